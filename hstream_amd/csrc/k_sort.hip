// gfx950 primitives: exclusive scan of u32/u64 counts and a stable LSD radix
// sort of (u32 key, u32 value) pairs, 8-bit digits, 256-thread workgroups.
//
// Sort pass = histogram (per-tile digit counts, digit-major) -> exclusive scan
// of the 256 x tiles counts -> stable scatter. Stability inside a tile comes
// from wave64 ballot match (8 ballots give each lane the mask of same-digit
// lanes) plus per-wave / per-round digit counters in LDS.
#include "hsg_sort.h"

namespace hsg {

constexpr int kSortThreads = 256;
constexpr int kSortItems = 16;  // rounds per tile
constexpr int kSortTile = kSortThreads * kSortItems;

// ---------------------------------------------------------------------------
// scan (u64 elements, exclusive), three kernels: reduce / top / apply
// ---------------------------------------------------------------------------
constexpr int kScanThreads = 256;
constexpr int kScanItems = 8;
constexpr int kScanTile = kScanThreads * kScanItems;

__device__ inline uint64_t wave_incl_sum64(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// block-wide exclusive scan of one value per thread (256 threads); returns the
// exclusive prefix, *total = block sum
__device__ inline uint64_t block_excl_sum256(uint64_t v, uint64_t *total) {
  __shared__ uint64_t sw[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t incl = wave_incl_sum64(v);
  if (lane == 63) sw[w] = incl;
  __syncthreads();
  uint64_t before = 0;
  for (int k = 0; k < w; ++k) before += sw[k];
  *total = sw[0] + sw[1] + sw[2] + sw[3];
  __syncthreads();
  return before + incl - v;
}

template <typename T>
__global__ __launch_bounds__(kScanThreads) void k_scan_reduce(const T *__restrict__ in, uint64_t n,
                                                              uint64_t *__restrict__ partial) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  uint64_t s = 0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    uint64_t i = base + (uint64_t)r * kScanThreads + threadIdx.x;
    if (i < n) s += (uint64_t)in[i];
  }
  uint64_t tot;
  block_excl_sum256(s, &tot);
  if (threadIdx.x == 0) partial[blockIdx.x] = tot;
}

// single workgroup: exclusive scan of the partials in place; total -> *total
__global__ __launch_bounds__(1024) void k_scan_top(uint64_t *__restrict__ partial, uint64_t m,
                                                   uint64_t *__restrict__ total) {
  __shared__ uint64_t sw[16];
  const uint64_t per = (m + 1023) / 1024;
  const uint64_t lo = threadIdx.x * per;
  const uint64_t hi = lo + per < m ? lo + per : m;
  uint64_t loc = 0;
  for (uint64_t i = lo; i < hi; ++i) loc += partial[i];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint64_t incl = wave_incl_sum64(loc);
  if (lane == 63) sw[w] = incl;
  __syncthreads();
  uint64_t run = incl - loc;
  for (int k = 0; k < w; ++k) run += sw[k];
  for (uint64_t i = lo; i < hi; ++i) {
    uint64_t v = partial[i];
    partial[i] = run;
    run += v;
  }
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int k = 0; k < 16; ++k) t += sw[k];
    if (total) *total = t;
  }
}

// out[i] = exclusive prefix of in (in and out may alias)
template <typename T, typename U>
__global__ __launch_bounds__(kScanThreads) void k_scan_apply(const T *in, uint64_t n,
                                                             const uint64_t *__restrict__ partial, U *out) {
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile;
  // each thread owns kScanItems consecutive elements
  const uint64_t t0 = base + (uint64_t)threadIdx.x * kScanItems;
  uint64_t v[kScanItems];
  uint64_t s = 0;
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    uint64_t i = t0 + r;
    v[r] = i < n ? (uint64_t)in[i] : 0;
    s += v[r];
  }
  uint64_t tot;
  uint64_t run = block_excl_sum256(s, &tot) + partial[blockIdx.x];
#pragma unroll
  for (int r = 0; r < kScanItems; ++r) {
    uint64_t i = t0 + r;
    if (i < n) out[i] = (U)run;
    run += v[r];
  }
}

// One workgroup for short inputs (n <= kScanSmall): each of 1024 threads owns
// kScanSmallPer consecutive elements, all loaded before the scan; one launch
// instead of three.
constexpr int kScanSmallPer = 8;
constexpr uint64_t kScanSmall = 1024 * kScanSmallPer;
template <typename T, typename U>
__global__ __launch_bounds__(1024) void k_scan_small(const T *in, uint64_t n, U *out, uint64_t *__restrict__ total) {
  __shared__ uint64_t sw[16];
  const uint64_t lo = (uint64_t)threadIdx.x * kScanSmallPer;
  uint64_t v[kScanSmallPer];
  uint64_t loc = 0;
#pragma unroll
  for (int r = 0; r < kScanSmallPer; ++r) {
    v[r] = lo + r < n ? (uint64_t)in[lo + r] : 0;  // in and out may alias: every read before any write
    loc += v[r];
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_sum64(loc);
  if (lane == 63) sw[w] = incl;
  __syncthreads();
  uint64_t run = incl - loc;
  for (int k = 0; k < w; ++k) run += sw[k];
#pragma unroll
  for (int r = 0; r < kScanSmallPer; ++r) {
    if (lo + r < n) out[lo + r] = (U)run;
    run += v[r];
  }
  if (threadIdx.x == 0 && total) {
    uint64_t t = 0;
    for (int k = 0; k < 16; ++k) t += sw[k];
    *total = t;
  }
}

uint64_t scan_partials_needed(uint64_t n) { return (n + kScanTile - 1) / kScanTile + 1; }

template <typename T, typename U>
static void scan_excl_impl(hipStream_t s, const T *in, U *out, uint64_t n, uint64_t *partial, uint64_t *total) {
  uint64_t blocks = (n + kScanTile - 1) / kScanTile;
  if (blocks == 0) {
    hipMemsetAsync(total, 0, 8, s);
    return;
  }
  if (n <= kScanSmall) {
    hipLaunchKernelGGL((k_scan_small<T, U>), dim3(1), dim3(1024), 0, s, in, n, out, total);
    return;
  }
  hipLaunchKernelGGL((k_scan_reduce<T>), dim3((unsigned)blocks), dim3(kScanThreads), 0, s, in, n, partial);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, s, partial, blocks, total);
  hipLaunchKernelGGL((k_scan_apply<T, U>), dim3((unsigned)blocks), dim3(kScanThreads), 0, s, in, n, partial, out);
}

void scan_excl_u32(hipStream_t s, const uint32_t *in, uint64_t *out, uint64_t n, uint64_t *partial, uint64_t *total) {
  scan_excl_impl<uint32_t, uint64_t>(s, in, out, n, partial, total);
}
void scan_excl_u8(hipStream_t s, const uint8_t *in, uint64_t *out, uint64_t n, uint64_t *partial, uint64_t *total) {
  scan_excl_impl<uint8_t, uint64_t>(s, in, out, n, partial, total);
}

// ---------------------------------------------------------------------------
// radix sort
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kSortThreads) void k_rs_hist(const uint32_t *__restrict__ keys, uint64_t n, int shift,
                                                          uint32_t *__restrict__ hist, uint64_t n_tiles) {
  __shared__ uint32_t cnt[256];
  cnt[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kSortTile;
#pragma unroll 4
  for (int r = 0; r < kSortItems; ++r) {
    uint64_t i = base + (uint64_t)r * kSortThreads + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & 255u], 1u);
  }
  __syncthreads();
  hist[(uint64_t)threadIdx.x * n_tiles + blockIdx.x] = cnt[threadIdx.x];
}

__global__ __launch_bounds__(kSortThreads) void k_rs_scatter(const uint32_t *__restrict__ kin,
                                                             const uint32_t *__restrict__ vin, uint64_t n, int shift,
                                                             const uint64_t *__restrict__ offs, uint64_t n_tiles,
                                                             uint32_t *__restrict__ kout, uint32_t *__restrict__ vout) {
  __shared__ uint64_t base_d[256];     // global offset of (digit, tile) + digits already placed
  __shared__ uint32_t wcnt[4][256];    // per-wave counts of the current round
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  base_d[threadIdx.x] = offs[(uint64_t)threadIdx.x * n_tiles + blockIdx.x];
  const uint64_t tile0 = (uint64_t)blockIdx.x * kSortTile;
  const uint64_t lt_mask = lane ? (~0ull >> (64 - lane)) : 0ull;
  for (int r = 0; r < kSortItems; ++r) {
    for (int k = 0; k < 4; ++k) wcnt[k][threadIdx.x] = 0;
    __syncthreads();
    uint64_t i = tile0 + (uint64_t)r * kSortThreads + threadIdx.x;
    bool in = i < n;
    uint32_t key = in ? kin[i] : 0;
    uint32_t val = in ? vin[i] : 0;
    uint32_t d = (key >> shift) & 255u;
    uint64_t peers = __ballot(in);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      uint64_t bal = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bal : ~bal;
    }
    uint32_t rank = (uint32_t)__popcll(peers & lt_mask);
    // the lowest lane of each peer group publishes the group's count
    if (in && rank == 0) wcnt[w][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (in) {
      uint64_t pos = base_d[d] + rank;
      for (int k = 0; k < w; ++k) pos += wcnt[k][d];
      kout[pos] = key;
      vout[pos] = val;
    }
    __syncthreads();
    uint32_t tot = wcnt[0][threadIdx.x] + wcnt[1][threadIdx.x] + wcnt[2][threadIdx.x] + wcnt[3][threadIdx.x];
    base_d[threadIdx.x] += tot;
    __syncthreads();
  }
}

uint64_t sort_tiles(uint64_t n) { return (n + kSortTile - 1) / kSortTile; }

// scratch: hist u32 [256*tiles], offs u64 [256*tiles], partial u64 [scan_partials_needed(256*tiles)]
uint64_t sort_scratch_bytes(uint64_t n) {
  uint64_t t = sort_tiles(n) + 1;
  return 256 * t * 4 + 256 * t * 8 + scan_partials_needed(256 * t) * 8 + 64;
}

// Sorts n pairs by the low `bits` of the key. Ping-pongs between (k0,v0) and
// (k1,v1); returns 0 if the result is in (k0,v0), 1 if in (k1,v1).
int radix_sort_pairs(hipStream_t s, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, int bits,
                     void *scratch) {
  if (n <= 1 || bits <= 0) return 0;
  uint64_t tiles = sort_tiles(n);
  uint32_t *hist = (uint32_t *)scratch;
  uint64_t *offs = (uint64_t *)((char *)scratch + 256 * (tiles + 1) * 4);
  uint64_t *partial = offs + 256 * (tiles + 1);
  int cur = 0;
  for (int shift = 0; shift < bits; shift += 8) {
    uint32_t *ki = cur ? k1 : k0, *vi = cur ? v1 : v0;
    uint32_t *ko = cur ? k0 : k1, *vo = cur ? v0 : v1;
    hipLaunchKernelGGL(k_rs_hist, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, ki, n, shift, hist, tiles);
    scan_excl_u32(s, hist, offs, 256 * tiles, partial, partial + scan_partials_needed(256 * tiles) - 1);
    hipLaunchKernelGGL(k_rs_scatter, dim3((unsigned)tiles), dim3(kSortThreads), 0, s, ki, vi, n, shift, offs, tiles,
                       ko, vo);
    cur ^= 1;
  }
  return cur;
}

}  // namespace hsg
