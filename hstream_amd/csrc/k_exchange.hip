// gfx950 kernels of the multi-GPU key exchange: owner = hash(key) mod G,
// stable partition by owner, packing into 8-byte-word records for one RCCL
// all-to-all-v, unpacking into columnar staging on the receiving rank.
//
// Record words: [key | valid bits << 32] [ts] [col 0..C-1] [seq]? [wm]?
// seq = the record's index in the global arrival order (rank slices in rank
// order), wm = its stream time (only when some record could be late).
#include "hsg_dev.h"
#include "hsg_exchange.h"

namespace hsg {

__device__ inline uint32_t owner_of(uint32_t key, uint32_t G) {
  return (uint32_t)(mix64((uint64_t)key ^ 0x5bd1e9955bd1e995ull) % G);
}

// min / max over the tile statistics -> info[0] = max ts (all records),
// info[1] = min ts of keyed records with ts >= 0, info[2] = n
__global__ __launch_bounds__(1024) void k_x_minmax(const int64_t *tmax, const int64_t *tmin, uint64_t n_tiles,
                                                   uint64_t n, int has_valid, int64_t *info) {
  __shared__ int64_t smax[16], smin[16];
  int64_t mx = INT64_MIN, mn = INT64_MAX;
  for (uint64_t t = threadIdx.x; t < n_tiles; t += 1024) {
    mx = tmax[t] > mx ? tmax[t] : mx;
    mn = tmin[t] < mn ? tmin[t] : mn;
  }
  mx = wave_max_i64(mx);
  mn = wave_min_i64(mn);
  if ((threadIdx.x & 63) == 0) {
    smax[threadIdx.x >> 6] = mx;
    smin[threadIdx.x >> 6] = mn;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 0; k < 16; ++k) {
      mx = smax[k] > mx ? smax[k] : mx;
      mn = smin[k] < mn ? smin[k] : mn;
    }
    info[0] = mx;
    info[1] = mn;
    info[2] = (int64_t)n;
    info[3] = has_valid;
  }
}

// owner digit per record (G = dropped: HSG_KEY_NONE records only move stream
// time, which the all-gathered maxima already carry) + histogram
__global__ void k_x_owner(Batch b, uint32_t G, uint32_t *owner, uint32_t *idx, unsigned long long *hist) {
  __shared__ unsigned int h[kMaxRanks + 1];
  if (threadIdx.x <= G) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < b.n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t key = b.key[i];
    uint32_t o = key == HSG_KEY_NONE ? G : owner_of(key, G);
    owner[i] = o;
    idx[i] = (uint32_t)i;
    atomicAdd(&h[o], 1u);
  }
  __syncthreads();
  if (threadIdx.x <= G && h[threadIdx.x]) atomicAdd(&hist[threadIdx.x], (unsigned long long)h[threadIdx.x]);
}

// per-record stream time in arrival order, seeded with the tile prefix
__global__ __launch_bounds__(kTileThreads) void k_x_recwm(Batch b, const int64_t *tprefix, int64_t *wm_out) {
  const uint64_t base = (uint64_t)blockIdx.x * kTileRecords;
  int64_t ts[kRecPerThread], wm[kRecPerThread];
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    ts[r] = i < b.n ? b.ts[i] : INT64_MIN;
  }
  tile_stream_time(ts, tprefix[blockIdx.x], wm);
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    if (i < b.n) wm_out[i] = wm[r];
  }
}

__global__ void k_x_pack(Batch b, XLayout L, const uint32_t *sidx, uint64_t m, uint64_t seq_base, const int64_t *wm,
                         uint64_t *send) {
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < m; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = sidx[q];
    uint64_t *w = send + q * L.words;
    uint64_t vb = 0;
    for (int c = 0; c < L.ncols; ++c) vb |= (uint64_t)(rec_present(b, c, i) ? 1u : 0u) << c;
    w[0] = (uint64_t)b.key[i] | (vb << 32);
    w[1] = (uint64_t)b.ts[i];
    for (int c = 0; c < L.ncols; ++c) w[2 + c] = (uint64_t)b.col[c][i];
    int k = 2 + L.ncols;
    if (L.has_seq) w[k++] = seq_base + i;
    if (L.has_wm) w[k++] = (uint64_t)wm[i];
  }
}

__global__ void k_x_unpack(XLayout L, const uint64_t *recv, uint64_t m, XStaging st) {
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < m; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t *w = recv + q * L.words;
    st.key[q] = (uint32_t)w[0];
    st.ts[q] = (int64_t)w[1];
    for (int c = 0; c < L.ncols; ++c) {
      st.col[c][q] = (int64_t)w[2 + c];
      if (L.has_valid) st.valid[c][q] = (uint8_t)((w[0] >> (32 + c)) & 1u);
    }
    int k = 2 + L.ncols;
    if (L.has_seq) st.seq[q] = (int64_t)w[k++];
    if (L.has_wm) st.wm[q] = (int64_t)w[k++];
  }
}

void launch_x_minmax(hipStream_t s, const int64_t *tmax, const int64_t *tmin, uint64_t n_tiles, uint64_t n,
                     int has_valid, int64_t *info) {
  hipLaunchKernelGGL(k_x_minmax, dim3(1), dim3(1024), 0, s, tmax, tmin, n_tiles, n, has_valid, info);
}
void launch_x_owner(hipStream_t s, const Batch &b, uint32_t G, uint32_t *owner, uint32_t *idx, uint64_t *hist) {
  if (b.n)
    hipLaunchKernelGGL(k_x_owner, dim3(grid_for(b.n, 256)), dim3(256), 0, s, b, G, owner, idx,
                       (unsigned long long *)hist);
}
void launch_x_recwm(hipStream_t s, const Batch &b, const int64_t *tprefix, int64_t *wm) {
  uint64_t tiles = (b.n + kTileRecords - 1) / kTileRecords;
  if (tiles) hipLaunchKernelGGL(k_x_recwm, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, tprefix, wm);
}
void launch_x_pack(hipStream_t s, const Batch &b, const XLayout &L, const uint32_t *sidx, uint64_t m,
                   uint64_t seq_base, const int64_t *wm, uint64_t *send) {
  if (m) hipLaunchKernelGGL(k_x_pack, dim3(grid_for(m, 256)), dim3(256), 0, s, b, L, sidx, m, seq_base, wm, send);
}
void launch_x_unpack(hipStream_t s, const XLayout &L, const uint64_t *recv, uint64_t m, const XStaging &st) {
  if (m) hipLaunchKernelGGL(k_x_unpack, dim3(grid_for(m, 256)), dim3(256), 0, s, L, recv, m, st);
}

}  // namespace hsg
