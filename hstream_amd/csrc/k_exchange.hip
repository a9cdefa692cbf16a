// gfx950 kernels of the multi-GPU key exchange: owner = hash(key) mod G,
// stable partition by owner, packing into 8-byte-word records for one RCCL
// all-to-all-v, unpacking into columnar staging on the receiving rank.
//
// Record words: [key | valid bits << 32 | literal-form bits << 40] [ts] [col 0..C-1] [seq]? [wm]?
// seq = the record's index in the global arrival order (rank slices in rank
// order), wm = its stream time (only when some record could be late).
#include "hsg_dev.h"
#include "hsg_exchange.h"

namespace hsg {

// owner GPU of a key: the top log2(G) bits of key_hash for a power-of-two rank
// count (the same bits the fast exchange partitions on; local buckets skip
// them), hash mod G otherwise
__device__ inline uint32_t owner_of(uint32_t key, uint32_t G, int lg) {
  if (lg >= 0) return lg ? (uint32_t)(key_hash(key) >> (64 - lg)) : 0u;
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
__global__ void k_x_owner(Batch b, uint32_t G, int lg, uint32_t *owner, uint32_t *idx, unsigned long long *hist) {
  __shared__ unsigned int h[kMaxRanks + 1];
  if (threadIdx.x <= G) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < b.n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t key = b.key[i];
    uint32_t o = key == HSG_KEY_NONE ? G : owner_of(key, G, lg);
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
    uint64_t vb = 0, db = 0;  // presence, and the literal-form bit of the valid bytes
    for (int c = 0; c < L.ncols; ++c) {
      vb |= (uint64_t)(rec_present(b, c, i) ? 1u : 0u) << c;
      db |= (uint64_t)(rec_decimal(b, c, i) ? 1u : 0u) << c;
    }
    w[0] = (uint64_t)b.key[i] | (vb << 32) | (db << 40);
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
      if (L.has_valid) st.valid[c][q] = (uint8_t)(((w[0] >> (32 + c)) & 1u) | (((w[0] >> (40 + c)) & 1u) << 1));
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
    hipLaunchKernelGGL(k_x_owner, dim3(grid_for(b.n, 256)), dim3(256), 0, s, b, G, log2_exact(G), owner, idx,
                       (unsigned long long *)hist);
}

// ---------------------------------------------------------------------------
// fast exchange (no LAST / per-record order / late records): owner partition
// with the partition-offsets pipeline, columnar send buffers, one all-to-all-v
// per column, the received columns are the owner's batch as they are
// ---------------------------------------------------------------------------
constexpr int kXT = 4096;   // records per tile
constexpr int kXNT = 512;   // threads

// a record travels iff it has a key and, for a time-window op, ts >= 0 (the
// others only move stream time, which the all-gathered maxima carry)
__device__ inline bool x_sends(const Batch &b, uint64_t i, bool unwin) {
  return b.key[i] != HSG_KEY_NONE && (unwin || b.ts[i] >= 0);
}

// tile-major owner counts hist[tile][P] + the ts extrema (scratch[21..22] images)
__global__ __launch_bounds__(kXNT) void k_x_hist(Batch b, int xl, int unwin, uint32_t *hist, uint64_t tiles,
                                                 uint64_t *text) {
  __shared__ uint32_t cnt[kMaxRanks];
  __shared__ uint64_t sext[2][kXNT / 64];
  const uint32_t P = 1u << xl;
  for (uint32_t o = threadIdx.x; o < P; o += kXNT) cnt[o] = 0;
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kXT;
  uint64_t mx = 0, mn = 0;
  for (int r = 0; r < kXT / kXNT; ++r) {
    const uint64_t i = base + (uint64_t)r * kXNT + threadIdx.x;
    if (i >= b.n) break;
    const uint32_t key = b.key[i];
    const int64_t ts = b.ts[i];
    const uint64_t o = (uint64_t)ts ^ 0x8000000000000000ull;
    mx = o > mx ? o : mx;
    if (key != HSG_KEY_NONE && ts >= 0) mn = ~o > mn ? ~o : mn;
    if (key != HSG_KEY_NONE && (unwin || ts >= 0)) atomicAdd(&cnt[owner_of(key, P, xl)], 1u);
  }
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    const uint64_t a = __shfl_xor(mx, s, 64), c = __shfl_xor(mn, s, 64);
    mx = a > mx ? a : mx;
    mn = c > mn ? c : mn;
  }
  if ((threadIdx.x & 63) == 0) {
    sext[0][threadIdx.x >> 6] = mx;
    sext[1][threadIdx.x >> 6] = mn;
  }
  __syncthreads();
  for (uint32_t o = threadIdx.x; o < P; o += kXNT) hist[blockIdx.x * (uint64_t)P + o] = cnt[o];
  if (threadIdx.x == 0) {
    for (int k = 0; k < kXNT / 64; ++k) {
      mx = sext[0][k] > mx ? sext[0][k] : mx;
      mn = sext[1][k] > mn ? sext[1][k] : mn;
    }
    // per-tile slots, reduced by k_x_info (no contended device-scope atomics)
    text[2 * blockIdx.x] = mx;
    text[2 * blockIdx.x + 1] = mn;
  }
}

// this rank's facts for the all-gather: [max ts, min keyed ts, n, has_valid, per-rank counts]
__global__ void k_x_info(DevScalars *sc, const uint64_t *bstart, int xl, uint32_t G, uint64_t n, int has_valid,
                         int64_t *info, const uint64_t *__restrict__ text, uint64_t tiles) {
  uint64_t tx = 0, tn = 0;
  for (uint64_t t = threadIdx.x; t < tiles; t += 64) {
    const uint64_t a = text[2 * t], c = text[2 * t + 1];
    tx = a > tx ? a : tx;
    tn = c > tn ? c : tn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t a = __shfl_xor(tx, o, 64), c = __shfl_xor(tn, o, 64);
    tx = a > tx ? a : tx;
    tn = c > tn ? c : tn;
  }
  if (threadIdx.x != 0) return;
  uint64_t mx = sc->scratch[21], mn = sc->scratch[22];
  mx = tx > mx ? tx : mx;
  mn = tn > mn ? tn : mn;
  sc->scratch[21] = mx;  // as the per-workgroup atomics left them before
  sc->scratch[22] = mn;
  info[0] = mx ? (int64_t)(mx ^ 0x8000000000000000ull) : INT64_MIN;
  info[1] = mn ? (int64_t)(~mn ^ 0x8000000000000000ull) : INT64_MAX;
  info[2] = (int64_t)n;
  info[3] = has_valid;
  const uint32_t per = (1u << xl) / G;  // owner regions per rank (1 unless a test partitions finer)
  // an empty slice: the offsets pipeline did not run (no tiles), so bstart
  // still holds the previous batch's owner runs -- this rank sends nothing
  for (uint32_t q = 0; q < G; ++q) info[4 + q] = n ? (int64_t)(bstart[(q + 1) * per] - bstart[q * per]) : 0;
}

// every sent record at offt[tile][owner] + its slot in the tile's run, columnar
__global__ __launch_bounds__(kXNT) void k_x_scatter(Batch b, int xl, int unwin, int write_valid, int ncols,
                                                    const uint32_t *offt, XCols send) {
  __shared__ uint32_t cnt[kMaxRanks];
  __shared__ uint32_t goff[kMaxRanks];
  const uint32_t P = 1u << xl;
  for (uint32_t o = threadIdx.x; o < P; o += kXNT) {
    cnt[o] = 0;
    goff[o] = offt[blockIdx.x * (uint64_t)P + o];
  }
  __syncthreads();
  const uint64_t base = (uint64_t)blockIdx.x * kXT;
  for (int r = 0; r < kXT / kXNT; ++r) {
    const uint64_t i = base + (uint64_t)r * kXNT + threadIdx.x;
    if (i >= b.n) break;
    const uint32_t key = b.key[i];
    const int64_t ts = b.ts[i];
    if (key == HSG_KEY_NONE || (!unwin && ts < 0)) continue;
    const uint32_t o = owner_of(key, P, xl);
    const uint64_t d = (uint64_t)goff[o] + atomicAdd(&cnt[o], 1u);
    send.key[d] = key;
    send.ts[d] = ts;
    for (int c = 0; c < ncols; ++c) {
      send.col[c][d] = b.col[c][i];
      if (write_valid) send.valid[c][d] = rec_present(b, c, i) ? 1 : 0;
    }
  }
}

// Stable variant (the sequenced exchange): records in arrival order (round r,
// thread t) keep that order within each owner's run. Per round, a record's
// place = the owner's records of earlier rounds (cnt) + of earlier waves in
// this round (wcnt prefix) + of lower lanes of its wave (ballot match on the
// owner bits); one wave-count table, three barriers per round.
__global__ __launch_bounds__(kXNT) void k_x_scatter_seq(Batch b, int xl, int all_ts, int write_valid, int ncols,
                                                        const uint32_t *offt, XCols send, uint64_t seq_base,
                                                        const int64_t *wm) {
  constexpr int NW = kXNT / 64;
  __shared__ uint32_t cnt[kMaxRanks];
  __shared__ uint32_t goff[kMaxRanks];
  __shared__ uint32_t wcnt[NW][kMaxRanks];
  const uint32_t P = 1u << xl;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint32_t o = threadIdx.x; o < P; o += kXNT) {
    cnt[o] = 0;
    goff[o] = offt[blockIdx.x * (uint64_t)P + o];
  }
  const uint64_t base = (uint64_t)blockIdx.x * kXT;
  const uint64_t below = (1ull << lane) - 1ull;
  for (int r = 0; r < kXT / kXNT; ++r) {
    for (uint32_t k = threadIdx.x; k < (uint32_t)NW * P; k += kXNT) wcnt[k / P][k % P] = 0;
    __syncthreads();
    const uint64_t i = base + (uint64_t)r * kXNT + threadIdx.x;
    bool go = false;
    uint32_t o = 0;
    if (i < b.n) {
      const uint32_t key = b.key[i];
      go = key != HSG_KEY_NONE && (all_ts || b.ts[i] >= 0);
      if (go) o = owner_of(key, P, xl);
    }
    // lanes of this wave with the same owner
    uint64_t peers = __ballot(go);
    for (int bit = 0; bit < xl; ++bit) {
      const uint64_t m = __ballot(go && ((o >> bit) & 1u));
      peers &= ((o >> bit) & 1u) ? m : ~m;
    }
    const uint32_t rk = (uint32_t)__popcll(peers & below);
    if (go && rk == 0) wcnt[w][o] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (go) {
      uint32_t pre = cnt[o];
      for (int k = 0; k < w; ++k) pre += wcnt[k][o];
      const uint64_t d = (uint64_t)goff[o] + pre + rk;
      send.key[d] = b.key[i];
      send.ts[d] = b.ts[i];
      for (int c = 0; c < ncols; ++c) {
        send.col[c][d] = b.col[c][i];
        // (the literal-form bit rides along: ops with literal forms use this exchange)
        if (write_valid) send.valid[c][d] = b.valid[c] ? b.valid[c][i] : (uint8_t)1;
      }
      send.seq[d] = (int64_t)(seq_base + i);
      if (wm) send.wm[d] = wm[i];
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < P; q += kXNT) {
      uint32_t t = 0;
      for (int k = 0; k < NW; ++k) t += wcnt[k][q];
      cnt[q] += t;
    }
    __syncthreads();  // (the next round clears wcnt)
  }
}

void launch_x_scatter_seq(hipStream_t s, const Batch &b, int xl, bool all_ts, bool write_valid, int ncols,
                          const uint32_t *offt, const XCols &send, uint64_t seq_base, const int64_t *wm) {
  const uint64_t tiles = x_tiles(b.n);
  if (tiles)
    hipLaunchKernelGGL(k_x_scatter_seq, dim3((unsigned)tiles), dim3(kXNT), 0, s, b, xl, all_ts ? 1 : 0,
                       write_valid ? 1 : 0, ncols, offt, send, seq_base, wm);
}

uint64_t x_tiles(uint64_t n) { return (n + kXT - 1) / kXT; }

void launch_x_hist(hipStream_t s, const Batch &b, int xl, bool unwin, uint32_t *hist, uint64_t *text, DevScalars *) {
  const uint64_t tiles = x_tiles(b.n);
  if (tiles)
    hipLaunchKernelGGL(k_x_hist, dim3((unsigned)tiles), dim3(kXNT), 0, s, b, xl, unwin ? 1 : 0, hist, tiles, text);
}
void launch_x_info(hipStream_t s, DevScalars *sc, const uint64_t *bstart, int xl, uint32_t G, uint64_t n,
                   bool has_valid, int64_t *info, const uint64_t *text, uint64_t tiles) {
  hipLaunchKernelGGL(k_x_info, dim3(1), dim3(64), 0, s, sc, bstart, xl, G, n, has_valid ? 1 : 0, info, text, tiles);
}
void launch_x_scatter(hipStream_t s, const Batch &b, int xl, bool unwin, bool write_valid, int ncols,
                      const uint32_t *offt, const XCols &send) {
  const uint64_t tiles = x_tiles(b.n);
  if (tiles)
    hipLaunchKernelGGL(k_x_scatter, dim3((unsigned)tiles), dim3(kXNT), 0, s, b, xl, unwin ? 1 : 0,
                       write_valid ? 1 : 0, ncols, offt, send);
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
