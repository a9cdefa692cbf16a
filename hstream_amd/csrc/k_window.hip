// gfx950 kernels for tumbling / hopping / unwindowed GROUP BY (per-batch and
// state-only modes): stream-time scan, window assignment fused with the HBM
// open-addressing (key, window) hash aggregation, and the touched-row emit /
// dump scans.
//
// Semantics follow the reference's per-record processor, restated for a batch:
//   windowsFor      hstream-processing/.../Stream/TimeWindowedStream.hs:105-117
//   grace check     TimeWindowedStream.hs:88-92 with stream time Processor.hs:139
//   state update    TimeWindowedStream.hs:93-100 (ksGet / aggF / ksPut)
//   SQL aggregates  hstream-sql/src/HStream/SQL/Codegen.hs:399-469
// The aggregates (COUNT/SUM/MIN/MAX, and LAST resolved by global arrival
// sequence) are commutative per group, so applying a batch's updates in any
// order gives the reference's final state; the exact per-record changelog is
// produced by the sort-based path in k_perrecord.hip.
#include "hsg_dev.h"
#include "hsg_sort.h"
#include "hsg_tw.h"

namespace hsg {

// ---------------------------------------------------------------------------
// fills
// ---------------------------------------------------------------------------
__global__ void k_fill_u64(uint64_t *__restrict__ p, uint64_t n, uint64_t v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ void k_fill_u32(uint32_t *__restrict__ p, uint64_t n, uint32_t v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    p[i] = v;
}
__global__ void k_fill_rows(int64_t *__restrict__ aggs, uint64_t rows, Program prog) {
  const uint64_t total = rows * (uint64_t)prog.n_slots;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < total; i += (uint64_t)gridDim.x * blockDim.x)
    aggs[i] = slot_identity_dev(prog.slot_op[i % prog.n_slots]);
}

// word wi of an empty row: key EMPTY, stamp 0, slot identities, padding 0
__device__ inline uint64_t tw_empty_word(const Program &prog, uint32_t wi) {
  if (wi == 0) return kEmpty;
  if (wi >= 2 && (int)(wi - 2) < prog.n_slots) return (uint64_t)slot_identity_dev(prog.slot_op[wi - 2]);
  return 0;
}

// Rows are an even number of words (tw_row_stride), so every 16-byte pair lies
// in one row: one 16-byte store per lane and iteration (the table is sized for
// the whole run, so this is a streaming write of hundreds of MB).
__global__ __launch_bounds__(256) void k_tw_reset(TwTable t, Program prog) {
  const uint64_t pairs = t.slots() * (uint64_t)t.stride / 2;  // regions + overflow rows
  const uint32_t sp = t.stride / 2;
  const bool pow2 = (sp & (sp - 1)) == 0;
  ulonglong2 *rows = reinterpret_cast<ulonglong2 *>(t.rows);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < pairs; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t wi = 2u * (pow2 ? (uint32_t)(i & (sp - 1)) : (uint32_t)(i % sp));
    rows[i] = make_ulonglong2(tw_empty_word(prog, wi), tw_empty_word(prog, wi + 1));
  }
}

// Clear of the claimed blocks only (t.dirty): a table sized for the worst
// batch holds few groups at a reset (C2: 4.3M of 32M slots, in ~1/8 of the
// blocks since a key's windows share a block), so this rewrites the rows of
// the claimed blocks instead of streaming the whole table. k_tw_dirty_count
// counts them first; when more than half the blocks are dirty (one-window
// keys spread over the table, C5) the whole table is streamed as by
// k_tw_reset.
__global__ __launch_bounds__(256) void k_tw_dirty_count(TwTable t, uint64_t nblk, unsigned long long *cnt) {
  uint64_t c = 0;
  const uint4 *m = reinterpret_cast<const uint4 *>(t.dirty);
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; 16 * i < nblk; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint4 v = m[i];  // the map is padded to 16 bytes (tw_dirty_bytes); bytes past nblk stay 0
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; ++k)
      c += ((w[k] & 0xFFu) != 0) + ((w[k] & 0xFF00u) != 0) + ((w[k] & 0xFF0000u) != 0) + ((w[k] >> 24) != 0);
  }
  c = wave_sum_u64(c);
  if ((threadIdx.x & 63) == 0 && c) atomicAdd(cnt, (unsigned long long)c);
}

// position of the r-th set bit of m (r < popcount(m)): binary search on
// popcounts of the low halves
__device__ inline uint32_t kth_set_bit(uint64_t m, uint32_t r) {
  uint32_t pos = 0;
#pragma unroll
  for (uint32_t w = 32; w; w >>= 1) {
    const uint32_t c = (uint32_t)__popcll((m >> pos) & ((1ull << w) - 1));
    if (c <= r) {
      r -= c;
      pos += w;
    }
  }
  return pos;
}

__global__ __launch_bounds__(256) void k_tw_reset_dirty(TwTable t, Program prog, uint64_t nblk, const uint64_t *cnt) {
  const uint32_t sp = t.stride / 2;
  const bool pow2 = (sp & (sp - 1)) == 0;
  ulonglong2 *rows = reinterpret_cast<ulonglong2 *>(t.rows);
  if (2 * *cnt > nblk) {  // uniform: most blocks dirty, stream the table and the map
    const uint64_t pairs = t.slots() * (uint64_t)sp;
    const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < pairs; i += step) {
      const uint32_t wi = 2u * (pow2 ? (uint32_t)(i & (sp - 1)) : (uint32_t)(i % sp));
      rows[i] = make_ulonglong2(tw_empty_word(prog, wi), tw_empty_word(prog, wi + 1));
    }
    uint4 *m = reinterpret_cast<uint4 *>(t.dirty);
    for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; 16 * i < nblk; i += step) m[i] = make_uint4(0, 0, 0, 0);
    return;
  }
  // a wave per 64 map bytes; the dirty blocks' 16-byte pairs spread over
  // all 64 lanes (pair q: the (q / ppb)-th dirty block of the ballot)
  const int lane = threadIdx.x & 63;
  const uint32_t ppb = 8u * sp;  // pairs per block
  const uint64_t waves = (uint64_t)gridDim.x * 4, w0 = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  for (uint64_t i0 = w0 * 64; i0 < nblk; i0 += waves * 64) {
    const uint64_t i = i0 + lane;
    const bool d = i < nblk && t.dirty[i] != 0;
    const uint64_t m = __ballot(d);
    if (d) t.dirty[i] = 0;
    const uint32_t total = (uint32_t)__popcll(m) * ppb;
    for (uint32_t q = lane; q < total; q += 64) {
      const uint32_t k = q / ppb, pr = q - k * ppb;
      const uint64_t blk = i0 + kth_set_bit(m, k);
      const uint32_t wi = 2u * (pow2 ? (pr & (sp - 1)) : (pr % sp));
      rows[blk * ppb + pr] = make_ulonglong2(tw_empty_word(prog, wi), tw_empty_word(prog, wi + 1));
    }
  }
}

// per-batch scalars: err .. touched, redo and scratch (wm / epoch / live persist)
__global__ void k_clear_scalars(DevScalars *sc) {
  const int t = threadIdx.x;
  if (t == 0) {
    sc->err = 0;
    sc->pairs = 0;
    sc->late = 0;
    sc->out_rows = 0;
    sc->touched = 0;
    sc->redo = 0;
    sc->packed = 0;
    sc->kbase = 0;
  }
  if (t < kScratchWords) sc->scratch[t] = 0;
}
void launch_clear_scalars(hipStream_t s, DevScalars *sc) { hipLaunchKernelGGL(k_clear_scalars, dim3(1), dim3(64), 0, s, sc); }

// The end of every push: the scalars into the pinned host mirror (one 8-byte
// word per lane, vector stores), then the per-batch ones cleared for the next
// batch -- one launch where a copy and a clear took two.
__global__ void k_fetch_clear_scalars(DevScalars *sc, DevScalars *h) {
  static_assert(sizeof(DevScalars) == 64 * 8, "one word per lane");
  const int t = threadIdx.x;
  reinterpret_cast<uint64_t *>(h)[t] = reinterpret_cast<const uint64_t *>(sc)[t];
  __syncthreads();
  if (t == 0) {
    sc->err = 0;
    sc->pairs = 0;
    sc->late = 0;
    sc->out_rows = 0;
    sc->touched = 0;
    sc->redo = 0;
    sc->packed = 0;
    sc->kbase = 0;
  }
  if (t < kScratchWords) sc->scratch[t] = 0;
}
void launch_fetch_clear_scalars(hipStream_t s, DevScalars *sc, DevScalars *h) {
  hipLaunchKernelGGL(k_fetch_clear_scalars, dim3(1), dim3(64), 0, s, sc, h);
}

// changelog rows [from, from + n) of src into device columns (null = skip), one launch
__global__ void k_copy_rows(OutCols src, uint64_t from, uint64_t n, int n_aggs, uint32_t *key, int64_t *ws, int64_t *we,
                            int64_t *si, RowPtrs aggs, uint32_t *form) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t q = from + i;
    if (key) key[i] = src.key[q];
    if (ws) ws[i] = src.ws[q];
    if (we) we[i] = src.we[q];
    if (si) si[i] = src.src[q];
    for (int j = 0; j < n_aggs; ++j)
      if (aggs.p[j]) aggs.p[j][i] = src.agg[j][q];
    if (form) form[i] = src.form ? src.form[q] : 0u;
  }
}
void launch_copy_rows(hipStream_t s, const OutCols &src, uint64_t from, uint64_t n, int n_aggs, uint32_t *key,
                      int64_t *ws, int64_t *we, int64_t *si, const RowPtrs &aggs, uint32_t *form) {
  if (n)
    hipLaunchKernelGGL(k_copy_rows, dim3(grid_for(n, 256)), dim3(256), 0, s, src, from, n, n_aggs, key, ws, we, si, aggs,
                       form);
}

unsigned grid_for(uint64_t n, unsigned tpb) {
  uint64_t g = (n + tpb - 1) / tpb;
  if (g > 4096) g = 4096;
  if (g == 0) g = 1;
  return (unsigned)g;
}

void launch_fill_u64(hipStream_t s, uint64_t *p, uint64_t n, uint64_t v) {
  if (n) hipLaunchKernelGGL(k_fill_u64, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n, v);
}
void launch_fill_u32(hipStream_t s, uint32_t *p, uint64_t n, uint32_t v) {
  if (n) hipLaunchKernelGGL(k_fill_u32, dim3(grid_for(n, 256)), dim3(256), 0, s, p, n, v);
}
void launch_tw_reset(hipStream_t s, const TwTable &t, const Program &prog) {
  hipLaunchKernelGGL(k_tw_reset, dim3(4096), dim3(256), 0, s, t, prog);
  if (t.dirty) hipMemsetAsync(t.dirty, 0, tw_dirty_bytes(t.slots()), s);
}
void launch_tw_reset_dirty(hipStream_t s, const TwTable &t, const Program &prog, uint64_t *cnt) {
  const uint64_t nblk = t.slots() >> 3;
  if (!nblk) return launch_tw_reset(s, t, prog);
  hipMemsetAsync(cnt, 0, 8, s);
  hipLaunchKernelGGL(k_tw_dirty_count, dim3(grid_for(nblk / 16 + 1, 256)), dim3(256), 0, s, t, nblk,
                     (unsigned long long *)cnt);
  hipLaunchKernelGGL(k_tw_reset_dirty, dim3(4096), dim3(256), 0, s, t, prog, nblk, (const uint64_t *)cnt);
}
// narrow transport -> full width: one pass, coalesced 2- / 4-byte loads and
// 4- / 8-byte stores
__global__ __launch_bounds__(256) void k_widen(WidenArgs w) {
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < w.n; i += step) {
    if (w.k16) w.key[i] = (uint32_t)w.k16[i];
    if (w.ts32) w.ts[i] = w.ts_base + (int64_t)w.ts32[i];
    if (w.ts16) w.ts[i] = w.frames[i / HSG_TS16_FRAME] + (int64_t)w.ts16[i];
#pragma unroll
    for (int c = 0; c < kMaxCols; ++c) {
      if (!w.c32[c]) continue;  // uniform
      const int32_t m = w.c32[c][i];
      // DEC32: the correctly rounded quotient of two exact doubles = the
      // double nearest the decimal m / 10^s, which its JSON text parses to
      w.col[c][i] = w.div[c] > 0.0 ? __builtin_bit_cast(int64_t, (double)m / w.div[c]) : (int64_t)m;
    }
  }
}

__global__ __launch_bounds__(256) void k_dump_keys(const int64_t *ws, uint64_t n, int64_t adv, int64_t k_epoch,
                                                  uint32_t *k, uint32_t *v) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    k[i] = adv > 0 ? (uint32_t)(ws[i] / adv - k_epoch) : 0u;
    v[i] = (uint32_t)i;
  }
}
__global__ __launch_bounds__(256) void k_gather_u32(const uint32_t *src, const uint32_t *perm, uint64_t n, uint32_t *dst) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[perm[i]];
}
__global__ __launch_bounds__(256) void k_gather_u64(const uint64_t *src, const uint32_t *perm, uint64_t n, uint64_t *dst) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    dst[i] = src[perm[i]];
}
void launch_dump_keys(hipStream_t s, const int64_t *ws, uint64_t n, int64_t adv, int64_t k_epoch, uint32_t *k, uint32_t *v) {
  if (n) hipLaunchKernelGGL(k_dump_keys, dim3(grid_for(n, 256)), dim3(256), 0, s, ws, n, adv, k_epoch, k, v);
}
void launch_gather_u32(hipStream_t s, const uint32_t *src, const uint32_t *perm, uint64_t n, uint32_t *dst) {
  if (n) hipLaunchKernelGGL(k_gather_u32, dim3(grid_for(n, 256)), dim3(256), 0, s, src, perm, n, dst);
}
void launch_gather_u64(hipStream_t s, const uint64_t *src, const uint32_t *perm, uint64_t n, uint64_t *dst) {
  if (n) hipLaunchKernelGGL(k_gather_u64, dim3(grid_for(n, 256)), dim3(256), 0, s, src, perm, n, dst);
}

void launch_widen(hipStream_t s, const WidenArgs &w) {
  if (w.n) hipLaunchKernelGGL(k_widen, dim3(grid_for(w.n, 256)), dim3(256), 0, s, w);
}

void launch_fill_rows(hipStream_t s, int64_t *aggs, uint64_t rows, const Program &prog) {
  if (rows && prog.n_slots)
    hipLaunchKernelGGL(k_fill_rows, dim3(grid_for(rows * prog.n_slots, 256)), dim3(256), 0, s, aggs, rows, prog);
}

// ---------------------------------------------------------------------------
// stream time (Processor.hs:139): per-tile max of every record's ts, then an
// exclusive prefix max over tiles seeded with the incoming watermark.
// Tile t covers records [t*kTileRecords, (t+1)*kTileRecords), record
// (r, thread) = t*kTileRecords + r*kTileThreads + thread.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(kTileThreads) void k_tile_stats(Batch b, int64_t *__restrict__ tmax,
                                                             int64_t *__restrict__ tmin) {
  __shared__ int64_t smax[kTileThreads / 64], smin[kTileThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kTileRecords;
  int64_t mx = INT64_MIN, mn = INT64_MAX;
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    if (i < b.n) {
      int64_t t = b.ts[i];
      mx = t > mx ? t : mx;
      if (b.key[i] != HSG_KEY_NONE && t >= 0) mn = t < mn ? t : mn;
    }
  }
  mx = wave_max_i64(mx);
  mn = wave_min_i64(mn);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) { smax[w] = mx; smin[w] = mn; }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int k = 1; k < kTileThreads / 64; ++k) {
      mx = smax[k] > mx ? smax[k] : mx;
      mn = smin[k] < mn ? smin[k] : mn;
    }
    tmax[blockIdx.x] = mx;
    tmin[blockIdx.x] = mn;
  }
}

// One workgroup: tile_prefix[t] = max(wm_in, tile_max[0..t-1]); sc->wm_out; epoch.
__global__ __launch_bounds__(1024) void k_tile_scan(const int64_t *__restrict__ tmax, const int64_t *__restrict__ tmin,
                                                    int64_t *__restrict__ tprefix, uint64_t n_tiles, int64_t wm_in,
                                                    int64_t adv, int set_epoch, int64_t grace, DevScalars *sc) {
  __shared__ int64_t swave[16];
  __shared__ int64_t swmin[16];
  const uint64_t per = (n_tiles + 1023) / 1024;
  const uint64_t lo = threadIdx.x * per;
  const uint64_t hi = lo + per < n_tiles ? lo + per : n_tiles;
  int64_t local = INT64_MIN, lmin = INT64_MAX;
  for (uint64_t t = lo; t < hi; ++t) {
    local = tmax[t] > local ? tmax[t] : local;
    lmin = tmin[t] < lmin ? tmin[t] : lmin;
  }
  int64_t incl = wave_incl_max(local);
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (lane == 63) swave[w] = incl;
  int64_t wmn = wave_min_i64(lmin);
  if (lane == 0) swmin[w] = wmn;
  __syncthreads();
  int64_t before = wm_in;
  for (int k = 0; k < w; ++k) before = swave[k] > before ? swave[k] : before;
  int64_t excl = __shfl_up(incl, 1, 64);
  if (lane > 0) before = excl > before ? excl : before;
  int64_t run = before;
  for (uint64_t t = lo; t < hi; ++t) {
    tprefix[t] = run;
    run = tmax[t] > run ? tmax[t] : run;
  }
  if (threadIdx.x == 0) {
    int64_t all = wm_in, amin = INT64_MAX;
    for (int k = 0; k < 16; ++k) {
      all = swave[k] > all ? swave[k] : all;
      amin = swmin[k] < amin ? swmin[k] : amin;
    }
    sc->wm_out = all;
    // every window of a record at ts t ends after t, so no window of this
    // batch can fail the grace check while stream time <= min ts + grace
    if (grace >= 0)
      sc->no_late = (amin == INT64_MAX || amin > INT64_MAX - grace || all <= amin + grace) ? 1u : 0u;
    else
      sc->no_late = 0;
    if (set_epoch && !sc->epoch_set && amin != INT64_MAX) {
      int64_t k0 = amin / adv - (int64_t)(1ll << 31);
      sc->k_epoch = k0 > 0 ? k0 : 0;
      sc->epoch_set = 1;
    }
  }
}

// One wave: the first keyed record with ts >= 0 (4 records per lane and
// step; usually record 0) sets the epoch 2^31 windows below its window, so
// the batch's windows fit 32 bits unless they span 2^31 windows. No keyed
// record: the epoch stays unset, as with k_tile_scan.
__global__ __launch_bounds__(64) void k_epoch_first(Batch b, int64_t adv, DevScalars *sc) {
  if (sc->epoch_set) return;
  const int lane = threadIdx.x;
  for (uint64_t base = 0; base < b.n; base += 256) {
    int64_t first = -1;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const uint64_t i = base + (uint64_t)u * 64 + lane;
      const bool ok = i < b.n && b.key[i] != HSG_KEY_NONE && b.ts[i] >= 0;
      const uint64_t m = __ballot(ok);
      if (m && first < 0) first = (int64_t)(base + (uint64_t)u * 64 + (__ffsll((long long)m) - 1));
    }
    if (first >= 0) {  // uniform
      if (lane == 0) {
        const int64_t k0 = b.ts[first] / adv - (int64_t)(1ll << 31);
        sc->k_epoch = k0 > 0 ? k0 : 0;
        sc->epoch_set = 1;
      }
      return;
    }
  }
}
void launch_epoch_first(hipStream_t s, const Batch &b, int64_t adv, DevScalars *sc) {
  hipLaunchKernelGGL(k_epoch_first, dim3(1), dim3(64), 0, s, b, adv, sc);
}

void launch_tile_stats(hipStream_t s, const Batch &b, int64_t *tile_max, int64_t *tile_min, uint64_t n_tiles) {
  if (n_tiles) hipLaunchKernelGGL(k_tile_stats, dim3((unsigned)n_tiles), dim3(kTileThreads), 0, s, b, tile_max, tile_min);
}
void launch_tile_scan(hipStream_t s, const int64_t *tile_max, const int64_t *tile_min, int64_t *tile_prefix,
                      uint64_t n_tiles, int64_t wm_in, int64_t adv, bool set_epoch, DevScalars *sc,
                      int64_t grace) {
  hipLaunchKernelGGL(k_tile_scan, dim3(1), dim3(1024), 0, s, tile_max, tile_min, tile_prefix, n_tiles, wm_in, adv,
                     set_epoch ? 1 : 0, grace, sc);
}

// ---------------------------------------------------------------------------
// window assignment + hash aggregation, one tile of kTileRecords per workgroup
// ---------------------------------------------------------------------------
// the tie words of MIN slot v: unset (the resolution pass takes the minimum
// over this batch's records holding the new value)
__device__ inline void tie_reset(const Program &prog, int64_t *__restrict__ row, int v) {
  for (int s = 0; s < prog.n_slots; ++s)
    if (prog.slot_op[s] == S_TIE_MIN && prog.slot_aux[s] == v)
      atomicExch((unsigned long long *)(row + s), ~0ull);
}

__device__ inline void apply_slots(const Program &prog, int64_t *__restrict__ row, const Batch &b, uint64_t i,
                                   uint64_t seq1) {
  for (int s = 0; s < prog.n_slots; ++s) {
    const int op = prog.slot_op[s];
    const int c = prog.slot_col[s];
    unsigned long long *u = (unsigned long long *)(row + s);
    switch (op) {
      case S_CNT_ALL: atomicAdd(u, 1ull); break;
      case S_CNT: if (rec_present(b, c, i)) atomicAdd(u, 1ull); break;
      case S_SUM_I: if (rec_present(b, c, i)) atomicAdd(u, (unsigned long long)b.col[c][i]); break;
      case S_SUM_F:
        if (rec_present(b, c, i)) unsafeAtomicAdd((double *)(row + s), __builtin_bit_cast(double, b.col[c][i]));
        break;
      case S_MIN_I:
        if (rec_present(b, c, i)) {
          const long long x = (long long)b.col[c][i];
          const long long old = atomicMin((long long *)(row + s), x);
          if (prog.ties && x < old) tie_reset(prog, row, s);
        }
        break;
      case S_MAX_I: if (rec_present(b, c, i)) atomicMax((long long *)(row + s), (long long)b.col[c][i]); break;
      case S_MIN_F:
        if (rec_present(b, c, i)) {
          const unsigned long long x = f64_ord(__builtin_bit_cast(double, b.col[c][i]));
          const unsigned long long old = atomicMin(u, x);
          if (prog.ties && x < old) tie_reset(prog, row, s);
        }
        break;
      case S_MAX_F:
        if (rec_present(b, c, i)) atomicMax(u, (unsigned long long)f64_ord(__builtin_bit_cast(double, b.col[c][i])));
        break;
      case S_LAST_SEQ: if (rec_present(b, c, i)) atomicMax(u, (unsigned long long)seq1); break;
      case S_CNT_DEC: if (rec_decimal(b, c, i)) atomicAdd(u, 1ull); break;
      case S_LAST_FORM: if (rec_present(b, c, i)) atomicMax(u, (unsigned long long)form_word(b, c, i, seq1)); break;
      default: break;  // S_LAST_VAL, S_TIE_*: the resolution pass
    }
  }
}

// Resolution pass, once the batch's LAST_SEQ / MIN / MAX words are final:
// the record whose sequence won LAST_SEQ writes LAST_VAL, and every record
// holding a MIN / MAX's value offers its literal to the tie word (the
// earliest for MIN, the latest for MAX: min n x = n, max n x = x). A MAX's
// word from earlier batches needs no reset (a record of this batch is later);
// a MIN's is reset by the aggregation pass when the batch lowers the minimum.
__device__ inline void apply_last(const Program &prog, int64_t *__restrict__ row, const Batch &b, uint64_t i,
                                  uint64_t seq1) {
  for (int s = 0; s < prog.n_slots; ++s) {
    const int op = prog.slot_op[s];
    const int c = prog.slot_col[s];
    if (op == S_LAST_SEQ) {
      if (rec_present(b, c, i) && (uint64_t)row[s] == seq1) row[s + 1] = b.col[c][i];
    } else if (slot_is_tie(op) && rec_present(b, c, i)) {
      const int v = prog.slot_aux[s], vop = prog.slot_op[v];
      const int64_t x = (vop == S_MIN_F || vop == S_MAX_F)
                            ? (int64_t)f64_ord(__builtin_bit_cast(double, b.col[c][i]))
                            : b.col[c][i];
      if (x != row[v]) continue;
      unsigned long long *u = (unsigned long long *)(row + s);
      const unsigned long long w = (unsigned long long)form_word(b, c, i, seq1);
      if (op == S_TIE_MIN) atomicMin(u, w);
      else atomicMax(u, w);
    }
  }
}

// pass 0 = aggregate, pass 1 = LAST resolution (lookups only)
template <int PASS>
__global__ __launch_bounds__(kTileThreads) void k_tw_agg(Batch b, TwParams p, TwTable t, Program prog,
                                                         const int64_t *__restrict__ tprefix,
                                                         const int64_t *__restrict__ rec_wm,
                                                         const int64_t *__restrict__ seq, DevScalars *sc) {
  __shared__ uint64_t sred[3][kTileThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kTileRecords;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t k_epoch = sc->k_epoch;

  uint32_t key[kRecPerThread];
  int64_t ts[kRecPerThread], wm[kRecPerThread];
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    bool in = i < b.n;
    key[r] = in ? b.key[i] : HSG_KEY_NONE;
    ts[r] = in ? b.ts[i] : INT64_MIN;
    if (rec_wm) wm[r] = in ? rec_wm[i] : INT64_MIN;
  }
  // 1) stream time per record (or the one computed before a key exchange)
  if (!rec_wm) tile_stream_time(ts, tprefix[blockIdx.x], wm);

  // 2) windows + hash aggregation
  uint64_t pairs = 0, late = 0;
  uint32_t fresh = 0, err = 0;
#pragma unroll 1
  for (int r = 0; r < kRecPerThread; ++r) {
    if (key[r] == HSG_KEY_NONE) continue;
    const uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    uint64_t k_lo, k_hi;
    if (!record_windows(p, ts[r], k_lo, k_hi)) continue;
    const uint64_t seq1 = (seq ? (uint64_t)seq[i] : p.rec_base + i) + 1;
    for (uint64_t k = k_lo; k <= k_hi; ++k) {
      if (!window_accepted(p, k, wm[r])) { late += 1; continue; }
      int64_t krel = (int64_t)k - k_epoch;
      if (krel < 0 || krel > 0xFFFFFFFFll) { err |= ERR_RANGE; continue; }
      uint64_t g = ((uint64_t)key[r] << 32) | (uint64_t)krel;
      if (PASS == 0) {
        int64_t slot = tw_find_or_insert(t, g, fresh);
        if (slot < 0) { err |= ERR_OOM; continue; }
        apply_slots(prog, t.aggs(slot), b, i, seq1);
        *t.stamp(slot) = (uint32_t)p.batch_id;
        pairs += 1;
      } else {
        int64_t slot = tw_find(t, g);
        if (slot >= 0) apply_last(prog, t.aggs(slot), b, i, seq1);
      }
    }
  }
  if (PASS != 0) return;

  // 3) per-workgroup counters
  pairs = wave_sum_u64(pairs);
  late = wave_sum_u64(late);
  uint64_t fr = wave_sum_u64(fresh);
  if (lane == 0) { sred[0][w] = pairs; sred[1][w] = late; sred[2][w] = fr; }
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a = 0, l = 0, f = 0;
    for (int k = 0; k < kTileThreads / 64; ++k) { a += sred[0][k]; l += sred[1][k]; f += sred[2][k]; }
    if (a) atomicAdd((unsigned long long *)&sc->pairs, (unsigned long long)a);
    if (l) atomicAdd((unsigned long long *)&sc->late, (unsigned long long)l);
    if (f) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)f);
  }
}

void launch_tw_agg(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const Program &prog,
                   const int64_t *tile_prefix, const int64_t *rec_wm, const int64_t *seq, DevScalars *sc,
                   bool last_pass) {
  uint64_t tiles = (b.n + kTileRecords - 1) / kTileRecords;
  if (!tiles) return;
  if (last_pass)
    hipLaunchKernelGGL(k_tw_agg<1>, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, p, t, prog, tile_prefix,
                       rec_wm, seq, sc);
  else
    hipLaunchKernelGGL(k_tw_agg<0>, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, p, t, prog, tile_prefix,
                       rec_wm, seq, sc);
}

// ---------------------------------------------------------------------------
// row emission: mode 0 = groups touched by this batch (per-batch changelog),
// mode 1 = every live group (ksDump). Deterministic: per-chunk counts, an
// exclusive scan, then rows written in slot order (no shared counter).
// ---------------------------------------------------------------------------
__device__ inline bool tw_hit(const TwTable &t, uint64_t s, uint64_t cap, int mode, uint32_t batch_id) {
  if (s >= cap) return false;
  uint64_t g = *t.key(s);
  if (g == kEmpty) return false;
  return mode == 1 || *t.stamp(s) == batch_id;
}

__global__ __launch_bounds__(256) void k_tw_emit_count(TwTable t, uint64_t cap, int mode, uint32_t batch_id,
                                                       uint32_t *cnt) {
  __shared__ uint64_t sw[4];
  const uint64_t c0 = (uint64_t)blockIdx.x * kEmitChunk;
  uint64_t h = 0;
  for (uint64_t s = c0 + threadIdx.x; s < c0 + kEmitChunk; s += 256) h += tw_hit(t, s, cap, mode, batch_id);
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = (uint32_t)(sw[0] + sw[1] + sw[2] + sw[3]);
}

__global__ __launch_bounds__(256) void k_tw_emit_rows(TwTable t, uint64_t cap, Program prog, TwParams p, int mode,
                                                      const uint64_t *off, OutCols out, uint64_t out_base,
                                                      uint64_t out_cap, DevScalars *sc) {
  __shared__ uint64_t swave[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t k_epoch = sc->k_epoch;
  const bool unwin = p.kind == HSG_UNWINDOWED;
  const uint64_t c0 = (uint64_t)blockIdx.x * kEmitChunk;
  uint64_t run = off[blockIdx.x];
  for (uint64_t blk = c0; blk < c0 + kEmitChunk; blk += 256) {
    const uint64_t s = blk + threadIdx.x;
    const bool hit = tw_hit(t, s, cap, mode, (uint32_t)p.batch_id);
    uint64_t f = hit ? 1 : 0;
    uint64_t incl = wave_incl_sum(f);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    uint64_t o = run + incl - f;
    for (int k = 0; k < w; ++k) o += swave[k];
    run += swave[0] + swave[1] + swave[2] + swave[3];
    __syncthreads();
    if (!hit) continue;
    o += out_base;
    if (o >= out_cap) {
      atomicOr(&sc->err, ERR_OOM);
      continue;
    }
    const uint64_t g = *t.key(s);
    const int64_t *row = t.aggs(s);
    out.key[o] = (uint32_t)(g >> 32);
    int64_t ws = 0, we = 0;
    if (!unwin) {
      int64_t k = k_epoch + (int64_t)(g & 0xFFFFFFFFull);
      ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
      we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
    }
    out.ws[o] = ws;
    out.we[o] = we;
    out.src[o] = -1;
    for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, row);
    if (out.form) out.form[o] = out_form(prog, row);
  }
}

uint64_t emit_chunks(uint64_t cap) { return (cap + kEmitChunk - 1) / kEmitChunk; }

// ---------------------------------------------------------------------------
// retention (retention.cpp): a window is closed once the stream time has
// reached its end + grace, since stream time never decreases, no later record
// passes the grace check of TimeWindowedStream.hs:92 for it. Closed rows are
// copied out whole (raw row words) to be kept on the host; the table is
// rebuilt from the rest, into the same or a larger capacity.
// ---------------------------------------------------------------------------
__device__ inline bool tw_row_closed(uint64_t g, int64_t k_epoch, const TwParams &p) {
  if (g == kEmpty || p.kind == HSG_UNWINDOWED) return false;
  const uint64_t k = (uint64_t)k_epoch + (g & 0xFFFFFFFFull);
  return !window_accepted(p, k, p.wm_in);
}

__global__ __launch_bounds__(256) void k_tw_closed_count(TwTable t, uint64_t cap, TwParams p, const DevScalars *sc,
                                                         uint32_t *cnt) {
  __shared__ uint64_t sw[4];
  const int64_t k_epoch = sc->k_epoch;
  const uint64_t c0 = (uint64_t)blockIdx.x * kEmitChunk;
  uint64_t h = 0;
  for (uint64_t s = c0 + threadIdx.x; s < c0 + kEmitChunk && s < cap; s += 256) h += tw_row_closed(*t.key(s), k_epoch, p);
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = (uint32_t)(sw[0] + sw[1] + sw[2] + sw[3]);
}

// closed rows, in slot order, to dst[row][stride] at the scanned chunk offsets
__global__ __launch_bounds__(256) void k_tw_closed_copy(TwTable t, uint64_t cap, TwParams p, const DevScalars *sc,
                                                        const uint64_t *off, uint64_t *__restrict__ dst) {
  __shared__ uint64_t swave[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t k_epoch = sc->k_epoch;
  const uint64_t c0 = (uint64_t)blockIdx.x * kEmitChunk;
  uint64_t run = off[blockIdx.x];
  for (uint64_t blk = c0; blk < c0 + kEmitChunk; blk += 256) {
    const uint64_t s = blk + threadIdx.x;
    const bool hit = s < cap && tw_row_closed(*t.key(s), k_epoch, p);
    const uint64_t f = hit ? 1 : 0;
    const uint64_t incl = wave_incl_sum(f);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    uint64_t o = run + incl - f;
    for (int k = 0; k < w; ++k) o += swave[k];
    run += swave[0] + swave[1] + swave[2] + swave[3];
    __syncthreads();
    if (!hit) continue;
    const uint64_t *src = t.key(s);
    for (uint32_t q = 0; q < t.stride; ++q) dst[o * t.stride + q] = src[q];
  }
}

// Rows src[0, n) (a table's slots or dense rows, `stride` words each) into
// table dst: empty rows skipped, closed rows too when skip_closed; every row
// is a distinct group, so an insert never meets a concurrent insert of its own
// group. *kept counts the rows inserted.
__global__ __launch_bounds__(256) void k_tw_reinsert(const uint64_t *__restrict__ src, uint64_t n, TwTable dst,
                                                     TwParams p, DevScalars *sc, int skip_closed,
                                                     unsigned long long *kept) {
  const int64_t k_epoch = sc->k_epoch;
  uint32_t fresh = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t *row = src + i * dst.stride;
    const uint64_t g = row[0];
    if (g == kEmpty || (skip_closed && tw_row_closed(g, k_epoch, p))) continue;
    const int64_t s = tw_find_or_insert(dst, g, fresh);
    if (s < 0) {
      atomicOr(&sc->err, ERR_OOM);
      continue;
    }
    uint64_t *d = dst.key((uint64_t)s);
    for (uint32_t q = 1; q < dst.stride; ++q) d[q] = row[q];
  }
  const uint64_t tot = wave_sum_u64(fresh);
  if ((threadIdx.x & 63) == 0 && tot) atomicAdd(kept, (unsigned long long)tot);
}

// A touched list across a table rebuild in the middle of a batch
// (op_device.cpp resume_deferred): its entries are slots of the old table,
// so they go through the group keys (k_touch_keys, before the rebuild) back
// to the slots of the new one (k_touch_slots, after it). kTouchSkip entries
// and groups the rebuild did not keep stay kTouchSkip.
__global__ __launch_bounds__(256) void k_touch_keys(TwTable t, const uint32_t *__restrict__ touched, uint64_t n,
                                                    uint64_t *__restrict__ keys) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t s = touched[i];
    keys[i] = s == kTouchSkipEntry ? kEmpty : *t.key(s);
  }
}
__global__ __launch_bounds__(256) void k_touch_slots(TwTable t, const uint64_t *__restrict__ keys, uint64_t n,
                                                     uint32_t *__restrict__ touched) {
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t g = keys[i];
    const int64_t s = g == kEmpty ? -1 : tw_find(t, g);
    touched[i] = s < 0 ? kTouchSkipEntry : (uint32_t)s;
  }
}
void launch_touch_keys(hipStream_t s, const TwTable &t, const uint32_t *touched, uint64_t n, uint64_t *keys) {
  if (n) hipLaunchKernelGGL(k_touch_keys, dim3(grid_for(n, 256)), dim3(256), 0, s, t, touched, n, keys);
}
void launch_touch_slots(hipStream_t s, const TwTable &t, const uint64_t *keys, uint64_t n, uint32_t *touched) {
  if (n) hipLaunchKernelGGL(k_touch_slots, dim3(grid_for(n, 256)), dim3(256), 0, s, t, keys, n, touched);
}

void launch_tw_closed(hipStream_t s, const TwTable &t, uint64_t cap, const TwParams &p, const DevScalars *sc,
                      const EmitScratch &es, uint64_t *total, uint64_t *dst) {
  const uint64_t nb = emit_chunks(cap);
  if (!dst) {
    hipLaunchKernelGGL(k_tw_closed_count, dim3((unsigned)nb), dim3(256), 0, s, t, cap, p, sc, es.cnt);
    scan_excl_u32(s, es.cnt, es.off, nb, es.partial, total);
  } else {
    hipLaunchKernelGGL(k_tw_closed_copy, dim3((unsigned)nb), dim3(256), 0, s, t, cap, p, sc, es.off, dst);
  }
}

void launch_tw_reinsert(hipStream_t s, const uint64_t *src, uint64_t n, const TwTable &dst, const TwParams &p,
                        DevScalars *sc, bool skip_closed, unsigned long long *kept) {
  if (n) hipLaunchKernelGGL(k_tw_reinsert, dim3(grid_for(n, 256)), dim3(256), 0, s, src, n, dst, p, sc,
                            skip_closed ? 1 : 0, kept);
}

void launch_tw_emit(hipStream_t s, const TwTable &t, uint64_t cap, const Program &prog, const TwParams &p, int mode,
                    OutCols out, uint64_t out_base, uint64_t out_cap, DevScalars *sc, const EmitScratch &es,
                    uint64_t *total) {
  uint64_t nb = emit_chunks(cap);
  hipLaunchKernelGGL(k_tw_emit_count, dim3((unsigned)nb), dim3(256), 0, s, t, cap, mode, (uint32_t)p.batch_id, es.cnt);
  scan_excl_u32(s, es.cnt, es.off, nb, es.partial, total);
  hipLaunchKernelGGL(k_tw_emit_rows, dim3((unsigned)nb), dim3(256), 0, s, t, cap, prog, p, mode, es.off, out, out_base,
                     out_cap, sc);
}

}  // namespace hsg
