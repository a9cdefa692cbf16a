// gfx950 kernels of the partitioned (key, window) aggregation:
//
//   hist     per-tile bucket counts of the records that have >= 1 accepted
//            window (bucket = top bits of hash(key): every window of a key
//            lands in one bucket)
//   scan     bucket-major exclusive prefix -> bucket ranges
//   scatter  each tile is bucket-sorted in LDS, then every bucket's run is
//            written by consecutive lanes as packed 8-byte-word records
//            [key|krel<<32][nwin|valid<<32][cols][seq+1]? (coalesced stores;
//            scattering 4-8 B fields per record directly ran at ~280 GB/s)
//   agg      one workgroup per <= kAggChunk records of a bucket: LDS hash table
//            of the chunk's groups fed by LDS atomics, then one flush per group
//            into the HBM table -- plain read-modify-write when the workgroup is
//            the bucket's only chunk (it owns those groups), atomics otherwise;
//            pairs that do not fit the LDS table go straight to HBM atomics.
//
// Window assignment and grace follow TimeWindowedStream.hs:86-103 / :105-117
// exactly as in k_window.hip (rejected windows are always the earliest ones, so
// the accepted windows of a record are one consecutive run).
#include "hsg_dev.h"
#include "hsg_part.h"
#include "hsg_tw.h"

namespace hsg {

constexpr uint16_t kNoBucket = 0xFFFF;

__device__ inline uint32_t bucket_of(uint32_t key, int np_log2) {
  return np_log2 ? (uint32_t)(mix64((uint64_t)key * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) >> (64 - np_log2))
                 : 0u;
}

// Accepted window run of one record: [krel, krel + nwin) relative to the epoch.
__device__ inline bool part_record(const TwParams &p, int64_t k_epoch, uint32_t key, int64_t ts, int64_t wm,
                                   uint32_t &krel, uint32_t &nwin, uint64_t &late, uint32_t &err) {
  if (key == HSG_KEY_NONE) return false;
  uint64_t k_lo, k_hi;
  if (!record_windows(p, ts, k_lo, k_hi)) return false;
  uint64_t k = k_lo;
  while (k <= k_hi && !window_accepted(p, k, wm)) {
    ++k;
    ++late;
  }
  if (k > k_hi) return false;
  int64_t a = (int64_t)k - k_epoch, z = (int64_t)k_hi - k_epoch;
  if (a < 0) {
    err |= ERR_RANGE;
    a = 0;
  }
  if (z > 0xFFFFFFFFll) {
    err |= ERR_RANGE;
    z = 0xFFFFFFFFll;
  }
  if (a > z) return false;
  krel = (uint32_t)a;
  nwin = (uint32_t)(z - a + 1);
  return true;
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so
// give workgroups b, b+8, b+16, ... (one XCD) consecutive tiles; a bucket's
// runs from consecutive tiles are adjacent in the output. Speed only.
__device__ inline uint64_t xcd_tile(uint64_t blk, uint64_t tiles) {
  const uint64_t per = tiles / 8, full = per * 8;
  if (blk >= full) return blk;
  return (blk & 7) * per + (blk >> 3);
}

// Per-record stream time in arrival order, only when some record of the batch
// may fail the grace check (sc->no_late == 0); otherwise every workgroup exits.
__global__ __launch_bounds__(kTileThreads) void k_part_recwm(Batch b, const int64_t *__restrict__ tprefix,
                                                             const DevScalars *sc, int64_t *__restrict__ wm_out) {
  if (sc->no_late) return;  // uniform
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

void launch_part_recwm(hipStream_t s, const Batch &b, const int64_t *tprefix, const DevScalars *sc, int64_t *wm) {
  uint64_t tiles = (b.n + kTileRecords - 1) / kTileRecords;
  if (tiles) hipLaunchKernelGGL(k_part_recwm, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, tprefix, sc, wm);
}

// stream time source: the exchange's per-record times, else our own unless no
// record can be late (then every window is accepted and none is needed)
__device__ inline const int64_t *pick_wm(const int64_t *rec_wm, const int64_t *own, const DevScalars *sc) {
  return rec_wm ? rec_wm : (sc->no_late ? nullptr : own);
}

// Walk the T records of one partition tile with NT threads (record (r, t) =
// tile*T + r*NT + t); calls f(j, i, key, krel, nwin) for every record with
// >= 1 accepted window (j = tile-local index, i = batch index). No barriers.
template <int T, int NT, typename F>
__device__ inline void walk_tile(const Batch &b, const TwParams &p, uint64_t tile, int64_t k_epoch,
                                 const int64_t *__restrict__ wm, uint64_t &late, uint32_t &err, F f) {
  constexpr int R = T / NT;
  const uint64_t base = tile * T;
  // every load of the tile is issued before the first record is processed
  uint32_t key[R];
  int64_t ts[R], w[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t i = base + (uint64_t)r * NT + threadIdx.x;
    const bool in = i < b.n;
    key[r] = in ? b.key[i] : HSG_KEY_NONE;
    ts[r] = in ? b.ts[i] : 0;
    w[r] = in && wm ? wm[i] : INT64_MIN;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = r * NT + threadIdx.x;
    uint32_t krel, nwin;
    if (!part_record(p, k_epoch, key[r], ts[r], w[r], krel, nwin, late, err)) continue;
    f(j, base + j, key[r], krel, nwin);
  }
}

constexpr int kPNT = 512;  // threads of the partition passes

template <int T>
__global__ __launch_bounds__(kPNT) void k_part_hist(Batch b, TwParams p, PartParams pp,
                                                    const int64_t *__restrict__ rec_wm,
                                                    const int64_t *__restrict__ own_wm, PartBuffers pb,
                                                    DevScalars *sc) {
  __shared__ uint32_t cnt[1 << kPartMaxLog2];
  __shared__ uint64_t sred[kPNT / 64];
  const int nb = 1 << pp.np_log2;
  const uint64_t tile = xcd_tile(blockIdx.x, pp.tiles);
  for (int i = threadIdx.x; i < nb; i += kPNT) cnt[i] = 0;
  __syncthreads();
  uint64_t late = 0;
  uint32_t err = 0;
  walk_tile<T, kPNT>(b, p, tile, sc->k_epoch, pick_wm(rec_wm, own_wm, sc), late, err,
                     [&](int, uint64_t, uint32_t key, uint32_t, uint32_t) {
                       atomicAdd(&cnt[bucket_of(key, pp.np_log2)], 1u);
                     });
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += kPNT) pb.hist[(uint64_t)i * pp.tiles + tile] = cnt[i];
  late = wave_sum_u64(late);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = late;
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t l = 0;
    for (int k = 0; k < kPNT / 64; ++k) l += sred[k];
    if (l) atomicAdd((unsigned long long *)&sc->late, (unsigned long long)l);
  }
}

// LDS holds only the tile's bucket sort (bucket, order, window run per record:
// 12 B) plus per-bucket run starts, so two workgroups fit a CU; the record
// words are gathered from the (L2-resident) input at write-out.
template <int T>
__global__ __launch_bounds__(kPNT) void k_part_scatter(Batch b, TwParams p, PartParams pp,
                                                       const int64_t *__restrict__ rec_wm,
                                                       const int64_t *__restrict__ own_wm,
                                                       const int64_t *__restrict__ seq, PartBuffers pb,
                                                       DevScalars *sc) {
  __shared__ uint16_t lbk[T];
  __shared__ uint16_t sidx[T];
  __shared__ uint64_t lkn[T];  // krel | nwin << 32
  __shared__ uint32_t lstart[1 << kPartMaxLog2];
  __shared__ uint32_t cursor[1 << kPartMaxLog2];
  __shared__ uint32_t goff[1 << kPartMaxLog2];
  __shared__ uint32_t swave[kPNT / 64];
  const int nb = 1 << pp.np_log2;
  const int W = pp.words;
  const int C = W - 2 - pp.has_seq;
  const uint64_t tile = xcd_tile(blockIdx.x, pp.tiles);
  const uint64_t q0 = wall_clock64();
  for (int i = threadIdx.x; i < nb; i += kPNT) cursor[i] = 0;
  for (int j = threadIdx.x; j < T; j += kPNT) lbk[j] = kNoBucket;
  __syncthreads();
  // 1) window runs and buckets of the tile's records, bucket histogram
  uint64_t late = 0;
  uint32_t err = 0;
  walk_tile<T, kPNT>(b, p, tile, sc->k_epoch, pick_wm(rec_wm, own_wm, sc), late, err,
                     [&](int j, uint64_t, uint32_t key, uint32_t krel, uint32_t nwin) {
                       const uint32_t bk = bucket_of(key, pp.np_log2);
                       lkn[j] = (uint64_t)krel | ((uint64_t)nwin << 32);
                       lbk[j] = (uint16_t)bk;
                       atomicAdd(&cursor[bk], 1u);
                     });
  __syncthreads();
  const uint64_t q1 = wall_clock64();
  // 2) tile-local exclusive scan of the histogram; global run starts
  const int per = (nb + kPNT - 1) / kPNT;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint32_t loc = 0;
  for (int k = lo; k < hi; ++k) loc += cursor[k];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) swave[wv] = incl;
  __syncthreads();
  uint32_t run = incl - loc;
  for (int k = 0; k < wv; ++k) run += swave[k];
  for (int k = lo; k < hi; ++k) {
    lstart[k] = run;
    run += cursor[k];
    cursor[k] = 0;
    goff[k] = (uint32_t)pb.off[(uint64_t)k * pp.tiles + tile];
  }
  uint32_t placed = 0;
  for (int k = 0; k < kPNT / 64; ++k) placed += swave[k];
  __syncthreads();
  const uint64_t q2 = wall_clock64();
  // 3) bucket-sorted order of the tile's records
  for (int j = threadIdx.x; j < T; j += kPNT) {
    const uint16_t bk = lbk[j];
    if (bk == kNoBucket) continue;
    sidx[lstart[bk] + atomicAdd(&cursor[bk], 1u)] = (uint16_t)j;
  }
  __syncthreads();
  const uint64_t q3 = wall_clock64();
  // 4) coalesced write-out: consecutive lanes write consecutive words of a run
  const uint32_t inv = (1u << 20) / (uint32_t)W + 1;  // t / W for t < 2^16, W <= 16
  const uint32_t total = placed * (uint32_t)W;
  const uint64_t base = tile * T;
#pragma unroll 4
  for (uint32_t t = threadIdx.x; t < total; t += kPNT) {
    const uint32_t q = (uint32_t)(((uint64_t)t * inv) >> 20);
    const uint32_t w = t - q * (uint32_t)W;
    const uint16_t j = sidx[q];
    const uint16_t bk = lbk[j];
    const uint64_t i = base + j;
    const uint64_t dest = (uint64_t)goff[bk] + (q - lstart[bk]);
    uint64_t v;
    if (w == 0) {
      v = (uint64_t)b.key[i] | (lkn[j] << 32);
    } else if (w == 1) {
      uint64_t vb = 0;
      for (int c = 0; c < C; ++c)
        if (!(pp.has_valid && b.valid[c] && !b.valid[c][i])) vb |= 1ull << c;
      v = (lkn[j] >> 32) | (vb << 32);
    } else if ((int)w < 2 + C) {
      v = (uint64_t)b.col[w - 2][i];
    } else {
      v = (uint64_t)((seq ? seq[i] : (int64_t)(p.rec_base + i)) + 1);
    }
    pb.rec[dest * W + w] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t q4 = wall_clock64();
    atomicAdd((unsigned long long *)&sc->scratch[13], (unsigned long long)(q1 - q0));
    atomicAdd((unsigned long long *)&sc->scratch[14], (unsigned long long)(q2 - q1));
    atomicAdd((unsigned long long *)&sc->scratch[15], (unsigned long long)(q3 - q2));
    atomicAdd((unsigned long long *)&sc->scratch[16], (unsigned long long)(q4 - q3));
    atomicAdd((unsigned long long *)&sc->scratch[17], 1ull);
  }
}

void launch_part_hist(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp, const int64_t *rec_wm,
                      const int64_t *own_wm, const PartBuffers &pb, DevScalars *sc) {
  if (!pp.tiles) return;
  hipLaunchKernelGGL(k_part_hist<kPartTileRecs>, dim3((unsigned)pp.tiles), dim3(kPNT), 0, s, b, p, pp, rec_wm, own_wm,
                     pb, sc);
}

void launch_part_scatter(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                         const int64_t *rec_wm, const int64_t *own_wm, const int64_t *seq, const PartBuffers &pb,
                         DevScalars *sc) {
  if (!pp.tiles) return;
  hipLaunchKernelGGL(k_part_scatter<kPartTileRecs>, dim3((unsigned)pp.tiles), dim3(kPNT), 0, s, b, p, pp, rec_wm,
                     own_wm, seq, pb, sc);
}

// ---------------------------------------------------------------------------
// chunk map: chunk_start[b] = first aggregation workgroup of bucket b
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_part_chunks(const uint64_t *off, uint64_t tiles, int np_log2,
                                                      uint32_t *chunk_start) {
  __shared__ uint32_t sw[16];
  const int nb = 1 << np_log2;
  const int per = (nb + 1023) / 1024;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint32_t loc = 0;
  for (int b = lo; b < hi; ++b) {
    uint64_t sz = off[(uint64_t)(b + 1) * tiles] - off[(uint64_t)b * tiles];
    loc += (uint32_t)((sz + kAggChunk - 1) / kAggChunk);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) sw[w] = incl;
  __syncthreads();
  uint32_t run = incl - loc;
  for (int k = 0; k < w; ++k) run += sw[k];
  for (int b = lo; b < hi; ++b) {
    chunk_start[b] = run;
    uint64_t sz = off[(uint64_t)(b + 1) * tiles] - off[(uint64_t)b * tiles];
    run += (uint32_t)((sz + kAggChunk - 1) / kAggChunk);
  }
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 16; ++k) t += sw[k];
    chunk_start[nb] = t;
  }
}

// ---------------------------------------------------------------------------
// LDS aggregation of one chunk
// ---------------------------------------------------------------------------
// One partitioned record held in registers: [w0 w1 col 0..C-1 seq+1?]. Runtime
// word selection is an unrolled compare chain, so the record never leaves VGPRs.
template <int WMAX>
struct PRec {
  uint64_t w[WMAX];
  int C;
  __device__ bool present(int c) const { return (w[1] >> (32 + c)) & 1ull; }
  __device__ int64_t word(int k) const {
    int64_t v = 0;
#pragma unroll
    for (int q = 2; q < WMAX; ++q)
      if (q == k) v = (int64_t)w[q];
    return v;
  }
  __device__ int64_t col(int c) const { return word(2 + c); }
  __device__ int64_t seq1() const { return word(2 + C); }
};

// contribution of the record to slot s (identity when absent)
template <typename R>
__device__ inline int64_t prec_elem(const Program &prog, int s, const R &r) {
  const int op = prog.slot_op[s];
  const int c = prog.slot_col[s];
  if (op == S_CNT_ALL) return 1;
  if (op == S_LAST_VAL) return 0;
  if (!r.present(c)) return slot_identity_dev(op);
  switch (op) {
    case S_CNT: return 1;
    case S_SUM_I:
    case S_SUM_F:
    case S_MIN_I:
    case S_MAX_I: return r.col(c);
    case S_MIN_F:
    case S_MAX_F: return (int64_t)f64_ord(__builtin_bit_cast(double, r.col(c)));
    case S_LAST_SEQ: return r.seq1();
    default: return 0;
  }
}

template <int MS, typename R>
__device__ inline void lds_apply(const Program &prog, int64_t *__restrict__ row, const R &r) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
    if (op == S_LAST_VAL) continue;
    if (op != S_CNT_ALL && !r.present(prog.slot_col[s])) continue;
    const int64_t x = prec_elem(prog, s, r);
    unsigned long long *u = (unsigned long long *)(row + s);
    switch (op) {
      case S_CNT_ALL:
      case S_CNT:
      case S_SUM_I: atomicAdd(u, (unsigned long long)x); break;
      case S_SUM_F: unsafeAtomicAdd((double *)(row + s), __builtin_bit_cast(double, x)); break;
      case S_MIN_I: atomicMin((long long *)(row + s), (long long)x); break;
      case S_MAX_I: atomicMax((long long *)(row + s), (long long)x); break;
      case S_MIN_F: atomicMin(u, (unsigned long long)x); break;
      case S_MAX_F:
      case S_LAST_SEQ: atomicMax(u, (unsigned long long)x); break;
      default: break;
    }
  }
}

// HBM-side combine of a finished row of partial aggregates (v) into `row`.
__device__ inline void flush_row(const Program &prog, int64_t *__restrict__ row, const int64_t *v, bool exclusive) {
  for (int s = 0; s < prog.n_slots; ++s) {
    const int op = prog.slot_op[s];
    const int64_t x = v[s];
    if (op == S_LAST_VAL) continue;
    if (x == slot_identity_dev(op)) continue;  // nothing to add
    if (exclusive) {
      row[s] = op == S_LAST_SEQ ? ((uint64_t)x > (uint64_t)row[s] ? x : row[s]) : slot_combine(op, row[s], x);
      continue;
    }
    unsigned long long *u = (unsigned long long *)(row + s);
    switch (op) {
      case S_CNT_ALL:
      case S_CNT:
      case S_SUM_I: atomicAdd(u, (unsigned long long)x); break;
      case S_SUM_F: unsafeAtomicAdd((double *)(row + s), __builtin_bit_cast(double, x)); break;
      case S_MIN_I: atomicMin((long long *)(row + s), (long long)x); break;
      case S_MAX_I: atomicMax((long long *)(row + s), (long long)x); break;
      case S_MIN_F: atomicMin(u, (unsigned long long)x); break;
      case S_MAX_F:
      case S_LAST_SEQ: atomicMax(u, (unsigned long long)x); break;
      default: break;
    }
  }
}

template <int MS, int E, int WMAX, int KU>
__global__ __launch_bounds__(kAggThreads, 4) void k_part_agg(Program prog, TwParams p, PartParams pp, TwTable t,
                                                          PartBuffers pb, DevScalars *sc) {
  __shared__ uint64_t lkey[E];
  __shared__ int64_t lagg[E * MS];
  __shared__ uint32_t lfill;
  __shared__ uint32_t sb, sc0, sc1;
  __shared__ uint64_t sred[3][kAggThreads / 64];
  __shared__ uint32_t ltouch[E];  // slots this workgroup touched first in this batch
  __shared__ uint32_t ltn;
  __shared__ uint16_t llive[E];   // live entries of the LDS table, compacted
  __shared__ uint32_t lnl;
  __shared__ uint64_t lbase;
  const int nb = 1 << pp.np_log2;
  const uint32_t *chunk_start = pb.chunk_start;
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) {
    // find this workgroup's bucket: chunk_start[b] <= blockIdx.x < chunk_start[b + 1]
    uint32_t w = blockIdx.x;
    int lo = 0, hi = nb;
    while (lo < hi) {
      int m = (lo + hi) >> 1;
      if (chunk_start[m + 1] <= w) lo = m + 1;
      else hi = m;
    }
    sb = (uint32_t)lo;
    sc0 = chunk_start[lo];
    sc1 = chunk_start[lo + 1];
    lfill = 0;
    ltn = 0;
    lnl = 0;
  }
  for (int e = threadIdx.x; e < E; e += kAggThreads) {
    lkey[e] = kEmpty;
#pragma unroll
    for (int s = 0; s < MS; ++s) lagg[e * MS + s] = s < prog.n_slots ? slot_identity_dev(prog.slot_op[s]) : 0;
  }
  __syncthreads();
  if (blockIdx.x >= chunk_start[nb]) return;  // uniform: grid is an upper bound
  const uint32_t b = sb;
  const uint64_t b0 = pb.off[(uint64_t)b * pp.tiles], b1 = pb.off[(uint64_t)(b + 1) * pp.tiles];
  const uint64_t c = blockIdx.x - sc0;
  const bool exclusive = (sc1 - sc0) == 1;
  const uint64_t r0 = b0 + c * kAggChunk, r1 = r0 + kAggChunk < b1 ? r0 + kAggChunk : b1;
  const uint32_t limit = (uint32_t)(E * 3 / 4);
  const int W = pp.words;
  const int C = W - 2 - pp.has_seq;
  const uint64_t t1 = wall_clock64();
  uint64_t pairs = 0;
  uint32_t fresh = 0, err = 0;
  // KU records (whole, in registers) are loaded per thread before any is processed
  for (uint64_t i0 = r0 + threadIdx.x; i0 < r1; i0 += (uint64_t)kAggThreads * KU) {
    PRec<WMAX> rr[KU];
#pragma unroll
    for (int u = 0; u < KU; ++u) {
      const uint64_t i = i0 + (uint64_t)u * kAggThreads;
      rr[u].C = C;
#pragma unroll
      for (int q = 0; q < WMAX; ++q) rr[u].w[q] = (i < r1 && q < W) ? pb.rec[i * W + q] : 0;
    }
    // one instance of the record body (a rolled loop over a shifting register
    // queue): unrolling it KU times overflowed the instruction cache.
    // Out-of-range records were loaded as zeros (no windows).
#pragma unroll 1
    for (int u = 0; u < KU; ++u) {
    const PRec<WMAX> r = rr[0];
#pragma unroll
    for (int k = 0; k + 1 < KU; ++k) rr[k] = rr[k + 1];
    const uint64_t w0 = r.w[0];
    const uint32_t key = (uint32_t)w0, krel = (uint32_t)(w0 >> 32);
    const uint32_t nw = (uint32_t)r.w[1];
    pairs += nw;
    for (uint32_t j = 0; j < nw; ++j) {
      const uint64_t g = ((uint64_t)key << 32) | (uint64_t)(krel + j);
      uint32_t h = (uint32_t)(mix64(g) & (E - 1));
      int e = -1;
      for (int probe = 0; probe < 32; ++probe) {
        uint64_t cur = lkey[h];
        if (cur == g) { e = (int)h; break; }
        if (cur == kEmpty) {
          if (lfill >= limit) break;  // table nearly full: leave new groups to HBM
          uint64_t old = atomicCAS((unsigned long long *)&lkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
          if (old == kEmpty) {
            atomicAdd(&lfill, 1u);
            e = (int)h;
            break;
          }
          if (old == g) { e = (int)h; break; }
        }
        h = (h + 1) & (E - 1);
      }
      if (e >= 0) {
        lds_apply<MS>(prog, &lagg[e * MS], r);
      } else {
        // overflow: straight to the HBM table
        int64_t slot = tw_find_or_insert(t, g, fresh);
        if (slot < 0) { err |= ERR_OOM; continue; }
        int64_t v[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) v[s] = s < prog.n_slots ? prec_elem(prog, s, r) : 0;
        flush_row(prog, t.aggs + (uint64_t)slot * prog.n_slots, v, false);
        if (atomicExch(&t.stamp[slot], (uint32_t)p.batch_id) != (uint32_t)p.batch_id)
          pb.touched[atomicAdd((unsigned long long *)&sc->scratch[1], 1ull)] = (uint32_t)slot;
      }
    }
    }
  }
  __syncthreads();
  const uint64_t t2 = wall_clock64();
  // flush: one HBM update per group of the chunk. Compact the live entries
  // first so a thread carries about one group; every HBM access of a group is
  // issued before any of its results is needed.
  for (int e = threadIdx.x; e < E; e += kAggThreads)
    if (lkey[e] != kEmpty) llive[atomicAdd(&lnl, 1u)] = (uint16_t)e;
  __syncthreads();
  const uint32_t nl = lnl;
  uint64_t groups = 0;
  for (uint32_t q = threadIdx.x; q < nl; q += kAggThreads) {
    const int e = llive[q];
    const uint64_t g = lkey[e];
    ++groups;
    const uint32_t f0 = fresh;
    const int64_t slot = tw_find_or_insert(t, g, fresh);
    if (slot < 0) { err |= ERR_OOM; continue; }
    int64_t v[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = lagg[e * MS + s];
    int64_t *row = t.aggs + (uint64_t)slot * prog.n_slots;
    bool first;
    if (exclusive && fresh != f0) {
      // inserted just now by the group's only writer: the row holds identities
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < prog.n_slots && prog.slot_op[s] != S_LAST_VAL) row[s] = v[s];
      t.stamp[slot] = (uint32_t)p.batch_id;
      first = true;
    } else if (exclusive) {
      int64_t cur[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) cur[s] = s < prog.n_slots ? row[s] : 0;
      const uint32_t st = t.stamp[slot];
#pragma unroll
      for (int s = 0; s < MS; ++s) {
        if (s >= prog.n_slots) break;
        const int op = prog.slot_op[s];
        if (op == S_LAST_VAL || v[s] == slot_identity_dev(op)) continue;
        row[s] = op == S_LAST_SEQ ? ((uint64_t)v[s] > (uint64_t)cur[s] ? v[s] : cur[s]) : slot_combine(op, cur[s], v[s]);
      }
      first = st != (uint32_t)p.batch_id;
      if (first) t.stamp[slot] = (uint32_t)p.batch_id;
    } else {
      flush_row(prog, row, v, false);
      first = atomicExch(&t.stamp[slot], (uint32_t)p.batch_id) != (uint32_t)p.batch_id;
    }
    // first touch of the group in this batch -> touched list (per-batch changelog)
    if (first) ltouch[atomicAdd(&ltn, 1u)] = (uint32_t)slot;
  }
  __syncthreads();
  const uint64_t t3 = wall_clock64();
  if (threadIdx.x == 0) lbase = ltn ? atomicAdd((unsigned long long *)&sc->scratch[1], (unsigned long long)ltn) : 0;
  __syncthreads();
  for (uint32_t q = threadIdx.x; q < ltn; q += kAggThreads) pb.touched[lbase + q] = ltouch[q];
  pairs = wave_sum_u64(pairs);
  uint64_t fr = wave_sum_u64(fresh);
  groups = wave_sum_u64(groups);
  if ((threadIdx.x & 63) == 0) {
    sred[0][threadIdx.x >> 6] = pairs;
    sred[1][threadIdx.x >> 6] = fr;
    sred[2][threadIdx.x >> 6] = groups;
  }
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a = 0, f = 0, gr = 0;
    for (int k = 0; k < kAggThreads / 64; ++k) {
      a += sred[0][k];
      f += sred[1][k];
      gr += sred[2][k];
    }
    if (a) atomicAdd((unsigned long long *)&sc->pairs, (unsigned long long)a);
    if (f) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)f);
    if (gr) atomicAdd((unsigned long long *)&sc->scratch[0], (unsigned long long)gr);
    // phase clock (100 MHz wall clock) sums: init, records, flush, tail, workgroups
    const uint64_t t4 = wall_clock64();
    atomicAdd((unsigned long long *)&sc->scratch[8], (unsigned long long)(t1 - t0));
    atomicAdd((unsigned long long *)&sc->scratch[9], (unsigned long long)(t2 - t1));
    atomicAdd((unsigned long long *)&sc->scratch[10], (unsigned long long)(t3 - t2));
    atomicAdd((unsigned long long *)&sc->scratch[11], (unsigned long long)(t4 - t3));
    atomicAdd((unsigned long long *)&sc->scratch[12], 1ull);
  }
}

bool part_supported(const Program &prog) { return prog.n_slots <= 8; }

// per-batch changelog: one row per group in the touched list
__global__ __launch_bounds__(256) void k_part_emit(TwTable t, Program prog, TwParams p, PartBuffers pb, OutCols out,
                                                   uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  const uint64_t n = sc->scratch[1];
  const int64_t k_epoch = sc->k_epoch;
  const bool unwin = p.kind == HSG_UNWINDOWED;
  if (blockIdx.x == 0 && threadIdx.x == 0) sc->out_rows = n;
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t o = out_base + q;
    if (o >= out_cap) {
      atomicOr(&sc->err, ERR_OOM);
      break;
    }
    const uint32_t s = pb.touched[q];
    const uint64_t g = t.keys[s];
    const int64_t *row = t.aggs + (uint64_t)s * prog.n_slots;
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
  }
}

void launch_part_emit(hipStream_t s, const TwTable &t, const Program &prog, const TwParams &p, const PartBuffers &pb,
                      OutCols out, uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  hipLaunchKernelGGL(k_part_emit, dim3(2048), dim3(256), 0, s, t, prog, p, pb, out, out_base, out_cap, sc);
}

template <int MS, int E>
static void agg_launch(hipStream_t s, dim3 g, int W, const Program &prog, const TwParams &p, const PartParams &pp,
                       const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  const dim3 th(kAggThreads);
  constexpr int KU4 = MS >= 6 ? 6 : 8;  // records in flight per thread, within 128 VGPRs
  if (W <= 4) hipLaunchKernelGGL((k_part_agg<MS, E, 4, KU4>), g, th, 0, s, prog, p, pp, t, pb, sc);
  else if (W <= 6) hipLaunchKernelGGL((k_part_agg<MS, E, 6, 4>), g, th, 0, s, prog, p, pp, t, pb, sc);
  else hipLaunchKernelGGL((k_part_agg<MS, E, kPartMaxWords, 2>), g, th, 0, s, prog, p, pp, t, pb, sc);
}

bool launch_part_agg(hipStream_t s, const Program &prog, const TwParams &p, const PartParams &pp, const TwTable &t,
                     const PartBuffers &pb, uint64_t n, DevScalars *sc) {
  if (!part_supported(prog)) return false;
  const uint64_t nb = 1ull << pp.np_log2;
  hipLaunchKernelGGL(k_part_chunks, dim3(1), dim3(1024), 0, s, pb.off, pp.tiles, pp.np_log2, pb.chunk_start);
  const dim3 g((unsigned)(nb + n / kAggChunk + 1));
  const int W = pp.words;
  if (prog.n_slots <= 2) agg_launch<2, 2048>(s, g, W, prog, p, pp, t, pb, sc);
  else if (prog.n_slots <= 4) agg_launch<4, 1024>(s, g, W, prog, p, pp, t, pb, sc);
  else if (prog.n_slots <= 6) agg_launch<6, 1024>(s, g, W, prog, p, pp, t, pb, sc);
  else agg_launch<8, 1024>(s, g, W, prog, p, pp, t, pb, sc);
  return true;
}

}  // namespace hsg
