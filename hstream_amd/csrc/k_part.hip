// gfx950 kernels of the partitioned (key, window) aggregation:
//
//   hist     per-tile bucket counts of the records that have >= 1 accepted
//            window (bucket = top bits of hash(key): every window of a key
//            lands in one bucket)
//   scan     bucket-major exclusive prefix -> bucket ranges
//   scatter  partitioned columnar copy: key, first accepted window, window
//            count, values (+ presence, + sequence when LAST is asked for)
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

uint64_t part_tiles(uint64_t n) { return (n + kPartTile - 1) / kPartTile; }

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

// Shared walk over the 4 stream-time sub-tiles of one partition tile.
template <int PASS>
__global__ __launch_bounds__(kPartThreads) void k_part(Batch b, TwParams p, PartParams pp,
                                                       const int64_t *__restrict__ tprefix,
                                                       const int64_t *__restrict__ rec_wm,
                                                       const int64_t *__restrict__ seq, PartBuffers pb,
                                                       DevScalars *sc) {
  __shared__ uint32_t cnt[1 << kPartMaxLog2];
  __shared__ uint64_t sred[2][kPartThreads / 64];
  const int nb = 1 << pp.np_log2;
  for (int i = threadIdx.x; i < nb; i += kPartThreads) cnt[i] = 0;
  __syncthreads();
  const int64_t k_epoch = sc->k_epoch;
  uint64_t late = 0;
  uint32_t err = 0;
  constexpr int kSub = kPartTile / kTileRecords;
  for (int sub = 0; sub < kSub; ++sub) {
    const uint64_t st = (uint64_t)blockIdx.x * kSub + sub;  // stream-time tile
    const uint64_t base = st * kTileRecords;
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
    if (base >= b.n) break;  // uniform across the workgroup
    if (!rec_wm) tile_stream_time(ts, tprefix[st], wm);
#pragma unroll
    for (int r = 0; r < kRecPerThread; ++r) {
      const uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
      uint32_t krel, nwin;
      uint64_t lt = 0;
      if (!part_record(p, k_epoch, key[r], ts[r], wm[r], krel, nwin, lt, err)) {
        late += lt;
        continue;
      }
      late += lt;
      const uint32_t bk = bucket_of(key[r], pp.np_log2);
      if (PASS == 0) {
        atomicAdd(&cnt[bk], 1u);
      } else {
        const uint32_t rank = atomicAdd(&cnt[bk], 1u);
        const uint64_t o = pb.off[(uint64_t)bk * pp.tiles + blockIdx.x] + rank;
        pb.key[o] = key[r];
        pb.krel[o] = krel;
        pb.nwin[o] = nwin;
        for (int c = 0; c < kMaxCols; ++c) {
          if (!b.col[c]) break;
          pb.col[c][o] = b.col[c][i];
          if (pp.has_valid) pb.valid[c][o] = b.valid[c] ? b.valid[c][i] : (uint8_t)1;
        }
        if (pp.has_seq) pb.seq1[o] = (seq ? seq[i] : (int64_t)(p.rec_base + i)) + 1;
      }
    }
  }
  __syncthreads();
  if (PASS == 0) {
    for (int i = threadIdx.x; i < nb; i += kPartThreads) pb.hist[(uint64_t)i * pp.tiles + blockIdx.x] = cnt[i];
    late = wave_sum_u64(late);
    if ((threadIdx.x & 63) == 0) sred[0][threadIdx.x >> 6] = late;
    if (err) atomicOr(&sc->err, err);
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t l = 0;
      for (int k = 0; k < kPartThreads / 64; ++k) l += sred[0][k];
      if (l) atomicAdd((unsigned long long *)&sc->late, (unsigned long long)l);
    }
  }
}

void launch_part_hist(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                      const int64_t *tprefix, const int64_t *rec_wm, const PartBuffers &pb, DevScalars *sc) {
  if (pp.tiles)
    hipLaunchKernelGGL(k_part<0>, dim3((unsigned)pp.tiles), dim3(kPartThreads), 0, s, b, p, pp, tprefix, rec_wm,
                       nullptr, pb, sc);
}
void launch_part_scatter(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                         const int64_t *tprefix, const int64_t *rec_wm, const int64_t *seq, const PartBuffers &pb,
                         DevScalars *sc) {
  if (pp.tiles)
    hipLaunchKernelGGL(k_part<1>, dim3((unsigned)pp.tiles), dim3(kPartThreads), 0, s, b, p, pp, tprefix, rec_wm, seq,
                       pb, sc);
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
__device__ inline void lds_apply(const Program &prog, int64_t *__restrict__ row, const PartBuffers &pb, bool has_valid,
                                 uint64_t i) {
  for (int s = 0; s < prog.n_slots; ++s) {
    const int op = prog.slot_op[s];
    const int c = prog.slot_col[s];
    const bool present = op == S_CNT_ALL || !has_valid || pb.valid[c][i];
    if (!present) continue;
    unsigned long long *u = (unsigned long long *)(row + s);
    switch (op) {
      case S_CNT_ALL:
      case S_CNT: atomicAdd(u, 1ull); break;
      case S_SUM_I: atomicAdd(u, (unsigned long long)pb.col[c][i]); break;
      case S_SUM_F: unsafeAtomicAdd((double *)(row + s), __builtin_bit_cast(double, pb.col[c][i])); break;
      case S_MIN_I: atomicMin((long long *)(row + s), (long long)pb.col[c][i]); break;
      case S_MAX_I: atomicMax((long long *)(row + s), (long long)pb.col[c][i]); break;
      case S_MIN_F: atomicMin(u, (unsigned long long)f64_ord(__builtin_bit_cast(double, pb.col[c][i]))); break;
      case S_MAX_F: atomicMax(u, (unsigned long long)f64_ord(__builtin_bit_cast(double, pb.col[c][i]))); break;
      case S_LAST_SEQ: atomicMax(u, (unsigned long long)pb.seq1[i]); break;
      default: break;
    }
  }
}

// HBM-side combine of a finished LDS row (v) into state row `row`.
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

template <int MS, int E>
__global__ __launch_bounds__(kAggThreads) void k_part_agg(Program prog, TwParams p, PartParams pp, TwTable t,
                                                          PartBuffers pb, const uint32_t *__restrict__ chunk_start,
                                                          DevScalars *sc) {
  __shared__ uint64_t lkey[E];
  __shared__ int64_t lagg[E * MS];
  __shared__ uint32_t lfill;
  __shared__ uint32_t sb, sc0, sc1;
  __shared__ uint64_t sred[3][kAggThreads / 64];
  const int nb = 1 << pp.np_log2;
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
  const bool has_valid = pp.has_valid != 0;
  uint64_t pairs = 0;
  uint32_t fresh = 0, err = 0;
  for (uint64_t i = r0 + threadIdx.x; i < r1; i += kAggThreads) {
    const uint32_t key = pb.key[i];
    const uint32_t krel = pb.krel[i];
    const uint32_t nw = pb.nwin[i];
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
        lds_apply(prog, &lagg[e * MS], pb, has_valid, i);
      } else {
        // overflow: straight to the HBM table
        int64_t slot = tw_find_or_insert(t, g, fresh);
        if (slot < 0) { err |= ERR_OOM; continue; }
        int64_t v[MS];
        identity_row<MS>(prog, v);
#pragma unroll
        for (int s = 0; s < MS; ++s) {
          if (s >= prog.n_slots) break;
          const int op = prog.slot_op[s];
          const int cc = prog.slot_col[s];
          const bool present = op == S_CNT_ALL || !has_valid || pb.valid[cc][i];
          if (!present) continue;
          switch (op) {
            case S_CNT_ALL:
            case S_CNT: v[s] = 1; break;
            case S_SUM_I:
            case S_SUM_F:
            case S_MIN_I:
            case S_MAX_I: v[s] = pb.col[cc][i]; break;
            case S_MIN_F:
            case S_MAX_F: v[s] = (int64_t)f64_ord(__builtin_bit_cast(double, pb.col[cc][i])); break;
            case S_LAST_SEQ: v[s] = pb.seq1[i]; break;
            default: break;
          }
        }
        flush_row(prog, t.aggs + (uint64_t)slot * prog.n_slots, v, false);
        t.stamp[slot] = (uint32_t)p.batch_id;
      }
    }
  }
  __syncthreads();
  // flush: one HBM update per group of the chunk
  uint64_t groups = 0;
  for (int e = threadIdx.x; e < E; e += kAggThreads) {
    const uint64_t g = lkey[e];
    if (g == kEmpty) continue;
    ++groups;
    int64_t slot = tw_find_or_insert(t, g, fresh);
    if (slot < 0) { err |= ERR_OOM; continue; }
    int64_t v[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = lagg[e * MS + s];
    flush_row(prog, t.aggs + (uint64_t)slot * prog.n_slots, v, exclusive);
    t.stamp[slot] = (uint32_t)p.batch_id;
  }
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
  }
}

bool part_supported(const Program &prog) { return prog.n_slots <= 8; }

bool launch_part_agg(hipStream_t s, const Program &prog, const TwParams &p, const PartParams &pp, const TwTable &t,
                     const PartBuffers &pb, uint64_t n, DevScalars *sc) {
  if (!part_supported(prog)) return false;
  const uint64_t nb = 1ull << pp.np_log2;
  uint32_t *chunk_start = pb.chunk_start;
  hipLaunchKernelGGL(k_part_chunks, dim3(1), dim3(1024), 0, s, pb.off, pp.tiles, pp.np_log2, chunk_start);
  const uint64_t grid = nb + n / kAggChunk + 1;
  if (prog.n_slots <= 2)
    hipLaunchKernelGGL((k_part_agg<2, 4096>), dim3((unsigned)grid), dim3(kAggThreads), 0, s, prog, p, pp, t, pb,
                       chunk_start, sc);
  else if (prog.n_slots <= 4)
    hipLaunchKernelGGL((k_part_agg<4, 2048>), dim3((unsigned)grid), dim3(kAggThreads), 0, s, prog, p, pp, t, pb,
                       chunk_start, sc);
  else if (prog.n_slots <= 6)
    hipLaunchKernelGGL((k_part_agg<6, 2048>), dim3((unsigned)grid), dim3(kAggThreads), 0, s, prog, p, pp, t, pb,
                       chunk_start, sc);
  else
    hipLaunchKernelGGL((k_part_agg<8, 1024>), dim3((unsigned)grid), dim3(kAggThreads), 0, s, prog, p, pp, t, pb,
                       chunk_start, sc);
  return true;
}

}  // namespace hsg
