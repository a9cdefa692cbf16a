// gfx950 kernels of the exact per-record changelog of time windows
// (HSG_EMIT_PER_RECORD, EMIT CHANGES) on the partitioned pipeline.
//
// The reference forwards, for every record in arrival order and each of its
// accepted windows in ascending start, the group's aggregate right after that
// record (TimeWindowedStream.hs:89-103). Batch restatement, after the
// partition passes of k_part.hip (records bucket-major by key hash, arrival
// order kept inside a bucket; every window of a key lands in one bucket):
//
//   k_pr_local  one workgroup per chunk of <= kPrPairs (record, window) pairs
//               of one bucket: groups into an LDS hash table, a stable LDS
//               radix sort of the pairs by table slot (arrival order kept per
//               group), a segmented inclusive scan = each pair's prefix over
//               the chunk. Each pair's prefix goes to its bucket-major pair
//               position, each group's chunk total to a compact partial list.
//   k_pr_carry  one workgroup per bucket, its chunks in order: each partial's
//               group is claimed / found in the HBM table; the row before the
//               chunk is the partial's carry (written over the total), the row
//               plus the total the group's state after it.
//   k_pr_emit   one workgroup per arrival tile: each record's windows again
//               (the partition's own window run), the pairs' output positions
//               (exclusive prefix of accepted windows in arrival order), and
//               row = carry (+) prefix for every pair, written in arrival order
//               (coalesced: consecutive records, consecutive rows).
//
// The order-dependent parts are exact: a group's prefix follows its records in
// arrival order inside a chunk, chunks of a bucket are applied in bucket (=
// arrival) order, LAST keeps the latest present record (combine_row).
#include "hsg_dev.h"
#include "hsg_part.h"
#include "hsg_perrecord.h"
#include "hsg_tw.h"

namespace hsg {

constexpr int kPrNT = 1024;              // threads of k_pr_local
constexpr int kPrNW = kPrNT / 64;        // its waves
constexpr int kPrTab = 4096;             // LDS table slots (>= 2 x pairs)
constexpr int kPrTabLog2 = 12;
static_assert(kPrPairs * 2 <= kPrTab && kPrPairs == 2 * kPrNT, "k_pr_local sizes");

// chunk of this workgroup: records [r0, r1) of bucket b; false past the chunks
__device__ inline bool pr_chunk(const PartParams &pp, const PartBuffers &pb, uint32_t &b, uint64_t &r0, uint64_t &r1) {
  const int nb = 1 << pp.np_log2;
  if (blockIdx.x >= pb.chunk_start[nb]) return false;
  b = pb.chunk_bucket[blockIdx.x];
  const uint32_t c0 = pb.chunk_start[b];
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  r0 = b0 + (uint64_t)(blockIdx.x - c0) * pp.chunk;
  r1 = r0 + pp.chunk < b1 ? r0 + pp.chunk : b1;
  return true;
}

// A partitioned record in memory (hsg_part.h layouts), runtime word count.
struct PrRecView {
  const uint64_t *w;
  bool pk;
  int C;
  __device__ uint32_t key() const { return (uint32_t)w[0]; }
  __device__ uint32_t krel(uint32_t kbase) const {
    return pk ? kbase + (uint32_t)((w[0] >> 32) & 0xFFFFull) : (uint32_t)(w[0] >> 32);
  }
  __device__ uint32_t nwin() const { return pk ? (uint32_t)((w[0] >> 48) & 0xFFull) : (uint32_t)w[1]; }
  __device__ bool present(int c) const { return pk ? (w[0] >> (56 + c)) & 1ull : (w[1] >> (32 + c)) & 1ull; }
  __device__ int64_t col(int c) const { return (int64_t)w[(pk ? 1 : 2) + c]; }
  __device__ int64_t seq1() const { return (int64_t)w[(pk ? 1 : 2) + C]; }
};

// contribution of the record to every slot (identity when the field is absent)
template <int MS>
__device__ inline void pr_elems(const Program &prog, const PrRecView &r, int64_t (&e)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    e[s] = 0;
    if (s >= prog.n_slots) continue;
    const int op = prog.slot_op[s], c = prog.slot_col[s];
    if (op == S_CNT_ALL) {
      e[s] = 1;
      continue;
    }
    const bool pr = r.present(c);
    if (op == S_LAST_VAL) {
      e[s] = pr ? r.col(c) : 0;
      continue;
    }
    if (!pr) {
      e[s] = slot_identity_dev(op);
      continue;
    }
    switch (op) {
      case S_CNT: e[s] = 1; break;
      case S_SUM_I:
      case S_SUM_F:
      case S_MIN_I:
      case S_MAX_I: e[s] = r.col(c); break;
      case S_MIN_F:
      case S_MAX_F: e[s] = (int64_t)f64_ord(__builtin_bit_cast(double, r.col(c))); break;
      case S_LAST_SEQ: e[s] = r.seq1(); break;
      default: break;
    }
  }
}

// (hf, v) <- (hf_u, v_u) (+) (hf, v), u earlier: segmented combine
template <int MS>
__device__ inline void pr_seg_earlier(const Program &prog, bool &hf, int64_t (&v)[MS], bool hf_u,
                                      const int64_t (&v_u)[MS]) {
  if (!hf) {
    int64_t t[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) t[s] = v_u[s];
    combine_row<MS>(prog, t, v);
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = t[s];
  }
  hf = hf || hf_u;
}

__device__ inline uint32_t pr_home(uint32_t key, uint32_t w) {
  uint32_t h = key * 0x9E3779B1u + w * 0x85EBCA77u;
  h ^= (h >> 16) * 0x7FEB352Du;
  return h >> (32 - kPrTabLog2);
}

// block-wide exclusive sum of one u32 per thread (kPrNT threads); *total = sum
__device__ inline uint32_t pr_block_excl(uint32_t v, uint32_t *sw, uint32_t &total) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)v);
  if (lane == 63) sw[w] = incl;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (int k = 0; k < kPrNW; ++k) {
    before += k < w ? sw[k] : 0u;
    total += sw[k];
  }
  __syncthreads();
  return before + incl - v;
}

template <int MS>
__global__ __launch_bounds__(kPrNT) void k_pr_local(Program prog, PartParams pp, PartBuffers pb, PrPart pr,
                                                    uint32_t wpr, DevScalars *sc) {
  __shared__ uint64_t lkey[kPrTab];
  __shared__ uint32_t sa[kPrPairs], sb[kPrPairs];  // slot << 16 | pair, sort ping-pong
  __shared__ uint32_t prp[kPrPairs];               // pair -> chunk record << 8 | window offset
  __shared__ uint32_t dcnt[kPrNW][64];             // radix digit counts per wave
  __shared__ uint32_t sw[kPrNW];
  __shared__ int64_t swv[kPrNW][MS];
  __shared__ uint32_t swf[kPrNW], swh[kPrNW];
  __shared__ uint32_t s_cbase;
  if (sc->redo) return;  // uniform: the optimistic pass found late records (bucket starts are stale)
  uint32_t b;
  uint64_t r0, r1;
  if (!pr_chunk(pp, pb, b, r0, r1)) return;  // uniform
  const bool pk = sc->packed != 0;
  const int W = pk ? pp.words - 1 : pp.words;
  const int C = pp.words - 2 - pp.has_seq;
  const uint32_t kbase = (uint32_t)sc->kbase;
  const uint32_t nrec = (uint32_t)(r1 - r0);  // <= kPrPairs / wpr
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ns = prog.n_slots;
  for (int k = threadIdx.x; k < kPrTab; k += kPrNT) lkey[k] = kEmpty;

  // 1) records 2t, 2t + 1 of the chunk: window runs, pair offsets
  uint32_t nw[2] = {0, 0}, key[2] = {0, 0}, kr[2] = {0, 0};
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t r = 2 * threadIdx.x + k;
    if (r < nrec) {
      const PrRecView v{pb.rec + (r0 + r) * (uint64_t)W, pk, C};
      key[k] = v.key();
      kr[k] = v.krel(kbase);
      nw[k] = v.nwin();
    }
  }
  uint32_t P;
  const uint32_t pbase = pr_block_excl(nw[0] + nw[1], sw, P);  // (barrier inside: the table clear is seen)
  // 2) groups into the LDS table; pair p = (slot << 16 | p) for the sort
  uint32_t p = pbase;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    for (uint32_t j = 0; j < nw[k]; ++j, ++p) {
      const uint32_t kw = kr[k] + j;
      const uint64_t g = ((uint64_t)key[k] << 32) | kw;
      uint32_t h = pr_home(key[k], kw);
      for (;;) {  // the table holds <= half its slots: every probe sequence ends
        const uint64_t c = lkey[h];
        if (c == g) break;
        if (c == kEmpty) {
          const uint64_t old =
              atomicCAS((unsigned long long *)&lkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
          if (old == kEmpty || old == g) break;
        }
        h = (h + 1) & (kPrTab - 1);
      }
      sa[p] = (h << 16) | p;
      prp[p] = ((2 * threadIdx.x + k) << 8) | j;
    }
  }
  __syncthreads();

  // 3) stable LSD radix sort of the pairs by slot (two 6-bit digits). Wave w
  // ranks positions [w * 128, w * 128 + 128) in two rounds of 64 lanes, so
  // equal digits keep their order; digit-major, wave-minor offsets.
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t *src = sa, *dst = sb;
#pragma unroll 1
  for (int pass = 0; pass < 2; ++pass) {
    const int shift = 16 + 6 * pass;
    for (int k = threadIdx.x; k < kPrNW * 64; k += kPrNT) (&dcnt[0][0])[k] = 0;
    __syncthreads();
    uint32_t val[2], dig[2], rank[2];
#pragma unroll
    for (int rd = 0; rd < 2; ++rd) {
      const uint32_t q = wv * 128 + rd * 64 + lane;
      const bool ok = q < P;
      val[rd] = ok ? src[q] : 0u;
      dig[rd] = ok ? (val[rd] >> shift) & 63u : 64u;
      uint64_t m = __ballot(ok);
#pragma unroll
      for (int bit = 0; bit < 6; ++bit) {
        const bool x = (dig[rd] >> bit) & 1u;
        const uint64_t bb = __ballot(x);
        m &= x ? bb : ~bb;
      }
      const uint32_t before = ok ? dcnt[wv][dig[rd]] : 0u;
      rank[rd] = before + (uint32_t)__popcll(m & lt);
      // the group's highest lane moves the wave's count past the group
      if (ok && (m >> lane) == 1ull) dcnt[wv][dig[rd]] = before + (uint32_t)__popcll(m);
    }
    __syncthreads();
    // offsets: digit-major, wave-minor (1024 counters, one per thread)
    const int d = threadIdx.x / kPrNW, ww = threadIdx.x % kPrNW;
    uint32_t tot;
    const uint32_t off = pr_block_excl(dcnt[ww][d], sw, tot);
    dcnt[ww][d] = off;
    __syncthreads();
#pragma unroll
    for (int rd = 0; rd < 2; ++rd)
      if (dig[rd] < 64u) dst[dcnt[wv][dig[rd]] + rank[rd]] = val[rd];
    __syncthreads();
    uint32_t *t = src;
    src = dst;
    dst = t;
  }
  const uint32_t *sorted = src;

  // 4) segmented inclusive scan in sorted order, thread t: positions 2t, 2t+1
  int64_t e[2][MS];
  bool hd[2];
  uint32_t nh = 0;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t q = 2 * threadIdx.x + k;
    hd[k] = false;
    if (q < P) {
      const uint32_t v = sorted[q];
      hd[k] = q == 0 || (sorted[q - 1] >> 16) != (v >> 16);
      const uint32_t rr = prp[v & 0xFFFFu] >> 8;
      const PrRecView rv{pb.rec + (r0 + rr) * (uint64_t)W, pk, C};
      pr_elems<MS>(prog, rv, e[k]);
    } else {
      identity_row<MS>(prog, e[k]);
    }
    nh += hd[k] ? 1u : 0u;
  }
  // thread aggregate (hf, v): its two elements combined
  bool hf = hd[0] || hd[1];
  int64_t tv[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) tv[s] = e[0][s];
  if (hd[1]) {
#pragma unroll
    for (int s = 0; s < MS; ++s) tv[s] = e[1][s];
  } else {
    combine_row<MS>(prog, tv, e[1]);
  }
  // wave inclusive segmented scan of (hf, tv), plus the head counts
  bool ihf = hf;
  int64_t iv[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) iv[s] = tv[s];
  uint32_t ih = nh;
#pragma unroll
  for (int dd = 1; dd < 64; dd <<= 1) {
    const bool uf = __shfl_up((int)ihf, dd, 64) != 0;
    int64_t uv[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) uv[s] = __shfl_up(iv[s], dd, 64);
    const uint32_t uh = __shfl_up(ih, dd, 64);
    if (lane >= dd) {
      pr_seg_earlier<MS>(prog, ihf, iv, uf, uv);
      ih += uh;
    }
  }
  if (lane == 63) {
    swf[wv] = ihf;
    swh[wv] = ih;
#pragma unroll
    for (int s = 0; s < MS; ++s) swv[wv][s] = iv[s];
  }
  // exclusive within the wave
  bool xf = __shfl_up((int)ihf, 1, 64) != 0;
  int64_t xv[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) xv[s] = __shfl_up(iv[s], 1, 64);
  uint32_t xh = __shfl_up(ih, 1, 64);
  __syncthreads();
  // prefix of the earlier waves
  bool pf = false;
  int64_t pv[MS];
  identity_row<MS>(prog, pv);
  uint32_t ph = 0, heads = 0;
  for (int k = 0; k < kPrNW; ++k) {
    if (k < wv) {
      int64_t wv2[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) wv2[s] = swv[k][s];
      bool wf = swf[k] != 0;
      pr_seg_earlier<MS>(prog, wf, wv2, pf, pv);
      pf = wf;
#pragma unroll
      for (int s = 0; s < MS; ++s) pv[s] = wv2[s];
      ph += swh[k];
    }
    heads += swh[k];
  }
  if (lane == 0) {
    xf = pf;
#pragma unroll
    for (int s = 0; s < MS; ++s) xv[s] = pv[s];
    xh = ph;
  } else {
    pr_seg_earlier<MS>(prog, xf, xv, pf, pv);
    xh += ph;
  }
  // the chunk's partials: one per group (head), allocated in one atomic
  if (threadIdx.x == 0) {
    const uint32_t base = (uint32_t)atomicAdd((unsigned long long *)pr.counter, (unsigned long long)heads);
    s_cbase = base;
    pr.cbase[blockIdx.x] = base;
    pr.ccnt[blockIdx.x] = heads;
  }
  __syncthreads();
  const uint32_t cbase = s_cbase;
  // 5) each pair's inclusive prefix at its bucket-major pair position; each
  // group's last prefix (its chunk total) and key as the partial
  int64_t run[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) run[s] = xv[s];
  uint32_t ent = xh;  // heads before this thread's first position
  const uint64_t rw = 1 + (uint64_t)ns;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const uint32_t q = 2 * threadIdx.x + k;
    if (q >= P) break;
    if (hd[k]) {
#pragma unroll
      for (int s = 0; s < MS; ++s) run[s] = e[k][s];
      ent += 1;
    } else {
      combine_row<MS>(prog, run, e[k]);
    }
    const uint32_t v = sorted[q];
    const uint32_t pp2 = prp[v & 0xFFFFu];
    const uint64_t gp = (r0 + (pp2 >> 8)) * (uint64_t)wpr + (pp2 & 0xFFu);
    const uint32_t gi = cbase + ent - 1;
    uint64_t *o = pr.inter + gp * rw;
    o[0] = gi;
#pragma unroll
    for (int s = 0; s < MS; ++s)
      if (s < ns) o[1 + s] = (uint64_t)run[s];
    const bool tail = q + 1 == P || (sorted[q + 1] >> 16) != (v >> 16);
    if (tail) {
      pr.gkey[gi] = lkey[v >> 16];
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < ns) pr.part[(uint64_t)gi * ns + s] = run[s];
    }
  }
}

// One workgroup per bucket, its chunks in order: claim / find each partial's
// group, carry = the row before the chunk, row = carry (+) chunk total. Only
// this workgroup updates these groups in the batch (a key's groups are all in
// its bucket): plain read-modify-write; the next chunk may update the same
// groups, hence agent-scope loads and a fence + barrier between chunks.
template <int MS>
__global__ __launch_bounds__(256) void k_pr_carry(Program prog, TwParams p, PartParams pp, TwTable t, PartBuffers pb,
                                                  PrPart pr, DevScalars *sc) {
  __shared__ uint64_t s_red[4], s_tch[4];
  if (sc->redo) return;  // uniform
  const uint32_t b = blockIdx.x;
  const uint32_t c0 = pb.chunk_start[b], c1 = pb.chunk_start[b + 1];
  const int ns = prog.n_slots;
  const uint32_t bid = (uint32_t)p.batch_id;
  uint32_t fresh = 0, err = 0;
  uint64_t touched = 0;
  for (uint32_t c = c0; c < c1; ++c) {
    const uint32_t base = pr.cbase[c], cnt = pr.ccnt[c];
    for (uint32_t e = threadIdx.x; e < cnt; e += 256) {
      const uint32_t gi = base + e;
      const uint64_t g = pr.gkey[gi];
      int64_t tot[MS], cur[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) tot[s] = s < ns ? pr.part[(uint64_t)gi * ns + s] : 0;
      // find or claim (agent-scope loads: an earlier chunk of this workgroup may have claimed it)
      const uint64_t rb = tw_region_base(t, g);
      uint64_t sl = tw_home_in(t, g);
      const uint64_t step = tw_step(t), np = (t.rmask + 1) / step;
      int64_t slot = -1;
      bool isnew = false;
      for (uint64_t probe = 0; probe < np && probe < kMaxProbes; ++probe) {
        uint64_t *kp = t.key(rb + sl);
        const uint64_t k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (k == g) {
          slot = (int64_t)(rb + sl);
          break;
        }
        if (k == kEmpty) {
          const uint64_t old = atomicCAS((unsigned long long *)kp, (unsigned long long)kEmpty, (unsigned long long)g);
          if (old == kEmpty) {
            t.mark(rb + sl);
            fresh += 1;
            isnew = true;
            slot = (int64_t)(rb + sl);
            break;
          }
          if (old == g) {
            slot = (int64_t)(rb + sl);
            break;
          }
        }
        sl = (sl + step) & t.rmask;
      }
      if (slot < 0) {
        err |= ERR_OOM;
        identity_row<MS>(prog, cur);
      } else {
        int64_t *row = t.aggs(slot);
        uint32_t *stp = t.stamp(slot);
        if (isnew) {
          identity_row<MS>(prog, cur);
        } else {
#pragma unroll
          for (int s = 0; s < MS; ++s)
            cur[s] = s < ns ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        }
        const uint32_t st = isnew ? 0u : __hip_atomic_load(stp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        int64_t nv[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) nv[s] = cur[s];
        combine_row<MS>(prog, nv, tot);
#pragma unroll
        for (int s = 0; s < MS; ++s)
          if (s < ns) row[s] = nv[s];
        if (st != bid) {
          *stp = bid;
          touched += 1;
        }
      }
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < ns) pr.part[(uint64_t)gi * ns + s] = cur[s];
    }
    __threadfence();  // this chunk's rows at the device before the next chunk reads them
    __syncthreads();
  }
  if (err) atomicOr(&sc->err, err);
  const uint64_t f = wave_sum_u64(fresh), tc = wave_sum_u64(touched);
  if ((threadIdx.x & 63) == 0) {
    s_red[threadIdx.x >> 6] = f;
    s_tch[threadIdx.x >> 6] = tc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t ff = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    const uint64_t tt = s_tch[0] + s_tch[1] + s_tch[2] + s_tch[3];
    if (ff) atomicAdd((unsigned long long *)&sc->live_x[blockIdx.x & 7], (unsigned long long)ff);
    if (tt) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tt);
  }
}

// One workgroup per kPrEmitRecs arrival-order records (kPrEmitThreads threads,
// consecutive records per thread): window runs as the partition computed
// them, output positions, rows.
constexpr int kPrEmitThreads = 1024;
constexpr int kPrEmitPer = kPrEmitRecs / kPrEmitThreads;
static_assert(kPrEmitRecs % kPartTileRecs == 0 && kPrEmitPer * kPrEmitThreads == kPrEmitRecs, "emit tile");

template <int MS>
__global__ __launch_bounds__(kPrEmitThreads) void k_pr_emit(Batch bt, Program prog, TwParams p, PartParams pp,
                                                            PartBuffers pb, PrPart pr, uint32_t wpr,
                                                            const int64_t *__restrict__ rec_wm,
                                                            const int64_t *__restrict__ seq, OutCols out,
                                                            uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  __shared__ uint32_t sw[kPrEmitThreads / 64];
  if (sc->redo) return;  // uniform
  const uint64_t i0 = (uint64_t)blockIdx.x * kPrEmitRecs + (uint64_t)threadIdx.x * kPrEmitPer;
  const int64_t k_epoch = sc->k_epoch;
  const int64_t *wm = rec_wm ? rec_wm : (sc->no_late ? nullptr : pb.wm);
  uint32_t krel[kPrEmitPer], nwin[kPrEmitPer], key[kPrEmitPer];
  uint64_t late = 0;
  uint32_t err = 0, mine = 0;
#pragma unroll
  for (int r = 0; r < kPrEmitPer; ++r) {
    const uint64_t i = i0 + r;
    nwin[r] = 0;
    key[r] = HSG_KEY_NONE;
    if (i >= bt.n) continue;
    key[r] = bt.key[i];
    const int64_t ts = bt.ts[i];
    uint32_t a = 0, n = 0;
    // same window run as the partition passes (k_part.hip part_record)
    if (key[r] != HSG_KEY_NONE) {
      uint64_t k_lo, k_hi;
      if (record_windows(p, ts, k_lo, k_hi)) {
        const int64_t w = wm ? wm[i] : INT64_MIN;
        uint64_t k = k_lo;
        while (k <= k_hi && !window_accepted(p, k, w)) ++k;
        if (k <= k_hi) {
          int64_t lo = (int64_t)k - k_epoch, hi = (int64_t)k_hi - k_epoch;
          if (lo < 0) lo = 0;
          if (hi > 0xFFFFFFFFll) hi = 0xFFFFFFFFll;
          if (lo <= hi) {
            a = (uint32_t)lo;
            n = (uint32_t)(hi - lo + 1);
          }
        }
      }
    }
    krel[r] = a;
    nwin[r] = n;
    mine += n;
  }
  // exclusive prefix of the pairs in arrival order: the tiles before this one
  // (histogram pair counts, scanned) + the threads before this one
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)mine);
  if (lane == 63) sw[wv] = incl;
  __syncthreads();
  uint64_t o = pr.tpoff[(uint64_t)blockIdx.x * (kPrEmitRecs / kPartTileRecs)] + incl - mine;
  for (int k = 0; k < wv; ++k) o += sw[k];
  const uint64_t rw = 1 + (uint64_t)prog.n_slots;
  const int ns = prog.n_slots;
#pragma unroll
  for (int r = 0; r < kPrEmitPer; ++r) {
    if (!nwin[r]) continue;
    const uint64_t i = i0 + r;
    const uint64_t pos = pr.pos[i];
    const int64_t src = seq ? seq[i] : (int64_t)(p.rec_base + i);
    if (pos >= pb.n_cap) {  // cannot happen: the scatter placed every record with a window
      err |= ERR_OOM;
      o += nwin[r];
      continue;
    }
    for (uint32_t j = 0; j < nwin[r]; ++j, ++o) {
      const uint64_t *it = pr.inter + (pos * wpr + j) * rw;
      const uint32_t gi = (uint32_t)it[0];
      if ((uint64_t)gi >= pb.n_cap * wpr) {
        err |= ERR_OOM;
        continue;
      }
      int64_t R[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) R[s] = s < ns ? pr.part[(uint64_t)gi * ns + s] : 0;
      int64_t L[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) L[s] = s < ns ? (int64_t)it[1 + s] : 0;
      combine_row<MS>(prog, R, L);
      const uint64_t ob = out_base + o;
      if (ob >= out_cap) {
        err |= ERR_OOM;
        continue;
      }
      out.key[ob] = key[r];
      int64_t ws = 0, we = 0;
      if (p.kind != HSG_UNWINDOWED) {
        const int64_t k = k_epoch + (int64_t)(krel[r] + j);
        ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
        we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
      }
      out.ws[ob] = ws;
      out.we[ob] = we;
      out.src[ob] = src;
      for (int jj = 0; jj < prog.n_out; ++jj) out.agg[jj][ob] = out_value_reg<MS>(prog, jj, R);
    }
  }
  if (err) atomicOr(&sc->err, err);
}

template <int MS>
static void pr_launch(hipStream_t s, const Batch &b, const Program &prog, const TwParams &p, const PartParams &pp,
                      const TwTable &t, const PartBuffers &pb, const PrPart &pr, uint32_t wpr, const int64_t *rec_wm,
                      const int64_t *seq, const OutCols &out, uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  const uint64_t nb = 1ull << pp.np_log2;
  const dim3 g((unsigned)(nb + b.n / pp.chunk + 1));
  hipLaunchKernelGGL(k_pr_local<MS>, g, dim3(kPrNT), 0, s, prog, pp, pb, pr, wpr, sc);
  hipLaunchKernelGGL(k_pr_carry<MS>, dim3((unsigned)nb), dim3(256), 0, s, prog, p, pp, t, pb, pr, sc);
  const uint64_t tiles = (b.n + kPrEmitRecs - 1) / kPrEmitRecs;
  hipLaunchKernelGGL(k_pr_emit<MS>, dim3((unsigned)tiles), dim3(kPrEmitThreads), 0, s, b, prog, p, pp, pb, pr, wpr,
                     rec_wm, seq, out, out_base, out_cap, sc);
}

void launch_pr_part(hipStream_t s, const Batch &b, const Program &prog, const TwParams &p, const PartParams &pp,
                    const TwTable &t, const PartBuffers &pb, const PrPart &pr, uint32_t wpr, const int64_t *rec_wm,
                    const int64_t *seq, const OutCols &out, uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  if (!b.n) return;
  if (prog.n_slots <= 2) pr_launch<2>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
  else if (prog.n_slots <= 4) pr_launch<4>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
  else pr_launch<8>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
}

}  // namespace hsg
