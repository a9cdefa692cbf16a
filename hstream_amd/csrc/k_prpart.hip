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
#include "hsg_agg.h"
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
__device__ inline bool pr_chunk(const PartParams &pp, const PartBuffers &pb, uint32_t cid, uint32_t &b, uint64_t &r0,
                                uint64_t &r1) {
  const int nb = 1 << pp.np_log2;
  if (cid >= pb.chunk_start[nb]) return false;
  b = pb.chunk_bucket[cid];
  const uint32_t c0 = pb.chunk_start[b];
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  r0 = b0 + (uint64_t)(cid - c0) * pp.chunk;
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
  // the sequence word (hsg_dev.h seq_word): seq + 1, decimal-literal bits
  __device__ int64_t seq1() const { return (int64_t)(w[(pk ? 1 : 2) + C] & kSeqMask); }
  __device__ bool dec(int c) const { return (w[(pk ? 1 : 2) + C] >> (56 + c)) & 1ull; }
};

// contribution of the record to every slot (identity when the field is absent)
template <int MS, class RV>
__device__ inline void pr_elems(const Program &prog, const RV &r, int64_t (&e)[MS]) {
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
      case S_CNT_DEC: e[s] = r.dec(c) ? 1 : 0; break;
      case S_TIE_MIN:
      case S_TIE_MAX:
      case S_LAST_FORM: e[s] = (int64_t)(((uint64_t)r.seq1() << 1) | (r.dec(c) ? 0u : 1u)); break;
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

// Multi-window ops: each bucket's records regrouped by key, arrival order kept
// within a key (a stable LSD radix sort on 12 key-hash bits below the bucket
// bits, two 6-bit digits). k_pr_keys then replays a key's records from one
// contiguous run. A bucket of up to kKsMax records sorts in LDS; up to
// kKsBig in global scratch (the roff buffer, written only later by
// k_pr_offs: record indices only, each digit recomputed from the record's
// key); a larger bucket (a very hot key) is copied as it is and sets
// pr.counter[1]: the batch then takes the chunked path, whose chunks also
// read the key-grouped records. kpos maps each partitioned position to its
// place in krec.
constexpr int kKsMax = 16384;  // records a workgroup sorts in LDS (2 x 64 KB)
constexpr int kKsBig = 65536;  // records it sorts in global scratch
// the 12 key-hash bits below the bucket bits (hs = bshift + np_log2)
__device__ inline uint32_t ks_digits(uint32_t key, int hs) { return (uint32_t)((key_hash(key) << hs) >> (64 - 12)); }

// one stable LSD pass over m entries src -> dst (6-bit digit `dig(v)`): wave w
// ranks positions [w * RW, (w + 1) * RW) in rounds of 64 lanes, digit-major
// wave-minor offsets (as k_pr_local)
template <class D>
__device__ inline void ks_pass(const uint32_t *src, uint32_t *dst, uint32_t m, D dig, uint32_t (&dcnt)[kPrNW][64],
                               uint32_t *sw) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t lt = (1ull << lane) - 1ull;
  const uint32_t RW = (m + kPrNW - 1) / kPrNW;
  for (int k = threadIdx.x; k < kPrNW * 64; k += kPrNT) (&dcnt[0][0])[k] = 0;
  __syncthreads();
  for (uint32_t q0 = 0; q0 < RW; q0 += 64) {  // count (wave-local, in order)
    const uint32_t q = wv * RW + q0 + lane;
    const bool ok = q0 + lane < RW && q < m;
    const uint32_t d = ok ? dig(src[q]) : 64u;
    uint64_t mm = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) {
      const bool x = (d >> bit) & 1u;
      const uint64_t bb = __ballot(x);
      mm &= x ? bb : ~bb;
    }
    if (ok && (mm >> lane) == 1ull) dcnt[wv][d] += (uint32_t)__popcll(mm);
  }
  __syncthreads();
  const int dd = threadIdx.x / kPrNW, ww = threadIdx.x % kPrNW;
  uint32_t tot;
  const uint32_t off = pr_block_excl(dcnt[ww][dd], sw, tot);
  dcnt[ww][dd] = off;
  __syncthreads();
  for (uint32_t q0 = 0; q0 < RW; q0 += 64) {  // place (the same order: stable)
    const uint32_t q = wv * RW + q0 + lane;
    const bool ok = q0 + lane < RW && q < m;
    const uint32_t v = ok ? src[q] : 0u;
    const uint32_t d = ok ? dig(v) : 64u;
    uint64_t mm = __ballot(ok);
#pragma unroll
    for (int bit = 0; bit < 6; ++bit) {
      const bool x = (d >> bit) & 1u;
      const uint64_t bb = __ballot(x);
      mm &= x ? bb : ~bb;
    }
    const uint32_t before = ok ? dcnt[wv][d] : 0u;
    if (ok) dst[before + (uint32_t)__popcll(mm & lt)] = v;
    if (ok && (mm >> lane) == 1ull) dcnt[wv][d] = before + (uint32_t)__popcll(mm);
  }
  __syncthreads();
}

__global__ __launch_bounds__(kPrNT) void k_pr_keysort(PartParams pp, PartBuffers pb, PrPart pr, DevScalars *sc) {
  __shared__ uint32_t ka[kKsMax], kb[kKsMax];  // hash digits << 16 | record (bucket-relative)
  __shared__ uint32_t dcnt[kPrNW][64];
  __shared__ uint32_t sw[kPrNW];
  if (sc->redo) return;  // uniform
  const uint32_t b = blockIdx.x;
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  const uint32_t m = (uint32_t)(b1 - b0);
  const int W = sc->packed ? pp.words - 1 : pp.words;
  const int hs = pp.bshift + pp.np_log2;
  const uint64_t *rec = pb.rec + b0 * (uint64_t)W;
  if (m > (uint32_t)kKsBig) {  // uniform: copied in partition order, and the batch takes the chunked path
    if (threadIdx.x == 0) __hip_atomic_store(&pr.counter[1], 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (uint64_t w = threadIdx.x; w < (uint64_t)m * W; w += kPrNT) pr.krec[b0 * W + w] = rec[w];
    for (uint32_t r = threadIdx.x; r < m; r += kPrNT) pr.kpos[b0 + r] = (uint32_t)(b0 + r);
    return;
  }
  const uint32_t *order;  // bucket-relative record of each sorted position
  uint32_t omask;
  if (m <= (uint32_t)kKsMax) {  // uniform
    for (uint32_t r = threadIdx.x; r < m; r += kPrNT) ka[r] = (ks_digits((uint32_t)rec[(uint64_t)r * W], hs) << 16) | r;
    __syncthreads();
    ks_pass(ka, kb, m, [](uint32_t v) { return (v >> 16) & 63u; }, dcnt, sw);
    ks_pass(kb, ka, m, [](uint32_t v) { return (v >> 22) & 63u; }, dcnt, sw);
    order = ka;
    omask = 0xFFFFu;
  } else {
    uint32_t *ga = reinterpret_cast<uint32_t *>(pr.roff) + b0, *gb = ga + pb.n_cap;
    for (uint32_t r = threadIdx.x; r < m; r += kPrNT) ga[r] = r;
    __syncthreads();
    ks_pass(ga, gb, m, [&](uint32_t r) { return ks_digits((uint32_t)rec[(uint64_t)r * W], hs) & 63u; }, dcnt, sw);
    ks_pass(gb, ga, m, [&](uint32_t r) { return (ks_digits((uint32_t)rec[(uint64_t)r * W], hs) >> 6) & 63u; }, dcnt,
            sw);
    order = ga;
    omask = 0xFFFFFFFFu;
  }
  // records to their key-grouped places, and the position map
  for (uint32_t q = threadIdx.x; q < m; q += kPrNT) pr.kpos[b0 + (order[q] & omask)] = (uint32_t)(b0 + q);
  for (uint64_t w = threadIdx.x; w < (uint64_t)m * W; w += kPrNT) {
    const uint32_t q = (uint32_t)(w / W), k = (uint32_t)(w - (uint64_t)q * W);
    pr.krec[(b0 + q) * W + k] = rec[(uint64_t)(order[q] & omask) * W + k];
  }
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
  if (sc->redo || !pr.counter[1]) return;  // uniform: stale bucket starts / the batch takes k_pr_keys
  // grid-stride over the chunks (the grid is capped: a batch that takes
  // k_pr_keys launches this kernel for nothing)
  for (uint32_t cid = blockIdx.x;; cid += gridDim.x) {
  uint32_t b;
  uint64_t r0, r1;
  if (!pr_chunk(pp, pb, cid, b, r0, r1)) break;  // uniform
  uint64_t ck = phase_clock(), c_rec = 0, c_ins = 0, c_sort = 0, c_scan = 0;
  auto lap = [&](uint64_t &acc) {
    if constexpr (kPhaseClocks) {
      const uint64_t c = phase_clock();
      acc += c - ck;
      ck = c;
    }
  };
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
  lap(c_rec);
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
  lap(c_ins);

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
  lap(c_sort);

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
  // the chunk's partials: one per group (head), at the chunk's own pair
  // range (partials <= pairs; chunks' record ranges are disjoint), so no
  // chunk waits on a shared counter (one device-scope atomic per chunk on a
  // single word serialised ~100K chunks per C3 batch)
  if (threadIdx.x == 0) {
    const uint32_t base = (uint32_t)(r0 * wpr);
    s_cbase = base;
    pr.cbase[cid] = base;
    pr.ccnt[cid] = heads;
  }
  __syncthreads();
  lap(c_scan);
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
  if (kPhaseClocks) {  // phase clocks (100 MHz), PHASES=1 builds with HSG_PHASES set
    __syncthreads();
    uint64_t c_out = 0;
    lap(c_out);
    if (threadIdx.x == 0) {
      atomicAdd((unsigned long long *)&sc->scratch[24], (unsigned long long)c_rec);
      atomicAdd((unsigned long long *)&sc->scratch[25], (unsigned long long)c_ins);
      atomicAdd((unsigned long long *)&sc->scratch[26], (unsigned long long)c_sort);
      atomicAdd((unsigned long long *)&sc->scratch[27], (unsigned long long)c_scan);
      atomicAdd((unsigned long long *)&sc->scratch[28], (unsigned long long)c_out);
      atomicAdd((unsigned long long *)&sc->scratch[29], 0ull);
      atomicAdd((unsigned long long *)&sc->scratch[30], 1ull);
    }
  }
  __syncthreads();  // the LDS table and sort arrays are reused by the next chunk
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
  if (sc->redo || !pr.counter[1]) return;  // uniform
  const uint32_t b = blockIdx.x;
  const uint32_t c0 = pb.chunk_start[b], c1 = pb.chunk_start[b + 1];
  const int ns = prog.n_slots;
  const uint32_t bid = (uint32_t)p.batch_id;
  uint32_t fresh = 0, err = 0;
  uint64_t touched = 0;
  // The chunks of a bucket form a chain (each reads the rows the one before
  // it wrote), so the latency per chunk is the bucket's time -- a hot key's
  // bucket has ~10^3 chunks. Per pass of CU partials per thread: the partials
  // were loaded during the previous pass (prefetch, overlapping its store
  // drain), and each one's home row -- key, stamp and slots share a line --
  // is loaded in one go: one round trip plus the drain per chunk where the
  // partial, home-key and row loads took three.
  constexpr int CU = 4;
  uint64_t gk[CU];
  int64_t tt[CU][MS];
  auto load_pass = [&](uint32_t base, uint32_t cnt, uint32_t e0) {
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const uint32_t e = e0 + u * 256;
      gk[u] = e < cnt ? pr.gkey[base + e] : kEmpty;
#pragma unroll
      for (int s = 0; s < MS; ++s) tt[u][s] = (e < cnt && s < ns) ? pr.part[(uint64_t)(base + e) * ns + s] : 0;
    }
  };
  uint32_t c = c0, pass = 0, base = 0, cnt = 0;
  if (c < c1) {
    base = pr.cbase[c];
    cnt = pr.ccnt[c];
    load_pass(base, cnt, threadIdx.x);
  }
  while (c < c1) {
    const uint32_t e0 = threadIdx.x + pass * (256 * CU);
    uint64_t hk[CU];
    uint32_t hst[CU];
    int64_t hrow[CU][MS];
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      hk[u] = kEmpty;
      if (gk[u] == kEmpty) continue;
      const uint64_t hs = tw_region_base(t, gk[u]) + tw_home_in(t, gk[u]);
      hk[u] = __hip_atomic_load(t.key(hs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      hst[u] = __hip_atomic_load(t.stamp(hs), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
      for (int s = 0; s < MS; ++s)
        hrow[u][s] = s < ns ? __hip_atomic_load(t.aggs(hs) + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    }
#pragma unroll
    for (int u = 0; u < CU; ++u) {
      const uint32_t e = e0 + u * 256;
      if (e >= cnt) continue;
      const uint32_t gi = base + e;
      const uint64_t g = gk[u];
      int64_t tot[MS], cur[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) tot[s] = tt[u][s];
      // find or claim (agent-scope loads: an earlier chunk of this workgroup may have claimed it)
      const uint64_t rb = tw_region_base(t, g);
      uint64_t sl = tw_home_in(t, g);
      const uint64_t step = tw_step(t), np = (t.rmask + 1) / step;
      int64_t slot = -1;
      bool isnew = false, loaded = false;
      uint32_t st = 0;
      if (hk[u] == g) {  // found at its home slot (the usual case), its row loaded with the key
        slot = (int64_t)(rb + sl);
        loaded = true;
        st = hst[u];
#pragma unroll
        for (int s = 0; s < MS; ++s) cur[s] = hrow[u][s];
      }
      for (uint64_t probe = 0; slot < 0 && probe < np && probe < kMaxProbes; ++probe) {
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
      if (slot < 0) {  // the region's sub-table is full
        slot = tw_ovf_claim_new(t, g, isnew);
        fresh += isnew ? 1 : 0;
      }
      if (slot < 0) {
        err |= ERR_OOM;
        identity_row<MS>(prog, cur);
      } else {
        int64_t *row = t.aggs(slot);
        uint32_t *stp = t.stamp(slot);
        if (isnew) {
          identity_row<MS>(prog, cur);
        } else if (!loaded) {
#pragma unroll
          for (int s = 0; s < MS; ++s)
            cur[s] = s < ns ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
          st = __hip_atomic_load(stp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        int64_t nv[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) nv[s] = cur[s];
        combine_row<MS>(prog, nv, tot);
#pragma unroll
        for (int s = 0; s < MS; ++s)
          if (s < ns) row[s] = nv[s];
        if (st != bid) {  // (a new row: st = 0)
          *stp = bid;
          touched += 1;
        }
      }
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < ns) pr.part[(uint64_t)gi * ns + s] = cur[s];
    }
    // the next pass (uniform): more of this chunk, else the next chunk --
    // its partials loaded now, beside this pass's stores
    uint32_t nc = c, npass = pass + 1;
    if ((uint64_t)npass * (256 * CU) >= cnt) {
      nc = c + 1;
      npass = 0;
    }
    if (nc < c1) {
      if (nc != c) {
        base = pr.cbase[nc];
        cnt = pr.ccnt[nc];
      }
      load_pass(base, cnt, threadIdx.x + npass * (256 * CU));
    }
    if (nc != c) {
      // this chunk's rows in L2 before the next chunk reads them: the same
      // workgroup (one CU, one L2) reads them back with L1-bypassing loads, so
      // draining the stores is enough (no device-scope fence: a whole-L2 write-
      // back per chunk)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
    }
    c = nc;
    pass = npass;
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

// One workgroup per kPrEmitRecs arrival-order records, in rounds of
// kPrEmitThreads consecutive records. A round's rows are consecutive in the
// changelog (its records' accepted pairs in arrival order), so after each
// thread has found its record's window run and the round's prefix, the rows
// are written row-parallel: thread t writes rows t, t + NT, ... of the round,
// each column store of a wave covering 64 consecutive rows (a record-per-
// thread loop over its windows stored 8-byte pieces 12 rows apart: partial
// lines that the L2 could not merge before writing them back). A row finds
// its record by a binary search over the round's record offsets in LDS.
constexpr int kPrEmitThreads = 1024;
constexpr int kPrEmitRounds = kPrEmitRecs / kPrEmitThreads;
static_assert(kPrEmitRecs % kPartTileRecs == 0 && kPrEmitRounds * kPrEmitThreads == kPrEmitRecs, "emit tile");

template <int MS>
__global__ __launch_bounds__(kPrEmitThreads) void k_pr_emit(Batch bt, Program prog, TwParams p, PartParams pp,
                                                            PartBuffers pb, PrPart pr, uint32_t wpr,
                                                            const int64_t *__restrict__ rec_wm,
                                                            const int64_t *__restrict__ seq, OutCols out,
                                                            uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  __shared__ uint32_t sw[kPrEmitThreads / 64];
  __shared__ uint32_t roff[kPrEmitThreads + 1];  // round-relative first row of each record
  __shared__ uint32_t rpos[kPrEmitThreads];      // its partitioned position
  __shared__ uint32_t rkey[kPrEmitThreads], rwin[kPrEmitThreads];
  if (sc->redo || !pr.counter[1]) return;  // uniform
  const int64_t k_epoch = sc->k_epoch;
  const int64_t *wm = rec_wm ? rec_wm : (sc->no_late ? nullptr : pb.wm);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t rw = 1 + (uint64_t)prog.n_slots;
  const int ns = prog.n_slots;
  uint32_t err = 0;
  // the workgroup's first changelog row: the tiles before it (histogram pair
  // counts, scanned); the rounds then advance it by their pair totals
  uint64_t base = pr.tpoff[(uint64_t)blockIdx.x * (kPrEmitRecs / kPartTileRecs)];
  for (int rd = 0; rd < kPrEmitRounds; ++rd) {
    const uint64_t i0 = (uint64_t)blockIdx.x * kPrEmitRecs + (uint64_t)rd * kPrEmitThreads;
    if (i0 >= bt.n) break;  // uniform
    const uint64_t i = i0 + threadIdx.x;
    uint32_t a = 0, n = 0, key = HSG_KEY_NONE;
    if (i < bt.n) {
      key = bt.key[i];
      const int64_t ts = bt.ts[i];
      // same window run as the partition passes (k_part.hip part_record)
      if (key != HSG_KEY_NONE) {
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
    }
    // exclusive prefix of the round's pairs in arrival order
    const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)n);
    if (lane == 63) sw[wv] = incl;
    lds_barrier();
    uint32_t before = incl - n, tot = 0;
    for (int k = 0; k < kPrEmitThreads / 64; ++k) {
      before += k < wv ? sw[k] : 0u;
      tot += sw[k];
    }
    roff[threadIdx.x] = before;
    if (threadIdx.x == kPrEmitThreads - 1) roff[kPrEmitThreads] = before + n;
    // (k_pr_keysort's place of the record; one-window ops: no key grouping)
    rpos[threadIdx.x] = n ? (pr.kpos ? pr.kpos[pr.pos[i]] : pr.pos[i]) : 0u;
    rkey[threadIdx.x] = key;
    rwin[threadIdx.x] = a;
    lds_barrier();
    // rows of the round, row-parallel: q -> its record (the last record whose
    // first row is <= q), window j = q - first row
    constexpr int EQ = MS <= 4 ? 4 : 2;  // rows per thread with their loads in flight together
    for (uint32_t q0 = 0; q0 < tot; q0 += (uint32_t)kPrEmitThreads * EQ) {
      uint32_t rr[EQ], jj[EQ], gq[EQ];
      int64_t Lq[EQ][MS], Rq[EQ][MS];
#pragma unroll
      for (int u = 0; u < EQ; ++u) {
        const uint32_t q = q0 + (uint32_t)u * kPrEmitThreads + threadIdx.x;
        uint32_t lo = 0, hi = kPrEmitThreads;  // roff[lo] <= q < roff[hi]
        while (hi - lo > 1) {
          const uint32_t mid = (lo + hi) >> 1;
          if (roff[mid] <= q) lo = mid;
          else hi = mid;
        }
        rr[u] = lo;
        jj[u] = q - roff[lo];
        const bool ok = q < tot;
        const uint64_t pos = rpos[lo];
        const uint64_t *it = pr.inter + (ok ? (pos * wpr + jj[u]) * rw : 0);
        gq[u] = ok ? (uint32_t)it[0] : 0u;
#pragma unroll
        for (int s = 0; s < MS; ++s) Lq[u][s] = (ok && s < ns) ? (int64_t)it[1 + s] : 0;
      }
#pragma unroll
      for (int u = 0; u < EQ; ++u) {
        const uint32_t q = q0 + (uint32_t)u * kPrEmitThreads + threadIdx.x;
        const bool ok = q < tot && (uint64_t)gq[u] < pb.n_cap * wpr;
#pragma unroll
        for (int s = 0; s < MS; ++s) Rq[u][s] = (ok && s < ns) ? pr.part[(uint64_t)gq[u] * ns + s] : 0;
      }
#pragma unroll
      for (int u = 0; u < EQ; ++u) {
        const uint32_t q = q0 + (uint32_t)u * kPrEmitThreads + threadIdx.x;
        if (q >= tot) break;
        if ((uint64_t)gq[u] >= pb.n_cap * wpr || rpos[rr[u]] >= pb.n_cap) {  // cannot happen
          err |= ERR_OOM;
          continue;
        }
        int64_t R[MS], L[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) {
          R[s] = Rq[u][s];
          L[s] = Lq[u][s];
        }
        combine_row<MS>(prog, R, L);
        const uint64_t ob = out_base + base + q;
        if (ob >= out_cap) {
          err |= ERR_OOM;
          continue;
        }
        const uint64_t irec = i0 + rr[u];
        out.key[ob] = rkey[rr[u]];
        int64_t ws = 0, we = 0;
        if (p.kind != HSG_UNWINDOWED) {
          const int64_t k = k_epoch + (int64_t)(rwin[rr[u]] + jj[u]);
          ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
          we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
        }
        out.ws[ob] = ws;
        out.we[ob] = we;
        out.src[ob] = seq ? seq[irec] : (int64_t)(p.rec_base + irec);
#pragma unroll
        for (int c = 0; c < kMaxAggs; ++c)  // static indices: the column pointers stay in registers
          if (c < prog.n_out) out.agg[c][ob] = out_value_reg<MS>(prog, c, R);
        if (out.form) out.form[ob] = out_form_reg<MS>(prog, R);
      }
    }
    base += tot;
    lds_barrier();  // sw / roff / rpos are rewritten by the next round
  }
  if (err) atomicOr(&sc->err, err);
}

// ---------------------------------------------------------------------------
// One-window ops (tumbling, unwindowed: one pair per partitioned record):
// k_pr_bucket, one workgroup per bucket, walks the bucket's records in arrival
// order and leaves each record's changelog state (the group's aggregate right
// after it) at the record's partitioned position; k_pr_emit1 then writes the
// rows in arrival order. No chunk carries: the bucket is its workgroup's.
//
//   per segment of the bucket (as many records as keep the LDS table at most
//   half full; one segment unless the bucket holds very many groups):
//   1. the segment's groups into an LDS table (in 256-record steps);
//   2. each group found / claimed in the HBM table, its row loaded into LDS
//      (all groups at once: one round of HBM latency per segment);
//   3. 256-record steps in arrival order: the four waves one after the other,
//      each group's lowest lane of the wave folds its lanes' records into the
//      group's LDS state in lane (= arrival) order and hands each record its
//      state (a step's records of one group are rare except for hot keys);
//   4. the LDS states written back to their rows.
// ---------------------------------------------------------------------------
constexpr int kPbNT = 256;
constexpr int kPbNW = kPbNT / 64;

// Slot-program helpers over a program view (ProgRT, or ProgSig<SIG> with the
// slot ops baked in: the common aggregate sets get straight-line combines)
template <int MS, class PV>
__device__ inline void combine_v(const PV &pv, int64_t (&a)[MS], const int64_t (&e)[MS]) {
  if constexpr (std::is_same<PV, ProgRT>::value) {
    // a runtime program: tie words, the LAST pair and the form slots
    // (combine_row)
    combine_row<MS>(pv.p, a, e);
    return;
  } else {
    // a baked program with tie words (the SQL shape): the words first, against
    // the MIN / MAX values before the combine (as combine_row)
    if constexpr (PV::has_ties()) {
#pragma unroll
      for (int s = 0; s < MS; ++s) {
        if (s >= pv.n()) break;
        const int op = pv.op(s);
        if (op != S_TIE_MIN && op != S_TIE_MAX) continue;
        const int v = PV::aux_of(s);
        a[s] = tie_combine(op, pv.op(v), reg_at<MS>(a, v), reg_at<MS>(e, v), a[s], e[s]);
      }
    }
  }
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= pv.n()) break;
    const int op = pv.op(s);
    if (op == S_LAST_SEQ) {
      if (e[s] != 0) {
        a[s] = e[s];
        if (s + 1 < MS) a[s + 1] = e[s + 1];
      }
    } else if (op != S_LAST_VAL) {
      a[s] = slot_combine(op, a[s], e[s]);
    }
  }
}
template <int MS, class PV>
__device__ inline void identity_v(const PV &pv, int64_t (&a)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) a[s] = s < pv.n() ? slot_identity_dev(pv.op(s)) : 0;
}
template <int MS, class PV, class RV>
__device__ inline void elems_v(const PV &pv, const RV &r, int64_t (&e)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    e[s] = 0;
    if (s >= pv.n()) continue;
    const int op = pv.op(s), c = pv.col(s);
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
      case S_CNT_DEC: e[s] = r.dec(c) ? 1 : 0; break;
      case S_TIE_MIN:
      case S_TIE_MAX:
      case S_LAST_FORM: e[s] = (int64_t)(((uint64_t)r.seq1() << 1) | (r.dec(c) ? 0u : 1u)); break;
      default: break;
    }
  }
}

__device__ inline uint32_t pb_home(uint64_t g, int log2tab) {
  uint32_t h = (uint32_t)g * 0x9E3779B1u + (uint32_t)(g >> 32) * 0x85EBCA77u;
  h ^= (h >> 15) * 0x7FEB352Du;
  return h >> (32 - log2tab);
}

// find or claim group g's row in the HBM table (the overflow rows when its
// region is full); -1 = those are full too (ERR_OOM)
__device__ inline int64_t pr_claim_row(const TwTable &t, uint64_t g, bool &isnew) {
  const uint64_t rb = tw_region_base(t, g);
  uint64_t sl = tw_home_in(t, g);
  const uint64_t step = tw_step(t), np = (t.rmask + 1) / step;
  isnew = false;
  for (uint64_t probe = 0; probe < np && probe < kMaxProbes; ++probe) {
    uint64_t *kp = t.key(rb + sl);
    const uint64_t k = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (k == g) return (int64_t)(rb + sl);
    if (k == kEmpty) {
      const uint64_t old = atomicCAS((unsigned long long *)kp, (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        t.mark(rb + sl);
        isnew = true;
        return (int64_t)(rb + sl);
      }
      if (old == g) return (int64_t)(rb + sl);
    }
    sl = (sl + step) & t.rmask;
  }
  return tw_ovf_claim_new(t, g, isnew);  // the region's sub-table is full
}

// A partitioned record with its first kPrRegWords words in registers
// (prefetched a step ahead); further words (more columns) from memory. Every
// word an op of <= 2 columns reads is a register: no load inside a step, whose
// wait would also wait for the step's stores (vmcnt counts both).
constexpr int kPrRegWords = 4;
template <bool REG>  // REG: the record has <= kPrRegWords words (no memory path)
struct PrRecRegs {
  uint64_t r0, r1, r2, r3;  // named, not an array: a runtime index would put an array on the stack
  const uint64_t *w;
  bool pk;
  int C;
  __device__ uint32_t key() const { return (uint32_t)r0; }
  __device__ uint32_t krel(uint32_t kbase) const {
    return pk ? kbase + (uint32_t)((r0 >> 32) & 0xFFFFull) : (uint32_t)(r0 >> 32);
  }
  __device__ uint32_t nwin() const { return pk ? (uint32_t)((r0 >> 48) & 0xFFull) : (uint32_t)r1; }
  __device__ bool present(int c) const { return pk ? (r0 >> (56 + c)) & 1ull : (r1 >> (32 + c)) & 1ull; }
  __device__ int64_t word(int k) const {
    if (!REG && k >= kPrRegWords) return (int64_t)w[k];
    return (int64_t)(k == 0 ? r0 : k == 1 ? r1 : k == 2 ? r2 : r3);
  }
  __device__ int64_t col(int c) const { return word((pk ? 1 : 2) + c); }
  // the sequence word (hsg_dev.h seq_word): seq + 1, decimal-literal bits
  __device__ int64_t seq1() const { return (int64_t)((uint64_t)word((pk ? 1 : 2) + C) & kSeqMask); }
  __device__ bool dec(int c) const { return ((uint64_t)word((pk ? 1 : 2) + C) >> (56 + c)) & 1ull; }
};

template <int MS, int LT, bool REG, uint64_t SIG, uint64_t SIG2 = 0>
__global__ __launch_bounds__(kPbNT) void k_pr_bucket(Program prog, TwParams p, PartParams pp, TwTable t,
                                                     PartBuffers pb, PrPart pr, DevScalars *sc) {
  const ProgView<SIG, SIG2> pv(prog);
  constexpr int TAB = 1 << LT;
  constexpr int EPT = TAB / kPbNT;  // table entries per thread
  constexpr int PF = 8;             // record loads in flight per thread in the one-pass insert
  constexpr int CAP = TAB / 2;      // groups of a segment (the table runs at most half full)
  __shared__ uint64_t tkey[TAB];
  __shared__ uint16_t tidx[TAB];    // group index (insertion order) of the key at each slot
  __shared__ int64_t tst[MS][CAP];  // per group index: state, row slot, owners of the step
  __shared__ uint32_t tslot[CAP];
  __shared__ int64_t stg[kPbNW][MS][64];  // each wave's records' contributions, then its groups' totals
  __shared__ uint8_t widx[kPbNW][CAP];     // per wave: 1 + owner lane of each group in the step, 0 = none
  __shared__ uint32_t s_fill;
  __shared__ uint64_t s_red[2][kPbNW];
  if (sc->redo || pr.counter[1]) return;  // uniform: stale bucket starts / a hot bucket: the chunked path runs
  const uint32_t b = blockIdx.x;
  const uint64_t r0 = pb.bstart[b], r1 = pb.bstart[b + 1];
  if (r0 >= r1) return;  // uniform
  const bool pk = sc->packed != 0;
  const int W = pk ? pp.words - 1 : pp.words;
  const int C = pp.words - 2 - pp.has_seq;
  const uint32_t kbase = (uint32_t)sc->kbase;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ns = pv.n();
  const uint32_t bid = (uint32_t)p.batch_id;
  const uint64_t *rec = pb.rec;
  uint32_t err = 0;
  uint64_t fresh = 0, touched = 0;
  uint64_t c_ins = 0, c_claim = 0, c_steps = 0, c_back = 0, nseg = 0;  // phase clocks (HSG_PHASES)
  uint64_t c_phase = 0, npeer = 0;
  const uint64_t c_start = phase_clock();
  // LDS insert of group g; returns false once the table passed half full
  // (then at most TAB / 2 + kPbNT - 1 entries: every probe sequence ends)
  auto insert = [&](uint64_t g) -> bool {
    uint32_t h = pb_home(g, LT);
    for (;;) {
      const uint64_t c = tkey[h];
      if (c == g) return true;
      if (c == kEmpty) {
        const uint64_t old = atomicCAS((unsigned long long *)&tkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
        if (old == kEmpty) {
          const uint32_t c = atomicAdd(&s_fill, 1u);
          if (c < (uint32_t)CAP) tidx[h] = (uint16_t)c;
          return c + 1 <= (uint32_t)CAP;
        }
        if (old == g) return true;
      }
      h = (h + 1) & (TAB - 1);
    }
  };
  for (int e = threadIdx.x; e < TAB; e += kPbNT) tkey[e] = kEmpty;
  for (int e = threadIdx.x; e < kPbNW * CAP; e += kPbNT) (&widx[0][0])[e] = 0;
  if (threadIdx.x == 0) s_fill = 0;
  __syncthreads();
  // 1a. one pass over the whole bucket, PF record loads in flight per thread:
  // one segment when its groups fill at most half the table (the common case)
  uint64_t ca = phase_clock();
  bool ok = true;
  for (uint64_t i0 = r0 + threadIdx.x; ok && i0 < r1; i0 += (uint64_t)PF * kPbNT) {
    uint64_t w0[PF];
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint64_t i = i0 + (uint64_t)u * kPbNT;
      w0[u] = i < r1 ? rec[i * (uint64_t)W] : 0;
    }
#pragma unroll
    for (int u = 0; u < PF; ++u) {
      const uint64_t i = i0 + (uint64_t)u * kPbNT;
      if (ok && i < r1) {
        const PrRecRegs<REG> v{w0[u], 0, 0, 0, nullptr, pk, C};
        ok = insert(((uint64_t)v.key() << 32) | v.krel(kbase));
      }
    }
    if (s_fill > (uint32_t)(TAB / 2)) ok = false;  // another thread passed it (racy read: only stops early)
  }
  lds_barrier();
  const bool one_segment = s_fill <= (uint32_t)(TAB / 2);  // uniform
  for (uint64_t s0 = r0; s0 < r1;) {
    ++nseg;
    uint64_t s1 = r1;
    if (!one_segment) {
      // 1b. the segment's groups in kPbNT-record steps while the table stays <= half full
      __syncthreads();
      for (int e = threadIdx.x; e < TAB; e += kPbNT) tkey[e] = kEmpty;
      if (threadIdx.x == 0) s_fill = 0;
      __syncthreads();
      s1 = s0;
      while (s1 < r1) {
        if (s_fill + kPbNT > (uint32_t)(TAB / 2)) break;  // uniform (read after the barrier)
        const uint64_t i = s1 + threadIdx.x;
        if (i < r1) {
          const PrRecRegs<REG> v{rec[i * (uint64_t)W], 0, 0, 0, nullptr, pk, C};
          insert(((uint64_t)v.key() << 32) | v.krel(kbase));
        }
        s1 = s1 + kPbNT < r1 ? s1 + kPbNT : r1;
        lds_barrier();
      }
    }
    { const uint64_t cb = phase_clock(); c_ins += cb - ca; ca = cb; }
    // 2. rows of the segment's groups into LDS: every entry's home probe
    // issued at once (agent-scope loads: an earlier segment of this workgroup
    // may have written the rows), then the rows
    {
      uint64_t g[EPT], kh[EPT], hs[EPT];
#pragma unroll
      for (int u = 0; u < EPT; ++u) {
        g[u] = tkey[threadIdx.x + u * kPbNT];
        hs[u] = 0;
        kh[u] = kEmpty;
        if (g[u] != kEmpty) {
          hs[u] = tw_region_base(t, g[u]) + tw_home_in(t, g[u]);
          kh[u] = __hip_atomic_load(t.key(hs[u]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      int64_t sl[EPT];
      bool isnew[EPT];
#pragma unroll
      for (int u = 0; u < EPT; ++u) {
        sl[u] = -1;
        isnew[u] = false;
        if (g[u] == kEmpty) continue;
        if (kh[u] == g[u]) {
          sl[u] = (int64_t)hs[u];
        } else {
          if (kh[u] == kEmpty) {
            const uint64_t old = atomicCAS((unsigned long long *)t.key(hs[u]), (unsigned long long)kEmpty,
                                           (unsigned long long)g[u]);
            if (old == kEmpty) {
              t.mark(hs[u]);
              isnew[u] = true;
              sl[u] = (int64_t)hs[u];
            } else if (old == g[u]) {
              sl[u] = (int64_t)hs[u];
            }
          }
          if (sl[u] < 0) sl[u] = pr_claim_row(t, g[u], isnew[u]);  // collision: the full probe
        }
      }
      int64_t cur[EPT][MS];
      uint32_t st[EPT];
#pragma unroll
      for (int u = 0; u < EPT; ++u) {
        identity_v<MS>(pv, cur[u]);
        st[u] = 0;
        if (sl[u] >= 0 && !isnew[u]) {
          const int64_t *row = t.aggs(sl[u]);
#pragma unroll
          for (int s = 0; s < MS; ++s)
            if (s < ns) cur[u][s] = __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          st[u] = __hip_atomic_load(t.stamp(sl[u]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
#pragma unroll
      for (int u = 0; u < EPT; ++u) {
        const int e = threadIdx.x + u * kPbNT;
        if (g[u] == kEmpty) continue;
        if (sl[u] < 0) {
          err |= ERR_OOM;
        } else {
          fresh += isnew[u] ? 1 : 0;
          if (st[u] != bid) {  // (a new row's stamp reads as 0)
            *t.stamp(sl[u]) = bid;
            touched += 1;
          }
        }
        const uint32_t c = tidx[e];
        tslot[c] = sl[u] < 0 ? ~0u : (uint32_t)sl[u];
#pragma unroll
        for (int s = 0; s < MS; ++s) tst[s][c] = cur[u][s];
      }
    }
    lds_barrier();
    { const uint64_t cb = phase_clock(); c_claim += cb - ca; ca = cb; }
    // 3. the segment's records in arrival order (the next step's first two
    // words loaded while this step runs). A step's four waves run side by
    // side: (A) each lane folds its wave's earlier records of its group (lane
    // order = arrival order) into its wave-local prefix; the group's highest
    // lane of the wave (its owner) holds the wave's total; (B) each owner
    // takes the group's state, folds in the totals of the earlier waves'
    // owners of the group, and hands the result (the state before its wave)
    // to its lanes; the owner in the group's last wave of the step keeps the
    // state after the step. Two barriers per step.
    // the step's record words: registers, loaded one step ahead at the top
    // of the previous step (before its stores: the wait for them at the top
    // of this step then leaves the stores in flight)
    uint64_t nx0 = 0, nx1 = 0, nx2 = 0, nx3 = 0;
    auto fetch = [&](uint64_t ii) {
      const uint64_t *q = rec + ii * (uint64_t)W;
      const bool f = ii < s1;
      nx0 = f ? q[0] : 0ull;
      nx1 = (f && W > 1) ? q[1] : 0ull;
      nx2 = (f && W > 2) ? q[2] : 0ull;
      nx3 = (f && W > 3) ? q[3] : 0ull;
    };
    fetch(s0 + threadIdx.x);
    for (uint64_t base = s0; base < s1; base += kPbNT) {
      const uint64_t i = base + threadIdx.x;
      const bool in = i < s1;
      const PrRecRegs<REG> v{nx0, nx1, nx2, nx3, rec + i * (uint64_t)W, pk, C};
      fetch(i + kPbNT);
      uint32_t h = 0;  // then the group's index
      int64_t pre[MS];
      identity_v<MS>(pv, pre);
      const uint64_t t0 = phase_clock();
      if (in) {
        const uint64_t g = ((uint64_t)v.key() << 32) | v.krel(kbase);
        h = pb_home(g, LT);
        while (tkey[h] != g) h = (h + 1) & (TAB - 1);  // inserted in step 1
        h = tidx[h];
        int64_t e[MS];
        elems_v<MS>(pv, v, e);
#pragma unroll
        for (int s = 0; s < MS; ++s) stg[wv][s][lane] = e[s];
      }
      // this wave's lanes of each group, found by one ballot per table bit
      uint64_t peers = __ballot(in);
#pragma unroll
      for (int bit = 0; bit < LT - 1; ++bit) {
        const bool x = (h >> bit) & 1u;
        const uint64_t bb = __ballot(x);
        peers &= x ? bb : ~bb;
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // the wave's elements in LDS
      const uint64_t t1 = phase_clock();
      npeer += in ? (uint64_t)__popcll(peers) : 0ull;
      // (A) wave-local inclusive prefix over the group's lanes up to this one
      if (in) {
        const uint64_t upto = peers & (lane == 63 ? ~0ull : ((2ull << lane) - 1ull));
        for (uint64_t m = upto; m; m &= m - 1) {
          const int q = __ffsll((long long)m) - 1;
          int64_t e[MS];
#pragma unroll
          for (int s = 0; s < MS; ++s) e[s] = stg[wv][s][q];
          combine_v<MS>(pv, pre, e);
        }
      }
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront", "local");  // every lane read its peers' elements
      const uint64_t t2 = phase_clock();
      const int owner_lane = in ? 63 - __clzll((long long)peers) : lane;
      const bool owner = in && owner_lane == lane;
      if (owner) {
#pragma unroll
        for (int s = 0; s < MS; ++s) stg[wv][s][lane] = pre[s];  // the wave's total for the group
        widx[wv][h] = (uint8_t)(lane + 1);
      }
      lds_barrier();  // (LDS only: the step's global loads and stores keep flowing)
      // (B) the owners: the state before this wave, and after the step
      int64_t carry[MS], after[MS];
      bool last = false;
      if (owner) {
#pragma unroll
        for (int s = 0; s < MS; ++s) carry[s] = tst[s][h];
        last = true;
        for (int w = 0; w < kPbNW; ++w) {
          const uint32_t k = widx[w][h];
          if (!k || w == wv) continue;
          if (w > wv) {
            last = false;
            continue;
          }
          int64_t e[MS];
#pragma unroll
          for (int s = 0; s < MS; ++s) e[s] = stg[w][s][k - 1];
          combine_v<MS>(pv, carry, e);
        }
#pragma unroll
        for (int s = 0; s < MS; ++s) after[s] = carry[s];
        combine_v<MS>(pv, after, pre);
      } else {
        identity_v<MS>(pv, carry);
      }
      // every lane takes its owner's carry (all lanes active: plain permutes)
#pragma unroll
      for (int s = 0; s < MS; ++s) carry[s] = __shfl(carry[s], owner_lane, 64);
      lds_barrier();  // every owner has read the totals and the states
      const uint64_t t3 = phase_clock();
      c_phase += (t1 - t0) | ((t2 - t1) << 21) | ((t3 - t2) << 42);  // 21-bit fields (per-step deltas)
      if (in) {
        int64_t fin[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) fin[s] = carry[s];
        combine_v<MS>(pv, fin, pre);
        // at the record's partitioned position: consecutive lanes, consecutive rows
        if (SIG != 0 && prog.fin_n == ns && !prog.fin_form) {  // (uniform: no projection)
          int64_t *o = pr.fin + i * (uint64_t)ns;
#pragma unroll
          for (int s = 0; s < MS; ++s)
            if (s < ns) o[s] = fin[s];
        } else {
          // the words the row's outputs read (hsg_internal.h fin_*)
          const int fw = prog.fin_n + prog.fin_form;
          int64_t *o = pr.fin + i * (uint64_t)fw;
#pragma unroll
          for (int k = 0; k < MS; ++k)
            if (k < prog.fin_n) o[k] = reg_at<MS>(fin, prog.fin_slot[k]);
          if (prog.fin_form) o[prog.fin_n] = (int64_t)out_form_reg<MS>(prog, fin);
        }
      }
      if (owner) {
        if (last) {
#pragma unroll
          for (int s = 0; s < MS; ++s) tst[s][h] = after[s];
        }
        widx[wv][h] = 0;
      }
    }
    lds_barrier();  // the last step's owners have written their groups' states
    { const uint64_t cb = phase_clock(); c_steps += cb - ca; ca = cb; }
    // 4. the groups' states back to their rows
    for (int e = threadIdx.x; e < TAB; e += kPbNT) {
      if (tkey[e] == kEmpty) continue;
      const uint32_t c = tidx[e];
      if (tslot[c] == ~0u) continue;
      int64_t *row = t.aggs(tslot[c]);
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < ns) row[s] = tst[s][c];
    }
    // the next segment reads these rows back (L1-bypassing loads): drain
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    c_back += phase_clock() - ca;
    ca = phase_clock();
    s0 = s1;
  }
  if (err) atomicOr(&sc->err, err);
  const uint64_t f = wave_sum_u64(fresh), tc = wave_sum_u64(touched);
  if (lane == 0) {
    s_red[0][wv] = f;
    s_red[1][wv] = tc;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t ff = 0, tt = 0;
    for (int k = 0; k < kPbNW; ++k) {
      ff += s_red[0][k];
      tt += s_red[1][k];
    }
    if (ff) atomicAdd((unsigned long long *)&sc->live_x[blockIdx.x & 7], (unsigned long long)ff);
    if (tt) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tt);
    if (kPhaseClocks) {
      atomicAdd((unsigned long long *)&sc->scratch[36], (unsigned long long)c_ins);
      atomicAdd((unsigned long long *)&sc->scratch[37], (unsigned long long)c_claim);
      atomicAdd((unsigned long long *)&sc->scratch[38], (unsigned long long)c_steps);
      atomicAdd((unsigned long long *)&sc->scratch[39], (unsigned long long)c_back);
      atomicAdd((unsigned long long *)&sc->scratch[40], (unsigned long long)nseg);
      atomicAdd((unsigned long long *)&sc->scratch[41], 1ull);
      atomicAdd((unsigned long long *)&sc->scratch[42], (unsigned long long)(phase_clock() - c_start));
      if (blockIdx.x == 0) sc->scratch[43] = c_phase;  // one workgroup's step sub-phases
    }
  }
  if (kPhaseClocks && lane == 0 && npeer) atomicAdd((unsigned long long *)&sc->scratch[44], (unsigned long long)npeer);
}

// Rows of one-window ops in arrival order: the record's window as the
// partition computed it, its state from k_pr_bucket (pr.fin at the record's
// partitioned position pr.pos). Each thread carries kE1 records of
// consecutive rounds (record = round base + thread: coalesced lanes), their
// state gathers issued together: kE1 row loads in flight per thread.
constexpr int kE1 = 4;
constexpr int kE1NT = 256;                         // threads of k_pr_emit1 (registers for kE1 records each)
constexpr int kE1Rounds = kPrEmitRecs / kE1NT;
static_assert(kE1Rounds % kE1 == 0 && kE1Rounds * kE1NT == kPrEmitRecs, "emit rounds");

template <int MS>
__global__ __launch_bounds__(kE1NT) void k_pr_emit1(Batch bt, Program prog, TwParams p, PartBuffers pb,
                                                             PrPart pr, const int64_t *__restrict__ rec_wm,
                                                             const int64_t *__restrict__ seq, OutCols out,
                                                             uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  __shared__ uint32_t sw[kE1][kE1NT / 64];
  if (sc->redo || pr.counter[1]) return;  // uniform (a hot bucket: the chunked path's k_pr_emit)
  const int64_t k_epoch = sc->k_epoch;
  const int64_t *wm = rec_wm ? rec_wm : (sc->no_late ? nullptr : pb.wm);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  // the state words k_pr_bucket left per record (hsg_internal.h fin_*; the
  // baked programs: the whole state)
  const int fw = prog_fin_words(prog) ;
  const bool proj = prog.fin_n != prog.n_slots || prog.fin_form;
  uint32_t err = 0;
  // consecutive tiles on one XCD: their rows of a bucket are neighbours in pr.fin
  const uint64_t tile = xcd_tile(blockIdx.x, gridDim.x);
  uint64_t base = pr.tpoff[tile * (kPrEmitRecs / kPartTileRecs)];
  for (int rd0 = 0; rd0 < kE1Rounds; rd0 += kE1) {
    if (tile * kPrEmitRecs + (uint64_t)rd0 * kE1NT >= bt.n) break;  // uniform
    // every load of the rounds is issued up front (indices clamped, no
    // branches), so a thread waits on two memory round trips: the record
    // columns + its position, then the state rows
    uint32_t a[kE1], n[kE1], key[kE1];
    uint64_t i[kE1], pz[kE1];
    int64_t tsv[kE1], wmv[kE1];
    const uint64_t last = bt.n - 1;
#pragma unroll
    for (int u = 0; u < kE1; ++u) {
      i[u] = tile * kPrEmitRecs + (uint64_t)(rd0 + u) * kE1NT + threadIdx.x;
      const uint64_t ic = i[u] < bt.n ? i[u] : last;
      key[u] = bt.key[ic];
      tsv[u] = bt.ts[ic];
      wmv[u] = wm ? wm[ic] : INT64_MIN;
      pz[u] = pr.pos[ic];
      if (i[u] >= bt.n) key[u] = HSG_KEY_NONE;
    }
    // the states (a record the partition dropped has a stale position: its
    // row is read, clamped into the buffer, and not used)
    int64_t R[kE1][MS];
#pragma unroll
    for (int u = 0; u < kE1; ++u) {
      const int64_t *f = pr.fin + (pz[u] < pb.n_cap ? pz[u] : 0) * (uint64_t)fw;
      if constexpr (MS % 2 == 0) {
        if ((fw & 1) == 0) {  // 16-B aligned rows
#pragma unroll
          for (int s = 0; s < MS; s += 2) {
            if (s < fw) {
              const longlong2 v = *reinterpret_cast<const longlong2 *>(f + s);
              R[u][s] = v.x;
              R[u][s + 1] = v.y;
            } else {
              R[u][s] = R[u][s + 1] = 0;
            }
          }
          continue;
        }
      }
#pragma unroll
      for (int s = 0; s < MS; ++s) R[u][s] = s < fw ? f[s] : 0;
    }
    // a projected state: the launcher's program indexes the projected words
    // (pr_launch fin_outputs), the form word stays at fin_n
    uint32_t F[kE1];
#pragma unroll
    for (int u = 0; u < kE1; ++u) F[u] = proj && prog.fin_form ? (uint32_t)reg_at<MS>(R[u], prog.fin_n) : 0u;
#pragma unroll
    for (int u = 0; u < kE1; ++u) {
      a[u] = 0;
      n[u] = 0;
      if (key[u] == HSG_KEY_NONE) continue;  // the window the partition passes accepted (k_part.hip part_record)
      uint64_t k_lo, k_hi;
      if (record_windows(p, tsv[u], k_lo, k_hi) && window_accepted(p, k_lo, wmv[u])) {
        const int64_t lo = (int64_t)k_lo - k_epoch;
        if (lo >= 0 && lo <= 0xFFFFFFFFll) {
          a[u] = (uint32_t)lo;
          n[u] = 1;
        }
      }
    }
    // exclusive prefixes of the rounds' rows in arrival order
    uint64_t o[kE1];
#pragma unroll
    for (int u = 0; u < kE1; ++u) {
      const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)n[u]);
      if (lane == 63) sw[u][wv] = incl;
      o[u] = incl - n[u];
    }
    lds_barrier();
#pragma unroll
    for (int u = 0; u < kE1; ++u) {
      uint64_t before = 0, tot = 0;
      for (int k = 0; k < kE1NT / 64; ++k) {
        before += k < wv ? sw[u][k] : 0u;
        tot += sw[u][k];
      }
      o[u] += base + before;
      base += tot;
    }
    lds_barrier();  // sw is rewritten by the next rounds
#pragma unroll
    for (int u = 0; u < kE1; ++u) {
      if (!n[u]) continue;
      const uint64_t ob = out_base + o[u];
      if (ob >= out_cap || pz[u] >= pb.n_cap) {  // cannot happen
        err |= ERR_OOM;
        continue;
      }
      out.key[ob] = key[u];
      int64_t ws = 0, we = 0;
      if (p.kind != HSG_UNWINDOWED) {
        const int64_t k = k_epoch + (int64_t)a[u];
        ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
        we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
      }
      out.ws[ob] = ws;
      out.we[ob] = we;
      out.src[ob] = seq ? seq[i[u]] : (int64_t)(p.rec_base + i[u]);
#pragma unroll
      for (int jj = 0; jj < kMaxAggs; ++jj)
        if (jj < prog.n_out) out.agg[jj][ob] = out_value_reg<MS>(prog, jj, R[u]);
      if (out.form) out.form[ob] = proj && prog.fin_form ? F[u] : out_form_reg<MS>(prog, R[u]);
    }
  }
  if (err) atomicOr(&sc->err, err);
}

// ---------------------------------------------------------------------------
// Multi-window ops when every bucket fits k_pr_keysort (the usual case; a
// larger bucket sets pr.counter[1] and the batch takes k_pr_local /
// k_pr_carry / k_pr_emit above instead): a key's records are contiguous in
// krec, arrival order kept, so one wave replays them straight into its rows.
//
//   k_pr_offs  one workgroup per arrival tile: each record's first changelog
//              row (exclusive prefix of accepted windows in arrival order) and
//              its arrival index, packed in one word at its krec position.
//   k_pr_keys  one workgroup per bucket, a wave per run of equal key digits
//              (one key, rarely a few sharing the 12 bits): lane l owns window
//              lo + l of the key's window range (one pass of 64 windows for a
//              hopping key's ~2 x size / advance windows in a batch), finds /
//              claims its HBM row, then the key's records in arrival order are
//              broadcast one by one: the lanes of the record's windows fold it
//              into their state and write its rows (consecutive in the
//              changelog: one contiguous store per column). The states go back
//              once per key. No chunk partials, no carries, no emit gathers.
// ---------------------------------------------------------------------------
constexpr int kPkNT = 256;  // k_pr_keys threads
constexpr int kPkNW = kPkNT / 64;

// record i's accepted window run in arrival order [a, a + n) (k_epoch-relative),
// the same run as the partition passes (k_part.hip part_record)
__device__ inline uint32_t pr_record_run(const Batch &bt, const TwParams &p, const int64_t *wm, int64_t k_epoch,
                                         uint64_t i, uint32_t &a, uint32_t &key) {
  a = 0;
  key = HSG_KEY_NONE;
  if (i >= bt.n) return 0;
  key = bt.key[i];
  if (key == HSG_KEY_NONE) return 0;
  uint64_t k_lo, k_hi;
  if (!record_windows(p, bt.ts[i], k_lo, k_hi)) return 0;
  const int64_t w = wm ? wm[i] : INT64_MIN;
  uint64_t k = k_lo;
  while (k <= k_hi && !window_accepted(p, k, w)) ++k;
  if (k > k_hi) return 0;
  int64_t lo = (int64_t)k - k_epoch, hi = (int64_t)k_hi - k_epoch;
  if (lo < 0) lo = 0;
  if (hi > 0xFFFFFFFFll) hi = 0xFFFFFFFFll;
  if (lo > hi) return 0;
  a = (uint32_t)lo;
  return (uint32_t)(hi - lo + 1);
}

__global__ __launch_bounds__(kPrEmitThreads) void k_pr_offs(Batch bt, TwParams p, PartBuffers pb, PrPart pr,
                                                            const int64_t *__restrict__ rec_wm, DevScalars *sc) {
  __shared__ uint32_t sw[kPrEmitThreads / 64];
  if (sc->redo || pr.counter[1]) return;  // uniform
  const int64_t k_epoch = sc->k_epoch;
  const int64_t *wm = rec_wm ? rec_wm : (sc->no_late ? nullptr : pb.wm);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t base = pr.tpoff[(uint64_t)blockIdx.x * (kPrEmitRecs / kPartTileRecs)];
  for (int rd = 0; rd < kPrEmitRounds; ++rd) {
    const uint64_t i0 = (uint64_t)blockIdx.x * kPrEmitRecs + (uint64_t)rd * kPrEmitThreads;
    if (i0 >= bt.n) break;  // uniform
    const uint64_t i = i0 + threadIdx.x;
    uint32_t a, key;
    const uint32_t n = pr_record_run(bt, p, wm, k_epoch, i, a, key);
    const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)n);
    if (lane == 63) sw[wv] = incl;
    lds_barrier();
    uint32_t before = incl - n, tot = 0;
    for (int k = 0; k < kPrEmitThreads / 64; ++k) {
      before += k < wv ? sw[k] : 0u;
      tot += sw[k];
    }
    if (n) {  // one 8-byte store per record: the row (batch-relative, < 2^32 pairs) and the arrival index
      const uint32_t x = pr.kpos[pr.pos[i]];
      pr.roff[x] = ((base + before) << 32) | (uint64_t)(uint32_t)i;
    }
    base += tot;
    lds_barrier();  // sw is rewritten by the next round
  }
}

__device__ inline int64_t rl64(int64_t v, int j) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, j);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), j);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}
__device__ inline uint32_t rl32(uint32_t v, int j) { return (uint32_t)__builtin_amdgcn_readlane((int)v, j); }

template <int MS, uint64_t SIG>
__global__ __launch_bounds__(kPkNT) void k_pr_keys(Program prog, TwParams p, PartParams pp, TwTable t,
                                                   PartBuffers pb, PrPart pr, const int64_t *__restrict__ seq,
                                                   OutCols out, uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  // each wave stages its rows' states (and record lane << 8 | window offset)
  // in LDS while it replays, then writes them row-parallel: the replay step
  // of a record (~12 active lanes) only folds and stages, the output
  // conversion runs on full waves
  constexpr int CAP = MS <= 2 ? 384 : MS <= 4 ? 192 : 128;  // staged rows per wave (>= 64: one record's pass)
  __shared__ int64_t sst[kPkNW][MS][CAP];
  __shared__ uint16_t smeta[kPkNW][CAP];
  __shared__ uint16_t gst[4096];  // group starts (bucket-relative), in no particular order: one per digit value
  __shared__ uint32_t s_ng, s_next;
  if (sc->redo || pr.counter[1]) return;  // uniform
  const ProgView<SIG> pv(prog);  // the slot program, baked in for the common aggregate sets
  const uint32_t b = blockIdx.x;
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  const uint32_t m = (uint32_t)(b1 - b0);  // <= kKsBig (else counter[1])
  if (m == 0) return;                      // uniform
  const bool pk = sc->packed != 0;
  const int W = pk ? pp.words - 1 : pp.words;
  const int C = pp.words - 2 - pp.has_seq;
  const uint32_t kbase = (uint32_t)sc->kbase;
  const int hs = pp.bshift + pp.np_log2;
  const int64_t k_epoch = sc->k_epoch;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int ns = pv.n();
  const uint32_t bid = (uint32_t)p.batch_id;
  const uint64_t *rec = pr.krec + b0 * (uint64_t)W;
  uint32_t err = 0;
  uint64_t fresh = 0, touched = 0;
  uint64_t ck = phase_clock(), c_head = 0, c_load = 0, c_claim = 0, c_replay = 0, c_flush = 0, c_wb = 0;
  auto lap = [&](uint64_t &acc) {
    if constexpr (kPhaseClocks) {
      const uint64_t c = phase_clock();
      acc += c - ck;
      ck = c;
    }
  };
  if (threadIdx.x == 0) {
    s_ng = 0;
    s_next = 0;
  }
  __syncthreads();
  // 1) group heads: the first record of each run of equal key digits
  for (uint32_t r = threadIdx.x; r < m; r += kPkNT) {
    const uint32_t d = ks_digits((uint32_t)rec[(uint64_t)r * W], hs);
    if (r == 0 || ks_digits((uint32_t)rec[(uint64_t)(r - 1) * W], hs) != d) gst[atomicAdd(&s_ng, 1u)] = (uint16_t)r;
  }
  __syncthreads();
  const uint32_t ng = s_ng;
  lap(c_head);
  int64_t(&st_v)[MS][CAP] = sst[wv];
  uint16_t(&st_m)[CAP] = smeta[wv];
  // 2) each wave takes the next group until none is left. A chunk's records
  // (each lane's record, its arrival index and first row) are one round of
  // loads; the next group's first chunk is loaded with this group's claims,
  // so a group waits for one round of memory before its replay
  struct ChunkRegs {
    uint64_t w0, w1, w2, w3, ro;
    uint32_t idx;
  };
  auto load_chunk = [&](uint32_t s_, uint32_t c0_) {
    const uint32_t r = c0_ + lane;
    const uint64_t rr = r < m ? r : s_;
    const uint64_t *wp = rec + rr * W;
    ChunkRegs c;
    c.w0 = wp[0];
    c.w1 = W > 1 ? wp[1] : 0ull;
    c.w2 = W > 2 ? wp[2] : 0ull;
    c.w3 = W > 3 ? wp[3] : 0ull;
    const uint64_t ri = pr.roff[b0 + rr];
    c.idx = (uint32_t)ri;
    c.ro = ri >> 32;
    return c;
  };
  auto take_group = [&]() {
    uint32_t g_ = 0;
    if (lane == 0) g_ = atomicAdd(&s_next, 1u);
    return rl32(g_, 0);
  };
  uint32_t gi = take_group();
  ChunkRegs pre{};
  if (gi < ng) pre = load_chunk(gst[gi], gst[gi]);
  while (gi < ng) {  // uniform (wave)
    const uint32_t s = gst[gi];
    uint32_t gnext = ng, d0 = 0;
    for (uint32_t c0 = s;; c0 += 64) {  // the group's records, 64 at a time
      const ChunkRegs cr = c0 == s ? pre : load_chunk(s, c0);
      const uint32_t r = c0 + lane;
      const uint64_t rr = r < m ? r : s;
      const PrRecRegs<false> v{cr.w0, cr.w1, cr.w2, cr.w3, rec + rr * W, pk, C};
      const uint32_t idx = cr.idx;
      const uint64_t ro = cr.ro;
      const uint32_t key = v.key();
      if (c0 == s) d0 = ks_digits(rl32(key, 0), hs);  // the group's digits (its first record)
      const bool in = r < m && ks_digits(key, hs) == d0;
      const uint64_t outm = __ballot(!in);
      const uint32_t len = outm ? (uint32_t)__builtin_ctzll(outm) : 64u;  // records of the group here
      const bool mine = (uint32_t)lane < len;
      const bool last = len < 64 || c0 + 64 >= m;  // uniform: the group's last chunk
      if (last) {
        gnext = take_group();
        if (gnext < ng) pre = load_chunk(gst[gnext], gst[gnext]);
      }
      const uint32_t kr = v.krel(kbase), nw = mine ? v.nwin() : 0u;
      const int64_t src = seq ? seq[idx] : (int64_t)(p.rec_base + idx);
      int64_t e[MS];
      elems_v<MS>(pv, v, e);
      lap(c_load);
      uint64_t todo = len == 64 ? ~0ull : ((1ull << len) - 1ull);
      while (todo) {  // each key of the chunk (one, unless keys share the digits)
        const uint32_t kk = rl32(key, __builtin_ctzll(todo));
        const uint64_t km = __ballot(mine && key == kk);
        todo &= ~km;
        const bool mk = (km >> lane) & 1ull;
        const uint32_t lo = (uint32_t)wave_min_i64(mk && nw ? (int64_t)kr : (int64_t)0xFFFFFFFFll);
        const uint32_t hi = (uint32_t)wave_max_i64(mk && nw ? (int64_t)kr + nw - 1 : 0);
        // the staged rows out, row-parallel: row q = (record lane j, window
        // offset jj) -> changelog row ro_j + jj, window kr_j + jj
        auto flush = [&](uint32_t nst) {
          lap(c_replay);
          __builtin_amdgcn_wave_barrier();
          for (uint32_t q0 = 0; q0 < nst; q0 += 64) {  // uniform trip count (the shuffles)
            const uint32_t q = q0 + lane;
            const bool ok = q < nst;
            const uint32_t mt = ok ? st_m[q] : 0u;
            const int j = (int)(mt >> 8), jj = (int)(mt & 0xFFu);
            const uint64_t roj = (uint64_t)__shfl((long long)ro, j, 64);
            const uint32_t krj = (uint32_t)__shfl((int)kr, j, 64);
            const int64_t srcj = __shfl((long long)src, j, 64);
            if (!ok) continue;
            int64_t R[MS];
#pragma unroll
            for (int z = 0; z < MS; ++z) R[z] = st_v[z][q];
            const uint64_t ob = out_base + roj + (uint64_t)jj;
            if (ob >= out_cap) {
              err |= ERR_OOM;
              continue;
            }
            int64_t ws = 0, we = 0;
            if (p.kind != HSG_UNWINDOWED) {
              ws = (int64_t)((uint64_t)(k_epoch + (int64_t)(krj + (uint32_t)jj)) * (uint64_t)p.adv);
              we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
            }
            out.key[ob] = kk;
            out.ws[ob] = ws;
            out.we[ob] = we;
            out.src[ob] = srcj;
#pragma unroll
            for (int c = 0; c < kMaxAggs; ++c)  // static indices: the column pointers stay in registers
              if (c < prog.n_out) out.agg[c][ob] = out_value_reg<MS>(prog, c, R);
            if (out.form) out.form[ob] = out_form_reg<MS>(prog, R);
          }
          __builtin_amdgcn_wave_barrier();
          lap(c_flush);
        };
        for (uint64_t wb = lo; wb <= hi; wb += 64) {  // windows, 64 lanes at a time
          const uint64_t w = wb + (uint64_t)lane;
          const uint64_t we_ = wb + 63 < hi ? wb + 63 : hi;
          // the lane's window is some record's (a key's records can leave gaps)
          bool act = false;
          for (uint64_t rm = km; rm; rm &= rm - 1ull) {
            const int j = __builtin_ctzll(rm);
            act = act || (w >= rl32(kr, j) && w - rl32(kr, j) < rl32(nw, j));
          }
          act = act && w <= hi;
          if (!__ballot(act)) continue;  // uniform
          int64_t cur[MS];
          identity_v<MS>(pv, cur);
          int64_t slot = -1;
          bool isnew = false;
          uint32_t stp = 0;
          bool pending = false;  // a claim at home whose result (cas) is read at the write-back
          uint64_t cas = kEmpty;
          if (act) {
            // find (or claim) at the home slot, the home row and stamp loaded
            // with its key (the group's usual place); else probe on
            const uint64_t g = ((uint64_t)kk << 32) | (uint32_t)w;
            const uint64_t h = tw_region_base(t, g) + tw_home_in(t, g);
            int64_t hv[MS];
#pragma unroll
            for (int q = 0; q < MS; ++q)
              hv[q] = q < ns ? __hip_atomic_load(t.aggs(h) + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
            const uint32_t hst = __hip_atomic_load(t.stamp(h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            uint64_t old = __hip_atomic_load(t.key(h), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            if (old == kEmpty) {
              // claimed at home; the claim's result is waited for at the write-back
              cas = atomicCAS((unsigned long long *)t.key(h), (unsigned long long)kEmpty, (unsigned long long)g);
              pending = true;
              isnew = true;
              slot = (int64_t)h;
            } else if (old == g) {
              slot = (int64_t)h;
              stp = hst;
#pragma unroll
              for (int q = 0; q < MS; ++q) cur[q] = hv[q];
            } else {
              slot = pr_claim_row(t, g, isnew);
              if (slot < 0) {
                err |= ERR_OOM;
              } else if (!isnew) {
                const int64_t *row = t.aggs(slot);
#pragma unroll
                for (int q = 0; q < MS; ++q)
                  if (q < ns) cur[q] = __hip_atomic_load(row + q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                stp = __hip_atomic_load(t.stamp(slot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
              }
              // vmcnt(0) here (the rare path): after the branches only a home
              // claim is outstanding, and the replay does not wait for it
              __builtin_amdgcn_s_waitcnt(0x0F70);
            }
          }
          // the key's records in arrival order: fold, stage each record's rows
          lap(c_claim);
          uint32_t nst = 0;
          for (uint64_t rm = km; rm; rm &= rm - 1ull) {
            const int j = __builtin_ctzll(rm);
            const uint32_t krj = rl32(kr, j), nwj = rl32(nw, j);
            const uint64_t a = krj > wb ? krj : wb, z = (uint64_t)krj + nwj - 1 < we_ ? (uint64_t)krj + nwj - 1 : we_;
            if (a > z) continue;  // uniform: none of the record's windows in this pass
            const uint32_t cnt = (uint32_t)(z - a + 1);
            if (nst + cnt > (uint32_t)CAP) {  // uniform
              flush(nst);
              nst = 0;
            }
            int64_t ej[MS];
#pragma unroll
            for (int q = 0; q < MS; ++q) ej[q] = q < ns ? rl64(e[q], j) : 0;
            if (act && w >= a && w <= z) {
              combine_v<MS>(pv, cur, ej);
              const uint32_t q = nst + (uint32_t)(w - a);
#pragma unroll
              for (int y = 0; y < MS; ++y) st_v[y][q] = cur[y];
              st_m[q] = (uint16_t)(((uint32_t)j << 8) | (uint32_t)(w - krj));
            }
            nst += cnt;
          }
          flush(nst);
          if (pending && cas == kEmpty) t.mark(slot);  // the home claim held
          if (pending && cas != kEmpty) {
            // another key took the home slot first: the next free one (the
            // group is new: only this wave holds the key's groups)
            bool nn;
            slot = pr_claim_row(t, ((uint64_t)kk << 32) | (uint32_t)w, nn);
            if (slot < 0) err |= ERR_OOM;
          }
          if (act && slot >= 0) {
            int64_t *row = t.aggs(slot);
#pragma unroll
            for (int q = 0; q < MS; ++q)
              if (q < ns) row[q] = cur[q];
            if (stp != bid) {
              *t.stamp(slot) = bid;
              touched += 1;
            }
            fresh += isnew ? 1 : 0;
          }
          lap(c_wb);
        }
      }
      if (last) break;
      // the rows in L2 before the group's next chunk loads them again
      // (L1-bypassing loads of this wave; vmcnt counts stores on gfx9)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    gi = gnext;
  }
  if (err) atomicOr(&sc->err, err);
  const uint64_t f = wave_sum_u64(fresh), tc = wave_sum_u64(touched);
  if (kPhaseClocks && lane == 0) {  // per-wave phase clocks (HSG_PHASES builds)
    atomicAdd((unsigned long long *)&sc->scratch[24], (unsigned long long)c_head);
    atomicAdd((unsigned long long *)&sc->scratch[25], (unsigned long long)c_load);
    atomicAdd((unsigned long long *)&sc->scratch[26], (unsigned long long)c_claim);
    atomicAdd((unsigned long long *)&sc->scratch[27], (unsigned long long)c_replay);
    atomicAdd((unsigned long long *)&sc->scratch[28], (unsigned long long)c_flush);
    atomicAdd((unsigned long long *)&sc->scratch[29], (unsigned long long)c_wb);
    atomicAdd((unsigned long long *)&sc->scratch[30], 1ull);
  }
  if (lane == 0) {
    if (f) atomicAdd((unsigned long long *)&sc->live_x[blockIdx.x & 7], (unsigned long long)f);
    if (tc) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tc);
  }
}

// One-window ops: a bucket of more than kPrHot records (a very hot key) would
// serialise k_pr_bucket on one workgroup; counter[1] then sends the batch to
// the chunked path (k_pr_local / k_pr_carry / k_pr_emit over the bucket's
// arrival-order records, chunks in parallel, carries in order)
constexpr uint64_t kPrHot = 65536;
__global__ __launch_bounds__(256) void k_pr_hot(const uint64_t *bstart, int nb, const DevScalars *sc, PrPart pr) {
  if (sc->redo) return;
  uint32_t hot = 0;
  for (int b = threadIdx.x; b < nb; b += 256) hot |= bstart[b + 1] - bstart[b] > kPrHot ? 1u : 0u;
  hot = __syncthreads_or(hot);
  if (threadIdx.x == 0 && hot) pr.counter[1] = 1;
}

// k_pr_emit1's program: with a projected per-record state (hsg_internal.h
// fin_*) the outputs read the projected words, so their slot indices are
// remapped to those words' positions (fin_n / fin_form stay: they tell the
// kernel the state is projected and where the form word is)
static Program fin_outputs(const Program &prog) {
  Program q = prog;
  if (prog.fin_n == prog.n_slots && !prog.fin_form) return q;
  auto at = [&](int s) {
    for (int k = 0; k < prog.fin_n; ++k)
      if (prog.fin_slot[k] == s) return k;
    return 0;  // (an output slot is always projected: build_program)
  };
  for (int j = 0; j < prog.n_out; ++j) {
    q.out_a[j] = at(prog.out_a[j]);
    q.out_b[j] = (prog.out_kind[j] == O_AVG_I || prog.out_kind[j] == O_AVG_F) ? at(prog.out_b[j]) : 0;
  }
  return q;
}

template <int MS>
static void pr_launch(hipStream_t s, const Batch &b, const Program &prog, const TwParams &p, const PartParams &pp,
                      const TwTable &t, const PartBuffers &pb, const PrPart &pr, uint32_t wpr, const int64_t *rec_wm,
                      const int64_t *seq, const OutCols &out, uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  const uint64_t nb = 1ull << pp.np_log2;
  if (wpr == 1) {
    hipLaunchKernelGGL(k_pr_hot, dim3(1), dim3(256), 0, s, pb.bstart, (int)nb, sc, pr);
    // LDS: 10 B per table slot, 8 MS + 4 + 4 per group (half the slots), staging 2 KB per state slot
    constexpr int LT = MS <= 6 ? 10 : 9;
    const dim3 gb((unsigned)nb), tb(kPbNT);
    const uint64_t sig = program_sig(prog);
    const bool reg = pp.words <= kPrRegWords;
    // the common aggregate sets run with their slot program baked in
    bool done = false;
    if constexpr (MS == 6) {
      if (reg && sig == kSigAllI) {
        hipLaunchKernelGGL((k_pr_bucket<MS, LT, true, kSigAllI>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      } else if (reg && sig == kSigAllF) {
        hipLaunchKernelGGL((k_pr_bucket<MS, LT, true, kSigAllF>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      }
    }
    if constexpr (MS == 2) {
      if (reg && sig == kSigCnt) {
        hipLaunchKernelGGL((k_pr_bucket<MS, LT, true, kSigCnt>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      } else if (reg && sig == kSigCntSumI) {
        hipLaunchKernelGGL((k_pr_bucket<MS, LT, true, kSigCntSumI>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      } else if (reg && sig == kSigSumMaxI) {
        hipLaunchKernelGGL((k_pr_bucket<MS, LT, true, kSigSumMaxI>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      }
    }
    if constexpr (MS == 8) {
      // the SQL drop-in's C5 query (its 7 slots exactly)
      uint64_t hi = 0;
      const uint64_t sq = program_sig(prog, &hi);
      if (reg && sq == kSigSqlSumMaxI && !hi) {
        hipLaunchKernelGGL((k_pr_bucket<7, LT, true, kSigSqlSumMaxI, 0>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      }
    }
    if constexpr (MS == 12) {
      // the SQL drop-in's C2 query (literal forms, a passthrough)
      uint64_t hi = 0;
      const uint64_t sq = program_sig(prog, &hi);
      // (a 1024-slot table, one segment for C2's ~350 groups per bucket at one
      // workgroup per CU, measured no faster: 2.18 against 2.10 ms per batch)
      // (its 11 slots exactly: 52 KB of LDS, three workgroups per CU instead of two)
      if (reg && sq == kSigSqlI && hi == kSigSqlI2) {
        hipLaunchKernelGGL((k_pr_bucket<11, LT, true, kSigSqlI, kSigSqlI2>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      } else if (reg && sq == kSigSqlF && hi == kSigSqlF2) {
        hipLaunchKernelGGL((k_pr_bucket<11, LT, true, kSigSqlF, kSigSqlF2>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
        done = true;
      }
    }
    if (!done) {
      if (reg) hipLaunchKernelGGL((k_pr_bucket<MS, LT, true, 0>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
      else hipLaunchKernelGGL((k_pr_bucket<MS, LT, false, 0>), gb, tb, 0, s, prog, p, pp, t, pb, pr, sc);
    }
    const uint64_t tiles = (b.n + kPrEmitRecs - 1) / kPrEmitRecs;
    // registers for the words the rows read (a projected state: fewer than MS)
    const Program ep = fin_outputs(prog);
    const int fw = prog_fin_words(prog);
    const dim3 ge((unsigned)tiles), te(kE1NT);
#define HSG_E1(M) hipLaunchKernelGGL(k_pr_emit1<M>, ge, te, 0, s, b, ep, p, pb, pr, rec_wm, seq, out, out_base, out_cap, sc)
    if (fw <= 2 && MS >= 2) HSG_E1(2);
    else if (fw <= 4 && MS >= 4) HSG_E1(4);
    else if (fw <= 6 && MS >= 6) HSG_E1(6);
    else if (fw <= 8 && MS >= 8) HSG_E1(8);
    else HSG_E1(MS);
#undef HSG_E1
    // ... or, with a hot bucket, the chunked path over the arrival-order
    // records (each kernel returns at once otherwise)
    const uint64_t nchunks = nb + b.n / pp.chunk + 1;
    const dim3 g((unsigned)(nchunks < 4096 ? nchunks : 4096));
    PrPart pr1 = pr;
    pr1.kpos = nullptr;  // (no key grouping: a record's pairs sit at its partitioned position)
    hipLaunchKernelGGL(k_pr_local<MS>, g, dim3(kPrNT), 0, s, prog, pp, pb, pr1, wpr, sc);
    hipLaunchKernelGGL(k_pr_carry<MS>, dim3((unsigned)nb), dim3(256), 0, s, prog, p, pp, t, pb, pr1, sc);
    hipLaunchKernelGGL(k_pr_emit<MS>, ge, dim3(kPrEmitThreads), 0, s, b, prog, p, pp, pb, pr1, wpr, rec_wm, seq, out,
                       out_base, out_cap, sc);
    return;
  }
  const uint64_t nchunks = nb + b.n / pp.chunk + 1;  // >= the partition's chunks
  const dim3 g((unsigned)(nchunks < 4096 ? nchunks : 4096));
  hipLaunchKernelGGL(k_pr_keysort, dim3((unsigned)nb), dim3(kPrNT), 0, s, pp, pb, pr, sc);
  const uint64_t etiles = (b.n + kPrEmitRecs - 1) / kPrEmitRecs;
  // the key-grouped replay (returns at once when a bucket was too large) ...
  hipLaunchKernelGGL(k_pr_offs, dim3((unsigned)etiles), dim3(kPrEmitThreads), 0, s, b, p, pb, pr, rec_wm, sc);
  {
    const uint64_t sig = program_sig(prog);
    const bool reg = pp.words <= kPrRegWords;  // (the specialised programs read one column)
    const dim3 gk((unsigned)nb), tk(kPkNT);
    bool done = false;
    if constexpr (MS == 2) {
      if (reg && sig == kSigCntSumI) {
        hipLaunchKernelGGL((k_pr_keys<MS, kSigCntSumI>), gk, tk, 0, s, prog, p, pp, t, pb, pr, seq, out, out_base,
                           out_cap, sc);
        done = true;
      } else if (reg && sig == kSigCntSumF) {
        hipLaunchKernelGGL((k_pr_keys<MS, kSigCntSumF>), gk, tk, 0, s, prog, p, pp, t, pb, pr, seq, out, out_base,
                           out_cap, sc);
        done = true;
      }
    }
    if constexpr (MS == 6) {
      if (reg && sig == kSigAllI) {
        hipLaunchKernelGGL((k_pr_keys<MS, kSigAllI>), gk, tk, 0, s, prog, p, pp, t, pb, pr, seq, out, out_base,
                           out_cap, sc);
        done = true;
      } else if (reg && sig == kSigAllF) {
        hipLaunchKernelGGL((k_pr_keys<MS, kSigAllF>), gk, tk, 0, s, prog, p, pp, t, pb, pr, seq, out, out_base,
                           out_cap, sc);
        done = true;
      }
    }
    if (!done)
      hipLaunchKernelGGL((k_pr_keys<MS, 0>), gk, tk, 0, s, prog, p, pp, t, pb, pr, seq, out, out_base, out_cap, sc);
  }
  // ... or the chunked path (returns at once otherwise)
  PartBuffers kpb = pb;
  kpb.rec = pr.krec;  // the chunks read the key-grouped records
  hipLaunchKernelGGL(k_pr_local<MS>, g, dim3(kPrNT), 0, s, prog, pp, kpb, pr, wpr, sc);
  hipLaunchKernelGGL(k_pr_carry<MS>, dim3((unsigned)nb), dim3(256), 0, s, prog, p, pp, t, kpb, pr, sc);
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
  else if (prog.n_slots <= 6) pr_launch<6>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
  else if (prog.n_slots <= 8) pr_launch<8>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
  // the SQL drop-in's op shape (literal forms, a passthrough: C2's five
  // aggregates take 11 slots)
  else if (prog.n_slots <= 12) pr_launch<12>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
  else pr_launch<16>(s, b, prog, p, pp, t, pb, pr, wpr, rec_wm, seq, out, out_base, out_cap, sc);
}

}  // namespace hsg
