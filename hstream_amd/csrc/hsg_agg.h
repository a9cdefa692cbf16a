// The LDS aggregation kernel of the partitioned path (k_part_agg) and its
// device helpers, included by the per-slot-count instantiation units
// k_agg_s{2,4,6,8}.hip so the variants compile in parallel. Not ABI.
#pragma once

#include <initializer_list>
#include <type_traits>

#include "hsg_dev.h"
#include "hsg_part.h"
#include "hsg_tw.h"

namespace hsg {

// ---------------------------------------------------------------------------
// Slot-program views
// ---------------------------------------------------------------------------
// The per-record LDS update dispatches on every slot's op. Read from the
// runtime Program (ProgRT) that dispatch is a scalar branch chain per slot and
// record; a program signature baked into the kernel (ProgSig<SIG>) folds it
// to the slot's one LDS atomic. SIG packs 7 bits per slot, slot 0 lowest:
// (op + 1) in the low 4 bits, the column in the high 3; 0 ends the program.
struct ProgRT {
  const Program &p;
  __device__ explicit ProgRT(const Program &q) : p(q) {}
  __device__ int n() const { return p.n_slots; }
  __device__ int op(int s) const { return p.slot_op[s]; }
  __device__ int col(int s) const { return p.slot_col[s]; }
};

template <uint64_t SIG, uint64_t SIG2 = 0>
struct ProgSig {
  // slot s's 7-bit code: slots 0..8 in SIG, 9..17 in SIG2 (programs of more
  // than 9 slots: the SQL drop-in's shape, literal forms and a passthrough)
  static constexpr uint32_t code(int s) {
    return s < 9 ? (uint32_t)((SIG >> (7 * s)) & 127u) : (uint32_t)((SIG2 >> (7 * (s - 9))) & 127u);
  }
  static constexpr int count() {
    int k = 0;
    while (k < 18 && (code(k) & 15u) != 0) ++k;
    return k;
  }
  static constexpr int op_of(int s) { return (int)(code(s) & 15u) - 1; }
  static constexpr int col_of(int s) { return (int)((code(s) >> 4) & 7u); }
  // the MIN / MAX slot a tie-word slot breaks ties of (build_program: the
  // one MIN (MAX) slot over the same column)
  static constexpr int aux_of(int s) {
    const int want = op_of(s) == S_TIE_MIN ? 0 : 1;
    for (int k = 0; k < count(); ++k) {
      const int o = op_of(k);
      const bool mn = o == S_MIN_I || o == S_MIN_F, mx = o == S_MAX_I || o == S_MAX_F;
      if (((want == 0 && mn) || (want == 1 && mx)) && col_of(k) == col_of(s)) return k;
    }
    return 0;
  }
  // the LAST_FORM slot over the column of LAST_SEQ slot s (-1: none): its
  // word is (seq + 1) << 1 | bit over the same present records, so the
  // LAST_SEQ slot is that word >> 1 and needs no update of its own
  static constexpr int last_form_of(int s) {
    for (int k = 0; k < count(); ++k)
      if (op_of(k) == S_LAST_FORM && col_of(k) == col_of(s)) return k;
    return -1;
  }
  static constexpr bool has_ties() {
    for (int k = 0; k < count(); ++k)
      if (op_of(k) == S_TIE_MIN || op_of(k) == S_TIE_MAX) return true;
    return false;
  }
  __device__ ProgSig() {}
  __device__ explicit ProgSig(const Program &) {}
  __device__ constexpr int n() const { return count(); }
  __device__ constexpr int op(int s) const { return op_of(s); }
  __device__ constexpr int col(int s) const { return col_of(s); }
};

template <uint64_t SIG, uint64_t SIG2 = 0>
using ProgView = typename std::conditional<SIG == 0, ProgRT, ProgSig<SIG, SIG2>>::type;

// tie-word helpers over either view
__device__ inline int pv_aux(const ProgRT &pv, int s) { return pv.p.slot_aux[s]; }
__device__ inline bool pv_ties(const ProgRT &pv) { return pv.p.ties != 0; }
template <uint64_t SIG, uint64_t SIG2>
__device__ constexpr int pv_aux(const ProgSig<SIG, SIG2> &, int s) { return ProgSig<SIG, SIG2>::aux_of(s); }
template <uint64_t SIG, uint64_t SIG2>
__device__ constexpr bool pv_ties(const ProgSig<SIG, SIG2> &) { return ProgSig<SIG, SIG2>::has_ties(); }
__device__ inline int pv_last_form(const ProgRT &, int) { return -1; }
template <uint64_t SIG, uint64_t SIG2>
__device__ constexpr int pv_last_form(const ProgSig<SIG, SIG2> &, int s) { return ProgSig<SIG, SIG2>::last_form_of(s); }

// signature of a runtime program (0: not expressible); slots past the ninth
// go to *sig2 when it is given (else such a program has no signature)
inline uint64_t program_sig(const Program &p, uint64_t *sig2 = nullptr) {
  if (p.n_slots > (sig2 ? 18 : 8)) return 0;
  uint64_t sig = 0, hi = 0;
  for (int s = 0; s < p.n_slots; ++s) {
    if (p.slot_op[s] < 0 || p.slot_op[s] > 14 || p.slot_col[s] < 0 || p.slot_col[s] > 7) return 0;
    // (a tie word's MIN / MAX slot is implied: the one over its column)
    if (slot_is_tie(p.slot_op[s])) {
      const int v = p.slot_aux[s], vo = p.slot_op[v];
      const bool ok = p.slot_col[v] == p.slot_col[s] &&
                      (p.slot_op[s] == S_TIE_MIN ? (vo == S_MIN_I || vo == S_MIN_F) : (vo == S_MAX_I || vo == S_MAX_F));
      if (!ok) return 0;
    }
    const uint64_t c = (uint64_t)((p.slot_op[s] + 1) | (p.slot_col[s] << 4));
    if (s < 9) sig |= c << (7 * s);
    else hi |= c << (7 * (s - 9));
  }
  if (sig2) *sig2 = hi;
  return sig;
}

// ---------------------------------------------------------------------------
// LDS aggregation of one chunk
// ---------------------------------------------------------------------------
// One partitioned record held in registers: [w0 w1 col 0..C-1 seq+1?]. Runtime
// word selection is an unrolled compare chain, so the record never leaves VGPRs.
// One partitioned record held in registers, in its memory layout (PK: packed,
// see hsg_part.h). Runtime word selection is an unrolled compare chain, so
// the record never leaves VGPRs.
template <int WMAX, bool PK>
struct PRec {
  static constexpr int CB = PK ? 1 : 2;  // first column word
  uint64_t w[WMAX];
  int C;
  __device__ uint32_t key() const { return (uint32_t)w[0]; }
  __device__ uint32_t krel(uint32_t kbase) const {
    return PK ? kbase + (uint32_t)((w[0] >> 32) & 0xFFFFull) : (uint32_t)(w[0] >> 32);
  }
  __device__ uint32_t nwin() const { return PK ? (uint32_t)((w[0] >> 48) & 0xFFull) : (uint32_t)w[1]; }
  __device__ bool present(int c) const { return PK ? (w[0] >> (56 + c)) & 1ull : (w[1] >> (32 + c)) & 1ull; }
  __device__ int64_t word(int k) const {
    int64_t v = 0;
#pragma unroll
    for (int q = CB; q < WMAX; ++q)
      if (q == k) v = (int64_t)w[q];
    return v;
  }
  __device__ int64_t col(int c) const { return word(CB + c); }
  // the sequence word (hsg_dev.h seq_word): seq + 1, decimal-literal bits
  __device__ int64_t seq1() const { return (int64_t)((uint64_t)word(CB + C) & kSeqMask); }
  __device__ bool dec(int c) const { return ((uint64_t)word(CB + C) >> (56 + c)) & 1ull; }
};

// contribution of the record to slot s (identity when absent)
template <class PG, typename R>
__device__ inline int64_t prec_elem(const PG &prog, int s, const R &r) {
  const int op = prog.op(s);
  const int c = prog.col(s);
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
    case S_CNT_DEC: return r.dec(c) ? 1 : 0;
    case S_TIE_MIN:
    case S_TIE_MAX:
    case S_LAST_FORM: return (int64_t)(((uint64_t)r.seq1() << 1) | (r.dec(c) ? 0u : 1u));
    default: return 0;
  }
}

// LDS aggregates are slot-major: slot s of entry e at agg[s * ST + e] (ST = the
// table's entry count), so the 64 lanes of one atomic instruction spread over
// the banks (entry-major rows of 48 B hit a quarter of them). `skip`: slots not
// updated in LDS (COUNT(col) of a batch without validity arrays = COUNT(*)).
template <int MS, int ST, typename R, class PG>
__device__ inline void lds_apply(const PG &prog, int64_t *__restrict__ row, const R &r, uint32_t skip) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n()) break;
    const int op = prog.op(s);
    if (op == S_LAST_VAL || ((skip >> s) & 1u)) continue;
    if (op != S_CNT_ALL && !r.present(prog.col(s))) continue;
    const int64_t x = prec_elem(prog, s, r);
    int64_t *a = row + s * ST;
    unsigned long long *u = (unsigned long long *)a;
    // min / max: a plain read first; the atomic only when x would change the
    // value (a stale read costs an atomic that changes nothing, never a wrong
    // result), so a group's later records mostly skip the LDS atomic unit
    switch (op) {
      case S_CNT_ALL:
      case S_CNT:
      case S_SUM_I: atomicAdd(u, (unsigned long long)x); break;
      case S_SUM_F: unsafeAtomicAdd((double *)a, __builtin_bit_cast(double, x)); break;
      case S_MIN_I:
        if (x < *(volatile int64_t *)a) atomicMin((long long *)a, (long long)x);
        break;
      case S_MAX_I:
        if (x > *(volatile int64_t *)a) atomicMax((long long *)a, (long long)x);
        break;
      case S_MIN_F:
        if ((uint64_t)x < *(volatile uint64_t *)a) atomicMin(u, (unsigned long long)x);
        break;
      case S_MAX_F:
      case S_LAST_SEQ:
        if ((uint64_t)x > *(volatile uint64_t *)a) atomicMax(u, (unsigned long long)x);
        break;
      default: break;
    }
  }
}

// a <- a (+) x over the aggregate slots (LAST_SEQ = latest sequence); x strided by ST
template <int MS, int ST, class PG>
__device__ inline void acc_combine(const PG &prog, int64_t (&a)[MS], const int64_t *x) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n()) break;
    const int op = prog.op(s);
    if (op == S_LAST_VAL) continue;
    const int64_t v = x[s * ST];
    a[s] = op == S_LAST_SEQ ? ((uint64_t)v > (uint64_t)a[s] ? v : a[s]) : slot_combine(op, a[s], v);
  }
}

// HBM-side atomic combine of a row of partial aggregates (v) into `row`.
template <int MS, class PG>
__device__ inline void flush_row_atomic(const PG &prog, int64_t *__restrict__ row, const int64_t (&v)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n()) break;
    const int op = prog.op(s);
    const int64_t x = v[s];
    if (op == S_LAST_VAL || x == slot_identity_dev(op)) continue;  // nothing to add
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

// One HBM update of group g with the chunk's partial aggregate v. `exclusive`:
// this workgroup is the only one updating the group in this launch, so a plain
// read-modify-write suffices (agent-scope loads, served by L2 not L1: this
// workgroup's own atomics may have updated the row). Returns the slot when this is the group's first update
// in the batch (-> per-batch changelog), else kTouchSkip.
template <int MS, class PG>
__device__ inline uint32_t flush_window(const PG &prog, const TwParams &p, const TwTable &t, uint64_t g,
                                        const int64_t (&v)[MS], bool exclusive, uint32_t &fresh, uint32_t &err,
                                        bool plain_claim = false) {
  const uint32_t f0 = fresh;
  const int64_t slot = plain_claim ? tw_claim_exclusive(t, g, fresh) : tw_find_or_insert(t, g, fresh);
  if (slot < 0) {
    err |= ERR_OOM;
    return kTouchSkip;
  }
  int64_t *row = t.aggs(slot);
  uint32_t *stp = t.stamp(slot);
  const uint32_t bid = (uint32_t)p.batch_id;
  bool first;
  if (exclusive && fresh != f0) {
    // inserted just now by the group's only writer: the row holds identities
#pragma unroll
    for (int s = 0; s < MS; ++s)
      if (s < prog.n() && prog.op(s) != S_LAST_VAL) row[s] = v[s];
    *stp = bid;
    first = true;
  } else if (exclusive) {
    int64_t cur[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s)
      cur[s] = s < prog.n() ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    const uint32_t st = __hip_atomic_load(stp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (s >= prog.n()) break;
      const int op = prog.op(s);
      if (op == S_LAST_VAL || v[s] == slot_identity_dev(op)) continue;
      row[s] = op == S_LAST_SEQ ? ((uint64_t)v[s] > (uint64_t)cur[s] ? v[s] : cur[s]) : slot_combine(op, cur[s], v[s]);
    }
    first = st != bid;
    if (first) *stp = bid;
  } else {
    flush_row_atomic<MS>(prog, row, v);
    first = atomicExch(stp, bid) != bid;
  }
  return first ? (uint32_t)slot : kTouchSkip;
}

__device__ inline void touch_append(const PartBuffers &pb, DevScalars *sc, uint32_t slot, uint32_t &err) {
  if (slot == kTouchSkip) return;
  const uint64_t o = atomicAdd((unsigned long long *)&sc->scratch[1], 1ull);
  if (o < pb.touched_cap) pb.touched[o] = slot;
  else err |= ERR_OOM;
}

// Windows [w0, w1] of one record straight into the HBM table (records whose
// earliest windows were rejected by grace, and LDS overflow in fan-out mode).
template <int MS, typename R, class PG>
__device__ inline void direct_windows(const PG &prog, const TwParams &p, const TwTable &t, const PartBuffers &pb,
                                      DevScalars *sc, uint32_t key, uint32_t w0, uint32_t w1, const R &r,
                                      uint32_t &fresh, uint32_t &err) {
  int64_t v[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) v[s] = s < prog.n() ? prec_elem(prog, s, r) : 0;
  atomicOr((unsigned int *)&sc->scratch[5], 1u);  // updated in-kernel: the batch is not clean
  for (uint32_t w = w0;; ++w) {
    touch_append(pb, sc, flush_window<MS>(prog, p, t, ((uint64_t)key << 32) | w, v, false, fresh, err), err);
    if (w == w1) break;
  }
}

// find or insert g; -1 when g is absent and the table is at its fill limit
template <int E>
__device__ inline int lds_insert(uint64_t *lkey, uint32_t *lfill, uint32_t limit, uint64_t g) {
  uint32_t h = (uint32_t)(mix64(g) & (E - 1));
  for (int probe = 0; probe < E; ++probe) {
    const uint64_t cur = lkey[h];
    if (cur == g) return (int)h;
    if (cur == kEmpty) {
      if (*(volatile uint32_t *)lfill >= limit) return -1;
      const uint64_t old = atomicCAS((unsigned long long *)&lkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        atomicAdd(lfill, 1u);
        return (int)h;
      }
      if (old == g) return (int)h;
    }
    h = (h + 1) & (E - 1);
  }
  return -1;
}

// slot of g in the LDS table, -1 when absent
template <int E>
__device__ inline int lds_find(const uint64_t *lkey, uint64_t g) {
  uint32_t h = (uint32_t)(mix64(g) & (E - 1));
  for (int probe = 0; probe < E; ++probe) {
    const uint64_t cur = lkey[h];
    if (cur == g) return (int)h;
    if (cur == kEmpty) return -1;
    h = (h + 1) & (E - 1);
  }
  return -1;
}

// sub-round of a key: the hash bits just below its bucket bits
__device__ inline uint32_t key_round(uint32_t key, int np_log2, int rbits, int bshift) {
  if (!rbits) return 0;
  return (uint32_t)((key_hash(key) << bshift) >> (64 - np_log2 - rbits)) & ((1u << rbits) - 1u);
}

// Aggregation of one chunk of a bucket (buckets are disjoint key sets, so when
// the bucket is one chunk this workgroup owns every group it updates).
//
// Pane mode (pp.pane_S = S >= 1, size = S * advance): a record of a full window
// run only updates its pane (key, last window P) in the LDS table. At a flush
// the live panes are sorted by (key, pane) in LDS; every pane P owns the
// windows [a, P] that contain no earlier pane in the table, and window
// w = combine(panes w .. w+S-1) gets one HBM update, with the panes summed
// incrementally from the sorted neighbours (w+1 adds the panes up to w+S).
// Tumbling is S = 1 (no sort). Fan-out mode (S = 0: size not a multiple of
// advance) keeps one entry per window.
//
// The chunk is walked in register-resident sub-chunks of NT * RPT records and
// the LDS table persists across them: it is flushed when full and at the end
// of each of the 2^rbits key-hash rounds (host-sized from the previous batch so
// that a round's panes fit), so a bucket's groups are normally flushed once.
// Pane grouping at a flush: a counting sort of the live panes by key hash
// (LDS counters per hash bucket) and an insertion sort of each bucket by
// (key, pane) puts every key's panes next to each other in pane order, which
// is all the window pass needs (the key order itself is irrelevant). Tables
// whose counters do not fit next to the aggregates (8-slot programs) sort
// the whole list (bitonic) instead, as do flushes with an oversized bucket.
template <int MS, int E>
struct PaneGroup {
  static constexpr bool kCount = MS <= 6;
  uint32_t cnt[kCount ? E : 1];     // per hash bucket: count, then end offset
  uint16_t order[kCount ? E : 1];   // live entries grouped by key
};

template <int MS, int E, int NT>
struct AggLds {
  uint64_t key[E];
  int64_t agg[E * MS];
  uint8_t nw[E];     // windows of the pane's records
  uint8_t run[E];    // owned windows - 1
  uint16_t live[E];  // compacted / key-grouped live entries
  uint32_t fill, nl, b, c0, c1, maxb;
  uint32_t wsum[NT / 64];
  uint64_t base;
  uint64_t pbase;        // deferred flush: first pane entry of this flush
  uint32_t nseg, dnow;   // deferred segments so far; this flush is deferred
  uint32_t pcnt;         // deferred entries of this workgroup
  uint64_t red[2][NT / 64];
  PaneGroup<MS, E> pg;
};

// Bitonic sort of the live list by (key, pane), padded to a power of two.
template <int MS, int E, int NT>
__device__ inline void sort_live_bitonic(AggLds<MS, E, NT> &L, uint32_t nl) {
  uint32_t M = 1;
  while (M < nl) M <<= 1;
  for (uint32_t q = nl + threadIdx.x; q < M; q += NT) L.live[q] = 0xFFFFu;
  __syncthreads();
  for (uint32_t k = 2; k <= M; k <<= 1) {
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      for (uint32_t i = threadIdx.x; i < M; i += NT) {
        const uint32_t ixj = i ^ j;
        if (ixj <= i) continue;
        const uint16_t x = L.live[i], y = L.live[ixj];
        const uint64_t kx = x == 0xFFFFu ? kEmpty : L.key[x];
        const uint64_t ky = y == 0xFFFFu ? kEmpty : L.key[y];
        if ((kx > ky) == ((i & k) == 0)) {
          L.live[i] = y;
          L.live[ixj] = x;
        }
      }
      __syncthreads();
    }
  }
}

// Group the live list by key, panes ascending within a key (see PaneGroup).
template <int MS, int E, int NT>
__device__ inline void group_live(AggLds<MS, E, NT> &L, uint32_t nl) {
  if constexpr (!PaneGroup<MS, E>::kCount) {
    sort_live_bitonic<MS, E, NT>(L, nl);
  } else {
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    constexpr uint32_t PER = E / NT;  // buckets per thread
    for (uint32_t h = threadIdx.x; h < E; h += NT) L.pg.cnt[h] = 0;
    if (threadIdx.x == 0) L.maxb = 0;
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nl; q += NT) {
      const uint32_t h = (uint32_t)(mix64(L.key[L.live[q]] >> 32) & (E - 1));
      const uint32_t c = atomicAdd(&L.pg.cnt[h], 1u) + 1u;
      atomicMax(&L.maxb, c);
    }
    __syncthreads();
    if (L.maxb > 48) {  // a hot key: one long bucket would make the insertion sort quadratic
      sort_live_bitonic<MS, E, NT>(L, nl);
      return;
    }
    // exclusive scan of the bucket counts (PER consecutive buckets per thread)
    uint32_t local = 0;
    for (uint32_t k = 0; k < PER; ++k) local += L.pg.cnt[threadIdx.x * PER + k];
    const uint64_t incl = wave_incl_sum((uint64_t)local);
    if (lane == 63) L.wsum[wv] = (uint32_t)incl;
    __syncthreads();
    uint32_t run = (uint32_t)(incl - local);
    for (int k = 0; k < wv; ++k) run += L.wsum[k];
    for (uint32_t k = 0; k < PER; ++k) {
      const uint32_t h = threadIdx.x * PER + k, c = L.pg.cnt[h];
      L.pg.cnt[h] = run;  // start, advanced to the end by the scatter
      run += c;
    }
    __syncthreads();
    for (uint32_t q = threadIdx.x; q < nl; q += NT) {
      const uint16_t e = L.live[q];
      const uint32_t h = (uint32_t)(mix64(L.key[e] >> 32) & (E - 1));
      L.pg.order[atomicAdd(&L.pg.cnt[h], 1u)] = e;
    }
    __syncthreads();
    // each bucket by (key, pane): every entry counts the entries of its
    // bucket that sort before it (one thread per entry; a bucket holds a key's
    // panes, ~size / advance of them, so a serial sort per bucket would keep
    // one thread busy for the whole bucket)
    for (uint32_t q = threadIdx.x; q < nl; q += NT) {
      const uint16_t x = L.pg.order[q];
      const uint64_t kx = L.key[x];
      const uint32_t h = (uint32_t)(mix64(kx >> 32) & (E - 1));
      const uint32_t end = L.pg.cnt[h], start = h ? L.pg.cnt[h - 1] : 0u;
      uint32_t rank = 0;
      for (uint32_t j = start; j < end; ++j) rank += L.key[L.pg.order[j]] < kx;
      L.live[start + rank] = x;
    }
    __syncthreads();
  }
}

// Flush every live entry of the table as window updates, then clear it.
// Block-wide: every thread calls. Returns the number of live entries.
template <int MS, int E, int NT, class PG>
__device__ __forceinline__ uint32_t agg_flush(AggLds<MS, E, NT> &L, const PG &prog, const TwParams &p, const TwTable &t,
                              const PartBuffers &pb, DevScalars *sc, int S, bool exclusive, bool plain_claim,
                              uint32_t skip, int cnt_all_slot, uint32_t &fresh, uint32_t &err, uint64_t &t_sort,
                              bool defer) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t SW = S ? (uint32_t)S : 1u;
  const uint64_t t0 = phase_clock();
  // compact the live entries (one LDS atomic per wave)
  for (int e0 = 0; e0 < E; e0 += NT) {
    const int e = e0 + threadIdx.x;
    const bool on = L.key[e] != kEmpty;
    const uint64_t m = __ballot(on);
    uint32_t wb = 0;
    if (lane == 0 && m) wb = atomicAdd(&L.nl, (uint32_t)__popcll(m));
    wb = __shfl(wb, 0, 64);
    if (on) L.live[wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)e;
  }
  __syncthreads();
  const uint32_t nl = L.nl;
  // pane mode: a key's panes become neighbours in pane order
  if (S > 1 && nl > 1) group_live<MS, E, NT>(L, nl);
  t_sort += phase_clock() - t0;
  // owned window run of every pane: [max(P - n + 1, previous pane + 1), P];
  // each thread takes a contiguous range of the (key-grouped) live list, so
  // the window positions below follow pane order
  const uint32_t per = (nl + NT - 1) / NT;
  const uint32_t q0 = threadIdx.x * per < nl ? threadIdx.x * per : nl;
  const uint32_t q1 = q0 + per < nl ? q0 + per : nl;
  uint32_t cnt = 0;
  for (uint32_t q = q0; q < q1; ++q) {
    const int e = L.live[q];
    const uint64_t g = L.key[e];
    const uint32_t P = (uint32_t)g;
    uint32_t a = P - (L.nw[e] - 1u);
    if (S > 1 && q > 0) {
      const uint64_t gp = L.key[L.live[q - 1]];
      if ((gp >> 32) == (g >> 32) && (uint32_t)gp + 1u > a) a = (uint32_t)gp + 1u;
    }
    L.run[e] = (uint8_t)(P - a);
    cnt += P - a + 1;
  }
  // block exclusive scan of the window counts -> positions in the flush
  const uint64_t incl = wave_incl_sum((uint64_t)cnt);
  if (lane == 63) L.wsum[wv] = (uint32_t)incl;
  __syncthreads();
  uint64_t o = incl - cnt, total = 0;
  for (int k = 0; k < NT / 64; ++k) {
    if (k < wv) o += L.wsum[k];
    total += L.wsum[k];
  }
  // first window position of every pane (reusing the grouping counters), so
  // that the windows can be spread one per thread: a key's first pane in the
  // batch owns up to size / advance windows, the others one each
  constexpr bool kSpread = PaneGroup<MS, E>::kCount;
  if constexpr (kSpread) {
    uint32_t run = (uint32_t)o;
    for (uint32_t q = q0; q < q1; ++q) {
      L.pg.cnt[q] = run;
      run += L.run[L.live[q]] + 1u;
    }
  }
  if (threadIdx.x == 0) {
    // deferred to k_seg_apply when this workgroup owns the bucket and the
    // segment fits; else updated here, with touched-list entries
    uint32_t df = 0;
    uint64_t pb0 = 0;
    if (defer && total && L.nseg < (uint32_t)kMaxSeg) {
      pb0 = atomicAdd((unsigned long long *)&sc->scratch[4], (unsigned long long)total);
      df = pb0 + total <= pb.pane_cap;
    }
    if (df) {
      pb.seg[((uint64_t)blockIdx.x * kMaxSeg + L.nseg) * 2] = pb0;
      pb.seg[((uint64_t)blockIdx.x * kMaxSeg + L.nseg) * 2 + 1] = total;
      L.nseg += 1;
      L.pcnt += (uint32_t)total;
    } else if (total) {
      atomicOr((unsigned int *)&sc->scratch[5], 1u);  // updated in-kernel: the batch is not clean
    }
    L.dnow = df;
    L.pbase = pb0;
    L.base = total && !df ? atomicAdd((unsigned long long *)&sc->scratch[1], (unsigned long long)total) : 0;
  }
  __syncthreads();
  const bool dnow = L.dnow != 0;
  const uint64_t pw = 1 + (uint64_t)prog.n();  // pane entry words
  // window w of the key of pane q (w in q's run): pane q plus the key's later
  // panes up to w + SW - 1, then its update at position `at`
  auto emit_window = [&](uint32_t q, uint32_t w, uint64_t at) {
    const int e = L.live[q];
    const uint64_t g = L.key[e];
    const uint64_t kb = g & 0xFFFFFFFF00000000ull;
    int64_t v[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = L.agg[s * E + e];
    const uint64_t top = (uint64_t)w + SW - 1;
    for (uint32_t j = q + 1; S > 1 && j < nl; ++j) {
      const int f = L.live[j];
      const uint64_t gj = L.key[f];
      if ((gj & 0xFFFFFFFF00000000ull) != kb || (uint64_t)(uint32_t)gj > top) break;
      acc_combine<MS, E>(prog, v, &L.agg[f]);
    }
    if (skip) {
      // COUNT(col) slots not kept in LDS: every record of the batch has the column
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if ((skip >> s) & 1u) v[s] = v[cnt_all_slot];
    }
    if (dnow) {
      // the window's update for k_seg_apply: [g][slot 0 .. n-1]
      uint64_t *ent = pb.pane + (L.pbase + at) * pw;
      ent[0] = kb | w;
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < prog.n()) ent[1 + s] = (uint64_t)v[s];
    } else {
      const uint32_t sl = flush_window<MS>(prog, p, t, kb | w, v, exclusive, fresh, err, plain_claim);
      if (L.base + at < pb.touched_cap) pb.touched[L.base + at] = sl;
      else err |= ERR_OOM;
    }
  };
  if constexpr (kSpread) {
    // one thread per window: its pane by binary search over the positions
    for (uint32_t at = threadIdx.x; at < total; at += NT) {
      uint32_t lo = 0, hi = nl;  // last pane whose first position is <= at
      while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (L.pg.cnt[mid] <= at) lo = mid;
        else hi = mid;
      }
      const int e = L.live[lo];
      const uint32_t P = (uint32_t)L.key[e];
      emit_window(lo, P - L.run[e] + (at - L.pg.cnt[lo]), at);
    }
  } else {
    for (uint32_t q = q0; q < q1; ++q) {
      const int e = L.live[q];
      const uint32_t P = (uint32_t)L.key[e];
      for (uint32_t w = P - L.run[e];; ++w) {
        emit_window(q, w, o++);
        if (w == P) break;
      }
    }
  }
  __syncthreads();
  // clear the table
  for (uint32_t q = threadIdx.x; q < nl; q += NT) {
    const int e = L.live[q];
    L.key[e] = kEmpty;
#pragma unroll
    for (int s = 0; s < MS; ++s) L.agg[s * E + e] = s < prog.n() ? slot_identity_dev(prog.op(s)) : 0;
  }
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.nl = 0;
  }
  __syncthreads();
  return nl;
}

// 4 waves per SIMD: two 512-thread or one 1024-thread workgroup per CU (<= 128 VGPRs)
template <int MS, int E, int WMAX, int RPT, int NT, bool FAN, bool PK, uint64_t SIG>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(4))) void k_part_agg(Program prog_, TwParams p, PartParams pp, TwTable t,
                                                            PartBuffers pb, DevScalars *sc) {
  __shared__ AggLds<MS, E, NT> L;
  const ProgView<SIG> prog(prog_);
  if (sc->redo) return;  // uniform: the optimistic pass found late records
  if ((sc->packed != 0) != PK) return;  // uniform: the other layout's variant runs
  if (pp.hold) {  // uniform: the table lacks room for this batch's worst case (host grows it, runs again)
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long *)&sc->scratch[32], 2ull);
    return;
  }
  constexpr int SUB = NT * RPT;
  const int nb = 1 << pp.np_log2;
  const uint32_t *chunk_start = pb.chunk_start;
  const uint64_t t0 = phase_clock();
  if (threadIdx.x == 0) {
    // this workgroup's bucket: chunk_start[b] <= blockIdx.x < chunk_start[b + 1]
    const uint32_t bk = blockIdx.x < chunk_start[nb] ? pb.chunk_bucket[blockIdx.x] : 0;
    L.b = bk;
    L.c0 = chunk_start[bk];
    L.c1 = chunk_start[bk + 1];
    L.fill = 0;
    L.nl = 0;
    L.nseg = 0;
    L.pcnt = 0;
  }
  for (int e = threadIdx.x; e < E; e += NT) {
    L.key[e] = kEmpty;
#pragma unroll
    for (int s = 0; s < MS; ++s) L.agg[s * E + e] = s < prog.n() ? slot_identity_dev(prog.op(s)) : 0;
  }
  __syncthreads();
  if (blockIdx.x >= chunk_start[nb]) return;  // uniform: the grid is an upper bound
  const uint32_t b = L.b;
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  const uint64_t c = blockIdx.x - L.c0;
  const bool exclusive = (L.c1 - L.c0) == 1;
  // the bucket's table regions are this workgroup's alone (hsg_tw.h)
  const bool plain_claim = exclusive && pp.np_log2 <= t.rbits && pp.bshift == t.bshift;
  const uint64_t r0 = b0 + c * pp.chunk, r1 = r0 + pp.chunk < b1 ? r0 + pp.chunk : b1;
  // window updates of a bucket this workgroup owns go to k_seg_apply
  const bool defer = pp.defer && exclusive;
  const uint32_t limit = (uint32_t)(E * 3 / 4);
  const int W = PK ? pp.words - 1 : pp.words;  // words per record in memory
  const int C = pp.words - 2 - pp.has_seq;
  const uint32_t kbase = (uint32_t)sc->kbase;
  const int S = pp.pane_S;
  const int nrounds = 1 << pp.rbits;
  // without validity arrays COUNT(col) = COUNT(*): derive those slots at flush
  int cnt_all_slot = -1;
  uint32_t skip = 0;
  for (int s = 0; s < prog.n() && s < MS; ++s)
    if (prog.op(s) == S_CNT_ALL && cnt_all_slot < 0) cnt_all_slot = s;
  if (!pp.has_valid && cnt_all_slot >= 0)
    for (int s = 0; s < prog.n() && s < MS; ++s)
      if (prog.op(s) == S_CNT) skip |= 1u << s;
  const int64_t k_epoch = sc->k_epoch;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t pairs = 0, groups = 0, t_rec = 0, t_flush = 0, t_sort = 0, flushes = 0;
  uint32_t fresh = 0, err = 0;
  const uint64_t t1 = phase_clock();

  for (int round = 0; round < nrounds; ++round) {
    for (uint64_t s0 = r0; s0 < r1; s0 += SUB) {
      uint64_t ta = phase_clock();
      PRec<WMAX, PK> rr[RPT];
      auto load = [&]() {
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
          const uint64_t i = s0 + (uint64_t)u * NT + threadIdx.x;
          const bool in = i < r1;
          rr[u].C = C;
#pragma unroll
          for (int q = 0; q < WMAX; ++q) rr[u].w[q] = (in && q < W) ? pb.rec[i * W + q] : 0;
        }
      };
      load();
      uint32_t pend = 0;
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        const uint64_t i = s0 + (uint64_t)u * NT + threadIdx.x;
        if (i < r1 && (nrounds == 1 || key_round(rr[u].key(), pp.np_log2, pp.rbits, pp.bshift) == (uint32_t)round))
          pend |= 1u << u;
      }
      uint32_t dpend = 0;  // records for the direct HBM path
      for (;;) {
        // one instance of the record body (a rolled loop over a rotating register
        // queue, back in order after RPT steps): unrolling it overflowed the
        // instruction cache
#pragma unroll 1
        for (int u = 0; u < RPT; ++u) {
          const PRec<WMAX, PK> r = rr[0];
#pragma unroll
          for (int k = 0; k + 1 < RPT; ++k) rr[k] = rr[k + 1];
          rr[RPT - 1] = r;
          if (!((pend >> u) & 1u)) continue;
          const uint32_t key = r.key(), krel = r.krel(kbase), nw = r.nwin();
          if (FAN) {
            // fan-out: one entry per window, overflow straight to HBM
            pairs += nw;
            for (uint32_t j = 0; j < nw; ++j) {
              const uint64_t g = ((uint64_t)key << 32) | (uint64_t)(krel + j);
              const int e = lds_insert<E>(L.key, &L.fill, limit, g);
              if (e >= 0) {
                lds_apply<MS, E>(prog, &L.agg[e], r, skip);
                L.nw[e] = 1;
              } else {
                direct_windows<MS>(prog, p, t, pb, sc, key, krel + j, krel + j, r, fresh, err);
              }
            }
            pend &= ~(1u << u);
            continue;
          }
          if (nw == 0) {  // never written by the scatter (cannot happen; keep loops bounded)
            pend &= ~(1u << u);
            continue;
          }
          const uint32_t P = krel + nw - 1;
          const int64_t pabs = (int64_t)P + k_epoch;
          const uint32_t full = pabs + 1 < (int64_t)S ? (uint32_t)(pabs + 1) : (uint32_t)S;
          if (nw != full) {
            // some earliest windows were rejected by grace: not a whole pane;
            // straight to HBM after this loop
            dpend |= 1u << u;
            pend &= ~(1u << u);
            continue;
          }
          const int e = lds_insert<E>(L.key, &L.fill, limit, ((uint64_t)key << 32) | P);
          if (e < 0) continue;  // table full: after the next flush
          pairs += nw;
          lds_apply<MS, E>(prog, &L.agg[e], r, skip);
          L.nw[e] = (uint8_t)nw;
          pend &= ~(1u << u);
        }
        const bool more = __syncthreads_or(pend != 0);
        const uint64_t tb = phase_clock();
        t_rec += tb - ta;
        if (!more) break;
        // table full with records left: flush and go on (the records are
        // loaded again afterwards, so they hold no registers across the flush)
        groups += agg_flush<MS, E, NT>(L, prog, p, t, pb, sc, S, exclusive, plain_claim, skip, cnt_all_slot, fresh, err,
                                   t_sort, defer);
        // a mid-round flush: a group may be updated again later in the batch
        if (threadIdx.x == 0) atomicOr((unsigned int *)&sc->scratch[5], 1u);
        ++flushes;
        load();
        ta = phase_clock();
        t_flush += ta - tb;
      }
      if (!FAN && __syncthreads_or(dpend != 0)) {
        load();
#pragma unroll 1
        for (int u = 0; u < RPT; ++u) {
          const PRec<WMAX, PK> r = rr[0];
#pragma unroll
          for (int k = 0; k + 1 < RPT; ++k) rr[k] = rr[k + 1];
          rr[RPT - 1] = r;
          if (!((dpend >> u) & 1u)) continue;
          const uint32_t key = r.key(), krel = r.krel(kbase), nw = r.nwin();
          pairs += nw;
          direct_windows<MS>(prog, p, t, pb, sc, key, krel, krel + nw - 1, r, fresh, err);
        }
      }
    }
    const uint64_t tb = phase_clock();
    groups += agg_flush<MS, E, NT>(L, prog, p, t, pb, sc, S, exclusive, plain_claim, skip, cnt_all_slot, fresh, err,
                                   t_sort, defer);
    ++flushes;
    t_flush += phase_clock() - tb;
  }
  const uint64_t t3 = phase_clock();
  pairs = wave_sum_u64(pairs);
  const uint64_t fr = wave_sum_u64(fresh);
  if (lane == 0) {
    L.red[0][wv] = pairs;
    L.red[1][wv] = fr;
  }
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    // the deferred segments of this workgroup (k_seg_apply)
    pb.pane_info[2 * blockIdx.x] = L.nseg;
    pb.pane_cnt[blockIdx.x] = L.pcnt;
    uint64_t a = 0, f = 0;
    for (int k = 0; k < NT / 64; ++k) {
      a += L.red[0][k];
      f += L.red[1][k];
    }
    if (a) atomicAdd((unsigned long long *)&sc->pairs, (unsigned long long)a);
    if (f) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)f);
    if (groups) atomicAdd((unsigned long long *)&sc->scratch[0], (unsigned long long)groups);
    // phase clock (100 MHz wall clock) sums: init, records, flush, tail, workgroups
    if (kPhaseClocks) {
      const uint64_t t4 = phase_clock();
      atomicAdd((unsigned long long *)&sc->scratch[8], (unsigned long long)(t1 - t0));
      atomicAdd((unsigned long long *)&sc->scratch[9], (unsigned long long)t_rec);
      atomicAdd((unsigned long long *)&sc->scratch[10], (unsigned long long)t_flush);
      atomicAdd((unsigned long long *)&sc->scratch[11], (unsigned long long)(t4 - t3));
      atomicAdd((unsigned long long *)&sc->scratch[12], 1ull);
      atomicAdd((unsigned long long *)&sc->scratch[18], (unsigned long long)t_sort);
      atomicAdd((unsigned long long *)&sc->scratch[20], (unsigned long long)flushes);
    }
  }
}

// Aggregation variants: small = E_s entries and 512 threads (two workgroups per
// CU), big = E_l entries and 1024 threads (one per CU). Records per thread
// keep the record queue within 128 VGPRs.
template <int MS, int E, int NT, int WM, int RPT, bool FAN, uint64_t SIG = 0>
static void agg_launch_pk(hipStream_t s, dim3 g, bool maybe_packed, const Program &prog, const TwParams &p,
                          const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  const dim3 th(NT);
  hipLaunchKernelGGL((k_part_agg<MS, E, WM, RPT, NT, FAN, false, SIG>), g, th, 0, s, prog, p, pp, t, pb, sc);
  if (maybe_packed)  // the layout is decided on the device: the variant not chosen exits at once
    hipLaunchKernelGGL((k_part_agg<MS, E, WM - 1, RPT, NT, FAN, true, SIG>), g, th, 0, s, prog, p, pp, t, pb, sc);
}

// Aggregate sets with a kernel specialised on their slot program (ProgSig):
// the SQL aggregates over one numeric column that a windowed GROUP BY most
// often asks for. Every other program runs the runtime-program kernel.
constexpr uint64_t sig_ops(std::initializer_list<int> ops) {
  uint64_t sig = 0;
  int k = 0;
  for (int op : ops) sig |= (uint64_t)(op + 1) << (7 * k++);
  return sig;
}
// COUNT(*), SUM, AVG, MIN, MAX of an i64 / f64 column
constexpr uint64_t kSigAllI = sig_ops({S_CNT_ALL, S_SUM_I, S_CNT, S_MIN_I, S_MAX_I});
constexpr uint64_t kSigAllF = sig_ops({S_CNT_ALL, S_SUM_F, S_CNT, S_MIN_F, S_MAX_F});
// COUNT(*); COUNT(*), SUM; SUM, MAX
constexpr uint64_t kSigCnt = sig_ops({S_CNT_ALL});
constexpr uint64_t kSigCntSumI = sig_ops({S_CNT_ALL, S_SUM_I});
constexpr uint64_t kSigCntSumF = sig_ops({S_CNT_ALL, S_SUM_F});
constexpr uint64_t kSigSumMaxI = sig_ops({S_SUM_I, S_MAX_I});
// the SQL drop-in's C2 query, `SELECT v, COUNT(*), SUM(v), AVG(v), MIN(v),
// MAX(v)` with literal forms (build_program's slot order): the passthrough's
// LAST pair and form, COUNT(*), SUM and its decimal count, COUNT(v), MIN / MAX
// with their tie words -- eleven slots, the last two in the second word
constexpr uint64_t sig_ops_at(std::initializer_list<int> ops, int first) {
  uint64_t sig = 0;
  int k = 0;
  for (int op : ops) {
    if (k >= first && k < first + 9) sig |= (uint64_t)(op + 1) << (7 * (k - first));
    ++k;
  }
  return sig;
}
#define HSG_SQL_C2_OPS(SUM, MIN, MAX) \
  {S_LAST_SEQ, S_LAST_VAL, S_LAST_FORM, S_CNT_ALL, SUM, S_CNT_DEC, S_CNT, MIN, S_TIE_MIN, MAX, S_TIE_MAX}
constexpr uint64_t kSigSqlI = sig_ops_at(HSG_SQL_C2_OPS(S_SUM_I, S_MIN_I, S_MAX_I), 0);
constexpr uint64_t kSigSqlI2 = sig_ops_at(HSG_SQL_C2_OPS(S_SUM_I, S_MIN_I, S_MAX_I), 9);
constexpr uint64_t kSigSqlF = sig_ops_at(HSG_SQL_C2_OPS(S_SUM_F, S_MIN_F, S_MAX_F), 0);
constexpr uint64_t kSigSqlF2 = sig_ops_at(HSG_SQL_C2_OPS(S_SUM_F, S_MIN_F, S_MAX_F), 9);
#undef HSG_SQL_C2_OPS
static_assert(ProgSig<kSigSqlI, kSigSqlI2>::count() == 11 && ProgSig<kSigSqlI, kSigSqlI2>::aux_of(8) == 7 &&
                  ProgSig<kSigSqlI, kSigSqlI2>::aux_of(10) == 9,
              "SQL C2 signature");
// and its C5 query, `SELECT v, SUM(v), MAX(v)` of an i64 column: seven slots
constexpr uint64_t kSigSqlSumMaxI =
    sig_ops_at({S_LAST_SEQ, S_LAST_VAL, S_LAST_FORM, S_SUM_I, S_CNT_DEC, S_MAX_I, S_TIE_MAX}, 0);
static_assert(ProgSig<kSigSqlSumMaxI, 0>::count() == 7 && ProgSig<kSigSqlSumMaxI, 0>::aux_of(6) == 5,
              "SQL C5 signature");

// the state-slot class (k_agg_s{2,4,6,8}.hip) a program of n slots runs in
constexpr int ms_class(int n) { return n <= 2 ? 2 : n <= 4 ? 4 : n <= 6 ? 6 : 8; }

template <int MS, int E, int NT, int RPT, uint64_t SIG>
static bool agg_launch_sig(uint64_t sig, hipStream_t s, dim3 g, bool mp, const Program &prog, const TwParams &p,
                           const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  if constexpr (ms_class(ProgSig<SIG>::count()) != MS) {
    return false;
  } else {
    if (sig != SIG) return false;
    agg_launch_pk<MS, E, NT, 3, RPT, false, SIG>(s, g, mp, prog, p, pp, t, pb, sc);
    return true;
  }
}

template <int MS, int E, int NT, int RPT4>
static void agg_launch_v(hipStream_t s, dim3 g, int W, bool mp, const Program &prog, const TwParams &p,
                         const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  constexpr int R6 = RPT4 / 2 > 0 ? RPT4 / 2 : 1, R11 = RPT4 / 4 > 0 ? RPT4 / 4 : 1;
  if (pp.pane_S == 0) {
    // fan-out (size not a multiple of advance): one generic-width variant
    agg_launch_pk<MS, E, NT, kPartMaxWords, R11, true>(s, g, mp, prog, p, pp, t, pb, sc);
    return;
  }
  if (W <= 3) {
    // records of at most one column: a specialised slot program if there is one
    const uint64_t sig = program_sig(prog);
    if (agg_launch_sig<MS, E, NT, RPT4, kSigAllI>(sig, s, g, mp, prog, p, pp, t, pb, sc) ||
        agg_launch_sig<MS, E, NT, RPT4, kSigAllF>(sig, s, g, mp, prog, p, pp, t, pb, sc) ||
        agg_launch_sig<MS, E, NT, RPT4, kSigCnt>(sig, s, g, mp, prog, p, pp, t, pb, sc) ||
        agg_launch_sig<MS, E, NT, RPT4, kSigCntSumI>(sig, s, g, mp, prog, p, pp, t, pb, sc) ||
        agg_launch_sig<MS, E, NT, RPT4, kSigCntSumF>(sig, s, g, mp, prog, p, pp, t, pb, sc) ||
        agg_launch_sig<MS, E, NT, RPT4, kSigSumMaxI>(sig, s, g, mp, prog, p, pp, t, pb, sc))
      return;
    agg_launch_pk<MS, E, NT, 3, RPT4, false>(s, g, mp, prog, p, pp, t, pb, sc);
  } else if (W <= 4) agg_launch_pk<MS, E, NT, 4, RPT4, false>(s, g, mp, prog, p, pp, t, pb, sc);
  else if (W <= 6) agg_launch_pk<MS, E, NT, 6, R6, false>(s, g, mp, prog, p, pp, t, pb, sc);
  else agg_launch_pk<MS, E, NT, kPartMaxWords, R11, false>(s, g, mp, prog, p, pp, t, pb, sc);
}

template <int MS>
static void agg_launch(hipStream_t s, dim3 g, int W, bool mp, const Program &prog, const TwParams &p,
                       const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  constexpr int ES = MS <= 2 ? 2048 : 1024, EL = MS <= 2 ? 4096 : 2048;
  if (pp.big) agg_launch_v<MS, EL, 1024, 8>(s, g, W, mp, prog, p, pp, t, pb, sc);
  else agg_launch_v<MS, ES, 512, 4>(s, g, W, mp, prog, p, pp, t, pb, sc);
}

}  // namespace hsg
