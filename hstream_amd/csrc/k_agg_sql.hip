// Lean aggregation of the SQL drop-in's op shape: every windowed GROUP BY that
// genGroupByNode dispatches prints its values through objectSerde with their
// Scientific literal forms (HSG_OPF_LITERAL_FORMS: MIN / MAX fold with
// `min n x` / `max n x`, Codegen.hs:436-461) and keeps every non-aggregate
// SELECT column as a passthrough, the value of the group's last record
// (HSG_LAST, Codegen.hs:463-469). For packed one-window batches (tumbling,
// unwindowed), in two launches, as k_agg_lean.hip:
//
//   k_agg_sql    one workgroup per bucket chunk: the chunk's packed records
//                [header][column(s)][sequence word] (hsg_dev.h seq_word: the
//                record's global sequence + 1 and its decimal-literal bits)
//                into an LDS hash table, then the live groups as partials
//                [g][slot 0 .. n-1] (the op's full slot program, global
//                sequence words) in HBM-home order;
//   k_sql_apply  one workgroup per aggregation workgroup: its partials into
//                the HBM (key, window) table with the full slot algebra
//                (hsg_dev.h combine_row: tie words, the LAST pair, form
//                slots) and the per-batch changelog rows written directly.
//
// The order-dependent slots need more than one LDS atomic per slot. The
// chunk's records are taken in blocks of RB x NT, each in two phases:
//   1. atomics: counts, sums, MIN / MAX, the LAST sequence (max of seq + 1),
//      LAST_FORM (max of (seq + 1) << 1 | integral); a record that lowers a
//      MIN (raises a MAX) clears the slot's tie word -- the words of earlier
//      records belong to a value that is no longer extreme;
//   2. after a barrier, the extremes and last sequences of the block are
//      final: the record whose sequence is the group's LAST sequence writes
//      the LAST value (one writer: sequences are unique), and every record
//      whose value equals the group's MIN (MAX) folds its tie word in with an
//      atomic min (max): the earliest literal among the minima (`min n x = n`),
//      the latest among the maxima (`max n x = x`).
// A second barrier ends the block when the program has tie words (the next
// block's resets must not meet this block's tie atomics); without them a
// later block's LAST writer always writes after this block's (it passes the
// next barrier only once every thread has finished this phase). Records never
// need to arrive in order: the sequence numbers carry it.
//
// A batch this kernel cannot finish exactly -- a bucket split over several
// workgroups, or a chunk whose groups overflow the LDS table (the partials of
// one group would then have to be combined in HBM in order) -- sets
// DevScalars::scratch[35]: k_sql_apply then changes nothing, and the host
// runs the batch on the careful path (k_window.hip's record kernels).
#include <cstring>
#include <type_traits>

#include "hsg_agg.h"

namespace hsg {

// LDS home of (key, window): the lean kernel's (k_agg_lean.hip lean_home)
template <int E>
__device__ inline uint32_t sql_home(uint32_t key, uint32_t w) {
  constexpr int LOG2E = __builtin_ctz(E);
  uint32_t h = key * 0x9E3779B1u + w * 0x85EBCA77u;
  h ^= (h >> 16) * 0x7FEB352Du;
  return h >> (32 - LOG2E);
}

// key-hash round of (key, window) among 2^rb (bits independent of sql_home's)
__device__ inline uint32_t sql_round(uint32_t key, uint32_t w, int rb) {
  uint32_t h = key * 0x85EBCA6Bu ^ w * 0xC2B2AE35u;
  h ^= h >> 13;
  h *= 0x27D4EB2Du;
  h ^= h >> 15;
  return h >> (32 - rb);
}

constexpr int kSqlSortBins = 1024;
// a partial's HBM home row bin (k_agg_lean.hip lean_sort_bin)
__device__ inline uint32_t sql_sort_bin(const TwTable &t, const PartParams &pp, uint64_t g) {
  const uint64_t slot = tw_region_base(t, g) + tw_home_in(t, g);
  const int cl = 64 - __builtin_clzll(t.mask);
  const int span = pp.np_log2 <= t.rbits ? cl - pp.np_log2 : cl - t.rbits;
  const uint64_t local = slot & ((1ull << span) - 1);
  return span > 10 ? (uint32_t)(local >> (span - 10)) : (uint32_t)local;
}

// chunk of this workgroup (k_agg_lean.hip lean_chunk)
__device__ inline bool sql_chunk(const PartParams &pp, const PartBuffers &pb, uint64_t &r0, uint64_t &r1,
                                 bool &exclusive) {
  const int nb = 1 << pp.np_log2;
  if (blockIdx.x >= pb.chunk_start[nb]) return false;
  const uint32_t b = pb.chunk_bucket[blockIdx.x];
  const uint32_t c0 = pb.chunk_start[b], c1 = pb.chunk_start[b + 1];
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  r0 = b0 + (uint64_t)(blockIdx.x - c0) * pp.chunk;
  r1 = r0 + pp.chunk < b1 ? r0 + pp.chunk : b1;
  exclusive = c1 - c0 == 1;
  return true;
}

// LDS columns of the state slots. A runtime program keeps one column per
// slot. A baked program (the SQL C2 query) packs its counts -- COUNT(*),
// COUNT(col), the SUM's decimal count, each < 2^21 in a chunk of <= 2^15
// records -- into one column updated by one atomic, and keeps no LAST
// sequence column (that word is the LAST_FORM word >> 1): 8 columns instead
// of 11, so a 2048-entry table fits the LDS beside its keys.
template <class PV>
struct SqlLay {
  static constexpr bool kPacked = false;
  static constexpr int ncols(int ms) { return ms; }
  __device__ static int col(const PV &, int s) { return s; }
  __device__ static int field(const PV &, int) { return -1; }
  __device__ static bool derived(const PV &, int) { return false; }
};
template <uint64_t A, uint64_t B>
struct SqlLay<ProgSig<A, B>> {
  using P = ProgSig<A, B>;
  static constexpr bool kPacked = true;
  static constexpr int field_of(int s) {
    return P::op_of(s) == S_CNT_ALL ? 0 : P::op_of(s) == S_CNT ? 1 : P::op_of(s) == S_CNT_DEC ? 2 : -1;
  }
  static constexpr bool derived_of(int s) { return P::op_of(s) == S_LAST_SEQ && P::last_form_of(s) >= 0; }
  static constexpr int col_of(int s) {
    if (field_of(s) >= 0) return 0;
    if (derived_of(s)) return -1;
    int c = 1;
    for (int k = 0; k < s; ++k)
      if (field_of(k) < 0 && !derived_of(k)) ++c;
    return c;
  }
  static constexpr int ncols(int) {
    int c = 1;
    for (int k = 0; k < P::count(); ++k)
      if (field_of(k) < 0 && !derived_of(k)) ++c;
    return c;
  }
  static constexpr bool packable() {  // one slot of each count op at most
    int n[3] = {0, 0, 0};
    for (int k = 0; k < P::count(); ++k)
      if (field_of(k) >= 0) ++n[field_of(k)];
    return n[0] <= 1 && n[1] <= 1 && n[2] <= 1;
  }
  __device__ static constexpr int col(const P &, int s) { return col_of(s); }
  __device__ static constexpr int field(const P &, int s) { return field_of(s); }
  __device__ static constexpr bool derived(const P &, int s) { return derived_of(s); }
};
static_assert(SqlLay<ProgSig<kSigSqlI, kSigSqlI2>>::ncols(12) == 8 && SqlLay<ProgSig<kSigSqlI, kSigSqlI2>>::packable(),
              "SQL C2 LDS layout");
static_assert(SqlLay<ProgSig<kSigSqlSumMaxI, 0>>::ncols(8) == 6 && SqlLay<ProgSig<kSigSqlSumMaxI, 0>>::packable(),
              "SQL C5 LDS layout");
constexpr int kCntBits = 21;

// phase 1 of one record on LDS entry e (column-major, ST entries per column)
template <int MS, int ST, int W, class PV>
__device__ inline void sql_phase1(const PV &pv, int64_t *__restrict__ agg, const PRec<W, true> &r,
                                  uint32_t skip) {
  using Lay = SqlLay<PV>;
  if constexpr (Lay::kPacked) {
    // every count slot in one atomic on column 0
    uint64_t add = 0;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (s >= pv.n()) break;
      const int f = Lay::field(pv, s), c = pv.col(s);
      if (f == 0) add += 1ull;
      if (f == 1 && r.present(c)) add += 1ull << kCntBits;
      if (f == 2 && r.present(c) && r.dec(c)) add += 1ull << (2 * kCntBits);
    }
    if (add) atomicAdd((unsigned long long *)agg, (unsigned long long)add);
  }
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= pv.n()) break;
    const int op = pv.op(s);
    if (op == S_LAST_VAL || slot_is_tie(op) || ((skip >> s) & 1u)) continue;
    if (Lay::field(pv, s) >= 0 || Lay::derived(pv, s)) continue;  // (packed counts / derived LAST sequence)
    if (op == S_LAST_SEQ && pv_last_form(pv, s) >= 0) continue;  // derived from the LAST_FORM word
    const int c = pv.col(s);
    if (op != S_CNT_ALL && !r.present(c)) continue;
    int64_t *a = agg + Lay::col(pv, s) * ST;
    unsigned long long *u = (unsigned long long *)a;
    switch (op) {
      case S_CNT_ALL:
      case S_CNT: atomicAdd(u, 1ull); break;
      case S_CNT_DEC:
        if (r.dec(c)) atomicAdd(u, 1ull);
        break;
      case S_SUM_I: atomicAdd(u, (unsigned long long)r.col(c)); break;
      case S_SUM_F: unsafeAtomicAdd((double *)a, __builtin_bit_cast(double, r.col(c))); break;
      case S_LAST_SEQ: {
        const uint64_t x = (uint64_t)r.seq1();
        if (x > *(volatile uint64_t *)a) atomicMax(u, (unsigned long long)x);
        break;
      }
      case S_LAST_FORM: {
        const uint64_t x = ((uint64_t)r.seq1() << 1) | (r.dec(c) ? 0u : 1u);
        if (x > *(volatile uint64_t *)a) atomicMax(u, (unsigned long long)x);
        break;
      }
      default: {
        // MIN / MAX (i64, or the order-preserving image of an f64): a plain
        // read first, the atomic only when x would change the value; a record
        // that lowers a MIN (raises a MAX) resets the slot's tie words
        const int64_t v = r.col(c);
        const uint64_t x = (op == S_MIN_F || op == S_MAX_F) ? f64_ord(__builtin_bit_cast(double, v)) : (uint64_t)v;
        bool moved = false;
        if (op == S_MIN_I) {
          if ((int64_t)x < *(volatile int64_t *)a) moved = atomicMin((long long *)a, (long long)x) > (long long)x;
        } else if (op == S_MAX_I) {
          if ((int64_t)x > *(volatile int64_t *)a) moved = atomicMax((long long *)a, (long long)x) < (long long)x;
        } else if (op == S_MIN_F) {
          if (x < *(volatile uint64_t *)a) moved = atomicMin(u, (unsigned long long)x) > x;
        } else if (op == S_MAX_F) {
          if (x > *(volatile uint64_t *)a) moved = atomicMax(u, (unsigned long long)x) < x;
        }
        // (to "no word yet": above every word for a MIN's atomic min -- its
        // identity, seq 0, is the initial value's word and would win every
        // tie -- below every word for a MAX's atomic max)
        if (moved && pv_ties(pv)) {
#pragma unroll
          for (int k = 0; k < MS; ++k)
            if (k < pv.n() && slot_is_tie(pv.op(k)) && pv_aux(pv, k) == s)
              agg[Lay::col(pv, k) * ST] = pv.op(k) == S_TIE_MIN ? (int64_t)~0ull : 0;
        }
        break;
      }
    }
  }
}

// phase 2: the LAST value of the group's last record, the tie words of the
// records holding the group's extreme
template <int MS, int ST, int W, class PV>
__device__ inline void sql_phase2(const PV &pv, int64_t *__restrict__ agg, const PRec<W, true> &r) {
  using Lay = SqlLay<PV>;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= pv.n()) break;
    const int op = pv.op(s);
    const int c = pv.col(s);
    if (op == S_LAST_VAL) {
      // the preceding slot is its LAST_SEQ (build_program last_pair)
      const int lf = s > 0 ? pv_last_form(pv, s - 1) : -1;
      const uint64_t last =
          lf >= 0 ? (uint64_t)agg[Lay::col(pv, lf) * ST] >> 1 : (uint64_t)agg[Lay::col(pv, s - 1) * ST];
      if (s > 0 && r.present(c) && last == (uint64_t)r.seq1()) agg[Lay::col(pv, s) * ST] = r.col(c);
    } else if (slot_is_tie(op)) {
      if (!r.present(c)) continue;
      const int v = pv_aux(pv, s), vop = pv.op(v);
      const int64_t x = r.col(c);
      const int64_t xv = (vop == S_MIN_F || vop == S_MAX_F) ? (int64_t)f64_ord(__builtin_bit_cast(double, x)) : x;
      if (agg[Lay::col(pv, v) * ST] != xv) continue;
      const uint64_t w = ((uint64_t)r.seq1() << 1) | (r.dec(c) ? 0u : 1u);
      unsigned long long *u = (unsigned long long *)(agg + Lay::col(pv, s) * ST);
      if (op == S_TIE_MIN) atomicMin(u, (unsigned long long)w);
      else atomicMax(u, (unsigned long long)w);
    }
  }
}

// one record's contribution to every slot, as a partial of its own (a record
// whose group found no room in the chunk's LDS table): the state of a group
// holding only this record
template <int MS, int W, class PV>
__device__ inline void sql_elems(const PV &pv, const PRec<W, true> &r, uint32_t skip, int64_t (&v)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    v[s] = 0;
    if (s >= pv.n()) continue;
    const int op = pv.op(s), c = pv.col(s);
    if (op == S_CNT_ALL || ((skip >> s) & 1u)) {  // (skip: COUNT(col) without validity arrays)
      v[s] = 1;
      continue;
    }
    if (!r.present(c)) {
      v[s] = slot_identity_dev(op);
      continue;
    }
    const int64_t x = r.col(c);
    const uint64_t w = ((uint64_t)r.seq1() << 1) | (r.dec(c) ? 0u : 1u);
    switch (op) {
      case S_CNT: v[s] = 1; break;
      case S_CNT_DEC: v[s] = r.dec(c) ? 1 : 0; break;
      case S_MIN_F:
      case S_MAX_F: v[s] = (int64_t)f64_ord(__builtin_bit_cast(double, x)); break;
      case S_LAST_SEQ: v[s] = r.seq1(); break;
      case S_LAST_FORM:
      case S_TIE_MIN:
      case S_TIE_MAX: v[s] = (int64_t)w; break;
      default: v[s] = x; break;  // SUM, MIN / MAX (i64), LAST_VAL
    }
  }
}

template <int MS, int E, int NT, int W, uint64_t SIG = 0, uint64_t SIG2 = 0>
__global__ __launch_bounds__(NT) void k_agg_sql(Program prog, PartParams pp, TwTable t, PartBuffers pb,
                                                DevScalars *sc) {
  const ProgView<SIG, SIG2> pv(prog);  // the SQL C2 query's slot program baked in (else the runtime one)
  constexpr int RB = 4;  // records per thread per block (one block in flight beside it)
  __shared__ uint64_t lkey[E];
  using Lay = SqlLay<ProgView<SIG, SIG2>>;
  constexpr int NC = Lay::ncols(MS);  // LDS columns
  __shared__ int64_t lagg[NC * E];
  __shared__ uint32_t s_cnt, s_ovf, s_fill, s_full;
  __shared__ uint32_t s_bin[kSqlSortBins];
  __shared__ uint32_t s_wsum[NT / 64];
  if (sc->redo || !sc->packed) return;  // uniform: the careful path runs the batch
  uint64_t r0, r1;
  bool exclusive;
  if (!sql_chunk(pp, pb, r0, r1, exclusive)) return;  // uniform
  const int ns = pv.n();
  const int PW = 1 + ns;  // partial words
  const int C = W - 2;    // packed: header, C columns, sequence word
  const uint32_t kbase = (uint32_t)sc->kbase;
  uint64_t *const pane = pb.pane + r0 * (uint64_t)PW;
  // (a bucket split over workgroups, or a record of a chunk whose LDS table is
  // full: several partials of one group, which k_sql_apply combines under the
  // row's lock)
  // without validity arrays COUNT(col) = COUNT(*): not kept in LDS
  int cnt_all_slot = -1;
  uint32_t skip = 0;
  for (int s = 0; s < ns && s < MS; ++s)
    if (pv.op(s) == S_CNT_ALL && cnt_all_slot < 0) cnt_all_slot = s;
  if (!pp.has_valid && cnt_all_slot >= 0)
    for (int s = 0; s < ns && s < MS; ++s)
      if (pv.op(s) == S_CNT) skip |= 1u << s;
  bool two = pv_ties(pv), need2 = pv_ties(pv);
  for (int s = 0; s < ns && s < MS; ++s) need2 |= pv.op(s) == S_LAST_VAL;
  // key-hash rounds: round k takes the groups whose round hash is k (one
  // pass over the chunk's records each), so a chunk with more groups than
  // the LDS table holds still gives one partial per group; the host's hint
  // (pp.rbits, from the last batch's groups per bucket) sets the first split,
  // a round whose groups overflow the table is split in two and run again
  constexpr int kMaxRb = 6;
  int rb = pp.rbits < kMaxRb ? pp.rbits : kMaxRb;
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_ovf = 0;
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t round = 0;
  while (round < (1u << rb)) {  // uniform
    for (int k = threadIdx.x; k < kSqlSortBins; k += NT) s_bin[k] = 0;
    for (int e = threadIdx.x; e < E; e += NT) {
      lkey[e] = kEmpty;
#pragma unroll
      for (int s = 0; s < MS; ++s) {
        if (s >= ns || Lay::derived(pv, s)) continue;
        lagg[Lay::col(pv, s) * E + e] = Lay::field(pv, s) >= 0 ? 0 : slot_identity_dev(pv.op(s));
      }
    }
    if (threadIdx.x == 0) {
      s_fill = 0;
      s_full = 0;
    }
    __syncthreads();
    const bool last_try = rb >= kMaxRb;  // (then a record that finds no room is a partial of its own)

    // records: block k holds records r0 + k*RB*NT + u*NT + tid; the next block's
    // loads are issued before the current one is processed (k_agg_lean.hip)
    PRec<W, true> rec[RB], nxt[RB];
    auto load = [&](uint64_t s0, PRec<W, true>(&d)[RB]) {
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        const uint64_t i = s0 + (uint64_t)u * NT + threadIdx.x;
        d[u].C = C;
#pragma unroll
        for (int q = 0; q < W; ++q) d[u].w[q] = i < r1 ? pb.rec[i * W + q] : 0;
        if (i >= r1) d[u].w[0] = kEmpty;
      }
    };
    load(r0, rec);
    for (uint64_t s0 = r0; s0 < r1; s0 += (uint64_t)RB * NT) {
      const bool more = s0 + (uint64_t)RB * NT < r1;  // uniform
      if (more) load(s0 + (uint64_t)RB * NT, nxt);
      int ent[RB];
      // phase 1
#pragma unroll
      for (int u = 0; u < RB; ++u) {
        ent[u] = -1;
        const PRec<W, true> &r = rec[u];
        if (r.w[0] == kEmpty) continue;
        const uint32_t key = r.key(), kw = r.krel(kbase);
        if (rb && sql_round(key, kw, rb) != round) continue;  // another round's group
        const uint64_t g = ((uint64_t)key << 32) | kw;
        uint32_t h = sql_home<E>(key, kw);
        for (int probe = 0; probe < E; ++probe) {
          const uint64_t c = lkey[h];
          if (c == g) {
            ent[u] = (int)h;
            break;
          }
          if (c == kEmpty) {
            if (*(volatile uint32_t *)&s_fill >= (uint32_t)(E - E / 8)) break;  // full: g is not in the table
            const uint64_t old =
                atomicCAS((unsigned long long *)&lkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
            if (old == kEmpty) atomicAdd(&s_fill, 1u);
            if (old == kEmpty || old == g) {
              ent[u] = (int)h;
              break;
            }
          }
          h = (h + 1) & (E - 1);
        }
        if (ent[u] >= 0) {
          sql_phase1<MS, E, W>(pv, &lagg[ent[u]], r, skip);
        } else if (!last_try) {
          s_full = 1;  // this round is split and run again
        } else {
          // no finer split left: this record is a partial of its own
          int64_t v[MS];
          sql_elems<MS, W>(pv, r, skip, v);
          const uint32_t q = atomicAdd(&s_cnt, 1u);
          uint64_t *o = pane + (uint64_t)q * PW;
          o[0] = g;
#pragma unroll
          for (int s = 0; s < MS; ++s)
            if (s < ns) o[1 + s] = (uint64_t)v[s];
          s_ovf = 1;
        }
      }
      if (need2) {
        lds_barrier();
        // phase 2
#pragma unroll
        for (int u = 0; u < RB; ++u)
          if (ent[u] >= 0) sql_phase2<MS, E, W>(pv, &lagg[ent[u]], rec[u]);
        if (two) lds_barrier();
      }
      if (more) {
#pragma unroll
        for (int u = 0; u < RB; ++u) rec[u] = nxt[u];
      }
    }
    __syncthreads();
    if (s_full) {  // uniform (read after the barrier): nothing of this round was written
      rb += 1;
      round *= 2;
      __syncthreads();  // every thread has read s_full before the reset above rewrites it
      continue;
    }
    // LAST_SEQ slots kept only through their LAST_FORM word (a runtime
    // program's column; the packed layout has none: the flush derives it)
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (Lay::kPacked || s >= ns || pv.op(s) != S_LAST_SEQ) continue;
      const int lf = pv_last_form(pv, s);
      if (lf < 0) continue;
      for (int e = threadIdx.x; e < E; e += NT) lagg[s * E + e] = (int64_t)((uint64_t)lagg[lf * E + e] >> 1);
    }

    // live entries -> partials, in the order of their HBM home rows (counting
    // sort over kSqlSortBins bins), after the partials written so far
    constexpr int PER = E / NT;
    uint32_t bin[PER], rank[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const uint64_t g = lkey[k * NT + threadIdx.x];
      bin[k] = g != kEmpty ? sql_sort_bin(t, pp, g) : ~0u;
      rank[k] = g != kEmpty ? atomicAdd(&s_bin[bin[k]], 1u) : 0u;
    }
    __syncthreads();
    constexpr int BPT = kSqlSortBins / NT > 0 ? kSqlSortBins / NT : 1;
    uint32_t loc = 0;
    if (threadIdx.x * BPT < kSqlSortBins) {
#pragma unroll
      for (int k = 0; k < BPT; ++k) loc += s_bin[threadIdx.x * BPT + k];
    }
    const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)loc);
    if (lane == 63) s_wsum[wv] = incl;
    __syncthreads();
    uint32_t run = incl - loc + s_cnt;
    for (int k = 0; k < wv; ++k) run += s_wsum[k];
    uint32_t live = 0;
    for (int k = 0; k < NT / 64; ++k) live += s_wsum[k];
    __syncthreads();
    if (threadIdx.x * BPT < kSqlSortBins) {
#pragma unroll
      for (int k = 0; k < BPT; ++k) {
        const uint32_t c = s_bin[threadIdx.x * BPT + k];
        s_bin[threadIdx.x * BPT + k] = run;
        run += c;
      }
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      if (bin[k] == ~0u) continue;
      const int e = k * NT + threadIdx.x;
      const uint32_t q = s_bin[bin[k]] + rank[k];
      uint64_t *o = pane + (uint64_t)q * PW;
      o[0] = lkey[e];
      if constexpr (Lay::kPacked) {
        const uint64_t cw = (uint64_t)lagg[e];  // the packed counts (column 0)
#pragma unroll
        for (int s = 0; s < MS; ++s) {
          if (s >= ns) continue;
          const int f = Lay::field(pv, s);
          uint64_t x;
          if (f >= 0) x = (cw >> (kCntBits * f)) & ((1ull << kCntBits) - 1);
          else if (Lay::derived(pv, s)) x = (uint64_t)lagg[Lay::col(pv, pv_last_form(pv, s)) * E + e] >> 1;
          else x = (uint64_t)lagg[Lay::col(pv, s) * E + e];
          o[1 + s] = x;
        }
      } else {
        const int64_t call = cnt_all_slot >= 0 ? lagg[cnt_all_slot * E + e] : 0;
#pragma unroll
        for (int s = 0; s < MS; ++s)
          if (s < ns) o[1 + s] = (uint64_t)(((skip >> s) & 1u) ? call : lagg[s * E + e]);
      }
    }
    __syncthreads();  // the flush has read the table (and s_cnt)
    if (threadIdx.x == 0) s_cnt += live;
    ++round;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint32_t total = s_cnt;
    atomicAdd((unsigned long long *)&sc->scratch[31], (unsigned long long)total);  // the apply's room check
    // count | record partials << 31 | split bucket << 30: a workgroup with
    // either applies under the rows' locks, and the batch's changelog then
    // comes from the touched list
    const uint32_t fl = (s_ovf ? 1u << 31 : 0u) | (exclusive ? 0u : 1u << 30);
    pb.pane_info[2 * blockIdx.x] = r0;
    pb.pane_info[2 * blockIdx.x + 1] = (uint64_t)total | ((uint64_t)fl << 32);
    pb.pane_cnt[blockIdx.x] = total | fl;
  }
}

// One workgroup per aggregation workgroup: its partials into the HBM table.
// A workgroup whose bucket is its own and which wrote no record partials has
// exactly one partial per group, so each thread owns its group's row: find or
// claim it (the bucket's regions are this workgroup's; claims arbitrated in an
// LDS claim set when the region bits allow, k_agg_lean.hip), combine with the
// full slot algebra and write the row. Otherwise (a split bucket, a chunk
// whose LDS table filled) several partials of one group meet here, from this
// and other workgroups: each is combined into the row under the row's lock
// (the high half of its stamp word), with agent-scope loads and stores (no
// stale L2 line across XCDs) and an order-free combine (the LAST pair by its
// sequence, tie words by their rule, the rest commutative). When every
// workgroup is of the first kind the changelog rows are written here;
// otherwise each partial leaves a touched-list entry (the group's slot on its
// first update of the batch, by the stamp) and the emit chain writes them.
constexpr int kSqlClaimSet = 4096;
__device__ inline bool sql_claim_insert(uint32_t *cset, uint32_t slot) {
  uint32_t h = (slot * 0x9E3779B1u) >> (32 - 12);
  for (int probe = 0; probe < kSqlClaimSet; ++probe) {
    const uint32_t old = atomicCAS(&cset[h], 0u, slot + 1u);
    if (old == 0u) return true;
    if (old == slot + 1u) return false;
    h = (h + 1) & (kSqlClaimSet - 1);
  }
  return false;
}

__device__ inline int64_t sql_claim_lds(const TwTable &t, uint64_t g, uint32_t *cset, uint32_t &fresh) {
  const uint64_t base = tw_region_base(t, g);
  uint64_t s = tw_home_in(t, g);
  const uint64_t step = tw_step(t), n = (t.rmask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    const uint64_t cur = *t.key(base + s);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty && sql_claim_insert(cset, (uint32_t)(base + s))) {
      *t.key(base + s) = g;
      t.mark(base + s);
      fresh += 1;
      return (int64_t)(base + s);
    }
    s = (s + step) & t.rmask;
  }
  return tw_ovf_claim(t, g, fresh);  // the region's sub-table is full
}

// a <- a (+) e in any order: combine_row with the LAST pair kept by sequence
template <int MS>
__device__ inline void sql_combine_any(const Program &prog, int64_t (&a)[MS], const int64_t (&e)[MS]) {
  int64_t f[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) f[s] = e[s];
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s + 1 < MS && s < prog.n_slots && prog.slot_op[s] == S_LAST_SEQ && (uint64_t)e[s] <= (uint64_t)a[s]) {
      f[s] = 0;  // combine_row then keeps a's pair
      f[s + 1] = 0;
    }
  combine_row<MS>(prog, a, f);
}

template <int MS>
__global__ __launch_bounds__(256) void k_sql_apply(Program prog, TwParams p, PartParams pp, TwTable t, PartBuffers pb,
                                                   OutCols out, uint64_t out_base, uint64_t out_cap,
                                                   DevScalars *sc) {
  __shared__ uint64_t s_red[4], s_tot[4];
  __shared__ uint32_t s_fl[4];
  __shared__ uint32_t cset[kSqlClaimSet];
  if (sc->redo || !sc->packed || sc->scratch[35]) return;  // uniform: the careful path runs the batch
  // the batch's groups (at most its partials) may not fit the table at the
  // load it is sized for: nothing is claimed, the host grows the table and
  // runs the batch again (uniform: k_agg_sql has finished)
  if (sc->scratch[31] > pp.room) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long *)&sc->scratch[32], 1ull);
    return;
  }
  uint64_t r0, r1;
  bool exclusive;
  if (!sql_chunk(pp, pb, r0, r1, exclusive)) return;  // uniform
  const int ns = prog.n_slots;
  const uint64_t PW = 1 + (uint64_t)ns;
  const uint64_t base = pb.pane_info[2 * blockIdx.x];
  const uint32_t cnt = (uint32_t)pb.pane_info[2 * blockIdx.x + 1];
  const bool shared = (pb.pane_info[2 * blockIdx.x + 1] >> 62) != 0;  // record partials or a split bucket
  const bool plain_claim = !shared && pp.np_log2 <= t.rbits && pp.bshift == t.bshift;
  const bool lds_claim = plain_claim && cnt <= kSqlClaimSet / 2 && t.mask < 0xFFFFFFFFull;
  if (lds_claim)
    for (int k = threadIdx.x; k < kSqlClaimSet; k += 256) cset[k] = 0;
  // every workgroup's partial count: this one's changelog / touched-list
  // position, the total, and whether any workgroup shares groups
  const int nb = 1 << pp.np_log2;
  const uint32_t nch = pb.chunk_start[nb];
  uint64_t before = 0, total = 0;
  uint32_t anyfl = 0;
  for (uint32_t k = threadIdx.x; k < nch; k += 256) {
    const uint32_t w = pb.pane_cnt[k];
    const uint64_t c = w & 0x3FFFFFFFu;
    anyfl |= w >> 30;
    total += c;
    if (k < blockIdx.x) before += c;
  }
  before = wave_sum_u64(before);
  total = wave_sum_u64(total);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) anyfl |= __shfl_xor(anyfl, o, 64);
  if ((threadIdx.x & 63) == 0) {
    s_red[threadIdx.x >> 6] = before;
    s_tot[threadIdx.x >> 6] = total;
    s_fl[threadIdx.x >> 6] = anyfl;
  }
  __syncthreads();
  before = s_red[0] + s_red[1] + s_red[2] + s_red[3];
  total = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
  const bool direct = (s_fl[0] | s_fl[1] | s_fl[2] | s_fl[3]) == 0;  // uniform over the batch
  const bool has_out = out.key != nullptr;
  if (threadIdx.x == 0 && blockIdx.x + 1 == nch) {
    // last workgroup: batch totals (every placed record updates one group)
    if (direct) {
      sc->scratch[1] = 0;
      sc->scratch[3] = has_out ? total : 0;
      sc->scratch[2] = 1;
    } else {
      sc->scratch[1] = total;  // the touched list: one entry per partial
      sc->scratch[3] = 0;
      sc->scratch[2] = 2;
    }
    sc->scratch[0] = total;
    sc->pairs = pb.bstart[nb];
  }
  const int64_t k_epoch = sc->k_epoch;
  __syncthreads();
  const uint64_t *pane = pb.pane + base * PW;
  const uint32_t bid = (uint32_t)p.batch_id;
  uint32_t fresh = 0, err = 0;
  for (uint32_t q = threadIdx.x; q < cnt; q += 256) {
    const uint64_t *ent = pane + (uint64_t)q * PW;
    const uint64_t g = ent[0];
    int64_t v[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = s < ns ? (int64_t)ent[1 + s] : 0;
    const uint32_t f0 = fresh;
    const int64_t slot = lds_claim ? sql_claim_lds(t, g, cset, fresh)
                         : plain_claim ? tw_claim_exclusive(t, g, fresh)
                                       : tw_find_or_insert(t, g, fresh);
    if (slot < 0) {
      err |= ERR_OOM;
      if (!direct) pb.touched[before + q] = kTouchSkip;
      continue;
    }
    int64_t *row = t.aggs(slot);
    uint32_t *stp = t.stamp(slot);
    bool first = true;
    if (shared) {
      // under the row's lock: one holder at a time, and a lane that takes it
      // finishes and releases it in the same pass (lanes of one wave never
      // wait on each other)
      // (a done flag, not a break out of the loop: the critical section must
      // stay inside the loop, where the compiler cannot move it past the
      // spinning lanes; a bound on the passes turns a lost lock into an error
      // instead of a hang)
      uint32_t *lk = stp + 1;
      bool done = false;
      for (uint32_t pass = 0; !done; ++pass) {
        if (pass > (1u << 24)) {
          err |= ERR_OOM;
          break;
        }
        if (atomicCAS(lk, 0u, 1u) == 0u) {
          int64_t c[MS];
#pragma unroll
          for (int s = 0; s < MS; ++s)
            c[s] = s < ns ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
          sql_combine_any<MS>(prog, c, v);
#pragma unroll
          for (int s = 0; s < MS; ++s)
            if (s < ns) __hip_atomic_store(row + s, c[s], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          first = __hip_atomic_load(stp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != bid;
          if (first) __hip_atomic_store(stp, bid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the row's stores before the release
          atomicExch(lk, 0u);
          done = true;
        }
      }
    } else {
      if (fresh == f0) {
        // an existing group (its window's earlier batches): the row first, then
        // this batch's partial (later in arrival order)
        int64_t c[MS];
#pragma unroll
        for (int s = 0; s < MS; ++s) c[s] = s < ns ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        combine_row<MS>(prog, c, v);
#pragma unroll
        for (int s = 0; s < MS; ++s) v[s] = c[s];
      }
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < ns) row[s] = v[s];
      if (!direct) first = *stp != bid;
      *stp = bid;
    }
    if (!direct) {
      pb.touched[before + q] = first ? (uint32_t)slot : kTouchSkip;
      continue;
    }
    if (has_out) {
      // v is the group's state after this batch: its changelog row
      const uint64_t o = out_base + before + q;
      if (o < out_cap) {
        out.key[o] = (uint32_t)(g >> 32);
        int64_t ws = 0, we = 0;
        if (p.kind != HSG_UNWINDOWED) {
          const int64_t k = k_epoch + (int64_t)(g & 0xFFFFFFFFull);
          ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
          we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
        }
        out.ws[o] = ws;
        out.we[o] = we;
        out.src[o] = -1;
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value_reg<MS>(prog, j, v);
        if (out.form) out.form[o] = out_form_reg<MS>(prog, v);
      } else {
        err |= ERR_OOM;
      }
    }
  }
  if (err) atomicOr(&sc->err, err);
  const uint64_t fr = wave_sum_u64(fresh);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = fr;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t f = s_red[0] + s_red[1] + s_red[2] + s_red[3];
    if (f) atomicAdd((unsigned long long *)&sc->live_x[blockIdx.x & 7], (unsigned long long)f);
  }
}

// LDS entries of the SQL lean kernel for this program (op_device.cpp
// adapt_partitions: buckets of at most half a table of groups)
uint64_t sql_lds_entries(const Program &prog) {
  uint64_t hi = 0;
  const uint64_t sq = program_sig(prog, &hi);
  return ((sq == kSigSqlI && hi == kSigSqlI2) || (sq == kSigSqlF && hi == kSigSqlF2) || (sq == kSigSqlSumMaxI && !hi))
             ? 2048
             : 1024;
}

// the op shape this path takes: one-window packed records with the sequence
// word (<= 2 columns), the full slot program in LDS (<= 16 slots)
bool sql_lean_eligible(const Program &prog, const PartParams &pp) {
  return pp.pane_S == 1 && pp.has_seq && (pp.words == 4 || pp.words == 5) && prog.n_slots <= 16;
}

template <int MS, int E, int NT, uint64_t SIG = 0, uint64_t SIG2 = 0>
static void sql_launch(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                       const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols &out, uint64_t out_base,
                       uint64_t out_cap) {
  if (pp.words - 1 == 3)
    hipLaunchKernelGGL((k_agg_sql<MS, E, NT, 3, SIG, SIG2>), g, dim3(NT), 0, s, prog, pp, t, pb, sc);
  else
    hipLaunchKernelGGL((k_agg_sql<MS, E, NT, 4, SIG, SIG2>), g, dim3(NT), 0, s, prog, pp, t, pb, sc);
  hipLaunchKernelGGL((k_sql_apply<MS>), g, dim3(256), 0, s, prog, p, pp, t, pb, out, out_base, out_cap, sc);
}

bool launch_part_agg_sql(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                         const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols *out,
                         uint64_t out_base, uint64_t out_cap) {
  if (!sql_lean_eligible(prog, pp)) return false;
  OutCols oc;
  memset(&oc, 0, sizeof(oc));
  if (out) oc = *out;
  // 1024 LDS entries (part_lds_entries: buckets of <= 512 groups): 8 + 8 MS
  // bytes each, one 1024-thread workgroup per CU at 12 slots
  // the SQL drop-in's C2 and C5 queries: their slot programs baked in, in
  // the packed LDS layout (a 2048-entry table, buckets of twice the groups)
  uint64_t hi = 0;
  const uint64_t sq = program_sig(prog, &hi);
  if (prog.n_slots <= 8) {
    if (sq == kSigSqlSumMaxI && !hi)
      sql_launch<8, 2048, 1024, kSigSqlSumMaxI, 0>(s, g, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
    else
      sql_launch<8, 1024, 512>(s, g, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
  } else if (prog.n_slots <= 12) {
    if (sq == kSigSqlI && hi == kSigSqlI2)
      sql_launch<12, 2048, 1024, kSigSqlI, kSigSqlI2>(s, g, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
    else if (sq == kSigSqlF && hi == kSigSqlF2)
      sql_launch<12, 2048, 1024, kSigSqlF, kSigSqlF2>(s, g, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
    else
      sql_launch<12, 1024, 1024>(s, g, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
  }
  else sql_launch<16, 1024, 1024>(s, g, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
  return true;
}

}  // namespace hsg
