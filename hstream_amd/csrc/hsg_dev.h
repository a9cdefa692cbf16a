// Device helpers shared by the gfx950 kernels (wave64 scans / reductions, the
// aggregate-slot algebra, output conversion). Not part of the ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

// Phase clocks of the HSG_PHASES diagnostics (per-workgroup time split of the
// partition, aggregation, per-record and session kernels, summed into
// DevScalars::scratch and printed by op_device.cpp). Compiled in only with
// -DHSG_PHASE_CLOCKS=1 (make PHASES=1): otherwise phase_clock() is 0 and every
// accumulation guarded by kPhaseClocks is dead code, so the product kernels
// carry neither the clock reads nor the atomics.
#ifndef HSG_PHASE_CLOCKS
#define HSG_PHASE_CLOCKS 0
#endif
constexpr bool kPhaseClocks = HSG_PHASE_CLOCKS != 0;
__device__ inline uint64_t phase_clock() {
  if constexpr (kPhaseClocks) return wall_clock64();
  return 0;
}

__device__ inline int64_t wave_max_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t u = __shfl_xor(v, o, 64);
    v = u > v ? u : v;
  }
  return v;
}
__device__ inline int64_t wave_min_i64(int64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    int64_t u = __shfl_xor(v, o, 64);
    v = u < v ? u : v;
  }
  return v;
}
__device__ inline uint64_t wave_sum_u64(uint64_t v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ inline int64_t wave_incl_max(int64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    int64_t u = __shfl_up(v, o, 64);
    if (lane >= o) v = u > v ? u : v;
  }
  return v;
}
__device__ inline uint64_t wave_incl_sum(uint64_t v) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint64_t u = __shfl_up(v, o, 64);
    if (lane >= o) v += u;
  }
  return v;
}

// Workgroup barrier that orders LDS only: __syncthreads() also waits for the
// wave's outstanding global stores (its workgroup-scope release), which costs
// microseconds after a burst of scattered stores that no one in the workgroup
// reads back. Use where the only data crossing the barrier is in LDS.
__device__ inline void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ inline int64_t slot_identity_dev(int32_t op) {
  switch (op) {
    case S_MIN_I: return INT64_MAX;
    case S_MAX_I: return INT64_MIN;
    case S_MIN_F: return (int64_t)f64_ord(9223372036854775807.0);
    case S_MAX_F: return (int64_t)f64_ord(-9223372036854775808.0);
    case S_SUM_F: return INT64_MIN;  // -0.0 (slot_identity)
    case S_TIE_MIN: return 1;        // seq 0, integral: the initial maxBound
    default: return 0;
  }
}

__device__ inline bool rec_present(const Batch &b, int c, uint64_t i) {
  return b.valid[c] == nullptr || b.valid[c][i] != 0;
}
// the value's JSON literal prints in Generic form (bit 1 of its valid byte,
// hstream_ingest.h literal_forms)
__device__ inline bool rec_decimal(const Batch &b, int c, uint64_t i) {
  return b.valid[c] != nullptr && (b.valid[c][i] & 2u) != 0;
}
// a form slot's word for a present record: (seq + 1) << 1 | integral literal
__device__ inline int64_t form_word(const Batch &b, int c, uint64_t i, uint64_t seq1) {
  return (int64_t)((seq1 << 1) | (rec_decimal(b, c, i) ? 0u : 1u));
}

// Sequence word of a partitioned record of an op with LAST / literal-form
// slots (hsg_part.h): (global seq + 1) in the low 56 bits, bit 56 + c set when
// column c's literal is decimal (bit 1 of its valid byte).
constexpr uint64_t kSeqMask = (1ull << 56) - 1;
__device__ inline uint64_t seq_word(const Batch &b, int C, int has_valid, int64_t seq, uint64_t i) {
  uint64_t w = (uint64_t)(seq + 1) & kSeqMask;
  if (has_valid)
    for (int c = 0; c < C && c < 8; ++c)
      if (b.valid[c] && (b.valid[c][i] & 2u)) w |= 1ull << (56 + c);
  return w;
}

// Contribution of record i to state slot s (identity when the field is absent).
__device__ inline int64_t slot_elem(const Program &prog, int s, const Batch &b, uint64_t i, uint64_t seq1) {
  const int op = prog.slot_op[s];
  const int c = prog.slot_col[s];
  if (op == S_CNT_ALL) return 1;
  if (op == S_LAST_VAL) {
    // paired with the preceding LAST_SEQ slot; value only meaningful when present
    return rec_present(b, c, i) ? b.col[c][i] : 0;
  }
  if (!rec_present(b, c, i)) return slot_identity_dev(op);
  switch (op) {
    case S_CNT: return 1;
    case S_SUM_I:
    case S_SUM_F:
    case S_MIN_I:
    case S_MAX_I: return b.col[c][i];
    case S_MIN_F:
    case S_MAX_F: return (int64_t)f64_ord(__builtin_bit_cast(double, b.col[c][i]));
    case S_LAST_SEQ: return (int64_t)seq1;
    case S_CNT_DEC: return rec_decimal(b, c, i) ? 1 : 0;
    case S_TIE_MIN:
    case S_TIE_MAX:
    case S_LAST_FORM: return form_word(b, c, i, seq1);
    default: return 0;
  }
}

// a <- a (+) e for one slot, where e comes later in arrival order than a.
// LAST_SEQ/LAST_VAL are combined as a pair by the caller (see combine_row).
__device__ inline int64_t slot_combine(int op, int64_t a, int64_t e) {
  switch (op) {
    case S_CNT_ALL:
    case S_CNT:
    case S_SUM_I: return (int64_t)((uint64_t)a + (uint64_t)e);
    case S_SUM_F: return __builtin_bit_cast(int64_t, __builtin_bit_cast(double, a) + __builtin_bit_cast(double, e));
    case S_MIN_I: return e < a ? e : a;
    case S_MAX_I: return e > a ? e : a;
    case S_MIN_F: return (uint64_t)e < (uint64_t)a ? e : a;
    case S_MAX_F: return (uint64_t)e > (uint64_t)a ? e : a;
    case S_CNT_DEC: return (int64_t)((uint64_t)a + (uint64_t)e);
    case S_LAST_FORM: return (uint64_t)e > (uint64_t)a ? e : a;
    default: return a;  // S_TIE_*: combined with their MIN / MAX slot (tie_combine)
  }
}

// "e is better than a" for the MIN / MAX slot op vop (equal: a tie)
__device__ inline bool extreme_better(int vop, int64_t e, int64_t a) {
  switch (vop) {
    case S_MIN_I: return e < a;
    case S_MAX_I: return e > a;
    case S_MIN_F: return (uint64_t)e < (uint64_t)a;
    case S_MAX_F: return (uint64_t)e > (uint64_t)a;
    default: return false;
  }
}
// tie word after a <- a (+) e, from the MIN / MAX values before the combine
// (va, ve): the better value's word; on a tie the earlier literal for MIN
// (min n x = n) and the later for MAX (max n x = x) -- by record sequence, so
// any grouping of a record fold gives the sequential fold's word
__device__ inline int64_t tie_combine(int op, int vop, int64_t va, int64_t ve, int64_t ta, int64_t te) {
  if (extreme_better(vop, ve, va)) return te;
  if (va != ve) return ta;
  if (op == S_TIE_MIN) return (uint64_t)te < (uint64_t)ta ? te : ta;
  return (uint64_t)te > (uint64_t)ta ? te : ta;
}

// Row-wise combine over MS compile-time-bounded slots (registers, no scratch).
// the value of slot v of a register row (v not a compile-time index)
template <int MS>
__device__ inline int64_t reg_at(const int64_t (&r)[MS], int v) {
  int64_t x = 0;
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s == v) x = r[s];
  return x;
}

// tie words first, against the MIN / MAX values before the combine
template <int MS>
__device__ inline void combine_ties(const Program &prog, int64_t (&a)[MS], const int64_t (&e)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
    if (!slot_is_tie(op)) continue;
    const int v = prog.slot_aux[s];
    a[s] = tie_combine(op, prog.slot_op[v], reg_at<MS>(a, v), reg_at<MS>(e, v), a[s], e[s]);
  }
}

template <int MS>
__device__ inline void combine_row(const Program &prog, int64_t (&a)[MS], const int64_t (&e)[MS]) {
  if (prog.ties) combine_ties<MS>(prog, a, e);
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
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

template <int MS>
__device__ inline void identity_row(const Program &prog, int64_t (&a)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) a[s] = s < prog.n_slots ? slot_identity_dev(prog.slot_op[s]) : 0;
}

template <int MS>
__device__ inline void elem_row(const Program &prog, int64_t (&e)[MS], const Batch &b, uint64_t i, uint64_t seq1) {
#pragma unroll
  for (int s = 0; s < MS; ++s) e[s] = s < prog.n_slots ? slot_elem(prog, s, b, i, seq1) : 0;
}

__device__ inline int64_t out_value_w(const Program &prog, int j, int64_t a, int64_t bcnt) {
  switch (prog.out_kind[j]) {
    case O_F64_ORD: return __builtin_bit_cast(int64_t, f64_unord((uint64_t)a));
    case O_AVG_I: {
      double d = bcnt ? (double)a / (double)bcnt : __builtin_nan("");
      return __builtin_bit_cast(int64_t, d);
    }
    case O_AVG_F: {
      double d = bcnt ? __builtin_bit_cast(double, a) / (double)bcnt : __builtin_nan("");
      return __builtin_bit_cast(int64_t, d);
    }
    default: return a;
  }
}

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so
// give workgroups b, b+8, b+16, ... (one XCD) consecutive tiles; a bucket's
// runs from consecutive tiles are adjacent in the output. Speed only.
__device__ inline uint64_t xcd_tile(uint64_t blk, uint64_t tiles) {
  const uint64_t per = tiles / 8, full = per * 8;
  if (blk >= full) return blk;
  return (blk & 7) * per + (blk >> 3);
}

// output column j from a state row in memory
__device__ inline int64_t out_value(const Program &prog, int j, const int64_t *row) {
  return out_value_w(prog, j, row[prog.out_a[j]], row[prog.out_b[j]]);
}

template <int MS>
__device__ inline int64_t out_value_reg(const Program &prog, int j, const int64_t (&r)[MS]) {
  int64_t a = 0, b = 0;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s == prog.out_a[j]) a = r[s];
    if (s == prog.out_b[j]) b = r[s];
  }
  return out_value_w(prog, j, a, b);
}

// Literal forms of a row's outputs (hsg_rows.form; hsg_internal.h FormKind):
// bit 2j = output j prints as an integer, bit 2j + 1 = it is the aggregate's
// initial value. fa = the output's form slot.
__device__ inline uint32_t form_bits_w(int kind, int64_t fa) {
  switch (kind) {
    case F_SUM: return fa == 0 ? 1u : 0u;
    case F_MIN: return fa == 1 ? 3u : (uint32_t)(fa & 1);
    case F_MAX:
    case F_LAST: return fa == 0 ? 3u : (uint32_t)(fa & 1);
    default: return 0u;
  }
}
__device__ inline uint32_t out_form(const Program &prog, const int64_t *row) {
  uint32_t f = 0;
  for (int j = 0; j < prog.n_out; ++j)
    if (prog.form_kind[j] != F_NONE) f |= form_bits_w(prog.form_kind[j], row[prog.form_a[j]]) << (2 * j);
  return f;
}
template <int MS>
__device__ inline uint32_t out_form_reg(const Program &prog, const int64_t (&r)[MS]) {
  uint32_t f = 0;
  for (int j = 0; j < prog.n_out; ++j)
    if (prog.form_kind[j] != F_NONE) f |= form_bits_w(prog.form_kind[j], reg_at<MS>(r, prog.form_a[j])) << (2 * j);
  return f;
}

// Session merge, acc <- sessionMergeF rk acc cur (SessionWindowedStream.hs
// :100-114; acc = the new record with the sessions merged so far, cur = the
// next overlapped session in end order): the aggregate components'
// aggregateMergeF (Codegen.hs:409-469) -- counts and sums add, MIN / MAX keep
// the extreme with min n1 n2 / max n1 n2 on ties (n1 = acc's literal for
// MIN, n2 = cur's for MAX), passthrough columns take cur's (o2)
template <int MS>
__device__ inline void merge_row(const Program &prog, int64_t (&acc)[MS], const int64_t (&cur)[MS]) {
  if (prog.ties) {
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (s >= prog.n_slots) break;
      const int op = prog.slot_op[s];
      if (!slot_is_tie(op)) continue;
      const int v = prog.slot_aux[s], vop = prog.slot_op[v];
      const int64_t va = reg_at<MS>(acc, v), vc = reg_at<MS>(cur, v);
      if (extreme_better(vop, vc, va) || (va == vc && op == S_TIE_MAX)) acc[s] = cur[s];
    }
  }
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
    if (op == S_LAST_SEQ || op == S_LAST_VAL || op == S_LAST_FORM) acc[s] = cur[s];
    else acc[s] = slot_combine(op, acc[s], cur[s]);
  }
}

// Per-record stream time for the records of one tile (record (r, thread) =
// tile_base + r*kTileThreads + thread), inclusive prefix max in arrival order
// seeded with the tile's exclusive prefix. Block-wide: every thread must call.
__device__ inline void tile_stream_time(const int64_t (&ts)[kRecPerThread], int64_t carry,
                                        int64_t (&wm)[kRecPerThread]) {
  __shared__ int64_t swave[kTileThreads / 64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    int64_t incl = wave_incl_max(ts[r]);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    int64_t before = carry;
    for (int k = 0; k < w; ++k) before = swave[k] > before ? swave[k] : before;
    wm[r] = incl > before ? incl : before;
    int64_t tot = carry;
    for (int k = 0; k < kTileThreads / 64; ++k) tot = swave[k] > tot ? swave[k] : tot;
    carry = tot;
    __syncthreads();
  }
}

// Window range [k_lo, k_hi] of a record (windowsFor, TimeWindowedStream.hs:105-117);
// returns false when the record has no window (ts < 0).
__device__ inline bool record_windows(const TwParams &p, int64_t ts, uint64_t &k_lo, uint64_t &k_hi) {
  if (p.kind == HSG_UNWINDOWED) {
    k_lo = 0;
    k_hi = 0;
    return true;
  }
  if (ts < 0) return false;
  k_hi = udiv(p.div, (uint64_t)ts);
  if (p.size == p.adv) {  // tumbling: the one window (uniform branch)
    k_lo = k_hi;
    return true;
  }
  int64_t t0 = (int64_t)((uint64_t)ts - (uint64_t)p.size + (uint64_t)p.adv);
  if (t0 < 0) t0 = 0;
  k_lo = udiv(p.div, (uint64_t)t0);
  return true;
}

// grace check of window k against the record's stream time (TimeWindowedStream.hs:92)
__device__ inline bool window_accepted(const TwParams &p, uint64_t k, int64_t wm) {
  if (p.kind == HSG_UNWINDOWED) return true;
  int64_t ws = (int64_t)(k * (uint64_t)p.adv);
  int64_t we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
  return wm < (int64_t)((uint64_t)we + (uint64_t)p.grace);
}

}  // namespace hsg
