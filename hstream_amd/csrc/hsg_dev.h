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
    default: return 0;
  }
}

__device__ inline bool rec_present(const Batch &b, int c, uint64_t i) {
  return b.valid[c] == nullptr || b.valid[c][i] != 0;
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
    default: return a;
  }
}

// Row-wise combine over MS compile-time-bounded slots (registers, no scratch).
template <int MS>
__device__ inline void combine_row(const Program &prog, int64_t (&a)[MS], const int64_t (&e)[MS]) {
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
// initial value. `own` = the output's own slot, fa / fb its form slots.
__device__ inline uint32_t form_bits_w(int kind, int64_t own, int64_t fa, int64_t fb) {
  switch (kind) {
    case F_SUM: return fa == 0 ? 1u : 0u;
    case F_MINMAX: return fb == 0 ? 3u : (fa == own ? 1u : 0u);
    case F_LAST:
      if (fa == 0 && fb == 0) return 3u;
      return (uint64_t)fb > (uint64_t)fa ? 1u : 0u;
    default: return 0u;
  }
}
__device__ inline uint32_t out_form(const Program &prog, const int64_t *row) {
  uint32_t f = 0;
  for (int j = 0; j < prog.n_out; ++j)
    if (prog.form_kind[j] != F_NONE)
      f |= form_bits_w(prog.form_kind[j], row[prog.out_a[j]], row[prog.form_a[j]], row[prog.form_b[j]]) << (2 * j);
  return f;
}
template <int MS>
__device__ inline uint32_t out_form_reg(const Program &prog, const int64_t (&r)[MS]) {
  uint32_t f = 0;
  for (int j = 0; j < prog.n_out; ++j) {
    if (prog.form_kind[j] == F_NONE) continue;
    int64_t own = 0, fa = 0, fb = 0;
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (s == prog.out_a[j]) own = r[s];
      if (s == prog.form_a[j]) fa = r[s];
      if (s == prog.form_b[j]) fb = r[s];
    }
    f |= form_bits_w(prog.form_kind[j], own, fa, fb) << (2 * j);
  }
  return f;
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
