// gfx950 kernels for session windows (SessionWindowedStream.hs:74-118 over the
// session store of Store.hs:177-272).
//
// State in HBM: a key -> slot hash table and, per slot, the key's sessions as
// a list sorted by start in an arena (structure of arrays). Sessions of one key
// stay more than `gap` apart, so the sessions findSessions returns for a point
// t (end >= t-gap, start <= t+gap) are one contiguous run of the list.
//
// Batch: slot per record -> stable radix sort of (slot, record) -> run heads
// -> one thread per touched key replays that key's records in arrival order
// against its list, exactly as the reference's per-record fold does (new point
// [t,t] with aggF init r, then mergeF over the overlapped sessions in end order,
// remove them, put the merged one). Keys are independent (findSessions filters
// by key), so the per-key replay is the reference's result for every order of
// interleaving between keys.
#include "hsg_dev.h"
#include "hsg_perrecord.h"
#include "hsg_session.h"

namespace hsg {

constexpr uint32_t kEmpty32 = 0xFFFFFFFFu;

__global__ void k_ss_reset(SessTable t, uint64_t cap) {
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    t.keys[s] = kEmpty32;
    t.list_off[s] = s * kSessInline;
    t.list_len[s] = 0;
    t.list_cap[s] = kSessInline;
  }
}

void launch_ss_reset(hipStream_t s, const SessTable &t, uint64_t cap) {
  hipLaunchKernelGGL(k_ss_reset, dim3(grid_for(cap, 256)), dim3(256), 0, s, t, cap);
}

__device__ inline int64_t ss_find_or_insert(const SessTable &t, uint32_t key) {
  uint64_t s = mix64(key) & t.mask;
  for (uint64_t probe = 0; probe <= t.mask; ++probe) {
    uint32_t cur = t.keys[s];
    if (cur == key) return (int64_t)s;
    if (cur == kEmpty32) {
      uint32_t old = atomicCAS(&t.keys[s], kEmpty32, key);
      if (old == kEmpty32 || old == key) return (int64_t)s;
    }
    s = (s + 1) & t.mask;
  }
  return -1;
}

// slot per record (cap for HSG_KEY_NONE / table full), record index, and the
// valid flag that numbers per-record changelog rows
__global__ void k_ss_slot(Batch b, SessTable t, uint32_t *rslot, uint32_t *ridx, uint32_t *vflag, DevScalars *sc) {
  const uint32_t cap = (uint32_t)(t.mask + 1);
  uint32_t err = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < b.n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t key = b.key[i];
    uint32_t sl = cap;
    if (key != HSG_KEY_NONE) {
      int64_t s = ss_find_or_insert(t, key);
      if (s < 0) err |= ERR_OOM;
      else sl = (uint32_t)s;
    }
    rslot[i] = sl;
    ridx[i] = (uint32_t)i;
    vflag[i] = key != HSG_KEY_NONE ? 1u : 0u;
  }
  if (err) atomicOr(&sc->err, err);
}

void launch_ss_slot(hipStream_t s, const Batch &b, const SessTable &t, uint32_t *rslot, uint32_t *ridx,
                    uint32_t *vflag, DevScalars *sc) {
  if (b.n) hipLaunchKernelGGL(k_ss_slot, dim3(grid_for(b.n, 256)), dim3(256), 0, s, b, t, rslot, ridx, vflag, sc);
}

// run heads over the sorted slots (valid records sort first)
__global__ void k_ss_heads(const uint32_t *slot, uint64_t n, uint32_t cap, uint8_t *flag) {
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x)
    flag[q] = (slot[q] < cap && (q == 0 || slot[q] != slot[q - 1])) ? 1 : 0;
}
__global__ void k_ss_runs(const uint8_t *flag, const uint64_t *runidx, uint64_t n, uint32_t *runs) {
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < n; q += (uint64_t)gridDim.x * blockDim.x)
    if (flag[q]) runs[runidx[q]] = (uint32_t)q;
}

void launch_ss_runs(hipStream_t s, const uint32_t *slot, uint64_t n, uint32_t cap, uint8_t *flag,
                    const uint64_t *runidx, uint32_t *runs, int phase) {
  if (!n) return;
  if (phase == 0) hipLaunchKernelGGL(k_ss_heads, dim3(grid_for(n, 256)), dim3(256), 0, s, slot, n, cap, flag);
  else hipLaunchKernelGGL(k_ss_runs, dim3(grid_for(n, 256)), dim3(256), 0, s, flag, runidx, n, runs);
}

// ---------------------------------------------------------------------------
// per-key replay
// ---------------------------------------------------------------------------
template <int MS>
__device__ inline void ss_load(const SessTable &t, const Program &prog, uint64_t idx, int64_t (&a)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) a[s] = s < prog.n_slots ? t.a_aggs[idx * prog.n_slots + s] : 0;
}
template <int MS>
__device__ inline void ss_store(const SessTable &t, const Program &prog, uint64_t idx, const int64_t (&a)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s < prog.n_slots) t.a_aggs[idx * prog.n_slots + s] = a[s];
}
__device__ inline void ss_move(const SessTable &t, int ns, uint64_t dst, uint64_t src) {
  t.a_start[dst] = t.a_start[src];
  t.a_end[dst] = t.a_end[src];
  t.a_stamp[dst] = t.a_stamp[src];
  for (int s = 0; s < ns; ++s) t.a_aggs[dst * ns + s] = t.a_aggs[src * ns + s];
}

template <int MS>
__global__ __launch_bounds__(256) void k_ss_process(Batch b, SessParams p, SessTable t, Program prog,
                                                    const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs,
                                                    uint64_t R, const uint64_t *out_pos, const int64_t *seq,
                                                    OutCols out, uint64_t out_base, uint64_t *arena_top,
                                                    DevScalars *sc) {
  __shared__ uint64_t swave[4];
  __shared__ uint64_t sbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const int ns = prog.n_slots;
  bool active = r < R;
  uint64_t q0 = 0, q1 = 0;
  uint32_t sl = 0, key = 0;
  uint64_t off = 0, lcap = 0, len = 0;
  uint32_t err = 0;
  int64_t live_delta = 0;
  if (active) {
    q0 = runs[r];
    q1 = runs[r + 1];
    sl = slot[q0];
    key = t.keys[sl];
    off = t.list_off[sl];
    len = t.list_len[sl];
    lcap = t.list_cap[sl];
  }
  // grow the key's list once for the whole run (each record adds <= 1 session);
  // one arena bump per wave
  uint64_t need = len + (q1 - q0);
  uint64_t new_cap = 0;
  if (active && need > lcap) {
    new_cap = lcap * 2;
    while (new_cap < need) new_cap *= 2;
  }
  uint64_t incl = wave_incl_sum(new_cap);
  uint64_t wtot = __shfl(incl, 63, 64);
  uint64_t wbase = 0;
  if (lane == 63 && wtot) wbase = atomicAdd((unsigned long long *)arena_top, (unsigned long long)wtot);
  wbase = __shfl(wbase, 63, 64);
  if (new_cap) {
    uint64_t noff = p.dyn_base + wbase + incl - new_cap;
    if (noff + new_cap > t.arena_cap) {
      err |= ERR_OOM;
      active = false;
    } else {
      for (uint64_t k = 0; k < len; ++k) ss_move(t, ns, noff + k, off + k);
      off = noff;
      lcap = new_cap;
      t.list_off[sl] = off;
      t.list_cap[sl] = (uint32_t)lcap;
    }
  }
  if (active) {
    for (uint64_t q = q0; q < q1; ++q) {
      const uint32_t i = ridx[q];
      const int64_t ts = b.ts[i];
      const uint64_t seq1 = (seq ? (uint64_t)seq[i] : p.rec_base + i) + 1;
      const int64_t lo = (int64_t)((uint64_t)ts - (uint64_t)p.gap);
      const int64_t hi = (int64_t)((uint64_t)ts + (uint64_t)p.gap);
      // first session with end >= lo (ends ascend: sessions are disjoint)
      uint64_t a = 0, z = len;
      while (a < z) {
        uint64_t m = (a + z) >> 1;
        if (t.a_end[off + m] < lo) a = m + 1;
        else z = m;
      }
      const uint64_t i0 = a;
      uint64_t i1 = i0;
      while (i1 < len && t.a_start[off + i1] <= hi) ++i1;
      // aggF initialValue r, then mergeF acc cur over the overlapped sessions
      int64_t acc[MS], e[MS];
      identity_row<MS>(prog, acc);
      elem_row<MS>(prog, e, b, i, seq1);
      combine_row<MS>(prog, acc, e);
      int64_t s0 = ts, e0 = ts;
      for (uint64_t k = i0; k < i1; ++k) {
        int64_t cs = t.a_start[off + k], ce = t.a_end[off + k];
        s0 = cs < s0 ? cs : s0;
        e0 = ce > e0 ? ce : e0;
        int64_t cur[MS];
        ss_load<MS>(t, prog, off + k, cur);
        combine_row<MS>(prog, acc, cur);
        // passthrough columns: aggregateMergeF _ _ o2 keeps the existing
        // session's value (Codegen.hs:467), so after the fold the last
        // overlapped session in end order (k = i1 - 1) decides
#pragma unroll
        for (int s = 0; s < MS; ++s)
          if (s < ns && (prog.slot_op[s] == S_LAST_SEQ || prog.slot_op[s] == S_LAST_VAL)) acc[s] = cur[s];
      }
      const uint64_t c = i1 - i0;
      if (c == 0) {
        for (uint64_t k = len; k > i0; --k) ss_move(t, ns, off + k, off + k - 1);
        len += 1;
      } else if (c > 1) {
        for (uint64_t k = i1; k < len; ++k) ss_move(t, ns, off + k - (c - 1), off + k);
        len -= c - 1;
      }
      live_delta += 1 - (int64_t)c;
      t.a_start[off + i0] = s0;
      t.a_end[off + i0] = e0;
      t.a_stamp[off + i0] = p.batch_id;
      ss_store<MS>(t, prog, off + i0, acc);
      if (p.emit_mode == HSG_EMIT_PER_RECORD) {
        const uint64_t o = out_base + out_pos[i];
        out.key[o] = key;
        out.ws[o] = s0;
        out.we[o] = e0;
        out.src[o] = (int64_t)(seq1 - 1);
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value_reg<MS>(prog, j, acc);
      }
    }
    t.list_len[sl] = (uint32_t)len;
  }
  // per-batch changelog: the key's sessions stamped by this batch
  uint64_t mine = 0;
  if (active && p.emit_mode == HSG_EMIT_PER_BATCH)
    for (uint64_t k = 0; k < len; ++k) mine += t.a_stamp[off + k] == p.batch_id;
  uint64_t inc2 = wave_incl_sum(mine);
  if (lane == 63) swave[w] = inc2;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = swave[0] + swave[1] + swave[2] + swave[3];
    sbase = tot ? atomicAdd((unsigned long long *)&sc->out_rows, (unsigned long long)tot) : 0;
    if (tot) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tot);
  }
  __syncthreads();
  if (mine) {
    uint64_t o = out_base + sbase + inc2 - mine;
    for (int k = 0; k < w; ++k) o += swave[k];
    for (uint64_t k = 0; k < len; ++k) {
      if (t.a_stamp[off + k] != p.batch_id) continue;
      out.key[o] = key;
      out.ws[o] = t.a_start[off + k];
      out.we[o] = t.a_end[off + k];
      out.src[o] = -1;
      const int64_t *row = t.a_aggs + (off + k) * ns;
      for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, row);
      ++o;
    }
  }
  // live sessions and errors
  uint64_t ld = wave_sum_u64((uint64_t)live_delta);
  if (lane == 0 && ld) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)ld);
  if (err) atomicOr(&sc->err, err);
}

template <int MS>
static void ss_process_launch(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t,
                              const Program &prog, const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs,
                              uint64_t R, const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base,
                              uint64_t *arena_top, DevScalars *sc) {
  uint64_t blocks = (R + 255) / 256;
  hipLaunchKernelGGL(k_ss_process<MS>, dim3((unsigned)blocks), dim3(256), 0, s, b, p, t, prog, slot, ridx, runs, R,
                     out_pos, seq, out, out_base, arena_top, sc);
}

void launch_ss_process(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                       const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs, uint64_t R,
                       const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base,
                       uint64_t *arena_top, DevScalars *sc) {
  if (!R) return;
  if (prog.n_slots <= 2) ss_process_launch<2>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, arena_top, sc);
  else if (prog.n_slots <= 4) ss_process_launch<4>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, arena_top, sc);
  else if (prog.n_slots <= 8) ss_process_launch<8>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, arena_top, sc);
  else ss_process_launch<kMaxSlots>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, arena_top, sc);
}

// ssDump: every live session (key, start, end, aggs)
__global__ __launch_bounds__(256) void k_ss_dump(SessTable t, uint64_t cap, Program prog, OutCols out,
                                                 uint64_t out_cap, uint64_t *counter) {
  __shared__ uint64_t swave[4];
  __shared__ uint64_t sbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t blk = blockIdx.x * 256ull; blk < cap; blk += (uint64_t)gridDim.x * 256ull) {
    const uint64_t s = blk + threadIdx.x;
    uint64_t len = 0, off = 0;
    uint32_t key = kEmpty32;
    if (s < cap) {
      key = t.keys[s];
      if (key != kEmpty32) {
        len = t.list_len[s];
        off = t.list_off[s];
      }
    }
    uint64_t incl = wave_incl_sum(len);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
      uint64_t tot = swave[0] + swave[1] + swave[2] + swave[3];
      sbase = tot ? atomicAdd((unsigned long long *)counter, (unsigned long long)tot) : 0;
    }
    __syncthreads();
    uint64_t o = sbase + incl - len;
    for (int k = 0; k < w; ++k) o += swave[k];
    for (uint64_t k = 0; k < len && o < out_cap; ++k, ++o) {
      out.key[o] = key;
      out.ws[o] = t.a_start[off + k];
      out.we[o] = t.a_end[off + k];
      out.src[o] = -1;
      const int64_t *row = t.a_aggs + (off + k) * prog.n_slots;
      for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, row);
    }
    __syncthreads();
  }
}

void launch_ss_dump(hipStream_t s, const SessTable &t, uint64_t cap, const Program &prog, OutCols out,
                    uint64_t out_cap, uint64_t *counter) {
  uint64_t blocks = (cap + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_ss_dump, dim3((unsigned)blocks), dim3(256), 0, s, t, cap, prog, out, out_cap, counter);
}

}  // namespace hsg
