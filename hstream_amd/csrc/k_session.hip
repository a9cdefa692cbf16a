// gfx950 kernels for session windows (SessionWindowedStream.hs:74-118 over the
// session store of Store.hs:177-272). Layout and paths: hsg_session.h.
#include "hsg_agg.h"
#include "hsg_dev.h"
#include "hsg_perrecord.h"
#include "hsg_session.h"
#include "hsg_sort.h"

namespace hsg {

// ---------------------------------------------------------------------------
// store helpers: key entries, session rows [start][end][stamp][aggs...]
// ---------------------------------------------------------------------------
__device__ inline uint64_t *ss_row(const SessTable &t, uint64_t i) { return t.rows + i * t.stride; }

__device__ inline void ss_copy(const SessTable &dt, uint64_t dst, const SessTable &st, uint64_t src) {
  const uint64_t *a = ss_row(st, src);
  uint64_t *b = ss_row(dt, dst);
  for (uint32_t w = 0; w < st.stride; ++w) b[w] = a[w];
}

// rows [base, base + n) from arena region r (bump); false when the region is
// exhausted (the host then compacts the arena and re-partitions the regions)
__device__ inline bool arena_take(const SessTable &t, uint32_t r, uint64_t n, uint64_t &base) {
  base = atomicAdd((unsigned long long *)&t.meta[M_RTOP + r * kRegionStride], (unsigned long long)n);
  return base + n <= t.meta[M_REND + r * kRegionStride];
}
__device__ inline uint32_t arena_region(uint32_t block) { return block % kArenaRegions; }

// rows reserved for a list of `need` sessions: 4, 16, 64, then doubling. A
// list that outgrows its rows moves (its rows are copied), so short lists,
// which grow by a session every few batches, grow 4x: C4's lists (~33
// sessions by the end of the stream) move twice instead of four times
__device__ inline uint32_t ss_grow_cap(uint64_t need) {
  uint32_t c = 4;
  while (c < need) c <<= (c < 64 ? 2 : 1);
  return c;
}

__device__ inline SessKey ss_blank(uint32_t key) {
  SessKey e;
  e.key = key;
  e.len = 0;
  e.off = 0;
  e.cap = 0;
  e.mvalid = 0;
  e.emark = ~0ull;
  e.ms = e.me = 0;
  e.ma[0] = e.ma[1] = 0;
  return e;
}

// one entry in four 16-byte loads, fields assigned one by one (a struct copy
// of the 64-byte entry can land on the stack)
__device__ inline SessKey ss_load_entry(const SessKey *p) {
  const uint4 *q = reinterpret_cast<const uint4 *>(p);
  const uint4 a = q[0], b = q[1], c = q[2], d = q[3];
  SessKey e;
  e.key = a.x;
  e.len = a.y;
  e.off = (uint64_t)a.z | ((uint64_t)a.w << 32);
  e.cap = b.x;
  e.mvalid = b.y;
  e.emark = (uint64_t)b.z | ((uint64_t)b.w << 32);
  e.ms = (int64_t)((uint64_t)c.x | ((uint64_t)c.y << 32));
  e.me = (int64_t)((uint64_t)c.z | ((uint64_t)c.w << 32));
  e.ma[0] = (int64_t)((uint64_t)d.x | ((uint64_t)d.y << 32));
  e.ma[1] = (int64_t)((uint64_t)d.z | ((uint64_t)d.w << 32));
  return e;
}

__global__ void k_ss_reset(SessTable t) {
  const uint64_t cap = t.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x)
    t.kt[s] = ss_blank(kSessEmptyKey);
}

void launch_ss_reset(hipStream_t s, const SessTable &t) {
  hipLaunchKernelGGL(k_ss_reset, dim3(grid_for(t.kmask + 1, 256)), dim3(256), 0, s, t);
}

// find key's slot, inserting it if absent; -1 = table full. `inserted` is set
// when this call claimed the slot (its entry then still holds an empty list).
// Home slot: the top key-hash bits below the owner bits, the same bits that
// pick the key's partition bucket (and sub-bucket), so the keys of a bucket
// occupy one stretch of the table and the merge path, which walks a bucket's
// keys in hash order, touches neighbouring entries from neighbouring lanes.
__device__ inline uint64_t ss_home(const SessTable &t, uint32_t key) {
  return t.kbits ? (uint64_t)((key_hash(key) << t.hshift) >> (64 - t.kbits)) : 0ull;
}

__device__ inline int64_t ss_find_or_insert(const SessTable &t, uint32_t key, bool &inserted) {
  uint64_t s = ss_home(t, key);
  inserted = false;
  for (uint64_t probe = 0; probe <= t.kmask; ++probe) {
    const uint32_t cur = t.kt[s].key;
    if (cur == key) return (int64_t)s;
    if (cur == kSessEmptyKey) {
      const uint32_t old = atomicCAS(&t.kt[s].key, kSessEmptyKey, key);
      if (old == kSessEmptyKey) {
        inserted = true;
        return (int64_t)s;
      }
      if (old == key) return (int64_t)s;
    }
    s = (s + 1) & t.kmask;
  }
  return -1;
}

// The same, loading the key's whole entry with the probe (one round trip
// when the key sits at its home slot, the common case): the found entry, or
// a blank one for a key this call inserted.
__device__ inline int64_t ss_find_entry(const SessTable &t, uint32_t key, SessKey &e, bool &inserted) {
  uint64_t s = ss_home(t, key);
  inserted = false;
  for (uint64_t probe = 0; probe <= t.kmask; ++probe) {
    e = ss_load_entry(&t.kt[s]);
    if (e.key == key) return (int64_t)s;
    if (e.key == kSessEmptyKey) {
      const uint32_t old = atomicCAS(&t.kt[s].key, kSessEmptyKey, key);
      if (old == kSessEmptyKey) {
        inserted = true;
        e = ss_blank(key);
        return (int64_t)s;
      }
      if (old == key) {
        e = ss_load_entry(&t.kt[s]);
        return (int64_t)s;
      }
    }
    s = (s + 1) & t.kmask;
  }
  return -1;
}

__global__ void k_ss_rehash(SessTable from, SessTable to) {
  const uint64_t cap = from.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    const SessKey e = from.kt[s];
    if (e.key == kSessEmptyKey) continue;
    bool ins;
    const int64_t d = ss_find_or_insert(to, e.key, ins);  // `to` is at most half full: d >= 0
    if (d >= 0) {
      SessKey x = e;
      x.emark = ~0ull;
      to.kt[d] = x;
    }
  }
}

void launch_ss_rehash(hipStream_t s, const SessTable &from, const SessTable &to) {
  launch_ss_reset(s, to);
  hipLaunchKernelGGL(k_ss_rehash, dim3(grid_for(from.kmask + 1, 256)), dim3(256), 0, s, from, to);
}

// ---------------------------------------------------------------------------
// arena compaction
// ---------------------------------------------------------------------------
__global__ void k_ss_ccount(SessTable t, uint32_t *newcap) {
  const uint64_t cap = t.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    const SessKey e = t.kt[s];
    const uint32_t len = e.key == kSessEmptyKey ? 0u : e.len;
    newcap[s] = len ? ss_grow_cap((uint64_t)len + 1) : 0u;
  }
}

__global__ void k_ss_ccopy(SessTable from, SessTable to, const uint32_t *newcap, const uint64_t *newoff) {
  const uint64_t cap = from.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    const SessKey e = from.kt[s];
    if (e.key == kSessEmptyKey) continue;
    const uint64_t o = newoff[s];
    for (uint32_t k = 0; k < e.len; ++k) ss_copy(to, o + k, from, e.off + k);
    to.kt[s].off = o;
    to.kt[s].cap = newcap[s];
  }
}

uint64_t ss_compact_scratch_bytes(uint64_t kcap) {
  return ((kcap * 4 + 255) & ~255ull) + (((kcap + 1) * 8 + 255) & ~255ull) + (scan_partials_needed(kcap) + 8) * 8;
}

static void compact_views(void *scratch, uint64_t kcap, uint32_t *&newcap, uint64_t *&newoff, uint64_t *&partial) {
  char *p = (char *)scratch;
  newcap = (uint32_t *)p;
  newoff = (uint64_t *)(p + ((kcap * 4 + 255) & ~255ull));
  partial = (uint64_t *)((char *)newoff + (((kcap + 1) * 8 + 255) & ~255ull));
}

void launch_ss_compact_plan(hipStream_t s, const SessTable &t, void *scratch, uint64_t *total) {
  const uint64_t kcap = t.kmask + 1;
  uint32_t *newcap;
  uint64_t *newoff, *partial;
  compact_views(scratch, kcap, newcap, newoff, partial);
  hipLaunchKernelGGL(k_ss_ccount, dim3(grid_for(kcap, 256)), dim3(256), 0, s, t, newcap);
  scan_excl_u32(s, newcap, newoff, kcap, partial, total);
}

void launch_ss_compact_copy(hipStream_t s, const SessTable &from, const SessTable &to, void *scratch) {
  const uint64_t kcap = from.kmask + 1;
  uint32_t *newcap;
  uint64_t *newoff, *partial;
  compact_views(scratch, kcap, newcap, newoff, partial);
  hipLaunchKernelGGL(k_ss_ccopy, dim3(grid_for(kcap, 256)), dim3(256), 0, s, from, to, newcap, newoff);
}

// ---------------------------------------------------------------------------
// replay path (per-record changelog, LAST)
// ---------------------------------------------------------------------------
// slot per record (kmask + 1 for HSG_KEY_NONE / table full), record index, and
// the valid flag that numbers per-record changelog rows
__global__ void k_ss_slot(Batch b, SessTable t, uint32_t *rslot, uint32_t *ridx, uint32_t *vflag, DevScalars *sc) {
  const uint32_t cap = (uint32_t)(t.kmask + 1);
  uint32_t err = 0;
  for (uint64_t i0 = blockIdx.x * (uint64_t)blockDim.x; i0 < b.n; i0 += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = i0 + threadIdx.x;
    bool ins = false;
    if (i < b.n) {
      const uint32_t key = b.key[i];
      uint32_t sl = cap;
      if (key != HSG_KEY_NONE) {
        const int64_t s = ss_find_or_insert(t, key, ins);
        if (s < 0) err |= ERR_OOM;
        else sl = (uint32_t)s;
      }
      rslot[i] = sl;
      ridx[i] = (uint32_t)i;
      vflag[i] = key != HSG_KEY_NONE ? 1u : 0u;
    }
    const uint64_t m = __ballot(ins);
    if ((threadIdx.x & 63) == 0 && m) atomicAdd((unsigned long long *)&t.meta[M_KEYS], (unsigned long long)__popcll(m));
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

// arena rows the replay's list growth needs, then the all-or-nothing decision
// (one thread, after every need has been added)
// (k_ss_process block q takes runs [256 q, 256 q + 256) and allocates from
// region arena_region(q): the need is summed per region)
__global__ __launch_bounds__(256) void k_ss_replay_need(SessTable t, const uint32_t *slot, const uint32_t *runs,
                                                        uint64_t R) {
  const uint64_t r = blockIdx.x * 256ull + threadIdx.x;
  uint64_t need = 0;
  if (r < R) {
    const SessKey e = t.kt[slot[runs[r]]];
    const uint64_t want = (uint64_t)e.len + (runs[r + 1] - runs[r]);
    if (want > e.cap) need = ss_grow_cap(want);
  }
  need = wave_sum_u64(need);
  if ((threadIdx.x & 63) == 0 && need)
    atomicAdd((unsigned long long *)&t.meta[M_RNEED + arena_region(blockIdx.x)], (unsigned long long)need);
}
__global__ void k_ss_replay_check(SessTable t) {
  const int r = threadIdx.x;
  if (r < kArenaRegions && t.meta[M_RTOP + r * kRegionStride] + t.meta[M_RNEED + r] > t.meta[M_REND + r * kRegionStride])
    t.meta[M_FAIL] = 1;
}

void launch_ss_replay_need(hipStream_t s, const SessTable &t, const uint32_t *slot, const uint32_t *runs, uint64_t R) {
  if (R) hipLaunchKernelGGL(k_ss_replay_need, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, s, t, slot, runs, R);
  hipLaunchKernelGGL(k_ss_replay_check, dim3(1), dim3(kArenaRegions), 0, s, t);
}

template <int MS>
__device__ inline void ss_load(const SessTable &t, uint64_t idx, int64_t (&a)[MS]) {
  const uint64_t *r = ss_row(t, idx) + 3;
#pragma unroll
  for (int s = 0; s < MS; ++s) a[s] = s < (int)t.ns ? (int64_t)r[s] : 0;
}
template <int MS>
__device__ inline void ss_store(const SessTable &t, uint64_t idx, int64_t st, int64_t en, uint32_t stamp,
                                const int64_t (&a)[MS]) {
  uint64_t *r = ss_row(t, idx);
  r[0] = (uint64_t)st;
  r[1] = (uint64_t)en;
  r[2] = stamp;
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s < (int)t.ns) r[3 + s] = (uint64_t)a[s];
}

// One thread per touched key replays the key's records in arrival order
// against its list (the reference's per-record fold: new point [t,t] with
// aggF init r, then mergeF over the overlapped sessions in end order, removed
// and replaced by the merged one). Keys are independent (findSessions filters
// by key), so this is the reference's result for any interleaving of keys.
template <int MS>
__global__ __launch_bounds__(256) void k_ss_process(Batch b, SessParams p, SessTable t, Program prog,
                                                    const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs,
                                                    uint64_t R, const uint64_t *out_pos, const int64_t *seq,
                                                    OutCols out, uint64_t out_base, DevScalars *sc) {
  __shared__ uint64_t swave[4];
  __shared__ uint64_t sbase;
  if (t.meta[M_FAIL]) return;  // uniform: the arena is refilled first, then this runs again
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const int ns = prog.n_slots;
  const bool active = r < R;
  uint64_t q0 = 0, q1 = 0;
  uint32_t sl = 0;
  SessKey e = ss_blank(0);
  int64_t live_delta = 0;
  if (active) {
    q0 = runs[r];
    q1 = runs[r + 1];
    sl = slot[q0];
    e = t.kt[sl];
  }
  const uint32_t key = e.key;
  // grow the key's list once for the whole run (each record adds <= 1
  // session); one arena bump per wave, within what k_ss_replay_need checked
  const uint64_t want = (uint64_t)e.len + (q1 - q0);
  const uint64_t new_cap = (active && want > e.cap) ? ss_grow_cap(want) : 0;
  const uint64_t incl = wave_incl_sum(new_cap);
  const uint64_t wtot = __shfl(incl, 63, 64);
  uint64_t wbase = 0;
  if (lane == 63 && wtot) arena_take(t, arena_region(blockIdx.x), wtot, wbase);  // within the checked need
  wbase = __shfl(wbase, 63, 64);
  uint64_t off = e.off, len = e.len;
  uint32_t lcap = e.cap;
  if (new_cap) {
    const uint64_t noff = wbase + incl - new_cap;
    for (uint64_t k = 0; k < len; ++k) ss_copy(t, noff + k, t, off + k);
    off = noff;
    lcap = (uint32_t)new_cap;
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
        const uint64_t m = (a + z) >> 1;
        if ((int64_t)ss_row(t, off + m)[1] < lo) a = m + 1;
        else z = m;
      }
      const uint64_t i0 = a;
      uint64_t i1 = i0;
      while (i1 < len && (int64_t)ss_row(t, off + i1)[0] <= hi) ++i1;
      // aggF initialValue r, then mergeF acc cur over the overlapped sessions
      int64_t acc[MS], ev[MS];
      identity_row<MS>(prog, acc);
      elem_row<MS>(prog, ev, b, i, seq1);
      combine_row<MS>(prog, acc, ev);
      int64_t s0 = ts, e0 = ts;
      for (uint64_t k = i0; k < i1; ++k) {
        const uint64_t *row = ss_row(t, off + k);
        const int64_t cs = (int64_t)row[0], ce = (int64_t)row[1];
        s0 = cs < s0 ? cs : s0;
        e0 = ce > e0 ? ce : e0;
        int64_t cur[MS];
        ss_load<MS>(t, off + k, cur);
        // passthrough columns: aggregateMergeF _ _ o2 keeps the existing
        // session's value (Codegen.hs:467), so after the fold the last
        // overlapped session in end order (k = i1 - 1) decides
        merge_row<MS>(prog, acc, cur);
      }
      const uint64_t c = i1 - i0;
      if (c == 0) {
        // insert at i0: near-sorted arrivals append (i0 == len), nothing moves
        for (uint64_t k = len; k > i0; --k) ss_copy(t, off + k, t, off + k - 1);
        len += 1;
      } else if (c > 1) {
        for (uint64_t k = i1; k < len; ++k) ss_copy(t, off + k - (c - 1), t, off + k);
        len -= c - 1;
      }
      live_delta += 1 - (int64_t)c;
      ss_store<MS>(t, off + i0, s0, e0, p.batch_id, acc);
      if (p.emit_mode == HSG_EMIT_PER_RECORD) {
        const uint64_t o = out_base + out_pos[i];
        out.key[o] = key;
        out.ws[o] = s0;
        out.we[o] = e0;
        out.src[o] = (int64_t)(seq1 - 1);
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value_reg<MS>(prog, j, acc);
        if (out.form) out.form[o] = out_form_reg<MS>(prog, acc);
      }
    }
    t.kt[sl].off = off;
    t.kt[sl].len = (uint32_t)len;
    t.kt[sl].cap = lcap;
    t.kt[sl].mvalid = 0;  // the replay path keeps no mirror of the last session
  }
  // per-batch changelog: the key's sessions stamped by this batch
  uint64_t mine = 0;
  if (active && p.emit_mode == HSG_EMIT_PER_BATCH)
    for (uint64_t k = 0; k < len; ++k) mine += (uint32_t)ss_row(t, off + k)[2] == p.batch_id;
  const uint64_t inc2 = wave_incl_sum(mine);
  if (lane == 63) swave[w] = inc2;
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t tot = swave[0] + swave[1] + swave[2] + swave[3];
    sbase = tot ? atomicAdd((unsigned long long *)&sc->out_rows, (unsigned long long)tot) : 0;
    if (tot) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tot);
  }
  __syncthreads();
  if (mine) {
    uint64_t o = out_base + sbase + inc2 - mine;
    for (int k = 0; k < w; ++k) o += swave[k];
    for (uint64_t k = 0; k < len; ++k) {
      const uint64_t *row = ss_row(t, off + k);
      if ((uint32_t)row[2] != p.batch_id) continue;
      out.key[o] = key;
      out.ws[o] = (int64_t)row[0];
      out.we[o] = (int64_t)row[1];
      out.src[o] = -1;
      for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, (const int64_t *)row + 3);
      if (out.form) out.form[o] = out_form(prog, (const int64_t *)row + 3);
      ++o;
    }
  }
  const uint64_t ld = wave_sum_u64((uint64_t)live_delta);
  if (lane == 0 && ld) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)ld);
}

template <int MS>
static void ss_process_launch(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t,
                              const Program &prog, const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs,
                              uint64_t R, const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base,
                              DevScalars *sc) {
  const uint64_t blocks = (R + 255) / 256;
  hipLaunchKernelGGL(k_ss_process<MS>, dim3((unsigned)blocks), dim3(256), 0, s, b, p, t, prog, slot, ridx, runs, R,
                     out_pos, seq, out, out_base, sc);
}

void launch_ss_process(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                       const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs, uint64_t R,
                       const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base, DevScalars *sc) {
  if (!R) return;
  if (prog.n_slots <= 2) ss_process_launch<2>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, sc);
  else if (prog.n_slots <= 4) ss_process_launch<4>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, sc);
  else if (prog.n_slots <= 8) ss_process_launch<8>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, sc);
  else ss_process_launch<kMaxSlots>(s, b, p, t, prog, slot, ridx, runs, R, out_pos, seq, out, out_base, sc);
}

// ---------------------------------------------------------------------------
// merge path: key-hash partition
// ---------------------------------------------------------------------------
constexpr int kSsTile = 4096;     // records per partition tile (= kPartTileRecs: the offsets pipeline)
constexpr int kSsPNT = 512;       // threads of the partition passes
constexpr int kSsSub = 1024;      // records per scatter sub-tile (LDS staging)

// bucket = the np_log2 key-hash bits below the `bshift` owner bits (multi-GPU:
// the owner of a key is the top log2(G) bits, so they carry no information here)
__device__ inline uint32_t ss_bucket(uint32_t key, int np_log2, int bshift) {
  return np_log2 ? (uint32_t)((key_hash(key) << bshift) >> (64 - np_log2)) : 0u;
}
__device__ inline uint64_t i64_img(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }

// per-tile bucket counts of the keyed records, tile-major; per-tile max ts
// image of EVERY record (stream time counts filtered records too)
__global__ __launch_bounds__(kSsPNT) void k_ss_phist(Batch b, int np_log2, int bshift, SessPart sp) {
  __shared__ uint32_t cnt[1 << 11];
  __shared__ uint64_t smx[kSsPNT / 64];
  __shared__ uint32_t skey[kSsPNT / 64];
  const int nb = 1 << np_log2;
  const uint64_t tile = blockIdx.x;
  for (int i = threadIdx.x; i < nb; i += kSsPNT) cnt[i] = 0;
  __syncthreads();
  const uint64_t base = tile * kSsTile;
  uint64_t mx = 0;
  uint32_t keyed = 0;
#pragma unroll
  for (int r = 0; r < kSsTile / kSsPNT; ++r) {
    const uint64_t i = base + (uint64_t)r * kSsPNT + threadIdx.x;
    if (i >= b.n) break;
    const uint32_t key = b.key[i];
    const uint64_t o = i64_img(b.ts[i]);
    mx = o > mx ? o : mx;
    if (key != HSG_KEY_NONE) {
      atomicAdd(&cnt[ss_bucket(key, np_log2, bshift)], 1u);
      ++keyed;
    }
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(mx, o, 64);
    mx = x > mx ? x : mx;
    keyed += __shfl_xor(keyed, o, 64);
  }
  if ((threadIdx.x & 63) == 0) {
    smx[threadIdx.x >> 6] = mx;
    skey[threadIdx.x >> 6] = keyed;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += kSsPNT) sp.hist[tile * (uint64_t)nb + i] = cnt[i];
  if (threadIdx.x == 0) {
    uint32_t kt = 0;
    for (int k = 0; k < kSsPNT / 64; ++k) {
      mx = smx[k] > mx ? smx[k] : mx;
      kt += skey[k];
    }
    sp.tmax[tile] = mx;
    if (sp.tkeyed) sp.tkeyed[tile] = kt;  // (bucket replay: the tile's changelog rows)
  }
}

void launch_ss_phist(hipStream_t s, const Batch &b, int np_log2, int bshift, uint64_t tiles, const SessPart &sp) {
  if (tiles) hipLaunchKernelGGL(k_ss_phist, dim3((unsigned)tiles), dim3(kSsPNT), 0, s, b, np_log2, bshift, sp);
}

// stream time after the batch (Processor.hs:139: max over every polled record)
__global__ __launch_bounds__(256) void k_ss_wm(SessPart sp, uint64_t tiles, int64_t wm_in, DevScalars *sc) {
  __shared__ uint64_t sw[4];
  uint64_t mx = 0;
  for (uint64_t t = threadIdx.x; t < tiles; t += 256) mx = sp.tmax[t] > mx ? sp.tmax[t] : mx;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(mx, o, 64);
    mx = x > mx ? x : mx;
  }
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = mx;
  __syncthreads();
  if (threadIdx.x) return;
  for (int k = 0; k < 4; ++k) mx = sw[k] > mx ? sw[k] : mx;
  const int64_t bmax = mx ? (int64_t)(mx ^ 0x8000000000000000ull) : INT64_MIN;
  sc->wm_out = bmax > wm_in ? bmax : wm_in;
}

void launch_ss_wm(hipStream_t s, const SessPart &sp, uint64_t tiles, int64_t wm_in, DevScalars *sc) {
  hipLaunchKernelGGL(k_ss_wm, dim3(1), dim3(256), 0, s, sp, tiles, wm_in, sc);
}

// Records of one tile to their bucket runs: sub-tiles of kSsSub records are
// counting-sorted by bucket into an LDS copy and written out with consecutive
// lanes on consecutive words of a run. Record: [key | valid bits << 32] [ts] [cols].
template <int W, bool IDX = false>
__global__ __launch_bounds__(kSsPNT) void k_ss_pscatter(Batch b, int np_log2, int bshift, int has_valid, SessPart sp) {
  __shared__ uint64_t stage[kSsSub * W];
  __shared__ uint32_t cursor[1 << 11];  // records of each bucket placed by earlier sub-tiles
  __shared__ uint32_t scnt[1 << 11];    // this sub-tile
  __shared__ uint32_t lstart[1 << 11];
  __shared__ uint16_t lbk[kSsSub];
  __shared__ uint32_t swave[kSsPNT / 64];
  constexpr int C = IDX ? W - 3 : W - 2;  // IDX: the record's arrival index in the last word
  constexpr int R = kSsSub / kSsPNT;
  const int nb = 1 << np_log2;
  const uint64_t tile = blockIdx.x;
  const uint32_t *orow = sp.offt + tile * (uint64_t)nb;
  uint64_t *out = IDX ? (uint64_t *)sp.srec : sp.rec;
  for (int i = threadIdx.x; i < nb; i += kSsPNT) cursor[i] = 0;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  for (int sub = 0; sub < kSsTile / kSsSub; ++sub) {
    const uint64_t base = tile * kSsTile + (uint64_t)sub * kSsSub;
    if (base >= b.n) break;  // uniform
    for (int i = threadIdx.x; i < nb; i += kSsPNT) scnt[i] = 0;
    __syncthreads();
    uint32_t key[R], pos[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t i = base + (uint64_t)r * kSsPNT + threadIdx.x;
      key[r] = i < b.n ? b.key[i] : HSG_KEY_NONE;
      pos[r] = key[r] != HSG_KEY_NONE ? atomicAdd(&scnt[ss_bucket(key[r], np_log2, bshift)], 1u) : ~0u;
    }
    __syncthreads();
    // sub-tile exclusive scan of the bucket counts -> LDS run starts
    const int per = (nb + kSsPNT - 1) / kSsPNT;
    const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
    uint32_t loc = 0;
    for (int k = lo; k < hi; ++k) loc += scnt[k];
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) swave[wv] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int k = 0; k < wv; ++k) run += swave[k];
    for (int k = lo; k < hi; ++k) {
      lstart[k] = run;
      run += scnt[k];
    }
    uint32_t placed = 0;
    for (int k = 0; k < kSsPNT / 64; ++k) placed += swave[k];
    __syncthreads();
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (pos[r] == ~0u) continue;
      const uint64_t i = base + (uint64_t)r * kSsPNT + threadIdx.x;
      const uint32_t bk = ss_bucket(key[r], np_log2, bshift);
      const uint32_t q = lstart[bk] + pos[r];
      uint64_t vb = 0;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        if (!(has_valid && b.valid[c] && !b.valid[c][i])) vb |= 1ull << c;
        if (IDX && has_valid && rec_decimal(b, c, i)) vb |= 1ull << (8 + c);  // literal-form bits
      }
      stage[q * W] = (uint64_t)key[r] | (vb << 32);
      stage[q * W + 1] = (uint64_t)b.ts[i];
#pragma unroll
      for (int c = 0; c < C; ++c) stage[q * W + 2 + c] = (uint64_t)b.col[c][i];
      if (IDX) stage[q * W + W - 1] = i;
      lbk[q] = (uint16_t)bk;
    }
    __syncthreads();
    // write-out: staged record q -> offt[tile][bk] + cursor[bk] + (q - lstart[bk])
    for (uint32_t t = threadIdx.x; t < placed * W; t += kSsPNT) {
      const uint32_t q = t / W, w = t - q * W;
      const uint32_t bk = lbk[q];
      const uint64_t dest = (uint64_t)orow[bk] + cursor[bk] + (q - lstart[bk]);
      out[dest * W + w] = stage[t];
    }
    lds_barrier();  // the next sub-tile reuses the LDS stage only
    for (int i = threadIdx.x; i < nb; i += kSsPNT) cursor[i] += scnt[i];
  }
}

void launch_ss_pscatter(hipStream_t s, const Batch &b, int np_log2, int bshift, uint64_t tiles, int words,
                        bool has_valid, const SessPart &sp) {
  if (!tiles) return;
  const dim3 g((unsigned)tiles), th(kSsPNT);
  const int hv = has_valid ? 1 : 0;
  switch (words) {
    case 2: hipLaunchKernelGGL(k_ss_pscatter<2>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 3: hipLaunchKernelGGL(k_ss_pscatter<3>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 4: hipLaunchKernelGGL(k_ss_pscatter<4>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 5: hipLaunchKernelGGL(k_ss_pscatter<5>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 6: hipLaunchKernelGGL(k_ss_pscatter<6>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 7: hipLaunchKernelGGL(k_ss_pscatter<7>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 8: hipLaunchKernelGGL(k_ss_pscatter<8>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    case 9: hipLaunchKernelGGL(k_ss_pscatter<9>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
    default: hipLaunchKernelGGL(k_ss_pscatter<10>, g, th, 0, s, b, np_log2, bshift, hv, sp); break;
  }
}

// ---------------------------------------------------------------------------
// merge path: runs and the sweep-merge of a key's runs with its sessions
// ---------------------------------------------------------------------------
constexpr int kMgTail = 2;  // resident sessions a key may rewrite in place (held in registers)

// contribution of one partitioned record to the slots (identity when absent)
template <int MS, class PV>
__device__ __attribute__((always_inline)) inline void ss_rec_elem(const PV &prog, const uint64_t *rec, int64_t (&e)[MS]) {
  const uint64_t vb = rec[0] >> 32;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    e[s] = 0;
    if (s >= prog.n()) continue;
    const int op = prog.op(s), c = prog.col(s);
    if (op == S_CNT_ALL) {
      e[s] = 1;
      continue;
    }
    if (!((vb >> c) & 1ull)) {
      e[s] = slot_identity_dev(op);
      continue;
    }
    const int64_t v = (int64_t)rec[2 + c];
    switch (op) {
      case S_CNT: e[s] = 1; break;
      case S_MIN_F:
      case S_MAX_F: e[s] = (int64_t)f64_ord(__builtin_bit_cast(double, v)); break;
      default: e[s] = v; break;
    }
  }
}

template <int MS, class PV>
__device__ __attribute__((always_inline)) inline void acc_row(const PV &prog, int64_t (&a)[MS], const int64_t (&e)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s < prog.n()) a[s] = slot_combine(prog.op(s), a[s], e[s]);
}

// One session of the sweep: start, end, aggregates, and whether a batch run
// is in it (-> stamped with the batch, a changelog row)
template <int MS>
struct MgSess {
  int64_t s, e;
  int64_t a[MS];
  uint32_t stamp;  // a resident's stamp (a session without a run is one resident, moved unchanged)
  bool fresh;
};
// the resident sessions a sweep may rewrite in place, in registers (kMgTail = 2)
template <int MS>
struct MgTail {
  MgSess<MS> t0, t1;
};
template <int MS>
__device__ __attribute__((always_inline)) inline void mg_clear(MgSess<MS> &x, uint32_t stamp) {
  x.s = x.e = 0;
  x.stamp = stamp;
  x.fresh = false;
#pragma unroll
  for (int s = 0; s < MS; ++s) x.a[s] = 0;
}

// Changelog rows of the fresh sessions of one key (per-batch mode), written
// by the sweep that produced them (k_ss_apply: every key once per batch).
struct EmitSink {
  OutCols out;
  uint64_t pos;   // next row; ~0 = count only
  uint32_t key;
  uint32_t n;     // fresh sessions seen
  const Program *rp;  // the op's program (output columns); unused when counting
};

template <int MS>
__device__ __attribute__((always_inline)) inline void mg_emit(EmitSink &k, const MgSess<MS> &c) {
  if (k.pos != ~0ull) {
    const Program &prog = *k.rp;
    const uint64_t o = k.pos++;
    k.out.key[o] = k.key;
    k.out.ws[o] = c.s;
    k.out.we[o] = c.e;
    k.out.src[o] = -1;
#pragma unroll
    for (int j = 0; j < kMaxAggs; ++j)  // static indices: the column pointers stay in registers
      if (j < prog.n_out) k.out.agg[j][o] = out_value_reg<MS>(prog, j, c.a);
    if (k.out.form) k.out.form[o] = out_form_reg<MS>(prog, c.a);
  }
  ++k.n;
}

template <int MS>
__device__ __attribute__((always_inline)) inline MgSess<MS> pick_tail(const MgTail<MS> &tail, uint64_t k) {
  // field-wise selects of two named sessions (an array picked by a runtime
  // index lands on the stack)
  static_assert(kMgTail == 2, "pick_tail");
  // bitwise blends: a select of two loads would be folded into a load through
  // a selected pointer, which keeps both sessions in stack memory
  const uint64_t m = k == 1 ? ~0ull : 0ull;
  auto blend = [m](int64_t a0, int64_t a1) { return (int64_t)(((uint64_t)a0 & ~m) | ((uint64_t)a1 & m)); };
  MgSess<MS> x;
  x.s = blend(tail.t0.s, tail.t1.s);
  x.e = blend(tail.t0.e, tail.t1.e);
#pragma unroll
  for (int s = 0; s < MS; ++s) x.a[s] = blend(tail.t0.a[s], tail.t1.a[s]);
  x.stamp = (uint32_t)blend(tail.t0.stamp, tail.t1.stamp);
  x.fresh = blend(tail.t0.fresh, tail.t1.fresh) != 0;
  return x;
}

// runs precomputed by k_ss_sort: rows [start][end][aggs]
struct RunsGlobal {
  const uint64_t *runs;
  uint32_t rstride;
  int ns;
  __device__ int64_t start(uint32_t r) const { return (int64_t)runs[(uint64_t)r * rstride]; }
  __device__ int64_t end(uint32_t r) const { return (int64_t)runs[(uint64_t)r * rstride + 1]; }
  template <int MS, class PV>
  __device__ void aggs(const PV &, uint32_t r, int64_t (&a)[MS]) const {
    const uint64_t *q = runs + (uint64_t)r * rstride + 2;
#pragma unroll
    for (int s = 0; s < MS; ++s) a[s] = s < ns ? (int64_t)q[s] : 0;
  }
};

// Sweep of one key: its resident sessions [i0, len) (in registers when
// `tail_regs`: then len - i0 <= kMgTail) and its runs [r0, r1), in start
// order; items closer than gap merge (next.start - running end <= gap). With
// APPLY the merged sessions are written at dst + i0 + k, else only counted.
template <int MS, bool APPLY, class RS, class PV>
__device__ __attribute__((always_inline)) inline uint32_t mg_sweep(const PV &prog, const SessTable &t, int64_t gap, const RS &rs, uint32_t r0,
                                    uint32_t r1, uint64_t off, uint64_t i0, uint64_t len, bool tail_regs,
                                    const MgTail<MS> &tail, uint64_t dst, uint32_t batch_id,
                                    EmitSink *sink = nullptr, SessKey *mirror = nullptr) {
  const int ns = prog.n();
  uint64_t j = i0;   // next resident
  uint32_t r = r0;   // next run
  uint32_t k = 0;    // merged sessions so far
  MgSess<MS> cur;
  bool have = false;
  for (;;) {
    // next item in start order: resident j or run r (ties: resident first)
    const bool has_res = j < len, has_run = r < r1;
    if (!has_res && !has_run) break;
    MgSess<MS> it;
    bool take_res = false;
    if (has_res) {
      if (tail_regs) {
        it = pick_tail<MS>(tail, j - i0);
      } else {
        const uint64_t *row = ss_row(t, off + j);
        it.s = (int64_t)row[0];
        it.e = (int64_t)row[1];
        if (APPLY) {
          it.stamp = (uint32_t)row[2];
#pragma unroll
          for (int s = 0; s < MS; ++s) it.a[s] = s < ns ? (int64_t)row[3 + s] : 0;
        }
      }
      take_res = !has_run || it.s <= rs.start(r);
    }
    if (take_res) {
      it.fresh = false;
      ++j;
    } else {
      it.s = rs.start(r);
      it.e = rs.end(r);
      it.fresh = true;
      it.stamp = batch_id;
      if (APPLY) rs.template aggs<MS>(prog, r, it.a);
      ++r;
    }
    if (have && (int64_t)((uint64_t)it.s - (uint64_t)cur.e) <= gap) {
      cur.e = it.e > cur.e ? it.e : cur.e;
      cur.fresh = cur.fresh || it.fresh;
      if (APPLY) acc_row<MS>(prog, cur.a, it.a);
    } else {
      if (have) {
        if (APPLY) ss_store<MS>(t, dst + i0 + k, cur.s, cur.e, cur.fresh ? batch_id : cur.stamp, cur.a);
        if (sink && cur.fresh) mg_emit<MS>(*sink, cur);
        ++k;
      }
      cur = it;
      have = true;
    }
  }
  if (have) {
    if (APPLY) ss_store<MS>(t, dst + i0 + k, cur.s, cur.e, cur.fresh ? batch_id : cur.stamp, cur.a);
    if (sink && cur.fresh) mg_emit<MS>(*sink, cur);
    ++k;
    if (mirror) {  // the list's new last session (the sweep runs to its end) into the entry's mirror
      const bool m = prog.n() <= kSessMirrorSlots;
      if (m) {
        mirror->ms = cur.s;
        mirror->me = cur.e;
#pragma unroll
        for (int s = 0; s < kSessMirrorSlots; ++s) mirror->ma[s] = s < MS ? cur.a[s] : 0;
      }
      mirror->mvalid = m ? 1u : 0u;
    }
  }
  return k;
}

// first resident session with end >= lo: galloping back from the end (near-
// sorted arrivals touch the last session or none), then binary search
__device__ __attribute__((always_inline)) inline uint64_t mg_first_end_ge(const SessTable &t, uint64_t off, uint64_t len, int64_t lo) {
  uint64_t hi = len, step = 1;
  while (hi > 0) {
    const uint64_t probe = hi > step ? hi - step : 0;
    if ((int64_t)ss_row(t, off + probe)[1] < lo) {
      uint64_t a = probe + 1, z = hi;  // answer in (probe, hi]
      while (a < z) {
        const uint64_t m = (a + z) >> 1;
        if ((int64_t)ss_row(t, off + m)[1] < lo) a = m + 1;
        else z = m;
      }
      return a;
    }
    hi = probe;
    step <<= 1;
  }
  return 0;
}

// Plan of one key against its list: the first resident its runs can reach,
// the merged count, and the rows of a fresh list when it cannot stay in place.
// fast: planned from the entry's mirror of the last session, no list read
// (mg_fast: the batch's first run starts at or after the last session's
// start, so no resident but the last can be reached, the one before ending
// more than gap before the last starts; the last is touched iff the first
// run comes within gap of its end).
template <int MS, class PV>
__device__ __attribute__((always_inline)) inline void mg_mirror_tail(const PV &prog, const SessKey &e, uint32_t batch_id,
                                      MgTail<MS> &tail);
template <class RS>
__device__ inline bool mg_fast(const RS &rs, uint32_t ra, const SessKey &e) {
  return e.mvalid && e.len > 0 && rs.start(ra) >= e.ms;
}
template <int MS, class RS, class PV>
__device__ __attribute__((always_inline)) inline void mg_plan(const PV &prog, const SessTable &t, int64_t gap, const RS &rs, uint32_t ra,
                               uint32_t rb, const SessKey &e, bool fast, uint32_t batch_id, uint64_t &i0, uint32_t &M,
                               uint32_t &newcap, uint32_t *fresh = nullptr) {
  const int64_t lo = (int64_t)((uint64_t)rs.start(ra) - (uint64_t)gap);
  MgTail<MS> tail;
  if (fast) {
    i0 = e.me >= lo ? e.len - 1 : e.len;
    mg_mirror_tail<MS>(prog, e, batch_id, tail);
  } else {
    i0 = mg_first_end_ge(t, e.off, e.len, lo);
  }
  EmitSink cnt{OutCols{}, ~0ull, 0, 0, nullptr};
  M = mg_sweep<MS, false>(prog, t, gap, rs, ra, rb, e.off, i0, e.len, fast, tail, 0, 0, &cnt);
  if (fresh) *fresh = cnt.n;
  // in place when the merged list fits and the rewritten tail fits the
  // registers, else a fresh list (prefix copied)
  newcap = (i0 + M > e.cap || e.len - i0 > kMgTail) ? ss_grow_cap(i0 + M + 1) : 0u;
}

// The key's last session from its entry's mirror (valid when e.mvalid).
template <int MS, class PV>
__device__ __attribute__((always_inline)) inline void mg_mirror_tail(const PV &prog, const SessKey &e, uint32_t batch_id,
                                      MgTail<MS> &tail) {
  mg_clear<MS>(tail.t0, batch_id);  // a fast-path resident always merges with a run: rewritten as fresh
  mg_clear<MS>(tail.t1, batch_id);
  tail.t0.s = e.ms;
  tail.t0.e = e.me;
#pragma unroll
  for (int s = 0; s < MS; ++s) tail.t0.a[s] = (s < kSessMirrorSlots && s < prog.n()) ? e.ma[s] : 0;
}

// The entry after a merge (its mirror was written by the sweep).
__device__ inline void ss_entry_commit(SessKey &ke, uint64_t off, uint32_t len, uint32_t newcap) {
  ke.off = off;
  ke.len = len;
  if (newcap) ke.cap = newcap;
}

// Apply a planned key: the list at dst (fresh rows: the prefix copied first).
// The rewritten residents come from registers: the mirror (fast) or the rows
// loaded here (in place), else from the old list (relocated).
template <int MS, class RS, class PV>
__device__ __attribute__((always_inline)) inline void mg_apply(const PV &prog, const SessTable &t, int64_t gap, const RS &rs, uint32_t ra,
                                uint32_t rb, const SessKey &e, bool fast, uint64_t i0, uint64_t dst, bool reloc,
                                uint32_t batch_id, EmitSink *sink = nullptr, SessKey *mirror = nullptr,
                                bool prefix_copied = false) {
  const int ns = prog.n();
  if (reloc && !prefix_copied)
    for (uint64_t k = 0; k < i0; ++k) ss_copy(t, dst + k, t, e.off + k);
  MgTail<MS> tail;
  if (fast) {
    mg_mirror_tail<MS>(prog, e, batch_id, tail);
  } else {
    auto fill = [&](MgSess<MS> &x, uint64_t j) {
      mg_clear<MS>(x, 0u);
      if (!reloc && j < e.len) {
        const uint64_t *row = ss_row(t, e.off + j);
        x.s = (int64_t)row[0];
        x.e = (int64_t)row[1];
        x.stamp = (uint32_t)row[2];
#pragma unroll
        for (int s = 0; s < MS; ++s) x.a[s] = s < ns ? (int64_t)row[3 + s] : 0;
      }
    };
    fill(tail.t0, i0);
    fill(tail.t1, i0 + 1);
  }
  mg_sweep<MS, true>(prog, t, gap, rs, ra, rb, e.off, i0, e.len, fast || !reloc, tail, dst, batch_id, sink, mirror);
}

// ---------------------------------------------------------------------------
// k_ss_sort: one workgroup per bucket, in sub-buckets (further key-hash bits)
// of about half a sort chunk each. A sub-bucket's records are grouped by key
// through an LDS hash table (count, scan, place with their values), each key's
// few records are sorted by ts by its thread and walked into gap-delimited
// runs (aggregates folded from the LDS copy) and one group record per key. A
// sub-bucket with a key of more than kSoSmall records (hot keys), or more than
// kSoCH records, is left to k_ss_merge_big (its bit in sp.bigmask).
// ---------------------------------------------------------------------------
#ifndef HSG_SO_CH_LOG2
#define HSG_SO_CH_LOG2 10
#endif
constexpr int kSoNT = 512;
constexpr int kSoCH = 1 << HSG_SO_CH_LOG2;  // records per sub-bucket
constexpr int kSoTabLog2 = HSG_SO_CH_LOG2 + 1;
constexpr int kSoTab = 1 << kSoTabLog2;  // LDS hash table entries
constexpr int kSoMaxSubLog2 = 6;   // up to 64 sub-buckets (buckets of < 2^16 records)
constexpr int kSoSmall = 32;       // a key's records sorted by its own thread

template <int W>
struct SortLds {
  uint32_t tkey[kSoTab];
  uint32_t tcnt[kSoTab];    // records of the key; after the scan the placement cursor
  uint32_t tstart[kSoTab];  // first position of the key's segment
  uint16_t tgid[kSoTab];    // group index of the key in the sub-bucket
  int64_t ts[kSoCH];        // segments: ts and the record's other words (word 0, columns)
  uint64_t vw[kSoCH * (W - 1)];
  uint16_t qslot[kSoCH];    // table slot of the record at each segment position
  uint32_t wsum[kSoNT / 64];
  uint32_t subcnt[1 << kSoMaxSubLog2];
  uint32_t suboff[1 << kSoMaxSubLog2];  // first entry of each sub-bucket in the bucket's index list
  uint32_t subgrp[1 << kSoMaxSubLog2];  // key groups of each sub-bucket
  uint32_t ngrp, nrun, maxseg;
  uint64_t grpbase;
};

// sub-bucket of a key: the sl key-hash bits below the owner and bucket bits
__device__ inline uint32_t ss_sub(uint32_t key, int hs, int sl) {
  return sl ? (uint32_t)((key_hash(key) << hs) >> (64 - sl)) : 0u;
}
// sub-bucket bits for a bucket of m records: sub-buckets of about kSoCH / 2
__device__ inline int ss_sub_log2(uint64_t m) {
  int sl = 0;
  while (((uint64_t)(kSoCH / 2) << sl) < m && sl < kSoMaxSubLog2) ++sl;
  return sl;
}

__device__ inline int64_t ts_of(uint64_t img) { return (int64_t)(img ^ 0x8000000000000000ull); }

// contribution of one record (word 0 and columns in `v`, as in the LDS copy:
// v[0] = key | valid bits << 32, v[1 + c] = column c)
template <int MS, class PV>
__device__ __attribute__((always_inline)) inline void ss_vw_elem(const PV &prog, const uint64_t *v, int64_t (&e)[MS]) {
  const uint64_t vb = v[0] >> 32;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    e[s] = 0;
    if (s >= prog.n()) continue;
    const int op = prog.op(s), c = prog.col(s);
    if (op == S_CNT_ALL) {
      e[s] = 1;
      continue;
    }
    if (!((vb >> c) & 1ull)) {
      e[s] = slot_identity_dev(op);
      continue;
    }
    const int64_t x = (int64_t)v[1 + c];
    switch (op) {
      case S_CNT: e[s] = 1; break;
      case S_MIN_F:
      case S_MAX_F: e[s] = (int64_t)f64_ord(__builtin_bit_cast(double, x)); break;
      default: e[s] = x; break;
    }
  }
}

template <int MS, int W>
__global__ __launch_bounds__(kSoNT) void k_ss_sort(SessParams p, SessTable t, Program prog, int np_log2, int bshift,
                                                   SessPart sp, DevScalars *sc) {
  __shared__ SortLds<W> L;
  const uint64_t c0 = phase_clock();
  uint64_t c_ins = 0, c_scan = 0, c_place = 0, c_key = 0, c1 = 0;
  constexpr int B = 8;  // loads in flight per thread in the bucket passes
  const uint32_t b = blockIdx.x;
  const uint64_t r0 = sp.bstart[b], r1 = sp.bstart[b + 1];
  const uint64_t m = r1 - r0;
  if (m == 0) {
    if (threadIdx.x == 0) sp.bigmask[b] = 0;
    return;
  }
  const uint64_t *recs = sp.rec + r0 * W;
  const int sl = ss_sub_log2(m), hs = bshift + np_log2;
  const int nsub = 1 << sl;
  // the bucket's records copied grouped by sub-bucket (sp.scopy, the bucket's
  // own range): every later pass reads only its sub-bucket's records
  uint64_t *scopy = sp.scopy + r0 * W;
  if (threadIdx.x < (1 << kSoMaxSubLog2)) {
    L.subcnt[threadIdx.x] = 0;
    L.subgrp[threadIdx.x] = 0;
  }
  __syncthreads();
  const bool indexable = m < 65536;
  // (lanes of a wave with the same sub-bucket found by ballots: one LDS
  // atomic per sub-bucket and wave instead of one per record)
  const int lane0 = threadIdx.x & 63;
  const uint64_t lt = lane0 ? (~0ull >> (64 - lane0)) : 0ull;
  auto peers = [&](uint32_t q, bool in) {
    uint64_t pm = __ballot(in);
#pragma unroll
    for (int bit = 0; bit < kSoMaxSubLog2; ++bit) {
      if (bit >= sl) break;
      const uint64_t bb = __ballot((q >> bit) & 1u);
      pm &= ((q >> bit) & 1u) ? bb : ~bb;
    }
    return pm;
  };
  if (indexable)
    for (uint64_t i0 = 0; i0 < m; i0 += (uint64_t)kSoNT * B) {
      uint32_t q[B];
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const uint64_t i = i0 + (uint64_t)u * kSoNT + threadIdx.x;
        q[u] = i < m ? ss_sub((uint32_t)recs[i * W], hs, sl) : ~0u;
      }
#pragma unroll
      for (int u = 0; u < B; ++u) {
        const bool in = q[u] != ~0u;
        const uint64_t pm = peers(q[u], in);
        if (in && (pm & lt) == 0) atomicAdd(&L.subcnt[q[u]], (uint32_t)__popcll(pm));
      }
    }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t o = 0;
    for (int q = 0; q < nsub; ++q) {
      L.suboff[q] = o;
      o += L.subcnt[q];
    }
  }
  __syncthreads();
  if (threadIdx.x < (1 << kSoMaxSubLog2)) L.subcnt[threadIdx.x] = 0;
  __syncthreads();
  // the records copied grouped by sub-bucket: each sub-bucket then reads its
  // records contiguously (no per-record index, no gather)
  constexpr int B2 = W <= 3 ? 4 : 2;
  if (indexable)
    for (uint64_t i0 = 0; i0 < m; i0 += (uint64_t)kSoNT * B2) {
      uint64_t v[B2][W];
#pragma unroll
      for (int u = 0; u < B2; ++u) {
        const uint64_t i = i0 + (uint64_t)u * kSoNT + threadIdx.x;
#pragma unroll
        for (int w = 0; w < W; ++w) v[u][w] = i < m ? recs[i * W + w] : 0;
      }
#pragma unroll
      for (int u = 0; u < B2; ++u) {
        const uint64_t i = i0 + (uint64_t)u * kSoNT + threadIdx.x;
        const uint32_t q = i < m ? ss_sub((uint32_t)v[u][0], hs, sl) : ~0u;
        const bool in = q != ~0u;
        const uint64_t pm = peers(q, in);
        const uint32_t rk = (uint32_t)__popcll(pm & lt);
        // the group's lowest lane reserves for the group; the others read its base
        uint32_t base = 0;
        if (in && rk == 0) base = atomicAdd(&L.subcnt[q], (uint32_t)__popcll(pm));
        const int leader = in ? __ffsll((long long)pm) - 1 : lane0;
        base = __shfl(base, leader, 64);
        if (in) {
          uint64_t *d = scopy + (uint64_t)(L.suboff[q] + base + rk) * W;
#pragma unroll
          for (int w = 0; w < W; ++w) d[w] = v[u][w];
        }
      }
    }
  __syncthreads();
  uint64_t bigmask = indexable ? 0ull : ~0ull;  // a bucket that cannot be indexed goes to the big path whole
  c1 = phase_clock();
  const uint32_t rstride = 2 + prog.n_slots;
  constexpr int RP = kSoCH / kSoNT;  // records per thread in a sub-bucket pass
  for (int sub = 0; indexable && sub < nsub; ++sub) {
    const uint32_t m2 = L.subcnt[sub];
    if (m2 == 0) continue;  // uniform
    if (m2 > (uint32_t)kSoCH) {
      bigmask |= 1ull << sub;
      continue;
    }
    const uint64_t *lst = scopy + (uint64_t)L.suboff[sub] * W;
    uint64_t ca = phase_clock();
    // 1. keys of the sub-bucket into the LDS table, records per key; the
    // records' words stay in registers for the placement
    for (int h = threadIdx.x; h < kSoTab; h += kSoNT) {
      L.tkey[h] = 0xFFFFFFFFu;
      L.tcnt[h] = 0;
    }
    if (threadIdx.x == 0) {
      L.ngrp = 0;
      L.nrun = 0;
      L.maxseg = 0;
    }
    uint64_t rw[RP][W];
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      const uint32_t j = u * kSoNT + threadIdx.x;
#pragma unroll
      for (int w = 0; w < W; ++w) rw[u][w] = j < m2 ? lst[(uint64_t)j * W + w] : 0;
    }
    lds_barrier();
    uint32_t hslot[RP];
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      hslot[u] = ~0u;
      if (u * kSoNT + threadIdx.x >= m2) continue;
      const uint32_t key = (uint32_t)rw[u][0];
      // the key-hash bits below the bucket and sub-bucket bits: the groups
      // come out in key-table home order (ss_home), so k_ss_apply's
      // neighbouring lanes touch neighbouring key entries
      uint32_t h = (uint32_t)((key_hash(key) << (hs + sl)) >> (64 - kSoTabLog2));
      for (;;) {
        const uint32_t cur = L.tkey[h];
        if (cur == key) break;
        if (cur == 0xFFFFFFFFu) {
          const uint32_t old = atomicCAS(&L.tkey[h], 0xFFFFFFFFu, key);
          if (old == 0xFFFFFFFFu || old == key) break;
        }
        h = (h + 1) & (kSoTab - 1);
      }
      hslot[u] = h;
      atomicAdd(&L.tcnt[h], 1u);
    }
    lds_barrier();
    { const uint64_t cb = phase_clock(); c_ins += cb - ca; ca = cb; }
    // 2. segment starts: exclusive scan of the counts
    // (records in the low 16 bits, occupied slots in the high: one scan gives
    // each key its segment start and its group index)
    constexpr int TP = kSoTab / kSoNT;
    uint32_t loc = 0, mx = 0;
#pragma unroll
    for (int u = 0; u < TP; ++u) {
      const uint32_t c = L.tcnt[threadIdx.x * TP + u];
      loc += c + (c ? 0x10000u : 0u);
      mx = c > mx ? c : mx;
    }
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t v = __shfl_up(incl, o, 64);
      if (lane >= o) incl += v;
    }
    if (lane == 63) L.wsum[wv] = incl;
    if (mx > (uint32_t)kSoSmall) atomicMax(&L.maxseg, mx);
    lds_barrier();
    if (L.maxseg > (uint32_t)kSoSmall) {  // uniform: a hot key, the big path takes the sub-bucket
      bigmask |= 1ull << sub;
      lds_barrier();
      continue;
    }
    uint32_t run = incl - loc, all = 0;
    for (int k = 0; k < kSoNT / 64; ++k) {
      if (k < wv) run += L.wsum[k];
      all += L.wsum[k];
    }
#pragma unroll
    for (int u = 0; u < TP; ++u) {
      const int h = threadIdx.x * TP + u;
      const uint32_t c = L.tcnt[h];
      L.tstart[h] = run & 0xFFFFu;
      L.tcnt[h] = run & 0xFFFFu;
      L.tgid[h] = (uint16_t)(run >> 16);
      run += c + (c ? 0x10000u : 0u);
    }
    if (threadIdx.x == 0) L.ngrp = all >> 16;
    if (threadIdx.x == 0) L.subgrp[sub] = L.ngrp;
    // a sub-bucket's sorted records and (sparse) group records live at its
    // records' positions in the bucket
    const uint64_t runbase = r0 + L.suboff[sub];
    uint32_t *gsp = sp.gsparse + (r0 + L.suboff[sub]) * 4;
    lds_barrier();
    { const uint64_t cb = phase_clock(); c_scan += cb - ca; ca = cb; }
    // 3. place (ts, words) in the key's segment
#pragma unroll
    for (int u = 0; u < RP; ++u) {
      if (hslot[u] == ~0u) continue;
      const uint32_t q = atomicAdd(&L.tcnt[hslot[u]], 1u);
      L.ts[q] = (int64_t)rw[u][1];
      L.vw[q * (W - 1)] = rw[u][0];
#pragma unroll
      for (int w = 2; w < W; ++w) L.vw[q * (W - 1) + w - 1] = rw[u][w];
      L.qslot[q] = (uint16_t)hslot[u];
    }
    lds_barrier();
    { const uint64_t cb = phase_clock(); c_place += cb - ca; ca = cb; }
    // 4. every record ranked by ts within its key's segment (<= kSoSmall) and
    // written out in (key, ts) order; one group record per key
    for (uint32_t q = threadIdx.x; q < m2; q += kSoNT) {
      const uint32_t h = L.qslot[q];
      const uint32_t sa = L.tstart[h], se = L.tcnt[h];
      const int64_t v = L.ts[q];
      uint32_t rank = 0;
      for (uint32_t j = sa; j < se; ++j) {
        const int64_t tj = L.ts[j];
        rank += (tj < v || (tj == v && j < q)) ? 1u : 0u;
      }
      uint64_t *row = sp.srec + (runbase + sa + rank) * W;
      row[0] = (uint64_t)v;
#pragma unroll
      for (int w = 0; w < W - 1; ++w) row[1 + w] = L.vw[q * (W - 1) + w];
    }
    for (int h = threadIdx.x; h < kSoTab; h += kSoNT) {
      const uint32_t key = L.tkey[h];
      if (key == 0xFFFFFFFFu) continue;
      const uint32_t sa = L.tstart[h];
      *reinterpret_cast<uint4 *>(gsp + (uint64_t)L.tgid[h] * 4) =
          make_uint4(key, (uint32_t)(runbase + sa), L.tcnt[h] - sa, 0u);
    }
    lds_barrier();
    c_key += phase_clock() - ca;
  }
  // the bucket's group records, dense: one reservation per bucket
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int q = 0; q < nsub; ++q) {
      if (!indexable || ((bigmask >> q) & 1ull) || L.subcnt[q] == 0 || L.subcnt[q] > (uint32_t)kSoCH) L.subgrp[q] = 0;
      tot += L.subgrp[q];
    }
    L.grpbase = tot ? atomicAdd((unsigned long long *)&t.meta[M_GRP], (unsigned long long)tot) : 0;
    sp.bigmask[b] = bigmask;
    if (bigmask) atomicAdd((unsigned long long *)&t.meta[M_BIG], 1ull);
  }
  __syncthreads();
  uint64_t d = L.grpbase;
  for (int q = 0; q < nsub; ++q) {
    const uint32_t c = L.subgrp[q];
    const uint4 *src = reinterpret_cast<const uint4 *>(sp.gsparse + (r0 + L.suboff[q]) * 4);
    for (uint32_t j = threadIdx.x; j < c; j += kSoNT) reinterpret_cast<uint4 *>(sp.groups)[d + j] = src[j];
    d += c;
  }
  if (kPhaseClocks && threadIdx.x == 0) {  // phase clocks (100 MHz), HSG_PHASES
    const uint64_t c2 = phase_clock();
    atomicAdd((unsigned long long *)&sc->scratch[24], (unsigned long long)(c1 - c0));
    atomicAdd((unsigned long long *)&sc->scratch[25], (unsigned long long)c_ins);
    atomicAdd((unsigned long long *)&sc->scratch[26], (unsigned long long)c_scan);
    atomicAdd((unsigned long long *)&sc->scratch[27], (unsigned long long)c_place);
    atomicAdd((unsigned long long *)&sc->scratch[28], (unsigned long long)c_key);
    atomicAdd((unsigned long long *)&sc->scratch[29], (unsigned long long)(c2 - c0));
    atomicAdd((unsigned long long *)&sc->scratch[30], 1ull);
  }
}

template <int MS>
static void sort_launch_w(hipStream_t s, int words, dim3 g, const SessParams &p, const SessTable &t,
                          const Program &prog, int np_log2, int bshift, const SessPart &sp, DevScalars *sc) {
  const dim3 th(kSoNT);
  switch (words) {
    case 2: hipLaunchKernelGGL((k_ss_sort<MS, 2>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 3: hipLaunchKernelGGL((k_ss_sort<MS, 3>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 4: hipLaunchKernelGGL((k_ss_sort<MS, 4>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 5: hipLaunchKernelGGL((k_ss_sort<MS, 5>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 6: hipLaunchKernelGGL((k_ss_sort<MS, 6>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 7: hipLaunchKernelGGL((k_ss_sort<MS, 7>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 8: hipLaunchKernelGGL((k_ss_sort<MS, 8>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    case 9: hipLaunchKernelGGL((k_ss_sort<MS, 9>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
    default: hipLaunchKernelGGL((k_ss_sort<MS, kSessMaxWords>), g, th, 0, s, p, t, prog, np_log2, bshift, sp, sc); break;
  }
}

void launch_ss_sort(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, int np_log2,
                    int bshift, int words, const SessPart &sp, DevScalars *sc) {
  const dim3 g(1u << np_log2);
  if (prog.n_slots <= 2) sort_launch_w<2>(s, words, g, p, t, prog, np_log2, bshift, sp, sc);
  else if (prog.n_slots <= 4) sort_launch_w<4>(s, words, g, p, t, prog, np_log2, bshift, sp, sc);
  else sort_launch_w<8>(s, words, g, p, t, prog, np_log2, bshift, sp, sc);
}

// a key's batch records, sorted by ts (k_ss_sort), as sweep items: record r
// is the point [ts, ts]; the sweep merges items closer than the gap, so
// feeding points instead of pre-merged runs gives the same sessions
template <int W>
struct RecItems {
  const uint64_t *rows;  // [n][W]: ts, word 0, columns
  __device__ int64_t start(uint32_t r) const { return (int64_t)rows[(uint64_t)r * W]; }
  __device__ int64_t end(uint32_t r) const { return (int64_t)rows[(uint64_t)r * W]; }
  template <int MS, class PV>
  __device__ void aggs(const PV &prog, uint32_t r, int64_t (&a)[MS]) const {
    ss_vw_elem<MS>(prog, rows + (uint64_t)r * W + 1, a);
  }
};

// The same with the key's first two records in registers, loaded right after
// the group record, beside the key-table probe: the sweeps of most keys (one
// or two records in a batch) then wait on no record load. W <= 3 (ts, word 0,
// one column); further records from memory.
template <int W>
struct RecItemsPf {
  static_assert(W >= 2 && W <= 3, "RecItemsPf");
  const uint64_t *rows;
  uint32_t ra;
  uint64_t t0, t1;           // ts of records ra, ra + 1
  uint64_t v0[W - 1], v1[W - 1];  // their word 0 and column
  __device__ void load(uint32_t a, uint32_t n) {
    ra = a;
    const uint64_t *p = rows + (uint64_t)a * W;
    t0 = n > 0 ? p[0] : 0;
    t1 = n > 1 ? p[W] : 0;
#pragma unroll
    for (int k = 0; k < W - 1; ++k) {
      v0[k] = n > 0 ? p[1 + k] : 0;
      v1[k] = n > 1 ? p[W + 1 + k] : 0;
    }
  }
  __device__ int64_t start(uint32_t r) const {
    return (int64_t)(r == ra ? t0 : r == ra + 1 ? t1 : rows[(uint64_t)r * W]);
  }
  __device__ int64_t end(uint32_t r) const { return start(r); }
  template <int MS, class PV>
  __device__ void aggs(const PV &prog, uint32_t r, int64_t (&a)[MS]) const {
    if (r - ra < 2) {
      uint64_t v[W - 1];
#pragma unroll
      for (int k = 0; k < W - 1; ++k) v[k] = r == ra ? v0[k] : v1[k];
      ss_vw_elem<MS>(prog, v, a);
    } else {
      ss_vw_elem<MS>(prog, rows + (uint64_t)r * W + 1, a);
    }
  }
};
template <int W, bool PF = (W <= 3)>
struct ApplyItems {
  using T = RecItems<W>;
};
template <int W>
struct ApplyItems<W, true> {
  using T = RecItemsPf<W>;
};

__device__ inline void ss_store_entry(SessKey *p, const SessKey &e) {
  uint4 *q = reinterpret_cast<uint4 *>(p);
  q[0] = make_uint4(e.key, e.len, (uint32_t)e.off, (uint32_t)(e.off >> 32));
  q[1] = make_uint4(e.cap, e.mvalid, (uint32_t)e.emark, (uint32_t)(e.emark >> 32));
  q[2] = make_uint4((uint32_t)(uint64_t)e.ms, (uint32_t)((uint64_t)e.ms >> 32), (uint32_t)(uint64_t)e.me,
                    (uint32_t)((uint64_t)e.me >> 32));
  q[3] = make_uint4((uint32_t)(uint64_t)e.ma[0], (uint32_t)((uint64_t)e.ma[0] >> 32), (uint32_t)(uint64_t)e.ma[1],
                    (uint32_t)((uint64_t)e.ma[1] >> 32));
}

// the key's slot (inserting it when absent) and its entry, probing from the
// slot whose entry `home` was already loaded; -1 = table full
__device__ inline int64_t ss_resolve(const SessTable &t, uint32_t key, uint64_t s, SessKey home, SessKey &e,
                                     bool &inserted) {
  inserted = false;
  for (uint64_t probe = 0; probe <= t.kmask; ++probe) {
    const SessKey cur = probe ? ss_load_entry(&t.kt[s]) : home;
    if (cur.key == key) {
      e = cur;
      return (int64_t)s;
    }
    if (cur.key == kSessEmptyKey) {
      const uint32_t old = atomicCAS(&t.kt[s].key, kSessEmptyKey, key);
      if (old == kSessEmptyKey) {
        inserted = true;
        e = ss_blank(key);
        return (int64_t)s;
      }
    }
    s = (s + 1) & t.kmask;
  }
  return -1;
}

// ---------------------------------------------------------------------------
// k_ss_apply: one thread per key group (every key once per batch). Plan,
// reserve the block's fresh lists in its arena region (all or nothing: a block
// that cannot stays undone, the host compacts and runs the pass again), apply
// and write the changelog rows of the fresh sessions.
// ---------------------------------------------------------------------------
constexpr int kApNT = 512;  // one arena / changelog reservation per 512 keys; two blocks per CU

template <int MS, int W, uint64_t SIG>
__global__ __launch_bounds__(kApNT) void k_ss_apply(SessParams p, SessTable t, Program prog, SessPart sp,
                                                    OutCols out, uint64_t out_base, DevScalars *sc) {
  const ProgView<SIG> pv(prog);  // the common aggregate sets: slot ops baked in
  __shared__ uint64_t ws[kApNT / 64];
  __shared__ uint64_t we[kApNT / 64];
  __shared__ uint64_t sbase, sobase, srbase;
  __shared__ int sfail;
  const uint32_t blk = blockIdx.x;
  if (sp.done[blk]) return;  // uniform: applied by an earlier pass of this batch
  const uint64_t ng = t.meta[M_GRP];
  const uint64_t g0 = (uint64_t)blk * kApNT;
  if (g0 >= ng) return;  // uniform
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t g = g0 + threadIdx.x;
  const bool act = g < ng;
  typename ApplyItems<W>::T rs{sp.srec};
  uint32_t key = 0, ra = 0, nr = 0, newcap = 0, M = 0, fresh = 0;
  uint64_t i0 = 0;
  int64_t sl = -1;
  bool ins = false, fast = false;
  SessKey e = ss_blank(0);
  uint32_t err = 0;
  if (act) {
    const uint4 gr = *reinterpret_cast<const uint4 *>(sp.groups + g * 4);
    key = gr.x;
    ra = gr.y;
    nr = gr.z;
    if constexpr (W <= 3) rs.load(ra, nr);  // in flight during the probe
    // the entry at the key's home slot, loaded whole with the probe (the key
    // is found there unless a collision displaced it)
    const uint64_t home = ss_home(t, key);
    sl = ss_resolve(t, key, home, ss_load_entry(&t.kt[home]), e, ins);
    if (sl < 0) err |= ERR_OOM;
    else {
      // near-sorted arrivals: planned from the entry's mirror, no list read
      fast = mg_fast(rs, ra, e);
      mg_plan<MS>(pv, t, p.gap, rs, ra, ra + nr, e, fast, p.batch_id, i0, M, newcap, &fresh);
    }
  }
  const bool live = act && sl >= 0;
  {
    // keys inserted count now: a block that fails below finds them next pass
    const uint64_t ksum = wave_sum_u64(ins ? 1ull : 0ull);
    if (lane == 0 && ksum) atomicAdd((unsigned long long *)&t.meta[M_KEYS], (unsigned long long)ksum);
    if (err) atomicOr(&sc->err, err);
  }
  // block exclusive scans of the fresh list rows and of the changelog rows
  // (with, in the high 32 bits, the relocated lists whose prefix
  // k_ss_reloc_copy copies after this kernel)
  const bool rel = live && newcap != 0 && i0 != 0;
  const uint64_t need = newcap, nem = (live ? fresh : 0) | ((uint64_t)(rel ? 1 : 0) << 32);
  const uint64_t incl = wave_incl_sum(need), einc = wave_incl_sum(nem);
  if (lane == 63) {
    ws[wv] = incl;
    we[wv] = einc;
  }
  __syncthreads();
  uint64_t before = 0, total = 0, ebefore = 0, etotal = 0;
  for (int k = 0; k < kApNT / 64; ++k) {
    if (k < wv) {
      before += ws[k];
      ebefore += we[k];
    }
    total += ws[k];
    etotal += we[k];
  }
  const uint64_t etot = etotal & 0xFFFFFFFFull, rtot = etotal >> 32;
  if (threadIdx.x == 0) {
    uint64_t base = 0;
    const int fail = total ? !arena_take(t, arena_region(blk), total, base) : 0;
    sfail = fail;
    sbase = base;
    sobase = 0;
    srbase = 0;
    if (fail) {
      atomicOr((unsigned int *)&t.meta[M_FAIL], 1u);
    } else {
      if (etot) {
        // per-batch mode: touched = rows (the host takes it from out_rows)
        if (p.emit_mode == HSG_EMIT_PER_BATCH) sobase = atomicAdd((unsigned long long *)&sc->out_rows, (unsigned long long)etot);
        else atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)etot);
      }
      if (rtot) srbase = atomicAdd((unsigned long long *)&t.meta[M_RELOC], (unsigned long long)rtot);
    }
  }
  __syncthreads();
  if (sfail) return;  // uniform: keys inserted above stay (idempotent); the block runs again
  int64_t ld = 0;
  if (live) {
    const bool reloc = newcap != 0;
    const uint64_t dst = reloc ? sbase + before + incl - need : e.off;
    const uint64_t eb = (ebefore & 0xFFFFFFFFull) + (einc & 0xFFFFFFFFull) - (nem & 0xFFFFFFFFull);
    EmitSink sink{out, p.emit_mode == HSG_EMIT_PER_BATCH ? out_base + sobase + eb : ~0ull, key, 0, &prog};
    if (rel) {
      // the untouched prefix [0, i0) of a relocated list is copied after this
      // kernel (k_ss_reloc_copy, every row of every list in parallel): a
      // thread copying its own list row by row would hold its whole wave
      // (~1 key in 12 per C4 batch outgrows its rows)
      uint64_t *r = sp.reloc + 3 * (srbase + (ebefore >> 32) + (einc >> 32) - 1);
      r[0] = e.off;
      r[1] = dst;
      r[2] = i0;
    }
    SessKey ne = e;
    mg_apply<MS>(pv, t, p.gap, rs, ra, ra + nr, e, fast, i0, dst, reloc, p.batch_id, &sink, &ne, true);
    ss_entry_commit(ne, dst, (uint32_t)(i0 + M), reloc ? newcap : 0u);
    ss_store_entry(&t.kt[sl], ne);
    ld = (int64_t)M - (int64_t)(e.len - i0);
  }
  const uint64_t lsum = wave_sum_u64((uint64_t)ld);
  if (lane == 0 && lsum) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)lsum);
  // (the done flag is read by a later launch only: no wait here for the
  // block's scattered stores, which a __syncthreads would add)
  lds_barrier();
  if (threadIdx.x == 0) sp.done[blk] = 1;
}

template <int MS, uint64_t SIG>
static void apply_launch_w(hipStream_t s, int words, dim3 g, const SessParams &p, const SessTable &t,
                           const Program &prog, const SessPart &sp, OutCols out, uint64_t out_base, DevScalars *sc) {
  const dim3 th(kApNT);
  switch (words) {
    case 2: hipLaunchKernelGGL((k_ss_apply<MS, 2, SIG>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 3: hipLaunchKernelGGL((k_ss_apply<MS, 3, SIG>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 4: hipLaunchKernelGGL((k_ss_apply<MS, 4, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 5: hipLaunchKernelGGL((k_ss_apply<MS, 5, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 6: hipLaunchKernelGGL((k_ss_apply<MS, 6, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 7: hipLaunchKernelGGL((k_ss_apply<MS, 7, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 8: hipLaunchKernelGGL((k_ss_apply<MS, 8, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    case 9: hipLaunchKernelGGL((k_ss_apply<MS, 9, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
    default: hipLaunchKernelGGL((k_ss_apply<MS, kSessMaxWords, 0>), g, th, 0, s, p, t, prog, sp, out, out_base, sc); break;
  }
}

void launch_ss_apply(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, uint64_t n_bound,
                     int words, const SessPart &sp, OutCols out, uint64_t out_base, DevScalars *sc) {
  const dim3 g((unsigned)((n_bound + kApNT - 1) / kApNT + 1));
  // the common aggregate sets of a session GROUP BY (one column or none) with
  // their slot program baked in; every other program reads it at run time
  const uint64_t sig = program_sig(prog);
  if (sig == kSigCntSumI) apply_launch_w<2, kSigCntSumI>(s, words, g, p, t, prog, sp, out, out_base, sc);
  else if (sig == kSigCntSumF) apply_launch_w<2, kSigCntSumF>(s, words, g, p, t, prog, sp, out, out_base, sc);
  else if (sig == kSigCnt) apply_launch_w<2, kSigCnt>(s, words, g, p, t, prog, sp, out, out_base, sc);
  else if (sig == kSigSumMaxI) apply_launch_w<2, kSigSumMaxI>(s, words, g, p, t, prog, sp, out, out_base, sc);
  else if (prog.n_slots <= 2) apply_launch_w<2, 0>(s, words, g, p, t, prog, sp, out, out_base, sc);
  else if (prog.n_slots <= 4) apply_launch_w<4, 0>(s, words, g, p, t, prog, sp, out, out_base, sc);
  else apply_launch_w<8, 0>(s, words, g, p, t, prog, sp, out, out_base, sc);
}

// the prefixes of relocated lists: 16 lanes per list on consecutive words
// (four loads in flight each; a list is ~10-60 rows of 3 + slots words)
constexpr int kRcLanes = 16;
__global__ __launch_bounds__(256) void k_ss_reloc_copy(SessTable t, SessPart sp) {
  const uint64_t n = t.meta[M_RELOC];
  const int lane = threadIdx.x & (kRcLanes - 1);
  const uint64_t w0 = (blockIdx.x * (uint64_t)blockDim.x + threadIdx.x) / kRcLanes;
  const uint64_t nw_all = ((uint64_t)gridDim.x * blockDim.x) / kRcLanes;
  const uint32_t sw = t.stride;
  for (uint64_t e = w0; e < n; e += nw_all) {
    const uint64_t src = sp.reloc[3 * e] * sw, dst = sp.reloc[3 * e + 1] * sw, nw = sp.reloc[3 * e + 2] * sw;
    for (uint64_t b = 0; b < nw; b += 4 * kRcLanes) {
      uint64_t v[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t w = b + (uint64_t)j * kRcLanes + lane;
        v[j] = w < nw ? t.rows[src + w] : 0;
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const uint64_t w = b + (uint64_t)j * kRcLanes + lane;
        if (w < nw) t.rows[dst + w] = v[j];
      }
    }
  }
}

void launch_ss_reloc_copy(hipStream_t s, const SessTable &t, const SessPart &sp, uint64_t n_bound) {
  uint64_t blocks = (n_bound / 4 * kRcLanes + 255) / 256;  // (lists: at most one per key)
  if (blocks > 8192) blocks = 8192;
  if (!blocks) blocks = 1;
  hipLaunchKernelGGL(k_ss_reloc_copy, dim3((unsigned)blocks), dim3(256), 0, s, t, sp);
}

// ---------------------------------------------------------------------------
// k_ss_merge_big: a bucket too large for one sort (hot keys) is merged chunk
// by chunk by one workgroup: each chunk sorted in LDS, its runs merged into the
// resident sessions before the next chunk (the aggregates commute, so the
// chunking does not change the result), one arena reservation per chunk.
// ---------------------------------------------------------------------------
constexpr int kMgNT = 512;
constexpr int kMgCH = 2048;
constexpr int kMgPer = kMgCH / kMgNT;

struct MgLds {
  uint32_t key[kMgCH];
  uint64_t tsu[kMgCH];
  uint16_t idx[kMgCH];
  int64_t rs[kMgCH];  // runs: start, end (inclusive), first sorted position
  int64_t re[kMgCH];
  uint16_t rbeg[kMgCH + 1];
  uint16_t gfirst[kMgCH + 1];  // key groups: first run
  uint32_t wsum[kMgNT / 64];
  uint64_t red[kMgNT / 64];
  uint64_t base;
  uint32_t tbase;
  uint32_t fill;
  int fail;
};

// runs of the LDS-sorted chunk, aggregates folded from the member records
template <int W>
struct RunsLds {
  const MgLds *L;
  const uint64_t *recs;
  __device__ int64_t start(uint32_t r) const { return L->rs[r]; }
  __device__ int64_t end(uint32_t r) const { return L->re[r]; }
  template <int MS, class PV>
  __device__ void aggs(const PV &prog, uint32_t r, int64_t (&a)[MS]) const {
#pragma unroll
    for (int s = 0; s < MS; ++s) a[s] = s < prog.n() ? slot_identity_dev(prog.op(s)) : 0;
    for (uint32_t q = L->rbeg[r]; q < L->rbeg[r + 1]; ++q) {
      int64_t e[MS];
      ss_rec_elem<MS>(prog, recs + (uint64_t)L->idx[q] * W, e);
      acc_row<MS>(prog, a, e);
    }
  }
};

__device__ inline uint32_t mg_scan(MgLds &L, uint32_t v, uint32_t &total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t incl = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) L.wsum[wv] = incl;
  __syncthreads();
  uint32_t before = 0;
  total = 0;
  for (int k = 0; k < kMgNT / 64; ++k) {
    if (k < wv) before += L.wsum[k];
    total += L.wsum[k];
  }
  __syncthreads();
  return before + incl - v;
}

__device__ inline uint64_t mg_scan64(MgLds &L, uint64_t v, uint64_t &total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint64_t incl = wave_incl_sum(v);
  if (lane == 63) L.red[wv] = incl;
  __syncthreads();
  uint64_t before = 0;
  total = 0;
  for (int k = 0; k < kMgNT / 64; ++k) {
    if (k < wv) before += L.red[k];
    total += L.red[k];
  }
  __syncthreads();
  return before + incl - v;
}

template <int MS, int W>
__global__ __launch_bounds__(kMgNT) void k_ss_merge_big(SessParams p, SessTable t, Program prog, int np_log2,
                                                        int bshift, SessPart sp, DevScalars *sc) {
  __shared__ MgLds L;
  const uint32_t b = blockIdx.x;
  const uint64_t bigmask = sp.bigmask[b];
  if (!bigmask) return;  // uniform
  const uint64_t r0 = sp.bstart[b], r1 = sp.bstart[b + 1];
  const uint32_t nch = (uint32_t)((r1 - r0 + kMgCH - 1) / kMgCH);
  const int sl = ss_sub_log2(r1 - r0), hs = bshift + np_log2;
  const int lane = threadIdx.x & 63;
  int64_t live_delta = 0;
  uint64_t keys_new = 0;
  uint32_t err = 0;
  for (uint32_t c = sp.progress[b]; c < nch; ++c) {
    // window c of the bucket's records, restricted to the big sub-buckets
    const uint64_t q0 = r0 + (uint64_t)c * kMgCH;
    const uint32_t mw = (uint32_t)(r1 - q0 < kMgCH ? r1 - q0 : kMgCH);
    const uint64_t *recs = sp.rec + q0 * W;
    if (threadIdx.x == 0) L.fill = 0;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < mw; i += kMgNT) {
      const uint32_t key = (uint32_t)recs[(uint64_t)i * W];
      if (!((bigmask >> ss_sub(key, hs, sl)) & 1ull)) continue;
      const uint32_t q = atomicAdd(&L.fill, 1u);
      L.key[q] = key;
      L.tsu[q] = (uint64_t)recs[(uint64_t)i * W + 1] ^ 0x8000000000000000ull;
      L.idx[q] = (uint16_t)i;
    }
    __syncthreads();
    const uint32_t m = L.fill;
    if (m == 0) {  // uniform
      if (c + 1 == nch && threadIdx.x == 0) sp.progress[b] = nch;
      __syncthreads();
      continue;
    }
    uint32_t N = 2;
    while (N < m) N <<= 1;
    for (uint32_t i = m + threadIdx.x; i < N; i += kMgNT) {
      L.key[i] = 0xFFFFFFFFu;
      L.tsu[i] = ~0ull;
      L.idx[i] = 0;
    }
    __syncthreads();
    for (uint32_t k = 2; k <= N; k <<= 1) {
      for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
        for (uint32_t i = threadIdx.x; i < N; i += kMgNT) {
          const uint32_t ixj = i ^ jj;
          if (ixj <= i) continue;
          const uint32_t ka = L.key[i], kb = L.key[ixj];
          const uint64_t ta = L.tsu[i], tb = L.tsu[ixj];
          const bool gt = ka > kb || (ka == kb && ta > tb);
          if (gt == ((i & k) == 0)) {
            L.key[i] = kb;
            L.key[ixj] = ka;
            L.tsu[i] = tb;
            L.tsu[ixj] = ta;
            const uint16_t x = L.idx[i];
            L.idx[i] = L.idx[ixj];
            L.idx[ixj] = x;
          }
        }
        __syncthreads();
      }
    }
    // runs
    uint32_t heads = 0, hmask = 0;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t i = threadIdx.x * kMgPer + u;
      if (i >= m) break;
      bool h = i == 0 || L.key[i] != L.key[i - 1];
      if (!h) h = (int64_t)((uint64_t)ts_of(L.tsu[i]) - (uint64_t)ts_of(L.tsu[i - 1])) > p.gap;
      if (h) {
        hmask |= 1u << u;
        ++heads;
      }
    }
    uint32_t nrun;
    uint32_t rpos = mg_scan(L, heads, nrun);
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      if (!((hmask >> u) & 1u)) continue;
      const uint32_t i = threadIdx.x * kMgPer + u;
      L.rbeg[rpos] = (uint16_t)i;
      L.rs[rpos] = ts_of(L.tsu[i]);
      if (rpos > 0) L.re[rpos - 1] = ts_of(L.tsu[i - 1]);
      ++rpos;
    }
    if (threadIdx.x == 0) {
      L.rbeg[nrun] = (uint16_t)m;
      L.re[nrun - 1] = ts_of(L.tsu[m - 1]);
    }
    __syncthreads();
    // key groups
    uint32_t gh = 0, gmask = 0;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t r = threadIdx.x * kMgPer + u;
      if (r >= nrun) break;
      if (r == 0 || L.key[L.rbeg[r]] != L.key[L.rbeg[r - 1]]) {
        gmask |= 1u << u;
        ++gh;
      }
    }
    uint32_t ngrp;
    uint32_t gpos = mg_scan(L, gh, ngrp);
#pragma unroll
    for (int u = 0; u < kMgPer; ++u)
      if ((gmask >> u) & 1u) L.gfirst[gpos++] = (uint16_t)(threadIdx.x * kMgPer + u);
    if (threadIdx.x == 0) L.gfirst[ngrp] = (uint16_t)nrun;
    __syncthreads();
    // plan every group of the chunk (thread owns groups tid, tid + NT, ...)
    const RunsLds<W> rsrc{&L, recs};
    int64_t gslot[kMgPer];
    uint64_t gi0[kMgPer];
    uint32_t gM[kMgPer], gcap[kMgPer];
    SessKey ge[kMgPer];
    uint64_t need = 0;
    uint32_t nt = 0;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t g = u * kMgNT + threadIdx.x;
      gslot[u] = -1;
      gcap[u] = 0;
      gM[u] = 0;
      gi0[u] = 0;
      ge[u] = ss_blank(0);
      if (g >= ngrp) continue;
      const uint32_t ra = L.gfirst[g], rb = L.gfirst[g + 1];
      bool ins;
      const int64_t sl = ss_find_or_insert(t, L.key[L.rbeg[ra]], ins);
      if (sl < 0) {
        err |= ERR_OOM;
        continue;
      }
      keys_new += ins ? 1 : 0;
      gslot[u] = sl;
      ++nt;
      if (!ins) ge[u] = t.kt[sl];
      mg_plan<MS>(ProgRT(prog), t, p.gap, rsrc, ra, rb, ge[u], false, p.batch_id, gi0[u], gM[u], gcap[u]);
      need += gcap[u];
    }
    uint64_t tneed;
    const uint64_t npos = mg_scan64(L, need, tneed);
    uint32_t ttot;
    const uint32_t tpos = mg_scan(L, nt, ttot);
    if (threadIdx.x == 0) {
      L.fail = 0;
      L.base = 0;
      if (tneed) {
        uint64_t base = 0;
        L.fail = !arena_take(t, arena_region(b), tneed, base);
        L.base = base;
      }
      L.tbase = (!L.fail && ttot) ? (uint32_t)atomicAdd((unsigned long long *)&t.meta[M_TLEN], (unsigned long long)ttot) : 0;
    }
    __syncthreads();
    if (L.fail) {
      // resumable at this chunk: nothing of it was applied (inserted keys stay)
      if (threadIdx.x == 0) {
        sp.progress[b] = c;
        atomicOr((unsigned int *)&t.meta[M_FAIL], 1u);
      }
      break;
    }
    uint64_t my_alloc = L.base + npos;
    uint32_t tp = L.tbase + tpos;
    const uint64_t bmark = (uint64_t)(~p.batch_id) << 32;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t g = u * kMgNT + threadIdx.x;
      if (g >= ngrp || gslot[u] < 0) continue;
      const uint32_t ra = L.gfirst[g], rb = L.gfirst[g + 1];
      const bool reloc = gcap[u] != 0;
      uint64_t dst = ge[u].off;
      if (reloc) {
        dst = my_alloc;
        my_alloc += gcap[u];
      }
      SessKey &ke = t.kt[gslot[u]];
      mg_apply<MS>(ProgRT(prog), t, p.gap, rsrc, ra, rb, ge[u], false, gi0[u], dst, reloc, p.batch_id, nullptr, &ke);
      ss_entry_commit(ke, dst, (uint32_t)(gi0[u] + gM[u]), reloc ? gcap[u] : 0u);
      atomicMin((unsigned long long *)&ke.emark, (unsigned long long)(bmark | gi0[u]));
      sp.touched[tp++] = (uint32_t)gslot[u];
      live_delta += (int64_t)gM[u] - (int64_t)(ge[u].len - gi0[u]);
    }
    __syncthreads();
    if (c + 1 == nch && threadIdx.x == 0) sp.progress[b] = nch;
  }
  const uint64_t ld = wave_sum_u64((uint64_t)live_delta);
  const uint64_t kn = wave_sum_u64(keys_new);
  if (lane == 0) {
    if (ld) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)ld);
    if (kn) atomicAdd((unsigned long long *)&t.meta[M_KEYS], (unsigned long long)kn);
  }
  if (err) atomicOr(&sc->err, err);
}

template <int MS>
static void big_launch_w(hipStream_t s, int words, dim3 g, const SessParams &p, const SessTable &t,
                         const Program &prog, int nl, int bs, const SessPart &sp, DevScalars *sc) {
  const dim3 th(kMgNT);
  switch (words) {
    case 2: hipLaunchKernelGGL((k_ss_merge_big<MS, 2>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 3: hipLaunchKernelGGL((k_ss_merge_big<MS, 3>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 4: hipLaunchKernelGGL((k_ss_merge_big<MS, 4>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 5: hipLaunchKernelGGL((k_ss_merge_big<MS, 5>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 6: hipLaunchKernelGGL((k_ss_merge_big<MS, 6>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 7: hipLaunchKernelGGL((k_ss_merge_big<MS, 7>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 8: hipLaunchKernelGGL((k_ss_merge_big<MS, 8>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    case 9: hipLaunchKernelGGL((k_ss_merge_big<MS, 9>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
    default: hipLaunchKernelGGL((k_ss_merge_big<MS, kSessMaxWords>), g, th, 0, s, p, t, prog, nl, bs, sp, sc); break;
  }
}

void launch_ss_merge_big(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, int np_log2,
                         int bshift, int words, const SessPart &sp, DevScalars *sc) {
  const dim3 g(1u << np_log2);
  if (prog.n_slots <= 2) big_launch_w<2>(s, words, g, p, t, prog, np_log2, bshift, sp, sc);
  else if (prog.n_slots <= 4) big_launch_w<4>(s, words, g, p, t, prog, np_log2, bshift, sp, sc);
  else big_launch_w<8>(s, words, g, p, t, prog, np_log2, bshift, sp, sc);
}

// ---------------------------------------------------------------------------
// per-batch changelog of the merge path: every session of a touched key at or
// after the lowest index the batch rewrote, stamped by this batch. A key may
// be in the touched list more than once (a big bucket: once per chunk); the
// entry that takes the key's mark (resetting it) emits. emit = 0: count only.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ss_emit(SessTable t, Program prog, SessPart sp, uint32_t batch_id, int emit,
                                                 OutCols out, uint64_t out_base, DevScalars *sc) {
  __shared__ uint64_t swave[4];
  __shared__ uint64_t sbase;
  const uint64_t n = t.meta[M_TLEN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t blk = blockIdx.x * 256ull; blk < n; blk += (uint64_t)gridDim.x * 256ull) {
    const uint64_t q = blk + threadIdx.x;
    uint64_t cnt = 0, i0 = 0, off = 0, len = 0;
    uint32_t key = 0;
    if (q < n) {
      const uint32_t sl = sp.touched[q];
      const uint64_t mk = atomicExch((unsigned long long *)&t.kt[sl].emark, ~0ull);
      if ((uint32_t)(mk >> 32) == ~batch_id) {
        i0 = mk & 0xFFFFFFFFull;
        const SessKey e = t.kt[sl];
        key = e.key;
        off = e.off;
        len = e.len;
        for (uint64_t k = i0; k < len; ++k) cnt += (uint32_t)ss_row(t, off + k)[2] == batch_id;
      }
    }
    const uint64_t incl = wave_incl_sum(cnt);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t tot = swave[0] + swave[1] + swave[2] + swave[3];
      sbase = tot && emit ? atomicAdd((unsigned long long *)&sc->out_rows, (unsigned long long)tot) : 0;
      if (tot) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tot);
    }
    __syncthreads();
    if (emit && cnt) {
      uint64_t o = out_base + sbase + incl - cnt;
      for (int k = 0; k < w; ++k) o += swave[k];
      for (uint64_t k = i0; k < len; ++k) {
        const uint64_t *row = ss_row(t, off + k);
        if ((uint32_t)row[2] != batch_id) continue;
        out.key[o] = key;
        out.ws[o] = (int64_t)row[0];
        out.we[o] = (int64_t)row[1];
        out.src[o] = -1;
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, (const int64_t *)row + 3);
      if (out.form) out.form[o] = out_form(prog, (const int64_t *)row + 3);
        ++o;
      }
    }
    __syncthreads();
  }
}

void launch_ss_emit(hipStream_t s, const SessTable &t, const Program &prog, const SessPart &sp, uint32_t batch_id,
                    int emit, uint64_t n_bound, OutCols out, uint64_t out_base, DevScalars *sc) {
  uint64_t blocks = (n_bound + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  if (!blocks) blocks = 1;
  hipLaunchKernelGGL(k_ss_emit, dim3((unsigned)blocks), dim3(256), 0, s, t, prog, sp, batch_id, emit, out, out_base,
                     sc);
}

// ---------------------------------------------------------------------------
// ssDump: every live session (key, start, end, aggs)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ss_dump(SessTable t, Program prog, OutCols out, uint64_t out_cap,
                                                 uint64_t *counter) {
  __shared__ uint64_t swave[4];
  __shared__ uint64_t sbase;
  const uint64_t cap = t.kmask + 1;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t blk = blockIdx.x * 256ull; blk < cap; blk += (uint64_t)gridDim.x * 256ull) {
    const uint64_t s = blk + threadIdx.x;
    uint64_t len = 0, off = 0;
    uint32_t key = kSessEmptyKey;
    if (s < cap) {
      const SessKey e = t.kt[s];
      key = e.key;
      if (key != kSessEmptyKey) {
        len = e.len;
        off = e.off;
      }
    }
    const uint64_t incl = wave_incl_sum(len);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint64_t tot = swave[0] + swave[1] + swave[2] + swave[3];
      sbase = tot ? atomicAdd((unsigned long long *)counter, (unsigned long long)tot) : 0;
    }
    __syncthreads();
    uint64_t o = sbase + incl - len;
    for (int k = 0; k < w; ++k) o += swave[k];
    for (uint64_t k = 0; k < len && o < out_cap; ++k, ++o) {
      const uint64_t *row = ss_row(t, off + k);
      out.key[o] = key;
      out.ws[o] = (int64_t)row[0];
      out.we[o] = (int64_t)row[1];
      out.src[o] = -1;
      for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, (const int64_t *)row + 3);
      if (out.form) out.form[o] = out_form(prog, (const int64_t *)row + 3);
    }
    __syncthreads();
  }
}

void launch_ss_dump(hipStream_t s, const SessTable &t, const Program &prog, OutCols out, uint64_t out_cap,
                    uint64_t *counter) {
  uint64_t blocks = (t.kmask + 1 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_ss_dump, dim3((unsigned)blocks), dim3(256), 0, s, t, prog, out, out_cap, counter);
}

// ---------------------------------------------------------------------------
// Bucket replay (hsg_session.h): per-record changelog, LAST, literal forms.
// ---------------------------------------------------------------------------
#ifndef HSG_BR_NT
#define HSG_BR_NT 512
#endif
constexpr int kBrNT = HSG_BR_NT;
// k_br_replay's register tail for records before the last session (ops of at
// most this many slots; 0: off). Measured on C4 EMIT CHANGES: the tail cuts
// the replay phase from 12.0 to 10.8 us per sub-pass, but its 166 VGPRs leave
// room for one 512-thread workgroup per CU instead of two: 2.61 -> 4.19 ms per
// batch. The replay is bound by how many sub-passes are in flight, not by one
// sub-pass's latency, so it stays off.
#ifndef HSG_BR_WPE
#define HSG_BR_WPE 1  // minimum waves per SIMD asked of the compiler for k_br_replay (1: none)
#endif
#ifndef HSG_BR_TAIL_MS
#define HSG_BR_TAIL_MS 0
#endif
constexpr int kBrTab = 2 * kBrCap;  // LDS key table entries (load <= 1/2)
constexpr int kBrMaxSubLog2 = 6;
constexpr int kBrSubNT = 256;

int br_words(int n_cols) { return 3 + n_cols; }

// sub-bucket bits of a bucket of m records: sub-buckets of about kBrCap / 2
__device__ inline int br_sub_log2(uint64_t m) {
  int sl = 0;
  while (((uint64_t)(kBrCap / 2) << sl) < m && sl < kBrMaxSubLog2) ++sl;
  return sl;
}

void launch_br_scatter(hipStream_t s, const Batch &b, int np_log2, int bshift, uint64_t tiles, int words,
                       const SessPart &sp) {
  if (!tiles) return;
  const dim3 g((unsigned)tiles), th(kSsPNT);
  bool hv = false;
  for (int c = 0; c < kMaxCols; ++c) hv = hv || b.valid[c] != nullptr;
  const int v = hv ? 1 : 0;
  switch (words) {
    case 3: hipLaunchKernelGGL((k_ss_pscatter<3, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 4: hipLaunchKernelGGL((k_ss_pscatter<4, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 5: hipLaunchKernelGGL((k_ss_pscatter<5, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 6: hipLaunchKernelGGL((k_ss_pscatter<6, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 7: hipLaunchKernelGGL((k_ss_pscatter<7, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 8: hipLaunchKernelGGL((k_ss_pscatter<8, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 9: hipLaunchKernelGGL((k_ss_pscatter<9, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    case 10: hipLaunchKernelGGL((k_ss_pscatter<10, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
    default: hipLaunchKernelGGL((k_ss_pscatter<11, true>), g, th, 0, s, b, np_log2, bshift, v, sp); break;
  }
}

// Per bucket: its records grouped by sub-bucket (copied into sp.scopy over
// the bucket's own range, so each sub-bucket pass of k_br_replay reads one
// contiguous stretch) and the sub-bucket starts (sp.subst[b][0 .. 2^sl]); a
// sub-bucket of more than kBrCap records flags the batch (M_BRBIG) before
// any state is touched.
template <int W>
__global__ __launch_bounds__(kBrSubNT) void k_br_subhist(SessTable t, int np_log2, int bshift, SessPart sp) {
  __shared__ uint32_t cnt[1 << kBrMaxSubLog2];
  __shared__ uint32_t cur[1 << kBrMaxSubLog2];
  const uint32_t b = blockIdx.x;
  const uint64_t r0 = sp.bstart[b], m = sp.bstart[b + 1] - r0;
  const int sl = br_sub_log2(m), nsub = 1 << sl, hs = bshift + np_log2;
  if (threadIdx.x < (1 << kBrMaxSubLog2)) cnt[threadIdx.x] = 0;
  lds_barrier();
  for (uint64_t q = threadIdx.x; q < m; q += kBrSubNT) {
    const uint32_t key = (uint32_t)sp.srec[(r0 + q) * W];
    atomicAdd(&cnt[ss_sub(key, hs, sl)], 1u);
  }
  lds_barrier();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    bool big = false;
    for (int k = 0; k < nsub; ++k) {
      cur[k] = run;
      sp.subst[b * 65ull + k] = run;
      run += cnt[k];
      big = big || cnt[k] > (uint32_t)kBrCap;
    }
    sp.subst[b * 65ull + nsub] = run;
    if (big) atomicOr((unsigned long long *)&t.meta[M_BRBIG], 1ull);
  }
  lds_barrier();
  for (uint64_t q = threadIdx.x; q < m; q += kBrSubNT) {
    const uint64_t *src = sp.srec + (r0 + q) * W;
    uint64_t v[W];
#pragma unroll
    for (int k = 0; k < W; ++k) v[k] = src[k];
    const uint32_t at = atomicAdd(&cur[ss_sub((uint32_t)v[0], hs, sl)], 1u);
    uint64_t *dst = sp.scopy + (r0 + at) * W;
#pragma unroll
    for (int k = 0; k < W; ++k) dst[k] = v[k];
  }
}

void launch_br_subhist(hipStream_t s, const SessTable &t, int np_log2, int bshift, int words, const SessPart &sp) {
  const dim3 g(1u << np_log2), th(kBrSubNT);
  switch (words) {
    case 3: hipLaunchKernelGGL(k_br_subhist<3>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 4: hipLaunchKernelGGL(k_br_subhist<4>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 5: hipLaunchKernelGGL(k_br_subhist<5>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 6: hipLaunchKernelGGL(k_br_subhist<6>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 7: hipLaunchKernelGGL(k_br_subhist<7>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 8: hipLaunchKernelGGL(k_br_subhist<8>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 9: hipLaunchKernelGGL(k_br_subhist<9>, g, th, 0, s, t, np_log2, bshift, sp); break;
    case 10: hipLaunchKernelGGL(k_br_subhist<10>, g, th, 0, s, t, np_log2, bshift, sp); break;
    default: hipLaunchKernelGGL(k_br_subhist<11>, g, th, 0, s, t, np_log2, bshift, sp); break;
  }
}

// contribution of a bucket-replay record (present bits 32..39, literal-form
// bits 40..47 of word 0) to every slot, LAST / form slots included
template <int MS>
__device__ inline void br_elem(const Program &prog, const uint64_t *rec, uint64_t seq1, int64_t (&e)[MS]) {
  const uint64_t vb = rec[0] >> 32;
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    e[s] = 0;
    if (s >= prog.n_slots) continue;
    const int op = prog.slot_op[s], c = prog.slot_col[s];
    if (op == S_CNT_ALL) {
      e[s] = 1;
      continue;
    }
    const bool present = ((vb >> c) & 1ull) != 0, dec = ((vb >> (8 + c)) & 1ull) != 0;
    const int64_t x = (int64_t)rec[2 + c];
    if (op == S_LAST_VAL) {
      e[s] = present ? x : 0;
      continue;
    }
    if (!present) {
      e[s] = slot_identity_dev(op);
      continue;
    }
    switch (op) {
      case S_CNT: e[s] = 1; break;
      case S_MIN_F:
      case S_MAX_F: e[s] = (int64_t)f64_ord(__builtin_bit_cast(double, x)); break;
      case S_LAST_SEQ: e[s] = (int64_t)seq1; break;
      case S_CNT_DEC: e[s] = dec ? 1 : 0; break;
      case S_TIE_MIN:
      case S_TIE_MAX:
      case S_LAST_FORM: e[s] = (int64_t)((seq1 << 1) | (dec ? 0u : 1u)); break;
      default: e[s] = x; break;
    }
  }
}

// LDS of k_br_replay. CW: words of each record cached here (its word 0, ts
// and columns, for records of <= 5 words), so the replay reads no record
// from HBM; wider records are read from the bucket (L2).
template <int W>
struct BrLds {
  static constexpr int CW = W <= 5 ? W - 1 : 0;
  uint32_t tkey[kBrTab];  // key table
  uint32_t tcnt[kBrTab];  // records per key; after the grouping: the key's group
  uint32_t ridx[kBrCap];  // record -> its arrival index
  uint16_t rtab[kBrCap];  // record -> its key's table entry, then its group
  uint16_t seg[kBrCap];   // records placed by group
  uint16_t ord[kBrCap];   // records placed by group, in arrival order within a group
  uint32_t gkey[kBrCap];
  uint16_t gstart[kBrCap];
  uint16_t gcnt[kBrCap];
  uint32_t gcur[kBrCap];
  uint64_t rw[CW ? kBrCap * CW : 1];
  uint64_t wsum64[kBrNT / 64];
  uint32_t ngrp;
  uint64_t abase, rbase;
  uint32_t fail;
};

template <int MS, int W>
__global__ __launch_bounds__(kBrNT) __attribute__((amdgpu_waves_per_eu(HSG_BR_WPE))) void k_br_replay(Batch b, SessParams p, SessTable t, Program prog, int np_log2,
                                                     int bshift, SessPart sp, const int64_t *seq, OutCols out,
                                                     uint64_t out_base, DevScalars *sc) {
  __shared__ BrLds<W> L;
  // every barrier here orders LDS only (lds_barrier): nothing in the
  // workgroup reads back the rows, entries or states its threads store, so
  // no barrier waits for those scattered stores (a __syncthreads would: its
  // release waits for the wave's outstanding stores, ~10 us per sub-bucket)
  constexpr int CW = BrLds<W>::CW;
  if (t.meta[M_BRBIG] || t.meta[M_FAIL]) return;  // uniform: the other replay runs / the arena is refilled first
  const uint32_t bk = blockIdx.x;
  const uint64_t r0 = sp.bstart[bk], m = sp.bstart[bk + 1] - r0;
  const int sl = br_sub_log2(m), nsub = 1 << sl;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t fs = 2 + (uint32_t)prog.n_slots;
  const uint32_t region = arena_region(bk);
  const bool mir = prog.n_slots <= kSessMirrorSlots;
  int64_t live_delta = 0;
  uint64_t inserted = 0;
  uint64_t ph[5] = {0, 0, 0, 0, 0}, pc = 0, nsp = 0;  // phase clocks (PHASES=1 builds), thread 0
  uint64_t n_slow = 0, n_deep = 0, n_grp = 0;  // PHASES=1: records off the mirror (past the tail), groups
  auto tick = [&](int k) {
    if constexpr (kPhaseClocks) {
      const uint64_t c = phase_clock();
      if (k >= 0) ph[k] += c - pc;
      pc = c;
    }
  };
  // block-wide exclusive scan of one value per thread (every thread calls)
  auto block_excl = [&](uint64_t v, uint64_t &total) -> uint64_t {
    const uint64_t incl = wave_incl_sum(v);
    lds_barrier();
    if (lane == 63) L.wsum64[w] = incl;
    lds_barrier();
    uint64_t pre = incl - v;
    total = 0;
    for (int k = 0; k < kBrNT / 64; ++k) {
      pre += k < w ? L.wsum64[k] : 0;
      total += L.wsum64[k];
    }
    return pre;
  };
  for (int sub = (int)sp.progress[bk]; sub < nsub; ++sub) {
    const uint32_t s0 = sp.subst[bk * 65ull + sub], cnt = sp.subst[bk * 65ull + sub + 1] - s0;
    tick(-1);
    ++nsp;
    // 1. group the sub-bucket's records by key (LDS hash table)
    for (int i = threadIdx.x; i < kBrTab; i += kBrNT) {
      L.tkey[i] = kSessEmptyKey;
      L.tcnt[i] = 0;
    }
    if (threadIdx.x == 0) L.fail = 0;
    lds_barrier();
    for (uint32_t q = threadIdx.x; q < cnt; q += kBrNT) {
      const uint32_t pos = (uint32_t)(r0 + s0 + q);
      const uint64_t *rec = sp.scopy + (uint64_t)pos * W;
      const uint32_t key = (uint32_t)rec[0];
      L.ridx[q] = (uint32_t)rec[W - 1];
#pragma unroll
      for (int k = 0; k < CW; ++k) L.rw[q * CW + k] = rec[k];
      uint32_t h = (uint32_t)key_hash(key) & (kBrTab - 1);
      for (;;) {
        const uint32_t old = atomicCAS(&L.tkey[h], kSessEmptyKey, key);
        if (old == kSessEmptyKey || old == key) break;
        h = (h + 1) & (kBrTab - 1);
      }
      atomicAdd(&L.tcnt[h], 1u);
      L.rtab[q] = (uint16_t)h;
    }
    lds_barrier();
    tick(0);
    // 2. groups: the keys in table order, their segments (block scan over the table)
    {
      constexpr int PER = kBrTab / kBrNT;
      uint32_t c[PER], nz = 0, tot = 0;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        c[k] = L.tcnt[threadIdx.x * PER + k];
        nz += c[k] ? 1u : 0u;
        tot += c[k];
      }
      uint64_t all;
      const uint64_t pre = block_excl(((uint64_t)nz << 32) | tot, all);
      uint32_t g = (uint32_t)(pre >> 32), at = (uint32_t)pre;
#pragma unroll
      for (int k = 0; k < PER; ++k) {
        const int slot = threadIdx.x * PER + k;
        if (!c[k]) continue;
        L.gkey[g] = L.tkey[slot];
        L.gstart[g] = (uint16_t)at;
        L.gcnt[g] = (uint16_t)c[k];
        L.gcur[g] = 0;
        L.tcnt[slot] = g;
        ++g;
        at += c[k];
      }
      if (threadIdx.x == 0) L.ngrp = (uint32_t)(all >> 32);
    }
    lds_barrier();
    tick(1);
    const uint32_t ngrp = L.ngrp;
    // 3. records into their group's segment, then ranked by arrival index
    for (uint32_t q = threadIdx.x; q < cnt; q += kBrNT) {
      const uint32_t g = L.tcnt[L.rtab[q]];
      L.seg[L.gstart[g] + atomicAdd(&L.gcur[g], 1u)] = (uint16_t)q;
      L.rtab[q] = (uint16_t)g;
    }
    lds_barrier();
    for (uint32_t x = threadIdx.x; x < cnt; x += kBrNT) {
      const uint32_t q = L.seg[x], g = L.rtab[q], st = L.gstart[g], c = L.gcnt[g], me = L.ridx[q];
      uint32_t rank = 0;
      for (uint32_t y = st; y < st + c; ++y) rank += L.ridx[L.seg[y]] < me ? 1u : 0u;
      L.ord[st + rank] = (uint16_t)q;
    }
    // 4. every group's key-table entry (rounds of kBrNT groups, one per
    //    thread), the fresh list rows it needs; one arena reservation for the
    //    sub-bucket before anything is written (L.tkey[g]: the entry's slot,
    //    L.gcur[g]: the group's fresh rows' offset in the reservation)
    SessKey E;  // the entry of this thread's group in the last round (one round: all of them)
    uint64_t need = 0;
    for (uint32_t g0 = 0; g0 < ngrp; g0 += kBrNT) {
      const uint32_t g = g0 + threadIdx.x;
      uint32_t nc = 0;
      if (g < ngrp) {
        bool ins = false;
        const int64_t ks = ss_find_entry(t, L.gkey[g], E, ins);
        inserted += ins ? 1u : 0u;
        if (ks < 0) {
          atomicOr(&sc->err, ERR_OOM);
        } else {
          const uint64_t want = (uint64_t)E.len + L.gcnt[g];
          nc = want > E.cap ? ss_grow_cap(want) : 0u;
        }
        L.tkey[g] = ks < 0 ? ~0u : (uint32_t)ks;
      }
      uint64_t tot;
      const uint64_t pre = block_excl(nc, tot);
      if (g < ngrp) L.gcur[g] = (uint32_t)(need + pre);
      need += tot;
    }
    if (threadIdx.x == 0) {
      uint64_t base = 0;
      if (need && !arena_take(t, region, need, base)) {
        // no room: nothing of this sub-bucket is written; it (and the rest of
        // the bucket) runs again after the host compacts / grows the arena
        // (sp.progress resumes it here)
        L.fail = 1;
        t.meta[M_FAIL] = 1;
        atomicAdd((unsigned long long *)&t.meta[M_RNEED + region], (unsigned long long)need);
      }
      L.abase = base;
    }
    lds_barrier();
    tick(2);
    if (L.fail) break;
    // 5. replay: one thread per key, its records in arrival order against its list
    for (uint32_t g0 = 0; g0 < ngrp; g0 += kBrNT) {
    const uint32_t g = g0 + threadIdx.x;
    uint64_t rl_src = 0, rl_dst = 0, rl_n = 0;  // this thread's moved list, if any
    uint32_t emitted = 0;                         // sessions of the key this batch stamped
    uint64_t klen = 0, koff = 0;
    uint32_t kkey = 0;
    if (g < ngrp && L.tkey[g] != ~0u) {
      n_grp += 1;
      const uint32_t ks = L.tkey[g];
      if (ngrp > kBrNT) E = ss_load_entry(&t.kt[ks]);
      uint64_t off = E.off, len = E.len;
      uint32_t lcap = E.cap;
      const uint64_t want = len + L.gcnt[g];
      // a list that outgrows its rows moves to fresh rows; its rows are not
      // copied by this thread (a row-by-row copy holds the whole wave, and
      // ~1 key in 8 per C4 batch moves) unless the slow path needs to read
      // them: rows [0, pfx) -- those no record rewrote -- are listed for
      // k_ss_reloc_copy after the kernel
      const uint64_t old_off = off;
      uint64_t pfx = 0;
      bool pending = false;
      if (want > lcap) {
        off = L.abase + L.gcur[g];
        lcap = ss_grow_cap(want);
        pfx = len;
        pending = len > 0;
      }
      // the list's last session in registers (the entry's mirror, <= 2 slots):
      // a record at or after its start can reach no other session (the one
      // before ends more than gap before it), so it either merges into the
      // last session or follows it, without reading the list
      bool lv = mir && E.mvalid && len > 0;
      bool lst = false;  // the list's last session carries this batch's stamp (no session of the key
                         // does before its records: one thread replays a key once per batch)
      int64_t ls = E.ms, le = E.me, la[MS];
#pragma unroll
      for (int s = 0; s < MS; ++s) la[s] = s < kSessMirrorSlots ? E.ma[s] : 0;
      const uint32_t st = L.gstart[g], c = L.gcnt[g];
      for (uint32_t x = st; x < st + c; ++x) {
        const uint32_t q = L.ord[x];
        const uint64_t *rec = CW ? &L.rw[q * CW] : sp.scopy + (r0 + s0 + q) * W;
        const uint32_t i = L.ridx[q];
        const int64_t ts = (int64_t)rec[1];
        const uint64_t seq1 = (seq ? (uint64_t)seq[i] : p.rec_base + i) + 1;
        const int64_t lo = (int64_t)((uint64_t)ts - (uint64_t)p.gap);
        const int64_t hi = (int64_t)((uint64_t)ts + (uint64_t)p.gap);
        // aggF initialValue r, then mergeF acc cur over the overlapped sessions
        int64_t acc[MS], ev[MS];
        identity_row<MS>(prog, acc);
        br_elem<MS>(prog, rec, seq1, ev);
        combine_row<MS>(prog, acc, ev);
        int64_t ss = ts, se = ts;
        if (lv && ts >= ls) {
          if (le >= lo) {  // overlaps the last session: merged into it
            merge_row<MS>(prog, acc, la);
            ss = ls;
            se = le > ts ? le : ts;
            ss_store<MS>(t, off + len - 1, ss, se, p.batch_id, acc);
            pfx = len - 1 < pfx ? len - 1 : pfx;
            emitted += lst ? 0u : 1u;
          } else {  // a new last session
            ss_store<MS>(t, off + len, ss, se, p.batch_id, acc);
            len += 1;
            live_delta += 1;
            emitted += 1;
          }
          lst = true;
          ls = ss;
          le = se;
#pragma unroll
          for (int s = 0; s < MS; ++s) la[s] = acc[s];
        } else {
          n_slow += 1;
          // a record before the last session: the list's tail rows (KT of
          // them) in one round of loads; when the row before the tail ends
          // before lo, every session the record reaches is among them, and the
          // merge, the shift and the mirror run from registers (no dependent
          // search, no load-then-store copies)
          constexpr int KT = MS <= HSG_BR_TAIL_MS ? 4 : 0;
          constexpr int RW = 3 + (MS <= 4 ? MS : 0);
          bool done = false;
          if constexpr (KT > 0) {
            const uint64_t tb = len > (uint64_t)KT ? len - KT : 0;
            uint64_t R[KT > 0 ? KT : 1][RW];
#pragma unroll
            for (int k = 0; k < KT; ++k) {
              const uint64_t idx = tb + k;
              const uint64_t *row = ss_row(t, (pending && idx < pfx ? old_off : off) + idx);
#pragma unroll
              for (int w2 = 0; w2 < RW; ++w2) R[k][w2] = idx < len && w2 < 3 + (int)t.ns ? row[w2] : 0;
            }
            if (tb == 0 || (int64_t)R[0][1] < lo) {
              done = true;
              // i0: first row ending at or after lo; i1: past the rows starting by hi
              uint64_t i0 = len, i1;
#pragma unroll
              for (int k = KT - 1; k >= 0; --k)
                if (tb + k < len && (int64_t)R[k][1] >= lo) i0 = tb + k;
              uint64_t mc = 0;
#pragma unroll
              for (int k = 0; k < KT; ++k) mc += tb + k >= i0 && tb + k < len && (int64_t)R[k][0] <= hi ? 1u : 0u;
              i1 = i0 + mc;
              uint32_t sm = 0;
              for (uint64_t j = i0; j < i1; ++j) {  // the merged rows, in end order
                uint64_t cw[RW];
#pragma unroll
                for (int w2 = 0; w2 < RW; ++w2) {
                  cw[w2] = 0;
#pragma unroll
                  for (int k = 0; k < KT; ++k) cw[w2] = tb + k == j ? R[k][w2] : cw[w2];
                }
                ss = (int64_t)cw[0] < ss ? (int64_t)cw[0] : ss;
                se = (int64_t)cw[1] > se ? (int64_t)cw[1] : se;
                sm += (uint32_t)cw[2] == p.batch_id ? 1u : 0u;
                int64_t cur[MS];
#pragma unroll
                for (int s2 = 0; s2 < MS; ++s2) cur[s2] = s2 + 3 < RW ? (int64_t)cw[3 + s2] : 0;
                merge_row<MS>(prog, acc, cur);
              }
              const bool to_end = i1 == len;
              // the rows after the merged stretch move (up one for an insert,
              // down mc - 1 for a merge of several), straight from registers;
              // in a moved list they are written at their new place even when
              // they keep their index (only rows before i0 are left to the copy)
              const int64_t sh = mc == 0 ? 1 : 1 - (int64_t)mc;
              if (sh != 0 || pending) {
#pragma unroll
                for (int k = 0; k < KT; ++k) {
                  const uint64_t idx = tb + k;
                  if (idx < i1 || idx >= len) continue;
                  uint64_t *d = ss_row(t, off + (uint64_t)((int64_t)idx + sh));
#pragma unroll
                  for (int w2 = 0; w2 < RW; ++w2)
                    if (w2 < 3 + (int)t.ns) d[w2] = R[k][w2];
                }
              }
              // the last session before the update, if the mirror did not hold it
              if (mir && !lv && len > 0 && !to_end) {
#pragma unroll
                for (int k = 0; k < KT; ++k)
                  if (tb + k == len - 1) {
                    ls = (int64_t)R[k][0];
                    le = (int64_t)R[k][1];
#pragma unroll
                    for (int s2 = 0; s2 < MS; ++s2) la[s2] = s2 + 3 < RW ? (int64_t)R[k][3 + s2] : 0;
                  }
              }
              len = (uint64_t)((int64_t)len + sh);
              live_delta += 1 - (int64_t)mc;
              ss_store<MS>(t, off + i0, ss, se, p.batch_id, acc);
              pfx = i0 < pfx ? i0 : pfx;  // a moved list: rows from i0 on are written at their new place
              emitted += 1u - sm;
              if (to_end) lst = true;
              if (mir) {
                if (i0 + 1 == len) {
                  ls = ss;
                  le = se;
#pragma unroll
                  for (int s2 = 0; s2 < MS; ++s2) la[s2] = acc[s2];
                }
                lv = true;
              }
            }
          }
          if (!done) {
          n_deep += 1;
          if (pending) {  // the list is read from here on: its moved rows first
            for (uint64_t k = 0; k < pfx; ++k) ss_copy(t, off + k, t, old_off + k);
            pending = false;
          }
          // first session with end >= lo (ends ascend: sessions are disjoint)
          uint64_t a = 0, z = len;
          while (a < z) {
            const uint64_t mid = (a + z) >> 1;
            if ((int64_t)ss_row(t, off + mid)[1] < lo) a = mid + 1;
            else z = mid;
          }
          const uint64_t i0 = a;
          uint64_t i1 = i0;
          while (i1 < len && (int64_t)ss_row(t, off + i1)[0] <= hi) ++i1;
          uint32_t sm = 0;  // merged sessions already stamped by this batch
          for (uint64_t k = i0; k < i1; ++k) {
            const uint64_t *row = ss_row(t, off + k);
            const int64_t cs = (int64_t)row[0], ce = (int64_t)row[1];
            ss = cs < ss ? cs : ss;
            se = ce > se ? ce : se;
            sm += (uint32_t)row[2] == p.batch_id ? 1u : 0u;
            int64_t cur[MS];
            ss_load<MS>(t, off + k, cur);
            merge_row<MS>(prog, acc, cur);
          }
          const uint64_t mc = i1 - i0;
          const bool to_end = i1 == len;  // the merged stretch reaches the last session
          if (mc == 0) {
            for (uint64_t k = len; k > i0; --k) ss_copy(t, off + k, t, off + k - 1);
            len += 1;
          } else if (mc > 1) {
            for (uint64_t k = i1; k < len; ++k) ss_copy(t, off + k - (mc - 1), t, off + k);
            len -= mc - 1;
          }
          live_delta += 1 - (int64_t)mc;
          ss_store<MS>(t, off + i0, ss, se, p.batch_id, acc);
          emitted += 1u - sm;
          if (to_end) lst = true;
          if (mir) {  // the last session again
            if (i0 + 1 == len) {
              ls = ss;
              le = se;
#pragma unroll
              for (int s = 0; s < MS; ++s) la[s] = acc[s];
            } else {
              const uint64_t *row = ss_row(t, off + len - 1);
              ls = (int64_t)row[0];
              le = (int64_t)row[1];
              ss_load<MS>(t, off + len - 1, la);
            }
            lv = true;
          }
          }
        }
        int64_t *f = sp.fin + (uint64_t)i * fs;
        f[0] = ss;
        f[1] = se;
#pragma unroll
        for (int s = 0; s < MS; ++s)
          if (s < prog.n_slots) f[2 + s] = acc[s];
      }
      E.off = off;
      E.len = (uint32_t)len;
      E.cap = lcap;
      E.mvalid = lv && len > 0 ? 1u : 0u;
      E.ms = ls;
      E.me = le;
      E.ma[0] = MS > 0 ? la[0] : 0;
      E.ma[1] = MS > 1 ? la[1] : 0;
      ss_store_entry(&t.kt[ks], E);
      klen = len;
      koff = off;
      kkey = E.key;
      if (pending && pfx) {
        rl_src = old_off;
        rl_dst = off;
        rl_n = pfx;
      }
    }
    // the moved lists' prefixes to copy: one counter update per round
    {
      uint64_t rtot;
      const uint64_t rpre = block_excl(rl_n ? 1u : 0u, rtot);
      tick(3);
      if (threadIdx.x == 0) L.rbase = rtot ? atomicAdd((unsigned long long *)&t.meta[M_RELOC], rtot) : 0;
      lds_barrier();
      if (rl_n) {
        uint64_t *r = sp.reloc + 3 * (L.rbase + rpre);
        r[0] = rl_src;
        r[1] = rl_dst;
        r[2] = rl_n;
      }
      lds_barrier();
    }
    // per-batch changelog (LAST / literal forms, or every op with
    // HSG_SS_REPLAY_ALL): the key's sessions this batch stamped, found from
    // the end of its list (near-sorted arrivals stamp only its last ones;
    // rows the slow path shifted were copied first, so every row read here
    // is the kernel's or was in place)
    if (p.emit_mode == HSG_EMIT_PER_BATCH) {
      uint64_t tot;
      const uint64_t pre = block_excl(emitted, tot);
      if (threadIdx.x == 0) {
        L.rbase = tot ? atomicAdd((unsigned long long *)&sc->out_rows, (unsigned long long)tot) : 0;
        if (tot) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tot);
      }
      lds_barrier();
      uint64_t o = out_base + L.rbase + pre;
      uint32_t left = emitted;
      for (uint64_t k = klen; k > 0 && left; --k) {
        const uint64_t *row = ss_row(t, koff + k - 1);
        if ((uint32_t)row[2] != p.batch_id) continue;
        out.key[o] = kkey;
        out.ws[o] = (int64_t)row[0];
        out.we[o] = (int64_t)row[1];
        out.src[o] = -1;
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, (const int64_t *)row + 3);
        if (out.form) out.form[o] = out_form(prog, (const int64_t *)row + 3);
        ++o;
        --left;
      }
      lds_barrier();
    } else {
      // the resident sessions this batch read and wrote (U of SURVEY.md 8d's
      // 2*U*R), counted as in per-batch mode: one atomic per wave
      const uint64_t e = wave_sum_u64(emitted);
      if ((threadIdx.x & 63) == 0 && e) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)e);
    }
    }
    lds_barrier();
    tick(4);
    if (threadIdx.x == 0) sp.progress[bk] = (uint32_t)(sub + 1);
  }
  if constexpr (kPhaseClocks) {
    if (threadIdx.x == 0) {
      for (int k = 0; k < 5; ++k) atomicAdd((unsigned long long *)&sc->scratch[24 + k], (unsigned long long)ph[k]);
      atomicAdd((unsigned long long *)&sc->scratch[30], (unsigned long long)nsp);
      sc->scratch[23] = 1;
    }
    const uint64_t a = wave_sum_u64(n_slow | n_deep << 32), z = wave_sum_u64(n_grp);
    if (lane == 0) {
      atomicAdd((unsigned long long *)&sc->scratch[43], (unsigned long long)a);
      atomicAdd((unsigned long long *)&sc->scratch[44], (unsigned long long)z);
    }
  }
  const uint64_t ld = wave_sum_u64((uint64_t)live_delta);
  if (lane == 0 && ld) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)ld);
  const uint64_t ins = wave_sum_u64(inserted);
  if (lane == 0 && ins) atomicAdd((unsigned long long *)&t.meta[M_KEYS], (unsigned long long)ins);
}

template <int MS>
static void br_replay_launch(hipStream_t s, int W, dim3 g, const Batch &b, const SessParams &p, const SessTable &t,
                             const Program &prog, int np_log2, int bshift, const SessPart &sp, const int64_t *seq,
                             OutCols out, uint64_t out_base, DevScalars *sc) {
  const dim3 th(kBrNT);
#define BR_W(WW)                                                                                              \
  case WW:                                                                                                    \
    hipLaunchKernelGGL((k_br_replay<MS, WW>), g, th, 0, s, b, p, t, prog, np_log2, bshift, sp, seq, out, out_base, \
                       sc);                                                                                   \
    break;
  switch (W) {
    BR_W(3) BR_W(4) BR_W(5) BR_W(6) BR_W(7) BR_W(8) BR_W(9) BR_W(10)
    default: hipLaunchKernelGGL((k_br_replay<MS, 11>), g, th, 0, s, b, p, t, prog, np_log2, bshift, sp, seq, out,
                                out_base, sc);
  }
#undef BR_W
}

void launch_br_replay(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                      int np_log2, int bshift, int words, const SessPart &sp, const int64_t *seq, OutCols out,
                      uint64_t out_base, DevScalars *sc) {
  const dim3 g(1u << np_log2);
  if (prog.n_slots <= 2) br_replay_launch<2>(s, words, g, b, p, t, prog, np_log2, bshift, sp, seq, out, out_base, sc);
  else if (prog.n_slots <= 4) br_replay_launch<4>(s, words, g, b, p, t, prog, np_log2, bshift, sp, seq, out, out_base, sc);
  else if (prog.n_slots <= 8) br_replay_launch<8>(s, words, g, b, p, t, prog, np_log2, bshift, sp, seq, out, out_base, sc);
  else if (prog.n_slots <= 16) br_replay_launch<16>(s, words, g, b, p, t, prog, np_log2, bshift, sp, seq, out, out_base, sc);
  else br_replay_launch<kMaxSlots>(s, words, g, b, p, t, prog, np_log2, bshift, sp, seq, out, out_base, sc);
}

// The per-record changelog in arrival order: tile t's keyed records take rows
// from sp.toff[t] on (an in-tile exclusive scan of the keyed flags), each row
// from the state its record left in sp.fin. Coalesced columns.
__global__ __launch_bounds__(256) void k_br_emit(Batch b, SessParams p, Program prog, SessPart sp, const int64_t *seq,
                                                 OutCols out, uint64_t out_base) {
  __shared__ uint32_t sw[4];
  const uint64_t base = (uint64_t)blockIdx.x * kSsTile;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const uint32_t fs = 2 + (uint32_t)prog.n_slots;
  uint64_t o = out_base + sp.toff[blockIdx.x];
  for (int r = 0; r < kSsTile / 256; ++r) {
    const uint64_t i = base + (uint64_t)r * 256 + threadIdx.x;
    const uint32_t key = i < b.n ? b.key[i] : HSG_KEY_NONE;
    const bool keyed = key != HSG_KEY_NONE;
    const uint64_t m = __ballot(keyed);
    const uint32_t pre = (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
    if (lane == 0) sw[w] = (uint32_t)__popcll(m);
    lds_barrier();  // (LDS only: the rows stored are read by no one here)
    uint32_t wpre = 0, tot = 0;
    for (int k = 0; k < 4; ++k) {
      wpre += k < w ? sw[k] : 0u;
      tot += sw[k];
    }
    if (keyed) {
      const uint64_t q = o + wpre + pre;
      const int64_t *f = sp.fin + i * fs;
      out.key[q] = key;
      out.ws[q] = f[0];
      out.we[q] = f[1];
      out.src[q] = seq ? seq[i] : (int64_t)(p.rec_base + i);
      for (int j = 0; j < prog.n_out; ++j) out.agg[j][q] = out_value(prog, j, f + 2);
      if (out.form) out.form[q] = out_form(prog, f + 2);
    }
    o += tot;
    lds_barrier();
  }
}

void launch_br_emit(hipStream_t s, const Batch &b, const SessParams &p, const Program &prog, const SessPart &sp,
                    uint64_t tiles, const int64_t *seq, OutCols out, uint64_t out_base) {
  if (tiles) hipLaunchKernelGGL(k_br_emit, dim3((unsigned)tiles), dim3(256), 0, s, b, p, prog, sp, seq, out, out_base);
}

}  // namespace hsg
