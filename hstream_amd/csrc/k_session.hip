// gfx950 kernels for session windows (SessionWindowedStream.hs:74-118 over the
// session store of Store.hs:177-272). Layout and paths: hsg_session.h.
#include "hsg_dev.h"
#include "hsg_perrecord.h"
#include "hsg_session.h"
#include "hsg_sort.h"

namespace hsg {

// ---------------------------------------------------------------------------
// key table
// ---------------------------------------------------------------------------
__global__ void k_ss_reset(SessTable t) {
  const uint64_t cap = t.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    t.keys[s] = kSessEmptyKey;
    t.lists[s] = SessList{0, 0, 0};
    t.emark[s] = ~0ull;
  }
}

void launch_ss_reset(hipStream_t s, const SessTable &t) {
  hipLaunchKernelGGL(k_ss_reset, dim3(grid_for(t.kmask + 1, 256)), dim3(256), 0, s, t);
}

// find key's slot, inserting it if absent; -1 = table full. `inserted` is set
// when this call claimed the slot.
__device__ inline int64_t ss_find_or_insert(const SessTable &t, uint32_t key, bool &inserted) {
  uint64_t s = mix64(key) & t.kmask;
  inserted = false;
  for (uint64_t probe = 0; probe <= t.kmask; ++probe) {
    uint32_t cur = t.keys[s];
    if (cur == key) return (int64_t)s;
    if (cur == kSessEmptyKey) {
      uint32_t old = atomicCAS(&t.keys[s], kSessEmptyKey, key);
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

__global__ void k_ss_rehash(SessTable from, SessTable to) {
  const uint64_t cap = from.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t key = from.keys[s];
    if (key == kSessEmptyKey) continue;
    bool ins;
    const int64_t d = ss_find_or_insert(to, key, ins);
    if (d >= 0) to.lists[d] = from.lists[s];  // `to` is at most half full: d >= 0
  }
}

void launch_ss_rehash(hipStream_t s, const SessTable &from, const SessTable &to) {
  launch_ss_reset(s, to);
  hipLaunchKernelGGL(k_ss_rehash, dim3(grid_for(from.kmask + 1, 256)), dim3(256), 0, s, from, to);
}

// ---------------------------------------------------------------------------
// arena: session copies and compaction
// ---------------------------------------------------------------------------
__device__ inline void ss_copy(const SessTable &dt, uint64_t dst, const SessTable &st, uint64_t src, int ns) {
  dt.a_start[dst] = st.a_start[src];
  dt.a_end[dst] = st.a_end[src];
  dt.a_stamp[dst] = st.a_stamp[src];
  for (int s = 0; s < ns; ++s) dt.a_aggs[dst * ns + s] = st.a_aggs[src * ns + s];
}

__device__ inline uint32_t ss_grow_cap(uint64_t need) {
  uint32_t c = 4;
  while (c < need) c <<= 1;
  return c;
}

__global__ void k_ss_ccount(SessTable t, uint32_t *newcap) {
  const uint64_t cap = t.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t len = t.keys[s] == kSessEmptyKey ? 0u : t.lists[s].len;
    newcap[s] = len ? ss_grow_cap((uint64_t)len + 1) : 0u;
  }
}

__global__ void k_ss_ccopy(SessTable from, SessTable to, int ns, const uint32_t *newcap, const uint64_t *newoff) {
  const uint64_t cap = from.kmask + 1;
  for (uint64_t s = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; s < cap; s += (uint64_t)gridDim.x * blockDim.x) {
    if (from.keys[s] == kSessEmptyKey) continue;
    const SessList L = from.lists[s];
    const uint64_t o = newoff[s];
    for (uint32_t k = 0; k < L.len; ++k) ss_copy(to, o + k, from, L.off + k, ns);
    to.lists[s] = SessList{o, L.len, newcap[s]};
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

// new list capacities and their offsets; the total (the compacted arena's
// top) -> *total (device)
void launch_ss_compact_plan(hipStream_t s, const SessTable &t, void *scratch, uint64_t *total) {
  const uint64_t kcap = t.kmask + 1;
  uint32_t *newcap;
  uint64_t *newoff, *partial;
  compact_views(scratch, kcap, newcap, newoff, partial);
  hipLaunchKernelGGL(k_ss_ccount, dim3(grid_for(kcap, 256)), dim3(256), 0, s, t, newcap);
  scan_excl_u32(s, newcap, newoff, kcap, partial, total);
}

// every list copied into `to`'s arena (to shares the key table with from;
// lists are rewritten in place)
void launch_ss_compact_copy(hipStream_t s, const SessTable &from, const SessTable &to, int n_slots, void *scratch) {
  const uint64_t kcap = from.kmask + 1;
  uint32_t *newcap;
  uint64_t *newoff, *partial;
  compact_views(scratch, kcap, newcap, newoff, partial);
  hipLaunchKernelGGL(k_ss_ccopy, dim3(grid_for(kcap, 256)), dim3(256), 0, s, from, to, n_slots, newcap, newoff);
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
    uint32_t sl = cap;
    uint32_t key = HSG_KEY_NONE;
    if (i < b.n) {
      key = b.key[i];
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

// arena sessions the replay's list growth needs, then the all-or-nothing
// decision (one workgroup, after every need has been added)
__global__ __launch_bounds__(256) void k_ss_replay_need(SessTable t, const uint32_t *slot, const uint32_t *runs,
                                                        uint64_t R) {
  uint64_t need = 0;
  for (uint64_t r = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; r < R; r += (uint64_t)gridDim.x * blockDim.x) {
    const SessList L = t.lists[slot[runs[r]]];
    const uint64_t want = (uint64_t)L.len + (runs[r + 1] - runs[r]);
    if (want > L.cap) need += ss_grow_cap(want);
  }
  need = wave_sum_u64(need);
  if ((threadIdx.x & 63) == 0 && need) atomicAdd((unsigned long long *)&t.meta[M_NEED], (unsigned long long)need);
}
__global__ void k_ss_replay_check(SessTable t) {
  if (t.meta[M_TOP] + t.meta[M_NEED] > t.arena_cap) t.meta[M_FAIL] = 1;
}

void launch_ss_replay_need(hipStream_t s, const SessTable &t, const uint32_t *slot, const uint32_t *runs, uint64_t R) {
  if (R) {
    uint64_t blocks = (R + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(k_ss_replay_need, dim3((unsigned)blocks), dim3(256), 0, s, t, slot, runs, R);
  }
  hipLaunchKernelGGL(k_ss_replay_check, dim3(1), dim3(1), 0, s, t);
}

template <int MS>
__device__ inline void ss_load(const SessTable &t, int ns, uint64_t idx, int64_t (&a)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) a[s] = s < ns ? t.a_aggs[idx * ns + s] : 0;
}
template <int MS>
__device__ inline void ss_store(const SessTable &t, int ns, uint64_t idx, const int64_t (&a)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s < ns) t.a_aggs[idx * ns + s] = a[s];
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
  uint32_t sl = 0, key = 0;
  SessList L = {0, 0, 0};
  int64_t live_delta = 0;
  if (active) {
    q0 = runs[r];
    q1 = runs[r + 1];
    sl = slot[q0];
    key = t.keys[sl];
    L = t.lists[sl];
  }
  // grow the key's list once for the whole run (each record adds <= 1
  // session); one arena bump per wave, within what k_ss_replay_need reserved
  const uint64_t want = (uint64_t)L.len + (q1 - q0);
  const uint64_t new_cap = (active && want > L.cap) ? ss_grow_cap(want) : 0;
  const uint64_t incl = wave_incl_sum(new_cap);
  const uint64_t wtot = __shfl(incl, 63, 64);
  uint64_t wbase = 0;
  if (lane == 63 && wtot) wbase = atomicAdd((unsigned long long *)&t.meta[M_TOP], (unsigned long long)wtot);
  wbase = __shfl(wbase, 63, 64);
  uint64_t off = L.off, len = L.len;
  if (new_cap) {
    const uint64_t noff = wbase + incl - new_cap;
    for (uint64_t k = 0; k < len; ++k) ss_copy(t, noff + k, t, off + k, ns);
    off = noff;
    L.cap = (uint32_t)new_cap;
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
        const int64_t cs = t.a_start[off + k], ce = t.a_end[off + k];
        s0 = cs < s0 ? cs : s0;
        e0 = ce > e0 ? ce : e0;
        int64_t cur[MS];
        ss_load<MS>(t, ns, off + k, cur);
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
        // insert at i0: near-sorted arrivals append (i0 == len), nothing moves
        for (uint64_t k = len; k > i0; --k) ss_copy(t, off + k, t, off + k - 1, ns);
        len += 1;
      } else if (c > 1) {
        for (uint64_t k = i1; k < len; ++k) ss_copy(t, off + k - (c - 1), t, off + k, ns);
        len -= c - 1;
      }
      live_delta += 1 - (int64_t)c;
      t.a_start[off + i0] = s0;
      t.a_end[off + i0] = e0;
      t.a_stamp[off + i0] = p.batch_id;
      ss_store<MS>(t, ns, off + i0, acc);
      if (p.emit_mode == HSG_EMIT_PER_RECORD) {
        const uint64_t o = out_base + out_pos[i];
        out.key[o] = key;
        out.ws[o] = s0;
        out.we[o] = e0;
        out.src[o] = (int64_t)(seq1 - 1);
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value_reg<MS>(prog, j, acc);
      }
    }
    t.lists[sl] = SessList{off, (uint32_t)len, L.cap};
  }
  // per-batch changelog: the key's sessions stamped by this batch
  uint64_t mine = 0;
  if (active && p.emit_mode == HSG_EMIT_PER_BATCH)
    for (uint64_t k = 0; k < len; ++k) mine += t.a_stamp[off + k] == p.batch_id;
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

__device__ inline uint32_t ss_bucket(uint32_t key, int np_log2) {
  return np_log2 ? (uint32_t)(key_hash(key) >> (64 - np_log2)) : 0u;
}
__device__ inline uint64_t i64_img(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }

// per-tile bucket counts of the keyed records, tile-major; per-tile max ts
// image of EVERY record (stream time counts filtered records too)
__global__ __launch_bounds__(kSsPNT) void k_ss_phist(Batch b, int np_log2, SessPart sp) {
  __shared__ uint32_t cnt[1 << 11];
  __shared__ uint64_t smx[kSsPNT / 64];
  const int nb = 1 << np_log2;
  const uint64_t tile = blockIdx.x;
  for (int i = threadIdx.x; i < nb; i += kSsPNT) cnt[i] = 0;
  __syncthreads();
  const uint64_t base = tile * kSsTile;
  uint64_t mx = 0;
#pragma unroll
  for (int r = 0; r < kSsTile / kSsPNT; ++r) {
    const uint64_t i = base + (uint64_t)r * kSsPNT + threadIdx.x;
    if (i >= b.n) break;
    const uint32_t key = b.key[i];
    const uint64_t o = i64_img(b.ts[i]);
    mx = o > mx ? o : mx;
    if (key != HSG_KEY_NONE) atomicAdd(&cnt[ss_bucket(key, np_log2)], 1u);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(mx, o, 64);
    mx = x > mx ? x : mx;
  }
  if ((threadIdx.x & 63) == 0) smx[threadIdx.x >> 6] = mx;
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += kSsPNT) sp.hist[tile * (uint64_t)nb + i] = cnt[i];
  if (threadIdx.x == 0) {
    for (int k = 0; k < kSsPNT / 64; ++k) mx = smx[k] > mx ? smx[k] : mx;
    sp.tmax[tile] = mx;
  }
}

void launch_ss_phist(hipStream_t s, const Batch &b, int np_log2, uint64_t tiles, const SessPart &sp) {
  if (tiles) hipLaunchKernelGGL(k_ss_phist, dim3((unsigned)tiles), dim3(kSsPNT), 0, s, b, np_log2, sp);
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
template <int W>
__global__ __launch_bounds__(kSsPNT) void k_ss_pscatter(Batch b, int np_log2, int has_valid, SessPart sp) {
  __shared__ uint64_t stage[kSsSub * W];
  __shared__ uint32_t cursor[1 << 11];  // records of each bucket placed by earlier sub-tiles
  __shared__ uint32_t scnt[1 << 11];    // this sub-tile
  __shared__ uint32_t lstart[1 << 11];
  __shared__ uint16_t lbk[kSsSub];
  __shared__ uint32_t swave[kSsPNT / 64];
  constexpr int C = W - 2;
  constexpr int R = kSsSub / kSsPNT;
  const int nb = 1 << np_log2;
  const uint64_t tile = blockIdx.x;
  const uint32_t *orow = sp.offt + tile * (uint64_t)nb;
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
      pos[r] = key[r] != HSG_KEY_NONE ? atomicAdd(&scnt[ss_bucket(key[r], np_log2)], 1u) : ~0u;
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
      const uint32_t bk = ss_bucket(key[r], np_log2);
      const uint32_t q = lstart[bk] + pos[r];
      uint64_t vb = 0;
#pragma unroll
      for (int c = 0; c < C; ++c)
        if (!(has_valid && b.valid[c] && !b.valid[c][i])) vb |= 1ull << c;
      stage[q * W] = (uint64_t)key[r] | (vb << 32);
      stage[q * W + 1] = (uint64_t)b.ts[i];
#pragma unroll
      for (int c = 0; c < C; ++c) stage[q * W + 2 + c] = (uint64_t)b.col[c][i];
      lbk[q] = (uint16_t)bk;
    }
    __syncthreads();
    // write-out: staged record q -> offt[tile][bk] + cursor[bk] + (q - lstart[bk])
    for (uint32_t t = threadIdx.x; t < placed * W; t += kSsPNT) {
      const uint32_t q = t / W, w = t - q * W;
      const uint32_t bk = lbk[q];
      const uint64_t dest = (uint64_t)orow[bk] + cursor[bk] + (q - lstart[bk]);
      sp.rec[dest * W + w] = stage[t];
    }
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += kSsPNT) cursor[i] += scnt[i];
  }
}

void launch_ss_pscatter(hipStream_t s, const Batch &b, int np_log2, uint64_t tiles, int words, bool has_valid,
                        const SessPart &sp) {
  if (!tiles) return;
  const dim3 g((unsigned)tiles), th(kSsPNT);
  const int hv = has_valid ? 1 : 0;
  switch (words) {
    case 2: hipLaunchKernelGGL(k_ss_pscatter<2>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 3: hipLaunchKernelGGL(k_ss_pscatter<3>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 4: hipLaunchKernelGGL(k_ss_pscatter<4>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 5: hipLaunchKernelGGL(k_ss_pscatter<5>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 6: hipLaunchKernelGGL(k_ss_pscatter<6>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 7: hipLaunchKernelGGL(k_ss_pscatter<7>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 8: hipLaunchKernelGGL(k_ss_pscatter<8>, g, th, 0, s, b, np_log2, hv, sp); break;
    case 9: hipLaunchKernelGGL(k_ss_pscatter<9>, g, th, 0, s, b, np_log2, hv, sp); break;
    default: hipLaunchKernelGGL(k_ss_pscatter<10>, g, th, 0, s, b, np_log2, hv, sp); break;
  }
}

// ---------------------------------------------------------------------------
// merge path: per-bucket sort, gap-delimited runs, sweep-merge with the
// resident sessions
// ---------------------------------------------------------------------------
constexpr int kMgNT = 512;               // threads
constexpr int kMgCH = 2048;              // records per chunk
constexpr int kMgPer = kMgCH / kMgNT;    // records / runs / groups per thread
constexpr int kMgTail = 2;               // resident sessions a group may rewrite in place

// contribution of one partitioned record to the slots (identity when absent)
template <int MS>
__device__ inline void ss_rec_elem(const Program &prog, const uint64_t *rec, int64_t (&e)[MS]) {
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

template <int MS>
__device__ inline void acc_row(const Program &prog, int64_t (&a)[MS], const int64_t (&e)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s)
    if (s < prog.n_slots) a[s] = slot_combine(prog.slot_op[s], a[s], e[s]);
}

struct MgLds {
  uint32_t key[kMgCH];      // sort: key, ts image, record index in the chunk
  uint64_t tsu[kMgCH];
  uint16_t idx[kMgCH];
  int64_t rs[kMgCH];        // runs: start, end (inclusive), first sorted position
  int64_t re[kMgCH];
  uint16_t rbeg[kMgCH + 1];
  uint16_t gfirst[kMgCH + 1];  // groups (keys): first run
  uint32_t wsum[kMgNT / 64];
  uint64_t red[kMgNT / 64];
  uint32_t nrun, ngrp;
  uint64_t base;            // arena reservation of this chunk
  uint32_t tbase;           // touched-list entries of this chunk
  int fail;
};

// block exclusive scan of one u32 per thread (kMgNT threads)
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

// block exclusive scan of one u64 per thread; total -> *total
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

__device__ inline uint64_t mg_sum64(MgLds &L, uint64_t v) {
  v = wave_sum_u64(v);
  if ((threadIdx.x & 63) == 0) L.red[threadIdx.x >> 6] = v;
  __syncthreads();
  uint64_t t = 0;
  for (int k = 0; k < kMgNT / 64; ++k) t += L.red[k];
  __syncthreads();
  return t;
}

// One session of the sweep: start, end, aggregates, and whether a batch run
// is in it (-> changelog row, stamp)
template <int MS>
struct MgSess {
  int64_t s, e;
  int64_t a[MS];
  uint32_t stamp;  // a resident session's stamp (sessions without a run are one resident, moved unchanged)
  bool fresh;
};

// Sweep of one key: its resident sessions [i0, len) (the first kMgTail of them
// in registers when `tail_regs`) and its runs, in start order; items closer
// than gap merge (next.start - running end <= gap). With APPLY the merged
// sessions are written at dst + i0 + k (a session with a run in it stamped
// with the batch) and counted, else only counted.
template <int MS, int W, bool APPLY>
__device__ inline uint32_t mg_sweep(const MgLds &L, const Program &prog, const SessTable &t, int64_t gap,
                                    const uint64_t *recs, uint32_t r0, uint32_t r1, uint64_t off, uint64_t i0,
                                    uint64_t len, bool tail_regs, const MgSess<MS> (&tail)[kMgTail], uint64_t dst,
                                    uint32_t batch_id) {
  const int ns = prog.n_slots;
  uint64_t j = i0;   // next resident
  uint32_t r = r0;   // next run
  uint32_t k = 0;    // merged sessions so far
  MgSess<MS> cur;
  bool have = false;
  auto flush = [&]() {
    if (APPLY) {
      const uint64_t d = dst + i0 + k;
      t.a_start[d] = cur.s;
      t.a_end[d] = cur.e;
      t.a_stamp[d] = cur.fresh ? batch_id : cur.stamp;
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < ns) t.a_aggs[d * ns + s] = cur.a[s];
    }
    ++k;
  };
  for (;;) {
    // next item in start order: resident j or run r (ties: resident first)
    const bool has_res = j < len, has_run = r < r1;
    if (!has_res && !has_run) break;
    int64_t rs_ = 0, re_ = 0;
    if (has_res) {
      if (tail_regs && j - i0 < kMgTail) {
        rs_ = tail[j - i0].s;
        re_ = tail[j - i0].e;
      } else {
        rs_ = t.a_start[off + j];
        re_ = t.a_end[off + j];
      }
    }
    const bool take_res = has_res && (!has_run || rs_ <= L.rs[r]);
    MgSess<MS> it;
    if (take_res) {
      it.s = rs_;
      it.e = re_;
      it.fresh = false;
      it.stamp = 0;
      if (APPLY) {
        if (tail_regs && j - i0 < kMgTail) {
          it.stamp = tail[j - i0].stamp;
#pragma unroll
          for (int s = 0; s < MS; ++s) it.a[s] = tail[j - i0].a[s];
        } else {
          it.stamp = t.a_stamp[off + j];
#pragma unroll
          for (int s = 0; s < MS; ++s) it.a[s] = s < ns ? t.a_aggs[(off + j) * ns + s] : 0;
        }
      }
      ++j;
    } else {
      it.s = L.rs[r];
      it.e = L.re[r];
      it.fresh = true;
      it.stamp = batch_id;
      if (APPLY) {
        identity_row<MS>(prog, it.a);
        for (uint32_t q = L.rbeg[r]; q < L.rbeg[r + 1]; ++q) {
          int64_t e[MS];
          ss_rec_elem<MS>(prog, recs + (uint64_t)L.idx[q] * W, e);
          acc_row<MS>(prog, it.a, e);
        }
      }
      ++r;
    }
    if (have && (int64_t)((uint64_t)it.s - (uint64_t)cur.e) <= gap) {
      cur.e = it.e > cur.e ? it.e : cur.e;
      cur.fresh = cur.fresh || it.fresh;
      if (APPLY) acc_row<MS>(prog, cur.a, it.a);
    } else {
      if (have) flush();
      cur = it;
      have = true;
    }
  }
  if (have) flush();
  return k;
}

// first resident session with end >= lo: galloping back from the end (near-
// sorted arrivals touch the last session or none), then binary search
__device__ inline uint64_t mg_first_end_ge(const SessTable &t, uint64_t off, uint64_t len, int64_t lo) {
  uint64_t hi = len, step = 1;
  while (hi > 0) {
    const uint64_t probe = hi > step ? hi - step : 0;
    if (t.a_end[off + probe] < lo) {
      // answer in (probe, hi]
      uint64_t a = probe + 1, z = hi;
      while (a < z) {
        const uint64_t m = (a + z) >> 1;
        if (t.a_end[off + m] < lo) a = m + 1;
        else z = m;
      }
      return a;
    }
    hi = probe;
    step <<= 1;
  }
  return 0;
}

template <int MS, int W>
__global__ __launch_bounds__(kMgNT) void k_ss_merge(SessParams p, SessTable t, Program prog, int np_log2,
                                                    SessPart sp, DevScalars *sc) {
  __shared__ MgLds L;
  const uint32_t b = blockIdx.x;
  const uint64_t r0 = sp.bstart[b], r1 = sp.bstart[b + 1];
  const uint32_t nch = (uint32_t)((r1 - r0 + kMgCH - 1) / kMgCH);
  const int ns = prog.n_slots;
  int64_t live_delta = 0;
  uint64_t keys_new = 0;
  uint32_t err = 0;
  for (uint32_t c = sp.progress[b]; c < nch; ++c) {
    const uint64_t q0 = r0 + (uint64_t)c * kMgCH;
    const uint32_t m = (uint32_t)(r1 - q0 < kMgCH ? r1 - q0 : kMgCH);
    const uint64_t *recs = sp.rec + q0 * W;
    uint32_t N = 2;
    while (N < m) N <<= 1;
    // 1. load (key, ts) of the chunk; pad to N with +inf
    for (uint32_t i = threadIdx.x; i < N; i += kMgNT) {
      if (i < m) {
        L.key[i] = (uint32_t)recs[(uint64_t)i * W];
        L.tsu[i] = i64_img((int64_t)recs[(uint64_t)i * W + 1]);
      } else {
        L.key[i] = 0xFFFFFFFFu;
        L.tsu[i] = ~0ull;
      }
      L.idx[i] = (uint16_t)i;
    }
    __syncthreads();
    // 2. bitonic sort by (key, ts)
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
    // 3. gap-delimited runs: thread owns sorted positions [tid*kMgPer, +kMgPer)
    uint32_t heads = 0, hmask = 0;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t i = threadIdx.x * kMgPer + u;
      if (i >= m) break;
      bool h = i == 0 || L.key[i] != L.key[i - 1];
      if (!h) {
        const int64_t ta = (int64_t)(L.tsu[i - 1] ^ 0x8000000000000000ull);
        const int64_t tb = (int64_t)(L.tsu[i] ^ 0x8000000000000000ull);
        h = (int64_t)((uint64_t)tb - (uint64_t)ta) > p.gap;
      }
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
      L.rs[rpos] = (int64_t)(L.tsu[i] ^ 0x8000000000000000ull);
      if (rpos > 0) L.re[rpos - 1] = (int64_t)(L.tsu[i - 1] ^ 0x8000000000000000ull);
      ++rpos;
    }
    if (threadIdx.x == 0) {
      L.rbeg[nrun] = (uint16_t)m;
      L.re[nrun - 1] = (int64_t)(L.tsu[m - 1] ^ 0x8000000000000000ull);
    }
    __syncthreads();
    // 4. groups = runs of one key: thread owns runs [tid*kMgPer, +kMgPer)
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
    for (int u = 0; u < kMgPer; ++u) {
      if (!((gmask >> u) & 1u)) continue;
      L.gfirst[gpos++] = (uint16_t)(threadIdx.x * kMgPer + u);
    }
    if (threadIdx.x == 0) L.gfirst[ngrp] = (uint16_t)nrun;
    __syncthreads();
    // 5. plan: per group (thread owns groups tid, tid + NT, ...): slot, the
    // first resident session the runs can reach, merged count, relocation
    int64_t gslot[kMgPer];
    uint64_t gi0[kMgPer];
    uint32_t gM[kMgPer], gcap[kMgPer];
    SessList gl[kMgPer];
    uint64_t need = 0;
    uint32_t nt = 0;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t g = u * kMgNT + threadIdx.x;
      gslot[u] = -1;
      gcap[u] = 0;
      gM[u] = 0;
      gi0[u] = 0;
      gl[u] = SessList{0, 0, 0};
      if (g >= ngrp) continue;
      const uint32_t ra = L.gfirst[g], rb = L.gfirst[g + 1];
      const uint32_t key = L.key[L.rbeg[ra]];
      bool ins;
      const int64_t sl = ss_find_or_insert(t, key, ins);
      if (sl < 0) {
        err |= ERR_OOM;
        continue;
      }
      keys_new += ins ? 1 : 0;
      gslot[u] = sl;
      ++nt;
      const SessList Ls = ins ? SessList{0, 0, 0} : t.lists[sl];
      gl[u] = Ls;
      const int64_t lo = (int64_t)((uint64_t)L.rs[ra] - (uint64_t)p.gap);
      const uint64_t i0 = mg_first_end_ge(t, Ls.off, Ls.len, lo);
      gi0[u] = i0;
      MgSess<MS> dummy[kMgTail];
      const uint32_t M = mg_sweep<MS, W, false>(L, prog, t, p.gap, recs, ra, rb, Ls.off, i0, Ls.len, false, dummy, 0,
                                                0);
      gM[u] = M;
      // in place when the merged list fits and the rewritten tail fits the
      // registers, else a fresh list (prefix copied)
      if (i0 + M > Ls.cap || Ls.len - i0 > kMgTail) gcap[u] = ss_grow_cap(i0 + M + 1);
      need += gcap[u];
    }
    // 6. reserve the chunk's relocations in the arena (all or nothing)
    uint64_t tneed;
    const uint64_t npos = mg_scan64(L, need, tneed);
    uint32_t ttot;
    const uint32_t tpos = mg_scan(L, nt, ttot);
    if (threadIdx.x == 0) {
      L.fail = 0;
      L.base = 0;
      if (tneed) {
        unsigned long long *top = (unsigned long long *)&t.meta[M_TOP];
        unsigned long long old = __hip_atomic_load(top, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        for (;;) {
          if (old + tneed > t.arena_cap) {
            L.fail = 1;
            break;
          }
          const unsigned long long seen = atomicCAS(top, old, old + tneed);
          if (seen == old) break;
          old = seen;
        }
        L.base = old;
      }
      L.tbase = (!L.fail && ttot) ? (uint32_t)atomicAdd((unsigned long long *)&t.meta[M_TLEN], (unsigned long long)ttot) : 0;
    }
    __syncthreads();
    if (L.fail) {
      // resumable: nothing of this chunk was applied (keys inserted stay, idempotent)
      if (threadIdx.x == 0) {
        sp.progress[b] = c;
        atomicOr((unsigned int *)&t.meta[M_FAIL], 1u);
      }
      break;
    }
    // 7. apply; the touched list + per-slot mark (lowest index this batch
    // rewrote) let k_ss_emit write each touched session once per batch
    uint64_t my_alloc = L.base + npos;
    uint32_t tp = L.tbase + tpos;
    const uint64_t bmark = (uint64_t)(~p.batch_id) << 32;
#pragma unroll
    for (int u = 0; u < kMgPer; ++u) {
      const uint32_t g = u * kMgNT + threadIdx.x;
      if (g >= ngrp || gslot[u] < 0) continue;
      const uint32_t ra = L.gfirst[g], rb = L.gfirst[g + 1];
      const SessList Ls = gl[u];
      const uint64_t i0 = gi0[u];
      const bool reloc = gcap[u] != 0;
      uint64_t dst = Ls.off;
      if (reloc) {
        dst = my_alloc;
        my_alloc += gcap[u];
        for (uint64_t k = 0; k < i0; ++k) ss_copy(t, dst + k, t, Ls.off + k, ns);
      }
      MgSess<MS> tail[kMgTail];
#pragma unroll
      for (int k = 0; k < kMgTail; ++k) {
        const uint64_t j = i0 + k;
        if (!reloc && j < Ls.len) {
          tail[k].s = t.a_start[Ls.off + j];
          tail[k].e = t.a_end[Ls.off + j];
          tail[k].stamp = t.a_stamp[Ls.off + j];
#pragma unroll
          for (int s = 0; s < MS; ++s) tail[k].a[s] = s < ns ? t.a_aggs[(Ls.off + j) * ns + s] : 0;
        } else {
          tail[k].s = tail[k].e = 0;
          tail[k].stamp = 0;
#pragma unroll
          for (int s = 0; s < MS; ++s) tail[k].a[s] = 0;
        }
        tail[k].fresh = false;
      }
      mg_sweep<MS, W, true>(L, prog, t, p.gap, recs, ra, rb, Ls.off, i0, Ls.len, !reloc, tail, dst, p.batch_id);
      t.lists[gslot[u]] = SessList{dst, (uint32_t)(i0 + gM[u]), reloc ? gcap[u] : Ls.cap};
      live_delta += (int64_t)gM[u] - (int64_t)(Ls.len - i0);
      atomicMin((unsigned long long *)&t.emark[gslot[u]], (unsigned long long)(bmark | i0));
      sp.touched[tp++] = (uint32_t)gslot[u];
    }
    __syncthreads();
    if (c + 1 == nch && threadIdx.x == 0) sp.progress[b] = nch;
  }
  // live sessions, keys, touched rows, errors
  const uint64_t ld = mg_sum64(L, (uint64_t)live_delta);
  const uint64_t kn = mg_sum64(L, keys_new);
  if (threadIdx.x == 0) {
    if (ld) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)ld);
    if (kn) atomicAdd((unsigned long long *)&t.meta[M_KEYS], (unsigned long long)kn);
  }
  if (err) atomicOr(&sc->err, err);
}

template <int MS>
static void merge_launch_w(hipStream_t s, int words, dim3 g, const SessParams &p, const SessTable &t,
                           const Program &prog, int np_log2, const SessPart &sp, DevScalars *sc) {
  const dim3 th(kMgNT);
  switch (words) {
    case 2: hipLaunchKernelGGL((k_ss_merge<MS, 2>), g, th, 0, s, p, t, prog, np_log2, sp, sc); break;
    case 3: hipLaunchKernelGGL((k_ss_merge<MS, 3>), g, th, 0, s, p, t, prog, np_log2, sp, sc); break;
    case 4: hipLaunchKernelGGL((k_ss_merge<MS, 4>), g, th, 0, s, p, t, prog, np_log2, sp, sc); break;
    case 5: hipLaunchKernelGGL((k_ss_merge<MS, 5>), g, th, 0, s, p, t, prog, np_log2, sp, sc); break;
    case 6: hipLaunchKernelGGL((k_ss_merge<MS, 6>), g, th, 0, s, p, t, prog, np_log2, sp, sc); break;
    default: hipLaunchKernelGGL((k_ss_merge<MS, kSessMaxWords>), g, th, 0, s, p, t, prog, np_log2, sp, sc); break;
  }
}

void launch_ss_merge(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, int np_log2,
                     int words, const SessPart &sp, DevScalars *sc) {
  const dim3 g(1u << np_log2);
  if (prog.n_slots <= 2) merge_launch_w<2>(s, words, g, p, t, prog, np_log2, sp, sc);
  else if (prog.n_slots <= 4) merge_launch_w<4>(s, words, g, p, t, prog, np_log2, sp, sc);
  else merge_launch_w<8>(s, words, g, p, t, prog, np_log2, sp, sc);
}

// Per-batch changelog of the merge path: every session of a touched key at or
// after the lowest index the batch rewrote, stamped by this batch. A key may
// appear once per chunk in the touched list; the first entry to take the
// slot's mark (resetting it) emits. emit = 0: count only (state-only ops).
__global__ __launch_bounds__(256) void k_ss_emit(SessTable t, Program prog, SessPart sp, uint32_t batch_id, int emit,
                                                 OutCols out, uint64_t out_base, DevScalars *sc) {
  __shared__ uint64_t swave[4];
  __shared__ uint64_t sbase;
  const uint64_t n = t.meta[M_TLEN];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  for (uint64_t blk = blockIdx.x * 256ull; blk < n; blk += (uint64_t)gridDim.x * 256ull) {
    const uint64_t q = blk + threadIdx.x;
    uint64_t cnt = 0, i0 = 0;
    SessList Ls = {0, 0, 0};
    uint32_t key = 0;
    if (q < n) {
      const uint32_t sl = sp.touched[q];
      const uint64_t m = atomicExch((unsigned long long *)&t.emark[sl], ~0ull);
      if ((uint32_t)(m >> 32) == ~batch_id) {
        i0 = m & 0xFFFFFFFFull;
        Ls = t.lists[sl];
        key = t.keys[sl];
        for (uint64_t k = i0; k < Ls.len; ++k) cnt += t.a_stamp[Ls.off + k] == batch_id;
      } else {
        Ls.len = 0;
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
      for (uint64_t k = i0; k < Ls.len; ++k) {
        const uint64_t a = Ls.off + k;
        if (t.a_stamp[a] != batch_id) continue;
        out.key[o] = key;
        out.ws[o] = t.a_start[a];
        out.we[o] = t.a_end[a];
        out.src[o] = -1;
        const int64_t *row = t.a_aggs + a * prog.n_slots;
        for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, row);
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
      key = t.keys[s];
      if (key != kSessEmptyKey) {
        const SessList Ls = t.lists[s];
        len = Ls.len;
        off = Ls.off;
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

void launch_ss_dump(hipStream_t s, const SessTable &t, const Program &prog, OutCols out, uint64_t out_cap,
                    uint64_t *counter) {
  uint64_t blocks = (t.kmask + 1 + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  hipLaunchKernelGGL(k_ss_dump, dim3((unsigned)blocks), dim3(256), 0, s, t, prog, out, out_cap, counter);
}

}  // namespace hsg
