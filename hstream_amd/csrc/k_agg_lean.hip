// Lean aggregation of packed one-window-per-record batches (tumbling and
// unwindowed ops, the BASELINE C2 / C5 shape), in two launches:
//
//   k_agg_lean   one workgroup per bucket chunk: the chunk's packed records
//                (register double-buffered, no barrier per record block) into
//                an LDS hash table at a 32-bit multiplicative hash of the key
//                plus the window; at the end the live entries are written as
//                group partials [g][slot 0 .. n-1] to the chunk's own range of
//                pb.pane (coalesced stores, nothing waited on). A record whose
//                LDS probe sequence finds no room becomes a one-record partial
//                of its own (rare: buckets are sized to half a table).
//   k_pane_apply one workgroup per aggregation workgroup: its partials into
//                the HBM (key, window) table -- claim / read-modify-write as
//                the general kernel's flush (hsg_agg.h flush_window), touched
//                list for the per-batch changelog.
//
// Splitting the HBM updates out of the aggregation workgroup takes their
// dependent HBM round trips (claim load, CAS, row read) off the LDS-resident
// workgroup: many apply workgroups per CU hide them instead.
//
// Semantics are those of k_part_agg with pane_S = 1 (TimeWindowedStream.hs:
// 86-103 per (key, window) group, commutative SQL aggregates of Codegen.hs:
// 399-469): every record updates exactly one group.
#include <cstring>

#include "hsg_agg.h"

namespace hsg {

// The LDS table takes new groups up to 7/8 of its entries (probe sequences
// stay short: buckets are sized to half a table); past that a record of a new
// group becomes a partial of its own, so a probe sequence always ends.

// LDS home of (key, window): a 32-bit multiplicative hash (top bits),
// linear probing
template <int E>
__device__ inline uint32_t lean_home(uint32_t key, uint32_t w) {
  constexpr int LOG2E = __builtin_ctz(E);
  uint32_t h = key * 0x9E3779B1u + w * 0x85EBCA77u;
  h ^= (h >> 16) * 0x7FEB352Du;
  return h >> (32 - LOG2E);
}

// Sort key of a partial for the write-out: its HBM home row within the slot
// range the bucket's groups can occupy, in kLeanSortBins bins, so that the
// apply's neighbouring lanes update neighbouring rows (shared lines, no
// line touched by two wave-instructions of one workgroup more than needed).
constexpr int kLeanSortBins = 1024;
__device__ inline uint32_t lean_sort_bin(const TwTable &t, const PartParams &pp, uint64_t g) {
  const uint64_t slot = tw_region_base(t, g) + tw_home_in(t, g);
  const int cl = 64 - __builtin_clzll(t.mask);  // log2(cap)
  const int span = pp.np_log2 <= t.rbits ? cl - pp.np_log2 : cl - t.rbits;  // log2 of the bucket's slot range
  const uint64_t local = slot & ((1ull << span) - 1);
  return span > 10 ? (uint32_t)(local >> (span - 10)) : (uint32_t)local;
}

// value of slot s for one packed record (COUNT(col) slots of batches without
// validity arrays are filled from COUNT(*) at write-out)
template <int NS, uint64_t SIG, int W>
__device__ inline void lean_elems(const PRec<W, true> &r, int64_t (&v)[NS]) {
  const ProgSig<SIG> prog;
#pragma unroll
  for (int s = 0; s < NS; ++s) v[s] = prec_elem(prog, s, r);
}

// chunk of this workgroup: records [r0, r1) of bucket b; false past the chunks
__device__ inline bool lean_chunk(const PartParams &pp, const PartBuffers &pb, uint32_t &b, uint64_t &r0,
                                  uint64_t &r1, bool &exclusive) {
  const int nb = 1 << pp.np_log2;
  if (blockIdx.x >= pb.chunk_start[nb]) return false;
  b = pb.chunk_bucket[blockIdx.x];
  const uint32_t c0 = pb.chunk_start[b], c1 = pb.chunk_start[b + 1];
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  r0 = b0 + (uint64_t)(blockIdx.x - c0) * pp.chunk;
  r1 = r0 + pp.chunk < b1 ? r0 + pp.chunk : b1;
  exclusive = c1 - c0 == 1;
  return true;
}

template <int E, int NT, int W, uint64_t SIG>
__global__ __launch_bounds__(NT) void k_agg_lean(PartParams pp, TwTable t, PartBuffers pb, DevScalars *sc) {
  constexpr int NS = ProgSig<SIG>::count();
  constexpr int PW = 1 + NS;  // pane entry words
  constexpr int RB = 4;       // records per thread per block (one block in flight beside it)
  __shared__ uint64_t lkey[E];
  __shared__ int64_t lagg[NS * E];
  __shared__ uint32_t s_cnt, s_ovf, s_fill;
  __shared__ uint32_t s_bin[kLeanSortBins];
  __shared__ uint32_t s_wsum[NT / 64];
  if (sc->redo || !sc->packed) return;  // uniform: the careful path / wide variant runs
  uint32_t b;
  uint64_t r0, r1;
  bool exclusive;
  if (!lean_chunk(pp, pb, b, r0, r1, exclusive)) return;  // uniform
  const ProgSig<SIG> prog;
  const uint32_t kbase = (uint32_t)sc->kbase;
  // without validity arrays COUNT(col) = COUNT(*): not kept in LDS
  int cnt_all_slot = -1;
  uint32_t skip = 0;
#pragma unroll
  for (int s = 0; s < NS; ++s)
    if (prog.op(s) == S_CNT_ALL && cnt_all_slot < 0) cnt_all_slot = s;
  if (!pp.has_valid && cnt_all_slot >= 0) {
#pragma unroll
    for (int s = 0; s < NS; ++s)
      if (prog.op(s) == S_CNT) skip |= 1u << s;
  }
  for (int k = threadIdx.x; k < kLeanSortBins; k += NT) s_bin[k] = 0;
  for (int e = threadIdx.x; e < E; e += NT) {
    lkey[e] = kEmpty;
#pragma unroll
    for (int s = 0; s < NS; ++s) lagg[s * E + e] = slot_identity_dev(prog.op(s));
  }
  if (threadIdx.x == 0) {
    s_cnt = 0;
    s_fill = 0;
    s_ovf = 0;
  }
  uint64_t *const pane = pb.pane + r0 * PW;
  __syncthreads();

  // records: block k holds records r0 + k*RB*NT + u*NT + tid; the next block's
  // loads are issued before the current one is processed
  PRec<W, true> cur[RB], nxt[RB];
  auto load = [&](uint64_t s0, PRec<W, true>(&d)[RB]) {
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const uint64_t i = s0 + (uint64_t)u * NT + threadIdx.x;
      d[u].C = W - 1;
      if (i < r1) {
        if constexpr (W == 2) {
          const ulonglong2 x = *reinterpret_cast<const ulonglong2 *>(pb.rec + i * 2);
          d[u].w[0] = x.x;
          d[u].w[1] = x.y;
        } else {
          d[u].w[0] = pb.rec[i];
        }
      } else {
        d[u].w[0] = kEmpty;  // no record (a real header has nwin = 1 in bits 48..55)
        if constexpr (W == 2) d[u].w[1] = 0;
      }
    }
  };
  load(r0, cur);
  for (uint64_t s0 = r0; s0 < r1; s0 += (uint64_t)RB * NT) {
    if (s0 + (uint64_t)RB * NT < r1) load(s0 + (uint64_t)RB * NT, nxt);
#pragma unroll
    for (int u = 0; u < RB; ++u) {
      const PRec<W, true> &r = cur[u];
      if (r.w[0] == kEmpty) continue;
      const uint32_t key = r.key(), kw = r.krel(kbase);
      const uint64_t g = ((uint64_t)key << 32) | kw;
      uint32_t h = lean_home<E>(key, kw);
      int e = -1;
      for (int probe = 0; probe < E; ++probe) {
        const uint64_t c = lkey[h];
        if (c == g) {
          e = (int)h;
          break;
        }
        if (c == kEmpty) {
          if (*(volatile uint32_t *)&s_fill >= (uint32_t)(E - E / 8)) break;  // full: g is not in the table
          const uint64_t old =
              atomicCAS((unsigned long long *)&lkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
          if (old == kEmpty) atomicAdd(&s_fill, 1u);
          if (old == kEmpty || old == g) {
            e = (int)h;
            break;
          }
        }
        h = (h + 1) & (E - 1);
      }
      if (e >= 0) {
        lds_apply<NS, E>(prog, &lagg[e], r, skip);
      } else {
        // no room: this record is a partial of its own
        int64_t v[NS];
        lean_elems<NS, SIG, W>(r, v);
        if (skip) {
#pragma unroll
          for (int s = 0; s < NS; ++s)
            if ((skip >> s) & 1u) v[s] = 1;
        }
        const uint32_t q = atomicAdd(&s_cnt, 1u);
        uint64_t *o = pane + (uint64_t)q * PW;
        o[0] = g;
#pragma unroll
        for (int s = 0; s < NS; ++s) o[1 + s] = (uint64_t)v[s];
        s_ovf = 1;
      }
    }
    if (s0 + (uint64_t)RB * NT < r1) {
#pragma unroll
      for (int u = 0; u < RB; ++u) cur[u] = nxt[u];
    }
  }
  __syncthreads();

  // live entries -> partials, in the order of their HBM home rows (counting
  // sort over kLeanSortBins bins), after the overflow partials
  constexpr int PER = E / NT;
  uint32_t bin[PER], rank[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const uint64_t g = lkey[k * NT + threadIdx.x];
    bin[k] = g != kEmpty ? lean_sort_bin(t, pp, g) : ~0u;
    rank[k] = g != kEmpty ? atomicAdd(&s_bin[bin[k]], 1u) : 0u;
  }
  __syncthreads();
  // exclusive scan of the bins (kLeanSortBins / NT consecutive bins per thread)
  constexpr int BPT = kLeanSortBins / NT > 0 ? kLeanSortBins / NT : 1;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t loc = 0;
  if (threadIdx.x * BPT < kLeanSortBins) {
#pragma unroll
    for (int k = 0; k < BPT; ++k) loc += s_bin[threadIdx.x * BPT + k];
  }
  const uint32_t incl = (uint32_t)wave_incl_sum((uint64_t)loc);
  if (lane == 63) s_wsum[wv] = incl;
  __syncthreads();
  uint32_t run = incl - loc + s_cnt;  // overflow partials first
  for (int k = 0; k < wv; ++k) run += s_wsum[k];
  uint32_t total = 0;
  for (int k = 0; k < NT / 64; ++k) total += s_wsum[k];
  __syncthreads();
  if (threadIdx.x * BPT < kLeanSortBins) {
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
    const int64_t call = cnt_all_slot >= 0 ? lagg[cnt_all_slot * E + e] : 0;
#pragma unroll
    for (int s = 0; s < NS; ++s) o[1 + s] = (uint64_t)(((skip >> s) & 1u) ? call : lagg[s * E + e]);
  }
  if (threadIdx.x == 0) {
    s_cnt += total;
    atomicAdd((unsigned long long *)&sc->scratch[31], (unsigned long long)s_cnt);  // the apply's room check
  }
  __syncthreads();
  // the batch totals (pairs = records placed, groups = partials) are set by
  // the last apply workgroup: no per-workgroup atomic on a shared counter
  if (threadIdx.x == 0) {
    pb.pane_info[2 * blockIdx.x] = r0;
    pb.pane_info[2 * blockIdx.x + 1] = (uint64_t)s_cnt | ((uint64_t)s_ovf << 32);
    // count | overflow << 31 | split bucket << 30: the apply writes the
    // changelog rows of workgroups with neither itself
    pb.pane_cnt[blockIdx.x] = s_cnt | (s_ovf << 31) | ((exclusive ? 0u : 1u) << 30);
  }
}

// Claim or find g in a table region only this workgroup writes, without a
// global atomic: the plain load of a slot is only a hint (it may show EMPTY
// for a slot another thread of this workgroup has just claimed); the LDS set
// of slots claimed in this launch decides, so a slot is claimed once.
constexpr int kClaimSet = 4096;  // LDS slots (u32 slot + 1); <= kClaimSet / 2 claims per workgroup
__device__ inline bool claim_set_insert(uint32_t *cset, uint32_t slot) {
  uint32_t h = (slot * 0x9E3779B1u) >> (32 - 12);
  for (int probe = 0; probe < kClaimSet; ++probe) {
    const uint32_t old = atomicCAS(&cset[h], 0u, slot + 1u);
    if (old == 0u) return true;
    if (old == slot + 1u) return false;
    h = (h + 1) & (kClaimSet - 1);
  }
  return false;
}

__device__ inline int64_t tw_claim_lds(const TwTable &t, uint64_t g, uint32_t *cset, uint32_t &fresh) {
  const uint64_t base = tw_region_base(t, g);
  uint64_t s = tw_home_in(t, g);
  const uint64_t step = tw_step(t), n = (t.rmask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    const uint64_t cur = *t.key(base + s);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty && claim_set_insert(cset, (uint32_t)(base + s))) {
      *t.key(base + s) = g;
      t.mark(base + s);
      fresh += 1;
      return (int64_t)(base + s);
    }
    s = (s + step) & t.rmask;
  }
  return tw_ovf_claim(t, g, fresh);  // the region's sub-table is full
}

// One workgroup per aggregation workgroup: its partials into the HBM table.
// exclusive (the bucket is one chunk): no other workgroup updates these groups
// in this batch; without overflow partials each group appears once, so a plain
// read-modify-write (plain stores into a row claimed just now) suffices; with
// them, workgroup-scope atomics (this workgroup's XCD L2). Split buckets use
// device-scope atomics, as the general kernel.
//
// Direct changelog (out.key != null, no bucket split, no overflow partial in
// the batch): every group of the batch has exactly one partial, so the row
// this thread leaves is the group's final state for the batch -- its
// per-batch changelog row (k_touch_emit's row) is written here, at the
// partial's position, and the touched list stays empty.
template <uint64_t SIG>
__global__ __launch_bounds__(256) void k_pane_apply(Program rprog, TwParams p, PartParams pp, TwTable t,
                                                    PartBuffers pb, OutCols out, uint64_t out_base, uint64_t out_cap,
                                                    DevScalars *sc) {
  constexpr int NS = ProgSig<SIG>::count();
  constexpr int PW = 1 + NS;
  __shared__ uint64_t s_red[4], s_tot[4], s_d[4], s_t[4];
  __shared__ uint32_t cset[kClaimSet];
  if (sc->redo || !sc->packed) return;  // uniform
  // the batch's groups (at most its partials) may not fit the table at the
  // load it is sized for: nothing is claimed, the host grows the table and
  // runs the batch again (uniform: k_agg_lean has finished)
  if (sc->scratch[31] > pp.room) {
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicOr((unsigned long long *)&sc->scratch[32], 1ull);
    return;
  }
  uint32_t b;
  uint64_t r0, r1;
  bool exclusive;
  if (!lean_chunk(pp, pb, b, r0, r1, exclusive)) return;  // uniform
  const ProgSig<SIG> prog;
  const uint64_t base = pb.pane_info[2 * blockIdx.x], ci = pb.pane_info[2 * blockIdx.x + 1];
  const uint32_t cnt = (uint32_t)ci;
  const bool ovf = (ci >> 32) != 0;
  const bool plain_claim = exclusive && pp.np_log2 <= t.rbits && pp.bshift == t.bshift;
  const bool plain_rmw = exclusive && !ovf;
  // claims arbitrated in LDS: region owned, every group once, slots < 2^32
  const bool lds_claim = plain_claim && plain_rmw && cnt <= kClaimSet / 2 && t.mask < 0xFFFFFFFFull;
  if (lds_claim)
    for (int k = threadIdx.x; k < kClaimSet; k += 256) cset[k] = 0;
  // every workgroup's partial count (a few L2-resident loads per thread instead
  // of a returning atomic on one counter from every workgroup). A workgroup
  // whose bucket is its own and that wrote no overflow partial has every group
  // of its partials exactly once in the batch: its rows go straight to the
  // changelog (positions after the direct rows of the workgroups before it);
  // the others' partials leave touched-list entries for the emit pass, whose
  // rows follow every direct row (sc->scratch[3]).
  const int nb = 1 << pp.np_log2;
  const uint32_t nch = pb.chunk_start[nb];
  const bool has_out = out.key != nullptr;
  uint64_t bd = 0, bt = 0, td = 0, tt = 0;  // before / total, direct / touched
  for (uint32_t k = threadIdx.x; 4 * k < nch; k += 256) {
    const uint4 c4 = reinterpret_cast<const uint4 *>(pb.pane_cnt)[k];
    const uint32_t c[4] = {c4.x, c4.y, c4.z, c4.w};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t w = 4 * k + j;
      if (w >= nch) break;
      const uint32_t n = c[j] & 0x3FFFFFFFu;
      const bool d = has_out && (c[j] >> 30) == 0;
      (d ? td : tt) += n;
      if (w < blockIdx.x) (d ? bd : bt) += n;
    }
  }
  bd = wave_sum_u64(bd);
  bt = wave_sum_u64(bt);
  td = wave_sum_u64(td);
  tt = wave_sum_u64(tt);
  if ((threadIdx.x & 63) == 0) {
    s_red[threadIdx.x >> 6] = bd;
    s_tot[threadIdx.x >> 6] = bt;
    s_d[threadIdx.x >> 6] = td;
    s_t[threadIdx.x >> 6] = tt;
  }
  __syncthreads();
  bd = s_red[0] + s_red[1] + s_red[2] + s_red[3];
  bt = s_tot[0] + s_tot[1] + s_tot[2] + s_tot[3];
  td = s_d[0] + s_d[1] + s_d[2] + s_d[3];
  tt = s_t[0] + s_t[1] + s_t[2] + s_t[3];
  const bool direct = has_out && exclusive && !ovf;
  const uint64_t tb = direct ? bd : bt;
  if (threadIdx.x == 0 && blockIdx.x + 1 == nch) {
    // last workgroup: batch totals (every placed record updates one group)
    sc->scratch[1] = tt;
    sc->scratch[3] = td;
    sc->scratch[2] = tt == 0 ? 1 : 2;
    sc->scratch[0] = td + tt;
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
    int64_t v[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) v[s] = (int64_t)ent[1 + s];
    const uint32_t f0 = fresh;
    const int64_t slot = lds_claim     ? tw_claim_lds(t, g, cset, fresh)
                         : plain_claim ? tw_claim_exclusive(t, g, fresh)
                                       : tw_find_or_insert(t, g, fresh);
    uint32_t tl = kTouchSkip;
    if (slot < 0) {
      err |= ERR_OOM;
    } else {
      int64_t *row = t.aggs(slot);
      uint32_t *stp = t.stamp(slot);
      bool first;
      if (plain_rmw) {
        if (fresh == f0) {
          // an existing group (its earlier windows' batches): combine
          int64_t c[NS];
#pragma unroll
          for (int s = 0; s < NS; ++s) c[s] = __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          const uint32_t st = __hip_atomic_load(stp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
          for (int s = 0; s < NS; ++s) v[s] = slot_combine(prog.op(s), c[s], v[s]);
          first = st != bid;
        } else {
          first = true;  // claimed just now by the group's only writer: the row holds identities
        }
#pragma unroll
        for (int s = 0; s < NS; ++s) row[s] = v[s];
        if (first) *stp = bid;
        if (direct) {
          // v is the group's state after this batch: its changelog row
          const uint64_t o = out_base + tb + q;
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
            for (int j = 0; j < rprog.n_out; ++j) out.agg[j][o] = out_value_reg<NS>(rprog, j, v);
            if (out.form) out.form[o] = out_form_reg<NS>(rprog, v);
          } else {
            err |= ERR_OOM;
          }
          continue;
        }
      } else if (exclusive) {
        // overflow partials: the same group may appear twice in this segment
#pragma unroll
        for (int s = 0; s < NS; ++s) {
          const int op = prog.op(s);
          const int64_t x = v[s];
          if (x == slot_identity_dev(op)) continue;
          switch (op) {
            case S_CNT_ALL:
            case S_CNT:
            case S_SUM_I:
              __hip_atomic_fetch_add((unsigned long long *)(row + s), (unsigned long long)x, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            case S_SUM_F:
              __hip_atomic_fetch_add((double *)(row + s), __builtin_bit_cast(double, x), __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            case S_MIN_I:
              __hip_atomic_fetch_min((long long *)(row + s), (long long)x, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            case S_MAX_I:
              __hip_atomic_fetch_max((long long *)(row + s), (long long)x, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            case S_MIN_F:
              __hip_atomic_fetch_min((unsigned long long *)(row + s), (unsigned long long)x, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            case S_MAX_F:
              __hip_atomic_fetch_max((unsigned long long *)(row + s), (unsigned long long)x, __ATOMIC_RELAXED,
                                     __HIP_MEMORY_SCOPE_WORKGROUP);
              break;
            default: break;
          }
        }
        first = __hip_atomic_exchange(stp, bid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != bid;
      } else {
        flush_row_atomic<NS>(prog, row, v);
        first = atomicExch(stp, bid) != bid;
      }
      if (first) tl = (uint32_t)slot;
    }
    const uint64_t o = tb + q;
    if (o < pb.touched_cap) pb.touched[o] = tl;
    else err |= ERR_OOM;
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

// ---------------------------------------------------------------------------
// k_seg_apply: the general kernel's deferred window updates (hsg_agg.h
// agg_flush with pp.defer), one workgroup per aggregation workgroup, its
// segments in flush order. Only a bucket's own workgroup defers, so the
// groups are this workgroup's alone: plain read-modify-write; a later segment
// may update a group an earlier one did (a mid-round flush), hence the
// barrier between segments and L2-served (agent-scope) key and row loads.
// Touched-list entries go after the ones the aggregation kernel appended
// itself (sc->scratch[1]); the list length is left in sc->scratch[6]. A clean
// batch (every window updated once: no split bucket, no in-kernel update, no
// mid-round flush, no LAST) gets its changelog rows here instead.
// ---------------------------------------------------------------------------
constexpr int kSegClaimSet = 16384;  // claims per workgroup up to half of it (else workgroup-scope CAS)
#ifndef HSG_SEG_NT
#define HSG_SEG_NT 512  // two workgroups per CU (their 64 KB claim sets); C3 +2 % over 1024 (profiles/r03)
#endif
constexpr int kSegNT = HSG_SEG_NT;  // threads per workgroup
__device__ inline bool seg_claim_insert(uint32_t *cset, uint32_t slot) {
  uint32_t h = (slot * 0x9E3779B1u) >> (32 - 14);
  for (int probe = 0; probe < kSegClaimSet; ++probe) {
    const uint32_t old = atomicCAS(&cset[h], 0u, slot + 1u);
    if (old == 0u) return true;
    if (old == slot + 1u) return false;
    h = (h + 1) & (kSegClaimSet - 1);
  }
  return false;
}

__device__ inline int64_t tw_claim_seg(const TwTable &t, uint64_t g, uint32_t *cset, uint32_t &fresh,
                                       uint64_t skip = 0) {
  const uint64_t base = tw_region_base(t, g);
  const uint64_t step = tw_step(t), n = (t.rmask + 1) / step;
  uint64_t s = (tw_home_in(t, g) + skip * step) & t.rmask;
  for (uint64_t probe = skip; probe < n && probe < kMaxProbes; ++probe) {
    const uint64_t cur = __hip_atomic_load(t.key(base + s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty && seg_claim_insert(cset, (uint32_t)(base + s))) {
      *t.key(base + s) = g;
      t.mark(base + s);
      fresh += 1;
      return (int64_t)(base + s);
    }
    s = (s + step) & t.rmask;
  }
  return tw_ovf_claim(t, g, fresh);  // the region's sub-table is full
}

template <int MS, uint64_t SIG>
__global__ __launch_bounds__(kSegNT) void k_seg_apply(Program prog, TwParams p, PartParams pp, TwTable t, PartBuffers pb,
                                                    OutCols out, uint64_t out_base, uint64_t out_cap, int lean,
                                                    DevScalars *sc) {
  constexpr int NT = kSegNT;
  __shared__ uint64_t s_red[NT / 64], s_tot[NT / 64];
  __shared__ uint32_t cset[kSegClaimSet];
  if (sc->redo || (lean && sc->packed)) return;  // uniform: late batch / the lean kernels took it
  if (pp.hold) return;                           // uniform: k_part_agg held back for table room
  uint32_t b;
  uint64_t r0, r1;
  bool exclusive;
  if (!lean_chunk(pp, pb, b, r0, r1, exclusive)) return;  // uniform
  const ProgView<SIG> pg(prog);  // the common aggregate sets: slot ops baked in
  const int ns = pg.n();
  const uint64_t pw = 1 + (uint64_t)ns;
  const uint32_t nseg = (uint32_t)pb.pane_info[2 * blockIdx.x];
  const uint32_t mine = pb.pane_cnt[blockIdx.x];
  const bool plain_claim = pp.np_log2 <= t.rbits && pp.bshift == t.bshift;
  const bool lds_claim = plain_claim && mine <= kSegClaimSet / 2 && t.mask < 0xFFFFFFFFull;
  if (lds_claim)
    for (int k = threadIdx.x; k < kSegClaimSet; k += NT) cset[k] = 0;
  // every workgroup's deferred count: this one's position and the total
  const int nb = 1 << pp.np_log2;
  const uint32_t nch = pb.chunk_start[nb];
  uint64_t before = 0, total = 0;
  for (uint32_t k = threadIdx.x; k < nch; k += NT) {
    const uint64_t c = pb.pane_cnt[k];
    total += c;
    if (k < blockIdx.x) before += c;
  }
  before = wave_sum_u64(before);
  total = wave_sum_u64(total);
  if ((threadIdx.x & 63) == 0) {
    s_red[threadIdx.x >> 6] = before;
    s_tot[threadIdx.x >> 6] = total;
  }
  __syncthreads();
  before = total = 0;
  for (int k = 0; k < NT / 64; ++k) {
    before += s_red[k];
    total += s_tot[k];
  }
  // the deferred updates (an upper bound on the groups they make) may not fit
  // the table at the load it is sized for: nothing is claimed here, the host
  // grows the table and launches this kernel again on the same segments
  // (k_part_agg's own updates are in; uniform: every workgroup sums the same)
  if (total > pp.room) {
    if (blockIdx.x == 0 && threadIdx.x == 0) {
      atomicOr((unsigned long long *)&sc->scratch[32], 4ull);
      sc->scratch[34] = total;
    }
    return;
  }
  bool has_last = false;
  for (int s = 0; s < ns; ++s) has_last |= pg.op(s) == S_LAST_SEQ;
  const bool direct = out.key != nullptr && pb.chunk_start[nb + 1] == 0 && sc->scratch[5] == 0 && !has_last;
  const uint64_t t0 = sc->scratch[1];  // touched entries the aggregation kernel appended itself
  if (threadIdx.x == 0 && blockIdx.x + 1 == nch) {
    sc->scratch[6] = direct ? 0 : t0 + total;
    if (direct) sc->scratch[3] = total;
    sc->scratch[2] = direct ? 3 : 4;
    sc->scratch[34] = total;  // the host sizes the next batch's table room from it
  }
  const uint32_t bid = (uint32_t)p.batch_id;
  const int64_t k_epoch = sc->k_epoch;
  uint32_t fresh = 0, err = 0;
  uint64_t run = before;
  // SU entries per thread per pass: their partial loads, then their home-key
  // loads, then their row loads are issued together, so one wait (which on
  // CDNA also waits for the pass's earlier stores) covers SU entries
  constexpr int SU = MS <= 2 ? 2 : 1;
  for (uint32_t sg = 0; sg < nseg; ++sg) {
    const uint64_t base = pb.seg[((uint64_t)blockIdx.x * kMaxSeg + sg) * 2];
    const uint64_t cnt = pb.seg[((uint64_t)blockIdx.x * kMaxSeg + sg) * 2 + 1];
    for (uint64_t q0 = threadIdx.x; q0 < cnt; q0 += (uint64_t)NT * SU) {
      uint64_t g[SU];
      int64_t v[SU][MS];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const uint64_t q = q0 + (uint64_t)u * NT;
        const uint64_t *ent = pb.pane + (base + (q < cnt ? q : 0)) * pw;
        g[u] = q < cnt ? ent[0] : kEmpty;
#pragma unroll
        for (int s = 0; s < MS; ++s) v[u][s] = (q < cnt && s < ns) ? (int64_t)ent[1 + s] : 0;
      }
      // the first NP probe positions of all SU groups loaded together (the
      // table runs at up to 3/4 load, where a linear probe often needs more
      // than its home: one round trip instead of one per probe), then
      // resolved in probe order: the group, or the first empty slot claimed
      // through the LDS claim set; past NP positions the full probe
      constexpr int NP = 4;
      uint64_t hb[SU], hh[SU], kh[SU][NP];
      const uint64_t pstep = tw_step(t);
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        hb[u] = hh[u] = 0;
#pragma unroll
        for (int j = 0; j < NP; ++j) kh[u][j] = ~kEmpty;
        if (g[u] != kEmpty && lds_claim) {
          hb[u] = tw_region_base(t, g[u]);
          hh[u] = tw_home_in(t, g[u]);
#pragma unroll
          for (int j = 0; j < NP; ++j)
            kh[u][j] = __hip_atomic_load(t.key(hb[u] + ((hh[u] + j * pstep) & t.rmask)), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      int64_t slot[SU];
      bool isnew[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        slot[u] = -1;
        isnew[u] = false;
        if (g[u] == kEmpty) continue;
        const uint32_t f0 = fresh;
        if (lds_claim) {
#pragma unroll
          for (int j = 0; j < NP; ++j) {
            if (slot[u] >= 0) break;
            const uint64_t pos = hb[u] + ((hh[u] + j * pstep) & t.rmask);
            if (kh[u][j] == g[u]) {
              slot[u] = (int64_t)pos;
            } else if (kh[u][j] == kEmpty && seg_claim_insert(cset, (uint32_t)pos)) {
              // (a failed claim: a peer took the slot for another group, since
              // a group is in one entry of a segment; the probe goes on)
              *t.key(pos) = g[u];
              t.mark(pos);
              fresh += 1;
              slot[u] = (int64_t)pos;
            }
          }
          if (slot[u] < 0) slot[u] = tw_claim_seg(t, g[u], cset, fresh, NP);
        } else {
          slot[u] = plain_claim ? tw_claim_exclusive(t, g[u], fresh) : tw_find_or_insert(t, g[u], fresh);
        }
        isnew[u] = fresh != f0;
      }
      // the rows of the groups found (agent-scope: an earlier segment may have written them)
      int64_t c[SU][MS];
      uint32_t st[SU];
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        st[u] = 0;
#pragma unroll
        for (int s = 0; s < MS; ++s) c[u][s] = 0;
        if (slot[u] < 0 || isnew[u]) continue;
        const int64_t *row = t.aggs(slot[u]);
#pragma unroll
        for (int s = 0; s < MS; ++s)
          c[u][s] = s < ns ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
        st[u] = __hip_atomic_load(t.stamp(slot[u]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
#pragma unroll
      for (int u = 0; u < SU; ++u) {
        const uint64_t q = q0 + (uint64_t)u * NT;
        if (q >= cnt) continue;
        uint32_t tl = kTouchSkip;
        if (slot[u] < 0) {
          err |= ERR_OOM;
        } else {
          int64_t *row = t.aggs(slot[u]);
          uint32_t *stp = t.stamp(slot[u]);
          bool first = true;
          if (!isnew[u]) {
#pragma unroll
            for (int s = 0; s < MS; ++s) {
              if (s >= ns) break;
              const int op = pg.op(s);
              if (op == S_LAST_VAL) continue;
              v[u][s] = op == S_LAST_SEQ ? ((uint64_t)v[u][s] > (uint64_t)c[u][s] ? v[u][s] : c[u][s])
                                         : slot_combine(op, c[u][s], v[u][s]);
            }
            first = st[u] != bid;
          }
#pragma unroll
          for (int s = 0; s < MS; ++s)
            if (s < ns && pg.op(s) != S_LAST_VAL) row[s] = v[u][s];
          if (first) *stp = bid;
          if (direct) {
            const uint64_t o = out_base + run + q;
            if (o < out_cap) {
              out.key[o] = (uint32_t)(g[u] >> 32);
              int64_t ws = 0, we = 0;
              if (p.kind != HSG_UNWINDOWED) {
                const int64_t k = k_epoch + (int64_t)(g[u] & 0xFFFFFFFFull);
                ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
                we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
              }
              out.ws[o] = ws;
              out.we[o] = we;
              out.src[o] = -1;
#pragma unroll
              for (int j = 0; j < kMaxAggs; ++j)
                if (j < prog.n_out) out.agg[j][o] = out_value_reg<MS>(prog, j, v[u]);
              if (out.form) out.form[o] = out_form_reg<MS>(prog, v[u]);
            } else {
              err |= ERR_OOM;
            }
            continue;
          }
          if (first) tl = (uint32_t)slot[u];
        }
        if (!direct) {
          const uint64_t o = t0 + run + q;
          if (o < pb.touched_cap) pb.touched[o] = tl;
          else err |= ERR_OOM;
        }
      }
    }
    run += cnt;
    __syncthreads();  // the next segment may update this one's groups
  }
  if (err) atomicOr(&sc->err, err);
  const uint64_t fr = wave_sum_u64(fresh);
  if ((threadIdx.x & 63) == 0) s_red[threadIdx.x >> 6] = fr;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t f = 0;
    for (int k = 0; k < NT / 64; ++k) f += s_red[k];
    if (f) atomicAdd((unsigned long long *)&sc->live_x[blockIdx.x & 7], (unsigned long long)f);
  }
}

void launch_seg_apply(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                      const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols *out, uint64_t out_base,
                      uint64_t out_cap, bool lean) {
  OutCols oc;
  memset(&oc, 0, sizeof(oc));
  if (out) oc = *out;
  const int l = lean ? 1 : 0;
  const uint64_t sig = program_sig(prog);
  const dim3 th(kSegNT);
  if (sig == kSigCntSumI)
    hipLaunchKernelGGL((k_seg_apply<2, kSigCntSumI>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
  else if (sig == kSigCntSumF)
    hipLaunchKernelGGL((k_seg_apply<2, kSigCntSumF>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
  else if (sig == kSigAllI)
    hipLaunchKernelGGL((k_seg_apply<6, kSigAllI>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
  else if (prog.n_slots <= 2)
    hipLaunchKernelGGL((k_seg_apply<2, 0>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
  else if (prog.n_slots <= 4)
    hipLaunchKernelGGL((k_seg_apply<4, 0>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
  else if (prog.n_slots <= 6)
    hipLaunchKernelGGL((k_seg_apply<6, 0>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
  else
    hipLaunchKernelGGL((k_seg_apply<8, 0>), g, th, 0, s, prog, p, pp, t, pb, oc, out_base, out_cap, l, sc);
}

template <int W, uint64_t SIG>
static bool lean_launch(uint64_t sig, hipStream_t s, dim3 g, bool big, const Program &prog, const TwParams &p,
                        const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc,
                        const OutCols &out, uint64_t out_base, uint64_t out_cap) {
  if (sig != SIG) return false;
  constexpr int NS = ProgSig<SIG>::count();
  constexpr int ES = NS <= 2 ? 2048 : 1024, EL = NS <= 2 ? 4096 : 2048;  // part_lds_entries
  if (big)
    hipLaunchKernelGGL((k_agg_lean<EL, 1024, W, SIG>), g, dim3(1024), 0, s, pp, t, pb, sc);
  else
    hipLaunchKernelGGL((k_agg_lean<ES, 512, W, SIG>), g, dim3(512), 0, s, pp, t, pb, sc);
  hipLaunchKernelGGL((k_pane_apply<SIG>), g, dim3(256), 0, s, prog, p, pp, t, pb, out, out_base, out_cap, sc);
  return true;
}

bool part_lean_eligible(const Program &prog, const PartParams &pp) {
  if (pp.pane_S != 1 || pp.rbits != 0 || pp.has_seq) return false;
  const uint64_t sig = program_sig(prog);
  const int W = pp.words - 1;
  if (W == 1) return sig == kSigCnt;
  return W == 2 && (sig == kSigAllI || sig == kSigAllF || sig == kSigCnt || sig == kSigCntSumI ||
                    sig == kSigCntSumF || sig == kSigSumMaxI);
}

bool launch_part_agg_lean(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                          const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols *out,
                          uint64_t out_base, uint64_t out_cap) {
  OutCols oc;
  memset(&oc, 0, sizeof(oc));
  if (out) oc = *out;
  if (!part_lean_eligible(prog, pp)) return false;
  const int W = pp.words - 1;  // packed words
  const uint64_t sig = program_sig(prog);
  const bool big = pp.big != 0;
  if (W == 1) return lean_launch<1, kSigCnt>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
  if (W != 2) return false;
  return lean_launch<2, kSigAllI>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap) ||
         lean_launch<2, kSigAllF>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap) ||
         lean_launch<2, kSigCnt>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap) ||
         lean_launch<2, kSigCntSumI>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap) ||
         lean_launch<2, kSigCntSumF>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap) ||
         lean_launch<2, kSigSumMaxI>(sig, s, g, big, prog, p, pp, t, pb, sc, oc, out_base, out_cap);
}

}  // namespace hsg
