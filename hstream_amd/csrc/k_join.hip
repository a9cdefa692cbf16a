// gfx950 kernels of the stream-stream join (hsg_join.h): batch entries, the
// LSD sort keys, rank merges with the resident state, the per-record probe
// (binary searches over the merged state, one thread per record) and the
// compactions that form the next state.
//
// Reference semantics (joinStreamProcessor, Stream.hs:267-300, over
// InMemoryTimestampedKVStore, Store.hs:316-385): a record's candidates are the
// other store's entries with its record key and a timestamp in
// [ts - before, ts + after] (the other side: [ts - after, ts + before]),
// ascending; the end points count only when the other store holds some entry
// at both end timestamps (Store.hs:365-372); a candidate is joined when its
// join key equals the record's, and a missing join key on either side stops
// the record's scan there.
#include "hsg_dev.h"
#include "hsg_join.h"

namespace hsg {

__device__ inline bool jless(const JEnt &a, const JEnt &b) {
  if (a.k != b.k) return a.k < b.k;
  if (a.side != b.side) return a.side < b.side;
  if (a.ts != b.ts) return a.ts < b.ts;
  return a.arr < b.arr;
}

__device__ inline bool tless(const TEnt &a, const TEnt &b) {
  if (a.side != b.side) return a.side < b.side;
  if (a.ts != b.ts) return a.ts < b.ts;
  return a.arr < b.arr;
}

// first index in a[0, n) whose element is not less than x
template <typename T, typename L>
__device__ inline uint64_t lower_bound_by(const T *a, uint64_t n, const T &x, L less) {
  uint64_t lo = 0, hi = n;
  while (lo < hi) {
    const uint64_t mid = (lo + hi) >> 1;
    if (less(a[mid], x)) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

#define GRID_LOOP(i, n) \
  for (uint64_t i = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; i < (n); i += (uint64_t)gridDim.x * blockDim.x)

__global__ void k_join_build(JoinBatchDev b, JEnt *out) {
  GRID_LOOP(i, b.n) {
    JEnt e;
    e.k = b.key[i];
    e.jkey = b.jkey[i];
    e.ts = b.ts[i];
    e.handle = b.handle[i];
    const bool own = b.nranks <= 1 || join_owner(e.k, b.nranks) == b.rank;
    e.side = e.k == HSG_KEY_NONE ? 2u : ((b.side[i] ? 1u : 0u) | (own ? 0u : 4u));
    e.arr = (uint32_t)i + 1;
    out[i] = e;
  }
}

__global__ void k_join_sortkey(const JEnt *e, const uint32_t *perm, uint64_t n, int pass, uint32_t *key) {
  GRID_LOOP(i, n) {
    const JEnt &x = e[perm[i]];
    uint32_t v;
    if (pass == 0) v = (uint32_t)(uint64_t)x.ts;
    else if (pass == 1) v = (uint32_t)((uint64_t)x.ts >> 32) ^ 0x80000000u;
    else if (pass == 2) v = x.side & 3u;  // (a record another rank owns sorts by its side: all of its key's are)
    else v = x.k;
    key[i] = v;
  }
}

__global__ void k_join_iota(uint32_t *perm, uint64_t n) { GRID_LOOP(i, n) perm[i] = (uint32_t)i; }

__global__ void k_join_gather(const JEnt *src, const uint32_t *perm, uint64_t n, JEnt *dst) {
  GRID_LOOP(i, n) dst[i] = src[perm[i]];
}

// R entries go to i + |{B < R[i]}|, B entries to j + |{R < B[j]}| (arrivals
// differ, so no element of one equals one of the other)
__global__ void k_join_merge_r(const JEnt *R, uint64_t nR, const JEnt *B, uint64_t nB, JEnt *M) {
  GRID_LOOP(i, nR) {
    const JEnt x = R[i];
    M[i + lower_bound_by(B, nB, x, jless)] = x;
  }
}
__global__ void k_join_merge_b(const JEnt *R, uint64_t nR, const JEnt *B, uint64_t nB, JEnt *M, uint32_t *pos) {
  GRID_LOOP(j, nB) {
    const JEnt x = B[j];
    const uint64_t p = j + lower_bound_by(R, nR, x, jless);
    M[p] = x;
    pos[x.arr - 1] = (uint32_t)p;
  }
}

__global__ void k_join_tflags(const JEnt *Bt, uint64_t n, uint32_t *flag) {
  GRID_LOOP(i, n) {
    const JEnt &x = Bt[i];
    // (a record another rank owns keeps its timestamp here: side & 3; the
    // 2-bit side sort pass already ordered the batch by it)
    const uint32_t sd = x.side & 3u;
    flag[i] = sd < 2 && (i == 0 || (Bt[i - 1].side & 3u) != sd || Bt[i - 1].ts != x.ts) ? 1u : 0u;
  }
}
__global__ void k_join_twrite(const JEnt *Bt, uint64_t n, const uint32_t *flag, const uint64_t *off, TEnt *out) {
  GRID_LOOP(i, n) {
    if (!flag[i]) continue;
    TEnt t;
    t.side = Bt[i].side & 3u;
    t.arr = Bt[i].arr;  // the group is in arrival order: its first is the smallest
    t.ts = Bt[i].ts;
    out[off[i]] = t;
  }
}
__global__ void k_join_tmerge_a(const TEnt *A, uint64_t nA, const TEnt *B, uint64_t nB, TEnt *M) {
  GRID_LOOP(i, nA) {
    const TEnt x = A[i];
    M[i + lower_bound_by(B, nB, x, tless)] = x;
  }
}
__global__ void k_join_tmerge_b(const TEnt *A, uint64_t nA, const TEnt *B, uint64_t nB, TEnt *M) {
  GRID_LOOP(j, nB) {
    const TEnt x = B[j];
    M[j + lower_bound_by(A, nA, x, tless)] = x;
  }
}

// does the side's store hold some entry at ts for a record arriving at arr?
__device__ inline bool ts_present(const TEnt *T, uint64_t nT, uint32_t side, int64_t ts, uint32_t arr) {
  TEnt q;
  q.side = side;
  q.ts = ts;
  q.arr = 0;
  const uint64_t p = lower_bound_by(T, nT, q, tless);
  return p < nT && T[p].side == side && T[p].ts == ts && T[p].arr < arr;
}

__global__ void k_join_probe(const JEnt *M, uint64_t nM, const uint32_t *pos, uint64_t n, const TEnt *T, uint64_t nT,
                             int64_t before, int64_t after, uint32_t *cnt, const uint64_t *off, JoinOut out,
                             uint64_t out_base) {
  GRID_LOOP(t, n) {
    const JEnt e = M[pos[t]];
    if (e.side > 1) {
      if (!out.this_h) cnt[t] = 0;
      continue;
    }
    const uint32_t other = 1u - e.side;
    const int64_t lo = (int64_t)((uint64_t)e.ts - (uint64_t)(e.side == 0 ? before : after));
    const int64_t hi = (int64_t)((uint64_t)e.ts + (uint64_t)(e.side == 0 ? after : before));
    // end points only when the other store holds both end timestamps
    const bool ends = lo != hi && ts_present(T, nT, other, lo, e.arr) && ts_present(T, nT, other, hi, e.arr);
    JEnt q;
    q.k = e.k;
    q.side = other;
    q.ts = lo;
    q.arr = 0;
    uint64_t x = lower_bound_by(M, nM, q, jless);
    uint32_t c = 0;
    uint64_t o = out.this_h ? out_base + off[t] : 0;
    while (x < nM && M[x].k == e.k && M[x].side == other && M[x].ts <= hi) {
      // one timestamp group: its entries in arrival order
      const int64_t g_ts = M[x].ts;
      uint64_t g_end = x + 1;
      while (g_end < nM && M[g_end].k == e.k && M[g_end].side == other && M[g_end].ts == g_ts) ++g_end;
      const bool inside = ends || (g_ts != lo && g_ts != hi);
      if (inside) {
        // the version the other store held when e arrived: the latest earlier one
        int64_t pick = -1;
        for (uint64_t y = g_end; y > x; --y)
          if (M[y - 1].arr < e.arr) {
            pick = (int64_t)(y - 1);
            break;
          }
        if (pick >= 0) {
          const JEnt &cand = M[pick];
          if (e.jkey == HSG_KEY_NONE || cand.jkey == HSG_KEY_NONE) break;  // the key selector throws here
          if (cand.jkey == e.jkey) {
            if (out.this_h) {
              out.this_h[o] = e.side == 0 ? e.handle : cand.handle;
              out.other_h[o] = e.side == 0 ? cand.handle : e.handle;
              out.jkey[o] = e.jkey;
              out.ts[o] = e.ts > cand.ts ? e.ts : cand.ts;
              ++o;
            }
            ++c;
          }
        }
      }
      x = g_end;
    }
    if (!out.this_h) cnt[t] = c;
  }
}

__global__ void k_join_rflags(const JEnt *M, uint64_t n, uint32_t *flag) {
  GRID_LOOP(i, n) {
    const JEnt &x = M[i];
    const bool last = i + 1 == n || M[i + 1].k != x.k || M[i + 1].side != x.side || M[i + 1].ts != x.ts;
    flag[i] = x.side < 2 && last ? 1u : 0u;
  }
}
__global__ void k_join_rwrite(const JEnt *M, uint64_t n, const uint32_t *flag, const uint64_t *off, JEnt *out) {
  GRID_LOOP(i, n) {
    if (!flag[i]) continue;
    JEnt x = M[i];
    x.arr = 0;
    out[off[i]] = x;
  }
}
__global__ void k_join_tkeep(const TEnt *T, uint64_t n, uint32_t *flag) {
  GRID_LOOP(i, n) flag[i] = (i == 0 || T[i - 1].side != T[i].side || T[i - 1].ts != T[i].ts) ? 1u : 0u;
}
__global__ void k_join_tkeep_write(const TEnt *T, uint64_t n, const uint32_t *flag, const uint64_t *off, TEnt *out) {
  GRID_LOOP(i, n) {
    if (!flag[i]) continue;
    TEnt t = T[i];
    t.arr = 0;
    out[off[i]] = t;
  }
}

#define LAUNCH(k, n, ...) \
  do { if (n) hipLaunchKernelGGL(k, dim3(grid_for(n, 256)), dim3(256), 0, s, __VA_ARGS__); } while (0)

void launch_join_build(hipStream_t s, const JoinBatchDev &b, JEnt *out) { LAUNCH(k_join_build, b.n, b, out); }

__global__ void k_join_compact(JoinBatchDev slots, uint64_t stride, const int64_t *off, int G, uint64_t n,
                               uint8_t *side, uint32_t *key, uint32_t *jkey, int64_t *ts, uint64_t *handle) {
  GRID_LOOP(i, n) {
    int q = 0;
    while (q + 1 < G && (uint64_t)off[q + 1] <= i) ++q;
    const uint64_t src = (uint64_t)q * stride + (i - (uint64_t)off[q]);
    side[i] = slots.side[src];
    key[i] = slots.key[src];
    jkey[i] = slots.jkey[src];
    ts[i] = slots.ts[src];
    handle[i] = slots.handle[src];
  }
}
void launch_join_compact(hipStream_t s, const JoinBatchDev &slots, uint64_t stride, const int64_t *off, int G,
                         uint64_t n, uint8_t *side, uint32_t *key, uint32_t *jkey, int64_t *ts, uint64_t *handle) {
  LAUNCH(k_join_compact, n, slots, stride, off, G, n, side, key, jkey, ts, handle);
}
void launch_join_sortkey(hipStream_t s, const JEnt *e, const uint32_t *perm, uint64_t n, int pass, uint32_t *key) {
  LAUNCH(k_join_sortkey, n, e, perm, n, pass, key);
}
void launch_join_iota(hipStream_t s, uint32_t *perm, uint64_t n) { LAUNCH(k_join_iota, n, perm, n); }
void launch_join_gather(hipStream_t s, const JEnt *src, const uint32_t *perm, uint64_t n, JEnt *dst) {
  LAUNCH(k_join_gather, n, src, perm, n, dst);
}
void launch_join_merge(hipStream_t s, const JEnt *R, uint64_t nR, const JEnt *B, uint64_t nB, JEnt *M, uint32_t *pos) {
  LAUNCH(k_join_merge_r, nR, R, nR, B, nB, M);
  LAUNCH(k_join_merge_b, nB, R, nR, B, nB, M, pos);
}
void launch_join_tflags(hipStream_t s, const JEnt *Bt, uint64_t n, uint32_t *flag) { LAUNCH(k_join_tflags, n, Bt, n, flag); }
void launch_join_twrite(hipStream_t s, const JEnt *Bt, uint64_t n, const uint32_t *flag, const uint64_t *off, TEnt *out) {
  LAUNCH(k_join_twrite, n, Bt, n, flag, off, out);
}
void launch_join_tmerge(hipStream_t s, const TEnt *A, uint64_t nA, const TEnt *B, uint64_t nB, TEnt *M) {
  LAUNCH(k_join_tmerge_a, nA, A, nA, B, nB, M);
  LAUNCH(k_join_tmerge_b, nB, A, nA, B, nB, M);
}
void launch_join_probe(hipStream_t s, const JEnt *M, uint64_t nM, const uint32_t *pos, uint64_t n, const TEnt *T,
                       uint64_t nT, int64_t before, int64_t after, uint32_t *cnt, const uint64_t *off, JoinOut out,
                       uint64_t out_base) {
  LAUNCH(k_join_probe, n, M, nM, pos, n, T, nT, before, after, cnt, off, out, out_base);
}
void launch_join_rflags(hipStream_t s, const JEnt *M, uint64_t n, uint32_t *flag) { LAUNCH(k_join_rflags, n, M, n, flag); }
void launch_join_rwrite(hipStream_t s, const JEnt *M, uint64_t n, const uint32_t *flag, const uint64_t *off, JEnt *out) {
  LAUNCH(k_join_rwrite, n, M, n, flag, off, out);
}
void launch_join_tkeep(hipStream_t s, const TEnt *T, uint64_t n, uint32_t *flag) { LAUNCH(k_join_tkeep, n, T, n, flag); }
void launch_join_tkeep_write(hipStream_t s, const TEnt *T, uint64_t n, const uint32_t *flag, const uint64_t *off,
                             TEnt *out) {
  LAUNCH(k_join_tkeep_write, n, T, n, flag, off, out);
}

}  // namespace hsg
