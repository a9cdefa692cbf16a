// gfx950 kernels for the exact per-record changelog of time windows
// (HSG_EMIT_PER_RECORD): the reference forwards, for every record and every
// accepted window in ascending start, the group's aggregate right after that
// record (TimeWindowedStream.hs:89-103). Batch restatement:
//   count   accepted windows per record (stream time + grace as in k_window)
//   scan    -> pair offsets (pair = (record, window) in arrival x window order)
//   expand  find/insert each pair's group slot
//   sort    stable radix sort of pairs by slot (arrival order kept per group)
//   scan    segmented inclusive scan of the pairs' contributions per group,
//           seeded with the group's state before the batch
//   apply   one changelog row per pair at its arrival position; final rows
//           go to a shadow table and are committed after every read is done
#include "hsg_dev.h"
#include "hsg_perrecord.h"
#include "hsg_tw.h"

namespace hsg {

constexpr int kSegThreads = 256;
constexpr int kSegItems = 8;
constexpr int kSegTile = kSegThreads * kSegItems;

// ---------------------------------------------------------------------------
// count / expand (one record tile per workgroup, same layout as k_tw_agg)
// ---------------------------------------------------------------------------
template <int PASS>
__global__ __launch_bounds__(kTileThreads) void k_pr_pairs(Batch b, TwParams p, TwTable t,
                                                           const int64_t *__restrict__ tprefix,
                                                           const int64_t *__restrict__ rec_wm, PrBuffers pb,
                                                           DevScalars *sc) {
  __shared__ uint64_t sred[3][kTileThreads / 64];
  const uint64_t base = (uint64_t)blockIdx.x * kTileRecords;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t k_epoch = sc->k_epoch;
  uint32_t key[kRecPerThread];
  int64_t ts[kRecPerThread], wm[kRecPerThread];
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    bool in = i < b.n;
    key[r] = in ? b.key[i] : HSG_KEY_NONE;
    ts[r] = in ? b.ts[i] : INT64_MIN;
    if (rec_wm) wm[r] = in ? rec_wm[i] : INT64_MIN;
  }
  if (!rec_wm) tile_stream_time(ts, tprefix[blockIdx.x], wm);
  uint64_t late = 0, pairs = 0;
  uint32_t fresh = 0, err = 0;
#pragma unroll 1
  for (int r = 0; r < kRecPerThread; ++r) {
    const uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    if (i >= b.n) continue;
    uint32_t c = 0;
    uint64_t k_lo, k_hi;
    uint64_t o = PASS == 1 ? pb.off[i] : 0;
    if (key[r] != HSG_KEY_NONE && record_windows(p, ts[r], k_lo, k_hi)) {
      for (uint64_t k = k_lo; k <= k_hi; ++k) {
        if (!window_accepted(p, k, wm[r])) { late += 1; continue; }
        int64_t krel = (int64_t)k - k_epoch;
        if (krel < 0 || krel > 0xFFFFFFFFll) { err |= ERR_RANGE; continue; }
        if (PASS == 1) {
          uint64_t g = ((uint64_t)key[r] << 32) | (uint64_t)krel;
          int64_t slot = tw_find_or_insert(t, g, fresh);
          uint32_t s32;
          if (slot < 0) { err |= ERR_OOM; s32 = (uint32_t)t.slots(); }
          else { s32 = (uint32_t)slot; *t.stamp(slot) = (uint32_t)p.batch_id; }
          pb.pslot[o + c] = s32;
          pb.pidx[o + c] = (uint32_t)(o + c);
          pb.prec[o + c] = (uint32_t)i;
        }
        c += 1;
      }
    }
    if (PASS == 0) pb.cnt[i] = c;
    pairs += c;
  }
  pairs = wave_sum_u64(pairs);
  late = wave_sum_u64(late);
  uint64_t fr = wave_sum_u64(fresh);
  if (lane == 0) { sred[0][w] = pairs; sred[1][w] = late; sred[2][w] = fr; }
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a = 0, l = 0, f = 0;
    for (int k = 0; k < kTileThreads / 64; ++k) { a += sred[0][k]; l += sred[1][k]; f += sred[2][k]; }
    if (PASS == 0) {
      if (a) atomicAdd((unsigned long long *)&sc->pairs, (unsigned long long)a);
      if (l) atomicAdd((unsigned long long *)&sc->late, (unsigned long long)l);
    } else if (f) {
      atomicAdd((unsigned long long *)&sc->live, (unsigned long long)f);
    }
  }
}

void launch_pr_count(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const int64_t *tprefix,
                     const int64_t *rec_wm, const PrBuffers &pb, DevScalars *sc) {
  uint64_t tiles = (b.n + kTileRecords - 1) / kTileRecords;
  if (tiles)
    hipLaunchKernelGGL(k_pr_pairs<0>, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, p, t, tprefix, rec_wm, pb,
                       sc);
}
void launch_pr_expand(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const int64_t *tprefix,
                      const int64_t *rec_wm, const PrBuffers &pb, DevScalars *sc) {
  uint64_t tiles = (b.n + kTileRecords - 1) / kTileRecords;
  if (tiles)
    hipLaunchKernelGGL(k_pr_pairs<1>, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, p, t, tprefix, rec_wm, pb,
                       sc);
}

// ---------------------------------------------------------------------------
// segmented scan over the sorted pairs
// ---------------------------------------------------------------------------
template <int MS>
struct SegVal {
  int64_t v[MS];
};

template <int MS>
__device__ inline void pair_elem(const Program &prog, const Batch &b, const PrBuffers &pb, const int64_t *seq,
                                 uint64_t rec_base, uint32_t pidx, int64_t (&e)[MS]) {
  const uint32_t rec = pb.prec[pidx];
  const uint64_t seq1 = (seq ? (uint64_t)seq[rec] : rec_base + rec) + 1;
  elem_row<MS>(prog, e, b, rec, seq1);
}

// (hf, v) <- (hf_u, v_u) (+) (hf, v): segmented combine, u earlier
template <int MS>
__device__ inline void seg_combine_earlier(const Program &prog, bool &hf, int64_t (&v)[MS], bool hf_u,
                                           const int64_t (&v_u)[MS]) {
  if (!hf) {
    int64_t tmp[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) tmp[s] = v_u[s];
    combine_row<MS>(prog, tmp, v);
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = tmp[s];
  }
  hf = hf || hf_u;
}

// Block-wide exclusive segmented scan of one (hf, v) per thread, seeded with
// (false, carry). Returns the exclusive prefix in (ehf, ev).
template <int MS>
__device__ inline void block_seg_excl(const Program &prog, bool hf, const int64_t (&v)[MS], const int64_t (&carry)[MS],
                                      bool &ehf, int64_t (&ev)[MS]) {
  __shared__ int64_t swv[4][MS];
  __shared__ int swf[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  // inclusive wave scan
  bool ihf = hf;
  int64_t iv[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) iv[s] = v[s];
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    bool uf = __shfl_up((int)ihf, d, 64) != 0;
    int64_t uv[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) uv[s] = __shfl_up(iv[s], d, 64);
    if (lane >= d) seg_combine_earlier<MS>(prog, ihf, iv, uf, uv);
  }
  if (lane == 63) {
    swf[w] = ihf;
#pragma unroll
    for (int s = 0; s < MS; ++s) swv[w][s] = iv[s];
  }
  // exclusive within the wave
  bool xf = __shfl_up((int)ihf, 1, 64) != 0;
  int64_t xv[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) xv[s] = __shfl_up(iv[s], 1, 64);
  __syncthreads();
  // prefix from the carry and earlier waves
  bool pf = false;
  int64_t pv[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) pv[s] = carry[s];
  for (int k = 0; k < w; ++k) {
    int64_t wv[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) wv[s] = swv[k][s];
    bool wf = swf[k] != 0;
    // (pf, pv) (+) (wf, wv)
    seg_combine_earlier<MS>(prog, wf, wv, pf, pv);
    pf = wf;
#pragma unroll
    for (int s = 0; s < MS; ++s) pv[s] = wv[s];
  }
  if (lane == 0) {
    ehf = pf;
#pragma unroll
    for (int s = 0; s < MS; ++s) ev[s] = pv[s];
  } else {
    seg_combine_earlier<MS>(prog, xf, xv, pf, pv);
    ehf = xf;
#pragma unroll
    for (int s = 0; s < MS; ++s) ev[s] = xv[s];
  }
  __syncthreads();
}

__device__ inline bool seg_head(const uint32_t *slot, uint64_t q) { return q == 0 || slot[q] != slot[q - 1]; }

// per-tile (hf, tail aggregate) of the batch contributions (state excluded)
template <int MS>
__global__ __launch_bounds__(kSegThreads) void k_seg_reduce(Batch b, Program prog, PrBuffers pb, const uint32_t *slot,
                                                            const uint32_t *pidx, uint64_t P, const int64_t *seq,
                                                            uint64_t rec_base, int64_t *blk_v, int32_t *blk_f) {
  const uint64_t q0 = (uint64_t)blockIdx.x * kSegTile + (uint64_t)threadIdx.x * kSegItems;
  bool hf = false;
  int64_t v[MS];
  identity_row<MS>(prog, v);
  for (int r = 0; r < kSegItems; ++r) {
    uint64_t q = q0 + r;
    if (q >= P) break;
    int64_t e[MS];
    pair_elem<MS>(prog, b, pb, seq, rec_base, pidx[q], e);
    if (seg_head(slot, q)) {
      hf = true;
      identity_row<MS>(prog, v);
    }
    combine_row<MS>(prog, v, e);
  }
  int64_t zero[MS];
  identity_row<MS>(prog, zero);
  bool ehf;
  int64_t ev[MS];
  block_seg_excl<MS>(prog, hf, v, zero, ehf, ev);
  if (threadIdx.x == kSegThreads - 1) {
    // inclusive total of the tile = exclusive of the last thread (+) its own
    seg_combine_earlier<MS>(prog, hf, v, ehf, ev);
    blk_f[blockIdx.x] = hf;
#pragma unroll
    for (int s = 0; s < MS; ++s) blk_v[(uint64_t)blockIdx.x * MS + s] = v[s];
  }
}

// single workgroup: carry[t] = segment prefix entering tile t (tiles 0..nb-1)
template <int MS>
__global__ __launch_bounds__(1024) void k_seg_carry(Program prog, const int64_t *blk_v, const int32_t *blk_f,
                                                    uint64_t nb, int64_t *carry) {
  if (threadIdx.x != 0) return;
  bool f = false;
  int64_t v[MS];
  identity_row<MS>(prog, v);
  for (uint64_t t = 0; t < nb; ++t) {
#pragma unroll
    for (int s = 0; s < MS; ++s) carry[t * MS + s] = v[s];
    int64_t bv[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) bv[s] = blk_v[t * MS + s];
    bool bf = blk_f[t] != 0;
    seg_combine_earlier<MS>(prog, bf, bv, f, v);
    f = bf;
#pragma unroll
    for (int s = 0; s < MS; ++s) v[s] = bv[s];
  }
}

template <int MS>
__global__ __launch_bounds__(kSegThreads) void k_seg_apply(Batch b, Program prog, PrBuffers pb, TwParams p,
                                                           TwTable t, const uint32_t *slot, const uint32_t *pidx,
                                                           uint64_t P, const int64_t *seq, const int64_t *carry,
                                                           OutCols out, uint64_t out_base, DevScalars *sc) {
  __shared__ uint64_t sseg[4];
  const uint64_t q0 = (uint64_t)blockIdx.x * kSegTile + (uint64_t)threadIdx.x * kSegItems;
  const uint64_t cap = t.slots();  // region + overflow slots; a pair without one has slot cap
  const int64_t k_epoch = sc->k_epoch;
  const bool unwin = p.kind == HSG_UNWINDOWED;
  // phase 1: thread-local aggregate
  bool hf = false;
  int64_t v[MS];
  identity_row<MS>(prog, v);
  for (int r = 0; r < kSegItems; ++r) {
    uint64_t q = q0 + r;
    if (q >= P) break;
    int64_t e[MS];
    pair_elem<MS>(prog, b, pb, seq, p.rec_base, pidx[q], e);
    if (seg_head(slot, q)) {
      hf = true;
      identity_row<MS>(prog, v);
    }
    combine_row<MS>(prog, v, e);
  }
  int64_t cin[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) cin[s] = carry[(uint64_t)blockIdx.x * MS + s];
  bool ehf;
  int64_t run[MS];
  block_seg_excl<MS>(prog, hf, v, cin, ehf, run);
  // phase 2: rows. run = segment prefix (batch contributions) before q.
  uint64_t segs = 0;
  uint32_t cur_slot = 0xFFFFFFFFu;
  int64_t basev[MS];
  for (int r = 0; r < kSegItems; ++r) {
    uint64_t q = q0 + r;
    if (q >= P) break;
    const uint32_t sl = slot[q];
    const uint32_t pi = pidx[q];
    int64_t e[MS];
    pair_elem<MS>(prog, b, pb, seq, p.rec_base, pi, e);
    if (seg_head(slot, q)) identity_row<MS>(prog, run);
    combine_row<MS>(prog, run, e);
    if (sl >= cap) continue;  // pair without a slot (table full): error already flagged
    if (sl != cur_slot) {
      cur_slot = sl;
#pragma unroll
      for (int s = 0; s < MS; ++s) basev[s] = s < prog.n_slots ? t.aggs(sl)[s] : 0;
    }
    int64_t R[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) R[s] = basev[s];
    combine_row<MS>(prog, R, run);
    // changelog row at the pair's arrival position
    const uint64_t o = out_base + pi;
    const uint32_t rec = pb.prec[pi];
    const uint64_t g = *t.key(sl);
    out.key[o] = (uint32_t)(g >> 32);
    int64_t ws = 0, we = 0;
    if (!unwin) {
      int64_t k = k_epoch + (int64_t)(g & 0xFFFFFFFFull);
      ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
      we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
    }
    out.ws[o] = ws;
    out.we[o] = we;
    out.src[o] = seq ? seq[rec] : (int64_t)(p.rec_base + rec);
    for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value_reg<MS>(prog, j, R);
    if (out.form) out.form[o] = out_form_reg<MS>(prog, R);
    // segment end: final state into the shadow table
    if (q + 1 == P || slot[q + 1] != sl) {
      segs += 1;
#pragma unroll
      for (int s = 0; s < MS; ++s)
        if (s < prog.n_slots) pb.shadow[(uint64_t)sl * prog.n_slots + s] = R[s];
    }
  }
  segs = wave_sum_u64(segs);
  if ((threadIdx.x & 63) == 0) sseg[threadIdx.x >> 6] = segs;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t tot = sseg[0] + sseg[1] + sseg[2] + sseg[3];
    if (tot) atomicAdd((unsigned long long *)&sc->touched, (unsigned long long)tot);
  }
}

// copy final rows of every segment end from the shadow table into the state
__global__ void k_seg_commit(const uint32_t *slot, uint64_t P, uint64_t cap, int n_slots, const int64_t *shadow,
                             TwTable t) {
  for (uint64_t q = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x; q < P; q += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t sl = slot[q];
    if (sl >= cap) continue;
    if (q + 1 == P || slot[q + 1] != sl)
      for (int s = 0; s < n_slots; ++s) t.aggs(sl)[s] = shadow[(uint64_t)sl * n_slots + s];
  }
}

uint64_t seg_tiles(uint64_t P) { return (P + kSegTile - 1) / kSegTile; }

template <int MS>
static void seg_launch(hipStream_t s, const Batch &b, const Program &prog, const PrBuffers &pb, const TwParams &p,
                       const TwTable &t, const uint32_t *slot, const uint32_t *pidx, uint64_t P, const int64_t *seq,
                       OutCols out, uint64_t out_base, DevScalars *sc) {
  uint64_t nb = seg_tiles(P);
  hipLaunchKernelGGL(k_seg_reduce<MS>, dim3((unsigned)nb), dim3(kSegThreads), 0, s, b, prog, pb, slot, pidx, P, seq,
                     p.rec_base, pb.blk_v, pb.blk_f);
  hipLaunchKernelGGL(k_seg_carry<MS>, dim3(1), dim3(1024), 0, s, prog, pb.blk_v, pb.blk_f, nb, pb.carry);
  hipLaunchKernelGGL(k_seg_apply<MS>, dim3((unsigned)nb), dim3(kSegThreads), 0, s, b, prog, pb, p, t, slot, pidx, P,
                     seq, pb.carry, out, out_base, sc);
  hipLaunchKernelGGL(k_seg_commit, dim3(grid_for(P, 256)), dim3(256), 0, s, slot, P, t.slots(), prog.n_slots,
                     pb.shadow, t);
}

void launch_pr_segscan(hipStream_t s, const Batch &b, const Program &prog, const PrBuffers &pb, const TwParams &p,
                       const TwTable &t, const uint32_t *slot, const uint32_t *pidx, uint64_t P, const int64_t *seq,
                       OutCols out, uint64_t out_base, DevScalars *sc) {
  if (P == 0) return;
  if (prog.n_slots <= 2) seg_launch<2>(s, b, prog, pb, p, t, slot, pidx, P, seq, out, out_base, sc);
  else if (prog.n_slots <= 4) seg_launch<4>(s, b, prog, pb, p, t, slot, pidx, P, seq, out, out_base, sc);
  else if (prog.n_slots <= 8) seg_launch<8>(s, b, prog, pb, p, t, slot, pidx, P, seq, out, out_base, sc);
  else if (prog.n_slots <= 16) seg_launch<16>(s, b, prog, pb, p, t, slot, pidx, P, seq, out, out_base, sc);
  else seg_launch<kMaxSlots>(s, b, prog, pb, p, t, slot, pidx, P, seq, out, out_base, sc);
}

}  // namespace hsg
