// gfx950 kernels of the partitioned (key, window) aggregation:
//
//   hist     per-tile bucket counts of the records that have >= 1 accepted
//            window (bucket = top bits of hash(key): every window of a key
//            lands in one bucket), tile-major
//   offsets  column sums / scan / column prefix -> each (tile, bucket) run's
//            place in the bucket-major record array
//   scatter  every record stored from registers at its run slot (LDS atomic),
//            packed 16-byte records for one-column ops
//   agg      one workgroup per bucket (or per <= kAggChunk records of a big
//            one): records -> panes in an LDS hash table, panes -> windows,
//            one update per window into the HBM table -- plain
//            read-modify-write when the workgroup is the bucket's only chunk
//            (it owns those groups), atomics otherwise
//   emit     per-batch changelog rows of the groups first updated this batch
//
// Window assignment and grace follow TimeWindowedStream.hs:86-103 / :105-117
// exactly as in k_window.hip (rejected windows are always the earliest ones, so
// the accepted windows of a record are one consecutive run).
#include <cstring>

#include "hsg_dev.h"
#include "hsg_part.h"
#include "hsg_sort.h"
#include "hsg_tw.h"

namespace hsg {

constexpr uint16_t kNoBucket = 0xFFFF;

// bucket = the np_log2 hash bits below the top `bshift` (owner) bits
__device__ inline uint32_t bucket_of(uint32_t key, int np_log2, int bshift) {
  return np_log2 ? (uint32_t)((key_hash(key) << bshift) >> (64 - np_log2)) : 0u;
}

// Accepted window run of one record: [krel, krel + nwin) relative to the epoch.
__device__ inline bool part_record(const TwParams &p, int64_t k_epoch, uint32_t key, int64_t ts, int64_t wm,
                                   uint32_t &krel, uint32_t &nwin, uint64_t &late, uint32_t &err) {
  if (key == HSG_KEY_NONE) return false;
  uint64_t k_lo, k_hi;
  if (!record_windows(p, ts, k_lo, k_hi)) return false;
  uint64_t k = k_lo;
  while (k <= k_hi && !window_accepted(p, k, wm)) {
    ++k;
    ++late;
  }
  if (k > k_hi) return false;
  int64_t a = (int64_t)k - k_epoch, z = (int64_t)k_hi - k_epoch;
  if (a < 0) {
    err |= ERR_RANGE;
    a = 0;
  }
  if (z > 0xFFFFFFFFll) {
    err |= ERR_RANGE;
    z = 0xFFFFFFFFll;
  }
  if (a > z) return false;
  krel = (uint32_t)a;
  nwin = (uint32_t)(z - a + 1);
  return true;
}


// Per-record stream time in arrival order, only when some record of the batch
// may fail the grace check (sc->no_late == 0); otherwise every workgroup exits.
__global__ __launch_bounds__(kTileThreads) void k_part_recwm(Batch b, const int64_t *__restrict__ tprefix,
                                                             const DevScalars *sc, int64_t *__restrict__ wm_out) {
  if (sc->no_late) return;  // uniform
  const uint64_t base = (uint64_t)blockIdx.x * kTileRecords;
  int64_t ts[kRecPerThread], wm[kRecPerThread];
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    ts[r] = i < b.n ? b.ts[i] : INT64_MIN;
  }
  tile_stream_time(ts, tprefix[blockIdx.x], wm);
#pragma unroll
  for (int r = 0; r < kRecPerThread; ++r) {
    uint64_t i = base + (uint64_t)r * kTileThreads + threadIdx.x;
    if (i < b.n) wm_out[i] = wm[r];
  }
}

void launch_part_recwm(hipStream_t s, const Batch &b, const int64_t *tprefix, const DevScalars *sc, int64_t *wm) {
  uint64_t tiles = (b.n + kTileRecords - 1) / kTileRecords;
  if (tiles) hipLaunchKernelGGL(k_part_recwm, dim3((unsigned)tiles), dim3(kTileThreads), 0, s, b, tprefix, sc, wm);
}

// stream time source: the exchange's per-record times, else our own unless no
// record can be late (then every window is accepted and none is needed)
__device__ inline const int64_t *pick_wm(const int64_t *rec_wm, const int64_t *own, const DevScalars *sc) {
  return rec_wm ? rec_wm : (sc->no_late ? nullptr : own);
}

// Order-preserving u64 image of an i64 (max of images = image of the max).
__device__ inline uint64_t i64_ord(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }

// Stable ranking for the per-record changelog, which needs a bucket's records
// in arrival order (k_prpart.hip): a tile's records are ranked in rounds of
// kPNT consecutive records (record = round * kPNT + thread), so within a
// round the lanes of earlier waves and lower lanes come first. Lanes of one
// wave with the same bucket find each other with one ballot per bucket bit;
// wcnt[w][b] holds wave w's count of bucket b in this round (cleared again by
// its writer before the next round). Returns this record's rank among its
// bucket's records of the round (earlier rounds are the caller's base).
constexpr int kPNT = 512;  // threads of the partition passes
constexpr int kPW = kPNT / 64;
__device__ inline uint32_t stable_round_rank(uint32_t bk, bool ok, int nbits, uint8_t (*wcnt)[1 << kPartMaxLog2],
                                             uint64_t &peers) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t m = __ballot(ok);
  for (int bit = 0; bit < nbits; ++bit) {
    const bool x = (bk >> bit) & 1u;
    const uint64_t bb = __ballot(x);
    m &= x ? bb : ~bb;
  }
  peers = m;
  const bool leader = ok && (m >> lane) == 1ull;
  if (leader) wcnt[wv][bk] = (uint8_t)__popcll(m);
  lds_barrier();
  uint32_t before = 0;
  if (ok)
    for (int w = 0; w < wv; ++w) before += wcnt[w][bk];
  return before + (uint32_t)__popcll(m & ((1ull << lane) - 1ull));
}
// Lanes of this wave whose (ok) bucket equals ours: one ballot per bucket bit.
__device__ inline uint64_t match_peers(uint32_t bk, bool ok, int nbits) {
  uint64_t m = __ballot(ok);
  for (int bit = 0; bit < nbits; ++bit) {
    const bool x = (bk >> bit) & 1u;
    const uint64_t bb = __ballot(x);
    m &= x ? bb : ~bb;
  }
  return m;
}
__device__ inline void stable_round_done(uint32_t bk, bool ok, uint64_t peers, uint8_t (*wcnt)[1 << kPartMaxLog2]) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (ok && (peers >> lane) == 1ull) wcnt[wv][bk] = 0;
}

// Walk the T records of one partition tile with NT threads (record (r, t) =
// tile*T + r*NT + t); calls f(j, i, key, krel, nwin) for every record with
// >= 1 accepted window (j = tile-local index, i = batch index). No barriers.
// ext (optional): ext[0] = max image of every record's ts, ext[1] = max of
// ~image of the ts of keyed records with ts >= 0 (i.e. their min); 0 = none.
template <int T, int NT, typename F>
__device__ inline void walk_tile(const Batch &b, const TwParams &p, uint64_t tile, int64_t k_epoch,
                                 const int64_t *__restrict__ wm, uint64_t &late, uint32_t &err, F f,
                                 uint64_t *ext = nullptr) {
  constexpr int R = T / NT;
  const uint64_t base = tile * T;
  // every load of the tile is issued before the first record is processed
  uint32_t key[R];
  int64_t ts[R], w[R];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t i = base + (uint64_t)r * NT + threadIdx.x;
    const bool in = i < b.n;
    key[r] = in ? b.key[i] : HSG_KEY_NONE;
    ts[r] = in ? b.ts[i] : 0;
    w[r] = in && wm ? wm[i] : INT64_MIN;
  }
  if (ext) {
    uint64_t mx = 0, mn = 0;
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t i = base + (uint64_t)r * NT + threadIdx.x;
      const uint64_t o = i64_ord(ts[r]);
      if (i < b.n) mx = o > mx ? o : mx;
      if (key[r] != HSG_KEY_NONE && ts[r] >= 0) mn = ~o > mn ? ~o : mn;
    }
    ext[0] = mx;
    ext[1] = mn;
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int j = r * NT + threadIdx.x;
    uint32_t krel, nwin;
    if (!part_record(p, k_epoch, key[r], ts[r], w[r], krel, nwin, late, err)) continue;
    f(j, base + j, key[r], krel, nwin);
  }
}


template <int T>
__global__ __launch_bounds__(kPNT) void k_part_hist(Batch b, TwParams p, PartParams pp,
                                                    const int64_t *__restrict__ rec_wm,
                                                    const int64_t *__restrict__ own_wm, PartBuffers pb,
                                                    DevScalars *sc, int opt) {
  __shared__ uint32_t cnt[1 << kPartMaxLog2];
  __shared__ uint64_t sred[kPNT / 64];
  __shared__ uint64_t sext[2][kPNT / 64];
  __shared__ uint64_t spairs[kPNT / 64];
  const int nb = 1 << pp.np_log2;
  const uint64_t tile = xcd_tile(blockIdx.x, pp.tiles);
  for (int i = threadIdx.x; i < nb; i += kPNT) cnt[i] = 0;
  __syncthreads();
  uint64_t late = 0;
  uint32_t err = 0;
  // optimistic pass: no record is assumed late (checked by k_part_decide); the
  // stream-time inputs of the batch come out of the same walk: max ts of every
  // record (Processor.hs:139), min ts of the keyed records (as k_tile_stats)
  uint64_t ext[2] = {0, 0};
  uint64_t npairs = 0;
  for (int st = 0; st < pp.sub; ++st) {
    uint64_t e2[2] = {0, 0};
    walk_tile<T, kPNT>(b, p, tile * pp.sub + st, sc->k_epoch, opt ? nullptr : pick_wm(rec_wm, own_wm, sc), late, err,
                       [&](int, uint64_t, uint32_t key, uint32_t, uint32_t nwin) {
                         atomicAdd(&cnt[bucket_of(key, pp.np_log2, pp.bshift)], 1u);
                         npairs += nwin;
                       },
                       opt ? e2 : nullptr);
    ext[0] = e2[0] > ext[0] ? e2[0] : ext[0];
    ext[1] = e2[1] > ext[1] ? e2[1] : ext[1];
  }
  if (opt) {
    uint64_t mx = ext[0], mn = ext[1];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const uint64_t a = __shfl_xor(mx, o, 64), c = __shfl_xor(mn, o, 64);
      mx = a > mx ? a : mx;
      mn = c > mn ? c : mn;
    }
    if ((threadIdx.x & 63) == 0) {
      sext[0][threadIdx.x >> 6] = mx;
      sext[1][threadIdx.x >> 6] = mn;
    }
  }
  __syncthreads();
  if (opt && threadIdx.x == 0) {
    uint64_t mx = 0, mn = 0;
    for (int k = 0; k < kPNT / 64; ++k) {
      mx = sext[0][k] > mx ? sext[0][k] : mx;
      mn = sext[1][k] > mn ? sext[1][k] : mn;
    }
    // per-tile slots, reduced by k_part_decide (one contended device-scope
    // atomic per workgroup would serialise thousands of workgroups)
    pb.text[2 * tile] = mx;
    pb.text[2 * tile + 1] = mn;
  }
  // tile-major counts: one contiguous row per tile (k_part_colsum / colscan
  // turn them into bucket-major offsets)
  for (int i = threadIdx.x; i < nb; i += kPNT) pb.hist[tile * (uint64_t)nb + i] = cnt[i];
  late = wave_sum_u64(late);
  npairs = wave_sum_u64(npairs);
  if ((threadIdx.x & 63) == 0) {
    sred[threadIdx.x >> 6] = late;
    spairs[threadIdx.x >> 6] = npairs;
  }
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0 && pb.tpairs) {
    uint64_t tp = 0;
    for (int k = 0; k < kPNT / 64; ++k) tp += spairs[k];
    pb.tpairs[tile] = (uint32_t)tp;
  }
  if (threadIdx.x == 0) {
    uint64_t l = 0;
    for (int k = 0; k < kPNT / 64; ++k) l += sred[k];
    if (l) atomicAdd((unsigned long long *)&sc->late, (unsigned long long)l);
  }
}

// Optimistic histogram (no record late): only the window range decides whether
// a record is placed (as part_record with an unreachable stream time), plus
// the batch's ts extrema for k_part_decide. Fewer live registers than the
// general walk, so more workgroups per CU hide the HBM latency.
template <int T>
__global__ __launch_bounds__(kPNT) void k_part_hist_opt(Batch b, TwParams p, PartParams pp, PartBuffers pb,
                                                        DevScalars *sc) {
  __shared__ uint32_t cnt[1 << kPartMaxLog2];
  __shared__ uint64_t sext[2][kPNT / 64];
  __shared__ uint32_t spairs[kPNT / 64];
  constexpr int R = T / kPNT;
  const int nb = 1 << pp.np_log2;
  const uint64_t tile = xcd_tile(blockIdx.x, pp.tiles);  // offsets row
  const int64_t k_epoch = sc->k_epoch;
  for (int i = threadIdx.x; i < nb; i += kPNT) cnt[i] = 0;
  __syncthreads();
  uint64_t mx = 0, mn = 0;
  uint32_t npairs = 0;
  for (int st = 0; st < pp.sub; ++st) {
  const uint64_t base = (tile * pp.sub + st) * T;
  if (base >= b.n) break;  // uniform
  uint32_t key[R];
  int64_t ts[R];
  // the counts are per tile, so which thread reads which record of the tile is
  // free: full tiles of 16-byte aligned columns load 4 consecutive records per
  // thread (one 16-byte key load, two 16-byte ts loads)
  static_assert(R % 4 == 0, "4 records per vector load");
  const bool vec = base + T <= b.n && ((((uintptr_t)b.key) | ((uintptr_t)b.ts)) & 15) == 0;
  if (vec) {
#pragma unroll
    for (int q = 0; q < R / 4; ++q) {
      const uint64_t i0 = base + ((uint64_t)q * kPNT + threadIdx.x) * 4;
      const uint4 k4 = *reinterpret_cast<const uint4 *>(b.key + i0);
      const longlong2 t01 = *reinterpret_cast<const longlong2 *>(b.ts + i0);
      const longlong2 t23 = *reinterpret_cast<const longlong2 *>(b.ts + i0 + 2);
      key[4 * q + 0] = k4.x;
      key[4 * q + 1] = k4.y;
      key[4 * q + 2] = k4.z;
      key[4 * q + 3] = k4.w;
      ts[4 * q + 0] = t01.x;
      ts[4 * q + 1] = t01.y;
      ts[4 * q + 2] = t23.x;
      ts[4 * q + 3] = t23.y;
    }
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t i = base + (uint64_t)r * kPNT + threadIdx.x;
      const bool in = i < b.n;
      key[r] = in ? b.key[i] : HSG_KEY_NONE;
      ts[r] = in ? b.ts[i] : INT64_MIN;
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const uint64_t o = i64_ord(ts[r]);
    if (ts[r] != INT64_MIN || base + (uint64_t)r * kPNT + threadIdx.x < b.n) mx = o > mx ? o : mx;
    if (key[r] == HSG_KEY_NONE) continue;
    if (ts[r] >= 0) mn = ~o > mn ? ~o : mn;
    uint64_t k_lo, k_hi;
    if (!record_windows(p, ts[r], k_lo, k_hi)) continue;
    int64_t a = (int64_t)k_lo - k_epoch, z = (int64_t)k_hi - k_epoch;
    if (a < 0) a = 0;
    if (z > 0xFFFFFFFFll) z = 0xFFFFFFFFll;
    if (a > z) continue;
    atomicAdd(&cnt[bucket_of(key[r], pp.np_log2, pp.bshift)], 1u);
    npairs += (uint32_t)(z - a + 1);
  }
  }  // sub-tiles
  npairs = (uint32_t)wave_sum_u64(npairs);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t x = __shfl_xor(mx, o, 64), c = __shfl_xor(mn, o, 64);
    mx = x > mx ? x : mx;
    mn = c > mn ? c : mn;
  }
  if ((threadIdx.x & 63) == 0) {
    sext[0][threadIdx.x >> 6] = mx;
    sext[1][threadIdx.x >> 6] = mn;
    spairs[threadIdx.x >> 6] = npairs;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += kPNT) pb.hist[tile * (uint64_t)nb + i] = cnt[i];
  if (threadIdx.x == 0 && pb.tpairs) {
    uint32_t tp = 0;
    for (int k = 0; k < kPNT / 64; ++k) tp += spairs[k];
    pb.tpairs[tile] = tp;  // accepted pairs of the tile (no record late: every window of the range)
  }
  if (threadIdx.x == 0) {
    for (int k = 0; k < kPNT / 64; ++k) {
      mx = sext[0][k] > mx ? sext[0][k] : mx;
      mn = sext[1][k] > mn ? sext[1][k] : mn;
    }
    // per-tile slots, reduced by k_part_decide (one contended device-scope
    // atomic per workgroup would serialise thousands of workgroups)
    pb.text[2 * tile] = mx;
    pb.text[2 * tile + 1] = mn;
  }
}

// LDS holds only the tile's bucket sort (bucket, order, window run per record:
// 12 B) plus per-bucket run starts, so two workgroups fit a CU; the record
// words are gathered from the (L2-resident) input at write-out, in bucket
// order, so consecutive lanes write consecutive words of a run. (Storing each
// record straight from registers at its run slot instead measured slower, in
// this kernel and in the aggregation that reads its output.)
//
// Record layouts (sc->packed, decided per batch on the device):
//   wide   [key | krel << 32] [nwin | valid bits << 32] [col 0 .. C-1] [seq + 1]?
//   packed [key | (krel - kbase) << 32 | nwin << 48 | valid bits << 56] [cols] [seq + 1]?
template <int T, bool STABLE>
__global__ __launch_bounds__(kPNT) void k_part_scatter(Batch b, TwParams p, PartParams pp,
                                                       const int64_t *__restrict__ rec_wm,
                                                       const int64_t *__restrict__ own_wm,
                                                       const int64_t *__restrict__ seq, PartBuffers pb,
                                                       DevScalars *sc, int staged) {
  __shared__ uint8_t wcnt[STABLE ? kPW : 1][1 << kPartMaxLog2];
  __shared__ uint16_t lbk[T];
  __shared__ uint16_t sidx[T];
  __shared__ uint64_t lkn[T];  // krel | nwin << 32
  __shared__ uint32_t lstart[1 << kPartMaxLog2];
  __shared__ uint32_t cursor[1 << kPartMaxLog2];
  __shared__ uint32_t goff[1 << kPartMaxLog2];  // the row's next output slot per bucket
  __shared__ uint32_t swave[kPNT / 64];
  if (sc->redo) return;  // uniform: the optimistic pass found late records
  if (staged && sc->packed) return;  // uniform: k_part_scatter_st wrote this batch
  const int nb = 1 << pp.np_log2;
  const int C = pp.words - 2 - pp.has_seq;
  const bool packed = sc->packed != 0;
  const int W = packed ? pp.words - 1 : pp.words;
  const uint32_t kbase = (uint32_t)sc->kbase;
  const uint64_t row = xcd_tile(blockIdx.x, pp.tiles);
  const uint64_t q0 = phase_clock();
  for (int i = threadIdx.x; i < nb; i += kPNT) {
    cursor[i] = 0;
    goff[i] = pb.offt[row * (uint64_t)nb + i];
  }
  if constexpr (STABLE)
    for (int i = threadIdx.x; i < kPW * nb; i += kPNT) wcnt[i / nb][i % nb] = 0;
  const int per = (nb + kPNT - 1) / kPNT;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t late = 0;
  uint32_t err = 0;
  uint64_t q1 = q0, q2 = q0, q3 = q0;
  // the row's sub-tiles in order: a bucket's runs of consecutive sub-tiles
  // are adjacent in the output
  for (int st = 0; st < pp.sub; ++st) {
    const uint64_t tile = row * pp.sub + st;
    if (tile * T >= b.n) break;  // uniform
    for (int j = threadIdx.x; j < T; j += kPNT) lbk[j] = kNoBucket;
    __syncthreads();
    // 1) window runs and buckets of the sub-tile's records, bucket histogram
    walk_tile<T, kPNT>(b, p, tile, sc->k_epoch, pick_wm(rec_wm, own_wm, sc), late, err,
                       [&](int j, uint64_t, uint32_t key, uint32_t krel, uint32_t nwin) {
                         const uint32_t bk = bucket_of(key, pp.np_log2, pp.bshift);
                         lkn[j] = (uint64_t)krel | ((uint64_t)nwin << 32);
                         lbk[j] = (uint16_t)bk;
                         atomicAdd(&cursor[bk], 1u);
                       });
    __syncthreads();
    q1 = phase_clock();
    // 2) sub-tile-local exclusive scan of the histogram
    uint32_t loc = 0;
    for (int k = lo; k < hi; ++k) loc += cursor[k];
    uint32_t incl = loc;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      uint32_t u = __shfl_up(incl, o, 64);
      if (lane >= o) incl += u;
    }
    if (lane == 63) swave[wv] = incl;
    __syncthreads();
    uint32_t run = incl - loc;
    for (int k = 0; k < wv; ++k) run += swave[k];
    for (int k = lo; k < hi; ++k) {
      lstart[k] = run;
      run += cursor[k];
      cursor[k] = 0;
    }
    uint32_t placed = 0;
    for (int k = 0; k < kPNT / 64; ++k) placed += swave[k];
    __syncthreads();
    q2 = phase_clock();
    // 3) bucket-sorted order of the sub-tile's records (STABLE: in arrival
    // order inside each bucket's run)
    if constexpr (STABLE) {
      for (int j = threadIdx.x; j < T; j += kPNT) {  // uniform trip count (T % kPNT == 0)
        const uint16_t bk = lbk[j];
        const bool ok = bk != kNoBucket;
        uint64_t peers;
        const uint32_t rk = stable_round_rank(ok ? bk : 0u, ok, pp.np_log2, wcnt, peers);
        const uint32_t base_rk = ok ? cursor[bk] : 0u;
        lds_barrier();  // every rank read before the counts move
        if (ok) {
          sidx[lstart[bk] + base_rk + rk] = (uint16_t)j;
          if ((peers >> (threadIdx.x & 63)) == 1ull) atomicAdd(&cursor[bk], (uint32_t)__popcll(peers));
        }
        stable_round_done(ok ? bk : 0u, ok, peers, wcnt);
      }
    } else {
      for (int j = threadIdx.x; j < T; j += kPNT) {
        const uint16_t bk = lbk[j];
        if (bk == kNoBucket) continue;
        sidx[lstart[bk] + atomicAdd(&cursor[bk], 1u)] = (uint16_t)j;
      }
    }
    __syncthreads();
    q3 = phase_clock();
    // 4) coalesced write-out: consecutive lanes write consecutive words of a run
    const uint32_t inv = (1u << 20) / (uint32_t)W + 1;  // t / W for t < 2^16, W <= 16
    const uint32_t total = placed * (uint32_t)W;
    const uint64_t base = tile * T;
#pragma unroll 4
    for (uint32_t t = threadIdx.x; t < total; t += kPNT) {
      const uint32_t q = (uint32_t)(((uint64_t)t * inv) >> 20);
      const uint32_t w = t - q * (uint32_t)W;
      const uint16_t j = sidx[q];
      const uint16_t bk = lbk[j];
      const uint64_t i = base + j;
      const uint64_t dest = (uint64_t)goff[bk] + (q - lstart[bk]);
      uint64_t v;
      if (w == 0 && pb.pos) pb.pos[i] = (uint32_t)dest;
      const uint32_t wc = packed ? w + 1 : w;  // word index in the wide layout (packed: 0 is both headers)
      if (w == 0 && packed) {
        uint64_t vb = 0;
        for (int c = 0; c < C; ++c)
          if (!(pp.has_valid && b.valid[c] && !b.valid[c][i])) vb |= 1ull << c;
        const uint64_t kn = lkn[j];
        v = (uint64_t)b.key[i] | ((uint64_t)(((uint32_t)kn - kbase) & 0xFFFFu) << 32) | ((kn >> 32) << 48) | (vb << 56);
      } else if (w == 0) {
        v = (uint64_t)b.key[i] | (lkn[j] << 32);
      } else if (wc == 1) {
        uint64_t vb = 0;
        for (int c = 0; c < C; ++c)
          if (!(pp.has_valid && b.valid[c] && !b.valid[c][i])) vb |= 1ull << c;
        v = (lkn[j] >> 32) | (vb << 32);
      } else if ((int)wc < 2 + C) {
        v = (uint64_t)b.col[wc - 2][i];
      } else {
        v = seq_word(b, C, pp.has_valid, seq ? seq[i] : (int64_t)(p.rec_base + i), i);
      }
      pb.rec[dest * W + w] = v;
    }
    __syncthreads();
    // 5) the row's next slots: past this sub-tile's runs
    for (int k = lo; k < hi; ++k) {
      goff[k] += cursor[k];
      cursor[k] = 0;
    }
    __syncthreads();
  }
  late = wave_sum_u64(late);
  if (err) atomicOr(&sc->err, err);
  if (kPhaseClocks && threadIdx.x == 0) {
    const uint64_t q4 = phase_clock();
    atomicAdd((unsigned long long *)&sc->scratch[13], (unsigned long long)(q1 - q0));
    atomicAdd((unsigned long long *)&sc->scratch[14], (unsigned long long)(q2 - q1));
    atomicAdd((unsigned long long *)&sc->scratch[15], (unsigned long long)(q3 - q2));
    atomicAdd((unsigned long long *)&sc->scratch[16], (unsigned long long)(q4 - q3));
    atomicAdd((unsigned long long *)&sc->scratch[17], 1ull);
  }
}

void launch_part_hist(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp, const int64_t *rec_wm,
                      const int64_t *own_wm, const PartBuffers &pb, DevScalars *sc, bool opt) {
  if (!pp.tiles) return;
  if (opt) {
    hipLaunchKernelGGL(k_part_hist_opt<kPartTileRecs>, dim3((unsigned)pp.tiles), dim3(kPNT), 0, s, b, p, pp, pb, sc);
    return;
  }
  hipLaunchKernelGGL(k_part_hist<kPartTileRecs>, dim3((unsigned)pp.tiles), dim3(kPNT), 0, s, b, p, pp, rec_wm, own_wm,
                     pb, sc, 0);
}

// Optimistic path, after the histogram: stream time out, and whether the
// no-late assumption held (same test as k_tile_scan); if not, every later
// kernel of the batch exits and the host runs the batch again carefully.
// Also picks the packed record layout when every record's first window lies
// within 2^16 windows of the batch's earliest (kbase).
struct DecideArgs {
  TwParams p;
  int64_t wm_in, grace;
  int can_pack, on;
  const uint64_t *text;
  uint64_t tiles;
};

// 256 threads of one workgroup
__device__ inline void part_decide_body(DevScalars *sc, const TwParams &p, int64_t wm_in, int64_t grace, int can_pack,
                                        const uint64_t *__restrict__ text, uint64_t tiles) {
  __shared__ uint64_t sred[2][4];
  uint64_t tx = 0, tn = 0;
  for (uint64_t t = threadIdx.x; t < tiles; t += 256) {
    const uint64_t a = text[2 * t], c = text[2 * t + 1];
    tx = a > tx ? a : tx;
    tn = c > tn ? c : tn;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const uint64_t a = __shfl_xor(tx, o, 64), c = __shfl_xor(tn, o, 64);
    tx = a > tx ? a : tx;
    tn = c > tn ? c : tn;
  }
  if ((threadIdx.x & 63) == 0) {
    sred[0][threadIdx.x >> 6] = tx;
    sred[1][threadIdx.x >> 6] = tn;
  }
  __syncthreads();
  if (threadIdx.x != 0) return;
  // scratch[21/22] may already hold extrema from an exchange step; the batch's
  // tiles add theirs
  uint64_t mx = sc->scratch[21], mn = sc->scratch[22];
  for (int k = 0; k < 4; ++k) {
    mx = sred[0][k] > mx ? sred[0][k] : mx;
    mn = sred[1][k] > mn ? sred[1][k] : mn;
  }
  const int64_t bmax = mx ? (int64_t)(mx ^ 0x8000000000000000ull) : INT64_MIN;
  const int64_t amin = mn ? (int64_t)(~mn ^ 0x8000000000000000ull) : INT64_MAX;
  const int64_t all = bmax > wm_in ? bmax : wm_in;
  sc->wm_out = all;
  const bool ok = amin == INT64_MAX || amin > INT64_MAX - grace || all <= amin + grace;
  sc->no_late = ok ? 1u : 0u;
  sc->redo = ok ? 0u : 1u;
  uint64_t pk = 0, kb = 0;
  if (ok && can_pack && amin != INT64_MAX) {
    // no record is late: a record's first window is k_lo(ts), monotone in ts
    uint64_t lo0, hi0, lo1, hi1;
    if (record_windows(p, amin, lo0, hi0) && record_windows(p, bmax, lo1, hi1)) {
      const int64_t a = (int64_t)lo0 - sc->k_epoch;
      if (a >= 0 && hi1 >= lo0 && hi1 - lo0 < 0xFFFFull) {
        pk = 1;
        kb = (uint64_t)a;
      }
    }
  }
  sc->packed = pk;
  sc->kbase = kb;
}

__global__ __launch_bounds__(256) void k_part_decide(DevScalars *sc, DecideArgs a) {
  part_decide_body(sc, a.p, a.wm_in, a.grace, a.can_pack, a.text, a.tiles);
}

static DecideArgs decide_args(const TwParams &p, int64_t wm_in, int64_t grace, bool can_pack, const PartBuffers &pb,
                              uint64_t tiles) {
  DecideArgs a;
  memset(&a, 0, sizeof(a));
  a.p = p;
  a.wm_in = wm_in;
  a.grace = grace;
  a.can_pack = can_pack ? 1 : 0;
  a.on = 1;
  a.text = pb.text;
  a.tiles = tiles;
  return a;
}

void launch_part_decide(hipStream_t s, DevScalars *sc, const TwParams &p, int64_t wm_in, int64_t grace,
                        bool can_pack, const PartBuffers &pb, uint64_t tiles) {
  hipLaunchKernelGGL(k_part_decide, dim3(1), dim3(256), 0, s, sc, decide_args(p, wm_in, grace, can_pack, pb, tiles));
}

void launch_part_offsets(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc,
                         const DecideArgs *da);
void launch_part_offsets(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc) {
  launch_part_offsets(s, pp, pb, sc, nullptr);
}
void launch_part_decide_offsets(hipStream_t s, DevScalars *sc, const TwParams &p, int64_t wm_in, int64_t grace,
                                bool can_pack, const PartParams &pp, const PartBuffers &pb) {
  const DecideArgs a = decide_args(p, wm_in, grace, can_pack, pb, pp.tiles);
  launch_part_offsets(s, pp, pb, sc, &a);
}

// Staged scatter for packed records of <= 2 words (<= 1 column, no LAST), or
// 3 words (one column and the sequence word of LAST / literal-form ops): the
// walk reads every input column once, in arrival order; each record's packed
// words go to its bucket-sorted slot of an LDS copy of the tile, written out
// with consecutive lanes on consecutive records of a run (16-byte stores).
// The gather scatter above re-read ~0.35 GB per 2^24-record batch from L2
// misses (PMC) and waited on them. LDS: the tile (T x W words), two u16
// counters per u32, u16 run starts: 72 KiB at W = 2, two workgroups per CU.
// The bucket of a staged record is recomputed from its key at write-out.
template <int T, int W, bool STABLE, bool ONEWIN = false>
__global__ __launch_bounds__(kPNT) void k_part_scatter_st(Batch b, TwParams p, PartParams pp, PartBuffers pb,
                                                          const int64_t *__restrict__ seq, DevScalars *sc) {
  // STABLE: wave w's running count of bucket b over its rounds, then the
  // exclusive prefix of those counts over the waves
  // SEQ3: the SQL op shape's one-window records [header][value][sequence
  // word] staged as two words -- the header carries the record's tile-local
  // index in its window-count field (one window: rebuilt at write-out) and
  // the decimal bit, the sequence word is made at write-out -- so whole tiles
  // fit two workgroups per CU
  constexpr bool SEQ3 = W == 3 && ONEWIN;
  constexpr int SW = SEQ3 ? 2 : W;  // staged words per record
  __shared__ uint16_t wcnt[STABLE ? kPW : 1][1 << kPartMaxLog2];
  __shared__ uint64_t stage[T * SW];
  __shared__ uint32_t cnt2[1 << (kPartMaxLog2 - 1)];  // two u16 counts per word, then the u16 run starts
  __shared__ uint32_t cursor[1 << kPartMaxLog2];      // the row's next output slot per bucket
  __shared__ uint32_t swave[kPNT / 64];
  // W == 3: each staged record's output slot, so the write-out can go word by
  // word (consecutive lanes, consecutive 8-byte words of a run) instead of
  // three 8-byte stores 24 bytes apart per lane
  __shared__ uint32_t sdest[W == 3 && !SEQ3 ? T : 1];
  if (sc->redo || !sc->packed) return;  // uniform: the gather variant runs
  constexpr int R = T / kPNT;
  const int nb = 1 << pp.np_log2;
  const uint32_t kbase = (uint32_t)sc->kbase;
  const int64_t k_epoch = sc->k_epoch;
  const uint64_t row = xcd_tile(blockIdx.x, pp.tiles);
  const uint64_t q0 = phase_clock();
  uint16_t *lstart = reinterpret_cast<uint16_t *>(cnt2);
  for (int i = threadIdx.x; i < (nb + 1) / 2; i += kPNT) cnt2[i] = 0;
  for (int i = threadIdx.x; i < nb; i += kPNT) cursor[i] = pb.offt[row * (uint64_t)nb + i];
  if constexpr (STABLE)
    for (int i = threadIdx.x; i < kPW * nb; i += kPNT) wcnt[i / nb][i % nb] = 0;
  // buckets [lo, hi) of this thread: whole words of cnt2 (scan, run starts)
  const int per = (nb + kPNT - 1) / kPNT;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t late = 0, q1 = q0;
  uint32_t err = 0;
  // T may be a fraction of the partition tile (less LDS for the staging:
  // more workgroups per CU); the row's pieces are walked in arrival order.
  // The stable variant (per-record changelog, 2048 buckets) runs on half
  // tiles: 2 workgroups per CU, 0.36 -> 0.29 ms per C2 batch; the plain one
  // stays on whole tiles (half tiles: 186 -> 246 us, twice the bucket scans
  // and half-length runs per write-out)
  constexpr int SPT = kPartTileRecs / T;
  static_assert(SPT * T == kPartTileRecs, "staging piece");
  for (int st = 0; st < pp.sub * SPT; ++st) {
    const uint64_t base = (row * pp.sub * SPT + st) * T;
    if (base >= b.n) break;  // uniform
    uint32_t key[R];
    int64_t ts[R];
    uint64_t col[R];
    uint64_t sqw[W == 3 ? R : 1];  // W == 3: the sequence word (seq + 1 | literal bits << 56); SEQ3: the decimal bit
    // STABLE: each wave takes R*64 consecutive records (64 per round), so a
    // record's arrival rank needs no block barrier per round
    auto rec_i = [&](int r) -> uint64_t {
      return STABLE ? base + (uint64_t)wv * (R * 64) + (uint64_t)r * 64 + lane : base + (uint64_t)r * kPNT + threadIdx.x;
    };
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const uint64_t i = rec_i(r);
      const bool in = i < b.n;
      key[r] = in ? b.key[i] : HSG_KEY_NONE;
      ts[r] = in ? b.ts[i] : 0;
      col[r] = (W >= 2 && in) ? (uint64_t)b.col[0][i] : 0;
      if constexpr (SEQ3) sqw[r] = in && pp.has_valid && b.valid[0] && (b.valid[0][i] & 2u) ? 1u : 0u;
      else if constexpr (W == 3) sqw[r] = in ? seq_word(b, 1, pp.has_valid, seq ? seq[i] : (int64_t)(p.rec_base + i), i) : 0;
    }
    __syncthreads();  // counters clear
    uint32_t slot[R];  // bucket << 16 | slot in the sub-tile's run of the bucket, ~0 = no window
#pragma unroll
    for (int r = 0; r < R; ++r) {
      uint32_t krel = 0, nwin = 0;
      slot[r] = ~0u;
      const bool ok = part_record(p, k_epoch, key[r], ts[r], INT64_MIN, krel, nwin, late, err);
      const uint32_t bk = ok ? bucket_of(key[r], pp.np_log2, pp.bshift) : 0u;
      const uint32_t sh = (bk & 1u) * 16u;
      uint32_t pos;
      if constexpr (STABLE) {
        // rank within this wave: its earlier rounds + this round's lower lanes
        // (the wave's own LDS row, read before its leader writes it)
        const uint64_t peers = match_peers(bk, ok, pp.np_log2);
        const uint32_t prev = ok ? wcnt[wv][bk] : 0u;
        pos = prev + (uint32_t)__popcll(peers & ((1ull << lane) - 1ull));
        if (ok && (peers >> lane) == 1ull) wcnt[wv][bk] = (uint16_t)(prev + __popcll(peers));
        if (!ok) continue;
      } else {
        if (!ok) continue;
        pos = (atomicAdd(&cnt2[bk >> 1], 1u << sh) >> sh) & 0xFFFFu;
      }
      slot[r] = (bk << 16) | pos;
      const uint64_t i = rec_i(r);
      uint64_t vb = 0;
      if (W >= 2 && !(pp.has_valid && b.valid[0] && !b.valid[0][i])) vb = 1;
      if constexpr (SEQ3) {
        // (one window per record on this path: tumbling / unwindowed)
        if (nwin != 1) err |= ERR_RANGE;
        const uint64_t local = i - base;  // < T <= 4096: 12 bits
        ts[r] = (int64_t)((uint64_t)key[r] | ((uint64_t)((krel - kbase) & 0xFFFFu) << 32) | (local << 48) |
                          (vb << 60) | (sqw[r] << 61));
      } else {
        ts[r] = (int64_t)((uint64_t)key[r] | ((uint64_t)((krel - kbase) & 0xFFFFu) << 32) | ((uint64_t)nwin << 48) |
                          (vb << 56));  // the packed header word, kept in the ts register
      }
    }
    __syncthreads();
    // sub-tile-local exclusive scan of the bucket counts -> run starts (in place)
    uint32_t c[4] = {0, 0, 0, 0};  // per <= 4 (2048 buckets / 512 threads)
    uint32_t loc = 0;
    for (int k = lo; k < hi; ++k) {
      if constexpr (STABLE) {
        uint32_t run = 0;  // the waves' counts -> their exclusive prefix
        for (int w = 0; w < kPW; ++w) {
          const uint32_t x = wcnt[w][k];
          wcnt[w][k] = (uint16_t)run;
          run += x;
        }
        c[k - lo] = run;
      } else {
        c[k - lo] = (cnt2[k >> 1] >> ((k & 1) * 16)) & 0xFFFFu;
      }
      loc += c[k - lo];
    }
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
      lstart[k] = (uint16_t)run;
      run += c[k - lo];
    }
    uint32_t placed = 0;
    for (int k = 0; k < kPNT / 64; ++k) placed += swave[k];
    __syncthreads();
    // place the packed records at their bucket-sorted positions
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (slot[r] == ~0u) continue;
      const uint32_t sb = slot[r] >> 16;
      const uint32_t rk = (slot[r] & 0xFFFFu) + (STABLE ? (uint32_t)wcnt[wv][sb] : 0u);
      if (pb.pos) pb.pos[rec_i(r)] = cursor[sb] + rk;
      const uint32_t q = lstart[sb] + rk;
      stage[q * SW] = (uint64_t)ts[r];
      if (W >= 2) stage[q * SW + 1] = col[r];
      if constexpr (W == 3 && !SEQ3) stage[q * W + 2] = sqw[r];
    }
    __syncthreads();
    q1 = phase_clock();
    // write-out: record q goes to the row's slot for its bucket + (q - run start)
    if constexpr (SEQ3) {
      // word by word: the header rebuilt (one window, the present bit), the
      // value, the sequence word (seq + 1 | decimal bit << 56)
      for (uint32_t w = threadIdx.x; w < placed * 3; w += kPNT) {
        const uint32_t q = w / 3, j = w - 3 * q;
        const uint64_t h = stage[q * 2];
        const uint32_t bk = bucket_of((uint32_t)h, pp.np_log2, pp.bshift);
        const uint64_t dest = (uint64_t)cursor[bk] + (q - lstart[bk]);
        uint64_t v;
        if (j == 0) {
          v = (h & 0x0000FFFFFFFFFFFFull) | (1ull << 48) | (((h >> 60) & 1ull) << 56);
        } else if (j == 1) {
          v = stage[q * 2 + 1];
        } else {
          const uint64_t i = base + ((h >> 48) & 0xFFFull);
          v = ((uint64_t)((seq ? seq[i] : (int64_t)(p.rec_base + i)) + 1) & kSeqMask) | (((h >> 61) & 1ull) << 56);
        }
        pb.rec[dest * 3 + j] = v;
      }
    }
    if constexpr (W == 3 && !SEQ3) {
      for (uint32_t q = threadIdx.x; q < placed; q += kPNT) {
        const uint32_t bk = bucket_of((uint32_t)stage[q * W], pp.np_log2, pp.bshift);
        sdest[q] = cursor[bk] + (q - lstart[bk]);
      }
      lds_barrier();
      for (uint32_t w = threadIdx.x; w < placed * 3; w += kPNT) {
        const uint32_t q = w / 3, j = w - 3 * q;
        pb.rec[(uint64_t)sdest[q] * 3 + j] = stage[w];
      }
    }
    for (uint32_t q = threadIdx.x; W != 3 && q < placed; q += kPNT) {
      const uint64_t h = stage[q * W];
      const uint32_t bk = bucket_of((uint32_t)h, pp.np_log2, pp.bshift);
      const uint64_t dest = (uint64_t)cursor[bk] + (q - lstart[bk]);
      if (W == 2) {
        const uint64_t cc = stage[q * W + 1];
        *(ulonglong2 *)(pb.rec + dest * 2) = make_ulonglong2(h, cc);
      } else {
        pb.rec[dest] = h;
      }
    }
    __syncthreads();
    // the row's next slots, past this sub-tile's runs; counters cleared
    for (int k = lo; k < hi; ++k) cursor[k] += c[k - lo];
    for (int k = lo; k < hi; k += 2) cnt2[k >> 1] = 0;
    if constexpr (STABLE)
      for (int k = lo; k < hi; ++k)
        for (int w = 0; w < kPW; ++w) wcnt[w][k] = 0;
  }
  if (err) atomicOr(&sc->err, err);
  if (kPhaseClocks && threadIdx.x == 0) {
    const uint64_t q4 = phase_clock();
    atomicAdd((unsigned long long *)&sc->scratch[13], (unsigned long long)(q1 - q0));
    atomicAdd((unsigned long long *)&sc->scratch[16], (unsigned long long)(q4 - q1));
    atomicAdd((unsigned long long *)&sc->scratch[17], 1ull);
  }
}

void launch_part_scatter(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                         const int64_t *rec_wm, const int64_t *own_wm, const int64_t *seq, const PartBuffers &pb,
                         DevScalars *sc, bool maybe_packed, bool wide) {
  if (!pp.tiles) return;
  const dim3 g((unsigned)pp.tiles);
  // packed words <= 2, or 3 with the sequence word (one column)
  const bool stage = maybe_packed && ((!pp.has_seq && pp.words - 1 <= 2) || (pp.has_seq && pp.words - 1 == 3));
  // the per-record changelog (pb.pos) needs arrival order inside a bucket's runs
  const bool stable = pb.pos != nullptr;
  if (stage) {
    const dim3 th(kPNT);
    if (pp.words - 1 == 3) {
      // (the stable variant on half tiles: 48 KB of staging, two workgroups
      // per CU; the per-batch one stages two words per record -- SEQ3 -- and
      // takes whole tiles at two workgroups per CU; three staged words on
      // whole tiles, one workgroup per CU, measured 0.43 against 0.34 ms per
      // C2 SQL batch on half tiles)
      // (SEQ3 needs one window per record: tumbling / unwindowed ops)
      const bool onewin = p.kind == HSG_TUMBLING || p.kind == HSG_UNWINDOWED;
      if (stable && onewin)
        hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs / 2, 3, true, true>), g, th, 0, s, b, p, pp, pb, seq, sc);
      else if (stable)
        hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs / 2, 3, true>), g, th, 0, s, b, p, pp, pb, seq, sc);
      else if (onewin)
        hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs, 3, false, true>), g, th, 0, s, b, p, pp, pb, seq, sc);
      else
        hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs / 2, 3, false>), g, th, 0, s, b, p, pp, pb, seq, sc);
    } else if (pp.words - 1 == 2) {
      if (stable) hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs / 2, 2, true>), g, th, 0, s, b, p, pp, pb, seq, sc);
      else hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs, 2, false>), g, th, 0, s, b, p, pp, pb, seq, sc);
    } else {
      if (stable) hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs / 2, 1, true>), g, th, 0, s, b, p, pp, pb, seq, sc);
      else hipLaunchKernelGGL((k_part_scatter_st<kPartTileRecs, 1, false>), g, th, 0, s, b, p, pp, pb, seq, sc);
    }
  }
  if (wide || !stage) {
    if (stable)
      hipLaunchKernelGGL((k_part_scatter<kPartTileRecs, true>), g, dim3(kPNT), 0, s, b, p, pp, rec_wm, own_wm, seq, pb,
                         sc, stage ? 1 : 0);
    else
      hipLaunchKernelGGL((k_part_scatter<kPartTileRecs, false>), g, dim3(kPNT), 0, s, b, p, pp, rec_wm, own_wm, seq,
                         pb, sc, stage ? 1 : 0);
  }
}

// ---------------------------------------------------------------------------
// bucket-major offsets from the tile-major counts hist[tile][bucket]:
//   off(b, t) = sum_{b' < b} total(b') + sum_{t' < t} hist[t'][b]
// colsum: per (64-bucket block, segment of kColSeg tiles) column sums, stored
// bucket-major; a scan of those (nb x nseg entries) gives each segment's base;
// colscan: the running column prefix inside a segment, written tile-major
// (offt[t][b], what a scatter workgroup reads as one contiguous row), plus
// the bucket starts bstart[b] (bstart[nb] = records placed).
// ---------------------------------------------------------------------------
constexpr uint64_t kColSeg = 256;

uint32_t part_nseg(uint64_t tiles) { return (uint32_t)((tiles + kColSeg - 1) / kColSeg); }

// The extra column of workgroups (blockIdx.x == gridDim.x - 1) is the decide
// step of an optimistic batch (one launch fewer); the column sums do not
// depend on it (a batch found late is run again from the start).
__global__ __launch_bounds__(256) void k_part_colsum(const uint32_t *__restrict__ hist, uint64_t tiles, int nb,
                                                     uint32_t nseg, uint32_t *__restrict__ segsum, DevScalars *sc,
                                                     DecideArgs da) {
  __shared__ uint32_t red[4][64];
  if (blockIdx.x == gridDim.x - 1) {
    if (da.on && blockIdx.y == 0) part_decide_body(sc, da.p, da.wm_in, da.grace, da.can_pack, da.text, da.tiles);
    return;
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + lane;
  const uint64_t t0 = (uint64_t)blockIdx.y * kColSeg, t1 = t0 + kColSeg < tiles ? t0 + kColSeg : tiles;
  uint32_t sum = 0;
  if (b < nb) {
#pragma unroll 16
    for (uint64_t t = t0 + w; t < t1; t += 4) sum += hist[t * nb + b];
  }
  red[w][lane] = sum;
  __syncthreads();
  if (w == 0 && b < nb) segsum[(uint64_t)b * nseg + blockIdx.y] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

// FUSED (segment sums of at most kColFused entries): no separate scan -- a
// workgroup's base is the sum of the contiguous bucket-major prefix of the
// segment sums before its 64 buckets (<= 128 KiB of L2 reads), plus a wave
// scan of its buckets' totals and the bucket's own earlier segments; three
// launches fewer per batch.
constexpr uint64_t kColFused = 32768;
template <bool FUSED>
__global__ __launch_bounds__(256) void k_part_colscan(const uint32_t *__restrict__ hist, uint64_t tiles, int nb,
                                                      uint32_t nseg, const uint64_t *__restrict__ segoff,
                                                      const uint32_t *__restrict__ segsum,
                                                      uint32_t *__restrict__ offt, uint64_t *__restrict__ bstart,
                                                      const DevScalars *sc) {
  __shared__ uint32_t red[4][64];
  __shared__ uint64_t s_pre[4];
  if (sc->redo) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + lane;
  uint64_t base = 0;  // FUSED: segoff[b * nseg + blockIdx.y]
  if constexpr (FUSED) {
    // (16-byte loads, 16 per thread in flight at once: pre_n is a multiple of 64)
    constexpr int NQ = 16;
    const uint32_t n4 = (uint32_t)((uint64_t)blockIdx.x * 64 * nseg / 4);
    const uint4 *s4 = reinterpret_cast<const uint4 *>(segsum);
    uint64_t acc = 0;
    for (uint32_t i0 = 0; i0 < n4; i0 += NQ * 256) {
      uint4 qv[NQ];
#pragma unroll
      for (int k = 0; k < NQ; ++k) {
        const uint32_t i = i0 + threadIdx.x + (uint32_t)k * 256;
        qv[k] = i < n4 ? s4[i] : make_uint4(0, 0, 0, 0);
      }
#pragma unroll
      for (int k = 0; k < NQ; ++k) acc += (uint64_t)qv[k].x + qv[k].y + qv[k].z + qv[k].w;
    }
    acc = wave_incl_sum(acc);
    if (lane == 63) s_pre[w] = acc;
    uint64_t tot = 0, mine = 0;
    if (b < nb)
      for (uint32_t q = 0; q < nseg; ++q) {
        const uint32_t v = segsum[(uint64_t)b * nseg + q];
        tot += v;
        if (q < blockIdx.y) mine += v;
      }
    const uint64_t incl = wave_incl_sum(tot);
    __syncthreads();
    const uint64_t pre = s_pre[0] + s_pre[1] + s_pre[2] + s_pre[3];
    base = pre + (incl - tot) + mine;
    // records placed: the last bucket block's end
    if (blockIdx.x == gridDim.x - 1 && blockIdx.y == 0 && threadIdx.x == 63) bstart[nb] = pre + incl;
  }
  const uint64_t t0 = (uint64_t)blockIdx.y * kColSeg, t1 = t0 + kColSeg < tiles ? t0 + kColSeg : tiles;
  // each wave a quarter of the segment's tiles: their sum, then the running
  // prefix (the second read is served by L2); loads unrolled so that many
  // are in flight
  constexpr int PER = kColSeg / 4;
  const uint64_t r0 = t0 + (uint64_t)w * PER;
  const uint32_t *hp = hist + r0 * nb + b;
  const int cnt = r0 < t1 ? (int)(t1 - r0 < (uint64_t)PER ? t1 - r0 : PER) : 0;
  uint32_t sum = 0;
  if (b < nb) {
#pragma unroll 16
    for (int k = 0; k < cnt; ++k) sum += hp[(uint64_t)k * nb];
  }
  red[w][lane] = sum;
  __syncthreads();
  if (b >= nb) return;
  uint64_t run = FUSED ? base : segoff[(uint64_t)b * nseg + blockIdx.y];
  const uint64_t b0 = run;  // blockIdx.y == 0: the bucket's start
  for (int k = 0; k < w; ++k) run += red[k][lane];
  uint32_t *op = offt + r0 * nb + b;
#pragma unroll 16
  for (int k = 0; k < cnt; ++k) {
    op[(uint64_t)k * nb] = (uint32_t)run;
    run += hp[(uint64_t)k * nb];
  }
  if (blockIdx.y == 0 && w == 0) bstart[b] = b0;
}

void launch_part_offsets(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc,
                         const DecideArgs *da) {
  if (!pp.tiles) return;
  const int nb = 1 << pp.np_log2;
  const uint32_t nseg = part_nseg(pp.tiles);
  const dim3 g((unsigned)((nb + 63) / 64), nseg);
  DecideArgs off;
  memset(&off, 0, sizeof(off));
  hipLaunchKernelGGL(k_part_colsum, dim3(g.x + 1, g.y), dim3(256), 0, s, pb.hist, pp.tiles, nb, nseg, pb.segsum, sc,
                     da ? *da : off);
  if ((uint64_t)nb * nseg <= kColFused) {
    hipLaunchKernelGGL(k_part_colscan<true>, g, dim3(256), 0, s, pb.hist, pp.tiles, nb, nseg, nullptr, pb.segsum,
                       pb.offt, pb.bstart, sc);
    return;
  }
  scan_excl_u32(s, pb.segsum, pb.segoff, (uint64_t)nb * nseg, pb.partial, pb.bstart + nb);
  hipLaunchKernelGGL(k_part_colscan<false>, g, dim3(256), 0, s, pb.hist, pp.tiles, nb, nseg, pb.segoff, pb.segsum,
                     pb.offt, pb.bstart, sc);
}

// ---------------------------------------------------------------------------
// chunk map: chunk_start[b] = first aggregation workgroup of bucket b
// (a bucket of more than `chunk` records is split over several workgroups)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_part_chunks(const uint64_t *bstart, int np_log2, uint64_t chunk,
                                                      uint32_t *chunk_start, uint32_t *chunk_bucket,
                                                      const DevScalars *sc) {
  __shared__ uint32_t sw[16];
  // a batch found late (the optimistic decide) has no fresh bucket starts:
  // every aggregation kernel exits too
  if (sc->redo) return;
  const int nb = 1 << np_log2;
  const int per = (nb + 1023) / 1024;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint32_t loc = 0;
  for (int b = lo; b < hi; ++b) {
    const uint64_t sz = bstart[b + 1] > bstart[b] ? bstart[b + 1] - bstart[b] : 0;
    loc += (uint32_t)((sz + chunk - 1) / chunk);
  }
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t incl = loc;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    uint32_t u = __shfl_up(incl, o, 64);
    if (lane >= o) incl += u;
  }
  if (lane == 63) sw[w] = incl;
  __syncthreads();
  uint32_t run = incl - loc;
  for (int k = 0; k < w; ++k) run += sw[k];
  for (int b = lo; b < hi; ++b) {
    chunk_start[b] = run;
    const uint64_t sz = bstart[b + 1] > bstart[b] ? bstart[b + 1] - bstart[b] : 0;
    const uint32_t k = (uint32_t)((sz + chunk - 1) / chunk);
    for (uint32_t q = 0; q < k; ++q) chunk_bucket[run + q] = (uint32_t)b;
    run += k;
  }
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 16; ++k) t += sw[k];
    chunk_start[nb] = t;
  }
  // chunk_start[nb + 1]: some bucket is split over several workgroups
  uint32_t split = 0;
  for (int b = lo; b < hi; ++b) split |= bstart[b + 1] > bstart[b] + chunk;
  split = __syncthreads_or(split);
  if (threadIdx.x == 0) chunk_start[nb + 1] = split;
}

// ops with literal forms read bit 1 of the valid bytes, which the partition
// layouts do not carry: the generic record kernels run them
bool part_supported(const Program &prog) { return prog.n_slots <= 8 && !prog_has_forms(prog); }

void launch_part_chunks(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc) {
  hipLaunchKernelGGL(k_part_chunks, dim3(1), dim3(1024), 0, s, pb.bstart, pp.np_log2, pp.chunk, pb.chunk_start,
                     pb.chunk_bucket, sc);
}

// ---------------------------------------------------------------------------
// per-batch changelog: one row per first update of a group in the touched list
// (entries of later updates are kTouchSkip); counts, scan, compacted rows.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_touch_count(const uint32_t *__restrict__ touched, const DevScalars *sc,
                                                     uint64_t cap, uint32_t *__restrict__ cnt) {
  __shared__ uint64_t sw[4];
  uint64_t n = sc->scratch[6] ? sc->scratch[6] : sc->scratch[1];  // after k_seg_apply: [6]
  if (n > cap) n = cap;
  if (sc->scratch[32] & 4) n = 0;  // k_seg_apply held back: the chain runs again after it
  const uint64_t c0 = (uint64_t)blockIdx.x * kTouchChunk;
  uint64_t h = 0;
  if (c0 < n)
    for (uint64_t q = c0 + threadIdx.x; q < c0 + kTouchChunk && q < n; q += 256) h += touched[q] != kTouchSkip;
  h = wave_sum_u64(h);
  if ((threadIdx.x & 63) == 0) sw[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) cnt[blockIdx.x] = (uint32_t)(sw[0] + sw[1] + sw[2] + sw[3]);
}

__global__ __launch_bounds__(256) void k_touch_emit(TwTable t, Program prog, TwParams p, const uint32_t *touched,
                                                    uint64_t cap, const uint64_t *off, OutCols out, uint64_t out_base,
                                                    uint64_t out_cap, DevScalars *sc) {
  __shared__ uint64_t swave[4];
  uint64_t n = sc->scratch[6] ? sc->scratch[6] : sc->scratch[1];  // after k_seg_apply: [6]
  if (n > cap) n = cap;
  if (sc->scratch[32] & 4) return;  // uniform: k_seg_apply held back (k_touch_count)
  const uint64_t c0 = (uint64_t)blockIdx.x * kTouchChunk;
  if (c0 >= n) return;  // uniform
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int64_t k_epoch = sc->k_epoch;
  const bool unwin = p.kind == HSG_UNWINDOWED;
  uint64_t run = off[blockIdx.x];
  for (uint64_t blk = c0; blk < c0 + kTouchChunk && blk < n; blk += 256) {
    const uint64_t q = blk + threadIdx.x;
    const uint32_t s = q < n ? touched[q] : kTouchSkip;
    const bool hit = s != kTouchSkip;
    const uint64_t f = hit ? 1 : 0;
    const uint64_t incl = wave_incl_sum(f);
    if (lane == 63) swave[w] = incl;
    __syncthreads();
    uint64_t o = run + incl - f;
    for (int k = 0; k < w; ++k) o += swave[k];
    run += swave[0] + swave[1] + swave[2] + swave[3];
    __syncthreads();
    if (!hit) continue;
    o += out_base + sc->scratch[3];  // after the rows the lean apply wrote itself
    if (o >= out_cap) {
      atomicOr(&sc->err, ERR_OOM);
      continue;
    }
    const uint64_t g = *t.key(s);
    const int64_t *row = t.aggs(s);
    out.key[o] = (uint32_t)(g >> 32);
    int64_t ws = 0, we = 0;
    if (!unwin) {
      int64_t k = k_epoch + (int64_t)(g & 0xFFFFFFFFull);
      ws = (int64_t)((uint64_t)k * (uint64_t)p.adv);
      we = (int64_t)((uint64_t)ws + (uint64_t)p.size);
    }
    out.ws[o] = ws;
    out.we[o] = we;
    out.src[o] = -1;
    for (int j = 0; j < prog.n_out; ++j) out.agg[j][o] = out_value(prog, j, row);
    if (out.form) out.form[o] = out_form(prog, row);
  }
}

void launch_part_emit(hipStream_t s, const TwTable &t, const Program &prog, const TwParams &p, const PartBuffers &pb,
                      OutCols out, uint64_t out_base, uint64_t out_cap, DevScalars *sc) {
  const uint64_t nc = touch_chunks(pb.touched_cap);
  hipLaunchKernelGGL(k_touch_count, dim3((unsigned)nc), dim3(256), 0, s, pb.touched, sc, pb.touched_cap, pb.tcnt);
  scan_excl_u32(s, pb.tcnt, pb.toff, nc, pb.tpartial, &sc->out_rows);
  hipLaunchKernelGGL(k_touch_emit, dim3((unsigned)nc), dim3(256), 0, s, t, prog, p, pb.touched, pb.touched_cap,
                     pb.toff, out, out_base, out_cap, sc);
}

// per slot count: k_agg_s{2,4,6,8}.hip
void agg_launch_ms2(hipStream_t s, dim3 g, int W, bool maybe_packed, const Program &prog, const TwParams &p,
                    const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc);
void agg_launch_ms4(hipStream_t s, dim3 g, int W, bool maybe_packed, const Program &prog, const TwParams &p,
                    const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc);
void agg_launch_ms6(hipStream_t s, dim3 g, int W, bool maybe_packed, const Program &prog, const TwParams &p,
                    const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc);
void agg_launch_ms8(hipStream_t s, dim3 g, int W, bool maybe_packed, const Program &prog, const TwParams &p,
                    const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc);

uint64_t part_lds_entries(const Program &prog, bool big) {
  return prog.n_slots <= 2 ? (big ? 4096 : 2048) : (big ? 2048 : 1024);
}

bool launch_part_agg(hipStream_t s, const Program &prog, const TwParams &p, const PartParams &pp, const TwTable &t,
                     const PartBuffers &pb, uint64_t n, DevScalars *sc, bool maybe_packed, const OutCols *out,
                     uint64_t out_base, uint64_t out_cap, bool wide, bool *lean) {
  bool took_lean = false;
  if (lean) *lean = false;
  const uint64_t nb = 1ull << pp.np_log2;
  if (sql_lean_eligible(prog, pp)) {
    // the SQL op shape: its lean kernels only (a wide or refused batch runs on
    // the careful path, op_device.cpp push_time_atomic)
    if (!maybe_packed) return false;
    hipLaunchKernelGGL(k_part_chunks, dim3(1), dim3(1024), 0, s, pb.bstart, pp.np_log2, pp.chunk, pb.chunk_start,
                       pb.chunk_bucket, sc);
    const dim3 g((unsigned)(nb + n / pp.chunk + 1));
    launch_part_agg_sql(s, g, prog, p, pp, t, pb, sc, out, out_base, out_cap);
    if (lean) *lean = true;
    return true;
  }
  if (!part_supported(prog)) return false;
  hipLaunchKernelGGL(k_part_chunks, dim3(1), dim3(1024), 0, s, pb.bstart, pp.np_log2, pp.chunk, pb.chunk_start,
                     pb.chunk_bucket, sc);
  const dim3 g((unsigned)(nb + n / pp.chunk + 1));
  // packed one-window batches of the common slot programs: the lean kernels
  // (k_agg_lean.hip); the general kernel below then only covers the wide layout
  if (maybe_packed && launch_part_agg_lean(s, g, prog, p, pp, t, pb, sc, out, out_base, out_cap)) {
    maybe_packed = false;
    took_lean = true;
    if (lean) *lean = true;
    if (!wide) return true;  // predicted packed: the wide variant is not launched
  }
  const int W = pp.words;
  if (prog.n_slots <= 2) agg_launch_ms2(s, g, W, maybe_packed, prog, p, pp, t, pb, sc);
  else if (prog.n_slots <= 4) agg_launch_ms4(s, g, W, maybe_packed, prog, p, pp, t, pb, sc);
  else if (prog.n_slots <= 6) agg_launch_ms6(s, g, W, maybe_packed, prog, p, pp, t, pb, sc);
  else agg_launch_ms8(s, g, W, maybe_packed, prog, p, pp, t, pb, sc);
  if (pp.defer) launch_seg_apply(s, g, prog, p, pp, t, pb, sc, out, out_base, out_cap, took_lean);
  return true;
}

}  // namespace hsg
