// gfx950 kernels of the partitioned (key, window) aggregation:
//
//   hist     per-tile bucket counts of the records that have >= 1 accepted
//            window (bucket = top bits of hash(key): every window of a key
//            lands in one bucket)
//   scan     bucket-major exclusive prefix -> bucket ranges
//   scatter  each tile is bucket-sorted in LDS, then every bucket's run is
//            written by consecutive lanes as packed 8-byte-word records
//            [key|krel<<32][nwin|valid<<32][cols][seq+1]? (coalesced stores;
//            scattering 4-8 B fields per record directly ran at ~280 GB/s)
//   agg      one workgroup per <= kAggChunk records of a bucket: LDS hash table
//            of the chunk's groups fed by LDS atomics, then one flush per group
//            into the HBM table -- plain read-modify-write when the workgroup is
//            the bucket's only chunk (it owns those groups), atomics otherwise;
//            pairs that do not fit the LDS table go straight to HBM atomics.
//
// Window assignment and grace follow TimeWindowedStream.hs:86-103 / :105-117
// exactly as in k_window.hip (rejected windows are always the earliest ones, so
// the accepted windows of a record are one consecutive run).
#include "hsg_dev.h"
#include "hsg_part.h"
#include "hsg_sort.h"
#include "hsg_tw.h"

namespace hsg {

constexpr uint16_t kNoBucket = 0xFFFF;

__device__ inline uint32_t bucket_of(uint32_t key, int np_log2) {
  return np_log2 ? (uint32_t)(mix64((uint64_t)key * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull) >> (64 - np_log2))
                 : 0u;
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

// XCD-aware tile order: workgroups are dealt round-robin over the 8 XCDs, so
// give workgroups b, b+8, b+16, ... (one XCD) consecutive tiles; a bucket's
// runs from consecutive tiles are adjacent in the output. Speed only.
__device__ inline uint64_t xcd_tile(uint64_t blk, uint64_t tiles) {
  const uint64_t per = tiles / 8, full = per * 8;
  if (blk >= full) return blk;
  return (blk & 7) * per + (blk >> 3);
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

// Walk the T records of one partition tile with NT threads (record (r, t) =
// tile*T + r*NT + t); calls f(j, i, key, krel, nwin) for every record with
// >= 1 accepted window (j = tile-local index, i = batch index). No barriers.
// Order-preserving u64 image of an i64 (max of images = image of the max).
__device__ inline uint64_t i64_ord(int64_t v) { return (uint64_t)v ^ 0x8000000000000000ull; }

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

constexpr int kPNT = 512;  // threads of the partition passes

template <int T>
__global__ __launch_bounds__(kPNT) void k_part_hist(Batch b, TwParams p, PartParams pp,
                                                    const int64_t *__restrict__ rec_wm,
                                                    const int64_t *__restrict__ own_wm, PartBuffers pb,
                                                    DevScalars *sc, int opt) {
  __shared__ uint32_t cnt[1 << kPartMaxLog2];
  __shared__ uint64_t sred[kPNT / 64];
  __shared__ uint64_t sext[2][kPNT / 64];
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
  walk_tile<T, kPNT>(b, p, tile, sc->k_epoch, opt ? nullptr : pick_wm(rec_wm, own_wm, sc), late, err,
                     [&](int, uint64_t, uint32_t key, uint32_t, uint32_t) {
                       atomicAdd(&cnt[bucket_of(key, pp.np_log2)], 1u);
                     },
                     opt ? ext : nullptr);
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
    if (mx) atomicMax((unsigned long long *)&sc->scratch[21], (unsigned long long)mx);
    if (mn) atomicMax((unsigned long long *)&sc->scratch[22], (unsigned long long)mn);
  }
  // tile-major counts: one contiguous row per tile (k_part_colsum / colscan
  // turn them into bucket-major offsets)
  for (int i = threadIdx.x; i < nb; i += kPNT) pb.hist[tile * (uint64_t)nb + i] = cnt[i];
  late = wave_sum_u64(late);
  if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = late;
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t l = 0;
    for (int k = 0; k < kPNT / 64; ++k) l += sred[k];
    if (l) atomicAdd((unsigned long long *)&sc->late, (unsigned long long)l);
  }
}

// LDS holds only the tile's bucket sort (bucket, order, window run per record:
// 12 B) plus per-bucket run starts, so two workgroups fit a CU; the record
// words are gathered from the (L2-resident) input at write-out.
template <int T>
__global__ __launch_bounds__(kPNT) void k_part_scatter(Batch b, TwParams p, PartParams pp,
                                                       const int64_t *__restrict__ rec_wm,
                                                       const int64_t *__restrict__ own_wm,
                                                       const int64_t *__restrict__ seq, PartBuffers pb,
                                                       DevScalars *sc) {
  __shared__ uint16_t lbk[T];
  __shared__ uint16_t sidx[T];
  __shared__ uint64_t lkn[T];  // krel | nwin << 32
  __shared__ uint32_t lstart[1 << kPartMaxLog2];
  __shared__ uint32_t cursor[1 << kPartMaxLog2];
  __shared__ uint32_t goff[1 << kPartMaxLog2];
  __shared__ uint32_t swave[kPNT / 64];
  if (sc->redo) return;  // uniform: the optimistic pass found late records
  const int nb = 1 << pp.np_log2;
  const int W = pp.words;
  const int C = W - 2 - pp.has_seq;
  const uint64_t tile = xcd_tile(blockIdx.x, pp.tiles);
  const uint64_t q0 = wall_clock64();
  for (int i = threadIdx.x; i < nb; i += kPNT) cursor[i] = 0;
  for (int j = threadIdx.x; j < T; j += kPNT) lbk[j] = kNoBucket;
  __syncthreads();
  // 1) window runs and buckets of the tile's records, bucket histogram
  uint64_t late = 0;
  uint32_t err = 0;
  walk_tile<T, kPNT>(b, p, tile, sc->k_epoch, pick_wm(rec_wm, own_wm, sc), late, err,
                     [&](int j, uint64_t, uint32_t key, uint32_t krel, uint32_t nwin) {
                       const uint32_t bk = bucket_of(key, pp.np_log2);
                       lkn[j] = (uint64_t)krel | ((uint64_t)nwin << 32);
                       lbk[j] = (uint16_t)bk;
                       atomicAdd(&cursor[bk], 1u);
                     });
  __syncthreads();
  const uint64_t q1 = wall_clock64();
  // 2) tile-local exclusive scan of the histogram; global run starts
  const int per = (nb + kPNT - 1) / kPNT;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint32_t loc = 0;
  for (int k = lo; k < hi; ++k) loc += cursor[k];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
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
    goff[k] = pb.offt[tile * (uint64_t)nb + k];
  }
  uint32_t placed = 0;
  for (int k = 0; k < kPNT / 64; ++k) placed += swave[k];
  __syncthreads();
  const uint64_t q2 = wall_clock64();
  // 3) bucket-sorted order of the tile's records
  for (int j = threadIdx.x; j < T; j += kPNT) {
    const uint16_t bk = lbk[j];
    if (bk == kNoBucket) continue;
    sidx[lstart[bk] + atomicAdd(&cursor[bk], 1u)] = (uint16_t)j;
  }
  __syncthreads();
  const uint64_t q3 = wall_clock64();
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
    if (w == 0) {
      v = (uint64_t)b.key[i] | (lkn[j] << 32);
    } else if (w == 1) {
      uint64_t vb = 0;
      for (int c = 0; c < C; ++c)
        if (!(pp.has_valid && b.valid[c] && !b.valid[c][i])) vb |= 1ull << c;
      v = (lkn[j] >> 32) | (vb << 32);
    } else if ((int)w < 2 + C) {
      v = (uint64_t)b.col[w - 2][i];
    } else {
      v = (uint64_t)((seq ? seq[i] : (int64_t)(p.rec_base + i)) + 1);
    }
    pb.rec[dest * W + w] = v;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    const uint64_t q4 = wall_clock64();
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
  hipLaunchKernelGGL(k_part_hist<kPartTileRecs>, dim3((unsigned)pp.tiles), dim3(kPNT), 0, s, b, p, pp, rec_wm, own_wm,
                     pb, sc, opt ? 1 : 0);
}

// Optimistic path, after the histogram: stream time out, and whether the
// no-late assumption held (same test as k_tile_scan); if not, every later
// kernel of the batch exits and the host runs the batch again carefully.
__global__ void k_part_decide(DevScalars *sc, int64_t wm_in, int64_t grace) {
  if (threadIdx.x != 0) return;
  const uint64_t mx = sc->scratch[21], mn = sc->scratch[22];
  const int64_t bmax = mx ? (int64_t)(mx ^ 0x8000000000000000ull) : INT64_MIN;
  const int64_t amin = mn ? (int64_t)(~mn ^ 0x8000000000000000ull) : INT64_MAX;
  const int64_t all = bmax > wm_in ? bmax : wm_in;
  sc->wm_out = all;
  const bool ok = amin == INT64_MAX || amin > INT64_MAX - grace || all <= amin + grace;
  sc->no_late = ok ? 1u : 0u;
  sc->redo = ok ? 0u : 1u;
}

void launch_part_decide(hipStream_t s, DevScalars *sc, int64_t wm_in, int64_t grace) {
  hipLaunchKernelGGL(k_part_decide, dim3(1), dim3(64), 0, s, sc, wm_in, grace);
}

void launch_part_scatter(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                         const int64_t *rec_wm, const int64_t *own_wm, const int64_t *seq, const PartBuffers &pb,
                         DevScalars *sc) {
  if (!pp.tiles) return;
  hipLaunchKernelGGL(k_part_scatter<kPartTileRecs>, dim3((unsigned)pp.tiles), dim3(kPNT), 0, s, b, p, pp, rec_wm,
                     own_wm, seq, pb, sc);
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

__global__ __launch_bounds__(256) void k_part_colsum(const uint32_t *__restrict__ hist, uint64_t tiles, int nb,
                                                     uint32_t nseg, uint32_t *__restrict__ segsum, const DevScalars *sc) {
  __shared__ uint32_t red[4][64];
  if (sc->redo) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + lane;
  const uint64_t t0 = (uint64_t)blockIdx.y * kColSeg, t1 = t0 + kColSeg < tiles ? t0 + kColSeg : tiles;
  uint32_t sum = 0;
  if (b < nb)
    for (uint64_t t = t0 + w; t < t1; t += 4) sum += hist[t * nb + b];
  red[w][lane] = sum;
  __syncthreads();
  if (w == 0 && b < nb) segsum[(uint64_t)b * nseg + blockIdx.y] = red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane];
}

__global__ __launch_bounds__(256) void k_part_colscan(const uint32_t *__restrict__ hist, uint64_t tiles, int nb,
                                                      uint32_t nseg, const uint64_t *__restrict__ segoff,
                                                      uint32_t *__restrict__ offt, uint64_t *__restrict__ bstart,
                                                      const DevScalars *sc) {
  __shared__ uint32_t red[4][64];
  if (sc->redo) return;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int b = blockIdx.x * 64 + lane;
  const uint64_t t0 = (uint64_t)blockIdx.y * kColSeg, t1 = t0 + kColSeg < tiles ? t0 + kColSeg : tiles;
  const uint64_t per = (t1 - t0 + 3) / 4;
  const uint64_t r0 = t0 + w * per < t1 ? t0 + w * per : t1, r1 = r0 + per < t1 ? r0 + per : t1;
  uint32_t sum = 0;
  if (b < nb)
    for (uint64_t t = r0; t < r1; ++t) sum += hist[t * nb + b];
  red[w][lane] = sum;
  __syncthreads();
  if (b >= nb) return;
  uint64_t run = segoff[(uint64_t)b * nseg + blockIdx.y];
  for (int k = 0; k < w; ++k) run += red[k][lane];
  for (uint64_t t = r0; t < r1; ++t) {
    offt[t * nb + b] = (uint32_t)run;
    run += hist[t * nb + b];
  }
  if (blockIdx.y == 0 && w == 0) bstart[b] = segoff[(uint64_t)b * nseg];
}

void launch_part_offsets(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc) {
  if (!pp.tiles) return;
  const int nb = 1 << pp.np_log2;
  const uint32_t nseg = part_nseg(pp.tiles);
  const dim3 g((unsigned)((nb + 63) / 64), nseg);
  hipLaunchKernelGGL(k_part_colsum, g, dim3(256), 0, s, pb.hist, pp.tiles, nb, nseg, pb.segsum, sc);
  scan_excl_u32(s, pb.segsum, pb.segoff, (uint64_t)nb * nseg, pb.partial, pb.bstart + nb);
  hipLaunchKernelGGL(k_part_colscan, g, dim3(256), 0, s, pb.hist, pp.tiles, nb, nseg, pb.segoff, pb.offt, pb.bstart,
                     sc);
}

// ---------------------------------------------------------------------------
// chunk map: chunk_start[b] = first aggregation workgroup of bucket b
// (a bucket of more than `chunk` records is split over several workgroups)
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_part_chunks(const uint64_t *bstart, int np_log2, uint64_t chunk,
                                                      uint32_t *chunk_start, uint32_t *chunk_bucket) {
  __shared__ uint32_t sw[16];
  const int nb = 1 << np_log2;
  const int per = (nb + 1023) / 1024;
  const int lo = threadIdx.x * per, hi = lo + per < nb ? lo + per : nb;
  uint32_t loc = 0;
  for (int b = lo; b < hi; ++b) {
    uint64_t sz = bstart[b + 1] - bstart[b];
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
    uint64_t sz = bstart[b + 1] - bstart[b];
    const uint32_t k = (uint32_t)((sz + chunk - 1) / chunk);
    for (uint32_t q = 0; q < k; ++q) chunk_bucket[run + q] = (uint32_t)b;
    run += k;
  }
  if (threadIdx.x == 0) {
    uint32_t t = 0;
    for (int k = 0; k < 16; ++k) t += sw[k];
    chunk_start[nb] = t;
  }
}

// ---------------------------------------------------------------------------
// LDS aggregation of one chunk
// ---------------------------------------------------------------------------
// One partitioned record held in registers: [w0 w1 col 0..C-1 seq+1?]. Runtime
// word selection is an unrolled compare chain, so the record never leaves VGPRs.
template <int WMAX>
struct PRec {
  uint64_t w[WMAX];
  int C;
  __device__ bool present(int c) const { return (w[1] >> (32 + c)) & 1ull; }
  __device__ int64_t word(int k) const {
    int64_t v = 0;
#pragma unroll
    for (int q = 2; q < WMAX; ++q)
      if (q == k) v = (int64_t)w[q];
    return v;
  }
  __device__ int64_t col(int c) const { return word(2 + c); }
  __device__ int64_t seq1() const { return word(2 + C); }
};

// contribution of the record to slot s (identity when absent)
template <typename R>
__device__ inline int64_t prec_elem(const Program &prog, int s, const R &r) {
  const int op = prog.slot_op[s];
  const int c = prog.slot_col[s];
  if (op == S_CNT_ALL) return 1;
  if (op == S_LAST_VAL) return 0;
  if (!r.present(c)) return slot_identity_dev(op);
  switch (op) {
    case S_CNT: return 1;
    case S_SUM_I:
    case S_SUM_F:
    case S_MIN_I:
    case S_MAX_I: return r.col(c);
    case S_MIN_F:
    case S_MAX_F: return (int64_t)f64_ord(__builtin_bit_cast(double, r.col(c)));
    case S_LAST_SEQ: return r.seq1();
    default: return 0;
  }
}

template <int MS, typename R>
__device__ inline void lds_apply(const Program &prog, int64_t *__restrict__ row, const R &r) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
    if (op == S_LAST_VAL) continue;
    if (op != S_CNT_ALL && !r.present(prog.slot_col[s])) continue;
    const int64_t x = prec_elem(prog, s, r);
    unsigned long long *u = (unsigned long long *)(row + s);
    switch (op) {
      case S_CNT_ALL:
      case S_CNT:
      case S_SUM_I: atomicAdd(u, (unsigned long long)x); break;
      case S_SUM_F: unsafeAtomicAdd((double *)(row + s), __builtin_bit_cast(double, x)); break;
      case S_MIN_I: atomicMin((long long *)(row + s), (long long)x); break;
      case S_MAX_I: atomicMax((long long *)(row + s), (long long)x); break;
      case S_MIN_F: atomicMin(u, (unsigned long long)x); break;
      case S_MAX_F:
      case S_LAST_SEQ: atomicMax(u, (unsigned long long)x); break;
      default: break;
    }
  }
}

// a <- a (+) x over the aggregate slots (LAST_SEQ = latest sequence)
template <int MS>
__device__ inline void acc_combine(const Program &prog, int64_t (&a)[MS], const int64_t *x) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
    if (op == S_LAST_VAL) continue;
    a[s] = op == S_LAST_SEQ ? ((uint64_t)x[s] > (uint64_t)a[s] ? x[s] : a[s]) : slot_combine(op, a[s], x[s]);
  }
}

// HBM-side atomic combine of a row of partial aggregates (v) into `row`.
template <int MS>
__device__ inline void flush_row_atomic(const Program &prog, int64_t *__restrict__ row, const int64_t (&v)[MS]) {
#pragma unroll
  for (int s = 0; s < MS; ++s) {
    if (s >= prog.n_slots) break;
    const int op = prog.slot_op[s];
    const int64_t x = v[s];
    if (op == S_LAST_VAL || x == slot_identity_dev(op)) continue;  // nothing to add
    unsigned long long *u = (unsigned long long *)(row + s);
    switch (op) {
      case S_CNT_ALL:
      case S_CNT:
      case S_SUM_I: atomicAdd(u, (unsigned long long)x); break;
      case S_SUM_F: unsafeAtomicAdd((double *)(row + s), __builtin_bit_cast(double, x)); break;
      case S_MIN_I: atomicMin((long long *)(row + s), (long long)x); break;
      case S_MAX_I: atomicMax((long long *)(row + s), (long long)x); break;
      case S_MIN_F: atomicMin(u, (unsigned long long)x); break;
      case S_MAX_F:
      case S_LAST_SEQ: atomicMax(u, (unsigned long long)x); break;
      default: break;
    }
  }
}

constexpr uint32_t kTouchSkip = 0xFFFFFFFFu;

// One HBM update of group g with the chunk's partial aggregate v. `exclusive`:
// this workgroup is the only one updating the group in this launch, so a plain
// read-modify-write suffices (agent-scope loads, served by L2 not L1: this
// workgroup's own atomics may have updated the row). Returns the slot when this is the group's first update
// in the batch (-> per-batch changelog), else kTouchSkip.
template <int MS>
__device__ inline uint32_t flush_window(const Program &prog, const TwParams &p, const TwTable &t, uint64_t g,
                                        const int64_t (&v)[MS], bool exclusive, uint32_t &fresh, uint32_t &err) {
  const uint32_t f0 = fresh;
  const int64_t slot = tw_find_or_insert(t, g, fresh);
  if (slot < 0) {
    err |= ERR_OOM;
    return kTouchSkip;
  }
  int64_t *row = t.aggs(slot);
  uint32_t *stp = t.stamp(slot);
  const uint32_t bid = (uint32_t)p.batch_id;
  bool first;
  if (exclusive && fresh != f0) {
    // inserted just now by the group's only writer: the row holds identities
#pragma unroll
    for (int s = 0; s < MS; ++s)
      if (s < prog.n_slots && prog.slot_op[s] != S_LAST_VAL) row[s] = v[s];
    *stp = bid;
    first = true;
  } else if (exclusive) {
    int64_t cur[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s)
      cur[s] = s < prog.n_slots ? __hip_atomic_load(row + s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0;
    const uint32_t st = __hip_atomic_load(stp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#pragma unroll
    for (int s = 0; s < MS; ++s) {
      if (s >= prog.n_slots) break;
      const int op = prog.slot_op[s];
      if (op == S_LAST_VAL || v[s] == slot_identity_dev(op)) continue;
      row[s] = op == S_LAST_SEQ ? ((uint64_t)v[s] > (uint64_t)cur[s] ? v[s] : cur[s]) : slot_combine(op, cur[s], v[s]);
    }
    first = st != bid;
    if (first) *stp = bid;
  } else {
    flush_row_atomic<MS>(prog, row, v);
    first = atomicExch(stp, bid) != bid;
  }
  return first ? (uint32_t)slot : kTouchSkip;
}

__device__ inline void touch_append(const PartBuffers &pb, DevScalars *sc, uint32_t slot, uint32_t &err) {
  if (slot == kTouchSkip) return;
  const uint64_t o = atomicAdd((unsigned long long *)&sc->scratch[1], 1ull);
  if (o < pb.touched_cap) pb.touched[o] = slot;
  else err |= ERR_OOM;
}

// Windows [w0, w1] of one record straight into the HBM table (records whose
// earliest windows were rejected by grace, and LDS overflow in fan-out mode).
template <int MS, typename R>
__device__ inline void direct_windows(const Program &prog, const TwParams &p, const TwTable &t, const PartBuffers &pb,
                                      DevScalars *sc, uint32_t key, uint32_t w0, uint32_t w1, const R &r,
                                      uint32_t &fresh, uint32_t &err) {
  int64_t v[MS];
#pragma unroll
  for (int s = 0; s < MS; ++s) v[s] = s < prog.n_slots ? prec_elem(prog, s, r) : 0;
  for (uint32_t w = w0;; ++w) {
    touch_append(pb, sc, flush_window<MS>(prog, p, t, ((uint64_t)key << 32) | w, v, false, fresh, err), err);
    if (w == w1) break;
  }
}

// find or insert g; -1 when g is absent and the table is at its fill limit
template <int E>
__device__ inline int lds_insert(uint64_t *lkey, uint32_t *lfill, uint32_t limit, uint64_t g) {
  uint32_t h = (uint32_t)(mix64(g) & (E - 1));
  for (int probe = 0; probe < E; ++probe) {
    const uint64_t cur = lkey[h];
    if (cur == g) return (int)h;
    if (cur == kEmpty) {
      if (*(volatile uint32_t *)lfill >= limit) return -1;
      const uint64_t old = atomicCAS((unsigned long long *)&lkey[h], (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        atomicAdd(lfill, 1u);
        return (int)h;
      }
      if (old == g) return (int)h;
    }
    h = (h + 1) & (E - 1);
  }
  return -1;
}

// sub-round of a key: the hash bits just below its bucket bits
__device__ inline uint32_t key_round(uint32_t key, int np_log2, int rbits) {
  if (!rbits) return 0;
  const uint64_t h = mix64((uint64_t)key * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull);
  return (uint32_t)(h >> (64 - np_log2 - rbits)) & ((1u << rbits) - 1u);
}

// Aggregation of one chunk of a bucket (buckets are disjoint key sets, so when
// the bucket is one chunk this workgroup owns every group it updates).
//
// Pane mode (pp.pane_S = S >= 1, size = S * advance): a record of a full window
// run only updates its pane (key, last window P) in the LDS table. At a flush
// the live panes are sorted by (key, pane) in LDS; every pane P owns the
// windows [a, P] that contain no earlier pane in the table, and window
// w = combine(panes w .. w+S-1) gets one HBM update, with the panes summed
// incrementally from the sorted neighbours (w+1 adds the panes up to w+S).
// Tumbling is S = 1 (no sort). Fan-out mode (S = 0: size not a multiple of
// advance) keeps one entry per window.
//
// The chunk is walked in register-resident sub-chunks of NT * RPT records and
// the LDS table persists across them: it is flushed when full and at the end
// of each of the 2^rbits key-hash rounds (host-sized from the previous batch so
// that a round's panes fit), so a bucket's groups are normally flushed once.
template <int MS, int E, int NT>
struct AggLds {
  uint64_t key[E];
  int64_t agg[E * MS];
  uint8_t nw[E];     // windows of the pane's records
  uint8_t run[E];    // owned windows - 1
  uint16_t live[E];  // compacted / sorted live entries
  uint32_t fill, nl, b, c0, c1;
  uint32_t wsum[NT / 64];
  uint64_t base;
  uint64_t red[2][NT / 64];
};

// Flush every live entry of the table as window updates, then clear it.
// Block-wide: every thread calls. Returns the number of live entries.
template <int MS, int E, int NT>
__device__ __forceinline__ uint32_t agg_flush(AggLds<MS, E, NT> &L, const Program &prog, const TwParams &p, const TwTable &t,
                              const PartBuffers &pb, DevScalars *sc, int S, bool exclusive, uint32_t &fresh,
                              uint32_t &err, uint64_t &t_sort) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t SW = S ? (uint32_t)S : 1u;
  const uint64_t t0 = wall_clock64();
  // compact the live entries (one LDS atomic per wave)
  for (int e0 = 0; e0 < E; e0 += NT) {
    const int e = e0 + threadIdx.x;
    const bool on = L.key[e] != kEmpty;
    const uint64_t m = __ballot(on);
    uint32_t wb = 0;
    if (lane == 0 && m) wb = atomicAdd(&L.nl, (uint32_t)__popcll(m));
    wb = __shfl(wb, 0, 64);
    if (on) L.live[wb + (uint32_t)__popcll(m & ((1ull << lane) - 1ull))] = (uint16_t)e;
  }
  __syncthreads();
  const uint32_t nl = L.nl;
  if (S > 1 && nl > 1) {
    // panes of one key become neighbours: bitonic sort of the live list by
    // (key, pane), padded to a power of two with +inf
    uint32_t M = 1;
    while (M < nl) M <<= 1;
    for (uint32_t q = nl + threadIdx.x; q < M; q += NT) L.live[q] = 0xFFFFu;
    __syncthreads();
    for (uint32_t k = 2; k <= M; k <<= 1) {
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = threadIdx.x; i < M; i += NT) {
          const uint32_t ixj = i ^ j;
          if (ixj <= i) continue;
          const uint16_t x = L.live[i], y = L.live[ixj];
          const uint64_t kx = x == 0xFFFFu ? kEmpty : L.key[x];
          const uint64_t ky = y == 0xFFFFu ? kEmpty : L.key[y];
          if ((kx > ky) == ((i & k) == 0)) {
            L.live[i] = y;
            L.live[ixj] = x;
          }
        }
        __syncthreads();
      }
    }
  }
  t_sort += wall_clock64() - t0;
  // owned window run of every pane: [max(P - n + 1, previous pane + 1), P]
  uint32_t cnt = 0;
  for (uint32_t q = threadIdx.x; q < nl; q += NT) {
    const int e = L.live[q];
    const uint64_t g = L.key[e];
    const uint32_t P = (uint32_t)g;
    uint32_t a = P - (L.nw[e] - 1u);
    if (S > 1 && q > 0) {
      const uint64_t gp = L.key[L.live[q - 1]];
      if ((gp >> 32) == (g >> 32) && (uint32_t)gp + 1u > a) a = (uint32_t)gp + 1u;
    }
    L.run[e] = (uint8_t)(P - a);
    cnt += P - a + 1;
  }
  // block exclusive scan of the window counts -> changelog list positions
  const uint64_t incl = wave_incl_sum((uint64_t)cnt);
  if (lane == 63) L.wsum[wv] = (uint32_t)incl;
  __syncthreads();
  uint64_t o = incl - cnt, total = 0;
  for (int k = 0; k < NT / 64; ++k) {
    if (k < wv) o += L.wsum[k];
    total += L.wsum[k];
  }
  if (threadIdx.x == 0) L.base = total ? atomicAdd((unsigned long long *)&sc->scratch[1], (unsigned long long)total) : 0;
  __syncthreads();
  o += L.base;
  for (uint32_t q = threadIdx.x; q < nl; q += NT) {
    const int e = L.live[q];
    const uint64_t g = L.key[e];
    const uint64_t kb = g & 0xFFFFFFFF00000000ull;
    const uint32_t P = (uint32_t)g;
    const uint32_t a = P - L.run[e];
    int64_t acc[MS];
#pragma unroll
    for (int s = 0; s < MS; ++s) acc[s] = L.agg[e * MS + s];
    // later panes of the key (sorted after q) that window w covers: pane <= w + SW - 1
    uint32_t j = q + 1;
    uint64_t top = (uint64_t)a + SW - 1;
    for (uint32_t w = a;; ++w) {
      while (S > 1 && j < nl) {
        const int f = L.live[j];
        const uint64_t gj = L.key[f];
        if ((gj & 0xFFFFFFFF00000000ull) != kb || (uint64_t)(uint32_t)gj > top) break;
        acc_combine<MS>(prog, acc, &L.agg[f * MS]);
        ++j;
      }
      const uint32_t sl = flush_window<MS>(prog, p, t, kb | w, acc, exclusive, fresh, err);
      if (o < pb.touched_cap) pb.touched[o] = sl;
      else err |= ERR_OOM;
      ++o;
      if (w == P) break;
      ++top;
    }
  }
  __syncthreads();
  // clear the table
  for (uint32_t q = threadIdx.x; q < nl; q += NT) {
    const int e = L.live[q];
    L.key[e] = kEmpty;
#pragma unroll
    for (int s = 0; s < MS; ++s) L.agg[e * MS + s] = s < prog.n_slots ? slot_identity_dev(prog.slot_op[s]) : 0;
  }
  if (threadIdx.x == 0) {
    L.fill = 0;
    L.nl = 0;
  }
  __syncthreads();
  return nl;
}

template <int MS, int E, int WMAX, int RPT, int NT, bool FAN>
__global__ __launch_bounds__(NT, 1024 / NT) void k_part_agg(Program prog, TwParams p, PartParams pp, TwTable t,
                                                            PartBuffers pb, DevScalars *sc) {
  __shared__ AggLds<MS, E, NT> L;
  if (sc->redo) return;  // uniform: the optimistic pass found late records
  constexpr int SUB = NT * RPT;
  const int nb = 1 << pp.np_log2;
  const uint32_t *chunk_start = pb.chunk_start;
  const uint64_t t0 = wall_clock64();
  if (threadIdx.x == 0) {
    // this workgroup's bucket: chunk_start[b] <= blockIdx.x < chunk_start[b + 1]
    const uint32_t bk = blockIdx.x < chunk_start[nb] ? pb.chunk_bucket[blockIdx.x] : 0;
    L.b = bk;
    L.c0 = chunk_start[bk];
    L.c1 = chunk_start[bk + 1];
    L.fill = 0;
    L.nl = 0;
  }
  for (int e = threadIdx.x; e < E; e += NT) {
    L.key[e] = kEmpty;
#pragma unroll
    for (int s = 0; s < MS; ++s) L.agg[e * MS + s] = s < prog.n_slots ? slot_identity_dev(prog.slot_op[s]) : 0;
  }
  __syncthreads();
  if (blockIdx.x >= chunk_start[nb]) return;  // uniform: the grid is an upper bound
  const uint32_t b = L.b;
  const uint64_t b0 = pb.bstart[b], b1 = pb.bstart[b + 1];
  const uint64_t c = blockIdx.x - L.c0;
  const bool exclusive = (L.c1 - L.c0) == 1;
  const uint64_t r0 = b0 + c * pp.chunk, r1 = r0 + pp.chunk < b1 ? r0 + pp.chunk : b1;
  const uint32_t limit = (uint32_t)(E * 3 / 4);
  const int W = pp.words;
  const int C = W - 2 - pp.has_seq;
  const int S = pp.pane_S;
  const int nrounds = 1 << pp.rbits;
  const int64_t k_epoch = sc->k_epoch;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t pairs = 0, groups = 0, t_rec = 0, t_flush = 0, t_sort = 0, flushes = 0;
  uint32_t fresh = 0, err = 0;
  const uint64_t t1 = wall_clock64();

  for (int round = 0; round < nrounds; ++round) {
    for (uint64_t s0 = r0; s0 < r1; s0 += SUB) {
      uint64_t ta = wall_clock64();
      PRec<WMAX> rr[RPT];
      auto load = [&]() {
#pragma unroll
        for (int u = 0; u < RPT; ++u) {
          const uint64_t i = s0 + (uint64_t)u * NT + threadIdx.x;
          const bool in = i < r1;
          rr[u].C = C;
#pragma unroll
          for (int q = 0; q < WMAX; ++q) rr[u].w[q] = (in && q < W) ? pb.rec[i * W + q] : 0;
        }
      };
      load();
      uint32_t pend = 0;
#pragma unroll
      for (int u = 0; u < RPT; ++u) {
        const uint64_t i = s0 + (uint64_t)u * NT + threadIdx.x;
        if (i < r1 && (nrounds == 1 || key_round((uint32_t)rr[u].w[0], pp.np_log2, pp.rbits) == (uint32_t)round))
          pend |= 1u << u;
      }
      uint32_t dpend = 0;  // records for the direct HBM path
      for (;;) {
        // one instance of the record body (a rolled loop over a rotating register
        // queue, back in order after RPT steps): unrolling it overflowed the
        // instruction cache
#pragma unroll 1
        for (int u = 0; u < RPT; ++u) {
          const PRec<WMAX> r = rr[0];
#pragma unroll
          for (int k = 0; k + 1 < RPT; ++k) rr[k] = rr[k + 1];
          rr[RPT - 1] = r;
          if (!((pend >> u) & 1u)) continue;
          const uint32_t key = (uint32_t)r.w[0], krel = (uint32_t)(r.w[0] >> 32);
          const uint32_t nw = (uint32_t)r.w[1];
          if (FAN) {
            // fan-out: one entry per window, overflow straight to HBM
            pairs += nw;
            for (uint32_t j = 0; j < nw; ++j) {
              const uint64_t g = ((uint64_t)key << 32) | (uint64_t)(krel + j);
              const int e = lds_insert<E>(L.key, &L.fill, limit, g);
              if (e >= 0) {
                lds_apply<MS>(prog, &L.agg[e * MS], r);
                L.nw[e] = 1;
              } else {
                direct_windows<MS>(prog, p, t, pb, sc, key, krel + j, krel + j, r, fresh, err);
              }
            }
            pend &= ~(1u << u);
            continue;
          }
          if (nw == 0) {  // never written by the scatter (cannot happen; keep loops bounded)
            pend &= ~(1u << u);
            continue;
          }
          const uint32_t P = krel + nw - 1;
          const int64_t pabs = (int64_t)P + k_epoch;
          const uint32_t full = pabs + 1 < (int64_t)S ? (uint32_t)(pabs + 1) : (uint32_t)S;
          if (nw != full) {
            // some earliest windows were rejected by grace: not a whole pane;
            // straight to HBM after this loop
            dpend |= 1u << u;
            pend &= ~(1u << u);
            continue;
          }
          if (pp.exp == 2) { pairs += nw; pend &= ~(1u << u); continue; }
          const int e = lds_insert<E>(L.key, &L.fill, limit, ((uint64_t)key << 32) | P);
          if (e < 0) continue;  // table full: after the next flush
          pairs += nw;
          if (pp.exp != 1) lds_apply<MS>(prog, &L.agg[e * MS], r);
          L.nw[e] = (uint8_t)nw;
          pend &= ~(1u << u);
        }
        const bool more = __syncthreads_or(pend != 0);
        const uint64_t tb = wall_clock64();
        t_rec += tb - ta;
        if (!more) break;
        // table full with records left: flush and go on (the records are
        // loaded again afterwards, so they hold no registers across the flush)
        groups += agg_flush<MS, E, NT>(L, prog, p, t, pb, sc, S, exclusive, fresh, err, t_sort);
        ++flushes;
        load();
        ta = wall_clock64();
        t_flush += ta - tb;
      }
      if (!FAN && __syncthreads_or(dpend != 0)) {
        load();
#pragma unroll 1
        for (int u = 0; u < RPT; ++u) {
          const PRec<WMAX> r = rr[0];
#pragma unroll
          for (int k = 0; k + 1 < RPT; ++k) rr[k] = rr[k + 1];
          rr[RPT - 1] = r;
          if (!((dpend >> u) & 1u)) continue;
          const uint32_t key = (uint32_t)r.w[0], krel = (uint32_t)(r.w[0] >> 32);
          const uint32_t nw = (uint32_t)r.w[1];
          pairs += nw;
          direct_windows<MS>(prog, p, t, pb, sc, key, krel, krel + nw - 1, r, fresh, err);
        }
      }
    }
    const uint64_t tb = wall_clock64();
    groups += agg_flush<MS, E, NT>(L, prog, p, t, pb, sc, S, exclusive, fresh, err, t_sort);
    ++flushes;
    t_flush += wall_clock64() - tb;
  }
  const uint64_t t3 = wall_clock64();
  pairs = wave_sum_u64(pairs);
  const uint64_t fr = wave_sum_u64(fresh);
  if (lane == 0) {
    L.red[0][wv] = pairs;
    L.red[1][wv] = fr;
  }
  if (err) atomicOr(&sc->err, err);
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t a = 0, f = 0;
    for (int k = 0; k < NT / 64; ++k) {
      a += L.red[0][k];
      f += L.red[1][k];
    }
    if (a) atomicAdd((unsigned long long *)&sc->pairs, (unsigned long long)a);
    if (f) atomicAdd((unsigned long long *)&sc->live, (unsigned long long)f);
    if (groups) atomicAdd((unsigned long long *)&sc->scratch[0], (unsigned long long)groups);
    // phase clock (100 MHz wall clock) sums: init, records, flush, tail, workgroups
    const uint64_t t4 = wall_clock64();
    atomicAdd((unsigned long long *)&sc->scratch[8], (unsigned long long)(t1 - t0));
    atomicAdd((unsigned long long *)&sc->scratch[9], (unsigned long long)t_rec);
    atomicAdd((unsigned long long *)&sc->scratch[10], (unsigned long long)t_flush);
    atomicAdd((unsigned long long *)&sc->scratch[11], (unsigned long long)(t4 - t3));
    atomicAdd((unsigned long long *)&sc->scratch[12], 1ull);
    atomicAdd((unsigned long long *)&sc->scratch[18], (unsigned long long)t_sort);
    atomicAdd((unsigned long long *)&sc->scratch[19], 0ull);
    atomicAdd((unsigned long long *)&sc->scratch[20], (unsigned long long)flushes);
  }
}

bool part_supported(const Program &prog) { return prog.n_slots <= 8; }

// ---------------------------------------------------------------------------
// per-batch changelog: one row per first update of a group in the touched list
// (entries of later updates are kTouchSkip); counts, scan, compacted rows.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_touch_count(const uint32_t *__restrict__ touched, const DevScalars *sc,
                                                     uint64_t cap, uint32_t *__restrict__ cnt) {
  __shared__ uint64_t sw[4];
  uint64_t n = sc->scratch[1];
  if (n > cap) n = cap;
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
  uint64_t n = sc->scratch[1];
  if (n > cap) n = cap;
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
    o += out_base;
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

// Aggregation variants: small = E_s entries and 512 threads (two workgroups per
// CU), big = E_l entries and 1024 threads (one per CU). Records per thread
// keep the record queue within 128 VGPRs.
template <int MS, int E, int NT, int RPT4>
static void agg_launch_v(hipStream_t s, dim3 g, int W, const Program &prog, const TwParams &p, const PartParams &pp,
                         const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  const dim3 th(NT);
  constexpr int R6 = RPT4 / 2 > 0 ? RPT4 / 2 : 1, R11 = RPT4 / 4 > 0 ? RPT4 / 4 : 1;
  if (pp.pane_S == 0) {
    // fan-out (size not a multiple of advance): one generic-width variant
    hipLaunchKernelGGL((k_part_agg<MS, E, kPartMaxWords, R11, NT, true>), g, th, 0, s, prog, p, pp, t, pb, sc);
    return;
  }
  if (W <= 3) hipLaunchKernelGGL((k_part_agg<MS, E, 3, RPT4, NT, false>), g, th, 0, s, prog, p, pp, t, pb, sc);
  else if (W <= 4) hipLaunchKernelGGL((k_part_agg<MS, E, 4, RPT4, NT, false>), g, th, 0, s, prog, p, pp, t, pb, sc);
  else if (W <= 6) hipLaunchKernelGGL((k_part_agg<MS, E, 6, R6, NT, false>), g, th, 0, s, prog, p, pp, t, pb, sc);
  else hipLaunchKernelGGL((k_part_agg<MS, E, kPartMaxWords, R11, NT, false>), g, th, 0, s, prog, p, pp, t, pb, sc);
}

template <int MS>
static void agg_launch(hipStream_t s, dim3 g, int W, const Program &prog, const TwParams &p, const PartParams &pp,
                       const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  constexpr int ES = MS <= 2 ? 2048 : 1024, EL = MS <= 2 ? 4096 : 2048;
  if (pp.big) agg_launch_v<MS, EL, 1024, 8>(s, g, W, prog, p, pp, t, pb, sc);
  else agg_launch_v<MS, ES, 512, 4>(s, g, W, prog, p, pp, t, pb, sc);
}

uint64_t part_lds_entries(const Program &prog, bool big) {
  return prog.n_slots <= 2 ? (big ? 4096 : 2048) : (big ? 2048 : 1024);
}

bool launch_part_agg(hipStream_t s, const Program &prog, const TwParams &p, const PartParams &pp, const TwTable &t,
                     const PartBuffers &pb, uint64_t n, DevScalars *sc) {
  if (!part_supported(prog)) return false;
  const uint64_t nb = 1ull << pp.np_log2;
  hipLaunchKernelGGL(k_part_chunks, dim3(1), dim3(1024), 0, s, pb.bstart, pp.np_log2, pp.chunk, pb.chunk_start,
                     pb.chunk_bucket);
  const dim3 g((unsigned)(nb + n / pp.chunk + 1));
  const int W = pp.words;
  if (prog.n_slots <= 2) agg_launch<2>(s, g, W, prog, p, pp, t, pb, sc);
  else if (prog.n_slots <= 4) agg_launch<4>(s, g, W, prog, p, pp, t, pb, sc);
  else if (prog.n_slots <= 6) agg_launch<6>(s, g, W, prog, p, pp, t, pb, sc);
  else agg_launch<8>(s, g, W, prog, p, pp, t, pb, sc);
  return true;
}

}  // namespace hsg
