// Multi-GPU key exchange over RCCL (xGMI on an MI355X node).
//
// Every rank ingests its own slice of each global batch; slices are ordered by
// rank in the global arrival order. Per batch:
//   1. local: tile maxima of ts, owner = hash(key) mod G, stable partition
//   2. one ncclAllGather of [max ts, min ts, n, has_valid, counts[G]] per rank
//      -> global watermark, each rank's stream-time carry and sequence base,
//      the all-to-all-v sizes, and whether any record can be late at all
//   3. (only if some record can be late) per-record stream time in global order
//   4. pack -> ncclAllToAllv -> unpack: each rank now holds, in global arrival
//      order, every record whose key it owns
//   5. the single-GPU path aggregates them with their global sequence numbers
//      (and stream times), so results equal one GPU fed the whole batch.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "hsg_exchange.h"
#include "hsg_kernels.h"
#include "hsg_part.h"
#include "hsg_sort.h"

namespace hsg {

#define DTRY(expr)                                                          \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) {                                                 \
      err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;          \
    }                                                                       \
  } while (0)

#define NTRY(expr)                                                          \
  do {                                                                      \
    ncclResult_t _r = (expr);                                               \
    if (_r != ncclSuccess) {                                                \
      err = std::string(#expr) + ": " + ncclGetErrorString(_r);             \
      return HSG_E_COMM;                                                    \
    }                                                                       \
  } while (0)

// all-gathered facts per rank: [max ts, min keyed ts, n, has_valid,
// records for each owner [G], changelog room, changelog row clamp]
static int info_words(int G) { return 6 + G; }

// This rank's changelog room (rows free in the changelog buffer) and the
// clamp on the rows one batch can make here (per-batch time windows: the
// table's slots), queued into its info words for the all-gather: every rank
// then sees every rank's room and the records each one will own, and all of
// them refuse the batch together before the all-to-all when any rank's room
// is short (a rank that failed alone would leave its peers waiting in it).
static int publish_room(OpDevice &d, const hsg_op_config &cfg, const PushArgs &a, int G, std::string &err) {
  XBuffers &x = *d.x;
  uint64_t room = UINT64_MAX, clamp = UINT64_MAX;
  if (cfg.emit_mode != HSG_EMIT_NONE) {
    room = d.out_cap > a.pending ? d.out_cap - a.pending : 0;
    if (cfg.emit_mode == HSG_EMIT_PER_BATCH && cfg.window_kind != HSG_SESSION) clamp = d.cap;
  }
  x.h_room[0] = (int64_t)room;
  x.h_room[1] = (int64_t)clamp;
  // (pinned source: the push synchronises on the all-gather before the next
  // batch rewrites it)
  DTRY(hipMemcpyAsync(x.info + 4 + G, x.h_room, 16, hipMemcpyHostToDevice, d.stream));
  return HSG_OK;
}

// the uniform refusal (same H on every rank): some rank's owned records could
// write more changelog rows than its buffer has room for
static int check_room(const OpDevice &d, const int64_t *H, int G, std::string &err) {
  const int IW = info_words(G);
  for (int q = 0; q < G; ++q) {
    uint64_t ro = 0;
    for (int p = 0; p < G; ++p) ro += (uint64_t)H[(uint64_t)p * IW + 4 + q];
    uint64_t need = ro * d.wpr;
    const uint64_t clamp = (uint64_t)H[(uint64_t)q * IW + 5 + G], room = (uint64_t)H[(uint64_t)q * IW + 4 + G];
    if (need > clamp) need = clamp;
    if (need > room) {
      err = "changelog buffer full on rank " + std::to_string(q) + ": drain before pushing (out_capacity)";
      return HSG_E_CAPACITY;  // the batch is applied on no rank
    }
  }
  return HSG_OK;
}

static XLayout layout_for(const hsg_op_config &cfg, bool has_seq, bool has_wm, bool has_valid) {
  XLayout L;
  L.ncols = cfg.n_cols;
  L.has_seq = has_seq;
  L.has_wm = has_wm;
  L.has_valid = has_valid;
  L.words = 2 + cfg.n_cols + (has_seq ? 1 : 0) + (has_wm ? 1 : 0);
  return L;
}

int exchange_device_init(OpDevice &d, const hsg_op_config &cfg, uint64_t batch_cap, std::string &err) {
  XBuffers *x = new XBuffers();
  memset(x, 0, sizeof(*x));
  d.x = x;
  const int G = d.nranks;
  const uint64_t n = batch_cap;
  // packed records of the classic path (key, ts, columns, seq, wm), or the
  // columnar buffers of the fast / sequenced paths (+ valid bytes)
  const uint64_t max_words = 2 + cfg.n_cols + 3;
  x->batch = n;
  DTRY(hipMalloc((void **)&x->owner, n * 4 + 4));
  DTRY(hipMalloc((void **)&x->idx, n * 4 + 4));
  DTRY(hipMalloc((void **)&x->k1, n * 4 + 4));
  DTRY(hipMalloc((void **)&x->v1, n * 4 + 4));
  DTRY(hipMalloc(&x->sort_scratch, sort_scratch_bytes(n)));
  DTRY(hipMalloc((void **)&x->hist, (kMaxRanks + 1) * 8));
  DTRY(hipMalloc((void **)&x->info, info_words(G) * 8));
  DTRY(hipMalloc((void **)&x->info_all, (uint64_t)G * info_words(G) * 8));
  DTRY(hipHostMalloc((void **)&x->h_info, (uint64_t)G * info_words(G) * 8, hipHostMallocDefault));
  DTRY(hipHostMalloc((void **)&x->h_room, 16, hipHostMallocDefault));
  DTRY(hipMalloc((void **)&x->wm_local, n * 8 + 8));
  DTRY(hipMalloc((void **)&x->send, n * max_words * 8 + 65536));
  DTRY(hipMalloc((void **)&x->recv, (uint64_t)G * n * max_words * 8 + 65536));
  DTRY(hipMalloc((void **)&d.st_seq, (uint64_t)G * n * 8 + 8));
  DTRY(hipMalloc((void **)&d.st_wm, (uint64_t)G * n * 8 + 8));
  if (!d.h_tmp) DTRY(hipHostMalloc((void **)&d.h_tmp, 8 * sizeof(uint64_t), hipHostMallocDefault));
  // owner partition of the fast exchange: log2(ranks) for a power-of-two rank
  // count; the HSG_KNOB_XPART_LOG2 testing knob partitions a single rank
  // finer, every region still going to rank 0
  d.xpart_log2 = log2_exact((uint32_t)G);
  {
    const int64_t v = testing_knob(HSG_KNOB_XPART_LOG2);
    if (G == 1 && v >= 0 && v <= 6) d.xpart_log2 = (int)v;
  }
  d.x_classic = testing_knob(HSG_KNOB_X_CLASSIC) > 0;
  d.bshift = d.xpart_log2 > 0 ? d.xpart_log2 : 0;
  if (d.bshift + kPartMaxLog2 > 60) d.bshift = 0;
  d.tw.bshift = d.bshift;  // table regions follow the local buckets
  return HSG_OK;
}

void exchange_device_free(OpDevice &d) {
  XBuffers *x = d.x;
  if (!x) return;
  hipFree(x->owner);
  hipFree(x->idx);
  hipFree(x->k1);
  hipFree(x->v1);
  hipFree(x->sort_scratch);
  hipFree(x->hist);
  hipFree(x->info);
  hipFree(x->info_all);
  hipHostFree(x->h_info);
  hipHostFree(x->h_room);
  hipFree(x->wm_local);
  hipFree(x->send);
  hipFree(x->recv);
  delete x;
  d.x = nullptr;
}

// Fast path: no LAST / per-record changelog / sessions (record order and
// global sequence irrelevant) and, decided after the all-gather, no late
// record. Owner partition through the partition-offsets pipeline (owner = top
// key-hash bits), columnar send buffers, one all-to-all-v per column; the
// received columns are the owner's batch as they are (no unpack, no sort).
// `fallback` = some record may be late: the caller runs the classic path.
static int push_sharded_fast(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                             PushResult &r, std::string &err, bool &fallback) {
  XBuffers &x = *d.x;
  const int G = a.nranks, me = a.rank;
  const int IW = info_words(G);
  const int xl = d.xpart_log2;
  Comm *comm = a.comm;
  hipStream_t s = d.stream;
  fallback = false;
  if (a.batch->n > x.batch) {
    err = "batch larger than batch_capacity";
    return HSG_E_CAPACITY;
  }
  Batch kb;
  int rc = stage_batch(d, a.batch, kb, err, a.staged_set);
  if (rc != HSG_OK) return rc;
  bool has_valid = false;
  for (int c = 0; c < cfg.n_cols; ++c) has_valid = has_valid || kb.valid[c] != nullptr;
  const bool unwin = cfg.window_kind == HSG_UNWINDOWED;
  const uint64_t n = kb.n;
  DTRY(hipEventRecord(d.ev_c, s));
  rc = clear_batch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  // 1. owner counts per tile (+ ts extrema), owner-major run offsets, facts
  launch_x_hist(s, kb, xl, unwin, d.part.hist, d.part.text, d.sc);
  PartParams xp;
  memset(&xp, 0, sizeof(xp));
  xp.np_log2 = xl;
  xp.tiles = x_tiles(n);
  launch_part_offsets(s, xp, d.part, d.sc);
  launch_x_info(s, d.sc, d.part.bstart, xl, (uint32_t)G, n, has_valid, x.info, d.part.text, x_tiles(n));
  if ((rc = publish_room(d, cfg, a, G, err)) != HSG_OK) return rc;
  // 2. all-gather the per-rank facts
  rc = comm_allgather(comm, x.info, x.info_all, IW, ncclInt64, 8, s, err);
  if (rc != HSG_OK) return rc;
  DTRY(hipMemcpyAsync(x.h_info, x.info_all, (uint64_t)G * IW * 8, hipMemcpyDeviceToHost, s));
  if ((rc = poll_stream(d, s, err)) != HSG_OK) return rc;
  const int64_t *H = x.h_info;
  if ((rc = check_room(d, H, G, err)) != HSG_OK) return rc;
  int64_t wm_global = a.wm_in, carry = a.wm_in, min_ts = INT64_MAX;
  uint64_t total = 0;
  bool any_valid = false;
  for (int q = 0; q < G; ++q) {
    const int64_t *I = H + (uint64_t)q * IW;
    if (I[2] > 0) {
      wm_global = I[0] > wm_global ? I[0] : wm_global;
      if (q < me) carry = I[0] > carry ? I[0] : carry;
      min_ts = I[1] < min_ts ? I[1] : min_ts;
    }
    total += (uint64_t)I[2];
    any_valid = any_valid || I[3] != 0;
  }
  const bool time_win = cfg.window_kind == HSG_TUMBLING || cfg.window_kind == HSG_HOPPING;
  if (time_win && min_ts != INT64_MAX && wm_global > (int64_t)((uint64_t)min_ts + (uint64_t)cfg.grace_ms)) {
    fallback = true;  // some record may be late: per-record stream time in global order
    return HSG_OK;
  }
  // 3. columnar scatter by owner, one all-to-all-v per column
  std::vector<size_t> scount(G), sdispl(G), rcount(G), rdispl(G);
  uint64_t so = 0, ro = 0;
  for (int q = 0; q < G; ++q) {
    scount[q] = (size_t)H[(uint64_t)me * IW + 4 + q];
    sdispl[q] = so;
    so += scount[q];
    rcount[q] = (size_t)H[(uint64_t)q * IW + 4 + me];
    rdispl[q] = ro;
    ro += rcount[q];
  }
  if (ro > d.batch_cap) {
    err = "received more records than the op's capacity";
    return HSG_E_CAPACITY;
  }
  const int C = cfg.n_cols;
  auto carve = [&](void *base, uint64_t cap) {
    XCols c;
    memset(&c, 0, sizeof(c));
    char *p = (char *)base;
    auto take = [&](uint64_t bytes) {
      char *q = p;
      p += (bytes + 255) & ~255ull;
      return q;
    };
    c.ts = (int64_t *)take(cap * 8);
    for (int k = 0; k < C; ++k) c.col[k] = (int64_t *)take(cap * 8);
    c.key = (uint32_t *)take(cap * 4);
    for (int k = 0; k < C; ++k) c.valid[k] = (uint8_t *)take(cap);
    return c;
  };
  const XCols snd = carve(x.send, x.batch), rcv = carve(x.recv, (uint64_t)G * x.batch);
  launch_x_scatter(s, kb, xl, unwin, any_valid, C, d.part.offt, snd);
  // this rank's own records never cross the fabric: they are copied into
  // their place in the receive columns on the device (one rank: aggregated
  // from the send columns where they are, no copy), the others travel in
  // one all-to-all-v per column without the self block
  const size_t self_n = scount[me];
  scount[me] = 0;
  rcount[me] = 0;
  XCols src = rcv;
  if (G == 1) {
    src = snd;
  } else if (self_n) {
    const size_t so_me = sdispl[me], ro_me = rdispl[me];
    DTRY(hipMemcpyAsync(rcv.key + ro_me, snd.key + so_me, self_n * 4, hipMemcpyDeviceToDevice, s));
    DTRY(hipMemcpyAsync(rcv.ts + ro_me, snd.ts + so_me, self_n * 8, hipMemcpyDeviceToDevice, s));
    for (int k = 0; k < C; ++k) {
      DTRY(hipMemcpyAsync(rcv.col[k] + ro_me, snd.col[k] + so_me, self_n * 8, hipMemcpyDeviceToDevice, s));
      if (any_valid) DTRY(hipMemcpyAsync(rcv.valid[k] + ro_me, snd.valid[k] + so_me, self_n, hipMemcpyDeviceToDevice, s));
    }
  }
  if (G > 1) {
#define XA2A(buf, dt, el)                                                                              \
  do {                                                                                                  \
    rc = comm_alltoallv(comm, snd.buf, scount.data(), sdispl.data(), rcv.buf, rcount.data(), rdispl.data(), \
                        dt, el, s, err);                                                                \
    if (rc != HSG_OK) return rc;                                                                        \
  } while (0)
    if ((rc = comm_group_start(comm, err)) != HSG_OK) return rc;
    XA2A(key, ncclUint32, 4);
    XA2A(ts, ncclInt64, 8);
    for (int k = 0; k < C; ++k) {
      XA2A(col[k], ncclInt64, 8);
      if (any_valid) XA2A(valid[k], ncclUint8, 1);
    }
    if ((rc = comm_group_end(comm, err)) != HSG_OK) return rc;
#undef XA2A
  }
  DTRY(hipEventRecord(d.ev_d, s));
  DTRY(hipGetLastError());
  // 4. aggregate the owned records (order irrelevant for these ops)
  Batch rb;
  memset(&rb, 0, sizeof(rb));
  rb.n = ro;
  rb.key = src.key;
  rb.ts = src.ts;
  for (int k = 0; k < C; ++k) {
    rb.col[k] = src.col[k];
    rb.valid[k] = any_valid ? src.valid[k] : nullptr;
  }
  PushArgs la = a;
  la.wm_in = carry;  // any value <= the records' stream times keeps grace exact
  rc = push_local(d, cfg, prog, la, rb, nullptr, nullptr, r, err);
  float ms = 0;
  if (hipEventElapsedTime(&ms, d.ev_c, d.ev_d) == hipSuccess) r.exchange_ms = ms;
  r.exchange_bytes = (uint64_t)(so - self_n) * (12 + 8 * C + (any_valid ? C : 0));
  r.wm_out = wm_global;
  r.owned = ro;
  r.global_records = total;
  return rc;
}

static int push_sharded_classic(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                                PushResult &r, std::string &err);

static int push_sharded_seq(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                            PushResult &r, std::string &err);

int push_sharded(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, PushResult &r,
                 std::string &err) {
  bool need_seq = cfg.emit_mode == HSG_EMIT_PER_RECORD || cfg.window_kind == HSG_SESSION;
  need_seq = need_seq || prog_needs_seq(prog) || prog_has_forms(prog);
  if (d.use_part && d.xpart_log2 >= 0 && !need_seq) {
    bool fallback = false;
    int rc = push_sharded_fast(d, cfg, prog, a, r, err, fallback);
    if (rc != HSG_OK || !fallback) return rc;
  }
  // (HSG_KNOB_X_CLASSIC: the packed classic exchange even where the
  // sequenced columnar one applies; tests, A/B)
  if (d.xpart_log2 >= 0 && d.part_mem && !d.x_classic) return push_sharded_seq(d, cfg, prog, a, r, err);
  return push_sharded_classic(d, cfg, prog, a, r, err);
}

// Sequenced exchange (per-record changelog, LAST, sessions, literal forms,
// or a batch with late records; power-of-two ranks): the fast path's owner
// partition and columnar all-to-all-v, with a stable scatter (each owner's
// records in arrival order) that also sends every record's global sequence
// number and, when some record may be late, its stream time. Rank slices
// arrive in rank order, so the received columns are the owned records in
// global arrival order: the single-GPU kernels give the single-stream result.
// No radix sort, no packing, no unpack.
static int push_sharded_seq(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                            PushResult &r, std::string &err) {
  XBuffers &x = *d.x;
  const int G = a.nranks, me = a.rank;
  const int IW = info_words(G);
  // one owner region per rank (not the testing knob's finer partition of a
  // single rank): a rank's received columns are then its owned records in
  // global arrival order (rank slices in rank order, each kept stable)
  const int xl = log2_exact((uint32_t)G);
  Comm *comm = a.comm;
  hipStream_t s = d.stream;
  if (a.batch->n > x.batch) {
    err = "batch larger than batch_capacity";
    return HSG_E_CAPACITY;
  }
  Batch kb;
  int rc = stage_batch(d, a.batch, kb, err, a.staged_set);
  if (rc != HSG_OK) return rc;
  bool has_valid = false;
  for (int c = 0; c < cfg.n_cols; ++c) has_valid = has_valid || kb.valid[c] != nullptr;
  // records of every ts travel for sessions / unwindowed ops; for time
  // windows a record before 0 has no window (windowsFor) and only moves
  // stream time, which the all-gathered maxima carry
  const bool all_ts = cfg.window_kind == HSG_SESSION || cfg.window_kind == HSG_UNWINDOWED;
  const uint64_t n = kb.n;
  DTRY(hipEventRecord(d.ev_c, s));
  rc = clear_batch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  // 1. owner counts per tile (+ ts extrema), owner-major run offsets, facts
  launch_x_hist(s, kb, xl, all_ts, d.part.hist, d.part.text, d.sc);
  PartParams xp;
  memset(&xp, 0, sizeof(xp));
  xp.np_log2 = xl;
  xp.tiles = x_tiles(n);
  launch_part_offsets(s, xp, d.part, d.sc);
  launch_x_info(s, d.sc, d.part.bstart, xl, (uint32_t)G, n, has_valid, x.info, d.part.text, x_tiles(n));
  if ((rc = publish_room(d, cfg, a, G, err)) != HSG_OK) return rc;
  // 2. all-gather the per-rank facts
  rc = comm_allgather(comm, x.info, x.info_all, IW, ncclInt64, 8, s, err);
  if (rc != HSG_OK) return rc;
  DTRY(hipMemcpyAsync(x.h_info, x.info_all, (uint64_t)G * IW * 8, hipMemcpyDeviceToHost, s));
  if ((rc = poll_stream(d, s, err)) != HSG_OK) return rc;
  const int64_t *H = x.h_info;
  if ((rc = check_room(d, H, G, err)) != HSG_OK) return rc;
  int64_t wm_global = a.wm_in, carry = a.wm_in, min_ts = INT64_MAX;
  uint64_t seq_base = a.rec_base, total = 0;
  bool any_valid = false;
  for (int q = 0; q < G; ++q) {
    const int64_t *I = H + (uint64_t)q * IW;
    if (I[2] > 0) {
      wm_global = I[0] > wm_global ? I[0] : wm_global;
      if (q < me) carry = I[0] > carry ? I[0] : carry;
      min_ts = I[1] < min_ts ? I[1] : min_ts;
    }
    if (q < me) seq_base += (uint64_t)I[2];
    total += (uint64_t)I[2];
    any_valid = any_valid || I[3] != 0;
  }
  const bool time_win = cfg.window_kind == HSG_TUMBLING || cfg.window_kind == HSG_HOPPING;
  const bool may_be_late =
      time_win && min_ts != INT64_MAX && wm_global > (int64_t)((uint64_t)min_ts + (uint64_t)cfg.grace_ms);
  // per-record stream time in the global order (rare): tile maxima, their
  // prefix seeded with the lower ranks' maxima, the inclusive scan per tile
  if (may_be_late) {
    const uint64_t tiles = (n + kTileRecords - 1) / kTileRecords;
    launch_tile_stats(s, kb, d.tile_max, d.tile_min, tiles);
    launch_tile_scan(s, d.tile_max, d.tile_min, d.tile_prefix, tiles, carry, 1, false, d.sc);
    launch_x_recwm(s, kb, d.tile_prefix, x.wm_local);
  }
  // 3. stable columnar scatter by owner, one all-to-all-v per column
  std::vector<size_t> scount(G), sdispl(G), rcount(G), rdispl(G);
  uint64_t so = 0, ro = 0;
  for (int q = 0; q < G; ++q) {
    scount[q] = (size_t)H[(uint64_t)me * IW + 4 + q];
    sdispl[q] = so;
    so += scount[q];
    rcount[q] = (size_t)H[(uint64_t)q * IW + 4 + me];
    rdispl[q] = ro;
    ro += rcount[q];
  }
  if (ro > d.batch_cap) {
    err = "received more records than the op's capacity";
    return HSG_E_CAPACITY;
  }
  const int C = cfg.n_cols;
  auto carve = [&](void *base, uint64_t cap) {
    XCols c;
    memset(&c, 0, sizeof(c));
    char *p = (char *)base;
    auto take = [&](uint64_t bytes) {
      char *q = p;
      p += (bytes + 255) & ~255ull;
      return q;
    };
    c.ts = (int64_t *)take(cap * 8);
    for (int k = 0; k < C; ++k) c.col[k] = (int64_t *)take(cap * 8);
    c.seq = (int64_t *)take(cap * 8);
    c.wm = (int64_t *)take(cap * 8);
    c.key = (uint32_t *)take(cap * 4);
    for (int k = 0; k < C; ++k) c.valid[k] = (uint8_t *)take(cap);
    return c;
  };
  const XCols snd = carve(x.send, x.batch), rcv = carve(x.recv, (uint64_t)G * x.batch);
  launch_x_scatter_seq(s, kb, xl, all_ts, any_valid, C, d.part.offt, snd, seq_base,
                       may_be_late ? x.wm_local : nullptr);
  const size_t self_n = scount[me];
  scount[me] = 0;
  rcount[me] = 0;
  XCols src = rcv;
  if (G == 1) {
    src = snd;
  } else if (self_n) {
    const size_t so_me = sdispl[me], ro_me = rdispl[me];
    DTRY(hipMemcpyAsync(rcv.key + ro_me, snd.key + so_me, self_n * 4, hipMemcpyDeviceToDevice, s));
    DTRY(hipMemcpyAsync(rcv.ts + ro_me, snd.ts + so_me, self_n * 8, hipMemcpyDeviceToDevice, s));
    DTRY(hipMemcpyAsync(rcv.seq + ro_me, snd.seq + so_me, self_n * 8, hipMemcpyDeviceToDevice, s));
    if (may_be_late) DTRY(hipMemcpyAsync(rcv.wm + ro_me, snd.wm + so_me, self_n * 8, hipMemcpyDeviceToDevice, s));
    for (int k = 0; k < C; ++k) {
      DTRY(hipMemcpyAsync(rcv.col[k] + ro_me, snd.col[k] + so_me, self_n * 8, hipMemcpyDeviceToDevice, s));
      if (any_valid) DTRY(hipMemcpyAsync(rcv.valid[k] + ro_me, snd.valid[k] + so_me, self_n, hipMemcpyDeviceToDevice, s));
    }
  }
  if (G > 1) {
#define XA2A(buf, dt, el)                                                                              \
  do {                                                                                                  \
    rc = comm_alltoallv(comm, snd.buf, scount.data(), sdispl.data(), rcv.buf, rcount.data(), rdispl.data(), \
                        dt, el, s, err);                                                                \
    if (rc != HSG_OK) return rc;                                                                        \
  } while (0)
    if ((rc = comm_group_start(comm, err)) != HSG_OK) return rc;
    XA2A(key, ncclUint32, 4);
    XA2A(ts, ncclInt64, 8);
    XA2A(seq, ncclInt64, 8);
    if (may_be_late) XA2A(wm, ncclInt64, 8);
    for (int k = 0; k < C; ++k) {
      XA2A(col[k], ncclInt64, 8);
      if (any_valid) XA2A(valid[k], ncclUint8, 1);
    }
    if ((rc = comm_group_end(comm, err)) != HSG_OK) return rc;
#undef XA2A
  }
  DTRY(hipEventRecord(d.ev_d, s));
  DTRY(hipGetLastError());
  // 4. aggregate the owned records, in global arrival order
  Batch rb;
  memset(&rb, 0, sizeof(rb));
  rb.n = ro;
  rb.key = src.key;
  rb.ts = src.ts;
  for (int k = 0; k < C; ++k) {
    rb.col[k] = src.col[k];
    rb.valid[k] = any_valid ? src.valid[k] : nullptr;
  }
  PushArgs la = a;
  la.wm_in = carry;  // any value <= the records' stream times keeps grace exact
  rc = push_local(d, cfg, prog, la, rb, src.seq, may_be_late ? src.wm : nullptr, r, err);
  float ms = 0;
  if (hipEventElapsedTime(&ms, d.ev_c, d.ev_d) == hipSuccess) r.exchange_ms = ms;
  r.exchange_bytes = (uint64_t)(so - self_n) * (20 + 8 * C + (any_valid ? C : 0) + (may_be_late ? 8 : 0));
  r.wm_out = wm_global;
  r.owned = ro;
  r.global_records = total;
  return rc;
}

static int push_sharded_classic(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                                PushResult &r, std::string &err) {
  XBuffers &x = *d.x;
  const int G = a.nranks, me = a.rank;
  const int IW = info_words(G);
  Comm *comm = a.comm;
  hipStream_t s = d.stream;
  if (a.batch->n > x.batch) {
    err = "batch larger than batch_capacity";
    return HSG_E_CAPACITY;
  }
  // 1. stage this rank's slice and compute local facts
  Batch kb;
  int rc = stage_batch(d, a.batch, kb, err, a.staged_set);
  if (rc != HSG_OK) return rc;
  bool has_valid = false;
  for (int c = 0; c < cfg.n_cols; ++c) has_valid = has_valid || kb.valid[c] != nullptr;
  const uint64_t n = kb.n;
  const uint64_t tiles = (n + kTileRecords - 1) / kTileRecords;
  DTRY(hipEventRecord(d.ev_c, s));
  launch_tile_stats(s, kb, d.tile_max, d.tile_min, tiles);
  launch_x_minmax(s, d.tile_max, d.tile_min, tiles, n, has_valid ? 1 : 0, x.info);
  DTRY(hipMemsetAsync(x.hist, 0, (kMaxRanks + 1) * 8, s));
  launch_x_owner(s, kb, (uint32_t)G, x.owner, x.idx, x.hist);
  DTRY(hipMemcpyAsync(x.info + 4, x.hist, (uint64_t)G * 8, hipMemcpyDeviceToDevice, s));
  if ((rc = publish_room(d, cfg, a, G, err)) != HSG_OK) return rc;
  // stable partition by owner: one 8-bit radix pass of (owner, record index)
  int which = radix_sort_pairs(s, x.owner, x.idx, x.k1, x.v1, n, 8, x.sort_scratch);
  const uint32_t *sidx = which ? x.v1 : x.idx;
  // 2. all-gather the per-rank facts
  rc = comm_allgather(comm, x.info, x.info_all, IW, ncclInt64, 8, s, err);
  if (rc != HSG_OK) return rc;
  DTRY(hipMemcpyAsync(x.h_info, x.info_all, (uint64_t)G * IW * 8, hipMemcpyDeviceToHost, s));
  if ((rc = poll_stream(d, s, err)) != HSG_OK) return rc;
  const int64_t *H = x.h_info;
  if ((rc = check_room(d, H, G, err)) != HSG_OK) return rc;
  int64_t wm_global = a.wm_in, carry = a.wm_in, min_ts = INT64_MAX;
  uint64_t seq_base = a.rec_base, total = 0;
  bool any_valid = false;
  for (int q = 0; q < G; ++q) {
    const int64_t *I = H + (uint64_t)q * IW;
    if (I[2] > 0) {
      wm_global = I[0] > wm_global ? I[0] : wm_global;
      if (q < me) carry = I[0] > carry ? I[0] : carry;
      min_ts = I[1] < min_ts ? I[1] : min_ts;
    }
    if (q < me) seq_base += (uint64_t)I[2];
    total += (uint64_t)I[2];
    any_valid = any_valid || I[3] != 0;
  }
  // can any (record, window) be rejected by grace? every window of a record at
  // ts t ends after t, so none is when stream time never exceeds t + grace
  const bool time_win = cfg.window_kind == HSG_TUMBLING || cfg.window_kind == HSG_HOPPING;
  const bool may_be_late =
      time_win && min_ts != INT64_MAX && wm_global > (int64_t)((uint64_t)min_ts + (uint64_t)cfg.grace_ms);
  const bool need_seq = cfg.emit_mode == HSG_EMIT_PER_RECORD || cfg.window_kind == HSG_SESSION || prog_needs_seq(prog);
  XLayout L = layout_for(cfg, need_seq, may_be_late, any_valid);
  // 3. per-record stream time in the global order (rare)
  if (may_be_late) {
    launch_tile_scan(s, d.tile_max, d.tile_min, d.tile_prefix, tiles, carry, 1, false, d.sc);
    launch_x_recwm(s, kb, d.tile_prefix, x.wm_local);
  }
  // 4. exchange
  std::vector<size_t> scount(G), sdispl(G), rcount(G), rdispl(G);
  uint64_t so = 0, ro = 0;
  for (int q = 0; q < G; ++q) {
    scount[q] = (size_t)H[(uint64_t)me * IW + 4 + q] * L.words;
    sdispl[q] = so;
    so += scount[q];
    rcount[q] = (size_t)H[(uint64_t)q * IW + 4 + me] * L.words;
    rdispl[q] = ro;
    ro += rcount[q];
  }
  const uint64_t m_send = so / L.words, m_recv = ro / L.words;
  if (m_recv > d.batch_cap) {
    err = "received more records than the op's capacity";
    return HSG_E_CAPACITY;
  }
  launch_x_pack(s, kb, L, sidx, m_send, seq_base, x.wm_local, x.send);
  rc = comm_alltoallv(comm, x.send, scount.data(), sdispl.data(), x.recv, rcount.data(), rdispl.data(), ncclUint64, 8,
                      s, err);
  if (rc != HSG_OK) return rc;
  XStaging st;
  memset(&st, 0, sizeof(st));
  // received records reuse the op's staging arrays (the local slice is packed already)
  st.key = d.st_key;
  st.ts = d.st_ts;
  for (int c = 0; c < cfg.n_cols; ++c) {
    st.col[c] = d.st_col[c];
    st.valid[c] = d.st_valid[c];
  }
  st.seq = d.st_seq;
  st.wm = d.st_wm;
  launch_x_unpack(s, L, x.recv, m_recv, st);
  DTRY(hipEventRecord(d.ev_d, s));
  DTRY(hipGetLastError());
  // 5. aggregate the owned records
  Batch rb;
  memset(&rb, 0, sizeof(rb));
  rb.n = m_recv;
  rb.key = d.st_key;
  rb.ts = d.st_ts;
  for (int c = 0; c < cfg.n_cols; ++c) {
    rb.col[c] = d.st_col[c];
    rb.valid[c] = any_valid ? d.st_valid[c] : nullptr;
  }
  PushArgs la = a;
  la.wm_in = carry;  // any value <= the records' stream times keeps grace exact
  rc = push_local(d, cfg, prog, la, rb, need_seq ? d.st_seq : nullptr, may_be_late ? d.st_wm : nullptr, r, err);
  float ms = 0;
  if (hipEventElapsedTime(&ms, d.ev_c, d.ev_d) == hipSuccess) r.exchange_ms = ms;
  r.exchange_bytes = (uint64_t)(so - scount[me]) * 8;
  r.wm_out = wm_global;
  r.owned = m_recv;
  r.global_records = total;
  return rc;
}

}  // namespace hsg
