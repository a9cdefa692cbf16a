// Host orchestration of one operator's batch on its HIP stream: staging, the
// stream-time scan, the aggregation kernels, changelog bookkeeping, dumps.
#include <cstdio>
#include <cstdlib>
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <chrono>
#include <algorithm>
#include <cstring>
#include <string>
#include <vector>

#include "hsg_internal.h"
#include "hsg_ops.h"
#include "hsg_kernels.h"
#include "hsg_session.h"
#include "hsg_sort.h"
#include "hsg_part.h"

namespace hsg {

#define DTRY(expr)                                                          \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) {                                                 \
      err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;          \
    }                                                                       \
  } while (0)

// Hopping ops on the partition path: k_seg_apply checks its deferred window
// updates against the table's room and holds back past it (op_device.cpp
// resume_deferred), so the table follows the groups the batches make.
static bool has_last(const Program &prog);
static bool defer_room_checked(const OpDevice &d, const hsg_op_config &cfg, const Program &prog) {
  return d.use_part && cfg.window_kind == HSG_HOPPING && cfg.emit_mode != HSG_EMIT_PER_RECORD && !has_last(prog);
}

static uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

template <typename T>
static hipError_t dalloc(T **p, uint64_t count) {
  if (count == 0) count = 1;
  return hipMalloc((void **)p, count * sizeof(T));
}

template <typename T>
static void dfree(T *&p) {
  if (p) hipFree((void *)p);
  p = nullptr;
}

// transport bytes of a batch's ts column; TS16 frame bases follow the offsets
// in the same staging buffer (n * 2 bytes, 256-aligned)
static uint64_t ts_bytes(const hsg_batch *b) {
  return b->ts_enc == HSG_ENC_TS32 ? 4 : b->ts_enc == HSG_ENC_TS16 ? 2 : 8;
}
static uint64_t ts16_frames(uint64_t n) { return (n + HSG_TS16_FRAME - 1) / HSG_TS16_FRAME; }
static int64_t *ts16_frames_at(const void *buf, uint64_t n) {
  return (int64_t *)((char *)buf + ((n * 2 + 255) & ~255ull));
}
// elements of T a ts staging buffer of `cap` records needs: the widest
// transport (T itself: int32 offsets or int64 ts), or TS16 offsets followed
// by their frame bases, whichever is larger
template <typename T>
static uint64_t ts_stage_count(uint64_t cap) {
  const uint64_t ts16 = ((cap * 2 + 255) & ~255ull) + ts16_frames(cap) * 8;
  const uint64_t full = cap * sizeof(T);
  return ((full > ts16 ? full : ts16) + sizeof(T) - 1) / sizeof(T);
}

// LAST, or literal-form slots: the records' global sequence numbers are needed
static bool has_last(const Program &prog) { return prog_needs_seq(prog); }

static int alloc_out(OutCols &o, uint64_t cap, int n_aggs, std::string &err, bool forms = false) {
  if (forms) DTRY(dalloc(&o.form, cap));
  DTRY(dalloc(&o.key, cap));
  DTRY(dalloc(&o.ws, cap));
  DTRY(dalloc(&o.we, cap));
  DTRY(dalloc(&o.src, cap));
  for (int j = 0; j < n_aggs; ++j) DTRY(dalloc(&o.agg[j], cap));
  return HSG_OK;
}

static void free_out(OutCols &o) {
  dfree(o.key);
  dfree(o.ws);
  dfree(o.we);
  dfree(o.src);
  for (int j = 0; j < kMaxAggs; ++j) dfree(o.agg[j]);
  dfree(o.form);
}

// Partitioned-aggregation scratch, carved from one allocation.
int part_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err) {
  PartBuffers &pb = d.part;
  const uint64_t n = d.batch_cap;
  const int words = part_words(cfg.n_cols, prog_part_seq(prog));
  const uint64_t tiles = part_tiles(n, part_tile_for(words)) + 1;
  const uint64_t nh = (1ull << kPartMaxLog2) * tiles;
  uint64_t off = 0;
  auto take = [&](uint64_t bytes) {
    off = (off + 255) & ~255ull;
    uint64_t o = off;
    off += bytes ? bytes : 1;
    return o;
  };
  const uint64_t ns = (1ull << kPartMaxLog2) * part_nseg(tiles);
  uint64_t o_hist = take(nh * 4), o_offt = take(nh * 4), o_segsum = take(ns * 4), o_segoff = take((ns + 1) * 8);
  uint64_t o_bstart = take(((1ull << kPartMaxLog2) + 1) * 8), o_part = take((scan_partials_needed(ns) + 8) * 8);
  // records per aggregation workgroup: >= 1024 (kAggChunk / 32 at least), the
  // per-record changelog's chunks of kPrPairs pairs (k_prpart.hip) fewer
  const bool per_record = cfg.emit_mode == HSG_EMIT_PER_RECORD;
  const uint64_t min_chunk = per_record ? (uint64_t)kPrPairs / (d.wpr ? d.wpr : 1) : 1024;
  const uint64_t nwg = (1ull << kPartMaxLog2) + n / (min_chunk ? min_chunk : 1) + 2;
  uint64_t o_rec = take(n * words * 8), o_chunk = take(((1ull << kPartMaxLog2) + 2) * 4);
  uint64_t o_cbk = take(nwg * 4);  // >= buckets + n / chunk + 1
  const uint64_t tcap = n * (d.wpr ? d.wpr : 1), nc = touch_chunks(tcap);
  uint64_t o_touch = take(tcap * 4), o_wm = take(n * 8);
  uint64_t o_tcnt = take(nc * 4), o_toff = take((nc + 1) * 8), o_tpart = take((scan_partials_needed(nc) + 8) * 8);
  // lean aggregation: one pane entry per record at most, [g][slots]; the
  // general kernel's deferred window updates: up to 2 per record, more fall
  // back to in-kernel updates
  // (the per-record changelog uses none of them)
  const uint64_t pcap = per_record ? 1 : n * (d.wpr > 1 ? 2 : 1);
  uint64_t o_pane = take(pcap * (1 + (uint64_t)prog.n_slots) * 8);
  uint64_t o_seg = take(nwg * kMaxSeg * 16);
  uint64_t o_pinfo = take(nwg * 16);
  uint64_t o_pcnt = take((nwg + 4) * 4);
  DTRY(hipMalloc(&d.part_mem, off));
  char *m = (char *)d.part_mem;
  pb.hist = (uint32_t *)(m + o_hist);
  pb.offt = (uint32_t *)(m + o_offt);
  pb.segsum = (uint32_t *)(m + o_segsum);
  pb.segoff = (uint64_t *)(m + o_segoff);
  pb.bstart = (uint64_t *)(m + o_bstart);
  pb.partial = (uint64_t *)(m + o_part);
  pb.rec = (uint64_t *)(m + o_rec);
  pb.chunk_start = (uint32_t *)(m + o_chunk);
  pb.chunk_bucket = (uint32_t *)(m + o_cbk);
  pb.touched = (uint32_t *)(m + o_touch);
  pb.touched_cap = tcap;
  pb.tcnt = (uint32_t *)(m + o_tcnt);
  pb.toff = (uint64_t *)(m + o_toff);
  pb.tpartial = (uint64_t *)(m + o_tpart);
  pb.wm = (int64_t *)(m + o_wm);
  pb.pane = (uint64_t *)(m + o_pane);
  pb.pane_info = (uint64_t *)(m + o_pinfo);
  pb.pane_cnt = (uint32_t *)(m + o_pcnt);
  pb.seg = (uint64_t *)(m + o_seg);
  pb.pane_cap = pcap;
  pb.n_cap = n;
  return HSG_OK;
}

// Partitions, aggregation variant and rounds for the next batch, from the
// groups (LDS entries) the last batch flushed: buckets of at most half an LDS
// table of groups, so a bucket is normally one workgroup's (plain
// read-modify-write flushes) and its table is flushed once; the small table
// (two workgroups per CU) when that needs at most 2^kPartMaxLog2 buckets;
// fewer buckets mean longer coalesced runs in the scatter. When the bucket
// count is at its maximum, key-hash rounds split a bucket's groups instead.
uint64_t sql_lds_entries(const Program &prog);  // k_agg_sql.hip

static void adapt_partitions(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t groups, uint64_t n) {
  const uint64_t by_size = (n + kAggChunk / 2 - 1) / (kAggChunk / 2);  // buckets of <= half a chunk on average
  auto entries = [&](bool big) { return d.sql_lean ? sql_lds_entries(prog) : part_lds_entries(prog, big); };
  auto need = [&](bool big) {
    const uint64_t per = entries(big) / 2;
    uint64_t w = (groups + per - 1) / per;
    return w > by_size ? w : by_size;
  };
  uint64_t want = need(false);
  // one-window ops of more than two slots take the big table whatever the
  // group count: half the buckets, so the scatter's runs per (tile, bucket)
  // are twice as long and the (tile, bucket) offsets matrix half the size
  // (C2: scatter 164 -> 137 us, aggregation 113 -> 126 us, 30.5 -> 32.3 G
  // records/s HBM-resident); HSG_AGG_SMALL keeps the small table (A/B)
  // (two-slot ops -- C5's SUM / MAX -- measured the same on either table:
  // 23.25 against 23.31 G records/s; hopping ops already take the big one)
  static const bool keep_small = getenv("HSG_AGG_SMALL") != nullptr;
  const bool prefer_big = !keep_small && cfg.window_kind != HSG_HOPPING && d.pane_S == 1 && prog.n_slots > 2;
  d.agg_big = (want > (1ull << kPartMaxLog2) || prefer_big) && !d.sql_lean;  // (the SQL lean kernels: one LDS variant)
  if (d.agg_big) want = need(true);
  int l = 0;
  while ((1ull << l) < want && l < kPartMaxLog2) ++l;
  d.np_log2 = l < 4 ? 4 : l;
  const uint64_t per_bucket = groups >> d.np_log2;
  const uint64_t fit = entries(d.agg_big) * 6 / 10;
  int rb = 0;
  while ((fit << rb) < per_bucket && rb < 4) ++rb;
  d.rbits = d.pane_S ? rb : 0;
}

void wait_table_reset(OpDevice &d) {
  if (!d.reset_pending) return;
  hipStreamWaitEvent(d.stream, d.ev_reset, 0);
  d.reset_pending = false;
}

int op_device_reset(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err) {
  DTRY(hipMemsetAsync(d.sc, 0, sizeof(DevScalars), d.stream));
  memset(d.h_sc, 0, sizeof(DevScalars));  // host mirror (epoch_set gates the optimistic path)
  d.ovf_rows = 0;  // the clear below empties the overflow rows with the regions
  d.sc_clean = false;
  if (cfg.window_kind == HSG_SESSION) {
    int rc = session_device_reset(d, err);
    if (rc != HSG_OK) return rc;
  } else {
    // the clear runs on the side stream after everything queued on the op's
    // stream; kernels that touch the table wait for it (wait_table_reset)
    DTRY(hipEventRecord(d.ev_pre, d.stream));
    DTRY(hipStreamWaitEvent(d.aux, d.ev_pre, 0));
    // (only the blocks claimed since the last clear, once the dirty map is
    // valid)
    if (d.tw_cnt_pending) {  // the previous clear's count (long finished)
      DTRY(hipEventSynchronize(d.ev_reset));
      d.tw_cnt_pending = false;
      if (2 * *d.h_tw_cnt > (d.tw.slots() >> 3)) {
        d.tw.dirty = nullptr;
        d.tw_map_valid = false;
      }
    }
    if (d.tw_map_valid) {
      launch_tw_reset_dirty(d.aux, d.tw, prog, d.tw_cnt);
      DTRY(hipMemcpyAsync(d.h_tw_cnt, d.tw_cnt, 8, hipMemcpyDeviceToHost, d.aux));
      d.tw_cnt_pending = true;
    } else {
      launch_tw_reset(d.aux, d.tw, prog);
    }
    d.tw_map_valid = d.tw.dirty != nullptr;
    DTRY(hipEventRecord(d.ev_reset, d.aux));
    d.reset_pending = true;
    tw_retention_reset(d);
    if (cfg.window_kind == HSG_UNWINDOWED) {
      // one implicit window: k = 0, epoch fixed at 0
      DevScalars init;
      memset(&init, 0, sizeof(init));
      init.epoch_set = 1;
      memcpy(d.h_sc, &init, sizeof(init));
      DTRY(hipMemcpyAsync(d.sc, d.h_sc, sizeof(DevScalars), hipMemcpyHostToDevice, d.stream));
    }
  }
  DTRY(hipGetLastError());
  DTRY(hipStreamSynchronize(d.stream));
  return HSG_OK;
}

int op_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t batch_cap, int nranks, bool sharded,
                   uint64_t wpr, std::string &err) {
  d.nranks = nranks;
  d.n_cols = cfg.n_cols;
  d.wpr = wpr;
  // after a key exchange a rank can receive up to nranks * batch_cap records
  d.batch_cap = batch_cap * (uint64_t)nranks;
  DTRY(hipStreamCreateWithFlags(&d.stream, hipStreamNonBlocking));
  DTRY(hipStreamCreateWithFlags(&d.aux, hipStreamNonBlocking));
  DTRY(hipEventCreateWithFlags(&d.ev_reset, hipEventDisableTiming));
  DTRY(hipEventCreateWithFlags(&d.ev_pre, hipEventDisableTiming));
  DTRY(hipEventCreate(&d.ev_a));
  DTRY(hipEventCreate(&d.ev_b));
  DTRY(hipEventCreate(&d.ev_c));
  DTRY(hipEventCreate(&d.ev_d));
  DTRY(hipEventCreateWithFlags(&d.ev_fetch, hipEventDisableTiming));
  DTRY(dalloc(&d.sc, 1));
  DTRY(hipHostMalloc((void **)&d.h_sc, sizeof(DevScalars), hipHostMallocDefault));
  d.n_tiles_cap = (d.batch_cap + kTileRecords - 1) / kTileRecords + 1;
  DTRY(dalloc(&d.tile_max, d.n_tiles_cap));
  DTRY(dalloc(&d.tile_min, d.n_tiles_cap));
  DTRY(dalloc(&d.tile_prefix, d.n_tiles_cap));
  // per-tile ts extrema of the optimistic and exchange histograms (4096-record
  // tiles, 2 words each) share the stream-time tile maxima (1024-record tiles)
  static_assert(kTileRecords * 2 <= kPartTileRecs, "tile extrema buffer");
  d.part.text = (uint64_t *)d.tile_max;
  DTRY(dalloc(&d.st_key, d.batch_cap));
  DTRY(dalloc(&d.st_ts, d.batch_cap));
  for (int c = 0; c < cfg.n_cols; ++c) {
    DTRY(dalloc(&d.st_col[c], d.batch_cap));
    DTRY(dalloc(&d.st_valid[c], d.batch_cap));
  }
  uint64_t rows = cfg.state_capacity ? cfg.state_capacity : (1ull << 21);
  d.cap = next_pow2(rows * 2);  // load factor <= 1/2
  // hopping: a key's windows share its 8-row blocks, probed in steps of 8
  // rows; past 1/2 load those chains dominate k_seg_apply (C3 at 71 %: 1.49
  // ms per batch against 1.07 ms at 36 %), and 288 GB of HBM holds the rows
  d.load8 = cfg.window_kind == HSG_HOPPING ? 4 : 6;
  if (cfg.window_kind == HSG_SESSION) {
    int rc = session_device_init(d, cfg, prog, rows, err);
    if (rc != HSG_OK) return rc;
  } else {
    d.tw.stride = tw_row_stride(prog.n_slots);
    d.region_log2 = 12;
    tw_configure(d.tw, d.cap, cfg.window_kind, d.region_log2);
    d.tw.ovf = &d.sc->scratch[33];
    DTRY(dalloc(&d.tw.rows, d.tw.slots() * (uint64_t)d.tw.stride));
    DTRY(dalloc(&d.tw_dirty_mem, tw_dirty_bytes(d.tw.slots())));
    d.tw.dirty = d.tw_dirty_mem;
    DTRY(dalloc(&d.tw_cnt, 1));
    DTRY(hipHostMalloc((void **)&d.h_tw_cnt, 8, hipHostMallocDefault));
    d.tw.bshift = 0;  // set with the exchange (exchange_device_init)
    uint64_t nb = emit_chunks(d.tw.slots());
    DTRY(dalloc(&d.emit.cnt, nb));
    DTRY(dalloc(&d.emit.off, nb));
    DTRY(dalloc(&d.emit.partial, scan_partials_needed(nb) + 8));
  }
  // changelog capacity
  uint64_t oc = cfg.out_capacity;
  if (!oc && cfg.emit_mode != HSG_EMIT_NONE) {
    oc = d.batch_cap * wpr;
    if (cfg.emit_mode == HSG_EMIT_PER_BATCH && cfg.window_kind != HSG_SESSION && oc > d.cap) oc = d.cap;
  }
  d.out_cap = oc;
  int rc = alloc_out(d.out, d.out_cap, cfg.n_aggs, err, d.forms);
  d.own_out = d.out;
  d.own_out_cap = d.out_cap;
  if (rc != HSG_OK) return rc;
  if (cfg.emit_mode == HSG_EMIT_PER_RECORD && cfg.window_kind != HSG_SESSION && perrecord_part_eligible(prog, wpr)) {
    rc = perrecord_part_init(d, cfg, prog, err);
    if (rc != HSG_OK) return rc;
  } else if (cfg.emit_mode == HSG_EMIT_PER_RECORD || (cfg.window_kind == HSG_SESSION && !d.ss_merge)) {
    rc = perrecord_device_init(d, cfg, prog, err);
    if (rc != HSG_OK) return rc;
  } else if ((cfg.window_kind == HSG_TUMBLING || cfg.window_kind == HSG_UNWINDOWED) && prog_part_seq(prog) &&
             (cfg.n_cols == 1 || cfg.n_cols == 2) && prog.n_slots <= 16) {
    // the SQL drop-in's op shape (LAST passthroughs, literal forms) of one-window
    // ops: packed records with their sequence word on the SQL lean kernels
    // (k_agg_sql.hip); a batch they refuse runs on the record kernels
    d.use_part = true;
    d.sql_lean = true;
    d.pane_S = 1;
    // no group count before the first batch: the most buckets (a bucket whose
    // groups overflow its LDS table sends the batch to the careful path)
    d.np_log2 = kPartMaxLog2;
    rc = part_device_init(d, cfg, prog, err);
    if (rc != HSG_OK) return rc;
  } else if (part_supported(prog)) {
    d.use_part = true;
    {
      // panes: size a multiple of advance (tumbling and unwindowed: one pane per window)
      const int64_t adv = cfg.window_kind == HSG_HOPPING ? cfg.advance_ms : 0;
      d.pane_S = 1;
      if (adv > 0) d.pane_S = (cfg.size_ms % adv == 0 && cfg.size_ms / adv <= 64) ? (int)(cfg.size_ms / adv) : 0;
      rc = part_device_init(d, cfg, prog, err);
      if (rc != HSG_OK) return rc;
    }
  }
  if (sharded) {
    rc = exchange_device_init(d, cfg, batch_cap, err);
    if (rc != HSG_OK) return rc;
  }
  return op_device_reset(d, cfg, prog, err);
}

void op_device_free(OpDevice &d) {
  if (d.aux) hipStreamSynchronize(d.aux);
  if (d.stream) hipStreamSynchronize(d.stream);
  exchange_device_free(d);
  dfree(d.sc);
  if (d.h_sc) hipHostFree(d.h_sc);
  d.h_sc = nullptr;
  dfree(d.tile_max);
  dfree(d.tile_min);
  dfree(d.tile_prefix);
  dfree(d.st_key);
  dfree(d.st_ts);
  for (int c = 0; c < kMaxCols; ++c) {
    dfree(d.st_col[c]);
    dfree(d.st_valid[c]);
  }
  dfree(d.st_seq);
  dfree(d.st_wm);
  dfree(d.nar_ts);
  dfree(d.nar_key);
  for (int c = 0; c < kMaxCols; ++c) dfree(d.nar_col[c]);
  if (d.h2d) hipStreamSynchronize(d.h2d);
  for (auto &s : d.pre) {
    dfree(s.key);
    dfree(s.ts);
    for (int c = 0; c < kMaxCols; ++c) {
      dfree(s.col[c]);
      dfree(s.valid[c]);
    }
  }
  for (auto &e : d.ev_h2d) {
    if (e) hipEventDestroy(e);
    e = nullptr;
  }
  if (d.h2d) hipStreamDestroy(d.h2d);
  d.h2d = nullptr;
  dfree(d.tw.rows);
  dfree(d.tw_dirty_mem);
  dfree(d.tw_cnt);
  if (d.h_tw_cnt) hipHostFree(d.h_tw_cnt);
  d.h_tw_cnt = nullptr;
  dfree(d.emit.cnt);
  dfree(d.emit.off);
  dfree(d.emit.partial);
  session_device_free(d);
  free_out(d.own_out);
  d.out = d.own_out;
  if (d.scratch) hipFree(d.scratch);
  d.scratch = nullptr;
  if (d.part_mem) hipFree(d.part_mem);
  d.part_mem = nullptr;
  if (d.tkeys) hipFree(d.tkeys);
  d.tkeys = nullptr;
  d.tkeys_cap = 0;
  if (d.xsend) hipFree(d.xsend);
  if (d.xrecv) hipFree(d.xrecv);
  d.xsend = d.xrecv = nullptr;
  dfree(d.d_counts);
  if (d.h_counts) hipHostFree(d.h_counts);
  if (d.h_tmp) hipHostFree(d.h_tmp);
  d.h_tmp = nullptr;
  d.h_counts = nullptr;
  if (d.ev_a) hipEventDestroy(d.ev_a);
  if (d.ev_b) hipEventDestroy(d.ev_b);
  if (d.ev_c) hipEventDestroy(d.ev_c);
  if (d.ev_d) hipEventDestroy(d.ev_d);
  d.ev_a = d.ev_b = d.ev_c = d.ev_d = nullptr;
  if (d.stream) hipStreamDestroy(d.stream);
  d.stream = nullptr;
  if (d.aux) hipStreamDestroy(d.aux);
  d.aux = nullptr;
  if (d.ev_reset) hipEventDestroy(d.ev_reset);
  if (d.ev_pre) hipEventDestroy(d.ev_pre);
  if (d.ev_fetch) hipEventDestroy(d.ev_fetch);
  d.ev_reset = d.ev_pre = d.ev_fetch = nullptr;
  d.reset_pending = false;
}

int op_prestage(OpDevice &d, const hsg_batch *b, int set, std::string &err) {
  // a rank's own ingest (d.batch_cap also counts what an exchange may deliver)
  const uint64_t pcap = d.batch_cap / (d.nranks > 0 ? d.nranks : 1);
  if (b->mem != HSG_MEM_HOST || set < 0 || set > 1 || b->n > pcap || b->n_cols != d.user_cols) {
    err = "prestage: not a host batch of this op";
    return HSG_E_INVALID;
  }
  if (!d.h2d) {
    DTRY(hipStreamCreateWithFlags(&d.h2d, hipStreamNonBlocking));
    DTRY(hipEventCreateWithFlags(&d.ev_h2d[0], hipEventDisableTiming));
    DTRY(hipEventCreateWithFlags(&d.ev_h2d[1], hipEventDisableTiming));
  }
  OpDevice::Staging &s = d.pre[set];
  if (!s.key) {
    DTRY(dalloc(&s.key, pcap));
    DTRY(dalloc(&s.ts, ts_stage_count<int64_t>(pcap)));
    for (int c = 0; c < d.n_cols; ++c) {
      DTRY(dalloc(&s.col[c], pcap));
      DTRY(dalloc(&s.valid[c], pcap));
    }
  }
  const uint64_t n = b->n;
  const hipMemcpyKind k = hipMemcpyHostToDevice;
  // narrow columns (hsg_enc) land in the first half of their full-width
  // buffers; stage_batch widens them on the op's stream
  if (n) {
    DTRY(hipMemcpyAsync(s.key, b->key_id, n * (b->key_enc == HSG_ENC_K16 ? 2 : 4), k, d.h2d));
    DTRY(hipMemcpyAsync(s.ts, b->ts, n * ts_bytes(b), k, d.h2d));
    if (b->ts_enc == HSG_ENC_TS16)
      DTRY(hipMemcpyAsync(ts16_frames_at(s.ts, n), b->ts_frames, ts16_frames(n) * 8, k, d.h2d));
    for (int c = 0; c < b->n_cols; ++c) {
      DTRY(hipMemcpyAsync(s.col[c], b->cols[c], n * (b->col_enc[c] != HSG_ENC_FULL ? 4 : 8), k, d.h2d));
      if (b->valid && b->valid[c]) DTRY(hipMemcpyAsync(s.valid[c], b->valid[c], n, k, d.h2d));
    }
  }
  DTRY(hipEventRecord(d.ev_h2d[set], d.h2d));
  return HSG_OK;
}

// Narrow transport columns (include/hstream_gpu.h hsg_enc) at device
// addresses k16 / ts32 / c32 (used for the arrays the batch sends narrow;
// TS16: offsets at ts32, frame bases at frames) -> the op's full-width
// staging; kb points there afterwards.
static int widen_batch(OpDevice &d, const hsg_batch *b, const void *k16, const void *ts32, const int64_t *frames,
                       const void *const *c32, Batch &kb, std::string &err) {
  WidenArgs w;
  memset(&w, 0, sizeof(w));
  w.n = b->n;
  if (b->key_enc == HSG_ENC_K16) {
    w.k16 = (const uint16_t *)k16;
    w.key = d.st_key;
    kb.key = d.st_key;
  }
  if (b->ts_enc == HSG_ENC_TS32 || b->ts_enc == HSG_ENC_TS16) {
    if (b->ts_enc == HSG_ENC_TS32) {
      w.ts32 = (const int32_t *)ts32;
      w.ts_base = b->ts_base;
    } else {
      w.ts16 = (const uint16_t *)ts32;
      w.frames = frames;
    }
    w.ts = d.st_ts;
    kb.ts = d.st_ts;
  }
  for (int c = 0; c < b->n_cols; ++c) {
    if (b->col_enc[c] == HSG_ENC_FULL) continue;
    w.c32[c] = (const int32_t *)c32[c];
    w.col[c] = d.st_col[c];
    double p = 1.0;
    for (int q = 0; q < b->col_scale[c]; ++q) p *= 10.0;  // exact for <= 22 digits
    w.div[c] = b->col_enc[c] == HSG_ENC_DEC32 ? p : 0.0;
    kb.col[c] = d.st_col[c];
  }
  launch_widen(d.stream, w);
  DTRY(hipGetLastError());
  return HSG_OK;
}

static int stage_batch_raw(OpDevice &d, const hsg_batch *b, Batch &kb, std::string &err, int staged_set);

// Resolve the batch into device pointers, copying host arrays into staging
// (or taking the ones op_prestage queued for it). The valid bytes go to the
// kernels as they are: bit 1 is the literal form the forms slots read.
int stage_batch(OpDevice &d, const hsg_batch *b, Batch &kb, std::string &err, int staged_set) {
  return stage_batch_raw(d, b, kb, err, staged_set);
}

static int stage_batch_raw(OpDevice &d, const hsg_batch *b, Batch &kb, std::string &err, int staged_set) {
  memset(&kb, 0, sizeof(kb));
  kb.n = b->n;
  const uint64_t n = b->n;
  if (staged_set >= 0 && b->mem == HSG_MEM_HOST) {
    const OpDevice::Staging &s = d.pre[staged_set];
    DTRY(hipStreamWaitEvent(d.stream, d.ev_h2d[staged_set], 0));
    kb.key = s.key;
    kb.ts = s.ts;
    for (int c = 0; c < b->n_cols; ++c) {
      kb.col[c] = s.col[c];
      kb.valid[c] = (b->valid && b->valid[c]) ? s.valid[c] : nullptr;
    }
    if (batch_narrow(b)) {
      const void *c32[kMaxCols];
      for (int c = 0; c < b->n_cols; ++c) c32[c] = s.col[c];
      return widen_batch(d, b, s.key, s.ts, ts16_frames_at(s.ts, n), c32, kb, err);
    }
    return HSG_OK;
  }
  if (b->mem == HSG_MEM_DEVICE) {
    // the producer's stream is not ordered with ours: wait on its event
    if (b->ready_event) DTRY(hipStreamWaitEvent(d.stream, (hipEvent_t)b->ready_event, 0));
    kb.key = b->key_id;
    kb.ts = b->ts;
    for (int c = 0; c < b->n_cols; ++c) {
      kb.col[c] = (const int64_t *)b->cols[c];
      kb.valid[c] = (b->valid && b->valid[c]) ? b->valid[c] : nullptr;
    }
    if (batch_narrow(b)) return widen_batch(d, b, b->key_id, b->ts, b->ts_frames, b->cols, kb, err);
    return HSG_OK;
  }
  if (batch_narrow(b)) {
    // host narrow batch, synchronous push: H2D into the narrow staging, widen
    if (!d.nar_ts) {
      DTRY(dalloc(&d.nar_ts, ts_stage_count<int32_t>(d.batch_cap)));
      DTRY(dalloc(&d.nar_key, d.batch_cap));
      for (int c = 0; c < d.n_cols; ++c) DTRY(dalloc(&d.nar_col[c], d.batch_cap));
    }
    const hipMemcpyKind k = hipMemcpyHostToDevice;
    const void *c32[kMaxCols] = {};
    if (n) {
      if (b->key_enc == HSG_ENC_K16) DTRY(hipMemcpyAsync(d.nar_key, b->key_id, n * 2, k, d.stream));
      else DTRY(hipMemcpyAsync(d.st_key, b->key_id, n * 4, k, d.stream));
      if (b->ts_enc != HSG_ENC_FULL) DTRY(hipMemcpyAsync(d.nar_ts, b->ts, n * ts_bytes(b), k, d.stream));
      else DTRY(hipMemcpyAsync(d.st_ts, b->ts, n * 8, k, d.stream));
      if (b->ts_enc == HSG_ENC_TS16)
        DTRY(hipMemcpyAsync(ts16_frames_at(d.nar_ts, n), b->ts_frames, ts16_frames(n) * 8, k, d.stream));
    }
    kb.key = d.st_key;
    kb.ts = d.st_ts;
    for (int c = 0; c < b->n_cols; ++c) {
      const bool nar = b->col_enc[c] != HSG_ENC_FULL;
      if (n) DTRY(hipMemcpyAsync(nar ? (void *)d.nar_col[c] : (void *)d.st_col[c], b->cols[c], n * (nar ? 4 : 8), k, d.stream));
      c32[c] = d.nar_col[c];
      kb.col[c] = d.st_col[c];
      if (b->valid && b->valid[c]) {
        if (n) DTRY(hipMemcpyAsync(d.st_valid[c], b->valid[c], n, k, d.stream));
        kb.valid[c] = d.st_valid[c];
      }
    }
    return widen_batch(d, b, d.nar_key, d.nar_ts, ts16_frames_at(d.nar_ts, n), c32, kb, err);
  }
  if (n) {
    DTRY(hipMemcpyAsync(d.st_key, b->key_id, n * 4, hipMemcpyHostToDevice, d.stream));
    DTRY(hipMemcpyAsync(d.st_ts, b->ts, n * 8, hipMemcpyHostToDevice, d.stream));
  }
  kb.key = d.st_key;
  kb.ts = d.st_ts;
  for (int c = 0; c < b->n_cols; ++c) {
    if (n) DTRY(hipMemcpyAsync(d.st_col[c], b->cols[c], n * 8, hipMemcpyHostToDevice, d.stream));
    kb.col[c] = d.st_col[c];
    if (b->valid && b->valid[c]) {
      if (n) DTRY(hipMemcpyAsync(d.st_valid[c], b->valid[c], n, hipMemcpyHostToDevice, d.stream));
      kb.valid[c] = d.st_valid[c];
    }
  }
  return HSG_OK;
}

TwParams make_tw_params(const hsg_op_config &cfg, const PushArgs &a) {
  TwParams p;
  memset(&p, 0, sizeof(p));
  p.kind = cfg.window_kind;
  p.batch_id = (int32_t)a.batch_id;
  p.size = cfg.size_ms;
  p.adv = cfg.window_kind == HSG_HOPPING ? cfg.advance_ms : (cfg.size_ms > 0 ? cfg.size_ms : 1);
  p.grace = cfg.grace_ms;
  p.wm_in = a.wm_in;
  p.rec_base = a.rec_base;
  p.div = make_divider((uint64_t)p.adv);
  return p;
}

// Stream time for a batch in arrival order: per-tile maxima, exclusive tile
// prefix (seeded with wm_in), epoch initialisation.
void launch_stream_time(OpDevice &d, const hsg_op_config &cfg, const Batch &kb, int64_t wm_in, int64_t adv) {
  uint64_t tiles = (kb.n + kTileRecords - 1) / kTileRecords;
  launch_tile_stats(d.stream, kb, d.tile_max, d.tile_min, tiles);
  const bool tw = cfg.window_kind == HSG_TUMBLING || cfg.window_kind == HSG_HOPPING;
  launch_tile_scan(d.stream, d.tile_max, d.tile_min, d.tile_prefix, tiles, wm_in, adv, tw, d.sc,
                   tw ? (cfg.grace_ms >= 0 ? cfg.grace_ms : 0) : -1);
}

// Copies the scalars to the host mirror, then (same stream, before the host
// waits) clears the per-batch ones for the next batch, so a push does not
// start with a dependent launch.
// The host waits on the stream inside every push (here, and on the exchange's
// all-gathered facts), so the wake-up latency is GPU idle time: poll an event
// for up to 5 ms (a batch's pipeline is well under that), then block.
int poll_stream(OpDevice &d, hipStream_t s, std::string &err) {
  DTRY(hipEventRecord(d.ev_fetch, s));
  const auto t0 = std::chrono::steady_clock::now();
  hipError_t e;
  while ((e = hipEventQuery(d.ev_fetch)) == hipErrorNotReady) {
    if (std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(5)) {
      e = hipEventSynchronize(d.ev_fetch);
      break;
    }
  }
  DTRY(e);
  return HSG_OK;
}

int fetch_scalars(OpDevice &d, std::string &err) {
  launch_fetch_clear_scalars(d.stream, d.sc, d.h_sc);
  DTRY(hipGetLastError());
  // (against hipStreamSynchronize plus a separate copy and clear: C2 34.7 ->
  // 34.8 G, C5 24.2 -> 24.5 G records/s HBM-resident, profiles/r06)
  const int rc = poll_stream(d, d.stream, err);
  if (rc != HSG_OK) return rc;
  for (int k = 0; k < 8; ++k) d.h_sc->live += d.h_sc->live_x[k];  // device: live + shards
  d.ovf_rows += d.h_sc->scratch[33];  // groups a full region sent to the overflow rows (cleared above)
  d.sc_clean = true;
  return HSG_OK;
}

int clear_batch_scalars(OpDevice &d, std::string &err) {
  // err, pairs, late, out_rows, touched, redo, scratch; wm/epoch/live persist
  if (d.sc_clean) {
    d.sc_clean = false;
    return HSG_OK;
  }
  launch_clear_scalars(d.stream, d.sc);
  DTRY(hipGetLastError());
  return HSG_OK;
}

static int status_from_err(uint32_t e, std::string &err) {
  if (e & ERR_OOM) {
    err = "HBM state table / arena full (raise state_capacity)";
    return HSG_E_OOM;
  }
  if (e & ERR_RANGE) {
    err = "window index outside the op's 2^32-window span around its first batch";
    return HSG_E_RANGE;
  }
  return HSG_OK;
}

int finish_batch(OpDevice &d, int64_t wm_in, uint64_t n, PushResult &r, std::string &err) {
  int rc = fetch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  const DevScalars &s = *d.h_sc;
#ifndef HSG_PHASE_CLOCKS
#define HSG_PHASE_CLOCKS 0
#endif
  // the phase clocks exist only in a PHASES=1 build (hsg_dev.h kPhaseClocks)
  static const bool phases = HSG_PHASE_CLOCKS && getenv("HSG_PHASES") != nullptr;
  if (phases && s.scratch[12])
    fprintf(stderr, "[hsg phases] agg wg=%llu init=%.1fus records=%.1fus flush=%.1fus tail=%.1fus (per-wg avg)\n",
            (unsigned long long)s.scratch[12], s.scratch[8] * 0.01 / s.scratch[12], s.scratch[9] * 0.01 / s.scratch[12],
            s.scratch[10] * 0.01 / s.scratch[12], s.scratch[11] * 0.01 / s.scratch[12]);
  if (phases && s.scratch[12])
    fprintf(stderr, "[hsg phases] agg flush: sort=%.1fus runs=%.1fus rounds/wg=%.2f panes=%llu updates=%llu\n",
            s.scratch[18] * 0.01 / s.scratch[12], s.scratch[19] * 0.01 / s.scratch[12],
            (double)s.scratch[20] / s.scratch[12], (unsigned long long)s.scratch[0], (unsigned long long)s.scratch[1]);
  if (phases && s.scratch[17])
    fprintf(stderr, "[hsg phases] scatter wg=%llu walk=%.1fus -=%.1fus -=%.1fus write=%.1fus (per-wg avg)\n",
            (unsigned long long)s.scratch[17], s.scratch[13] * 0.01 / s.scratch[17], s.scratch[14] * 0.01 / s.scratch[17],
            s.scratch[15] * 0.01 / s.scratch[17], s.scratch[16] * 0.01 / s.scratch[17]);
  if (phases && s.scratch[30] && s.scratch[23] == 1)
    fprintf(stderr, "[hsg phases] bucket replay sub-passes=%llu load=%.2fus group=%.2fus rank+probe+reserve=%.2fus replay=%.2fus tail=%.2fus (per sub-pass)\n",
            (unsigned long long)s.scratch[30], s.scratch[24] * 0.01 / s.scratch[30], s.scratch[25] * 0.01 / s.scratch[30],
            s.scratch[26] * 0.01 / s.scratch[30], s.scratch[27] * 0.01 / s.scratch[30], s.scratch[28] * 0.01 / s.scratch[30]);
  if (phases && s.scratch[30] && s.scratch[23] == 1)
    fprintf(stderr, "[hsg phases] bucket replay records off the mirror=%llu (past the tail %llu) groups=%llu\n",
            (unsigned long long)(s.scratch[43] & 0xFFFFFFFFu), (unsigned long long)(s.scratch[43] >> 32),
            (unsigned long long)s.scratch[44]);
  else if (phases && s.scratch[30])
    fprintf(stderr, "[hsg phases] session sort wg=%llu buckets=%.1fus insert=%.1fus scan=%.1fus place=%.1fus keys=%.1fus total=%.1fus (per-wg avg)\n",
            (unsigned long long)s.scratch[30], s.scratch[24] * 0.01 / s.scratch[30], s.scratch[25] * 0.01 / s.scratch[30],
            s.scratch[26] * 0.01 / s.scratch[30], s.scratch[27] * 0.01 / s.scratch[30], s.scratch[28] * 0.01 / s.scratch[30],
            s.scratch[29] * 0.01 / s.scratch[30]);
  if (phases && s.scratch[41])
    fprintf(stderr, "[hsg phases] per-record bucket wg=%llu segments/wg=%.2f insert=%.1fus claim=%.1fus steps=%.1fus writeback=%.1fus total=%.1fus (per-wg avg)\n",
            (unsigned long long)s.scratch[41], (double)s.scratch[40] / s.scratch[41], s.scratch[36] * 0.01 / s.scratch[41],
            s.scratch[37] * 0.01 / s.scratch[41], s.scratch[38] * 0.01 / s.scratch[41], s.scratch[39] * 0.01 / s.scratch[41],
            s.scratch[42] * 0.01 / s.scratch[41]);
  if (phases && s.scratch[41])
    fprintf(stderr, "[hsg phases] per-record bucket: pre=%.1fus A=%.1fus B=%.1fus (thread 0) peer-lanes per keyed lane=%.2f\n",
            (s.scratch[43] & 0x1FFFFF) * 0.01, ((s.scratch[43] >> 21) & 0x1FFFFF) * 0.01,
            ((s.scratch[43] >> 42) & 0x1FFFFF) * 0.01, (double)s.scratch[44] / (16777216.0 / 64));

  r.wm_out = n ? s.wm_out : wm_in;
  r.pairs = s.pairs;
  r.late = s.late;
  r.out_rows = s.out_rows + s.scratch[3];  // touched-list emit, or rows the lean apply wrote itself
  r.touched = s.touched;
  r.state_rows = s.live + d.spilled_rows;
  return status_from_err(s.err, err);
}

static int push_time_atomic(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                            const Batch &kb, const int64_t *seq, const int64_t *rec_wm, PushResult &r,
                            std::string &err) {
  TwParams p = make_tw_params(cfg, a);
  // Optimistic partitioned path: assume no record of the batch is late, fold
  // the stream-time inputs into the histogram pass and decide afterwards (one
  // tiny kernel); a batch that does have late records is run again with the
  // per-record stream time. Needs the window epoch (set by an earlier batch).
  // The first batch after create/reset has no epoch yet: k_epoch_first sets it
  // (device side) from the batch's first keyed record ahead of the optimistic
  // kernels, which then run as on every later batch.
  // the SQL lean kernels (d.sql_lean) run only optimistic packed batches; a
  // batch they refuse (late records, a wide layout, a split bucket or an
  // overflowing chunk: scratch[35]) runs again on the record kernels
  // (k_window.hip k_tw_agg and its LAST / tie resolution pass)
  const bool sql = d.sql_lean;
  const bool opt = d.use_part && !rec_wm && (!has_last(prog) || sql) && cfg.grace_ms >= 0 &&
                   cfg.window_kind != HSG_SESSION;
  const bool need_epoch = !d.h_sc->epoch_set;
  // Table room (see table_bound_hint): the partition path's claiming kernels
  // check the batch against pp.room (3/4 load) before they claim anything --
  // the lean apply its partials, the general kernels one group per (record,
  // window) -- and hold back past it; the batch then runs again on a table
  // grown for that bound. The other paths were given the worst case by op_push.
  // Launch prediction (speed only): the variants a batch does not take exit at
  // once on the device, but each costs a launch. After a packed batch whose
  // changelog the lean apply wrote itself, the next batch's wide-layout
  // variants and touched-list emit chain are not launched; a batch that turns
  // out otherwise is completed after the fetch (wide: run again -- the packed
  // kernels exited without touching the state; emit: the chain runs on the
  // touched list the apply left).
  bool skipped_wide = false, skipped_emit = false;
  // hopping ops: the general kernel defers its window updates to k_seg_apply,
  // which checks them against the room (its partials bound the batch's new
  // groups), so the table is sized from the last batch's deferred updates
  // rather than one group per (record, window) (table_bound_hint)
  const bool defer_sized = defer_room_checked(d, cfg, prog);
  PartParams last_pp;
  memset(&last_pp, 0, sizeof(last_pp));
  auto run = [&](bool optimistic) -> int {
    skipped_wide = skipped_emit = false;  // (this run's launch prediction)
    int rc = clear_batch_scalars(d, err);
    if (rc != HSG_OK) return rc;
    if (!kb.n) return HSG_OK;
    // stream time (and the window epoch on the first batch); after a key exchange
    // the per-record stream time arrives in rec_wm and only the epoch is used
    // the optimistic kernels fold stream time into the histogram; the first
    // batch after create/reset takes its epoch from its first keyed record
    if (!optimistic) launch_stream_time(d, cfg, kb, a.wm_in, p.adv);
    else if (need_epoch) launch_epoch_first(d.stream, kb, p.adv, d.sc);
    DTRY(hipEventRecord(d.ev_a, d.stream));
    const bool part_now = d.use_part && (!sql || optimistic);
    if (part_now) {
      PartParams pp;
      memset(&pp, 0, sizeof(pp));
      pp.np_log2 = d.np_log2;
      pp.bshift = d.bshift;
      for (int c = 0; c < cfg.n_cols; ++c) pp.has_valid |= kb.valid[c] != nullptr;
      pp.has_seq = prog_part_seq(prog);
      pp.words = part_words(cfg.n_cols, pp.has_seq);
      pp.tile = part_tile_for(pp.words);
      pp.sub = optimistic ? kRowSub : 1;  // offsets rows of kRowSub tiles (the careful path: one)
      pp.tiles = part_tiles(kb.n, pp.tile * pp.sub);
      pp.pane_S = d.pane_S;
      pp.rbits = d.rbits;
      pp.chunk = kAggChunk;
      pp.big = d.agg_big ? 1 : 0;
      pp.defer = 1;
      const uint64_t lim = d.cap / 8 * d.load8;
      pp.room = lim > d.h_sc->live ? lim - d.h_sc->live : 0;
      pp.hold = !defer_sized && kb.n * d.wpr > pp.room ? 1 : 0;
      last_pp = pp;
      if (!rec_wm && !optimistic) launch_part_recwm(d.stream, kb, d.tile_prefix, d.sc, d.part.wm);
      launch_part_hist(d.stream, kb, p, pp, rec_wm, d.part.wm, d.part, d.sc, optimistic);
      const bool can_pack = optimistic && cfg.n_cols <= 8 && d.wpr < 256;
      if (optimistic)
        launch_part_decide_offsets(d.stream, d.sc, p, a.wm_in, cfg.grace_ms, can_pack, pp, d.part);
      else
        launch_part_offsets(d.stream, pp, d.part, d.sc);
      skipped_wide = can_pack && d.pred_packed && part_lean_eligible(prog, pp);
      // (the SQL kernels have no wide variant: a wide batch runs again carefully)
      launch_part_scatter(d.stream, kb, p, pp, rec_wm, d.part.wm, seq, d.part, d.sc, can_pack, !skipped_wide && !sql);
      const bool emit_batch = cfg.emit_mode == HSG_EMIT_PER_BATCH;
      bool lean = false;
      wait_table_reset(d);  // the partition passes above do not touch the table
      launch_part_agg(d.stream, prog, p, pp, d.tw, d.part, kb.n, d.sc, can_pack, emit_batch ? &d.out : nullptr,
                      a.pending, d.out_cap, !skipped_wide, &lean);
      if (!lean) skipped_wide = false;  // the general kernel ran both layouts
      skipped_emit = emit_batch && d.pred_direct;  // the lean or the deferred (k_seg_apply) path
    } else {
      wait_table_reset(d);
      launch_tw_agg(d.stream, kb, p, d.tw, prog, d.tile_prefix, rec_wm, seq, d.sc, false);
    }
    if (has_last(prog) && !(sql && part_now))
      launch_tw_agg(d.stream, kb, p, d.tw, prog, d.tile_prefix, rec_wm, seq, d.sc, true);
    if (cfg.emit_mode == HSG_EMIT_PER_BATCH) {
      if (part_now) {
        if (!skipped_emit) launch_part_emit(d.stream, d.tw, prog, p, d.part, d.out, a.pending, d.out_cap, d.sc);
      } else {
        launch_tw_emit(d.stream, d.tw, d.tw.slots(), prog, p, 0, d.out, a.pending, d.out_cap, d.sc, d.emit,
                       (uint64_t *)&d.sc->out_rows);
      }
    }
    // ev_a .. ev_b: the batch's device pipeline (aggregation + changelog rows)
    DTRY(hipEventRecord(d.ev_b, d.stream));
    DTRY(hipGetLastError());
    return HSG_OK;
  };
  // k_seg_apply held its deferred window updates back for table room after
  // k_part_agg's own updates went in (the batch is half applied, so it is not
  // run again): grow the table for the deferred updates, restore the batch's
  // scalars (the fetch cleared them on the device) and launch k_seg_apply, and
  // the changelog chain after it, again on the same segments
  auto resume_deferred = [&]() -> int {
    DevScalars keep;
    memcpy(&keep, d.h_sc, sizeof(keep));
    const uint64_t bound = keep.scratch[34];
    // the touched-list entries k_part_agg made (its in-kernel updates) are
    // slots of the table tw_maintain may rebuild: carried through their group
    // keys (k_seg_apply lists only the groups the batch had not touched yet,
    // by their stamps, which the rebuild keeps)
    const uint64_t t0 = cfg.emit_mode == HSG_EMIT_PER_BATCH
                            ? (keep.scratch[1] < d.part.touched_cap ? keep.scratch[1] : d.part.touched_cap)
                            : 0;
    // (a grow-only buffer kept with the op: no hipFree, and its device-wide
    // synchronisation, on this path; tw_maintain's rebuild allocates anyway)
    if (t0 > d.tkeys_cap) {
      if (d.tkeys) hipFree(d.tkeys);
      d.tkeys = nullptr;
      d.tkeys_cap = 0;
      const uint64_t want = t0 > d.part.touched_cap / 8 ? t0 : d.part.touched_cap / 8;
      DTRY(hipMalloc((void **)&d.tkeys, want * sizeof(uint64_t)));
      d.tkeys_cap = want;
    }
    uint64_t *tkeys = d.tkeys;
    if (t0) launch_touch_keys(d.stream, d.tw, d.part.touched, t0, tkeys);
    int rc = tw_maintain(d, cfg, prog, kb.n, a.wm_in, a.pending, err, bound);
    if (rc != HSG_OK) return rc;
    if (t0) launch_touch_slots(d.stream, d.tw, tkeys, t0, d.part.touched);
    keep.live = d.h_sc->live;  // the rebuilt table's rows, the batch's claims so far included
    memset(keep.live_x, 0, sizeof(keep.live_x));
    keep.scratch[32] = 0;
    keep.scratch[33] = 0;  // (counted into ovf_rows by the fetch)
    memcpy(d.h_sc, &keep, sizeof(keep));
    DTRY(hipMemcpyAsync(d.sc, d.h_sc, sizeof(DevScalars), hipMemcpyHostToDevice, d.stream));
    d.sc_clean = false;
    PartParams pp = last_pp;
    const uint64_t lim = d.cap / 8 * d.load8;
    pp.room = lim > keep.live ? lim - keep.live : 0;  // >= bound (tw_maintain)
    const bool emit_batch = cfg.emit_mode == HSG_EMIT_PER_BATCH;
    DTRY(hipEventRecord(d.ev_a, d.stream));
    const dim3 g((unsigned)((1ull << pp.np_log2) + kb.n / pp.chunk + 1));
    launch_seg_apply(d.stream, g, prog, p, pp, d.tw, d.part, d.sc, emit_batch ? &d.out : nullptr, a.pending, d.out_cap,
                     false);
    if (emit_batch && !skipped_emit) launch_part_emit(d.stream, d.tw, prog, p, d.part, d.out, a.pending, d.out_cap, d.sc);
    DTRY(hipEventRecord(d.ev_b, d.stream));
    DTRY(hipGetLastError());
    rc = finish_batch(d, a.wm_in, kb.n, r, err);
    if (rc == HSG_OK && d.h_sc->scratch[32]) {
      err = "deferred updates held back after the table grew for them (internal)";
      return HSG_E_DEVICE;
    }
    return rc;
  };
  // a run whose claiming kernels held back for table room: grow the table for
  // the bound they saw (the lean partials, else the worst case), run again
  auto run_room = [&](bool optimistic) -> int {
    int rc = run(optimistic);
    if (rc != HSG_OK) return rc;
    rc = finish_batch(d, a.wm_in, kb.n, r, err);
    if (rc != HSG_OK || !kb.n || !d.h_sc->scratch[32]) return rc;
    d.replays += 1;
    if (d.h_sc->scratch[32] & 4) return resume_deferred();
    const uint64_t bound = (d.h_sc->scratch[32] & 2) ? UINT64_MAX : d.h_sc->scratch[31];
    rc = tw_maintain(d, cfg, prog, kb.n, a.wm_in, a.pending, err, bound);
    if (rc != HSG_OK) return rc;
    if (cfg.emit_mode == HSG_EMIT_PER_BATCH && a.pending + (kb.n * d.wpr < d.cap ? kb.n * d.wpr : d.cap) > d.out_cap) {
      err = "changelog buffer full: drain before pushing (out_capacity)";
      return HSG_E_CAPACITY;  // the batch is not applied
    }
    rc = run(optimistic);
    if (rc != HSG_OK) return rc;
    rc = finish_batch(d, a.wm_in, kb.n, r, err);
    if (rc != HSG_OK || !d.h_sc->scratch[32]) return rc;
    // held back again (the lean partial count depends on the LDS tables' fill
    // races, so a rerun may count more): the worst case, one group per
    // (record, window), then a last run that must not hold back
    rc = tw_maintain(d, cfg, prog, kb.n, a.wm_in, a.pending, err, UINT64_MAX);
    if (rc != HSG_OK) return rc;
    rc = run(optimistic);
    if (rc != HSG_OK) return rc;
    rc = finish_batch(d, a.wm_in, kb.n, r, err);
    if (rc == HSG_OK && d.h_sc->scratch[32]) {
      err = "batch held back for table room after growing for its worst case (internal)";
      return HSG_E_DEVICE;
    }
    return rc;
  };
  const uint64_t live0 = d.h_sc->live;  // rows before the batch (after its tw_maintain)
  // a run of SQL refusals at the most buckets there are (groups beyond what the
  // LDS tables hold): the careful path directly for a while
  const bool sql_try = !sql || d.sql_skip == 0;
  if (!sql_try) d.sql_skip -= 1;
  int rc = run_room(opt && sql_try);
  if (rc != HSG_OK) return rc;
  const bool sql_refused = sql && opt && sql_try && kb.n && (!d.h_sc->packed || d.h_sc->scratch[35]);
  // (a refusal is a split bucket or a chunk whose groups overflowed its LDS
  // table: more buckets for the next batch -- the careful run below leaves no
  // group count to size them by)
  const bool sql_ovf = sql_refused && d.h_sc->packed && d.h_sc->scratch[35];
  const int np_refused = d.np_log2;
  if (sql_refused) d.replays += 1;  // (hsg_stats: a lean SQL batch is counted in lean_batches)
  if (opt && kb.n && (d.h_sc->redo || sql_refused)) {
    if (sql) {
      // the record kernels check no table room: the batch's worst case first
      rc = tw_maintain(d, cfg, prog, kb.n, a.wm_in, a.pending, err, UINT64_MAX);
      if (rc != HSG_OK) return rc;
    }
    rc = run_room(false);
  } else if (kb.n && skipped_wide && !d.h_sc->packed) {
    d.pred_packed = false;  // a wide batch: nothing was aggregated, run it with every variant
    d.replays += 1;
    rc = run_room(opt);
  }
  const uint64_t groups = d.h_sc->scratch[0];
  if (kb.n && d.use_part && !(sql && (d.h_sc->redo || sql_refused))) {
    d.pred_packed = d.h_sc->packed != 0;
    const uint64_t how = d.h_sc->scratch[2];  // 1/2 lean, 3/4 deferred; odd: changelog written directly
    d.pred_direct = how == 1 || how == 3;
    // next batch's table room: twice this batch's new-group bound (its partials)
    const uint64_t parts = d.h_sc->scratch[31];
    d.lean_pred = (how == 1 || how == 2) ? (2 * parts > (1ull << 16) ? 2 * parts : (1ull << 16)) : 0;
    // and for a deferred (hopping) batch: twice its new groups plus twice its
    // in-kernel window updates (k_part_agg's touched-list entries, the claims
    // no room check covers); k_seg_apply checks the deferred ones itself
    const uint64_t grew = d.h_sc->live > live0 ? d.h_sc->live - live0 : 0;
    const uint64_t dfr = 2 * grew + 2 * d.h_sc->scratch[1];
    if (how == 3 || how == 4) d.defer_pred = dfr > (1ull << 16) ? dfr : (1ull << 16);
    d.lean_batches += how == 1 || how == 2;
    d.direct_batches += how == 1 || how == 3;
  }
  const uint64_t how = d.h_sc->scratch[2];
  if (rc == HSG_OK && kb.n && skipped_emit && how != 1 && how != 3 && (d.h_sc->scratch[1] | d.h_sc->scratch[6])) {
    // the touched list was filled: the emit chain that was not launched runs on
    // it (its lengths, scratch[1] / [6], back on the device)
    d.replays += 1;
    PushResult r1 = r;
    DTRY(hipMemcpyAsync(&d.sc->scratch[1], &d.h_sc->scratch[1], 6 * 8, hipMemcpyHostToDevice, d.stream));
    d.sc_clean = false;
    launch_part_emit(d.stream, d.tw, prog, p, d.part, d.out, a.pending, d.out_cap, d.sc);
    DTRY(hipEventRecord(d.ev_b, d.stream));
    rc = finish_batch(d, a.wm_in, kb.n, r1, err);
    r.out_rows = r1.out_rows;
    if (rc != HSG_OK) return rc;
  }
  if (kb.n) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, d.ev_a, d.ev_b) == hipSuccess) r.agg_ms = ms;
    r.agg_launches = 1;
    if (d.use_part) adapt_partitions(d, cfg, prog, groups, kb.n);
    if (sql_ovf) {
      const int want = np_refused + 1 < kPartMaxLog2 ? np_refused + 1 : kPartMaxLog2;
      if (d.np_log2 < want) d.np_log2 = want;
      // already at the most buckets: give the lean SQL kernels a rest
      if (np_refused >= kPartMaxLog2) d.sql_skip = 16;
    }
  }
  r.touched = cfg.emit_mode == HSG_EMIT_PER_BATCH ? r.out_rows : d.h_sc->scratch[0];
  return rc;
}

// New groups to make room for ahead of a batch. The partition path's kernels
// check their own bound against the room left and hold back past it
// (push_time_atomic), so a lean-eligible op is sized for twice the partials
// of its last lean batch (none before its first: the batch's own check grows
// the table) rather than for one new group per (record, window); every other
// path gets that worst case.
static uint64_t table_bound_hint(const OpDevice &d, const hsg_op_config &cfg, const Program &prog) {
  // hopping: twice the last batch's window updates (k_part_agg's own and the
  // deferred ones: a superset of its new groups); the first batch, whose
  // in-kernel updates have no check of their own, gets the worst case
  if (defer_room_checked(d, cfg, prog)) return d.defer_pred ? d.defer_pred : UINT64_MAX;
  if (d.sql_lean) return cfg.grace_ms >= 0 ? d.lean_pred : UINT64_MAX;  // k_sql_apply checks its partials
  if (!d.use_part || has_last(prog) || cfg.emit_mode == HSG_EMIT_PER_RECORD || cfg.grace_ms < 0 ||
      cfg.window_kind == HSG_SESSION || cfg.n_cols > 8 || d.wpr >= 256)
    return UINT64_MAX;
  PartParams q;
  memset(&q, 0, sizeof(q));
  q.pane_S = d.pane_S;
  q.rbits = d.rbits;
  q.words = part_words(cfg.n_cols, false);
  return part_lean_eligible(prog, q) ? d.lean_pred : UINT64_MAX;
}

int op_push(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, PushResult &r,
            std::string &err) {
  const hsg_batch *b = a.batch;
  // room in the table for the batch's worst case (sharded ops: in push_local,
  // once the records this rank owns are known)
  if (!a.comm) {
    int rc = tw_maintain(d, cfg, prog, b->n, a.wm_in, a.pending, err, table_bound_hint(d, cfg, prog));
    if (rc != HSG_OK) return rc;
  }
  // the changelog must have room for the worst case of this batch (sharded
  // ops: decided after the all-gather, from the records each rank will own and
  // every rank's room, uniformly on all ranks -- exchange.cpp check_room)
  if (cfg.emit_mode != HSG_EMIT_NONE && !a.comm) {
    uint64_t bound = b->n * d.wpr;
    if (cfg.emit_mode == HSG_EMIT_PER_BATCH && cfg.window_kind != HSG_SESSION && bound > d.cap) bound = d.cap;
    if (a.pending + bound > d.out_cap) {
      err = "changelog buffer full: drain before pushing (out_capacity)";
      return HSG_E_CAPACITY;
    }
  }
  if (a.comm) return push_sharded(d, cfg, prog, a, r, err);
  Batch kb;
  int rc = stage_batch(d, b, kb, err, a.staged_set);
  if (rc != HSG_OK) return rc;
  r.owned = kb.n;
  r.global_records = kb.n;
  return push_local(d, cfg, prog, a, kb, nullptr, nullptr, r, err);
}

// Aggregate an already-staged (and, for multi-GPU, already-exchanged) batch.
// seq / rec_wm, when given, carry each record's global sequence number and the
// watermark it saw in the global arrival order (computed before the exchange).
int push_local(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, const Batch &kb,
               const int64_t *seq, const int64_t *rec_wm, PushResult &r, std::string &err) {
  if (cfg.window_kind == HSG_SESSION) return push_session(d, cfg, prog, a, kb, seq, r, err);
  if (a.comm) {
    int rc = tw_maintain(d, cfg, prog, kb.n, a.wm_in, a.pending, err);
    if (rc != HSG_OK) return rc;
  }
  if (cfg.emit_mode == HSG_EMIT_PER_RECORD) return push_time_perrecord(d, cfg, prog, a, kb, seq, rec_wm, r, err);
  return push_time_atomic(d, cfg, prog, a, kb, seq, rec_wm, r, err);
}

int op_copy_rows(OpDevice &d, const OutCols &src, uint64_t from, uint64_t n, int n_aggs, const hsg_rows *out,
                 std::string &err, uint64_t dst_off) {
  if (n == 0) return HSG_OK;
  const uint64_t o = dst_off;
  uint32_t *key = out->key_id ? (uint32_t *)out->key_id + o : nullptr;
  int64_t *ws = out->win_start ? out->win_start + o : nullptr;
  int64_t *we = out->win_end ? out->win_end + o : nullptr;
  int64_t *si = out->src_index ? out->src_index + o : nullptr;
  RowPtrs ap;
  memset(&ap, 0, sizeof(ap));
  for (int j = 0; j < n_aggs && out->aggs; ++j) ap.p[j] = out->aggs[j] ? (int64_t *)out->aggs[j] + o : nullptr;
  uint32_t *fm = out->form ? out->form + o : nullptr;
  if (out->mem == HSG_MEM_DEVICE) {
    // device-resident destination: every column in one launch
    launch_copy_rows(d.stream, src, from, n, n_aggs, key, ws, we, si, ap, fm);
    DTRY(hipGetLastError());
    DTRY(hipStreamSynchronize(d.stream));
    return HSG_OK;
  }
  hipMemcpyKind k = hipMemcpyDeviceToHost;
  if (key) DTRY(hipMemcpyAsync(key, src.key + from, n * 4, k, d.stream));
  if (ws) DTRY(hipMemcpyAsync(ws, src.ws + from, n * 8, k, d.stream));
  if (we) DTRY(hipMemcpyAsync(we, src.we + from, n * 8, k, d.stream));
  if (si) DTRY(hipMemcpyAsync(si, src.src + from, n * 8, k, d.stream));
  for (int j = 0; j < n_aggs; ++j)
    if (ap.p[j]) DTRY(hipMemcpyAsync(ap.p[j], src.agg[j] + from, n * 8, k, d.stream));
  if (fm && src.form) DTRY(hipMemcpyAsync(fm, src.form + from, n * 4, k, d.stream));
  else if (fm) memset(fm, 0, n * 4);
  DTRY(hipStreamSynchronize(d.stream));
  return HSG_OK;
}

// A dump lists the rows in (key, window start, window end) order, the order of
// the reference's ordered stores (ksDump / ssDump over Data.Map, Store.hs:81,
// 238-241), independent of where the rows sit in the HBM table. Host-side
// permutation of the caller's columns (views are read back rarely; the rows
// of a device-memory dump make one round trip).
// The same order on the device, for a device-memory dump of time windows
// (views of large states: C3's 731M rows would take minutes on the host): the
// rows' window index (32 bits relative to the epoch, HSG_E_RANGE keeps it
// there) then the key, two stable LSD radix sorts of (u32, row) pairs, every
// column gathered through the permutation. Rows of one (key, window) are one
// row, so the order is the host sort's.
static int sort_dump_rows_device(OpDevice &d, const hsg_op_config &cfg, const hsg_rows *out, uint64_t n, int n_aggs,
                                 std::string &err) {
  struct Tmp {
    void *p = nullptr;
    ~Tmp() {
      if (p) hipFree(p);
    }
  } scratch, gat;
  const uint64_t sb = sort_scratch_bytes(n);
  DTRY(hipMalloc(&scratch.p, 4 * n * 4 + sb + 256));
  DTRY(hipMalloc(&gat.p, n * 8));
  uint32_t *k0 = (uint32_t *)scratch.p, *v0 = k0 + n, *k1 = v0 + n, *v1 = k1 + n;
  void *ss = (void *)(((uintptr_t)(v1 + n) + 255) & ~(uintptr_t)255);
  const int64_t adv = cfg.window_kind == HSG_UNWINDOWED ? 0
                      : cfg.window_kind == HSG_HOPPING  ? cfg.advance_ms
                                                        : cfg.size_ms;
  launch_dump_keys(d.stream, out->win_start, n, adv, d.h_sc->k_epoch, k0, v0);
  uint32_t *perm = v0;
  if (adv > 0) {
    const int w = radix_sort_pairs(d.stream, k0, v0, k1, v1, n, 32, ss);
    perm = w ? v1 : v0;
  }
  // keys in window order, then a stable sort by key
  uint32_t *kk = perm == v0 ? k1 : k0, *kv = perm == v0 ? v1 : v0;
  launch_gather_u32(d.stream, out->key_id, perm, n, kk);
  hipMemcpyAsync(kv, perm, n * 4, hipMemcpyDeviceToDevice, d.stream);
  uint32_t *ok = perm == v0 ? k0 : k1, *ov = perm == v0 ? v0 : v1;  // (ok, ov) the free pair
  const int w2 = radix_sort_pairs(d.stream, kk, kv, ok, ov, n, 32, ss);
  const uint32_t *fin = w2 ? ov : kv;
  // every column through the permutation (a column at a time through gat)
  auto col = [&](void *c, int bytes) -> int {
    if (!c) return HSG_OK;
    if (bytes == 4) launch_gather_u32(d.stream, (const uint32_t *)c, fin, n, (uint32_t *)gat.p);
    else launch_gather_u64(d.stream, (const uint64_t *)c, fin, n, (uint64_t *)gat.p);
    DTRY(hipMemcpyAsync(c, gat.p, n * (uint64_t)bytes, hipMemcpyDeviceToDevice, d.stream));
    return HSG_OK;
  };
  int rc = col(out->key_id, 4);
  if (rc == HSG_OK) rc = col(out->win_start, 8);
  if (rc == HSG_OK) rc = col(out->win_end, 8);
  if (rc == HSG_OK) rc = col(out->src_index, 8);
  for (int j = 0; rc == HSG_OK && j < n_aggs && out->aggs; ++j) rc = col(out->aggs[j], 8);
  if (rc == HSG_OK) rc = col(out->form, 4);
  if (rc != HSG_OK) return rc;
  DTRY(hipGetLastError());
  DTRY(hipStreamSynchronize(d.stream));
  return HSG_OK;
}

static int sort_dump_rows(OpDevice &d, const hsg_rows *out, uint64_t n, int n_aggs, std::string &err) {
  if (n < 2) return HSG_OK;
  const bool dev = out->mem == HSG_MEM_DEVICE;
  const hipMemcpyKind d2h = hipMemcpyDeviceToHost, h2d = hipMemcpyHostToDevice;
  std::vector<uint32_t> key(n), form(out->form ? n : 0);
  std::vector<int64_t> ws(n), we(n);
  std::vector<std::vector<int64_t>> cols;  // src + aggs, 8-byte words
  std::vector<int64_t *> ptrs;
  if (out->src_index) ptrs.push_back(out->src_index);
  for (int j = 0; j < n_aggs && out->aggs; ++j)
    if (out->aggs[j]) ptrs.push_back((int64_t *)out->aggs[j]);
  auto fetch = [&](void *dst, const void *src, uint64_t bytes) -> int {
    if (dev) DTRY(hipMemcpy(dst, src, bytes, d2h));
    else memcpy(dst, src, bytes);
    return HSG_OK;
  };
  auto store = [&](void *dst, const void *src, uint64_t bytes) -> int {
    if (dev) DTRY(hipMemcpy(dst, src, bytes, h2d));
    else memcpy(dst, src, bytes);
    return HSG_OK;
  };
  if (!out->key_id || !out->win_start || !out->win_end) return HSG_OK;  // nothing to order by
  int rc = fetch(key.data(), out->key_id, n * 4);
  if (rc == HSG_OK) rc = fetch(ws.data(), out->win_start, n * 8);
  if (rc == HSG_OK) rc = fetch(we.data(), out->win_end, n * 8);
  if (rc == HSG_OK && out->form) rc = fetch(form.data(), out->form, n * 4);
  cols.resize(ptrs.size());
  for (size_t c = 0; rc == HSG_OK && c < ptrs.size(); ++c) {
    cols[c].resize(n);
    rc = fetch(cols[c].data(), ptrs[c], n * 8);
  }
  if (rc != HSG_OK) return rc;
  std::vector<uint64_t> ord(n);
  for (uint64_t i = 0; i < n; ++i) ord[i] = i;
  std::stable_sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
    if (key[a] != key[b]) return key[a] < key[b];
    if (ws[a] != ws[b]) return ws[a] < ws[b];
    return we[a] < we[b];
  });
  auto permute = [&](auto &v) {
    auto tmp = v;
    for (uint64_t i = 0; i < n; ++i) v[i] = tmp[ord[i]];
  };
  permute(key);
  permute(ws);
  permute(we);
  if (out->form) permute(form);
  for (auto &c : cols) permute(c);
  rc = store(out->key_id, key.data(), n * 4);
  if (rc == HSG_OK) rc = store(out->win_start, ws.data(), n * 8);
  if (rc == HSG_OK) rc = store(out->win_end, we.data(), n * 8);
  if (rc == HSG_OK && out->form) rc = store(out->form, form.data(), n * 4);
  for (size_t c = 0; rc == HSG_OK && c < ptrs.size(); ++c) rc = store(ptrs[c], cols[c].data(), n * 8);
  (void)d;
  return rc;
}

int op_dump(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const hsg_rows *out, uint64_t *n_out,
            std::string &err) {
  wait_table_reset(d);
  int rc = fetch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  uint64_t live = d.h_sc->live;
  *n_out = 0;
  if (live == 0) return tw_dump_spilled(d, cfg, prog, out, 0, n_out, err);
  OutCols tmp;
  memset(&tmp, 0, sizeof(tmp));
  rc = alloc_out(tmp, live, cfg.n_aggs, err, d.forms);
  if (rc == HSG_OK) {
    uint64_t *counter = nullptr;
    if (hipMalloc((void **)&counter, 8) != hipSuccess) {
      free_out(tmp);
      err = "hipMalloc counter";
      return HSG_E_DEVICE;
    }
    hipMemsetAsync(counter, 0, 8, d.stream);
    if (cfg.window_kind == HSG_SESSION) {
      launch_session_dump(d, cfg, prog, tmp, live, counter);
    } else {
      PushArgs a;
      TwParams p = make_tw_params(cfg, a);
      launch_tw_emit(d.stream, d.tw, d.tw.slots(), prog, p, 1, tmp, 0, live, d.sc, d.emit, counter);
    }
    uint64_t got = 0;
    hipMemcpyAsync(&got, counter, 8, hipMemcpyDeviceToHost, d.stream);
    hipError_t e = hipStreamSynchronize(d.stream);
    hipFree(counter);
    if (e != hipSuccess) {
      free_out(tmp);
      err = std::string("dump: ") + hipGetErrorString(e);
      return HSG_E_DEVICE;
    }
    if (got > live) got = live;
    rc = op_copy_rows(d, tmp, 0, got, cfg.n_aggs, out, err);
    *n_out = got;
  }
  free_out(tmp);
  if (rc == HSG_OK && cfg.window_kind != HSG_SESSION) {
    // closed windows kept on the host (retention.cpp) follow the resident rows
    uint64_t more = 0;
    rc = tw_dump_spilled(d, cfg, prog, out, *n_out, &more, err);
    *n_out += more;
  }
  if (rc == HSG_OK) {
    const bool dev_sort = out->mem == HSG_MEM_DEVICE && cfg.window_kind != HSG_SESSION && *n_out >= (1ull << 20) &&
                          *n_out < 0xFFFFFFFFull && out->key_id && out->win_start && out->win_end;
    rc = dev_sort ? sort_dump_rows_device(d, cfg, out, *n_out, cfg.n_aggs, err)
                  : sort_dump_rows(d, out, *n_out, cfg.n_aggs, err);
  }
  return rc;
}

}  // namespace hsg
