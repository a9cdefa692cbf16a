// Host orchestration of session windows (SessionWindowedStream.hs:74-118 over
// Store.hs:139-272): store allocation and growth, and the two batch paths of
// hsg_session.h (merge: partition + per-bucket sort / runs / sweep-merge;
// replay: per-key arrival-order replay for the per-record changelog and LAST).
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <cstring>
#include <string>

#include "hsg_kernels.h"
#include "hsg_part.h"
#include "hsg_perrecord.h"
#include "hsg_session.h"
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

static uint64_t pow2_at_least(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

static int log2u(uint64_t v) {
  int l = 0;
  while ((1ull << l) < v) ++l;
  return l;
}

// LAST, or literal-form slots: the records' global sequence numbers are needed
static bool has_last(const Program &prog) { return prog_needs_seq(prog); }

static int alloc_keys(SessTable &t, uint64_t kcap, std::string &err) {
  DTRY(hipMalloc((void **)&t.kt, kcap * sizeof(SessKey)));
  t.kmask = kcap - 1;
  t.kbits = log2u(kcap);
  return HSG_OK;
}

static void free_keys(SessTable &t) {
  if (t.kt) hipFree(t.kt);
  t.kt = nullptr;
}

static int alloc_arena(SessTable &t, uint64_t cap, std::string &err) {
  DTRY(hipMalloc((void **)&t.rows, cap * t.stride * sizeof(uint64_t)));
  t.arena_cap = cap;
  return HSG_OK;
}

static void free_arena(SessTable &t) {
  if (t.rows) hipFree(t.rows);
  t.rows = nullptr;
}

// Arena regions over the free rows [used, arena_cap): bump pointers and ends
// (hsg_session.h), written on the op's stream. The pinned staging words are
// the op's own (d.h_regions), never reused while a copy may be pending: the
// call synchronises the stream first.
static int set_regions(OpDevice &d, uint64_t used, std::string &err) {
  DTRY(hipStreamSynchronize(d.stream));
  const uint64_t cap = d.ss.arena_cap, per = (cap - used) / kArenaRegions;
  memset(d.h_regions, 0, kArenaRegions * kRegionStride * sizeof(uint64_t));
  for (int r = 0; r < kArenaRegions; ++r) {
    d.h_regions[r * kRegionStride] = used + (uint64_t)r * per;
    d.h_regions[r * kRegionStride + 1] = r + 1 == kArenaRegions ? cap : used + (uint64_t)(r + 1) * per;
  }
  DTRY(hipMemcpyAsync(d.ss.meta + M_RTOP, d.h_regions, kArenaRegions * kRegionStride * sizeof(uint64_t),
                      hipMemcpyHostToDevice, d.stream));
  DTRY(hipStreamSynchronize(d.stream));
  return HSG_OK;
}

// Session partition scratch (besides d.part's histogram, offsets and
// records): per-tile ts maxima, per-bucket progress and big flags, the touched
// list, the runs and key groups of k_ss_sort, the apply blocks' done flags.
static uint64_t ss_part_layout(uint64_t n, int words, SessPart *sp, char *m, bool br = false, uint32_t ns = 0) {
  uint64_t off = 0;
  auto take = [&](uint64_t bytes) {
    off = (off + 255) & ~255ull;
    const uint64_t o = off;
    off += bytes ? bytes : 1;
    return m ? m + o : nullptr;
  };
  const uint64_t tiles = part_tiles(n, kPartTileRecs) + 1, nb = 1ull << kPartMaxLog2;
  SessPart x;
  memset(&x, 0, sizeof(x));
  x.tmax = (uint64_t *)take(tiles * 8);
  x.progress = (uint32_t *)take(nb * 4);
  x.srec = (uint64_t *)take(n * (uint64_t)words * 8);
  if (br) {
    // bucket replay: its records (srec, with their arrival index), the
    // states by arrival index, the tiles' changelog offsets, the sub-buckets
    x.fin = (int64_t *)take(n * (2ull + ns) * 8);
    x.tkeyed = (uint32_t *)take(tiles * 4);
    x.toff = (uint64_t *)take((tiles + 1) * 8);
    x.tpartial = (uint64_t *)take((scan_partials_needed(tiles) + 8) * 8);
    x.subst = (uint32_t *)take(nb * 65 * 4);
    x.scopy = (uint64_t *)take(n * (uint64_t)words * 8);
    x.reloc = (uint64_t *)take(n * 24);
  } else {
    x.bigmask = (uint64_t *)take(nb * 8);
    x.touched = (uint32_t *)take(n * 4);
    x.groups = (uint32_t *)take(n * 16);
    x.done = (uint8_t *)take(n / 256 + 2);
    x.scopy = (uint64_t *)take(n * (uint64_t)words * 8);
    x.gsparse = (uint32_t *)take(n * 16);
    x.reloc = (uint64_t *)take(n * 24);
  }
  if (sp) *sp = x;
  return off;
}

static SessPart sess_part(OpDevice &d, int words, bool br = false) {
  SessPart sp;
  ss_part_layout(d.batch_cap, words, &sp, (char *)d.ss_part, br, d.ss.ns);
  sp.hist = d.part.hist;
  sp.offt = d.part.offt;
  sp.bstart = d.part.bstart;
  sp.rec = d.part.rec;
  return sp;
}

int session_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t rows, std::string &err) {
  SessTable &t = d.ss;
  memset(&t, 0, sizeof(t));
  t.ns = (uint32_t)prog.n_slots;
  t.stride = 3 + (uint32_t)prog.n_slots;
  // key table: keys <= sessions; grown by rehash as keys arrive (push_session)
  uint64_t kc = rows < d.batch_cap ? rows : d.batch_cap;
  const uint64_t kcap = pow2_at_least(2 * (kc > (1u << 14) ? kc : (1u << 14)));
  int rc = alloc_keys(t, kcap, err);
  if (rc != HSG_OK) return rc;
  d.cap = kcap;
  // arena: the expected live sessions, grown by compaction when a batch needs
  // more (the HSG_KNOB_SESS_ARENA_MIN testing knob: a smaller floor, so tests
  // reach the refills)
  uint64_t amin = 1u << 20;
  if (const int64_t v = testing_knob(HSG_KNOB_SESS_ARENA_MIN); v > 0) amin = (uint64_t)v;
  rc = alloc_arena(t, pow2_at_least(rows > amin ? rows : amin), err);
  if (rc != HSG_OK) return rc;
  DTRY(hipMalloc((void **)&t.meta, M_WORDS * sizeof(uint64_t)));
  DTRY(hipHostMalloc((void **)&d.h_meta, M_WORDS * sizeof(uint64_t), hipHostMallocDefault));
  DTRY(hipHostMalloc((void **)&d.h_regions, kArenaRegions * kRegionStride * sizeof(uint64_t), hipHostMallocDefault));
  // HSG_SS_REPLAY_ALL=1: per-batch / state-only ops on the bucket replay too (A/B)
  static const bool replay_all = getenv("HSG_SS_REPLAY_ALL") != nullptr;
  d.ss_merge = cfg.emit_mode != HSG_EMIT_PER_RECORD && !has_last(prog) && !prog_has_forms(prog) &&
               prog.n_slots <= 8 && !replay_all;
  rc = part_device_init(d, cfg, prog, err);
  if (rc != HSG_OK) return rc;
  if (d.ss_merge) {
    DTRY(hipMalloc(&d.ss_part, ss_part_layout(d.batch_cap, 2 + cfg.n_cols, nullptr, nullptr)));
  } else {
    // the bucket replay (the sort-based replay's buffers, perrecord_device_init,
    // stay for batches with a hot key)
    DTRY(hipMalloc(&d.ss_part, ss_part_layout(d.batch_cap, br_words(cfg.n_cols), nullptr, nullptr, true,
                                              (uint32_t)prog.n_slots)));
  }
  return HSG_OK;
}

int session_device_reset(OpDevice &d, std::string &err) {
  launch_ss_reset(d.stream, d.ss);
  DTRY(hipMemsetAsync(d.ss.meta, 0, M_WORDS * sizeof(uint64_t), d.stream));
  d.ss_keys = 0;
  return set_regions(d, 0, err);
}

void session_device_free(OpDevice &d) {
  free_keys(d.ss);
  free_arena(d.ss);
  if (d.ss.meta) hipFree(d.ss.meta);
  d.ss.meta = nullptr;
  if (d.h_meta) hipHostFree(d.h_meta);
  d.h_meta = nullptr;
  if (d.h_regions) hipHostFree(d.h_regions);
  d.h_regions = nullptr;
  if (d.ss_part) hipFree(d.ss_part);
  d.ss_part = nullptr;
}

// Key table with room for `incoming` more keys at load <= 1/2 (rehash).
static int ensure_keys(OpDevice &d, uint64_t incoming, std::string &err) {
  const uint64_t kcap = d.ss.kmask + 1;
  if (2 * (d.ss_keys + incoming) <= kcap) return HSG_OK;
  const uint64_t ncap = pow2_at_least(2 * (d.ss_keys + incoming) + 1);
  SessTable to = d.ss;
  to.kt = nullptr;
  int rc = alloc_keys(to, ncap, err);
  if (rc != HSG_OK) {
    free_keys(to);
    return rc;
  }
  launch_ss_rehash(d.stream, d.ss, to);
  DTRY(hipGetLastError());
  DTRY(hipStreamSynchronize(d.stream));
  free_keys(d.ss);
  d.ss.kt = to.kt;
  d.ss.kmask = to.kmask;
  d.ss.kbits = to.kbits;
  d.cap = ncap;
  d.grow_events += 1;
  return HSG_OK;
}

// Compact the arena into a fresh one with room for `extra` more sessions
// beyond the compacted lists (at least twice what they use). Between batches or
// between the passes of one batch: nothing is in flight on the stream.
static int refill_arena(OpDevice &d, const Program &prog, uint64_t extra, std::string &err) {
  SessTable &t = d.ss;
  const uint64_t kcap = t.kmask + 1;
  void *scratch = nullptr;
  DTRY(hipMalloc(&scratch, ss_compact_scratch_bytes(kcap)));
  launch_ss_compact_plan(d.stream, t, scratch, t.meta + M_SCRATCH);
  hipMemcpyAsync(d.h_meta + M_SCRATCH, t.meta + M_SCRATCH, 8, hipMemcpyDeviceToHost, d.stream);
  hipError_t e = hipStreamSynchronize(d.stream);
  if (e != hipSuccess) {
    hipFree(scratch);
    err = std::string("session compaction: ") + hipGetErrorString(e);
    return HSG_E_DEVICE;
  }
  const uint64_t used = d.h_meta[M_SCRATCH];
  uint64_t cap = t.arena_cap;
  while (cap < 2 * used + extra) cap <<= 1;
  SessTable to = t;
  to.rows = nullptr;
  int rc = alloc_arena(to, cap, err);
  if (rc != HSG_OK) {
    free_arena(to);
    hipFree(scratch);
    return rc;
  }
  launch_ss_compact_copy(d.stream, t, to, scratch);
  e = hipStreamSynchronize(d.stream);
  hipFree(scratch);
  if (e != hipSuccess) {
    free_arena(to);
    err = std::string("session compaction: ") + hipGetErrorString(e);
    return HSG_E_DEVICE;
  }
  free_arena(t);
  t.rows = to.rows;
  t.arena_cap = to.arena_cap;
  return set_regions(d, used, err);
}

static int finish_session_batch(OpDevice &d, int64_t wm_in, uint64_t n, PushResult &r, std::string &err) {
  DTRY(hipMemcpyAsync(d.h_meta, d.ss.meta, M_WORDS * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
  return finish_batch(d, wm_in, n, r, err);
}

static int clear_fail(OpDevice &d, std::string &err) {
  DTRY(hipMemsetAsync(d.ss.meta + M_FAIL, 0, sizeof(uint64_t), d.stream));
  DTRY(hipMemsetAsync(d.ss.meta + M_RNEED, 0, kArenaRegions * sizeof(uint64_t), d.stream));
  return HSG_OK;
}

// merge path: partition by key hash, per bucket sort / runs / key groups,
// one thread per key merges its runs into its sessions
static int push_session_merge(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                              const Batch &kb, PushResult &r, std::string &err) {
  const uint64_t n = kb.n;
  SessParams sp;
  sp.gap = cfg.gap_ms;
  sp.rec_base = a.rec_base;
  sp.batch_id = a.batch_id;
  sp.emit_mode = cfg.emit_mode;
  SessPart pt = sess_part(d, 2 + cfg.n_cols);
  const uint64_t tiles = part_tiles(n, kPartTileRecs);
  // buckets of about two sorts (k_ss_sort splits them in sub-buckets)
  int nl = log2u((n + 4095) / 4096);
  nl = nl < 4 ? 4 : (nl > kPartMaxLog2 ? kPartMaxLog2 : nl);
  bool has_valid = false;
  for (int c = 0; c < cfg.n_cols; ++c) has_valid = has_valid || kb.valid[c] != nullptr;
  const int words = 2 + cfg.n_cols;
  PartParams pp;
  memset(&pp, 0, sizeof(pp));
  pp.np_log2 = nl;
  pp.tiles = tiles;
  DTRY(hipEventRecord(d.ev_a, d.stream));
  DTRY(hipMemsetAsync(pt.progress, 0, (1ull << nl) * 4, d.stream));
  DTRY(hipMemsetAsync(pt.done, 0, n / 256 + 2, d.stream));
  launch_ss_phist(d.stream, kb, nl, d.bshift, tiles, pt);
  launch_ss_wm(d.stream, pt, tiles, a.wm_in, d.sc);
  launch_part_offsets(d.stream, pp, d.part, d.sc);
  launch_ss_pscatter(d.stream, kb, nl, d.bshift, tiles, words, has_valid, pt);
  launch_ss_sort(d.stream, sp, d.ss, prog, nl, d.bshift, words, pt, d.sc);
  // the key groups k_ss_sort found size the apply grid
  DTRY(hipMemcpyAsync(d.h_meta + M_GRP, d.ss.meta + M_GRP, sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
  DTRY(hipStreamSynchronize(d.stream));
  const uint64_t ngrp = d.h_meta[M_GRP];
  // a pass stops short (M_FAIL) only where the arena could not take a key's
  // fresh list: those apply blocks / big-bucket chunks were left untouched;
  // compact / grow the arena, then run the pass again (done work is skipped)
  for (int attempt = 0;; ++attempt) {
    launch_ss_apply(d.stream, sp, d.ss, prog, ngrp, words, pt, d.out, a.pending, d.sc);
    launch_ss_reloc_copy(d.stream, d.ss, pt, n);
    DTRY(hipMemsetAsync(d.ss.meta + M_RELOC, 0, sizeof(uint64_t), d.stream));
    launch_ss_merge_big(d.stream, sp, d.ss, prog, nl, d.bshift, words, pt, d.sc);
    DTRY(hipMemcpyAsync(d.h_meta, d.ss.meta, M_WORDS * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
    DTRY(hipStreamSynchronize(d.stream));
    DTRY(hipGetLastError());
    if (!d.h_meta[M_FAIL]) break;
    if (attempt >= 8) {
      err = "session arena: no room after compaction";
      return HSG_E_OOM;
    }
    int rc = refill_arena(d, prog, (2 * n) << attempt, err);
    if (rc != HSG_OK) return rc;
    rc = clear_fail(d, err);
    if (rc != HSG_OK) return rc;
  }
  launch_ss_emit(d.stream, d.ss, prog, pt, a.batch_id, cfg.emit_mode == HSG_EMIT_PER_BATCH ? 1 : 0, n, d.out,
                 a.pending, d.sc);
  DTRY(hipEventRecord(d.ev_b, d.stream));
  DTRY(hipGetLastError());
  int rc = finish_session_batch(d, a.wm_in, n, r, err);
  if (cfg.emit_mode == HSG_EMIT_PER_BATCH) r.touched = r.out_rows;
  else r.out_rows = 0;
  return rc;
}

// bucket replay (hsg_session.h): key-hash partition with the records'
// arrival indices, per bucket sub-buckets grouped by key in LDS and replayed
// one key per thread, the state after each record at its arrival index, the
// changelog written in arrival order. false in *done when a sub-bucket holds
// more than kBrCap records (a hot key): nothing was touched, the sort-based
// replay runs the batch.
static int push_session_bucket(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                               const Batch &kb, const int64_t *seq, PushResult &r, bool &done, std::string &err) {
  done = false;
  const uint64_t n = kb.n;
  SessParams sp;
  sp.gap = cfg.gap_ms;
  sp.rec_base = a.rec_base;
  sp.batch_id = a.batch_id;
  sp.emit_mode = cfg.emit_mode;
  const int words = br_words(cfg.n_cols);
  SessPart pt = sess_part(d, words, true);
  const uint64_t tiles = part_tiles(n, kPartTileRecs);
  // buckets of about 8 sub-buckets (k_br_replay's LDS holds kBrCap records)
  int nl = log2u((n + 4 * kBrCap - 1) / (4 * kBrCap));
  nl = nl < 4 ? 4 : (nl > kPartMaxLog2 ? kPartMaxLog2 : nl);
  PartParams pp;
  memset(&pp, 0, sizeof(pp));
  pp.np_log2 = nl;
  pp.tiles = tiles;
  DTRY(hipEventRecord(d.ev_a, d.stream));
  DTRY(hipMemsetAsync(pt.progress, 0, (1ull << nl) * 4, d.stream));
  launch_ss_phist(d.stream, kb, nl, d.bshift, tiles, pt);
  launch_ss_wm(d.stream, pt, tiles, a.wm_in, d.sc);
  launch_part_offsets(d.stream, pp, d.part, d.sc);
  launch_br_scatter(d.stream, kb, nl, d.bshift, tiles, words, pt);
  launch_br_subhist(d.stream, d.ss, nl, d.bshift, words, pt);
  scan_excl_u32(d.stream, pt.tkeyed, pt.toff, tiles, pt.tpartial, d.ss.meta + M_BRROWS);
  for (int attempt = 0;; ++attempt) {
    launch_br_replay(d.stream, kb, sp, d.ss, prog, nl, d.bshift, words, pt, seq, d.out, a.pending, d.sc);
    DTRY(hipMemcpyAsync(d.h_meta, d.ss.meta, M_WORDS * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
    DTRY(hipStreamSynchronize(d.stream));
    DTRY(hipGetLastError());
    if (d.h_meta[M_BRBIG]) return HSG_OK;  // (done stays false)
    // the moved lists' prefixes (listed by the sub-buckets that ran), before
    // anything else reads those lists: the next batch or a compaction
    if (d.h_meta[M_RELOC]) {
      launch_ss_reloc_copy(d.stream, d.ss, pt, n);
      DTRY(hipMemsetAsync(d.ss.meta + M_RELOC, 0, sizeof(uint64_t), d.stream));
    }
    if (!d.h_meta[M_FAIL]) break;
    if (attempt >= 8) {
      err = "session arena: no room after compaction";
      return HSG_E_OOM;
    }
    // regions are equal after compaction: room for the largest region's need in each
    uint64_t need = 0;
    for (int q = 0; q < kArenaRegions; ++q) need = d.h_meta[M_RNEED + q] > need ? d.h_meta[M_RNEED + q] : need;
    int rc = refill_arena(d, prog, (kArenaRegions * need + 2 * n) << attempt, err);
    if (rc != HSG_OK) return rc;
    rc = clear_fail(d, err);
    if (rc != HSG_OK) return rc;
  }
  if (cfg.emit_mode == HSG_EMIT_PER_RECORD)
    launch_br_emit(d.stream, kb, sp, prog, pt, tiles, seq, d.out, a.pending);
  DTRY(hipEventRecord(d.ev_b, d.stream));
  DTRY(hipGetLastError());
  done = true;
  int rc = finish_session_batch(d, a.wm_in, n, r, err);
  const uint64_t V = d.h_meta[M_BRROWS];
  if (cfg.emit_mode == HSG_EMIT_PER_RECORD) r.out_rows = V;
  else if (cfg.emit_mode == HSG_EMIT_PER_BATCH) r.touched = r.out_rows;
  r.pairs = V;
  return rc;
}

// replay path: stable sort by key slot, one thread per key replays its
// records in arrival order
static int push_session_replay(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                               const Batch &kb, const int64_t *seq, PushResult &r, std::string &err) {
  PrBuffers &pb = d.pr;
  const uint64_t n = kb.n;
  const uint32_t cap = (uint32_t)(d.ss.kmask + 1);
  SessParams sp;
  sp.gap = cfg.gap_ms;
  sp.rec_base = a.rec_base;
  sp.batch_id = a.batch_id;
  sp.emit_mode = cfg.emit_mode;
  launch_stream_time(d, cfg, kb, a.wm_in, 1);
  DTRY(hipEventRecord(d.ev_a, d.stream));
  launch_ss_slot(d.stream, kb, d.ss, pb.pslot, pb.pidx, pb.cnt, d.sc);
  scan_excl_u32(d.stream, pb.cnt, pb.off, n, pb.partial, pb.totals + 1);  // changelog positions, V
  const int which = radix_sort_pairs(d.stream, pb.pslot, pb.pidx, pb.k1, pb.v1, n, log2u(cap) + 1, pb.sort_scratch);
  const uint32_t *slot = which ? pb.k1 : pb.pslot;
  const uint32_t *ridx = which ? pb.v1 : pb.pidx;
  launch_ss_runs(d.stream, slot, n, cap, pb.flags, nullptr, nullptr, 0);
  scan_excl_u8(d.stream, pb.flags, pb.runidx, n, pb.partial, pb.totals + 2);  // R
  launch_ss_runs(d.stream, slot, n, cap, pb.flags, pb.runidx, pb.runs, 1);
  DTRY(hipMemcpyAsync(d.h_tmp, pb.totals, 4 * sizeof(uint64_t), hipMemcpyDeviceToHost, d.stream));
  DTRY(hipStreamSynchronize(d.stream));
  const uint64_t V = d.h_tmp[1];
  const uint64_t R = d.h_tmp[2];
  // runs[R] = V closes the last run (valid records sort before HSG_KEY_NONE)
  uint32_t *v32 = (uint32_t *)(d.h_tmp + 4);  // pinned
  *v32 = (uint32_t)V;
  DTRY(hipMemcpyAsync(pb.runs + R, v32, sizeof(uint32_t), hipMemcpyHostToDevice, d.stream));
  int rc = HSG_OK;
  for (int attempt = 0;; ++attempt) {
    launch_ss_replay_need(d.stream, d.ss, slot, pb.runs, R);
    launch_ss_process(d.stream, kb, sp, d.ss, prog, slot, ridx, pb.runs, R, pb.off, seq, d.out, a.pending, d.sc);
    DTRY(hipEventRecord(d.ev_b, d.stream));
    DTRY(hipGetLastError());
    rc = finish_session_batch(d, a.wm_in, n, r, err);
    if (rc != HSG_OK || !d.h_meta[M_FAIL] || attempt > 0) break;
    // not enough arena for the lists that grow: compact / grow, then again
    // regions are equal after compaction: room for the largest region's need in each
    uint64_t need = 0;
    for (int q = 0; q < kArenaRegions; ++q) need = d.h_meta[M_RNEED + q] > need ? d.h_meta[M_RNEED + q] : need;
    rc = refill_arena(d, prog, kArenaRegions * need + 2 * n, err);
    if (rc != HSG_OK) return rc;
    rc = clear_fail(d, err);
    if (rc != HSG_OK) return rc;
  }
  if (rc == HSG_OK && d.h_meta[M_FAIL]) {
    err = "session arena: no room after compaction";
    return HSG_E_OOM;
  }
  if (cfg.emit_mode == HSG_EMIT_PER_RECORD) r.out_rows = V;
  r.pairs = V;
  return rc;
}

int push_session(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, const Batch &kb,
                 const int64_t *seq, PushResult &r, std::string &err) {
  d.ss.hshift = d.bshift;  // fixed once the exchange is set up (before the first batch)
  int rc = clear_batch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  if (!kb.n) return finish_batch(d, a.wm_in, 0, r, err);
  rc = ensure_keys(d, kb.n, err);
  if (rc != HSG_OK) return rc;
  // per-batch words: need, fail, touched list, groups, runs, big buckets
  DTRY(hipMemsetAsync(d.ss.meta + M_FAIL, 0, (M_BRROWS - M_FAIL + 1) * sizeof(uint64_t), d.stream));
  DTRY(hipMemsetAsync(d.ss.meta + M_RNEED, 0, kArenaRegions * sizeof(uint64_t), d.stream));
  if (d.ss_merge) {
    rc = push_session_merge(d, cfg, prog, a, kb, r, err);
  } else {
    // HSG_SS_SORT_REPLAY=1: every batch on the sort-based replay (tests, A/B)
    static const bool sort_replay = getenv("HSG_SS_SORT_REPLAY") != nullptr;
    bool done = false;
    if (!sort_replay) rc = push_session_bucket(d, cfg, prog, a, kb, seq, r, done, err);
    if (rc == HSG_OK && !done) {
      d.replays += sort_replay ? 0 : 1;
      DTRY(hipMemsetAsync(d.ss.meta + M_FAIL, 0, (M_BRROWS - M_FAIL + 1) * sizeof(uint64_t), d.stream));
      rc = clear_batch_scalars(d, err);
      if (rc == HSG_OK) rc = push_session_replay(d, cfg, prog, a, kb, seq, r, err);
    }
  }
  if (d.ss_merge) r.pairs = kb.n;  // keyed records (HSG_KEY_NONE are counted too; stats only)
  d.ss_keys = d.h_meta[M_KEYS];
  float ms = 0;
  if (hipEventElapsedTime(&ms, d.ev_a, d.ev_b) == hipSuccess) r.agg_ms = ms;
  r.agg_launches = 1;
  return rc;
}

void launch_session_dump(OpDevice &d, const hsg_op_config &cfg, const Program &prog, OutCols out, uint64_t cap,
                         uint64_t *counter) {
  launch_ss_dump(d.stream, d.ss, prog, out, cap, counter);
}

}  // namespace hsg
