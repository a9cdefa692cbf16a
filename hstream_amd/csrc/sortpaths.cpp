// Host orchestration of the exact per-record changelog of time windows (and
// the scratch it shares with the session replay path).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "hsg_kernels.h"
#include "hsg_part.h"
#include "hsg_perrecord.h"
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

static int log2u(uint64_t v) {
  int l = 0;
  while ((1ull << l) < v) ++l;
  return l;
}

// bump allocator over one device block
struct Carve {
  char *base;
  uint64_t used = 0;
  template <typename T>
  T *take(uint64_t count) {
    used = (used + 255) & ~255ull;
    T *p = (T *)(base ? base + used : nullptr);
    used += (count ? count : 1) * sizeof(T);
    return p;
  }
};

static void carve_layout(Carve &c, PrBuffers &pb, uint64_t n, uint64_t P, uint64_t shadow_words) {
  uint64_t nseg = seg_tiles(P) + 1;
  uint64_t scan_n = n > P ? n : P;
  pb.cnt = c.take<uint32_t>(n);
  pb.off = c.take<uint64_t>(n + 1);
  pb.pslot = c.take<uint32_t>(P);
  pb.pidx = c.take<uint32_t>(P);
  pb.k1 = c.take<uint32_t>(P);
  pb.v1 = c.take<uint32_t>(P);
  pb.prec = c.take<uint32_t>(P);
  pb.shadow = c.take<int64_t>(shadow_words);
  pb.blk_v = c.take<int64_t>(nseg * kMaxSlots);
  pb.blk_f = c.take<int32_t>(nseg);
  pb.carry = c.take<int64_t>(nseg * kMaxSlots);
  pb.partial = c.take<uint64_t>(scan_partials_needed(scan_n) + 8);
  pb.totals = c.take<uint64_t>(8);
  pb.flags = c.take<uint8_t>(P);
  pb.runs = c.take<uint32_t>(n + 1);
  pb.runidx = c.take<uint64_t>(n + 1);
  pb.sort_scratch = c.take<char>(sort_scratch_bytes(P));
  pb.max_pairs = P;
}

int perrecord_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err) {
  const uint64_t n = d.batch_cap;
  const uint64_t P = n * d.wpr;
  if (P >= 0xFFFFFFFFull) {
    err = "batch_capacity x windows per record must be < 2^32 for the per-record / session paths";
    return HSG_E_INVALID;
  }
  if (d.tw.slots() > 0x7FFFFFFFull) {
    err = "state table too large for the sort-based paths (max 2^31 slots)";
    return HSG_E_INVALID;
  }
  uint64_t shadow = cfg.window_kind == HSG_SESSION ? 0 : d.tw.slots() * (uint64_t)prog.n_slots;
  Carve probe{nullptr};
  PrBuffers tmp;
  carve_layout(probe, tmp, n, P, shadow);
  DTRY(hipMalloc(&d.scratch, probe.used));
  d.scratch_bytes = probe.used;
  Carve real{(char *)d.scratch};
  carve_layout(real, d.pr, n, P, shadow);
  if (!d.h_tmp) DTRY(hipHostMalloc((void **)&d.h_tmp, 8 * sizeof(uint64_t), hipHostMallocDefault));
  return HSG_OK;
}

// ---------------------------------------------------------------------------
// Per-record changelog on the partitioned pipeline (k_prpart.hip): ops with
// <= 8 state slots and < 256 windows per record. Others: the sort path below.
// ---------------------------------------------------------------------------
// LAST, or literal-form slots: the records' sequence words (global seq +
// literal bits) ride in the partitioned records
static bool has_last_slot(const Program &prog) { return prog_part_seq(prog); }

// the per-record kernels fold with the full slot algebra (combine_row: the
// LAST pair, tie words, literal-form slots), up to 16 slots
bool perrecord_part_eligible(const Program &prog, uint64_t wpr) { return prog.n_slots <= 16 && wpr < 256; }

int perrecord_part_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err) {
  int rc = part_device_init(d, cfg, prog, err);
  if (rc != HSG_OK) return rc;
  const uint64_t n = d.batch_cap, wpr = d.wpr ? d.wpr : 1, P = n * wpr, ns = (uint64_t)prog.n_slots;
  if (P >= 0xFFFFFFFFull) {
    err = "batch_capacity x windows per record must be < 2^32 for the per-record changelog";
    return HSG_E_INVALID;
  }
  const uint64_t tiles = part_tiles(n, kPartTileRecs) + 2;
  const uint64_t chunks = (1ull << kPartMaxLog2) + n / (kPrPairs / wpr) + 2;
  auto layout = [&](Carve &c, PrPart &x) {
    x.tpairs = c.take<uint32_t>(tiles);
    x.tpoff = c.take<uint64_t>(tiles + 1);
    x.pos = c.take<uint32_t>(n);
    x.inter = c.take<uint64_t>(P * (1 + ns));
    x.gkey = c.take<uint64_t>(P);
    x.part = c.take<int64_t>(P * ns);
    x.cbase = c.take<uint32_t>(chunks);
    x.ccnt = c.take<uint32_t>(chunks);
    x.counter = c.take<uint64_t>(8);
    x.partial = c.take<uint64_t>(scan_partials_needed(tiles) + 8);
    x.fin = c.take<int64_t>(wpr == 1 ? n * (uint64_t)prog_fin_words(prog) : 1);
    x.krec = c.take<uint64_t>(wpr == 1 ? 1 : n * (uint64_t)part_words(cfg.n_cols, true));
    x.kpos = c.take<uint32_t>(wpr == 1 ? 1 : n);
    x.roff = c.take<uint64_t>(wpr == 1 ? 1 : n);
  };
  Carve probe{nullptr};
  PrPart tmp;
  layout(probe, tmp);
  DTRY(hipMalloc(&d.scratch, probe.used));
  d.scratch_bytes = probe.used;
  Carve real{(char *)d.scratch};
  layout(real, d.prp);
  d.part.tpairs = d.prp.tpairs;
  d.part.pos = d.prp.pos;
  d.pr_part = true;
  return HSG_OK;
}

// buckets of about four chunks: k_pr_carry walks a bucket's chunks in order,
// and k_pr_emit's gathers read runs of (records per emit tile / buckets)
static int pr_buckets_log2(uint64_t n, uint64_t chunk) {
  const uint64_t want = n / (4 * chunk);
  int l = 0;
  while ((1ull << l) < want && l < kPartMaxLog2) ++l;
  return l < 4 ? 4 : l;
}

static int push_time_perrecord_part(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                                    const Batch &kb, const int64_t *seq, const int64_t *rec_wm, PushResult &r,
                                    std::string &err) {
  TwParams p = make_tw_params(cfg, a);
  const uint32_t wpr = (uint32_t)(d.wpr ? d.wpr : 1);
  // optimistic: the histogram assumes no record is late and the decide step
  // checks it on the device (as the per-batch pipeline, op_device.cpp); a
  // batch with late records runs again with per-record stream time
  const bool opt = !rec_wm && cfg.grace_ms >= 0;
  const bool need_epoch = !d.h_sc->epoch_set;
  const bool last = has_last_slot(prog);
  auto run = [&](bool optimistic) -> int {
    int rc = clear_batch_scalars(d, err);
    if (rc != HSG_OK) return rc;
    if (!kb.n) return HSG_OK;
    if (!optimistic) launch_stream_time(d, cfg, kb, a.wm_in, p.adv);
    else if (need_epoch) launch_epoch_first(d.stream, kb, p.adv, d.sc);
    DTRY(hipEventRecord(d.ev_a, d.stream));
    PartParams pp;
    memset(&pp, 0, sizeof(pp));
    pp.chunk = kPrPairs / wpr;
    // one-window ops: a workgroup walks each bucket (k_pr_bucket), as many
    // buckets as the partition makes; else buckets of a few k_pr_local chunks
    // (multi-window: ~2048 records per bucket, ~128 keys for k_pr_keys' waves)
    pp.np_log2 = pr_buckets_log2(kb.n, wpr == 1 ? 1024 : 512);
    pp.bshift = d.bshift;
    for (int c = 0; c < cfg.n_cols; ++c) pp.has_valid |= kb.valid[c] != nullptr;
    pp.has_seq = last ? 1 : 0;
    pp.words = part_words(cfg.n_cols, last);
    pp.tile = part_tile_for(pp.words);
    pp.sub = 1;
    pp.tiles = part_tiles(kb.n, pp.tile);
    pp.pane_S = 1;
    if (!rec_wm && !optimistic) launch_part_recwm(d.stream, kb, d.tile_prefix, d.sc, d.part.wm);
    launch_part_hist(d.stream, kb, p, pp, rec_wm, d.part.wm, d.part, d.sc, optimistic);
    const bool can_pack = optimistic && cfg.n_cols <= 8 && wpr < 256;
    if (optimistic)
      launch_part_decide_offsets(d.stream, d.sc, p, a.wm_in, cfg.grace_ms, can_pack, pp, d.part);
    else
      launch_part_offsets(d.stream, pp, d.part, d.sc);
    // each tile's first changelog row; the batch's rows in sc->out_rows
    scan_excl_u32(d.stream, d.prp.tpairs, d.prp.tpoff, pp.tiles, d.prp.partial, &d.sc->out_rows);
    launch_part_scatter(d.stream, kb, p, pp, rec_wm, d.part.wm, seq, d.part, d.sc, can_pack, true);
    wait_table_reset(d);  // the passes above do not touch the table
    DTRY(hipMemsetAsync(d.prp.counter, 0, 16, d.stream));
    // HSG_PR_CHUNKED=1: multi-window batches take the chunked path (k_pr_local /
    // k_pr_carry / k_pr_emit) even when every bucket fits the key sort (tests, A/B)
    static const bool chunked = getenv("HSG_PR_CHUNKED") != nullptr;
    if (wpr != 1 && chunked) DTRY(hipMemsetAsync(d.prp.counter + 1, 1, 1, d.stream));
    launch_part_chunks(d.stream, pp, d.part, d.sc);  // (one-window ops: for a hot bucket's chunked path)
    launch_pr_part(d.stream, kb, prog, p, pp, d.tw, d.part, d.prp, wpr, rec_wm, seq, d.out, a.pending, d.out_cap,
                   d.sc);
    DTRY(hipEventRecord(d.ev_b, d.stream));
    DTRY(hipGetLastError());
    return HSG_OK;
  };
  int rc = run(opt);
  if (rc != HSG_OK) return rc;
  rc = finish_batch(d, a.wm_in, kb.n, r, err);
  if (opt && kb.n && d.h_sc->redo) {
    rc = run(false);
    if (rc != HSG_OK) return rc;
    rc = finish_batch(d, a.wm_in, kb.n, r, err);
  }
  r.pairs = r.out_rows;
  if (kb.n) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, d.ev_a, d.ev_b) == hipSuccess) r.agg_ms = ms;
    r.agg_launches = 1;
  }
  return rc;
}

int push_time_perrecord(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                        const Batch &kb, const int64_t *seq, const int64_t *rec_wm, PushResult &r, std::string &err) {
  if (d.pr_part) return push_time_perrecord_part(d, cfg, prog, a, kb, seq, rec_wm, r, err);
  wait_table_reset(d);
  TwParams p = make_tw_params(cfg, a);
  int rc = clear_batch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  uint64_t P = 0;
  if (kb.n) {
    PrBuffers &pb = d.pr;
    launch_stream_time(d, cfg, kb, a.wm_in, p.adv);
    DTRY(hipEventRecord(d.ev_a, d.stream));
    launch_pr_count(d.stream, kb, p, d.tw, d.tile_prefix, rec_wm, pb, d.sc);
    scan_excl_u32(d.stream, pb.cnt, pb.off, kb.n, pb.partial, pb.totals);
    DTRY(hipMemcpyAsync(d.h_tmp, pb.totals, 8, hipMemcpyDeviceToHost, d.stream));
    DTRY(hipStreamSynchronize(d.stream));
    P = d.h_tmp[0];
    if (P > pb.max_pairs) {
      err = "internal: pair count exceeds scratch";
      return HSG_E_DEVICE;
    }
    if (P) {
      launch_pr_expand(d.stream, kb, p, d.tw, d.tile_prefix, rec_wm, pb, d.sc);
      int which = radix_sort_pairs(d.stream, pb.pslot, pb.pidx, pb.k1, pb.v1, P, log2u(d.tw.slots()) + 1, pb.sort_scratch);
      const uint32_t *slot = which ? pb.k1 : pb.pslot;
      const uint32_t *idx = which ? pb.v1 : pb.pidx;
      launch_pr_segscan(d.stream, kb, prog, pb, p, d.tw, slot, idx, P, seq, d.out, a.pending, d.sc);
    }
    DTRY(hipEventRecord(d.ev_b, d.stream));
    DTRY(hipGetLastError());
  }
  rc = finish_batch(d, a.wm_in, kb.n, r, err);
  r.out_rows = P;
  if (kb.n) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, d.ev_a, d.ev_b) == hipSuccess) r.agg_ms = ms;
    r.agg_launches = 1;
  }
  return rc;
}

}  // namespace hsg
