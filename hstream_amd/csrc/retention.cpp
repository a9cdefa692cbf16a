// Retention of the time-window table (tumbling / hopping / unwindowed).
//
// The reference's window store only grows: every (key, window) the
// aggregateProcessor ever wrote stays in the KV store and every view reads it
// back with ksDump (TimeWindowedStream.hs:96-100, Store.hs:81,
// hstream/src/HStream/Server/Handler.hs:273-315). HBM is bounded, so before a
// batch that could take the table past 3/4 load the op
//   * moves closed windows (end + grace <= stream time: no later record passes
//     the grace check of TimeWindowedStream.hs:92 for them, and stream time never
//     decreases, Processor/Internal.hs:156-159) to host memory as raw rows, and
//   * rebuilds the table from the open rows, doubling its capacity until those
//     rows plus the batch's worst case fit at load 1/2.
// The check happens before any kernel of the batch runs, so a batch never
// stops half applied for lack of room. hsg_dump_state appends the spilled
// rows (rendered by the same emit kernel as the resident ones), so views see
// the store the reference would hold. A caller that lowers the watermark below
// one a spill used (not something runTask does) gets every spilled row back in
// HBM before its batch, so the result stays exact.
//
// Sessions do not spill: any later record within the gap of a session's end
// merges with it (there is no grace for sessions, SessionWindowedStream.hs:84-118),
// so none is ever closed; their key table and arena grow instead (session.cpp).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "hsg_kernels.h"
#include "hsg_sort.h"
#include "hsg_ops.h"

namespace hsg {

#define DTRY(expr)                                                          \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) {                                                 \
      err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;          \
    }                                                                       \
  } while (0)

void tw_configure(TwTable &t, uint64_t cap, int window_kind, int region_log2) {
  t.mask = cap - 1;
  t.omask = tw_ovf_slots(cap) - 1;
  t.blocked = window_kind != HSG_UNWINDOWED && cap >= 64 ? 1u : 0u;
  // regions of >= 2^region_log2 slots (4096 unless overflow claims made the
  // op widen them: small spread of the per-region load), at most one per
  // partition bucket (hsg_tw.h)
  int cl = 0;
  while ((1ull << cl) < cap) ++cl;
  const int rb = cl - region_log2;
  t.rbits = rb < 0 ? 0 : (rb > kPartMaxLog2 ? kPartMaxLog2 : rb);
  t.rmask = (cap >> t.rbits) - 1;
}

void tw_retention_reset(OpDevice &d) {
  d.spill.clear();
  d.spill.shrink_to_fit();
  d.spilled_rows = 0;
  d.spill_wm = INT64_MIN;
}

static TwParams retention_params(const hsg_op_config &cfg, int64_t wm) {
  PushArgs a;
  a.wm_in = wm;
  return make_tw_params(cfg, a);
}

// Own changelog buffer large enough for a per-batch emission over the grown
// table (its rows were sized by the capacity at create); pending rows move.
static int grow_out(OpDevice &d, const hsg_op_config &cfg, uint64_t ncap, uint64_t pending, std::string &err) {
  if (d.ext_out || cfg.out_capacity || cfg.emit_mode != HSG_EMIT_PER_BATCH) return HSG_OK;
  uint64_t want = d.batch_cap * d.wpr;
  if (want > ncap) want = ncap;
  want += pending;
  if (want <= d.own_out_cap) return HSG_OK;
  OutCols n;
  memset(&n, 0, sizeof(n));
  auto alloc = [&](void **p, uint64_t bytes) { return hipMalloc(p, bytes ? bytes : 1); };
  hipError_t e = alloc((void **)&n.key, want * 4);
  if (e == hipSuccess) e = alloc((void **)&n.ws, want * 8);
  if (e == hipSuccess) e = alloc((void **)&n.we, want * 8);
  if (e == hipSuccess) e = alloc((void **)&n.src, want * 8);
  for (int j = 0; j < cfg.n_aggs && e == hipSuccess; ++j) e = alloc((void **)&n.agg[j], want * 8);
  if (d.forms && e == hipSuccess) e = alloc((void **)&n.form, want * 4);
  auto release = [](OutCols &o) {
    hipFree(o.key);
    hipFree(o.ws);
    hipFree(o.we);
    hipFree(o.src);
    for (int j = 0; j < kMaxAggs; ++j)
      if (o.agg[j]) hipFree(o.agg[j]);
    if (o.form) hipFree(o.form);
    memset(&o, 0, sizeof(o));
  };
  if (e != hipSuccess) {
    release(n);
    err = std::string("changelog buffer growth: ") + hipGetErrorString(e);
    return e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;
  }
  if (pending) {
    const hipMemcpyKind k = hipMemcpyDeviceToDevice;
    DTRY(hipMemcpyAsync(n.key, d.own_out.key, pending * 4, k, d.stream));
    DTRY(hipMemcpyAsync(n.ws, d.own_out.ws, pending * 8, k, d.stream));
    DTRY(hipMemcpyAsync(n.we, d.own_out.we, pending * 8, k, d.stream));
    DTRY(hipMemcpyAsync(n.src, d.own_out.src, pending * 8, k, d.stream));
    for (int j = 0; j < cfg.n_aggs; ++j) DTRY(hipMemcpyAsync(n.agg[j], d.own_out.agg[j], pending * 8, k, d.stream));
    if (n.form && d.own_out.form) DTRY(hipMemcpyAsync(n.form, d.own_out.form, pending * 4, k, d.stream));
  }
  DTRY(hipStreamSynchronize(d.stream));
  release(d.own_out);
  d.own_out = n;
  d.own_out_cap = want;
  d.out = n;
  d.out_cap = want;
  return HSG_OK;
}

int tw_maintain(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t n_in, int64_t wm_in,
                uint64_t pending, std::string &err, uint64_t groups_bound) {
  if (cfg.window_kind == HSG_SESSION || !d.tw.rows) return HSG_OK;
  const bool reopen = d.spilled_rows && wm_in < d.spill_wm;
  const uint64_t live = d.h_sc->live;
  // new groups of the batch: one per (record, window) at worst, or the bound
  // of a batch whose apply checks its room (op_device.cpp push_time_atomic)
  const uint64_t bound = n_in * d.wpr < groups_bound ? n_in * d.wpr : groups_bound;
  // a region was full (overflow rows in use): rebuild with larger regions
  const bool widen = d.ovf_rows != 0;
  if (!reopen && !widen && 8 * (live + bound) <= (uint64_t)d.load8 * d.cap) return HSG_OK;
  wait_table_reset(d);
  const TwParams p = retention_params(cfg, wm_in);
  // small pinned block for the counters read back here
  uint64_t *h = nullptr;
  DTRY(hipHostMalloc((void **)&h, 4 * sizeof(uint64_t), hipHostMallocDefault));
  struct HostFree {
    uint64_t *p;
    ~HostFree() { hipHostFree(p); }
  } hf{h};
  struct DevFree {
    void *p = nullptr;
    ~DevFree() {
      if (p) hipFree(p);
    }
  };
  DevFree dw, dense, up, fresh, fresh_map;
  uint64_t *dwords = nullptr;  // [0] closed total, [1] rows kept by the rebuild
  DTRY(hipMalloc((void **)&dwords, 2 * sizeof(uint64_t)));
  dw.p = dwords;
  DTRY(hipMemsetAsync(dwords, 0, 2 * sizeof(uint64_t), d.stream));
  uint64_t closed = 0;
  if (!reopen && cfg.window_kind != HSG_UNWINDOWED) {
    launch_tw_closed(d.stream, d.tw, d.tw.slots(), p, d.sc, d.emit, dwords, nullptr);
    DTRY(hipMemcpyAsync(h, dwords, 8, hipMemcpyDeviceToHost, d.stream));
    DTRY(hipStreamSynchronize(d.stream));
    DTRY(hipGetLastError());
    closed = h[0];
  }
  const uint64_t back = reopen ? d.spilled_rows : 0;
  const uint64_t keep = live - closed + back;
  uint64_t ncap = widen ? 2 * d.cap : d.cap;
  while (2 * (keep + bound) > ncap) ncap <<= 1;
  // each overflow rebuild doubles the regions (a key's windows share its
  // region: a few keys with many open windows need larger regions, not more)
  const int rlog2 = widen ? d.region_log2 + 1 : d.region_log2;
  if (cfg.emit_mode == HSG_EMIT_PER_RECORD && ncap > 0x80000000ull) {
    err = "state table would pass 2^31 slots (per-record changelog path)";
    return HSG_E_OOM;
  }
  // every allocation first: a failure leaves the op as it was
  TwTable nt = d.tw;
  nt.rows = nullptr;
  tw_configure(nt, ncap, cfg.window_kind, rlog2);
  DTRY(hipMalloc((void **)&nt.rows, nt.slots() * (uint64_t)nt.stride * 8));
  fresh.p = nt.rows;
  if (d.tw.dirty) {  // claims still mark: a map for the new table
    nt.dirty = nullptr;
    DTRY(hipMalloc((void **)&nt.dirty, tw_dirty_bytes(nt.slots())));
    fresh_map.p = nt.dirty;
  }
  if (closed) DTRY(hipMalloc(&dense.p, closed * d.tw.stride * 8));
  if (back) DTRY(hipMalloc(&up.p, back * d.tw.stride * 8));
  const uint64_t at = d.spill.size();
  d.spill.resize(at + closed * d.tw.stride);
  auto undo = [&](const std::string &why, int code) {
    d.spill.resize(at);
    err = why;
    return code;
  };
  // 1. closed rows to the host
  if (closed) {
    launch_tw_closed(d.stream, d.tw, d.tw.slots(), p, d.sc, d.emit, nullptr, (uint64_t *)dense.p);
    hipMemcpyAsync(d.spill.data() + at, dense.p, closed * d.tw.stride * 8, hipMemcpyDeviceToHost, d.stream);
  }
  // 2. the open rows (and, after a lowered watermark, the spilled ones) into
  //    the fresh table
  launch_tw_reset(d.stream, nt, prog);
  DTRY(hipMemsetAsync(nt.ovf, 0, 8, d.stream));  // overflow claims of the rebuild
  launch_tw_reinsert(d.stream, d.tw.rows, d.tw.slots(), nt, p, d.sc, closed != 0, (unsigned long long *)(dwords + 1));
  if (back) {
    hipMemcpyAsync(up.p, d.spill.data(), back * d.tw.stride * 8, hipMemcpyHostToDevice, d.stream);
    launch_tw_reinsert(d.stream, (const uint64_t *)up.p, back, nt, p, d.sc, false, (unsigned long long *)(dwords + 1));
  }
  h[2] = 0;
  hipMemcpyAsync(h + 1, dwords + 1, 8, hipMemcpyDeviceToHost, d.stream);
  hipMemcpyAsync(h + 2, &d.sc->err, 4, hipMemcpyDeviceToHost, d.stream);
  hipMemcpyAsync(h + 3, nt.ovf, 8, hipMemcpyDeviceToHost, d.stream);
  hipError_t e = hipStreamSynchronize(d.stream);
  if (e == hipSuccess) e = hipGetLastError();
  if (e != hipSuccess) return undo(std::string("table rebuild: ") + hipGetErrorString(e), HSG_E_DEVICE);
  if (((uint32_t)h[2] & ERR_OOM) || h[1] != keep) return undo("table rebuild: rows lost (internal)", HSG_E_DEVICE);
  // commit
  fresh.p = nullptr;
  fresh_map.p = nullptr;
  hipFree(d.tw.rows);
  if (nt.dirty || ncap != d.cap) {
    // the old-size map goes: the new table's map, or none once claims stopped
    // marking (they never mark again: whole-table clears from then on)
    hipFree(d.tw_dirty_mem);
    d.tw_dirty_mem = nt.dirty;
  }
  // a clear's pending count of dirty blocks describes the old table
  if (ncap != d.cap) d.tw_cnt_pending = false;
  d.tw = nt;  // its dirty map: cleared with it, then marked by the reinsert
  d.region_log2 = rlog2;
  if (widen) d.ovf_events += 1;
  d.ovf_rows = h[3];  // rows the larger regions still could not take (rebuilt again next batch)
  DTRY(hipMemsetAsync(nt.ovf, 0, 8, d.stream));
  if (closed) {
    d.spilled_rows += closed;
    d.spill_events += 1;
    if (wm_in > d.spill_wm) d.spill_wm = wm_in;
  }
  if (back) tw_retention_reset(d);
  d.h_sc->live = keep;
  DTRY(hipMemcpyAsync(&d.sc->live, &d.h_sc->live, 8, hipMemcpyHostToDevice, d.stream));
  DTRY(hipMemsetAsync(d.sc->live_x, 0, sizeof(d.sc->live_x), d.stream));
  if (ncap != d.cap) {
    d.grow_events += 1;
    // emit / dump scratch for the larger table
    const uint64_t nb = emit_chunks(nt.slots());
    if (nb > emit_chunks(tw_ovf_slots(d.cap) + d.cap)) {
      DTRY(hipStreamSynchronize(d.stream));
      hipFree(d.emit.cnt);
      hipFree(d.emit.off);
      hipFree(d.emit.partial);
      d.emit = EmitScratch{};
      DTRY(hipMalloc((void **)&d.emit.cnt, nb * 4));
      DTRY(hipMalloc((void **)&d.emit.off, nb * 8));
      DTRY(hipMalloc((void **)&d.emit.partial, (scan_partials_needed(nb) + 8) * 8));
    }
    d.cap = ncap;
    // the sort-based per-record path keeps a [slots][n_slots] shadow table
    // (the partitioned one, d.pr_part, keeps nothing sized by the table)
    if (cfg.emit_mode == HSG_EMIT_PER_RECORD && !d.pr_part) {
      DTRY(hipStreamSynchronize(d.stream));
      hipFree(d.scratch);
      d.scratch = nullptr;
      int rc = perrecord_device_init(d, cfg, prog, err);
      if (rc != HSG_OK) return rc;
    }
    int rc = grow_out(d, cfg, ncap, pending, err);
    if (rc != HSG_OK) return rc;
  }
  DTRY(hipStreamSynchronize(d.stream));
  return HSG_OK;
}

int tw_dump_spilled(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const hsg_rows *out,
                    uint64_t dst_off, uint64_t *n_out, std::string &err) {
  *n_out = 0;
  if (!d.spilled_rows) return HSG_OK;
  // render in chunks through the resident rows' emit kernel (mode 1 = every
  // row of a "table" whose slots are the dense spilled rows)
  const uint64_t chunk_rows = d.spilled_rows < (1ull << 22) ? d.spilled_rows : (1ull << 22);
  const uint64_t nb = emit_chunks(chunk_rows);
  uint64_t *rows = nullptr, *total = nullptr;
  EmitScratch es;
  memset(&es, 0, sizeof(es));
  OutCols tmp;
  memset(&tmp, 0, sizeof(tmp));
  hipError_t e = hipMalloc((void **)&rows, chunk_rows * d.tw.stride * 8);
  if (e == hipSuccess) e = hipMalloc((void **)&total, 8);
  if (e == hipSuccess) e = hipMalloc((void **)&es.cnt, nb * 4);
  if (e == hipSuccess) e = hipMalloc((void **)&es.off, nb * 8);
  if (e == hipSuccess) e = hipMalloc((void **)&es.partial, (scan_partials_needed(nb) + 8) * 8);
  if (e == hipSuccess) e = hipMalloc((void **)&tmp.key, chunk_rows * 4);
  if (e == hipSuccess) e = hipMalloc((void **)&tmp.ws, chunk_rows * 8);
  if (e == hipSuccess) e = hipMalloc((void **)&tmp.we, chunk_rows * 8);
  if (e == hipSuccess) e = hipMalloc((void **)&tmp.src, chunk_rows * 8);
  for (int j = 0; j < cfg.n_aggs && e == hipSuccess; ++j) e = hipMalloc((void **)&tmp.agg[j], chunk_rows * 8);
  if (d.forms && e == hipSuccess) e = hipMalloc((void **)&tmp.form, chunk_rows * 4);
  int rc = HSG_OK;
  if (e != hipSuccess) {
    err = std::string("dump of spilled rows: ") + hipGetErrorString(e);
    rc = e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;
  }
  const TwParams p = retention_params(cfg, INT64_MIN);
  for (uint64_t at = 0; rc == HSG_OK && at < d.spilled_rows; at += chunk_rows) {
    const uint64_t m = d.spilled_rows - at < chunk_rows ? d.spilled_rows - at : chunk_rows;
    TwTable st = d.tw;
    st.rows = rows;
    e = hipMemcpyAsync(rows, d.spill.data() + at * d.tw.stride, m * d.tw.stride * 8, hipMemcpyHostToDevice, d.stream);
    if (e != hipSuccess) {
      err = std::string("dump of spilled rows: ") + hipGetErrorString(e);
      rc = HSG_E_DEVICE;
      break;
    }
    launch_tw_emit(d.stream, st, m, prog, p, 1, tmp, 0, m, d.sc, es, total);
    rc = op_copy_rows(d, tmp, 0, m, cfg.n_aggs, out, err, dst_off + at);
    *n_out += m;
  }
  hipStreamSynchronize(d.stream);
  hipFree(rows);
  hipFree(total);
  hipFree(es.cnt);
  hipFree(es.off);
  hipFree(es.partial);
  hipFree(tmp.key);
  hipFree(tmp.ws);
  hipFree(tmp.we);
  hipFree(tmp.src);
  for (int j = 0; j < kMaxAggs; ++j)
    if (tmp.agg[j]) hipFree(tmp.agg[j]);
  if (tmp.form) hipFree(tmp.form);
  return rc;
}

}  // namespace hsg
