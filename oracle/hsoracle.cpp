// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A sequential CPU restatement of the reference's windowed-aggregation path
// (Yu-zh/hstream @ 2025-01-17). Only tests/, __graft_entry__.smoke() and
// bench.py's cpu_baseline leg may load this library, and only as the checker /
// the timed CPU baseline; the product (hstream_amd/, libhstream_gpu) never links
// or calls it.
//
// Parity pinning: the reference is Haskell and cannot be built here (no GHC, see
// SURVEY.md §8c), so this restatement is pinned by (1) the windowed / grouped
// results the reference's own tests hold (hstream/test/HStream/RegressionSpec.hs:42-56
// #394_SESSION, :58-74 #403_RAW, :76-94 HS352_INT; RunSQLSpec.hs:66-83, :178-189),
// transcribed in tests/golden/reference_kat.json, and (2) the hand-derived
// windowsFor / findSessions vectors of SURVEY.md §8a. TUMBLING and HOPPING
// aggregate values are not pinned by any reference test ("parity partially
// pinned").
//
// Data structures follow the reference on purpose (they are what the CPU baseline
// times): the KV store is an ordered map (Store.hs:43-81, Data.Map behind an
// IORef) and the session store is the nested end -> key -> start map with the
// same findSessions scan (Store.hs:177-272). Arbitrary-precision Scientific
// arithmetic (Codegen.hs:404-461) is stood in for by __int128 (integer columns,
// overflow of the int64 output is reported) and __float128 (double columns).
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <unordered_map>
#include <vector>

#include "../include/hstream_gpu.h"

namespace {

typedef __int128 i128;
typedef __float128 f128;

// Haskell Int64 arithmetic wraps; do the same.
static inline int64_t wadd(int64_t a, int64_t b) { return (int64_t)((uint64_t)a + (uint64_t)b); }
static inline int64_t wsub(int64_t a, int64_t b) { return (int64_t)((uint64_t)a - (uint64_t)b); }

struct AggVal {
  i128 iv = 0;   // integer sum / min / max / last
  f128 fv = 0;   // double sum / min / max / last
  int64_t cnt = 0;
};

struct Acc {
  std::vector<AggVal> v;
};

struct Row {
  uint32_t key;
  int64_t ws, we, src;
  std::vector<AggVal> v;
};

struct Op {
  hsg_op_config cfg;
  std::vector<int32_t> col_types;
  std::vector<hsg_agg> aggs;
  bool faithful_sessions = true;
  uint64_t records = 0;
  uint64_t batches = 0;
  std::string err;
  bool overflow = false;

  // Time windows / unwindowed: Map (winStart, key) acc  (Store.hs:43-81; the SQL
  // state key is {"winStart": ws} ∪ {col: v}, TimeWindows.hs:68-73).
  std::map<std::pair<int64_t, uint32_t>, Acc> kv;
  // Sessions, faithful: Map end (Map key (Map start acc))  (Store.hs:177-179).
  std::map<int64_t, std::map<uint32_t, std::map<int64_t, Acc>>> ss;
  // Sessions, fast variant (same results, per-key ordered by start) used only to
  // generate larger fixtures; cross-checked against the faithful one in tests.
  std::unordered_map<uint32_t, std::map<int64_t, std::pair<int64_t, Acc>>> ssf;

  std::vector<Row> pending;
  uint64_t pending_head = 0;
};

// ---- aggregate components (Codegen.hs:399-477) -----------------------------

static Acc acc_init(const Op &op) {
  Acc a;
  a.v.resize(op.aggs.size());
  for (size_t j = 0; j < op.aggs.size(); ++j) {
    const hsg_agg &g = op.aggs[j];
    AggVal &x = a.v[j];
    switch (g.kind) {
      case HSG_MIN:  // init maxBound :: Int  (Codegen.hs:451)
        x.iv = (i128)INT64_MAX;
        x.fv = (f128)INT64_MAX;
        break;
      case HSG_MAX:  // init minBound :: Int  (Codegen.hs:438)
        x.iv = (i128)INT64_MIN;
        x.fv = (f128)INT64_MIN;
        break;
      default:       // Number 0 (Codegen.hs:406,414,425,465)
        break;
    }
  }
  return a;
}

struct RecView {
  const hsg_batch *b;
  uint64_t i;
  bool present(int c) const {
    if (!b->valid || !b->valid[c]) return true;
    return b->valid[c][i] != 0;
  }
  int64_t ival(int c) const { return ((const int64_t *)b->cols[c])[i]; }
  double fval(int c) const { return ((const double *)b->cols[c])[i]; }
};

// aggregateF: fold of every component over one record. The components touch
// disjoint aliases, so foldr order (Codegen.hs:475) does not change the result.
static void acc_apply(const Op &op, Acc &a, const RecView &r) {
  for (size_t j = 0; j < op.aggs.size(); ++j) {
    const hsg_agg &g = op.aggs[j];
    AggVal &x = a.v[j];
    if (g.kind == HSG_COUNT_ALL) { x.cnt += 1; continue; }
    int c = g.column;
    if (!r.present(c)) continue;  // HM.lookup … Nothing -> o
    bool isf = op.col_types[c] == HSG_F64;
    switch (g.kind) {
      case HSG_COUNT: x.cnt += 1; break;
      case HSG_SUM:
        if (isf) x.fv += (f128)r.fval(c); else x.iv += (i128)r.ival(c);
        break;
      case HSG_MIN:
        if (isf) { f128 v = r.fval(c); if (v < x.fv) x.fv = v; }
        else { i128 v = r.ival(c); if (v < x.iv) x.iv = v; }
        break;
      case HSG_MAX:
        if (isf) { f128 v = r.fval(c); if (v > x.fv) x.fv = v; }
        else { i128 v = r.ival(c); if (v > x.iv) x.iv = v; }
        break;
      case HSG_AVG:
        if (isf) x.fv += (f128)r.fval(c); else x.iv += (i128)r.ival(c);
        x.cnt += 1;
        break;
      case HSG_LAST:
        if (isf) x.fv = r.fval(c); else x.iv = r.ival(c);
        break;
    }
  }
}

// aggregateMergeF o1 o2 with o1 = running merged acc, o2 = existing session
// (SessionWindowedStream.hs:109): sums add, min/max combine, passthrough takes o2.
static void acc_merge(const Op &op, Acc &a, const Acc &cur) {
  for (size_t j = 0; j < op.aggs.size(); ++j) {
    const hsg_agg &g = op.aggs[j];
    AggVal &x = a.v[j];
    const AggVal &y = cur.v[j];
    switch (g.kind) {
      case HSG_COUNT_ALL:
      case HSG_COUNT: x.cnt += y.cnt; break;
      case HSG_SUM: x.iv += y.iv; x.fv += y.fv; break;
      case HSG_MIN: if (y.iv < x.iv) x.iv = y.iv; if (y.fv < x.fv) x.fv = y.fv; break;
      case HSG_MAX: if (y.iv > x.iv) x.iv = y.iv; if (y.fv > x.fv) x.fv = y.fv; break;
      case HSG_AVG: x.iv += y.iv; x.fv += y.fv; x.cnt += y.cnt; break;
      case HSG_LAST: x.iv = y.iv; x.fv = y.fv; break;
    }
  }
}

// ---- windowsFor (TimeWindowedStream.hs:105-117) -------------------------------
// windowStart = max 0 (ts - size + adv) `quot` adv * adv; emit [s, s+size) while s <= ts.
static int windows_for(int64_t ts, int64_t size, int64_t adv, std::vector<int64_t> &starts) {
  starts.clear();
  int64_t t0 = wadd(wsub(ts, size), adv);
  if (t0 < 0) t0 = 0;
  int64_t s = (t0 / adv) * adv;  // quot on a non-negative value
  while (s <= ts) {
    starts.push_back(s);
    if (s > INT64_MAX - adv) break;  // the reference would wrap and loop forever
    s += adv;
  }
  return (int)starts.size();
}

static void emit_row(Op &op, uint32_t key, int64_t ws, int64_t we, int64_t src, const Acc &a) {
  Row r;
  r.key = key; r.ws = ws; r.we = we; r.src = src; r.v = a.v;
  op.pending.push_back(std::move(r));
}

// ---- time-windowed and grouped aggregation ---------------------------------
static int push_time(Op &op, const hsg_batch *b, int64_t *wm, const int64_t *rec_wm, const int64_t *seq) {
  const bool unwin = op.cfg.window_kind == HSG_UNWINDOWED;
  const int64_t size = op.cfg.size_ms;
  const int64_t adv = op.cfg.window_kind == HSG_TUMBLING ? op.cfg.size_ms : op.cfg.advance_ms;
  const int64_t grace = op.cfg.grace_ms;
  const int mode = op.cfg.emit_mode;
  // per-batch mode: last per-record row per group
  std::map<std::pair<uint32_t, int64_t>, size_t> last;
  std::vector<Row> batch_rows;
  std::vector<int64_t> starts;
  int64_t w = *wm;
  for (uint64_t i = 0; i < b->n; ++i) {
    int64_t ts = b->ts[i];
    if (ts > w) w = ts;  // updateTimestampInTaskContext (Processor.hs:139)
    uint32_t key = b->key_id[i];
    if (key == HSG_KEY_NONE) continue;
    RecView rv{b, i};
    int64_t src = seq ? seq[i] : (int64_t)(op.records + i);
    // sharded-protocol tests hand in the stream time each record saw in the
    // global arrival order
    const int64_t wr = rec_wm ? rec_wm[i] : w;
    if (unwin) {  // GroupedStream.aggregateProcessor (GroupedStream.hs:79-87)
      auto it = op.kv.find({0, key});
      if (it == op.kv.end()) it = op.kv.emplace(std::make_pair((int64_t)0, key), acc_init(op)).first;
      acc_apply(op, it->second, rv);
      if (mode == HSG_EMIT_PER_RECORD) emit_row(op, key, 0, 0, src, it->second);
      else if (mode == HSG_EMIT_PER_BATCH) {
        Row r{key, 0, 0, src, it->second.v};
        auto lk = last.find({key, 0});
        if (lk == last.end()) { last[{key, 0}] = batch_rows.size(); batch_rows.push_back(std::move(r)); }
        else batch_rows[lk->second] = std::move(r);
      }
      continue;
    }
    windows_for(ts, size, adv, starts);  // TimeWindowedStream.hs:86
    for (int64_t ws : starts) {
      int64_t we = wadd(ws, size);
      if (!(wr < wadd(we, grace))) continue;  // :92, "Skipping record for expired window."
      auto it = op.kv.find({ws, key});
      if (it == op.kv.end()) it = op.kv.emplace(std::make_pair(ws, key), acc_init(op)).first;
      acc_apply(op, it->second, rv);  // :96-100
      if (mode == HSG_EMIT_PER_RECORD) emit_row(op, key, ws, we, src, it->second);  // :101
      else if (mode == HSG_EMIT_PER_BATCH) {
        Row r{key, ws, we, -1, it->second.v};
        auto lk = last.find({key, ws});
        if (lk == last.end()) { last[{key, ws}] = batch_rows.size(); batch_rows.push_back(std::move(r)); }
        else batch_rows[lk->second] = std::move(r);
      }
    }
  }
  if (mode == HSG_EMIT_PER_BATCH) {
    std::sort(batch_rows.begin(), batch_rows.end(), [](const Row &a, const Row &c) {
      return std::tie(a.key, a.ws) < std::tie(c.key, c.ws);
    });
    for (auto &r : batch_rows) { r.src = -1; op.pending.push_back(std::move(r)); }
  }
  *wm = w;
  return HSG_OK;
}

// ---- sessions (SessionWindowedStream.hs:84-118, Store.hs:189-272) -------------
struct SessHit { int64_t start, end; Acc acc; };

// findSessions key earliestEnd latestStart: every end >= earliestEnd (all keys),
// then that key's starts <= latestStart; ordered by end asc, start asc.
static void find_sessions_faithful(Op &op, uint32_t key, int64_t lo, int64_t hi, std::vector<SessHit> &out) {
  out.clear();
  for (auto it = op.ss.lower_bound(lo); it != op.ss.end(); ++it) {
    auto kt = it->second.find(key);
    if (kt == it->second.end()) continue;
    for (auto st = kt->second.begin(); st != kt->second.end() && st->first <= hi; ++st)
      out.push_back({st->first, it->first, st->second});
  }
}

static void ss_remove_faithful(Op &op, uint32_t key, int64_t start, int64_t end) {
  auto it = op.ss.find(end);
  if (it == op.ss.end()) return;
  auto kt = it->second.find(key);
  if (kt == it->second.end()) return;
  kt->second.erase(start);  // empty inner maps stay behind, as in Store.hs:223-235
}

static void find_sessions_fast(Op &op, uint32_t key, int64_t lo, int64_t hi, std::vector<SessHit> &out) {
  out.clear();
  auto kt = op.ssf.find(key);
  if (kt == op.ssf.end()) return;
  auto &m = kt->second;  // start -> (end, acc), disjoint sessions
  auto it = m.upper_bound(hi);
  // walk backwards over sessions with start <= hi while end >= lo
  std::vector<SessHit> rev;
  while (it != m.begin()) {
    --it;
    if (it->second.first < lo) break;
    rev.push_back({it->first, it->second.first, it->second.second});
  }
  // order by end asc, start asc (disjoint sessions: same as start asc)
  for (auto r = rev.rbegin(); r != rev.rend(); ++r) out.push_back(*r);
}

static int push_session(Op &op, const hsg_batch *b, int64_t *wm, const int64_t *seq) {
  const int64_t gap = op.cfg.gap_ms;
  const int mode = op.cfg.emit_mode;
  std::set<std::tuple<uint32_t, int64_t, int64_t>> touched;  // (key, start, end)
  std::vector<SessHit> hits;
  int64_t w = *wm;
  for (uint64_t i = 0; i < b->n; ++i) {
    int64_t ts = b->ts[i];
    if (ts > w) w = ts;
    uint32_t key = b->key_id[i];
    if (key == HSG_KEY_NONE) continue;
    RecView rv{b, i};
    int64_t lo = wsub(ts, gap), hi = wadd(ts, gap);
    if (op.faithful_sessions) find_sessions_faithful(op, key, lo, hi, hits);
    else find_sessions_fast(op, key, lo, hi, hits);
    Acc acc = acc_init(op);
    acc_apply(op, acc, rv);  // aggF initialValue r
    int64_t s = ts, e = ts;
    for (auto &h : hits) {  // foldM (SessionWindowedStream.hs:99-115)
      s = std::min(s, h.start);
      e = std::max(e, h.end);
      acc_merge(op, acc, h.acc);
      if (op.faithful_sessions) ss_remove_faithful(op, key, h.start, h.end);
      else op.ssf[key].erase(h.start);
      touched.erase({key, h.start, h.end});
    }
    if (op.faithful_sessions) op.ss[e][key][s] = acc;  // ssPut
    else op.ssf[key][s] = {e, acc};
    touched.insert({key, s, e});
    if (mode == HSG_EMIT_PER_RECORD) emit_row(op, key, s, e, seq ? seq[i] : (int64_t)(op.records + i), acc);
  }
  if (mode == HSG_EMIT_PER_BATCH) {
    for (auto &t : touched) {
      uint32_t key; int64_t s, e;
      std::tie(key, s, e) = t;
      const Acc *a;
      if (op.faithful_sessions) a = &op.ss[e][key][s];
      else a = &op.ssf[key][s].second;
      emit_row(op, key, s, e, -1, *a);
    }
  }
  *wm = w;
  return HSG_OK;
}

// ---- output conversion --------------------------------------------------------
static bool agg_is_f64(const Op &op, const hsg_agg &g) {
  if (g.kind == HSG_COUNT_ALL || g.kind == HSG_COUNT) return false;
  if (g.kind == HSG_AVG) return true;
  return op.col_types[g.column] == HSG_F64;
}

static void write_rows(Op &op, const std::vector<const Row *> &rows, hsg_rows *out) {
  for (size_t r = 0; r < rows.size(); ++r) {
    const Row &x = *rows[r];
    if (out->key_id) out->key_id[r] = x.key;
    if (out->win_start) out->win_start[r] = x.ws;
    if (out->win_end) out->win_end[r] = x.we;
    if (out->src_index) out->src_index[r] = x.src;
    for (size_t j = 0; j < op.aggs.size(); ++j) {
      const hsg_agg &g = op.aggs[j];
      const AggVal &v = x.v[j];
      void *dst = out->aggs ? out->aggs[j] : nullptr;
      if (!dst) continue;
      if (agg_is_f64(op, g)) {
        double d;
        bool isf = g.kind != HSG_COUNT_ALL && g.kind != HSG_COUNT && op.col_types[g.column] == HSG_F64;
        if (g.kind == HSG_AVG) {
          if (v.cnt == 0) d = NAN;
          else d = isf ? (double)(v.fv / (f128)v.cnt) : (double)((f128)v.iv / (f128)v.cnt);
        } else {
          d = (double)v.fv;
        }
        ((double *)dst)[r] = d;
      } else {
        int64_t o;
        if (g.kind == HSG_COUNT_ALL || g.kind == HSG_COUNT) o = v.cnt;
        else {
          if (v.iv > (i128)INT64_MAX || v.iv < (i128)INT64_MIN) op.overflow = true;
          o = (int64_t)v.iv;
        }
        ((int64_t *)dst)[r] = o;
      }
    }
  }
}

static int validate(const hsg_op_config *c, std::string &err) {
  if (!c) { err = "null config"; return HSG_E_INVALID; }
  if (c->window_kind < 0 || c->window_kind > HSG_UNWINDOWED) { err = "bad window_kind"; return HSG_E_INVALID; }
  if (c->window_kind == HSG_TUMBLING || c->window_kind == HSG_HOPPING) {
    if (c->size_ms <= 0) { err = "size_ms must be > 0"; return HSG_E_INVALID; }
    if (c->window_kind == HSG_HOPPING && c->advance_ms <= 0) { err = "advance_ms must be > 0"; return HSG_E_INVALID; }
  }
  if (c->window_kind == HSG_SESSION && c->gap_ms < 0) { err = "gap_ms must be >= 0"; return HSG_E_INVALID; }
  if (c->n_aggs <= 0 || !c->aggs) { err = "no aggregates"; return HSG_E_INVALID; }
  if (c->n_cols < 0 || (c->n_cols > 0 && !c->col_types)) { err = "bad columns"; return HSG_E_INVALID; }
  for (int j = 0; j < c->n_aggs; ++j) {
    const hsg_agg &g = c->aggs[j];
    if (g.kind < 0 || g.kind > HSG_LAST) { err = "bad agg kind"; return HSG_E_INVALID; }
    if (g.kind != HSG_COUNT_ALL && (g.column < 0 || g.column >= c->n_cols)) { err = "bad agg column"; return HSG_E_INVALID; }
  }
  return HSG_OK;
}

}  // namespace

extern "C" {

struct hso_op;

int hso_op_create_ex(const hsg_op_config *cfg, int faithful_sessions, hso_op **out) {
  std::string err;
  int rc = validate(cfg, err);
  if (rc != HSG_OK) return rc;
  Op *op = new Op();
  op->cfg = *cfg;
  op->col_types.assign(cfg->col_types, cfg->col_types + cfg->n_cols);
  op->aggs.assign(cfg->aggs, cfg->aggs + cfg->n_aggs);
  op->cfg.col_types = nullptr;
  op->cfg.aggs = nullptr;
  op->faithful_sessions = faithful_sessions != 0;
  *out = (hso_op *)op;
  return HSG_OK;
}

int hso_op_create(const hsg_op_config *cfg, hso_op **out) { return hso_op_create_ex(cfg, 1, out); }

void hso_op_destroy(hso_op *h) { delete (Op *)h; }

int hso_op_reset(hso_op *h) {
  Op *op = (Op *)h;
  op->kv.clear(); op->ss.clear(); op->ssf.clear();
  op->pending.clear(); op->pending_head = 0;
  op->records = 0; op->batches = 0; op->overflow = false;
  return HSG_OK;
}

const char *hso_last_error(const hso_op *h) { return ((const Op *)h)->err.c_str(); }

// rec_wm / seq (optional): per-record stream time and global sequence number,
// used by the tests that restate the multi-GPU sharding protocol.
int hso_push_batch_ex(hso_op *h, const hsg_batch *b, int64_t *wm, const int64_t *rec_wm, const int64_t *seq) {
  Op *op = (Op *)h;
  if (!b || !wm) { op->err = "null argument"; return HSG_E_INVALID; }
  if (b->mem != HSG_MEM_HOST) { op->err = "oracle takes host batches only"; return HSG_E_INVALID; }
  if (b->n_cols != (int32_t)op->col_types.size()) { op->err = "n_cols mismatch"; return HSG_E_INVALID; }
  if (b->n && (!b->key_id || !b->ts)) { op->err = "null key/ts"; return HSG_E_INVALID; }
  int rc = op->cfg.window_kind == HSG_SESSION ? push_session(*op, b, wm, seq) : push_time(*op, b, wm, rec_wm, seq);
  op->records += b->n;
  op->batches += 1;
  return rc;
}

int hso_push_batch(hso_op *h, const hsg_batch *b, int64_t *wm) { return hso_push_batch_ex(h, b, wm, nullptr, nullptr); }

int hso_pending_rows(const hso_op *h, uint64_t *n) {
  const Op *op = (const Op *)h;
  *n = op->pending.size() - op->pending_head;
  return HSG_OK;
}

int hso_drain(hso_op *h, hsg_rows *out, uint64_t *n_out) {
  Op *op = (Op *)h;
  uint64_t n = op->pending.size() - op->pending_head;
  *n_out = n;
  if (out->capacity < n) { op->err = "drain: out capacity too small"; return HSG_E_CAPACITY; }
  std::vector<const Row *> rows;
  rows.reserve(n);
  for (uint64_t i = op->pending_head; i < op->pending.size(); ++i) rows.push_back(&op->pending[i]);
  op->overflow = false;
  write_rows(*op, rows, out);
  op->pending.clear();
  op->pending_head = 0;
  if (op->overflow) { op->err = "int64 overflow of an exact SUM"; return HSG_E_RANGE; }
  return HSG_OK;
}

static void collect_state(Op &op, std::vector<Row> &rows) {
  if (op.cfg.window_kind == HSG_SESSION) {
    if (op.faithful_sessions) {
      for (auto &e : op.ss)
        for (auto &k : e.second)
          for (auto &s : k.second) rows.push_back({k.first, s.first, e.first, -1, s.second.v});
    } else {
      for (auto &k : op.ssf)
        for (auto &s : k.second) rows.push_back({k.first, s.first, s.second.first, -1, s.second.second.v});
    }
  } else {
    const bool unwin = op.cfg.window_kind == HSG_UNWINDOWED;
    for (auto &kv : op.kv) {
      int64_t ws = kv.first.first;
      rows.push_back({kv.first.second, ws, unwin ? 0 : wadd(ws, op.cfg.size_ms), -1, kv.second.v});
    }
  }
  std::sort(rows.begin(), rows.end(), [](const Row &a, const Row &c) {
    return std::tie(a.key, a.ws) < std::tie(c.key, c.ws);
  });
}

int hso_state_rows(hso_op *h, uint64_t *n) {
  Op *op = (Op *)h;
  std::vector<Row> rows;
  collect_state(*op, rows);
  *n = rows.size();
  return HSG_OK;
}

int hso_dump_state(hso_op *h, hsg_rows *out, uint64_t *n_out) {
  Op *op = (Op *)h;
  std::vector<Row> rows;
  collect_state(*op, rows);
  *n_out = rows.size();
  if (out->capacity < rows.size()) { op->err = "dump: out capacity too small"; return HSG_E_CAPACITY; }
  std::vector<const Row *> ptrs;
  for (auto &r : rows) ptrs.push_back(&r);
  op->overflow = false;
  write_rows(*op, ptrs, out);
  if (op->overflow) { op->err = "int64 overflow of an exact SUM"; return HSG_E_RANGE; }
  return HSG_OK;
}

// windowsFor exposed for the known-answer tests; returns the window count and
// writes up to cap starts.
int hso_windows_for(int64_t ts, int64_t size, int64_t adv, int64_t *starts, int cap) {
  std::vector<int64_t> s;
  windows_for(ts, size, adv, s);
  for (int i = 0; i < (int)s.size() && i < cap; ++i) starts[i] = s[i];
  return (int)s.size();
}

}  // extern "C"
