// libhstream_gpu host runtime: the C ABI of include/hstream_gpu.h.
//
// One hsg_engine per process and GPU (device selection, RCCL communicator);
// one hsg_op per windowed GROUP BY operator. Each op owns a HIP stream, its
// HBM state (hash table of (key, window) rows, or the session arena), staging
// buffers for host batches and an HBM changelog buffer drained by hsg_drain.
// Every entry point catches everything: no C++ exception crosses the ABI.
#include <hip/hip_runtime.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "hsg_internal.h"
#include "hsg_ops.h"

using namespace hsg;

// ---------------------------------------------------------------------------
// error helpers
// ---------------------------------------------------------------------------
#define HIP_TRY(obj, expr)                                                         \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      (obj)->err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;                 \
    }                                                                              \
  } while (0)

namespace {

int fail(std::string &err, int code, const std::string &msg) {
  err = msg;
  return code;
}

uint64_t next_pow2(uint64_t v) {
  uint64_t p = 1;
  while (p < v) p <<= 1;
  return p;
}

double now_ms() {
  using namespace std::chrono;
  return duration<double, std::milli>(steady_clock::now().time_since_epoch()).count();
}

}  // namespace

// ---------------------------------------------------------------------------
// program (aggregates -> state slots -> output columns)
// ---------------------------------------------------------------------------
namespace hsg {

int build_program(const hsg_op_config &cfg, const std::vector<int32_t> &col_types, const std::vector<hsg_agg> &aggs,
                  Program &prog, std::string &err, bool forms) {
  memset(&prog, 0, sizeof(prog));
  auto find_slot = [&](int op, int col) -> int {
    for (int s = 0; s < prog.n_slots; ++s)
      if (prog.slot_op[s] == op && prog.slot_col[s] == col) return s;
    return -1;
  };
  auto add_slot = [&](int op, int col) -> int {
    int s = find_slot(op, col);
    if (s >= 0) return s;
    if (prog.n_slots >= kMaxSlots) return -1;
    prog.slot_op[prog.n_slots] = op;
    prog.slot_col[prog.n_slots] = col;
    return prog.n_slots++;
  };
  // LAST: the (record seq, value) slot pair of column c; -1 = no room
  auto last_pair = [&](int c) -> int {
    int s = find_slot(S_LAST_SEQ, c);
    if (s < 0) {
      if (prog.n_slots + 2 > kMaxSlots) return -1;
      s = add_slot(S_LAST_SEQ, c);
      prog.slot_op[prog.n_slots] = S_LAST_VAL;
      prog.slot_col[prog.n_slots] = c;
      prog.n_slots++;
    }
    return s;
  };
  if ((int)aggs.size() > kMaxAggs) return fail(err, HSG_E_INVALID, "too many aggregates (max 16)");
  for (size_t j = 0; j < aggs.size(); ++j) {
    const hsg_agg &g = aggs[j];
    int a = -1, b = 0, kind = O_I64;
    bool isf = g.kind != HSG_COUNT_ALL && col_types[g.column] == HSG_F64;
    int c = g.kind == HSG_COUNT_ALL ? 0 : g.column;
    switch (g.kind) {
      case HSG_COUNT_ALL: a = add_slot(S_CNT_ALL, 0); break;
      case HSG_COUNT: a = add_slot(S_CNT, c); break;
      case HSG_SUM: a = add_slot(isf ? S_SUM_F : S_SUM_I, c); kind = isf ? O_F64 : O_I64; break;
      case HSG_MIN: a = add_slot(isf ? S_MIN_F : S_MIN_I, c); kind = isf ? O_F64_ORD : O_I64; break;
      case HSG_MAX: a = add_slot(isf ? S_MAX_F : S_MAX_I, c); kind = isf ? O_F64_ORD : O_I64; break;
      case HSG_AVG:
        a = add_slot(isf ? S_SUM_F : S_SUM_I, c);
        b = add_slot(S_CNT, c);
        kind = isf ? O_AVG_F : O_AVG_I;
        break;
      case HSG_LAST: {
        // sessions: merges keep the existing session's value (k_session.hip)
        const int s = last_pair(c);
        if (s < 0) return fail(err, HSG_E_INVALID, "too many state slots");
        a = s + 1;
        kind = isf ? O_F64 : O_I64;
        break;
      }
      default: return fail(err, HSG_E_INVALID, "bad aggregate kind");
    }
    if (a < 0 || b < 0) return fail(err, HSG_E_INVALID, "too many state slots");
    prog.out_kind[j] = kind;
    prog.out_a[j] = a;
    prog.out_b[j] = b;
    // the literal form (hsg_internal.h FormKind): a form slot over the
    // output's column that reads bit 1 of its valid bytes
    int fk = F_NONE, fa = 0;
    if (forms) {
      switch (g.kind) {
        case HSG_SUM: fk = F_SUM, fa = add_slot(S_CNT_DEC, c); break;
        case HSG_MIN:
        case HSG_MAX: {
          const int op = g.kind == HSG_MIN ? S_TIE_MIN : S_TIE_MAX;
          fk = g.kind == HSG_MIN ? F_MIN : F_MAX;
          fa = add_slot(op, c);
          if (fa >= 0) prog.slot_aux[fa] = a;  // the MIN / MAX slot it breaks ties of
          break;
        }
        case HSG_LAST: fk = F_LAST, fa = add_slot(S_LAST_FORM, c); break;
        default: break;
      }
      if (fa < 0) return fail(err, HSG_E_INVALID, "too many state slots");
    }
    prog.form_kind[j] = fk;
    prog.form_a[j] = fa;
  }
  prog.n_out = (int)aggs.size();
  for (int s = 0; s < prog.n_slots; ++s) prog.ties |= slot_is_tie(prog.slot_op[s]) ? 1 : 0;
  // the per-record state projection (hsg_internal.h fin_*): the slots the
  // outputs read, plus the form word, when that is smaller than the state
  bool used[kMaxSlots] = {};
  bool forms_any = false;
  for (int j = 0; j < prog.n_out; ++j) {
    used[prog.out_a[j]] = true;
    if (prog.out_kind[j] == O_AVG_I || prog.out_kind[j] == O_AVG_F) used[prog.out_b[j]] = true;
    forms_any |= prog.form_kind[j] != F_NONE;
  }
  int nf = 0;
  for (int s = 0; s < prog.n_slots; ++s)
    if (used[s]) prog.fin_slot[nf++] = s;
  if (nf + (forms_any ? 1 : 0) < prog.n_slots) {
    prog.fin_n = nf;
    prog.fin_form = forms_any ? 1 : 0;
  } else {
    prog.fin_n = prog.n_slots;
    prog.fin_form = 0;
    for (int s = 0; s < prog.n_slots; ++s) prog.fin_slot[s] = s;
  }
  return HSG_OK;
}

}  // namespace hsg

// ---------------------------------------------------------------------------
// engine
// ---------------------------------------------------------------------------
struct hsg_engine {
  int device = 0;
  int rank = 0;
  int nranks = 1;
  uint64_t batch_cap = 0;
  std::string err;
  std::mutex mu;  // guards the engine communicator (op creation splits it)
  Comm *comm = nullptr;
};

extern "C" int hsg_comm_unique_id(uint8_t *out, size_t len) {
  try {
    if (!out || len < HSG_COMM_ID_BYTES) return HSG_E_INVALID;
    return comm_unique_id(out);
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" int hsg_engine_create(const hsg_engine_config *cfg, hsg_engine **out) {
  try {
    if (!cfg || !out) return HSG_E_INVALID;
    *out = nullptr;
    if (cfg->nranks < 1 || cfg->rank < 0 || cfg->rank >= cfg->nranks) return HSG_E_INVALID;
    if (cfg->nranks > 1 && !cfg->comm_id) return HSG_E_INVALID;
    if (cfg->batch_capacity == 0) return HSG_E_INVALID;
    hsg_engine *e = new (std::nothrow) hsg_engine();
    if (!e) return HSG_E_OOM;
    int dev = cfg->device;
    if (dev < 0) {
      if (hipGetDevice(&dev) != hipSuccess) { delete e; return HSG_E_DEVICE; }
    }
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || dev >= ndev) { delete e; return HSG_E_DEVICE; }
    if (hipSetDevice(dev) != hipSuccess) { delete e; return HSG_E_DEVICE; }
    e->device = dev;
    e->rank = cfg->rank;
    e->nranks = cfg->nranks;
    e->batch_cap = cfg->batch_capacity;
    if (cfg->transport != HSG_TRANSPORT_RCCL && cfg->transport != HSG_TRANSPORT_HOST) { delete e; return HSG_E_INVALID; }
    if (cfg->nranks > 1 || cfg->comm_id) {
      int rc = comm_create(cfg->comm_id, cfg->rank, cfg->nranks, dev, cfg->transport, cfg->batch_capacity, &e->comm,
                           e->err);
      if (rc != HSG_OK) { delete e; return rc; }
    }
    *out = e;
    return HSG_OK;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" void hsg_engine_destroy(hsg_engine *e) {
  if (!e) return;
  try {
    hipSetDevice(e->device);
    if (e->comm) comm_destroy(e->comm);
  } catch (...) {
  }
  delete e;
}

extern "C" const char *hsg_engine_last_error(const hsg_engine *e) { return e ? e->err.c_str() : "null engine"; }

// testing knobs (include/hstream_gpu.h): process-wide, read at op creation
static std::atomic<int64_t> g_knob_xpart{-1}, g_knob_arena{0}, g_knob_xclassic{0};

namespace hsg {
int64_t testing_knob(int knob) {
  switch (knob) {
    case HSG_KNOB_XPART_LOG2: return g_knob_xpart.load();
    case HSG_KNOB_SESS_ARENA_MIN: return g_knob_arena.load();
    case HSG_KNOB_X_CLASSIC: return g_knob_xclassic.load();
    default: return 0;
  }
}
}  // namespace hsg

extern "C" int hsg_testing_set_knob(int32_t knob, int64_t value) {
  switch (knob) {
    case HSG_KNOB_XPART_LOG2:
      if (value < -1 || value > 6) return HSG_E_INVALID;
      g_knob_xpart.store(value);
      return HSG_OK;
    case HSG_KNOB_SESS_ARENA_MIN:
      if (value < 0) return HSG_E_INVALID;
      g_knob_arena.store(value);
      return HSG_OK;
    case HSG_KNOB_X_CLASSIC:
      if (value < 0 || value > 1) return HSG_E_INVALID;
      g_knob_xclassic.store(value);
      return HSG_OK;
    default: return HSG_E_INVALID;
  }
}

// ---------------------------------------------------------------------------
// op
// ---------------------------------------------------------------------------
// One queued asynchronous push: the batch descriptor is copied (the caller's
// struct may live on its stack); the arrays it points to are the caller's.
struct AsyncJob {
  hsg_batch b;
  std::vector<const void *> cols;
  std::vector<const uint8_t *> valid;
  int64_t *wm = nullptr;
  hsg_done_fn done = nullptr;
  void *ctx = nullptr;
  int staged_set = -1;  // host arrays already queued for H2D (op_prestage)
};

struct hsg_op {
  hsg_engine *eng = nullptr;
  hsg_op_config cfg;
  std::vector<int32_t> col_types;  // the user's value columns
  std::vector<hsg_agg> aggs;
  int32_t user_cols = 0;           // value columns of the caller's batches (= cfg.n_cols)
  Program prog;
  OpDevice dev;  // every HBM buffer + stream + events (hsg_ops.h)
  // Sharded ops own a communicator split from the engine's at creation, so
  // pushes of distinct ops never share RCCL call ordering (ranks may run their
  // queries' pushes in any interleaving) and need no engine-wide lock.
  Comm *comm = nullptr;
  std::string err;
  uint64_t pending = 0;
  uint64_t state_rows = 0;
  uint32_t batch_id = 0;
  uint64_t rec_base = 0;
  hsg_stats stats;
  // asynchronous pushes (hsg_push_batch_async): one completion thread per op
  std::mutex qmu;
  std::condition_variable qcv;
  std::deque<AsyncJob> queue;
  bool busy = false;       // a job is running
  bool stopping = false;
  int async_rc = HSG_OK;   // first failure since the last hsg_op_wait
  std::thread worker;
  int next_set = 0;        // staging set of the next prestaged batch
};

static int push_sync(hsg_op *op, const hsg_batch *b, int64_t *inout_watermark, int staged_set = -1);

// Queue the H2D copies of a queued host batch so that they
// overlap the batch before it; the sets alternate, so the set a prestage
// fills was last read by a push that has completed (pushes are synchronous on
// the op's completion thread). Failure only means the push stages itself.
static void prestage_job(hsg_op *op, AsyncJob &job) {
  if (job.staged_set >= 0 || job.b.mem != HSG_MEM_HOST || job.b.n == 0) return;
  if (job.b.n > op->eng->batch_cap || job.b.n_cols != op->user_cols || !job.b.key_id || !job.b.ts)
    return;  // push_sync reports it
  hsg_batch b = job.b;
  b.cols = job.cols.empty() ? nullptr : job.cols.data();
  b.valid = job.valid.empty() ? nullptr : job.valid.data();
  for (int c = 0; c < b.n_cols; ++c)
    if (!b.cols || !b.cols[c]) return;
  if (hipSetDevice(op->eng->device) != hipSuccess) return;
  std::string err;
  const int set = op->next_set;
  if (op_prestage(op->dev, &b, set, err) == HSG_OK) {
    job.staged_set = set;
    op->next_set ^= 1;
  }
}

// Wait for the op's queued asynchronous pushes; returns (and clears) the first
// failure among them.
static int drain_async(hsg_op *op) {
  std::unique_lock<std::mutex> lk(op->qmu);
  op->qcv.wait(lk, [&] { return op->queue.empty() && !op->busy; });
  int rc = op->async_rc;
  op->async_rc = HSG_OK;
  return rc;
}

// Same wait, keeping a failure for the next hsg_op_wait / hsg_push_batch.
static void wait_idle(const hsg_op *cop) {
  hsg_op *op = const_cast<hsg_op *>(cop);
  std::unique_lock<std::mutex> lk(op->qmu);
  op->qcv.wait(lk, [&] { return op->queue.empty() && !op->busy; });
}

static void async_loop(hsg_op *op) {
  std::unique_lock<std::mutex> lk(op->qmu);
  for (;;) {
    op->qcv.wait(lk, [&] { return op->stopping || !op->queue.empty(); });
    if (op->queue.empty()) return;  // stopping with nothing left
    AsyncJob job = std::move(op->queue.front());
    op->queue.pop_front();
    op->busy = true;
    // the next queued job stays in the deque (only this thread pops it, and
    // push_back keeps references to elements valid)
    AsyncJob *next = op->queue.empty() ? nullptr : &op->queue.front();
    lk.unlock();
    prestage_job(op, job);
    if (next) prestage_job(op, *next);
    job.b.cols = job.cols.empty() ? nullptr : job.cols.data();
    job.b.valid = job.valid.empty() ? nullptr : job.valid.data();
    const int rc = push_sync(op, &job.b, job.wm, job.staged_set);
    if (job.done) job.done(job.ctx, rc);
    lk.lock();
    if (rc != HSG_OK && op->async_rc == HSG_OK) op->async_rc = rc;
    op->busy = false;
    op->qcv.notify_all();
  }
}

static int validate_config(const hsg_op_config *c, std::string &err) {
  if (!c) return fail(err, HSG_E_INVALID, "null config");
  if (c->window_kind < HSG_TUMBLING || c->window_kind > HSG_UNWINDOWED) return fail(err, HSG_E_INVALID, "bad window_kind");
  if (c->emit_mode < HSG_EMIT_PER_RECORD || c->emit_mode > HSG_EMIT_NONE) return fail(err, HSG_E_INVALID, "bad emit_mode");
  if (c->window_kind == HSG_TUMBLING || c->window_kind == HSG_HOPPING) {
    if (c->size_ms <= 0) return fail(err, HSG_E_INVALID, "size_ms must be > 0");
    if (c->window_kind == HSG_HOPPING && c->advance_ms <= 0) return fail(err, HSG_E_INVALID, "advance_ms must be > 0");
  }
  if (c->window_kind == HSG_SESSION && c->gap_ms < 0) return fail(err, HSG_E_INVALID, "gap_ms must be >= 0");
  if (c->n_aggs <= 0 || !c->aggs) return fail(err, HSG_E_INVALID, "no aggregates");
  if (c->n_cols < 0 || c->n_cols > kMaxCols || (c->n_cols > 0 && !c->col_types))
    return fail(err, HSG_E_INVALID, "bad value columns (max 8)");
  for (int i = 0; i < c->n_cols; ++i)
    if (c->col_types[i] != HSG_I64 && c->col_types[i] != HSG_F64) return fail(err, HSG_E_INVALID, "bad column type");
  for (int j = 0; j < c->n_aggs; ++j) {
    const hsg_agg &g = c->aggs[j];
    if (g.kind < HSG_COUNT_ALL || g.kind > HSG_LAST) return fail(err, HSG_E_INVALID, "bad aggregate kind");
    if (g.kind != HSG_COUNT_ALL && (g.column < 0 || g.column >= c->n_cols))
      return fail(err, HSG_E_INVALID, "aggregate column out of range");
  }
  return HSG_OK;
}

uint64_t hsg_windows_per_record(const hsg_op_config &c) {
  if (c.window_kind == HSG_HOPPING) return (uint64_t)((c.size_ms + c.advance_ms - 1) / c.advance_ms);
  return 1;
}

extern "C" int hsg_op_create(hsg_engine *eng, const hsg_op_config *cfg, hsg_op **out) {
  try {
    if (!eng || !out) return HSG_E_INVALID;
    *out = nullptr;
    int rc = validate_config(cfg, eng->err);
    if (rc != HSG_OK) return rc;
    hsg_op *op = new (std::nothrow) hsg_op();
    if (!op) return HSG_E_OOM;
    op->eng = eng;
    op->cfg = *cfg;
    op->col_types.assign(cfg->col_types, cfg->col_types + cfg->n_cols);
    op->aggs.assign(cfg->aggs, cfg->aggs + cfg->n_aggs);
    op->cfg.col_types = nullptr;
    op->cfg.aggs = nullptr;
    if (op->cfg.window_kind == HSG_TUMBLING) op->cfg.advance_ms = op->cfg.size_ms;
    memset(&op->stats, 0, sizeof(op->stats));
    // literal forms: extra slots read the literal bit of the valid bytes
    const bool forms = (cfg->flags & HSG_OPF_LITERAL_FORMS) != 0;
    const std::vector<int32_t> &itypes = op->col_types;
    const std::vector<hsg_agg> &iaggs = op->aggs;
    op->user_cols = cfg->n_cols;
    rc = build_program(op->cfg, itypes, iaggs, op->prog, eng->err, forms);
    if (rc != HSG_OK) { delete op; return rc; }
    op->dev.user_cols = cfg->n_cols;
    op->dev.forms = forms;
    if (hipSetDevice(eng->device) != hipSuccess) { delete op; return HSG_E_DEVICE; }
    if (eng->comm) {
      // collective over the engine's ranks: every rank creates its sharded ops
      // in the same order (the same queries)
      std::lock_guard<std::mutex> lk(eng->mu);
      rc = comm_split(eng->comm, &op->comm, eng->err);
      if (rc != HSG_OK) {
        comm_destroy(op->comm);
        delete op;
        return rc;
      }
    }
    // a sharded op's ranks must all reach the agreement below, whatever
    // happened here: exceptions become a status
    try {
      rc = op_device_init(op->dev, op->cfg, op->prog, eng->batch_cap, eng->nranks, op->comm != nullptr,
                          hsg_windows_per_record(op->cfg), eng->err);
    } catch (const std::bad_alloc &) {
      rc = HSG_E_OOM;
      eng->err = "op_device_init: out of host memory";
    } catch (...) {
      rc = HSG_E_DEVICE;
      eng->err = "op_device_init: exception";
    }
    if (op->comm) {
      // the ranks agree on the creation: a rank whose shard failed (e.g. out
      // of memory) takes every rank's shard down with it, so no rank keeps an
      // op whose first exchange would wait forever on the missing one. The
      // failed shard's memory goes first, and the agreement's stream and
      // buffer were made with the communicator (comm_split), so nothing can
      // fail between here and the collective.
      if (rc != HSG_OK) op_device_free(op->dev);
      std::string aerr;
      const int arc = comm_agree(op->comm, rc, aerr);
      if (rc == HSG_OK && arc != HSG_OK) {
        rc = arc;
        eng->err = aerr;
      }
    }
    if (rc != HSG_OK) {
      op_device_free(op->dev);
      comm_destroy(op->comm);
      delete op;
      return rc;
    }
    op->stats.state_slots = (uint64_t)op->prog.n_slots;
    op->stats.state_row_bytes = 8ull * (uint64_t)op->prog.n_slots + (cfg->window_kind == HSG_SESSION ? 16ull : 8ull);
    op->stats.table_slots = op->dev.cap;
    *out = op;
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" void hsg_op_destroy(hsg_op *op) {
  if (!op) return;
  try {
    {
      std::lock_guard<std::mutex> lk(op->qmu);
      op->stopping = true;
    }
    op->qcv.notify_all();
    if (op->worker.joinable()) op->worker.join();  // runs what is queued first
    hipSetDevice(op->eng->device);
    op_device_free(op->dev);
    comm_destroy(op->comm);
  } catch (...) {
  }
  delete op;
}

extern "C" const char *hsg_last_error(const hsg_op *op) { return op ? op->err.c_str() : "null op"; }

extern "C" int hsg_op_reset(hsg_op *op) {
  try {
    if (!op) return HSG_E_INVALID;
    wait_idle(op);
    HIP_TRY(op, hipSetDevice(op->eng->device));
    int rc = op_device_reset(op->dev, op->cfg, op->prog, op->err);
    if (rc != HSG_OK) return rc;
    // counters in hsg_stats are cumulative since create; only the state goes
    op->pending = 0;
    op->state_rows = 0;
    op->rec_base = 0;
    op->stats.state_rows = 0;
    op->stats.pending_rows = 0;
    op->stats.spilled_rows = 0;
    return HSG_OK;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

static int validate_batch(hsg_op *op, const hsg_batch *b, const int64_t *inout_watermark) {
  if (!b || !inout_watermark) return fail(op->err, HSG_E_INVALID, "null batch or watermark");
  if (b->n_cols != op->user_cols) return fail(op->err, HSG_E_INVALID, "batch n_cols != op n_cols");
  if (b->mem != HSG_MEM_HOST && b->mem != HSG_MEM_DEVICE) return fail(op->err, HSG_E_INVALID, "bad batch mem");
  if (b->n > op->eng->batch_cap) return fail(op->err, HSG_E_CAPACITY, "batch larger than the engine's batch_capacity");
  if (b->n && (!b->key_id || !b->ts)) return fail(op->err, HSG_E_INVALID, "null key_id / ts");
  for (int c = 0; c < b->n_cols; ++c)
    if (b->n && (!b->cols || !b->cols[c])) return fail(op->err, HSG_E_INVALID, "null value column");
  // narrow transport (hsg_enc): ts as TS32 / TS16, i64 columns as I32, f64 columns as DEC32
  if (b->ts_enc != HSG_ENC_FULL && b->ts_enc != HSG_ENC_TS32 && b->ts_enc != HSG_ENC_TS16)
    return fail(op->err, HSG_E_INVALID, "bad ts_enc");
  if (b->ts_enc == HSG_ENC_TS16 && b->n && !b->ts_frames) return fail(op->err, HSG_E_INVALID, "TS16 without ts_frames");
  if (b->key_enc != HSG_ENC_FULL && b->key_enc != HSG_ENC_K16) return fail(op->err, HSG_E_INVALID, "bad key_enc");
  for (int c = 0; c < b->n_cols; ++c) {
    const int e = b->col_enc[c];
    const bool f64 = op->col_types[c] == HSG_F64;
    if (e != HSG_ENC_FULL && e != (f64 ? HSG_ENC_DEC32 : HSG_ENC_I32))
      return fail(op->err, HSG_E_INVALID, "bad col_enc for the column's type");
    if (e == HSG_ENC_DEC32 && b->col_scale[c] > 18) return fail(op->err, HSG_E_INVALID, "col_scale > 18");
  }
  return HSG_OK;
}

// The push itself (caller: hsg_push_batch, or the op's completion thread).
static int push_sync(hsg_op *op, const hsg_batch *b, int64_t *inout_watermark, int staged_set) {
  try {
    int rc = validate_batch(op, b, inout_watermark);
    if (rc != HSG_OK) return rc;
    HIP_TRY(op, hipSetDevice(op->eng->device));
    double t0 = now_ms();
    PushResult res;
    PushArgs args;
    args.batch = b;
    args.wm_in = *inout_watermark;
    args.batch_id = ++op->batch_id;
    args.rec_base = op->rec_base;
    args.pending = op->pending;
    args.comm = op->comm;
    args.rank = op->eng->rank;
    args.nranks = op->eng->nranks;
    args.staged_set = staged_set;
    rc = op_push(op->dev, op->cfg, op->prog, args, res, op->err);
    if (rc != HSG_OK && rc != HSG_E_RANGE && rc != HSG_E_OOM) return rc;
    // state was mutated: account for what happened even on OOM / RANGE
    *inout_watermark = res.wm_out;
    op->pending += res.out_rows;
    op->state_rows = res.state_rows;
    op->rec_base += res.global_records;
    op->stats.batches += 1;
    op->stats.records += b->n;
    op->stats.records_owned += res.owned;
    op->stats.pairs = res.pairs;
    op->stats.late_dropped = res.late;
    op->stats.touched = res.touched;
    op->stats.pairs_total += res.pairs;
    op->stats.touched_total += res.touched;
    op->stats.state_rows = op->state_rows;
    op->stats.spilled_rows = op->dev.spilled_rows;
    op->stats.spill_events = op->dev.spill_events;
    op->stats.table_slots = op->dev.cap;
    op->stats.grow_events = op->dev.grow_events;
    op->stats.lean_batches = op->dev.lean_batches;
    op->stats.direct_batches = op->dev.direct_batches;
    op->stats.replays = op->dev.replays;
    op->stats.overflow_rows = op->dev.ovf_rows;
    op->stats.overflow_rebuilds = op->dev.ovf_events;
    op->stats.pending_rows = op->pending;
    op->stats.last_batch_ms = now_ms() - t0;
    op->stats.agg_kernel_ms += res.agg_ms;
    op->stats.agg_kernel_launches += res.agg_launches;
    op->stats.exchange_ms += res.exchange_ms;
    op->stats.exchange_bytes += res.exchange_bytes;
    return rc;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  } catch (...) {
    op->err = "unexpected exception";
    return HSG_E_DEVICE;
  }
}

extern "C" int hsg_push_batch(hsg_op *op, const hsg_batch *b, int64_t *inout_watermark) {
  if (!op) return HSG_E_INVALID;
  int rc = drain_async(op);
  if (rc != HSG_OK) return rc;
  return push_sync(op, b, inout_watermark);
}

extern "C" int hsg_push_batch_async(hsg_op *op, const hsg_batch *b, int64_t *inout_watermark, hsg_done_fn done,
                                    void *ctx) {
  try {
    if (!op) return HSG_E_INVALID;
    int rc = validate_batch(op, b, inout_watermark);
    if (rc != HSG_OK) return rc;
    AsyncJob job;
    job.b = *b;
    if (b->cols) job.cols.assign(b->cols, b->cols + b->n_cols);
    if (b->valid) job.valid.assign(b->valid, b->valid + b->n_cols);
    job.wm = inout_watermark;
    job.done = done;
    job.ctx = ctx;
    std::lock_guard<std::mutex> lk(op->qmu);
    if (op->stopping) return fail(op->err, HSG_E_INVALID, "op is being destroyed");
    if (!op->worker.joinable()) op->worker = std::thread(async_loop, op);
    op->queue.push_back(std::move(job));
    op->qcv.notify_all();
    return HSG_OK;
  } catch (const std::bad_alloc &) {
    return HSG_E_OOM;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" int hsg_op_wait(hsg_op *op) {
  if (!op) return HSG_E_INVALID;
  return drain_async(op);
}

extern "C" int hsg_pending_rows(const hsg_op *op, uint64_t *n) {
  if (!op || !n) return HSG_E_INVALID;
  wait_idle(op);
  *n = op->pending;
  return HSG_OK;
}

static int check_rows(hsg_op *op, const hsg_rows *out) {
  if (!out) return fail(op->err, HSG_E_INVALID, "null rows");
  if (out->n_aggs != op->cfg.n_aggs) return fail(op->err, HSG_E_INVALID, "rows n_aggs != op n_aggs");
  if (out->mem != HSG_MEM_HOST && out->mem != HSG_MEM_DEVICE) return fail(op->err, HSG_E_INVALID, "bad rows mem");
  return HSG_OK;
}

extern "C" int hsg_op_set_changelog(hsg_op *op, const hsg_rows *dst) {
  try {
    if (!op) return HSG_E_INVALID;
    wait_idle(op);
    if (op->pending) return fail(op->err, HSG_E_INVALID, "set_changelog: drain the pending rows first");
    OpDevice &d = op->dev;
    if (!dst) {
      d.out = d.own_out;
      d.out_cap = d.own_out_cap;
      d.ext_out = false;
      return HSG_OK;
    }
    int rc = check_rows(op, dst);
    if (rc != HSG_OK) return rc;
    if (dst->mem != HSG_MEM_DEVICE) return fail(op->err, HSG_E_INVALID, "set_changelog: device columns only");
    if (!dst->key_id || !dst->win_start || !dst->win_end || !dst->src_index || dst->capacity == 0 ||
        (op->cfg.n_aggs && !dst->aggs))
      return fail(op->err, HSG_E_INVALID, "set_changelog: every column is required");
    OutCols o;
    memset(&o, 0, sizeof(o));
    o.key = dst->key_id;
    o.ws = dst->win_start;
    o.we = dst->win_end;
    o.src = dst->src_index;
    for (int j = 0; j < op->cfg.n_aggs; ++j) {
      if (!dst->aggs[j]) return fail(op->err, HSG_E_INVALID, "set_changelog: every column is required");
      o.agg[j] = (int64_t *)dst->aggs[j];
    }
    o.form = op->dev.forms ? dst->form : nullptr;  // (optional: rows then carry no forms)
    d.out = o;
    d.out_cap = dst->capacity;
    d.ext_out = true;
    return HSG_OK;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" int hsg_drain(hsg_op *op, hsg_rows *out, uint64_t *n_out) {
  try {
    if (!op || !n_out) return HSG_E_INVALID;
    wait_idle(op);
    int rc = op->dev.ext_out && !out ? HSG_OK : check_rows(op, out);
    if (rc != HSG_OK) return rc;
    *n_out = op->pending;
    if (!op->dev.ext_out) {
      if (out->capacity < op->pending) return fail(op->err, HSG_E_CAPACITY, "drain: rows capacity < pending rows");
      HIP_TRY(op, hipSetDevice(op->eng->device));
      rc = op_copy_rows(op->dev, op->dev.out, 0, op->pending, op->cfg.n_aggs, out, op->err);
      if (rc != HSG_OK) return rc;
    }
    op->pending = 0;
    op->stats.pending_rows = 0;
    return HSG_OK;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" int hsg_state_rows(hsg_op *op, uint64_t *n) {
  if (!op || !n) return HSG_E_INVALID;
  wait_idle(op);
  *n = op->state_rows;
  return HSG_OK;
}

extern "C" int hsg_dump_state(hsg_op *op, hsg_rows *out, uint64_t *n_out) {
  try {
    if (!op || !n_out) return HSG_E_INVALID;
    wait_idle(op);
    int rc = check_rows(op, out);
    if (rc != HSG_OK) return rc;
    *n_out = op->state_rows;
    if (out->capacity < op->state_rows) return fail(op->err, HSG_E_CAPACITY, "dump: rows capacity < state rows");
    HIP_TRY(op, hipSetDevice(op->eng->device));
    uint64_t n = 0;
    rc = op_dump(op->dev, op->cfg, op->prog, out, &n, op->err);
    *n_out = n;
    return rc;
  } catch (...) {
    return HSG_E_DEVICE;
  }
}

extern "C" int hsg_op_stats(const hsg_op *op, hsg_stats *out) {
  if (!op || !out) return HSG_E_INVALID;
  wait_idle(op);
  *out = op->stats;
  return HSG_OK;
}

namespace hsg {
// For the sink encoder (sink.cpp): the op's device and which changelog
// aggregate columns hold f64 bits.
int op_sink_info(const hsg_op *op, int *device, int *n_aggs, uint32_t *f64_mask, uint32_t *form_mask, int8_t *ident) {
  if (!op) return HSG_E_INVALID;
  *device = op->eng->device;
  *n_aggs = op->prog.n_out;
  uint32_t m = 0, fm = 0;
  for (int j = 0; j < op->prog.n_out; ++j) {
    if (op->prog.out_kind[j] != O_I64) m |= 1u << j;
    if (op->prog.form_kind[j] != F_NONE) fm |= 1u << j;
    // the reference's initial values: SUM Number 0, MIN maxBound, MAX minBound
    // (Codegen.hs:425-469); -1: an aggregate whose f64 prints exactly
    const int32_t kd = op->aggs[j].kind;
    ident[j] = kd == HSG_MIN ? 1 : kd == HSG_MAX ? 2 : kd == HSG_SUM ? 0 : -1;
  }
  *f64_mask = m;
  *form_mask = fm;
  return HSG_OK;
}
}  // namespace hsg

namespace hsg {
// For the join (join.cpp): the engine's device.
int engine_device(const hsg_engine *e) { return e ? e->device : 0; }
int engine_split_comm(hsg_engine *e, Comm **out, int *rank, int *nranks, std::string &err) {
  *out = nullptr;
  *rank = e ? e->rank : 0;
  *nranks = e ? e->nranks : 1;
  if (!e || e->nranks <= 1 || !e->comm) {
    *rank = 0;
    *nranks = 1;
    return HSG_OK;
  }
  std::lock_guard<std::mutex> lk(e->mu);
  return comm_split(e->comm, out, err);
}
}  // namespace hsg
