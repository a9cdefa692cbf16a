// Device-side operator state and the host orchestration entry points used by
// hsg_api.cpp. Not part of the ABI.
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "hsg_internal.h"
#include "hsg_part.h"
#include "hsg_perrecord.h"

namespace hsg {

struct Comm;      // RCCL communicator wrapper (hsg_exchange.h)
struct XBuffers;  // exchange scratch (hsg_exchange.h)

int comm_unique_id(uint8_t *out);

// hsg_testing_set_knob (include/hstream_gpu.h): read at op creation
int64_t testing_knob(int knob);
int comm_create(const uint8_t *id, int rank, int nranks, int device, int transport, uint64_t batch_cap, Comm **out,
                std::string &err);
int comm_split(Comm *parent, Comm **out, std::string &err);
// every rank's status of a collective step: the first failing rank's code, else HSG_OK
int comm_agree(Comm *c, int rc_local, std::string &err);
void comm_destroy(Comm *c);

// Session store in HBM (k_session.hip, hsg_session.h): a growable key table
// of 64-byte entries (key, the key's session list, the per-batch emit mark, a
// mirror of the list's last session) and the sessions, sorted by start per
// key, as array-of-struct rows [start][end][stamp][aggs...] in an arena. The
// home slot of a key is the top bits of its key hash below the owner bits, so
// the keys of one partition bucket live in one contiguous stretch of entries.
struct SessKey {
  uint32_t key;    // kSessEmptyKey = free
  uint32_t len;    // sessions
  uint64_t off;    // arena row of the first session
  uint32_t cap;    // rows reserved at off
  uint32_t mvalid; // merge path, <= 2 state slots: ms / me / ma mirror session len - 1
  uint64_t emark;  // merge path: ~batch << 32 | lowest index the batch rewrote (~0 = none)
  int64_t ms, me;  // mirror of the last session: start, end
  int64_t ma[2];   // and its state slots
};
static_assert(sizeof(SessKey) == 64, "SessKey");
constexpr int kSessMirrorSlots = 2;
struct SessTable {
  SessKey *kt;         // [kmask + 1]
  uint64_t kmask;
  uint64_t *rows;      // [arena_cap][stride]
  uint32_t stride;     // 3 + n_slots words
  uint32_t ns;         // n_slots
  uint64_t arena_cap;  // rows
  uint64_t *meta;      // [M_WORDS] device bookkeeping (hsg_session.h SessMeta)
  int32_t kbits;       // log2(kmask + 1)
  int32_t hshift;      // key-hash owner bits skipped by the home slot (multi-GPU)
};

struct OpDevice {
  hipStream_t stream = nullptr;
  hipEvent_t ev_a = nullptr, ev_b = nullptr, ev_c = nullptr, ev_d = nullptr;
  // the time-window table is cleared on a side stream by hsg_op_reset, so the
  // next batch's partition passes (which do not touch it) overlap the clear;
  // the first kernel that touches the table waits for it (wait_table_reset)
  hipStream_t aux = nullptr;
  hipEvent_t ev_reset = nullptr, ev_pre = nullptr;
  bool reset_pending = false;
  // dirty-block map of the table (hsg_internal.h TwTable::dirty): tw.dirty is
  // the map while claims mark it, null once a clear found most blocks dirty
  // (marking then costs more than it saves; whole-table clears from then on)
  bool tw_map_valid = false;  // tw.dirty covers every claim since the last whole-table clear
  uint8_t *tw_dirty_mem = nullptr;
  uint64_t *tw_cnt = nullptr;    // device: dirty blocks the last clear counted
  uint64_t *h_tw_cnt = nullptr;  // pinned copy (read at the next reset)
  bool tw_cnt_pending = false;
  DevScalars *sc = nullptr;     // device
  DevScalars *h_sc = nullptr;   // pinned host mirror
  bool sc_clean = false;        // per-batch scalars already cleared on the stream
  hipEvent_t ev_fetch = nullptr;  // after the fetch of the scalars (fetch_scalars)
  uint64_t batch_cap = 0;       // records this op can take in one push (after exchange)
  int32_t user_cols = 0;        // value columns of the caller's batches (n_cols: the kernels', internal)
  bool forms = false;           // HSG_OPF_LITERAL_FORMS: rows carry literal forms (hsg_rows.form)
  uint64_t wpr = 1;             // max windows per record
  bool sql_lean = false;        // per-batch LAST / literal-form op on the SQL lean kernels (k_agg_sql.hip)
  int sql_skip = 0;             // batches left that skip the SQL lean kernels (refused at the most buckets)
  uint64_t *tkeys = nullptr;    // touched-list group keys across a mid-batch table rebuild (grow-only)
  uint64_t tkeys_cap = 0;
  uint64_t n_tiles_cap = 0;
  int64_t *tile_max = nullptr, *tile_min = nullptr, *tile_prefix = nullptr;
  // staging (host batches, exchange receive side)
  uint32_t *st_key = nullptr;
  int64_t *st_ts = nullptr;
  int64_t *st_col[kMaxCols] = {};
  uint8_t *st_valid[kMaxCols] = {};
  int64_t *st_seq = nullptr;    // global record seq of received records (multi-GPU)
  int64_t *st_wm = nullptr;     // per-record watermark of received records (multi-GPU)
  int32_t *nar_ts = nullptr;    // narrow transport staging of synchronous host pushes (hsg_enc)
  uint16_t *nar_key = nullptr;
  int32_t *nar_col[kMaxCols] = {};
  // prestaged host batches of asynchronous pushes: the H2D
  // copies of the next queued batch run on their own stream, into the other
  // of two staging sets, while the current batch computes (op_prestage)
  struct Staging {
    uint32_t *key = nullptr;
    int64_t *ts = nullptr;
    int64_t *col[kMaxCols] = {};
    uint8_t *valid[kMaxCols] = {};
  };
  Staging pre[2];
  hipStream_t h2d = nullptr;
  hipEvent_t ev_h2d[2] = {nullptr, nullptr};
  // time windows
  TwTable tw = {};
  uint64_t cap = 0;             // table slots (regions; tw.slots() adds the overflow rows)
  uint32_t load8 = 6;           // the table's load limit in eighths: 3/4, and 1/2 for hopping
                                // tables, whose window-block probes grow long past it (the
                                // room checks and growth, op_device.cpp / retention.cpp)
  uint64_t ovf_rows = 0;        // groups in the overflow rows (a region was full): the next batch
                                // first rebuilds the table with twice the slots and larger regions
  int region_log2 = 12;         // log2 of the smallest region (raised by each overflow rebuild)
  uint64_t ovf_events = 0;      // rebuilds an overflow caused
  EmitScratch emit = {};
  // partitioned aggregation (hsg_part.h)
  PartBuffers part = {};
  void *part_mem = nullptr;
  bool use_part = false;
  int np_log2 = 10;             // partitions of the next batch (adapted per batch)
  int rbits = 0;                // key-hash aggregation rounds of the next batch (log2)
  int pane_S = 1;               // panes per window (0: one LDS entry per window)
  int bshift = 0;               // key-hash bits that pick the owner GPU (skipped by local buckets)
  int xpart_log2 = -1;          // owner partition of the fast exchange: log2(ranks), -1 = not a power of two
  bool x_classic = false;       // HSG_KNOB_X_CLASSIC: sequenced batches take the packed classic exchange
  bool agg_big = true;          // aggregation variant of the next batch (big LDS table)
  bool pred_packed = false;     // launch prediction: the last batch was packed (wide variants not launched)
  bool pred_direct = false;     // launch prediction: the last batch's changelog came from the lean apply
  uint64_t lean_batches = 0, direct_batches = 0, replays = 0;  // hsg_stats
  uint64_t lean_pred = 0;  // new groups the next lean batch may make (2x the last one's partials), 0 = none
  uint64_t defer_pred = 0; // hopping: new groups the next batch may make (2x the last one's deferred updates)
  // sessions
  SessTable ss = {};
  uint64_t *h_meta = nullptr;     // pinned mirror of ss.meta
  uint64_t *h_regions = nullptr;  // pinned staging of the arena regions
  uint64_t ss_keys = 0;           // live keys after the last batch (host mirror)
  uint64_t ss_live_max = 0;       // sessions the arena was last compacted for
  void *ss_part = nullptr;        // session partition scratch (tmax, progress)
  bool ss_merge = false;          // sessions take the sort + runs + merge path (else replay)
  // retention (retention.cpp): closed windows moved out of HBM, raw rows of
  // tw.stride words in host memory; hsg_dump_state appends them
  std::vector<uint64_t> spill;
  uint64_t spilled_rows = 0;
  uint64_t spill_events = 0;
  uint64_t grow_events = 0;
  int64_t spill_wm = INT64_MIN;   // highest stream time a spill closed windows at
  // changelog buffer: the op's own, or caller-owned device columns
  // registered with hsg_op_set_changelog (rows land there directly)
  OutCols out = {};
  uint64_t out_cap = 0;
  OutCols own_out = {};
  uint64_t own_out_cap = 0;
  bool ext_out = false;
  // per-record / session scratch (sort + scan)
  PrBuffers pr = {};
  PrPart prp = {};              // per-record changelog on the partitioned pipeline (k_prpart.hip)
  bool pr_part = false;
  void *scratch = nullptr;
  uint64_t scratch_bytes = 0;
  // exchange buffers (multi-GPU)
  void *xsend = nullptr;
  void *xrecv = nullptr;
  uint64_t xbytes = 0;
  uint64_t *h_counts = nullptr;   // pinned [2 * nranks]
  uint64_t *h_tmp = nullptr;      // pinned [8] small host<->device scalars
  XBuffers *x = nullptr;          // key exchange (engines with a communicator)
  uint64_t *d_counts = nullptr;
  int nranks = 1;
  int n_cols = 0;
  int32_t col_types[kMaxCols] = {};
};

struct PushArgs {
  const hsg_batch *batch = nullptr;
  int64_t wm_in = -1;
  uint32_t batch_id = 0;
  uint64_t rec_base = 0;  // global seq of this batch's first record (all ranks)
  uint64_t pending = 0;
  Comm *comm = nullptr;
  int rank = 0;
  int nranks = 1;
  int staged_set = -1;    // host batch already copied into OpDevice::pre[staged_set] (op_prestage)
};

struct PushResult {
  int64_t wm_out = -1;
  uint64_t out_rows = 0;
  uint64_t pairs = 0;
  uint64_t late = 0;
  uint64_t touched = 0;
  uint64_t state_rows = 0;
  uint64_t owned = 0;           // records aggregated here after the exchange
  uint64_t global_records = 0;  // records in this batch over all ranks
  double agg_ms = 0;
  uint64_t agg_launches = 0;
  double exchange_ms = 0;
  uint64_t exchange_bytes = 0;
};

int op_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t batch_cap, int nranks, bool sharded,
                   uint64_t wpr, std::string &err);
void op_device_free(OpDevice &d);
int op_device_reset(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err);
int op_push(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, PushResult &r,
            std::string &err);
// Queue the H2D copies of a host batch into staging set
// `set` on the op's copy stream; the push that names the set (PushArgs::
// staged_set) waits for them on the op's stream. The set must not be in use
// by a push still running.
int op_prestage(OpDevice &d, const hsg_batch *b, int set, std::string &err);
// rows [from, from + n) of src into out at row dst_off
int op_copy_rows(OpDevice &d, const OutCols &src, uint64_t from, uint64_t n, int n_aggs, const hsg_rows *out,
                 std::string &err, uint64_t dst_off = 0);

// retention (retention.cpp)
// table geometry for `cap` slots (stride and bshift kept)
void tw_configure(TwTable &t, uint64_t cap, int window_kind, int region_log2 = 12);
// Before a time-window batch of n_in records at stream time wm_in: when the
// table could pass 3/4 load, move closed windows to the host and rebuild the
// table (growing it until the open rows plus the batch's bound fit at 1/2).
// A watermark below the last spill's brings every spilled row back first.
int tw_maintain(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t n_in, int64_t wm_in,
                uint64_t pending, std::string &err, uint64_t groups_bound = UINT64_MAX);
// append the spilled rows to a dump at row dst_off (*n_out = rows written)
int tw_dump_spilled(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const hsg_rows *out,
                    uint64_t dst_off, uint64_t *n_out, std::string &err);
void tw_retention_reset(OpDevice &d);
// order the op's stream after a pending table clear (no-op when none)
void wait_table_reset(OpDevice &d);
int op_dump(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const hsg_rows *out, uint64_t *n_out,
            std::string &err);

}  // namespace hsg
