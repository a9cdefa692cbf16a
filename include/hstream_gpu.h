/*
 * hstream_gpu.h — C ABI of libhstream_gpu, the MI355X (gfx950) engine behind
 * HStreamDB's windowed GROUP BY operators.
 *
 * What it replaces (reference = Yu-zh/hstream @ 2025-01-17, paths relative to
 * its root):
 *
 *   hsg_op_create (HSG_TUMBLING / HSG_HOPPING)
 *       TimeWindowedStream.aggregate / count
 *         hstream-processing/src/HStream/Processing/Stream/TimeWindowedStream.hs:32-70
 *       with the window spec of mkTumblingWindow / mkHoppingWindow
 *         .../Stream/TimeWindows.hs:23-43
 *   hsg_op_create (HSG_SESSION)
 *       SessionWindowedStream.aggregate / count
 *         .../Stream/SessionWindowedStream.hs:33-72, mkSessionWindows SessionWindows.hs:25-30
 *   hsg_op_create (HSG_UNWINDOWED)
 *       GroupedStream.aggregate / count  .../Stream/GroupedStream.hs:35-87
 *   hsg_push_batch
 *       the per-record processors TimeWindowedStream.aggregateProcessor (:72-117),
 *       SessionWindowedStream.aggregateProcessor (:74-118),
 *       GroupedStream.aggregateProcessor (:71-87), driven for a whole poll batch
 *       instead of record by record by runTask (Processor.hs:128-144), with the
 *       stream-time update of Processor.hs:139 / Processor/Internal.hs:160-166.
 *   hsg_drain
 *       the `forward` of every updated (key, window) row (TimeWindowedStream.hs:101,
 *       SessionWindowedStream.hs:97,118, GroupedStream.hs:87).
 *   hsg_dump_state
 *       ksDump / ssDump (Store.hs:59,81 and :143,238-241) used by views
 *       (hstream/src/HStream/Server/Handler.hs:274-321).
 *   hsg_agg kinds
 *       the SQL aggregate components of hstream-sql/src/HStream/SQL/Codegen.hs:399-469
 *       (COUNT(*), COUNT(col), SUM, MIN, MAX, non-aggregate passthrough = HSG_LAST)
 *       plus AVG, which the reference rejects at codegen (Codegen.hs:462) and which
 *       this ABI defines as SUM(col) / COUNT(col).
 *
 * Conventions (mirroring the reference's own FFI, hstream-store cbits and
 * common/HStream/Stats.hs): opaque handles freed by *_destroy functions that
 * are usable as ForeignPtr finalizers, plain pointers + sizes, int status codes
 * (0 = OK, negative = error), no C++ exception crosses the ABI, a per-handle
 * last-error string. Calls on one op handle must be serialized by the caller;
 * distinct op handles may be used concurrently from different OS threads.
 * hsg_push_batch blocks until the GPU work is done: bind it as a *safe* ccall.
 */
#ifndef HSTREAM_GPU_H
#define HSTREAM_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes --------------------------------------------------------- */
#define HSG_OK           0
#define HSG_E_INVALID   (-1) /* bad argument / unsupported combination           */
#define HSG_E_OOM       (-2) /* HBM state table or session arena full            */
#define HSG_E_CAPACITY  (-3) /* batch larger than capacity / changelog not drained / out buffer too small */
#define HSG_E_DEVICE    (-4) /* HIP runtime error                                */
#define HSG_E_COMM      (-5) /* RCCL error                                       */
#define HSG_E_RANGE     (-6) /* window index outside the op's 2^32-window span   */

/* key id reserved for records that only advance stream time (filtered by WHERE,
 * failed decode, aggregate type error): Processor.hs:139 updates the task
 * timestamp before the topology runs, so such records still move the watermark. */
#define HSG_KEY_NONE 0xFFFFFFFFu

#define HSG_COMM_ID_BYTES 128

/* grace used by every reference window spec: 24 h (TimeWindows.hs:34,42; SessionWindows.hs:29) */
#define HSG_DEFAULT_GRACE_MS 86400000LL

enum hsg_window_kind {
  HSG_TUMBLING   = 0, /* mkTumblingWindow size            (advance = size)      */
  HSG_HOPPING    = 1, /* mkHoppingWindow size advance                           */
  HSG_SESSION    = 2, /* mkSessionWindows gap (grace unused, as in the reference) */
  HSG_UNWINDOWED = 3  /* GroupedStream.aggregate: one implicit window per key   */
};

enum hsg_emit_mode {
  HSG_EMIT_PER_RECORD = 0, /* exact reference changelog: one row per (record, accepted window),
                              arrival order, windows in ascending start              */
  HSG_EMIT_PER_BATCH  = 1, /* one row per group touched by the batch = the last per-record
                              row of that group; order unspecified                     */
  HSG_EMIT_NONE       = 2  /* state only (views)                                       */
};

enum hsg_col_type { HSG_I64 = 0, HSG_F64 = 1 };

enum hsg_agg_kind {
  HSG_COUNT_ALL = 0, /* COUNT(*)   Codegen.hs:404-411, DSL count TimeWindowedStream.hs:59-70 */
  HSG_COUNT     = 1, /* COUNT(col) Codegen.hs:412-422: +1 when the field is present          */
  HSG_SUM       = 2, /* SUM(col)   Codegen.hs:423-435                                        */
  HSG_MIN       = 3, /* MIN(col)   Codegen.hs:449-461, identity maxBound::Int                */
  HSG_MAX       = 4, /* MAX(col)   Codegen.hs:436-448, identity minBound::Int                */
  HSG_AVG       = 5, /* SUM(col)/COUNT(col) as f64 (NaN when COUNT(col) = 0)                 */
  HSG_LAST      = 6  /* non-aggregate SELECT column, Codegen.hs:463-469 (time windows and
                        unwindowed only)                                                     */
};

enum hsg_mem { HSG_MEM_HOST = 0, HSG_MEM_DEVICE = 1 };

/* Narrow transport encodings of a batch's columns (hsg_batch ts_enc / col_enc).
 * A poll batch crosses PCIe before any kernel sees it, so its bytes per record
 * bound a host-fed op's throughput; a producer that knows a column's range
 * (the decoder sees every value) may send it narrower. Lossless: the library
 * widens on the device before the batch runs. */
enum hsg_enc {
  HSG_ENC_FULL  = 0, /* the column's own type: int64 ts, int64 / double values          */
  HSG_ENC_TS32  = 1, /* ts only: int32 offsets from hsg_batch.ts_base                   */
  HSG_ENC_I32   = 2, /* an HSG_I64 column sent as int32 (every value fits)              */
  HSG_ENC_DEC32 = 3, /* an HSG_F64 column sent as int32 decimal mantissas m:
                        value = m / 10^col_scale, the double nearest that decimal,
                        i.e. the double the JSON text of the decimal parses to       */
  HSG_ENC_K16   = 4, /* key_id only: uint16 ids (a dictionary of <= 65536 keys, and
                        no HSG_KEY_NONE record in the batch)                        */
  HSG_ENC_TS16  = 5  /* ts only: uint16 offsets from per-frame bases (frame of
                        reference): record i's ts = ts_frames[i / HSG_TS16_FRAME] +
                        offset[i]; a poll batch's near-sorted timestamps fit when
                        every frame of HSG_TS16_FRAME records spans < 65536 ms     */
};
#define HSG_TS16_FRAME 4096

typedef struct hsg_engine hsg_engine;
typedef struct hsg_op hsg_op;

/* transports of the key exchange */
#define HSG_TRANSPORT_RCCL 0  /* one process per GPU over RCCL (xGMI)                       */
#define HSG_TRANSPORT_HOST 1  /* ranks of one host through shared memory (several ranks may
                                 share one GPU): for testing the multi-rank sequencing    */

typedef struct {
  int32_t device;          /* HIP device ordinal; -1 = the calling thread's current device */
  int32_t rank;            /* this process's rank in the key-sharded group                */
  int32_t nranks;          /* 1 = single GPU, no communicator                              */
  int32_t transport;       /* HSG_TRANSPORT_RCCL (0) or HSG_TRANSPORT_HOST                  */
  const uint8_t *comm_id;  /* RCCL: HSG_COMM_ID_BYTES from hsg_comm_unique_id() on rank 0,
                              shared out of band; HOST: a NUL-terminated segment name (the
                              same on every rank, no '/'); NULL when nranks == 1           */
  uint64_t batch_capacity; /* max records per hsg_push_batch on this rank                   */
} hsg_engine_config;

typedef struct {
  int32_t kind;   /* hsg_agg_kind                                  */
  int32_t column; /* value column index; ignored for HSG_COUNT_ALL */
} hsg_agg;

typedef struct {
  int32_t window_kind;     /* hsg_window_kind                                            */
  int32_t emit_mode;       /* hsg_emit_mode                                              */
  int64_t size_ms;         /* TUMBLING / HOPPING window size  (twSizeMs)                 */
  int64_t advance_ms;      /* HOPPING advance (twAdvanceMs); TUMBLING: = size_ms         */
  int64_t gap_ms;          /* SESSION inactivity gap (swInactivityGap)                   */
  int64_t grace_ms;        /* twGraceMs; use HSG_DEFAULT_GRACE_MS for reference parity  */
  int32_t n_cols;          /* value columns carried by every batch                       */
  int32_t n_aggs;
  const int32_t *col_types;/* n_cols hsg_col_type                                        */
  const hsg_agg *aggs;     /* n_aggs output aggregates, in output order                  */
  uint64_t state_capacity; /* HBM state rows (groups or sessions) to start with; 0 = engine
                            * default (2^21). Time-window tables then grow before a batch
                            * that could pass 3/4 load: by the groups the batch makes on
                            * the lean one-window path (which checks and, if short of
                            * room, grows and runs the batch again), else by one group
                            * per (record, window)                                      */
  uint64_t out_capacity;   /* changelog rows buffered in HBM between drains; 0 = default */
  uint32_t flags;          /* HSG_OPF_* (0 = none)                                        */
  uint32_t reserved;       /* 0                                                           */
} hsg_op_config;

/* hsg_op_config.flags */
#define HSG_OPF_LITERAL_FORMS 1u /* Track how aeson prints each SUM / MIN / MAX / LAST output:
   the reference aggregates Data.Scientific values, and aeson prints a Scientific
   whose exponent is >= 0 as an integer, else in Generic form ("6" vs "6.0",
   hstream-sql/src/HStream/SQL/Codegen/Boilerplate.hs:32-37 objectSerde over
   Codegen.hs:423-469). Batches then mark, in bit 1 of each valid byte, the values
   whose JSON literal had a negative exponent (hstream_ingest.h literal_forms); a
   SUM prints as an integer iff none of its values did (a Scientific sum takes the
   smaller exponent), a MIN / MAX / LAST as its winning literal was spelled, an
   aggregate nothing reached as the reference's initial value. Ties between equal
   values spelled differently (7 and 7.0) resolve as the reference's folds do:
   a time window's or a session's record fold keeps the earlier literal for MIN
   and takes the later for MAX (min n x = n, max n x = x, Codegen.hs:442,455); a
   session merge keeps the merged side's for MIN and takes the existing
   session's for MAX (min n1 n2 / max n1 n2, Codegen.hs:447,460). Changelog and
   dump rows then carry hsg_rows.form. Any number of value columns; such ops run
   on the generic record kernels (the fast partition layouts carry no literal
   bits). */

/* One micro-batch in columnar form, records in arrival order.
 *
 * Device-resident batches (mem = HSG_MEM_DEVICE) are read on the op's own HIP
 * stream, which is not ordered after the stream that produced them: either
 * the producer's writes are complete when hsg_push_batch is called (e.g. the
 * producer synchronised its stream), or ready_event names a hipEvent_t
 * recorded on the producing stream after its last write, and the op's stream
 * waits on it before reading. Host batches are copied to the device inside
 * the call (sync) or before completion is signalled (async). */
typedef struct {
  uint64_t n;
  int32_t mem;                  /* hsg_mem of every pointer below                        */
  int32_t n_cols;               /* must equal the op's n_cols                            */
  const uint32_t *key_id;       /* dictionary-encoded group-by key, HSG_KEY_NONE = skip   */
  const int64_t *ts;            /* event timestamp, ms (record header publish time)      */
  const void *const *cols;      /* n_cols arrays of int64_t or double                    */
  const uint8_t *const *valid;  /* n_cols presence arrays (1 byte/record, 0 = field absent);
                                   NULL or a NULL entry = all present                    */
  void *ready_event;            /* optional hipEvent_t the op's stream waits on (device
                                   batches); NULL = inputs already complete              */
  /* narrow transport (all zero = the full-width arrays above) */
  int32_t ts_enc;               /* HSG_ENC_FULL, HSG_ENC_TS32 (`ts` points at int32_t[n]) or
                                   HSG_ENC_TS16 (`ts` points at uint16_t[n], + ts_frames) */
  int32_t key_enc;              /* HSG_ENC_FULL, or HSG_ENC_K16: `key_id` points at uint16_t[n] */
  int64_t ts_base;              /* HSG_ENC_TS32: ts of a record = ts_base + its offset     */
  uint8_t col_enc[8];           /* per value column: HSG_ENC_FULL, HSG_ENC_I32 (HSG_I64
                                   columns) or HSG_ENC_DEC32 (HSG_F64 columns)            */
  uint8_t col_scale[8];         /* HSG_ENC_DEC32: decimal digits after the point, <= 18   */
  const int64_t *ts_frames;     /* HSG_ENC_TS16: ceil(n / HSG_TS16_FRAME) frame bases (the
                                   batch's hsg_mem); NULL otherwise                       */
} hsg_batch;

/* Columnar changelog / state rows. */
typedef struct {
  uint64_t capacity;   /* rows every array can hold                                    */
  int32_t mem;         /* hsg_mem of every pointer below                               */
  int32_t n_aggs;      /* must equal the op's n_aggs                                   */
  uint32_t *key_id;
  int64_t *win_start;  /* time windows: window start; sessions: session start          */
  int64_t *win_end;    /* time windows: start + size; sessions: session end (inclusive) */
  int64_t *src_index;  /* per-record mode: global index of the producing record; else -1 */
  void *const *aggs;   /* n_aggs arrays: int64_t (COUNT*, SUM/MIN/MAX/LAST of i64) or double */
  uint32_t *form;      /* optional (NULL = not wanted), ops with HSG_OPF_LITERAL_FORMS:
                          per row, bits 2j / 2j+1 of aggregate j: aeson prints it as an
                          integer / it is the aggregate's initial value (nothing reached it) */
} hsg_rows;

typedef struct {
  uint64_t batches;           /* batches pushed since create/reset                     */
  uint64_t records;           /* records pushed (this rank's ingest)                    */
  uint64_t records_owned;     /* records aggregated on this rank after the key exchange */
  uint64_t pairs;             /* accepted (record, window) updates, last batch          */
  uint64_t late_dropped;      /* (record, window) pairs rejected by grace, last batch   */
  uint64_t touched;           /* groups / sessions touched, last batch                  */
  uint64_t state_rows;        /* live groups / sessions                                 */
  uint64_t pending_rows;      /* changelog rows waiting for hsg_drain                   */
  double   last_batch_ms;     /* wall time of the last hsg_push_batch                   */
  double   agg_kernel_ms;     /* cumulative device time of the dominant kernel          */
  uint64_t agg_kernel_launches;
  double   exchange_ms;       /* cumulative device time of the key exchange             */
  uint64_t exchange_bytes;    /* cumulative bytes this rank sent to peers               */
  uint64_t pairs_total;       /* cumulative accepted (record, window) updates           */
  uint64_t touched_total;     /* cumulative groups / sessions touched (summed per batch) */
  uint64_t state_slots;       /* 8-byte aggregate words per state row (the op's program) */
  uint64_t state_row_bytes;   /* algorithmic state row: group key 8 B + 8 B per slot
                                 (sessions: start + end + slots)                        */
  uint64_t spilled_rows;      /* closed windows kept in host memory (counted in state_rows;
                                 hsg_dump_state returns them after the HBM rows)        */
  uint64_t spill_events;      /* retention passes that moved closed windows to the host */
  uint64_t table_slots;       /* HBM hash-table slots (time windows) / key-table slots
                                 (sessions) now                                          */
  uint64_t grow_events;       /* times the HBM table was rebuilt larger                   */
  uint64_t lean_batches;      /* batches aggregated by the lean one-window path            */
  uint64_t direct_batches;    /* ... whose changelog rows the lean apply wrote itself      */
  uint64_t replays;           /* batches completed after the fetch because the predicted
                                 kernel variants did not match the batch (speed only)     */
  uint64_t overflow_rows;     /* groups in the table's overflow rows now: a key-hash region
                                 was full when they were claimed (skewed keys, or keys with
                                 many open windows); the next batch rebuilds the table    */
  uint64_t overflow_rebuilds; /* table rebuilds (twice the slots, twice the region size)
                                 that overflow rows caused                               */
} hsg_stats;

/* Completion callback of hsg_push_batch_async: rc is what hsg_push_batch
 * would have returned. Runs on the op's completion thread; it must not call
 * back into the same op. The Haskell binding passes a C shim that stores rc
 * and calls hs_try_putmvar(cap, mvar), the pattern of
 * hstream-store/cbits/logdevice/hs_writer.cpp:29-44. */
typedef void (*hsg_done_fn)(void *ctx, int rc);

/* ---- engine: one per process and GPU ---------------------------------------- */
int  hsg_comm_unique_id(uint8_t *out, size_t len);
int  hsg_engine_create(const hsg_engine_config *cfg, hsg_engine **out);
void hsg_engine_destroy(hsg_engine *eng);
const char *hsg_engine_last_error(const hsg_engine *eng);

/* ---- operator: one per windowed GROUP BY -------------------------------------- */
int  hsg_op_create(hsg_engine *eng, const hsg_op_config *cfg, hsg_op **out);
void hsg_op_destroy(hsg_op *op);
int  hsg_op_reset(hsg_op *op);            /* drop all state and pending rows          */
const char *hsg_last_error(const hsg_op *op);

/* Process one batch. *inout_watermark is the task's stream time (initially -1,
 * Processor/Internal.hs:151); it is read as the value before the batch and
 * overwritten with the value after it (max over all ranks' records). */
int  hsg_push_batch(hsg_op *op, const hsg_batch *batch, int64_t *inout_watermark);

/* Asynchronous hsg_push_batch: validates and queues the batch, returns at
 * once (HSG_OK = queued, or an argument error). Queued batches of one op run
 * in call order on the op's completion thread; *inout_watermark is read when
 * the batch starts (so consecutive pushes may share one watermark variable)
 * and written before done(ctx, rc) is called. The batch's arrays (not the
 * hsg_batch struct itself, which is copied) must stay valid until done runs.
 * Any other call on the op first waits for the queue to drain. Bind as an
 * unsafe ccall: it never blocks on the GPU. */
int  hsg_push_batch_async(hsg_op *op, const hsg_batch *batch, int64_t *inout_watermark, hsg_done_fn done,
                          void *ctx);
/* Block until every queued asynchronous push of the op has completed; returns
 * the first non-OK status among them (HSG_OK if none), and clears it. */
int  hsg_op_wait(hsg_op *op);

int  hsg_pending_rows(const hsg_op *op, uint64_t *n);
/* Move up to out->capacity pending changelog rows into out (oldest first). If
 * the pending rows do not fit, copies nothing, sets *n_out to the number
 * pending and returns HSG_E_CAPACITY. */
int  hsg_drain(hsg_op *op, hsg_rows *out, uint64_t *n_out);

/* Zero-copy changelog: register caller-owned DEVICE columns (every column,
 * capacity rows) that pushes then write their changelog rows into directly, at
 * the pending offset; hsg_drain only reports and resets the pending count
 * (rows are at [0, n) of the registered columns; `out` may be NULL). NULL
 * restores the op's own buffer. Pending rows must be drained first. No
 * counterpart in the reference, whose forward hands rows to the sink one by
 * one (Processor.hs:221-266); here it saves a device copy per drain. */
int  hsg_op_set_changelog(hsg_op *op, const hsg_rows *dst);

int  hsg_state_rows(hsg_op *op, uint64_t *n);
/* Copy every live state row (views). Same capacity rule as hsg_drain. */
int  hsg_dump_state(hsg_op *op, hsg_rows *out, uint64_t *n_out);

/* Counters are cumulative since hsg_op_create (hsg_op_reset keeps them);
 * "last batch" fields describe the most recent hsg_push_batch. */
int  hsg_op_stats(const hsg_op *op, hsg_stats *out);

/* ---- testing hooks (not used by the drop-in) ----------------------------------
 * Process-wide knobs that let tests reach rare paths at small sizes; they apply
 * to ops created afterwards. Production code never sets them (defaults). */
#define HSG_KNOB_XPART_LOG2     1 /* a 1-rank exchange partitions its records into 2^v owner
                                     regions, all its own (0..6); -1 = log2(ranks)          */
#define HSG_KNOB_SESS_ARENA_MIN 2 /* floor of the session arena in rows (> 0); 0 = 2^20      */
#define HSG_KNOB_X_CLASSIC      3 /* 1: sequenced batches of a sharded op take the packed
                                     classic exchange instead of the columnar one            */
int  hsg_testing_set_knob(int32_t knob, int64_t value);

#ifdef __cplusplus
}
#endif
#endif /* HSTREAM_GPU_H */
