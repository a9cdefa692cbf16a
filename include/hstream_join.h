/* libhstream_gpu — stream-stream join within a time window, on the GPU.
 *
 * Replaces joinStream / joinStreamProcessor
 * (hstream-processing/src/HStream/Processing/Stream.hs:222-300) over the two
 * InMemoryTimestampedKVStores (Store.hs:316-385) that the SQL
 * `s1 INNER JOIN s2 WITHIN (INTERVAL ...) ON s1.a = s2.b` plan builds
 * (hstream-sql/src/HStream/SQL/Codegen.hs:219-265). Per record, in arrival
 * order over both streams, the reference
 *   1. stores the record in its side's store under (record key, timestamp),
 *      replacing an entry with the same key and timestamp,
 *   2. range-scans the other side's store for the same record key over
 *      [ts - before, ts + after] (this side; the other side swaps before and
 *      after), in ascending timestamp,
 *   3. forwards, for every candidate whose join key equals the record's,
 *      (join key, joiner(this value, other value), max of the timestamps).
 * Two quirks of the reference are kept: the scan includes its end points
 * only when the other store holds some entry (any key) at both end
 * timestamps, else neither (tksRange's Maybe-chained splitLookup,
 * Store.hs:365-372); and a record or candidate without the join field
 * (HSG_KEY_NONE here) ends that record's scan at the first candidate, where
 * the reference's key selector throws (Codegen.hs:241-243; runTask's catch,
 * Processor.hs:140-143).
 *
 * Values stay with the caller: each record carries a 64-bit handle, and the
 * output rows name the two handles the joiner combines. The stores are never
 * pruned, as in the reference.
 */
#ifndef HSTREAM_JOIN_H
#define HSTREAM_JOIN_H

#include "hstream_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int64_t before_ms;        /* JoinWindows jwBeforeMs (SQL: the WITHIN interval) */
  int64_t after_ms;         /* JoinWindows jwAfterMs                             */
  uint64_t batch_capacity;  /* records per push (both sides together)            */
} hsg_join_config;

/* one poll batch, both streams interleaved in arrival order */
typedef struct {
  uint64_t n;
  int32_t mem;                /* hsg_mem of every array                               */
  int32_t reserved0;
  const uint8_t *side;        /* 0 = this stream (left), 1 = the other stream         */
  const uint32_t *key_id;     /* record key (the stores' key), dictionary-encoded     */
  const uint32_t *join_key;   /* join key ({"SelectedKey": field}); HSG_KEY_NONE =
                                 the field is missing                                */
  const int64_t *ts;
  const uint64_t *handle;     /* the caller's reference to the record's value         */
} hsg_join_batch;

/* output rows: joiner(this value, other value) under join_key at ts */
typedef struct {
  uint64_t capacity;
  int32_t mem;
  int32_t reserved0;
  uint64_t *this_handle;
  uint64_t *other_handle;
  uint32_t *join_key;
  int64_t *ts;                /* max of the two records' timestamps */
} hsg_join_rows;

typedef struct hsg_join hsg_join;
int  hsg_join_create(hsg_engine *eng, const hsg_join_config *cfg, hsg_join **out);
void hsg_join_destroy(hsg_join *j);
const char *hsg_join_last_error(const hsg_join *j);
/* Records with key_id == HSG_KEY_NONE are dropped (the reference throws
 * before storing them). Output rows queue until hsg_join_drain. */
int  hsg_join_push(hsg_join *j, const hsg_join_batch *b);
int  hsg_join_pending(const hsg_join *j, uint64_t *n);
/* Same capacity rule as hsg_drain. */
int  hsg_join_drain(hsg_join *j, hsg_join_rows *out, uint64_t *n_out);
/* entries held by the two stores together */
int  hsg_join_state_rows(const hsg_join *j, uint64_t *n);

#ifdef __cplusplus
}
#endif

#endif /* HSTREAM_JOIN_H */
