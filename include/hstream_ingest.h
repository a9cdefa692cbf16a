/* libhstream_gpu — host ingest: poll batches of JSON records into the columnar
 * hsg_batch of hstream_gpu.h, with the group key dictionary-encoded.
 *
 * Replaces, for the windowed GROUP BY path, the per-record work the reference
 * does between the poll and the aggregate:
 *   - value decode of every SourceRecord (buildSourceProcessor,
 *     hstream-processing/src/HStream/Processing/Processor.hs:192-204: Aeson
 *     decode to an Object),
 *   - the GROUP BY key (hstream-sql/src/HStream/SQL/Codegen.hs:485-487:
 *     HM.singleton col (getFieldByName value col)), whose identity in the
 *     store is Aeson Value equality (Data.Scientific for numbers, so 1, 1.0,
 *     10e-1 and 1E0 are one key; objects compare as maps),
 *   - the field reads of the aggregate components (Codegen.hs:412-461:
 *     HM.lookup of the column, absent = the accumulator is left alone, a
 *     non-Number under SUM/MIN/MAX throws and the record is dropped by
 *     runTask's catch, Processor.hs:140-143).
 * A record that the reference would drop (undecodable value, missing GROUP BY
 * field, wrong-typed aggregated field) gets key_id = HSG_KEY_NONE: it still
 * moves stream time (Processor.hs:139), exactly as there.
 *
 * Key spellings: equal keys can print differently, because aeson prints a
 * number by its literal's exponent (1 and 1e0 print "1", 1.0 and 10e-1
 * "1.0"). The reference forwards each record with its own recordKey
 * (TimeWindowedStream.hs:94,101), so under EMIT CHANGES a row's key prints as
 * its record spelled it. hsg_decode_json_spelled reports each record's
 * spelling: the key id when it prints like the key's first spelling, else an
 * alternate spelling (HSG_SPELL_ALT | index) with its own text; the sink
 * (hstream_sink.h hsg_sink_encode_spelled) prints each row's key with it.
 *
 * Where the GPU's fixed-width columns cannot hold what Scientific holds, the
 * record is rejected with its own status instead of being rounded: a
 * non-integral number, or one outside int64, in an HSG_I64 column (declare
 * the column HSG_F64 for decimal data).
 *
 * Thread safety: one decoder / dictionary per operator; calls on one object
 * are serialized by the caller (the operator's runTask loop), distinct objects
 * are independent. Decoding itself fans out over n_threads host threads.
 */
#ifndef HSTREAM_INGEST_H
#define HSTREAM_INGEST_H

#include <stddef.h>
#include <stdint.h>

#include "hstream_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* per-record decode status (status[] of hsg_decode_json) */
enum hsg_decode_status {
  HSG_DEC_OK = 0,
  HSG_DEC_NOT_OBJECT = 1,   /* value is not a JSON object / malformed JSON        */
  HSG_DEC_NO_KEY = 2,       /* GROUP BY field absent (getFieldByName throws)       */
  HSG_DEC_TYPE = 3,         /* aggregated field present but not a Number           */
  HSG_DEC_NOT_INTEGRAL = 4, /* non-integral Number in an HSG_I64 column            */
  HSG_DEC_RANGE = 5         /* integral Number outside int64 in an HSG_I64 column   */
};

/* spelling of a record's key (hsg_decode_json_spelled): a key id, or this bit
 * with the index of an alternate spelling */
#define HSG_SPELL_ALT 0x80000000u

/* ---- key dictionary: Aeson Value -> dense u32 id (first-seen order) ------- */
typedef struct hsg_keydict hsg_keydict;
int  hsg_keydict_create(hsg_keydict **out);
void hsg_keydict_destroy(hsg_keydict *d);
uint64_t hsg_keydict_size(const hsg_keydict *d);
/* Id of one JSON value (text), inserting it if new. HSG_E_INVALID for
 * malformed JSON, HSG_E_CAPACITY when 2^32 - 1 keys exist. */
int  hsg_keydict_encode(hsg_keydict *d, const char *json, size_t len, uint32_t *id);
/* The key's JSON text as Aeson's encode prints the value (numbers in
 * Scientific's shortest form: 1.0 -> 1, 0.001 -> 1.0e-3; object members in
 * sorted order). *len = bytes needed; HSG_E_CAPACITY (nothing copied) when
 * cap is smaller, HSG_E_INVALID for an unknown id. */
int  hsg_keydict_text(const hsg_keydict *d, uint32_t id, char *buf, size_t cap, size_t *len);
/* The text of a spelling from hsg_decode_json_spelled (a key id: its first
 * spelling's text, as hsg_keydict_text). Same capacity rule. */
int  hsg_keydict_spelling_text(const hsg_keydict *d, uint32_t spell, char *buf, size_t cap, size_t *len);

/* ---- record decoder --------------------------------------------------------- */
typedef struct {
  const char *key_field;          /* GROUP BY column name (composeColName stream field) */
  int32_t n_cols;                 /* aggregated fields, in hsg_batch column order       */
  const char *const *col_fields;
  const int32_t *col_types;       /* hsg_col_type                                       */
  const uint8_t *col_numeric;     /* 1: must be a Number (SUM/MIN/MAX/AVG/LAST);
                                     0: presence only (COUNT(col): any value, null too) */
  int32_t literal_forms;          /* 1: valid bytes are 1 | (the number's JSON literal had a
                                     negative Scientific exponent, e.g. 2.0 or 25e-1) << 1, for
                                     ops with HSG_OPF_LITERAL_FORMS (hstream_gpu.h)        */
} hsg_decoder_config;

typedef struct hsg_decoder hsg_decoder;
int  hsg_decoder_create(const hsg_decoder_config *cfg, hsg_decoder **out);
void hsg_decoder_destroy(hsg_decoder *d);

/* Decode n records into caller-owned host columns (an hsg_batch's arrays):
 * record i is buf[off[i], off[i+1]) (off has n + 1 entries), its timestamp
 * rec_ts[i] (SourceRecord srcTimestamp) is copied to ts[i]; key_id[i] from
 * the dictionary (ids handed out in record order); cols[c][i] int64 or double;
 * valid[c][i] = 1 when the field is present. status (optional) receives
 * hsg_decode_status per record, *rejected (optional) the records passed as
 * HSG_KEY_NONE. n_threads <= 0: one per hardware thread (at most 32). */
int  hsg_decode_json(hsg_decoder *dec, hsg_keydict *dict, uint64_t n, const char *buf, const uint64_t *off,
                     const int64_t *rec_ts, uint32_t *key_id, int64_t *ts, void *const *cols,
                     uint8_t *const *valid, uint8_t *status, uint64_t *rejected, int n_threads);
/* hsg_decode_json plus spell[i], record i's key spelling (HSG_KEY_NONE for a
 * rejected record): its key id when the key prints like its first spelling,
 * else HSG_SPELL_ALT | an alternate spelling (texts: hsg_keydict_spelling_text). */
int  hsg_decode_json_spelled(hsg_decoder *dec, hsg_keydict *dict, uint64_t n, const char *buf, const uint64_t *off,
                             const int64_t *rec_ts, uint32_t *key_id, int64_t *ts, void *const *cols,
                             uint8_t *const *valid, uint8_t *status, uint64_t *rejected, uint32_t *spell,
                             int n_threads);

/* ---- narrow transport ---------------------------------------------------------
 * A poll batch crosses PCIe before any kernel sees it, so its bytes per record
 * bound a host-fed operator (hstream_gpu.h hsg_enc). The decoder sees every
 * value, so it can pick, per batch, the narrowest encoding that is lossless
 * for the values it decoded; the library widens on the device. */
#define HSG_NARROW_K16   1u  /* key ids as uint16 when every id < 2^16                    */
#define HSG_NARROW_TS16  2u  /* ts as uint16 offsets from per-frame minima (HSG_TS16_FRAME) */
#define HSG_NARROW_TS32  4u  /* ts as int32 offsets from the batch's minimum               */
#define HSG_NARROW_I32   8u  /* HSG_I64 columns as int32 when every value fits             */
#define HSG_NARROW_DEC32 16u /* HSG_F64 columns as int32 decimal mantissas (scale <= 9)     */
#define HSG_NARROW_ALL   31u

/* Rewrite a full-width host batch in place into the narrowest lossless
 * transport `allow` permits: io's arrays are reinterpreted (K16 keys in the
 * first 2n bytes of key_id, TS16 / TS32 offsets in the first 2n / 4n bytes of
 * ts, I32 / DEC32 values in the first 4n bytes of a column) and its encoding
 * fields set. ts_frames: ceil(n / HSG_TS16_FRAME) entries for TS16 (NULL: no
 * TS16). *present_mask (optional): bit c = column c is present in every
 * record with no literal-form bit, so its valid array may be left out.
 * HSG_E_INVALID for a device batch or one already narrow. */
int  hsg_batch_narrow(hsg_batch *io, const int32_t *col_types, uint32_t allow, int64_t *ts_frames,
                      uint32_t *present_mask, int n_threads);

/* Caller-owned host arrays one decoded batch is built in (pinned memory for
 * hsg_push_batch_async), sized for `capacity` records at full width. */
typedef struct {
  uint64_t capacity;
  uint32_t *key_id;             /* capacity entries                                   */
  int64_t *ts;                  /* capacity entries                                   */
  int64_t *ts_frames;           /* ceil(capacity / HSG_TS16_FRAME) entries (TS16)     */
  void *const *cols;            /* n_cols arrays of capacity 8-byte values            */
  uint8_t *const *valid;        /* n_cols arrays of capacity bytes                    */
  uint32_t allow;               /* HSG_NARROW_* the consumer takes; 0 = full width    */
  uint32_t reserved;
  const void *col_ptrs[8];      /* filled by the decoder: the batch's column pointers */
  const uint8_t *valid_ptrs[8]; /* filled: valid pointers, NULL for a column present in every
                                   record (no valid bytes to send)                     */
} hsg_decode_buffers;

/* hsg_decode_json_spelled into `bufs`, then hsg_batch_narrow: *out is a
 * ready hsg_batch (mem = HSG_MEM_HOST) over bufs' arrays, in the narrowest
 * lossless transport bufs->allow permits. spell optional. At most 8 value
 * columns. The batch stays valid until bufs is reused. */
int  hsg_decode_json_batch(hsg_decoder *dec, hsg_keydict *dict, uint64_t n, const char *buf, const uint64_t *off,
                           const int64_t *rec_ts, hsg_decode_buffers *bufs, hsg_batch *out, uint8_t *status,
                           uint64_t *rejected, uint32_t *spell, int n_threads);

#ifdef __cplusplus
}
#endif

#endif /* HSTREAM_INGEST_H */
