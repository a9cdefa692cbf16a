/* libhstream_gpu — sink encoding of changelog rows, on the GPU.
 *
 * Replaces what happens to each changelog row after the aggregate in the
 * reference's SQL plan (hstream-sql/src/HStream/SQL/Codegen.hs:540-575):
 *   - alias projection of the value object (genTimeWindowKeyMapR,
 *     Codegen.hs:355-369: the members named in the SELECT list),
 *   - the sink's key serde: for windowed GROUP BY timeWindowKeySerde
 *     objectSerde (timeWindowSerde 3000) (Codegen.hs:202-212, Boilerplate.hs:60-74,
 *     TimeWindows.hs:68-73) = int64BE win_start ++ int64BE 0 ++ encode key;
 *     without a window objectSerde (Codegen.hs:213-217) = encode key,
 *   - the value serde objectSerde = aeson encode of the value object,
 * so the bytes handed to the stream append (Processor.hs:252-266) come out of
 * one kernel pass over the changelog instead of one Aeson encode per row.
 * The key object is {key_field: key value} (Codegen.hs:485-487) with the key's
 * text from the ingest dictionary (hstream_ingest.h): under EMIT CHANGES each
 * row's key in its own record's spelling (hsg_sink_encode_spelled with the
 * batch's spellings from hsg_decode_json_spelled: 1 vs 1.0), as the reference
 * forwards each record with its own key (TimeWindowedStream.hs:94,101).
 * Numbers print as aeson prints the reference's Data.Scientific
 * (Boilerplate.hs:32-37 objectSerde): an exponent >= 0 as an integer, else
 * Scientific's Generic form of the shortest round-trip decimal ("2.5", "4.0",
 * "1.0e-3"). For an op with HSG_OPF_LITERAL_FORMS the rows' form column says
 * which (a SUM of integer literals prints "6", of decimal ones "6.0"; a MIN /
 * MAX / LAST as its winning value was written) and which rows hold an
 * aggregate's initial value ("0", MIN "9223372036854775807", MAX
 * "-9223372036854775808", Codegen.hs:404-469). Rows without forms print
 * integer columns plainly and f64 columns in Generic form, identities as those
 * initial values.
 * Members are written in aeson's order for an Object, the traversal order of
 * its HashMap (hashable-1.3.0.0 Text hash, unordered-containers-0.2.10.0,
 * Stack lts-16.21; restated in sink.cpp, pinned by that restatement only: no
 * reference test prints an encoded object).
 */
#ifndef HSTREAM_SINK_H
#define HSTREAM_SINK_H

#include "hstream_gpu.h"
#include "hstream_ingest.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
  int32_t windowed;            /* 1: key = int64BE start ++ int64BE 0 ++ key object; 0: key object */
  int32_t n_members;           /* value object members (<= 16)                                   */
  const char *key_field;       /* the key object is {key_field: value}                            */
  const char *const *aliases;  /* member names, SELECT order                                      */
  const int32_t *agg_index;    /* changelog aggregate column of each member; -1 = the GROUP BY
                                  value itself (SELECT of the grouping column)                    */
} hsg_sink_config;

typedef struct {
  int32_t mem;                 /* hsg_mem of the four arrays                                      */
  int32_t reserved0;
  uint64_t key_capacity;       /* bytes of key_bytes                                              */
  uint64_t value_capacity;     /* bytes of value_bytes                                            */
  char *key_bytes;             /* record i's key: key_bytes[key_off[i], key_off[i+1])             */
  uint64_t *key_off;           /* n + 1 entries                                                   */
  char *value_bytes;
  uint64_t *value_off;         /* n + 1 entries                                                   */
} hsg_sink_records;

typedef struct hsg_sink hsg_sink;

/* The op gives the aggregate columns' types and the device; the dictionary
 * the keys' text (it may keep growing: new keys are uploaded per encode). */
int  hsg_sink_create(hsg_op *op, const hsg_keydict *dict, const hsg_sink_config *cfg, hsg_sink **out);
void hsg_sink_destroy(hsg_sink *s);
/* Encode n changelog rows (host or device columns, as hsg_drain or
 * hsg_op_set_changelog deliver them; key_id, win_start and the aggregates are
 * read). *key_need / *value_need receive the bytes the records take; when
 * they exceed the capacities nothing is written and HSG_E_CAPACITY returned. */
int  hsg_sink_encode(hsg_sink *s, const hsg_rows *rows, uint64_t n, hsg_sink_records *out, uint64_t *key_need,
                     uint64_t *value_need);

/* The records' own key spellings (hsg_decode_json_spelled) for the rows of
 * hsg_sink_encode_spelled: a row whose src_index is in [src_base, src_base + n)
 * prints its key as spell[src_index - src_base]; other rows (per-batch rows,
 * src_index -1) print the key's first spelling. */
typedef struct {
  const uint32_t *spell;
  uint64_t n;
  int64_t src_base;    /* global index of spell[0]'s record (the batch's first record) */
  int32_t mem;         /* hsg_mem of spell */
  int32_t reserved;
} hsg_sink_spellings;
/* hsg_sink_encode with the records' key spellings (sp may be NULL); rows'
 * src_index is read when sp is given. */
int  hsg_sink_encode_spelled(hsg_sink *s, const hsg_rows *rows, uint64_t n, const hsg_sink_spellings *sp,
                             hsg_sink_records *out, uint64_t *key_need, uint64_t *value_need);
/* The order the value object's members are written in: order[k] = index (in
 * aliases) of the k-th member written. For tests and hosts that build the
 * same objects. */
int  hsg_sink_member_order(const char *const *aliases, int32_t n, int32_t *order);
/* One value's text as the encoder prints it (is_f64: 0 bits is an int64, 1 a
 * double's bit pattern printed exactly, 2 / 3 / 4 the double of a SUM / MIN /
 * MAX aggregate of a row without literal forms, whose identity -0.0 / 2^63 /
 * -2^63 prints as the reference's initial value 0 / maxBound / minBound).
 * *len = text bytes; HSG_E_CAPACITY if cap < *len. */
int  hsg_format_number(int32_t is_f64, int64_t bits, char *buf, size_t cap, size_t *len);

#ifdef __cplusplus
}
#endif

#endif /* HSTREAM_SINK_H */
