// Sink encoder internals (k_sink.hip, sink.cpp). Not part of the ABI.
#pragma once

#include "hsg_internal.h"
#include "../../include/hstream_ingest.h"

namespace hsg {

constexpr int kSinkMaxMembers = 16;

// Constant text of a record: fragment f = frag[frag_off[f], frag_off[f + 1])
//   0          {"<key_field>":      key object prefix
//   1          }                    key object suffix
//   2 + m      {"<alias 0>":  /  ,"<alias m>":
//   2 + M      }  (or {} when the value object has no member)
struct SinkDev {
  int32_t windowed;
  int32_t n_members;
  const char *frag;
  uint32_t frag_off[2 + kSinkMaxMembers + 2];
  int32_t agg_index[kSinkMaxMembers];
  uint32_t f64_mask;   // bit j: aggregate column j holds f64 bits
  uint32_t form_mask;  // bit j: aggregate j has literal-form bits in `form` (HSG_OPF_LITERAL_FORMS)
  int8_t ident[kMaxAggs];  // text of aggregate j's initial value: 0 "0", 1 maxBound (MIN), 2 minBound (MAX)
  const char *ktext;   // key texts back to back (the ingest dictionary's)
  const uint64_t *ktoff;
  uint64_t nkeys;
  const char *atext;   // alternate key spellings (hsg_decode_json_spelled), index after index
  const uint64_t *atoff;
  uint64_t nalt;
  // changelog rows (device)
  const uint32_t *key;
  const int64_t *ws;
  const int64_t *agg[kMaxAggs];
  const uint32_t *form;   // per row literal forms (hsg_rows.form), null = none
  const int64_t *src;     // per row source record (spellings only)
  const uint32_t *spell;  // spell[src - src_base] for src in [src_base, src_base + nspell)
  int64_t src_base;
  uint64_t nspell;
};

// per-row key / value byte counts
void launch_sink_len(hipStream_t s, const SinkDev &S, uint64_t n, uint32_t *klen, uint32_t *vlen);
// the records at the scanned offsets
void launch_sink_write(hipStream_t s, const SinkDev &S, uint64_t n, const uint64_t *koff, const uint64_t *voff,
                       char *kbytes, char *vbytes);

}  // namespace hsg
