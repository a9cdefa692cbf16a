// Sink encoder internals (k_sink.hip, sink.cpp). Not part of the ABI.
#pragma once

#include "hsg_internal.h"

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
  const char *ktext;   // key texts back to back (the ingest dictionary's)
  const uint64_t *ktoff;
  uint64_t nkeys;
  // changelog rows (device)
  const uint32_t *key;
  const int64_t *ws;
  const int64_t *agg[kMaxAggs];
};

// per-row key / value byte counts
void launch_sink_len(hipStream_t s, const SinkDev &S, uint64_t n, uint32_t *klen, uint32_t *vlen);
// the records at the scanned offsets
void launch_sink_write(hipStream_t s, const SinkDev &S, uint64_t n, const uint64_t *koff, const uint64_t *voff,
                       char *kbytes, char *vbytes);

}  // namespace hsg
