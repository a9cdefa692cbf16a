// Scratch of the sort-based paths (per-record changelog, sessions). Not ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

struct PrBuffers {
  uint32_t *cnt;     // [batch] accepted windows per record / valid flags
  uint64_t *off;     // [batch] exclusive prefix of cnt / output positions
  uint32_t *pslot;   // [pairs] sort key (group slot), buffer 0
  uint32_t *pidx;    // [pairs] sort value (pair index / record index), buffer 0
  uint32_t *k1;      // [pairs] sort ping-pong
  uint32_t *v1;      // [pairs]
  uint32_t *prec;    // [pairs] record of each pair
  int64_t *shadow;   // [cap][n_slots] final rows before commit (per-record time windows)
  int64_t *blk_v;    // [seg tiles][kMaxSlots]
  int32_t *blk_f;    // [seg tiles]
  int64_t *carry;    // [seg tiles][kMaxSlots]
  uint64_t *partial; // scan partials
  uint64_t *totals;  // [4] device scalars written by scans
  uint8_t *flags;    // [pairs] head flags (sessions)
  uint32_t *runs;    // [batch + 1] run starts (sessions)
  uint64_t *runidx;  // [batch] exclusive scan of head flags (sessions)
  void *sort_scratch;
  uint64_t max_pairs;
};

void launch_pr_count(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const int64_t *tprefix,
                     const int64_t *rec_wm, const PrBuffers &pb, DevScalars *sc);
void launch_pr_expand(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const int64_t *tprefix,
                      const int64_t *rec_wm, const PrBuffers &pb, DevScalars *sc);
void launch_pr_segscan(hipStream_t s, const Batch &b, const Program &prog, const PrBuffers &pb, const TwParams &p,
                       const TwTable &t, const uint32_t *slot, const uint32_t *pidx, uint64_t P, const int64_t *seq,
                       OutCols out, uint64_t out_base, DevScalars *sc);
uint64_t seg_tiles(uint64_t P);

}  // namespace hsg
