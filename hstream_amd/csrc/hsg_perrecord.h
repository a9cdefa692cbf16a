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

// Per-record changelog of time windows on the partitioned pipeline
// (k_prpart.hip). Pairs = (record, accepted window); "bucket-major pair
// position" = the record's index in the partitioned array x wpr + window.
constexpr int kPrPairs = 2048;         // pairs per k_pr_local chunk (its LDS sort)
#ifndef HSG_PR_EMIT_RECS
#define HSG_PR_EMIT_RECS 4096  // one partition tile (C2 per-record 8.21 -> 8.53 G records/s against 16384)
#endif
constexpr int kPrEmitRecs = HSG_PR_EMIT_RECS;  // arrival-order records per k_pr_emit workgroup
struct PrPart {
  uint32_t *tpairs;   // [tiles] accepted pairs of each partition tile (the histogram pass)
  uint64_t *tpoff;    // [tiles] exclusive prefix of tpairs: the tile's first changelog row
  uint32_t *pos;      // [n] partitioned (bucket-major) index of each arrival-order record (the scatter)
  uint64_t *inter;    // [n * wpr][1 + ns] per pair: its partial's index, its inclusive prefix in the chunk
  uint64_t *gkey;     // [n * wpr] group key of each partial
  int64_t *part;      // [n * wpr][ns] each partial's chunk total, then its carry (the row before the chunk)
  uint32_t *cbase;    // [chunks] first partial of each k_pr_local chunk
  uint32_t *ccnt;     // [chunks] partials of each chunk
  uint64_t *counter;  // [8] per-batch device words: [1] != 0 = a bucket too large for k_pr_keysort
                      // (the batch takes the chunked path); cleared before each batch
  uint64_t *partial;  // scan partials
  int64_t *fin;       // one-window ops (k_pr_bucket): [n][ns] each record's changelog state, at its
                      // partitioned position
  uint64_t *krec;     // multi-window ops: [n][words] the partitioned records, key-grouped in each bucket
  uint32_t *kpos;     // [n] partitioned position -> its position in krec
  uint64_t *roff;     // [n] at krec positions: the record's first changelog row << 32 | its arrival index
};

void launch_pr_count(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const int64_t *tprefix,
                     const int64_t *rec_wm, const PrBuffers &pb, DevScalars *sc);
void launch_pr_expand(hipStream_t s, const Batch &b, const TwParams &p, const TwTable &t, const int64_t *tprefix,
                      const int64_t *rec_wm, const PrBuffers &pb, DevScalars *sc);
void launch_pr_segscan(hipStream_t s, const Batch &b, const Program &prog, const PrBuffers &pb, const TwParams &p,
                       const TwTable &t, const uint32_t *slot, const uint32_t *pidx, uint64_t P, const int64_t *seq,
                       OutCols out, uint64_t out_base, DevScalars *sc);
uint64_t seg_tiles(uint64_t P);
struct PartParams;
struct PartBuffers;
// k_pr_local + k_pr_carry + k_pr_emit over a partitioned batch (chunks mapped)
void launch_pr_part(hipStream_t s, const Batch &b, const Program &prog, const TwParams &p, const PartParams &pp,
                    const TwTable &t, const PartBuffers &pb, const PrPart &pr, uint32_t wpr, const int64_t *rec_wm,
                    const int64_t *seq, const OutCols &out, uint64_t out_base, uint64_t out_cap, DevScalars *sc);

}  // namespace hsg
