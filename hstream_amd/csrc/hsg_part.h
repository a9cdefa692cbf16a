// Partitioned aggregation for tumbling / hopping / unwindowed ops (per-batch
// and state-only modes): radix-partition the batch by key hash, aggregate each
// partition chunk in an LDS hash table, flush one update per group. Not ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

constexpr int kPartThreads = 256;
constexpr int kPartMaxLog2 = 11;                      // up to 2048 partitions
constexpr int kPartMaxWords = 11;                     // 2 + 8 columns + seq
constexpr uint64_t kTouchChunk = 4096;                // touched-list entries per emit workgroup
constexpr uint32_t kTouchSkip = kTouchSkipEntry;          // touched-list entry of a later update of a group
constexpr int kMaxSeg = 8;                            // deferred flush segments per aggregation workgroup

// A partitioned record is `words` 8-byte words (wide layout):
//   [key | krel << 32] [nwin | valid bits << 32] [col 0 .. C-1] [seq + 1]?
// krel = first accepted window relative to the epoch, nwin = accepted windows.
// Packed layout (optimistic batches whose windows span < 2^16 advances, C <= 8,
// nwin < 256): words - 1 words, the first one
//   [key | (krel - kbase) << 32 | nwin << 48 | valid bits << 56]
struct PartBuffers {
  uint32_t *hist;         // [tiles][np] tile-major per-tile bucket counts
  uint32_t *offt;         // [tiles][np] tile-major bucket-major-order offsets of each (tile, bucket) run
  uint32_t *segsum;       // [np][nseg] column sums over segments of kColSeg tiles
  uint64_t *segoff;       // [np * nseg] exclusive prefix of segsum (bucket-major)
  uint64_t *bstart;       // [np + 1] first record of each bucket; bstart[np] = records placed
  uint64_t *partial;      // scan partials
  uint64_t *rec;          // [n * words] partitioned records
  uint32_t *chunk_start;  // [np + 1] first aggregation workgroup of each bucket
  uint32_t *chunk_bucket; // [workgroups] bucket of each aggregation workgroup
  uint32_t *touched;      // [touched_cap] one entry per HBM window update: the slot on the group's first
                          // update in the batch, else kTouchSkip (length: sc->scratch[1])
  uint64_t touched_cap;   // records x windows per record: bounds the updates of one batch
  uint64_t *text;         // [2 * tiles] optimistic histogram: per-tile ts extrema images for the decide step
  uint32_t *tcnt;         // [touch_chunks] emit: non-skip entries per chunk
  uint64_t *toff;         // [touch_chunks + 1] exclusive prefix
  uint64_t *tpartial;     // scan partials
  int64_t *wm;            // [n] per-record stream time (written only when late records are possible)
  uint64_t *pane;         // lean aggregation: [n][pane_words] group partials [g][slot 0 .. n_slots-1], each
                          // workgroup's entries at its chunk's record range
  uint64_t *pane_info;    // [workgroups][2]: first entry, entry count | overflow flag << 32
  uint32_t *pane_cnt;     // [workgroups] entry counts, dense (the apply's touched-list prefix)
  uint64_t *seg;          // [workgroups][kMaxSeg][2] general kernel: deferred flush segments (first entry, count)
  uint64_t pane_cap;      // entries pb.pane holds
  uint64_t n_cap;
  uint32_t *tpairs;       // per-record changelog only (else null): [tiles] accepted (record, window)
                          // pairs of each tile, written by the histogram pass
  uint32_t *pos;          // per-record changelog only (else null): [n] partitioned index of each
                          // arrival-order record, written by the scatter
};

struct PartParams {
  int32_t np_log2;    // partitions = 1 << np_log2 (np_log2 + bshift <= 64)
  int32_t has_valid;
  int32_t has_seq;
  int32_t words;
  int32_t tile;       // records per partition-pass workgroup (1024, 2048 or 4096)
  int32_t pane_S;     // aggregation: panes per window (size / advance), 0 = one LDS entry per window
  int32_t rbits;      // aggregation: 2^rbits key-hash rounds per sub-chunk
  int32_t big;        // aggregation variant: 1 = big LDS table, 1024 threads
  int32_t bshift;     // owner bits above the bucket bits in the key hash (multi-GPU, power-of-two ranks)
  int32_t defer;      // aggregation: window updates of exclusive buckets go to pb.pane segments (k_seg_apply)
  int32_t sub;        // partition passes: kPartTileRecs-record sub-tiles per offsets row (one workgroup per row)
  int32_t hold;       // aggregation, general kernels: the worst case (one group per (record, window))
                      // passes `room`: claim nothing, hold back (DevScalars scratch[32] bit 1)
  uint64_t tiles;     // offsets rows of this batch     // partition-pass tiles of this batch
  uint64_t chunk;     // records per aggregation workgroup
  uint64_t room;      // lean path: new groups the table takes this batch (load <= 3/4); past it the
                      // apply claims nothing and the host grows the table and runs the batch again
};

inline int part_words(int n_cols, bool has_seq) { return 2 + n_cols + (has_seq ? 1 : 0); }
constexpr int kPartTileRecs = 4096;                   // records per partition-pass workgroup
inline int part_tile_for(int) { return kPartTileRecs; }
inline uint64_t part_tiles(uint64_t n, int tile) { return (n + tile - 1) / tile; }
// Sub-tiles per offsets row of the optimistic pipeline (the partition
// kernels walk a row's sub-tiles in order). Rows of 2 or 8 tiles shrink the
// (row, bucket) offsets matrix 2x / 8x but measured slower overall on C2
// (staged scatter 184 -> 228 / 249 us: half / an eighth of the workgroups,
// each waiting on its sub-tiles' loads in turn), so one tile per row.
constexpr int kRowSub = 1;

// per-record stream time into wm unless sc->no_late (decided by launch_tile_scan)
void launch_part_recwm(hipStream_t s, const Batch &b, const int64_t *tprefix, const DevScalars *sc, int64_t *wm);
// rec_wm: per-record stream time from a key exchange (else own_wm / none)
// opt: optimistic pass (no record assumed late; also collects the batch's ts
// extrema for launch_part_decide)
void launch_part_hist(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp, const int64_t *rec_wm,
                      const int64_t *own_wm, const PartBuffers &pb, DevScalars *sc, bool opt);
void launch_part_decide(hipStream_t s, DevScalars *sc, const TwParams &p, int64_t wm_in, int64_t grace,
                        bool can_pack, const PartBuffers &pb, uint64_t tiles);
// bucket-major run offsets (offt, bstart) from the tile-major histogram
void launch_part_offsets(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc);
// launch_part_decide + launch_part_offsets in the launches of the offsets
void launch_part_decide_offsets(hipStream_t s, DevScalars *sc, const TwParams &p, int64_t wm_in, int64_t grace,
                                bool can_pack, const PartParams &pp, const PartBuffers &pb);
uint32_t part_nseg(uint64_t tiles);
// maybe_packed: the batch may be in the packed layout (staged variant too)
// wide = false: the wide-layout variant is not launched (predicted packed)
void launch_part_scatter(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                         const int64_t *rec_wm, const int64_t *own_wm, const int64_t *seq, const PartBuffers &pb,
                         DevScalars *sc, bool maybe_packed, bool wide = true);
// returns false when the op's slot count has no LDS variant (caller falls back)
// maybe_packed: the batch may be in the packed layout (launch both variants)
// out (per-batch changelog, else null): the lean path may write the rows itself
bool launch_part_agg(hipStream_t s, const Program &prog, const TwParams &p, const PartParams &pp, const TwTable &t,
                     const PartBuffers &pb, uint64_t n, DevScalars *sc, bool maybe_packed, const OutCols *out,
                     uint64_t out_base, uint64_t out_cap, bool wide = true, bool *lean = nullptr);
bool part_supported(const Program &prog);
// chunk map of the aggregation workgroups (buckets split into pp.chunk records)
void launch_part_chunks(hipStream_t s, const PartParams &pp, const PartBuffers &pb, DevScalars *sc);
// Lean aggregation of packed tumbling / unwindowed batches (pane_S = 1, no key
// rounds, a specialised slot program): records -> LDS table -> group partials
// in pb.pane, applied to the HBM table by a separate launch (k_agg_lean.hip).
// When every group of the batch gets exactly one partial (no bucket split over
// workgroups, no overflow partial) and out is given, the apply writes the
// per-batch changelog rows itself (count in sc->scratch[3]) and leaves the
// touched list empty (sc->scratch[2] = 1; 2 when it filled the touched list
// instead; k_seg_apply: 3 / 4). Returns false when the batch's shape has no lean variant.
bool part_lean_eligible(const Program &prog, const PartParams &pp);
// After the general aggregation kernel with pp.defer: its deferred window
// updates into the HBM table (one workgroup per aggregation workgroup, its
// segments in order), per-batch changelog rows written directly when the
// batch is clean (every window updated once, no split bucket).
void launch_seg_apply(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                      const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols *out, uint64_t out_base,
                      uint64_t out_cap, bool lean);
bool launch_part_agg_lean(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                          const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols *out,
                          uint64_t out_base, uint64_t out_cap);
// The SQL drop-in's op shape (LAST / literal-form slots, k_agg_sql.hip) on
// packed one-window batches: records with their sequence word, the full slot
// algebra; false when the shape has no such variant. A batch the kernels
// cannot finish exactly (a split bucket, an overflowing chunk) leaves
// DevScalars::scratch[35] set and changes nothing: the careful path runs it.
bool sql_lean_eligible(const Program &prog, const PartParams &pp);
bool launch_part_agg_sql(hipStream_t s, dim3 g, const Program &prog, const TwParams &p, const PartParams &pp,
                         const TwTable &t, const PartBuffers &pb, DevScalars *sc, const OutCols *out,
                         uint64_t out_base, uint64_t out_cap);
// per-batch changelog rows of the groups in pb.touched
void launch_part_emit(hipStream_t s, const TwTable &t, const Program &prog, const TwParams &p, const PartBuffers &pb,
                      OutCols out, uint64_t out_base, uint64_t out_cap, DevScalars *sc);
// LDS table entries of the small (2 workgroups per CU) / big (1 per CU) variant
uint64_t part_lds_entries(const Program &prog, bool big);
inline uint64_t touch_chunks(uint64_t cap) { return (cap + kTouchChunk - 1) / kTouchChunk; }
constexpr uint64_t kAggChunk = 32768;                 // most records per aggregation workgroup

}  // namespace hsg
