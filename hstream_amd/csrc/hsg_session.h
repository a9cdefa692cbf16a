// Session windows (k_session.hip, session.cpp). Not part of the ABI.
//
// State (SessTable, hsg_ops.h): a growable open-addressing key table (64-byte
// entries: key, the key's list, an emit mark, a mirror of its last session)
// and, per key, its sessions as a
// list of array-of-struct rows sorted by start in an HBM arena. Sessions of one
// key stay more than `gap` apart (the closure of SessionWindowedStream.hs:84-118
// over the findSessions test of Store.hs:243-272), so a point or a batch run
// touches one contiguous stretch of the list. Lists are bump-allocated; the
// host compacts (and grows) the arena and rehashes the key table between
// kernel passes, never inside one.
//
// Batch paths:
//   merge   (per-batch / state-only emission, no LAST): key-hash partition;
//           per bucket (k_ss_sort) sub-buckets by further key-hash bits, each
//           grouped by key in an LDS hash table and written out sorted by
//           (key, ts), one group record per key; then one thread per key
//           (k_ss_apply) sweep-merges its points with its resident sessions
//           (points closer than the gap chain into one session).
//           Buckets whose sub-buckets do not fit one sort (hot keys) are merged
//           chunk by chunk by one workgroup (k_ss_merge_big). Order-free: the
//           aggregates commute.
//   replay  (per-record changelog or LAST, where arrival order matters):
//           stable sort by key slot, then the key's records replayed in
//           arrival order against its list, exactly as the reference's fold.
#pragma once

#include "hsg_internal.h"
#include "hsg_ops.h"

namespace hsg {

constexpr uint32_t kSessEmptyKey = 0xFFFFFFFFu;

// The arena's free rows are split into regions, each with its own bump
// pointer, so thousands of workgroups reserving lists do not serialise on one
// atomic; a workgroup allocates from region (block id mod kArenaRegions).
constexpr int kArenaRegions = 64;
constexpr int kRegionStride = 16;  // words between region pointers: one 128-byte line each

// arena bookkeeping words (device, SessTable::meta)
enum SessMeta : int {
  M_KEYS = 1,       // live keys in the key table
  M_FAIL = 3,       // a workgroup could not reserve arena rows (the host compacts, then resumes)
  M_TLEN = 4,       // merge path: touched-list entries this batch
  M_GRP = 5,        // merge path: key groups written by k_ss_sort
  M_RUNS = 6,       // merge path: runs written by k_ss_sort
  M_BIG = 7,        // merge path: buckets left to k_ss_merge_big
  M_RELOC = 8,      // merge path: relocated lists whose prefix k_ss_reloc_copy still copies
  M_BRBIG = 9,      // bucket replay: a sub-bucket exceeds kBrCap records (the sort-based replay runs)
  M_BRROWS = 10,    // bucket replay: keyed records of the batch (its per-record changelog rows)
  M_SCRATCH = 15,   // device landing word (compaction total)
  M_RNEED = 16,                              // [kArenaRegions] replay path: rows its list growth needs
  M_RTOP = M_RNEED + kArenaRegions,          // [kArenaRegions x kRegionStride] region bump pointers
  M_REND = M_RTOP + 1,                       //   and ends, interleaved
  M_WORDS = M_RTOP + kArenaRegions * kRegionStride
};

struct SessParams {
  int64_t gap;
  uint64_t rec_base;
  uint32_t batch_id;
  int32_t emit_mode;
};

// Session records after the key-hash partition: [key | valid bits << 32] [ts] [col 0 .. C-1]
constexpr int kSessMaxWords = 2 + kMaxCols;

void launch_ss_reset(hipStream_t s, const SessTable &t);
// key table into a larger one (keys, lists; emit marks start clear)
void launch_ss_rehash(hipStream_t s, const SessTable &from, const SessTable &to);
// arena compaction: plan (new caps = next pow2 of len + 1, >= 4; total ->
// *total), then every list copied into `to`'s arena (same key table)
uint64_t ss_compact_scratch_bytes(uint64_t kcap);
void launch_ss_compact_plan(hipStream_t s, const SessTable &t, void *scratch, uint64_t *total);
void launch_ss_compact_copy(hipStream_t s, const SessTable &from, const SessTable &to, void *scratch);

// replay path
void launch_ss_slot(hipStream_t s, const Batch &b, const SessTable &t, uint32_t *rslot, uint32_t *ridx,
                    uint32_t *vflag, DevScalars *sc);
// phase 0: head flags; phase 1: compact run starts using runidx = exclusive scan of flags
void launch_ss_runs(hipStream_t s, const uint32_t *slot, uint64_t n, uint32_t cap, uint8_t *flag,
                    const uint64_t *runidx, uint32_t *runs, int phase);
// arena rows the replay's list growth needs (-> meta[M_NEED]) and the all-or-nothing check
void launch_ss_replay_need(hipStream_t s, const SessTable &t, const uint32_t *slot, const uint32_t *runs, uint64_t R);
void launch_ss_process(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                       const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs, uint64_t R,
                       const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base, DevScalars *sc);

// merge path
struct SessPart {
  uint32_t *hist;      // [tiles][nb]
  uint32_t *offt;      // [tiles][nb]
  uint64_t *bstart;    // [nb + 1]
  uint64_t *rec;       // [n * words] partitioned records
  uint64_t *tmax;      // [tiles] ts max image per tile (stream time)
  uint32_t *progress;  // [nb] chunks of each big bucket applied (resumable after an arena refill)
  uint32_t *touched;   // [n] key slots rewritten (a big bucket: one entry per chunk and key)
  uint64_t *srec;      // [n][words] records sorted by (key, ts): ts, word 0, columns
  uint32_t *groups;    // [n][4] key groups: key, first record in srec, records, -
  uint8_t *done;       // [n / 256 + 1] apply blocks done (resumable)
  uint64_t *bigmask;   // [nb] sub-buckets left to k_ss_merge_big
  uint64_t *scopy;     // [n][words] per bucket: its records grouped by sub-bucket (k_ss_sort, k_br_subhist)
  uint32_t *gsparse;   // [n][4] group records at their sub-bucket's record positions
  uint64_t *reloc;     // [n][3] relocated lists (old row, new row, rows of the prefix to copy)
  // bucket replay (per-record changelog, LAST, literal forms)
  uint32_t *tkeyed;    // [tiles] keyed records of each arrival tile (k_ss_phist)
  uint64_t *toff;      // [tiles + 1] exclusive prefix: the tile's first changelog row
  uint32_t *subst;     // [nb][65] each bucket's sub-bucket starts (k_br_subhist)
  int64_t *fin;        // [n][2 + n_slots] per arrival index: session start, end, state after the record
  uint64_t *tpartial;  // scan partials over the tiles
};
// bshift: owner bits of the key hash above the bucket bits (multi-GPU)
void launch_ss_phist(hipStream_t s, const Batch &b, int np_log2, int bshift, uint64_t tiles, const SessPart &sp);
void launch_ss_wm(hipStream_t s, const SessPart &sp, uint64_t tiles, int64_t wm_in, DevScalars *sc);
void launch_ss_pscatter(hipStream_t s, const Batch &b, int np_log2, int bshift, uint64_t tiles, int words,
                        bool has_valid, const SessPart &sp);
void launch_ss_sort(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, int np_log2,
                    int bshift, int words, const SessPart &sp, DevScalars *sc);
// n_bound: records of the batch (an upper bound on the groups); writes the
// changelog rows of its keys at out_base + sc->out_rows
void launch_ss_apply(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, uint64_t n_bound,
                     int words, const SessPart &sp, OutCols out, uint64_t out_base, DevScalars *sc);
void launch_ss_merge_big(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, int np_log2,
                         int bshift, int words, const SessPart &sp, DevScalars *sc);
// the prefixes of the lists k_ss_apply relocated (sp.reloc, t.meta[M_RELOC]
// entries), copied after it and before anything reads those lists
void launch_ss_reloc_copy(hipStream_t s, const SessTable &t, const SessPart &sp, uint64_t n_bound);
// per-batch changelog of the keys k_ss_merge_big touched (emit = 0: count only)
void launch_ss_emit(hipStream_t s, const SessTable &t, const Program &prog, const SessPart &sp, uint32_t batch_id,
                    int emit, uint64_t n_bound, OutCols out, uint64_t out_base, DevScalars *sc);

// bucket replay (per-record changelog, LAST, literal forms): records carry
// their arrival index ([word 0 | literal-form bits << 40] [ts] [cols] [index]);
// per bucket, sub-buckets of at most kBrCap records are grouped by key in LDS
// and each key's records replayed in arrival order against its list, the
// state after every record written to sp.fin at its arrival index; the
// changelog is then written in arrival order (k_br_emit). A sub-bucket of more
// than kBrCap records (a hot key) sets M_BRBIG before anything is modified,
// and the batch takes the sort-based replay instead.
#ifndef HSG_BR_CAP
#define HSG_BR_CAP 1024
#endif
constexpr int kBrCap = HSG_BR_CAP;
int br_words(int n_cols);
void launch_br_scatter(hipStream_t s, const Batch &b, int np_log2, int bshift, uint64_t tiles, int words,
                       const SessPart &sp);
void launch_br_subhist(hipStream_t s, const SessTable &t, int np_log2, int bshift, int words, const SessPart &sp);
void launch_br_replay(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                      int np_log2, int bshift, int words, const SessPart &sp, const int64_t *seq, OutCols out,
                      uint64_t out_base, DevScalars *sc);
void launch_br_emit(hipStream_t s, const Batch &b, const SessParams &p, const Program &prog, const SessPart &sp,
                    uint64_t tiles, const int64_t *seq, OutCols out, uint64_t out_base);

void launch_ss_dump(hipStream_t s, const SessTable &t, const Program &prog, OutCols out, uint64_t out_cap,
                    uint64_t *counter);

}  // namespace hsg
