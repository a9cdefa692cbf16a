// Session windows (k_session.hip, sortpaths.cpp). Not part of the ABI.
//
// State (SessTable, hsg_ops.h): a growable open-addressing key table
// (key -> slot) and, per slot, the key's sessions as a list sorted by start in
// an HBM arena (structure of arrays). Sessions of one key stay more than `gap`
// apart (the closure of SessionWindowedStream.hs:84-118 over the findSessions
// test of Store.hs:243-272), so a point or a batch run touches one contiguous
// stretch of the list. Lists are bump-allocated; the host compacts (and grows)
// the arena and rehashes the key table between batches, never mid-batch.
//
// Batch paths:
//   merge   (per-batch / state-only emission, no LAST): key-hash partition,
//           then one workgroup per bucket: chunks sorted by (key, ts) in LDS,
//           gap-delimited runs, and per key a sweep-merge of its runs with the
//           key's resident sessions (order-free: COUNT/SUM/MIN/MAX commute).
//   replay  (per-record changelog or LAST, where arrival order matters):
//           stable sort by key slot, then the key's records replayed in
//           arrival order against its list, exactly as the reference's fold.
#pragma once

#include "hsg_internal.h"
#include "hsg_ops.h"

namespace hsg {

constexpr uint32_t kSessEmptyKey = 0xFFFFFFFFu;

// arena bookkeeping words (device, SessTable::meta)
enum SessMeta : int {
  M_TOP = 0,        // arena bump pointer (sessions)
  M_KEYS = 1,       // live keys in the key table
  M_NEED = 2,       // replay path: arena sessions its growth needs this batch
  M_FAIL = 3,       // a workgroup could not reserve arena space (host compacts, resumes)
  M_TLEN = 4,       // merge path: touched-list entries this batch
  M_WORDS = 8
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
// key table into a new table of new_cap slots (keys, list metadata)
void launch_ss_rehash(hipStream_t s, const SessTable &from, const SessTable &to);
// arena compaction: plan (new caps = next pow2 of len + 1, >= 4; total ->
// *total), then every list copied into `to`'s arena (same key table)
uint64_t ss_compact_scratch_bytes(uint64_t kcap);
void launch_ss_compact_plan(hipStream_t s, const SessTable &t, void *scratch, uint64_t *total);
void launch_ss_compact_copy(hipStream_t s, const SessTable &from, const SessTable &to, int n_slots, void *scratch);

// replay path
void launch_ss_slot(hipStream_t s, const Batch &b, const SessTable &t, uint32_t *rslot, uint32_t *ridx,
                    uint32_t *vflag, DevScalars *sc);
// phase 0: head flags; phase 1: compact run starts using runidx = exclusive scan of flags
void launch_ss_runs(hipStream_t s, const uint32_t *slot, uint64_t n, uint32_t cap, uint8_t *flag,
                    const uint64_t *runidx, uint32_t *runs, int phase);
// arena sessions the replay's list growth needs (-> meta[M_NEED])
void launch_ss_replay_need(hipStream_t s, const SessTable &t, const uint32_t *slot, const uint32_t *runs, uint64_t R);
void launch_ss_process(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                       const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs, uint64_t R,
                       const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base, DevScalars *sc);

// merge path
struct SessPart {
  uint32_t *hist;      // [tiles][nb]
  uint32_t *offt;      // [tiles][nb]
  uint64_t *bstart;    // [nb + 1]
  uint64_t *rec;       // [n * words]
  uint64_t *tmax;      // [tiles] ts max image per tile (stream time)
  uint32_t *progress;  // [nb] chunks of each bucket applied (resumable after an arena refill)
  uint32_t *touched;   // [n] key slots a chunk rewrote (one entry per chunk and key)
};
void launch_ss_phist(hipStream_t s, const Batch &b, int np_log2, uint64_t tiles, const SessPart &sp);
void launch_ss_wm(hipStream_t s, const SessPart &sp, uint64_t tiles, int64_t wm_in, DevScalars *sc);
void launch_ss_pscatter(hipStream_t s, const Batch &b, int np_log2, uint64_t tiles, int words, bool has_valid,
                        const SessPart &sp);
void launch_ss_merge(hipStream_t s, const SessParams &p, const SessTable &t, const Program &prog, int np_log2,
                     int words, const SessPart &sp, DevScalars *sc);
// per-batch changelog of the merge path (emit = 0: count the touched sessions only)
void launch_ss_emit(hipStream_t s, const SessTable &t, const Program &prog, const SessPart &sp, uint32_t batch_id,
                    int emit, uint64_t n_bound, OutCols out, uint64_t out_base, DevScalars *sc);

void launch_ss_dump(hipStream_t s, const SessTable &t, const Program &prog, OutCols out, uint64_t out_cap,
                    uint64_t *counter);

}  // namespace hsg
