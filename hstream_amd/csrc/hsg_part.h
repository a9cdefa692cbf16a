// Partitioned aggregation for tumbling / hopping / unwindowed ops (per-batch
// and state-only modes): radix-partition the batch by key hash, aggregate each
// partition chunk in an LDS hash table, flush one update per group. Not ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

constexpr int kPartThreads = 256;
constexpr int kPartItems = 16;
constexpr int kPartTile = kPartThreads * kPartItems;  // records per partition-pass workgroup
constexpr int kPartMaxLog2 = 12;                      // up to 4096 partitions
constexpr int kAggThreads = 512;
constexpr uint64_t kAggChunk = 16384;                 // records per aggregation workgroup

struct PartBuffers {
  uint32_t *hist;     // [np * tiles] bucket-major per-tile counts
  uint64_t *off;      // [np * tiles + 1] exclusive prefix
  uint64_t *partial;  // scan partials
  uint64_t *total;    // [4] device scalars
  uint32_t *key;      // [n] partitioned records
  uint32_t *krel;     // [n] first accepted window, relative to the epoch
  uint32_t *nwin;     // [n] accepted windows (consecutive from krel)
  int64_t *col[kMaxCols];
  uint8_t *valid[kMaxCols];
  int64_t *seq1;      // [n] global sequence + 1 (LAST only)
  uint32_t *chunk_start;  // [4097] first aggregation workgroup of each bucket
  uint64_t n_cap;
  uint64_t tiles_cap;
};

struct PartParams {
  int32_t np_log2;    // partitions = 1 << np_log2
  int32_t has_valid;
  int32_t has_seq;
  int32_t pad;
  uint64_t tiles;     // partition-pass tiles of this batch
};

uint64_t part_tiles(uint64_t n);
void launch_part_hist(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                      const int64_t *tprefix, const int64_t *rec_wm, const PartBuffers &pb, DevScalars *sc);
void launch_part_scatter(hipStream_t s, const Batch &b, const TwParams &p, const PartParams &pp,
                         const int64_t *tprefix, const int64_t *rec_wm, const int64_t *seq, const PartBuffers &pb,
                         DevScalars *sc);
// returns false when the op's slot count has no LDS variant (caller falls back)
bool launch_part_agg(hipStream_t s, const Program &prog, const TwParams &p, const PartParams &pp, const TwTable &t,
                     const PartBuffers &pb, uint64_t n, DevScalars *sc);
bool part_supported(const Program &prog);
inline uint64_t part_lds_entries(const Program &prog) {
  return prog.n_slots <= 2 ? 4096 : prog.n_slots <= 6 ? 2048 : 1024;
}

}  // namespace hsg
