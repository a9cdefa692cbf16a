// Stream-stream join internals (k_join.hip, join.cpp). Not part of the ABI.
//
// State (both sides in one array, never pruned, as the reference's stores):
//   R  entries (record key, side, ts) -> (join key, handle), sorted by
//      (key, side, ts); one entry per (key, side, ts): the latest record's;
//   T  the timestamps each side's store holds (any key), sorted by (side, ts):
//      tksRange includes its end points only when both are present.
// A batch's records get arrival numbers 1..n (resident entries count as 0);
// sorted by (key, side, ts, arrival) they merge into R by rank, so every
// record can see, by binary search, what the other side held when it
// arrived: per timestamp the latest entry with a smaller arrival.
#pragma once

#include "hsg_internal.h"

namespace hsg {

struct JEnt {
  uint32_t k;       // record key id
  uint32_t jkey;    // join key id (HSG_KEY_NONE: the join field is missing)
  int64_t ts;
  uint64_t handle;
  uint32_t side;    // 0 this, 1 other, 2 dropped (no record key)
  uint32_t arr;     // 0 resident, 1..n batch arrival
};
static_assert(sizeof(JEnt) == 32, "JEnt");

struct TEnt {
  uint32_t side;
  uint32_t arr;     // smallest arrival holding this timestamp (0 resident)
  int64_t ts;
};
static_assert(sizeof(TEnt) == 16, "TEnt");

struct JoinBatchDev {
  uint64_t n;
  const uint8_t *side;
  const uint32_t *key;
  const uint32_t *jkey;
  const int64_t *ts;
  const uint64_t *handle;
  uint32_t rank;    // sharded joins (nranks > 1): this rank stores and probes the
  uint32_t nranks;  // records whose key it owns (join_owner); every record's timestamp
                    // still enters the timestamp set (side | 4 marks a record owned elsewhere)
};

// the rank that stores and probes record key k
__host__ __device__ inline uint32_t join_owner(uint32_t k, uint32_t nranks) {
  return nranks > 1 ? (uint32_t)((key_hash(k) >> 32) % nranks) : 0u;
}
// the rank slices of an all-gathered batch (G slots of `stride` records, slice q
// holding n_q at off[q] .. off[q + 1] of the global batch) -> the global batch
void launch_join_compact(hipStream_t s, const JoinBatchDev &slots, uint64_t stride, const int64_t *off, int G,
                         uint64_t n, uint8_t *side, uint32_t *key, uint32_t *jkey, int64_t *ts, uint64_t *handle);

struct JoinOut {
  uint64_t *this_h;
  uint64_t *other_h;
  uint32_t *jkey;
  int64_t *ts;
};

void launch_join_build(hipStream_t s, const JoinBatchDev &b, JEnt *out);
// sort key of pass p (0: ts low word, 1: ts high word (sign flipped), 2: side,
// 3: record key; order 1 skips pass 3: the timestamp-set sort) for perm[i]
void launch_join_sortkey(hipStream_t s, const JEnt *e, const uint32_t *perm, uint64_t n, int pass, uint32_t *key);
void launch_join_iota(hipStream_t s, uint32_t *perm, uint64_t n);
void launch_join_gather(hipStream_t s, const JEnt *src, const uint32_t *perm, uint64_t n, JEnt *dst);
// merge sorted resident R and sorted batch B into M by rank; pos[arr - 1] =
// the batch entry's index in M
void launch_join_merge(hipStream_t s, const JEnt *R, uint64_t nR, const JEnt *B, uint64_t nB, JEnt *M, uint32_t *pos);
// timestamp set: batch entries sorted by (side, ts, arr) -> one TEnt per
// group head (flags / scan / write), then merge with the resident set
void launch_join_tflags(hipStream_t s, const JEnt *Bt, uint64_t n, uint32_t *flag);
void launch_join_twrite(hipStream_t s, const JEnt *Bt, uint64_t n, const uint32_t *flag, const uint64_t *off, TEnt *out);
void launch_join_tmerge(hipStream_t s, const TEnt *A, uint64_t nA, const TEnt *B, uint64_t nB, TEnt *M);
// probe: count (out == nullptr) or write matches of every batch record
void launch_join_probe(hipStream_t s, const JEnt *M, uint64_t nM, const uint32_t *pos, uint64_t n, const TEnt *T,
                       uint64_t nT, int64_t before, int64_t after, uint32_t *cnt, const uint64_t *off, JoinOut out,
                       uint64_t out_base);
// new state: last entry of every (key, side, ts) group of M (sides 0/1)
void launch_join_rflags(hipStream_t s, const JEnt *M, uint64_t n, uint32_t *flag);
void launch_join_rwrite(hipStream_t s, const JEnt *M, uint64_t n, const uint32_t *flag, const uint64_t *off, JEnt *out);
// new timestamp set: first TEnt of every (side, ts) group, arrival reset
void launch_join_tkeep(hipStream_t s, const TEnt *T, uint64_t n, uint32_t *flag);
void launch_join_tkeep_write(hipStream_t s, const TEnt *T, uint64_t n, const uint32_t *flag, const uint64_t *off,
                             TEnt *out);

}  // namespace hsg
