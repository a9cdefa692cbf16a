// The (key, window) open-addressing hash table in HBM, shared by the atomic
// and the per-record time-window kernels. Not part of the ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

// Returns the slot of group g, inserting it if absent; -1 when the table is full.
// A plain load is only a hint (a stale EMPTY costs one failed CAS); the CAS
// result is authoritative, and a slot moves EMPTY -> g at most once per reset.
__device__ inline int64_t tw_find_or_insert(const TwTable &t, uint64_t g, uint32_t &fresh) {
  uint64_t s = mix64(g) & t.mask;
  for (uint64_t probe = 0; probe <= t.mask; ++probe) {
    uint64_t cur = t.keys[s];
    if (cur == g) return (int64_t)s;
    if (cur == kEmpty) {
      uint64_t old = atomicCAS((unsigned long long *)&t.keys[s], (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        fresh += 1;
        return (int64_t)s;
      }
      if (old == g) return (int64_t)s;
    }
    s = (s + 1) & t.mask;
  }
  return -1;
}

// Lookup only (after the aggregation pass has inserted every group).
__device__ inline int64_t tw_find(const TwTable &t, uint64_t g) {
  uint64_t s = mix64(g) & t.mask;
  for (uint64_t probe = 0; probe <= t.mask; ++probe) {
    uint64_t cur = t.keys[s];
    if (cur == g) return (int64_t)s;
    if (cur == kEmpty) return -1;
    s = (s + 1) & t.mask;
  }
  return -1;
}

}  // namespace hsg
