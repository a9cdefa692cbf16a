// The (key, window) open-addressing hash table in HBM, shared by the atomic
// and the per-record time-window kernels. Not part of the ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

// Home slot of group g: the 8 windows of an aligned block of one key share one
// hash and take 8 consecutive rows, so a key's run of windows in a batch is a
// few lines of HBM instead of one random line per window. Collisions probe in
// steps of 8 rows: the table is 8 interleaved linear-probing tables (one per
// window index mod 8), so a displaced block stays together and a probe
// sequence is as short as plain linear probing at the same load.
// Unwindowed tables (every group is window 0) hash plainly and probe by 1.
__device__ inline uint64_t tw_home(const TwTable &t, uint64_t g) {
  if (!t.blocked) return mix64(g) & t.mask;
  return ((mix64((g >> 3) * 0x9E3779B97F4A7C15ull) << 3) | (g & 7ull)) & t.mask;
}
__device__ inline uint64_t tw_step(const TwTable &t) { return t.blocked ? 8 : 1; }

// Longest probe sequence: the table runs at load <= 1/2, so a longer one means
// the table is (nearly) full; report that instead of scanning all of HBM.
constexpr uint64_t kMaxProbes = 1ull << 14;

// Returns the slot of group g, inserting it if absent; -1 when the table is full.
// A plain load is only a hint (a stale EMPTY costs one failed CAS); the CAS
// result is authoritative, and a slot moves EMPTY -> g at most once per reset.
__device__ inline int64_t tw_find_or_insert(const TwTable &t, uint64_t g, uint32_t &fresh) {
  uint64_t s = tw_home(t, g);
  const uint64_t step = tw_step(t), n = (t.mask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    uint64_t cur = *t.key(s);
    if (cur == g) return (int64_t)s;
    if (cur == kEmpty) {
      uint64_t old = atomicCAS((unsigned long long *)t.key(s), (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        fresh += 1;
        return (int64_t)s;
      }
      if (old == g) return (int64_t)s;
    }
    s = (s + step) & t.mask;
  }
  return -1;
}

// Lookup only (after the aggregation pass has inserted every group).
__device__ inline int64_t tw_find(const TwTable &t, uint64_t g) {
  uint64_t s = tw_home(t, g);
  const uint64_t step = tw_step(t), n = (t.mask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    uint64_t cur = *t.key(s);
    if (cur == g) return (int64_t)s;
    if (cur == kEmpty) return -1;
    s = (s + step) & t.mask;
  }
  return -1;
}

}  // namespace hsg
