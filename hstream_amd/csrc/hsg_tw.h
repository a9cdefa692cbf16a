// The (key, window) open-addressing hash table in HBM, shared by the atomic
// and the per-record time-window kernels. Not part of the ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

// The table is split into 2^rbits regions by the key-hash bits that also pick
// the partition bucket (below the owner bits): every group of a key lives in
// its region, and a bucket of np <= rbits bits covers whole regions, so the
// workgroup that owns a bucket is the only writer of those regions and may
// claim empty slots with plain stores (tw_claim_exclusive).
//
// Home slot of group g inside its region: the 8 windows of an aligned block of
// one key share one hash and take 8 consecutive rows, so a key's run of
// windows in a batch is a few lines of HBM instead of one random line per
// window. Collisions probe in steps of 8 rows: the region is 8 interleaved
// linear-probing tables (one per window index mod 8), so a displaced block
// stays together and a probe sequence is as short as plain linear probing at
// the same load. Unwindowed tables (every group is window 0) hash plainly and
// probe by 1.
__device__ inline uint64_t tw_region_base(const TwTable &t, uint64_t g) {
  if (!t.rbits) return 0;
  const uint64_t r = (key_hash((uint32_t)(g >> 32)) << t.bshift) >> (64 - t.rbits);
  return r * (t.rmask + 1);
}
__device__ inline uint64_t tw_home_in(const TwTable &t, uint64_t g) {
  if (!t.blocked) return mix64(g) & t.rmask;
  return ((mix64((g >> 3) * 0x9E3779B97F4A7C15ull) << 3) | (g & 7ull)) & t.rmask;
}
__device__ inline uint64_t tw_step(const TwTable &t) { return t.blocked ? 8 : 1; }

// Longest probe sequence: the table runs at load <= 1/2, so a longer one means
// the table is (nearly) full; report that instead of scanning all of HBM.
constexpr uint64_t kMaxProbes = 1ull << 14;

// Overflow rows. A region's sub-table can fill while the table as a whole is
// moderately loaded (a few keys with many open windows each, or a region that
// drew more than its share of keys). The group then goes to the overflow rows
// after the regions, a plain linear-probing table every workgroup may claim
// in with device-scope CAS (only the group's owner ever updates its row, as
// in the regions). The reference's store never refuses a row (ksPut =
// Map.insert, Store.hs:66-68), so neither does a region: every claim that
// counts here makes the host rebuild the table with larger regions before the
// next batch (retention.cpp tw_maintain). Invariant: a group is in the
// overflow only if the probe of its sub-table found no free slot, and slots
// are never freed between rebuilds, so a lookup whose probe meets a free slot
// stops there and one whose probe ends without meeting one continues here.
__device__ inline uint64_t tw_ovf_home(const TwTable &t, uint64_t g) {
  return mix64(g ^ 0x5851F42D4C957F2Dull) & t.omask;
}
__device__ inline int64_t tw_ovf_claim(const TwTable &t, uint64_t g, uint32_t &fresh) {
  const uint64_t base = t.mask + 1;
  uint64_t s = tw_ovf_home(t, g);
  for (uint64_t probe = 0; probe <= t.omask && probe < kMaxProbes; ++probe) {
    uint64_t *kp = t.key(base + s);
    const uint64_t cur = __hip_atomic_load(kp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty) {
      const uint64_t old = atomicCAS((unsigned long long *)kp, (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        t.mark(base + s);
        fresh += 1;
        atomicAdd((unsigned long long *)t.ovf, 1ull);
        return (int64_t)(base + s);
      }
      if (old == g) return (int64_t)(base + s);
    }
    s = (s + 1) & t.omask;
  }
  return -1;  // the overflow rows are full too: ERR_OOM
}
// the same, reporting a claim through isnew instead of a counter
__device__ inline int64_t tw_ovf_claim_new(const TwTable &t, uint64_t g, bool &isnew) {
  uint32_t f = 0;
  const int64_t s = tw_ovf_claim(t, g, f);
  isnew = f != 0;
  return s;
}
__device__ inline int64_t tw_ovf_find(const TwTable &t, uint64_t g) {
  const uint64_t base = t.mask + 1;
  uint64_t s = tw_ovf_home(t, g);
  for (uint64_t probe = 0; probe <= t.omask && probe < kMaxProbes; ++probe) {
    const uint64_t cur = __hip_atomic_load(t.key(base + s), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty) return -1;
    s = (s + 1) & t.omask;
  }
  return -1;
}

// Returns the slot of group g, inserting it if absent (in the overflow rows
// when its region's sub-table is full); -1 only when those are full too. A plain load is only a hint (a stale EMPTY costs one failed CAS); the
// CAS result is authoritative, and a slot moves EMPTY -> g once per reset.
__device__ inline int64_t tw_find_or_insert(const TwTable &t, uint64_t g, uint32_t &fresh) {
  const uint64_t base = tw_region_base(t, g);
  uint64_t s = tw_home_in(t, g);
  const uint64_t step = tw_step(t), n = (t.rmask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    uint64_t cur = *t.key(base + s);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty) {
      uint64_t old =
          atomicCAS((unsigned long long *)t.key(base + s), (unsigned long long)kEmpty, (unsigned long long)g);
      if (old == kEmpty) {
        t.mark(base + s);
        fresh += 1;
        return (int64_t)(base + s);
      }
      if (old == g) return (int64_t)(base + s);
    }
    s = (s + step) & t.rmask;
  }
  return tw_ovf_claim(t, g, fresh);
}

// Same, for the only workgroup writing g's region in this launch: its threads
// claim empty slots with a workgroup-scope CAS, which the XCD's L2 performs
// (no trip to the memory-side atomic unit that device scope needs). A slot
// moves EMPTY -> g once, so a stale plain load can only show EMPTY.
__device__ inline int64_t tw_claim_exclusive(const TwTable &t, uint64_t g, uint32_t &fresh) {
  const uint64_t base = tw_region_base(t, g);
  uint64_t s = tw_home_in(t, g);
  const uint64_t step = tw_step(t), n = (t.rmask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    const uint64_t cur = *t.key(base + s);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty) {
      uint64_t expected = kEmpty;
      if (__hip_atomic_compare_exchange_strong(t.key(base + s), &expected, g, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP)) {
        t.mark(base + s);
        fresh += 1;
        return (int64_t)(base + s);
      }
      if (expected == g) return (int64_t)(base + s);
    }
    s = (s + step) & t.rmask;
  }
  return tw_ovf_claim(t, g, fresh);
}

// Lookup only (after the aggregation pass has inserted every group).
__device__ inline int64_t tw_find(const TwTable &t, uint64_t g) {
  const uint64_t base = tw_region_base(t, g);
  uint64_t s = tw_home_in(t, g);
  const uint64_t step = tw_step(t), n = (t.rmask + 1) / step;
  for (uint64_t probe = 0; probe < n && probe < kMaxProbes; ++probe) {
    uint64_t cur = *t.key(base + s);
    if (cur == g) return (int64_t)(base + s);
    if (cur == kEmpty) return -1;
    s = (s + step) & t.rmask;
  }
  return tw_ovf_find(t, g);  // the probe met no free slot
}

}  // namespace hsg
