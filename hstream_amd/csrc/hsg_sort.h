// Scan and radix-sort primitives (k_sort.hip). Not part of the ABI.
#pragma once

#include "hsg_internal.h"

namespace hsg {

uint64_t scan_partials_needed(uint64_t n);
// exclusive prefix sums into u64; total written to *total (device)
void scan_excl_u32(hipStream_t s, const uint32_t *in, uint64_t *out, uint64_t n, uint64_t *partial, uint64_t *total);
void scan_excl_u8(hipStream_t s, const uint8_t *in, uint64_t *out, uint64_t n, uint64_t *partial, uint64_t *total);

uint64_t sort_scratch_bytes(uint64_t n);
// Stable LSD sort of n (key, value) pairs on the low `bits` key bits.
// Returns which buffer pair holds the result (0: k0/v0, 1: k1/v1).
int radix_sort_pairs(hipStream_t s, uint32_t *k0, uint32_t *v0, uint32_t *k1, uint32_t *v1, uint64_t n, int bits,
                     void *scratch);

}  // namespace hsg
