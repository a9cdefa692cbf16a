// Session-window kernels (k_session.hip). Not part of the ABI.
#pragma once

#include "hsg_internal.h"
#include "hsg_ops.h"

namespace hsg {

constexpr uint64_t kSessInline = 2;  // sessions reserved per key slot before the dynamic arena

struct SessParams {
  int64_t gap;
  uint64_t rec_base;
  uint64_t dyn_base;   // first arena index of the dynamic region (= cap * kSessInline)
  uint32_t batch_id;
  int32_t emit_mode;
};

void launch_ss_reset(hipStream_t s, const SessTable &t, uint64_t cap);
void launch_ss_slot(hipStream_t s, const Batch &b, const SessTable &t, uint32_t *rslot, uint32_t *ridx,
                    uint32_t *vflag, DevScalars *sc);
// phase 0: head flags; phase 1: compact run starts using runidx = exclusive scan of flags
void launch_ss_runs(hipStream_t s, const uint32_t *slot, uint64_t n, uint32_t cap, uint8_t *flag,
                    const uint64_t *runidx, uint32_t *runs, int phase);
void launch_ss_process(hipStream_t s, const Batch &b, const SessParams &p, const SessTable &t, const Program &prog,
                       const uint32_t *slot, const uint32_t *ridx, const uint32_t *runs, uint64_t R,
                       const uint64_t *out_pos, const int64_t *seq, OutCols out, uint64_t out_base,
                       uint64_t *arena_top, DevScalars *sc);
void launch_ss_dump(hipStream_t s, const SessTable &t, uint64_t cap, const Program &prog, OutCols out,
                    uint64_t out_cap, uint64_t *counter);

}  // namespace hsg
