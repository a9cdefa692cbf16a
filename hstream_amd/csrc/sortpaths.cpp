// Host orchestration of the exact per-record changelog of time windows (and
// the scratch it shares with the session replay path).
#include <hip/hip_runtime.h>

#include <cstring>
#include <string>

#include "hsg_kernels.h"
#include "hsg_perrecord.h"
#include "hsg_sort.h"

namespace hsg {

#define DTRY(expr)                                                          \
  do {                                                                      \
    hipError_t _e = (expr);                                                 \
    if (_e != hipSuccess) {                                                 \
      err = std::string(#expr) + ": " + hipGetErrorString(_e);              \
      return _e == hipErrorOutOfMemory ? HSG_E_OOM : HSG_E_DEVICE;          \
    }                                                                       \
  } while (0)

static int log2u(uint64_t v) {
  int l = 0;
  while ((1ull << l) < v) ++l;
  return l;
}

// bump allocator over one device block
struct Carve {
  char *base;
  uint64_t used = 0;
  template <typename T>
  T *take(uint64_t count) {
    used = (used + 255) & ~255ull;
    T *p = (T *)(base ? base + used : nullptr);
    used += (count ? count : 1) * sizeof(T);
    return p;
  }
};

static void carve_layout(Carve &c, PrBuffers &pb, uint64_t n, uint64_t P, uint64_t shadow_words) {
  uint64_t nseg = seg_tiles(P) + 1;
  uint64_t scan_n = n > P ? n : P;
  pb.cnt = c.take<uint32_t>(n);
  pb.off = c.take<uint64_t>(n + 1);
  pb.pslot = c.take<uint32_t>(P);
  pb.pidx = c.take<uint32_t>(P);
  pb.k1 = c.take<uint32_t>(P);
  pb.v1 = c.take<uint32_t>(P);
  pb.prec = c.take<uint32_t>(P);
  pb.shadow = c.take<int64_t>(shadow_words);
  pb.blk_v = c.take<int64_t>(nseg * kMaxSlots);
  pb.blk_f = c.take<int32_t>(nseg);
  pb.carry = c.take<int64_t>(nseg * kMaxSlots);
  pb.partial = c.take<uint64_t>(scan_partials_needed(scan_n) + 8);
  pb.totals = c.take<uint64_t>(8);
  pb.flags = c.take<uint8_t>(P);
  pb.runs = c.take<uint32_t>(n + 1);
  pb.runidx = c.take<uint64_t>(n + 1);
  pb.sort_scratch = c.take<char>(sort_scratch_bytes(P));
  pb.max_pairs = P;
}

int perrecord_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err) {
  const uint64_t n = d.batch_cap;
  const uint64_t P = n * d.wpr;
  if (P >= 0xFFFFFFFFull) {
    err = "batch_capacity x windows per record must be < 2^32 for the per-record / session paths";
    return HSG_E_INVALID;
  }
  if (d.cap > 0x7FFFFFFFull) {
    err = "state table too large for the sort-based paths (max 2^31 slots)";
    return HSG_E_INVALID;
  }
  uint64_t shadow = cfg.window_kind == HSG_SESSION ? 0 : d.cap * (uint64_t)prog.n_slots;
  Carve probe{nullptr};
  PrBuffers tmp;
  carve_layout(probe, tmp, n, P, shadow);
  DTRY(hipMalloc(&d.scratch, probe.used));
  d.scratch_bytes = probe.used;
  Carve real{(char *)d.scratch};
  carve_layout(real, d.pr, n, P, shadow);
  if (!d.h_tmp) DTRY(hipHostMalloc((void **)&d.h_tmp, 8 * sizeof(uint64_t), hipHostMallocDefault));
  return HSG_OK;
}

int push_time_perrecord(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                        const Batch &kb, const int64_t *seq, const int64_t *rec_wm, PushResult &r, std::string &err) {
  wait_table_reset(d);
  TwParams p = make_tw_params(cfg, a);
  int rc = clear_batch_scalars(d, err);
  if (rc != HSG_OK) return rc;
  uint64_t P = 0;
  if (kb.n) {
    PrBuffers &pb = d.pr;
    launch_stream_time(d, cfg, kb, a.wm_in, p.adv);
    DTRY(hipEventRecord(d.ev_a, d.stream));
    launch_pr_count(d.stream, kb, p, d.tw, d.tile_prefix, rec_wm, pb, d.sc);
    scan_excl_u32(d.stream, pb.cnt, pb.off, kb.n, pb.partial, pb.totals);
    DTRY(hipMemcpyAsync(d.h_tmp, pb.totals, 8, hipMemcpyDeviceToHost, d.stream));
    DTRY(hipStreamSynchronize(d.stream));
    P = d.h_tmp[0];
    if (P > pb.max_pairs) {
      err = "internal: pair count exceeds scratch";
      return HSG_E_DEVICE;
    }
    if (P) {
      launch_pr_expand(d.stream, kb, p, d.tw, d.tile_prefix, rec_wm, pb, d.sc);
      int which = radix_sort_pairs(d.stream, pb.pslot, pb.pidx, pb.k1, pb.v1, P, log2u(d.cap) + 1, pb.sort_scratch);
      const uint32_t *slot = which ? pb.k1 : pb.pslot;
      const uint32_t *idx = which ? pb.v1 : pb.pidx;
      launch_pr_segscan(d.stream, kb, prog, pb, p, d.tw, slot, idx, P, seq, d.out, a.pending, d.sc);
    }
    DTRY(hipEventRecord(d.ev_b, d.stream));
    DTRY(hipGetLastError());
  }
  rc = finish_batch(d, a.wm_in, kb.n, r, err);
  r.out_rows = P;
  if (kb.n) {
    float ms = 0;
    if (hipEventElapsedTime(&ms, d.ev_a, d.ev_b) == hipSuccess) r.agg_ms = ms;
    r.agg_launches = 1;
  }
  return rc;
}

}  // namespace hsg
