// Multi-GPU key exchange (k_exchange.hip, exchange.cpp). Not part of the ABI.
#pragma once

#include <rccl/rccl.h>

#include "hsg_internal.h"
#include "hsg_ops.h"

namespace hsg {

constexpr int kMaxRanks = 64;

struct HostComm;  // shared-memory transport (comm.cpp)

struct Comm {
  ncclComm_t comm = nullptr;   // RCCL
  HostComm *host = nullptr;    // HSG_TRANSPORT_HOST (tests: several ranks on one GPU)
  uint64_t slot_bytes = 0;
  int rank = 0;
  int nranks = 1;
  // comm_agree's stream and [nranks + 1] buffer, made with the communicator so
  // that a rank whose op creation failed (out of memory) still reaches the
  // collective without allocating anything
  hipStream_t agree_s = nullptr;
  int64_t *agree_buf = nullptr;
};

// collectives over either transport (RCCL calls, or the host copies)
int comm_group_start(Comm *c, std::string &err);
int comm_group_end(Comm *c, std::string &err);
int comm_allgather(Comm *c, const void *send, void *recv, size_t count, ncclDataType_t dt, size_t elem,
                   hipStream_t s, std::string &err);
int comm_alltoallv(Comm *c, const void *send, const size_t *scount, const size_t *sdispl, void *recv,
                   const size_t *rcount, const size_t *rdispl, ncclDataType_t dt, size_t elem, hipStream_t s,
                   std::string &err);

struct XLayout {
  int32_t words;     // 8-byte words per record
  int32_t ncols;
  int32_t has_seq;
  int32_t has_wm;
  int32_t has_valid;
};

struct XStaging {
  uint32_t *key;
  int64_t *ts;
  int64_t *col[kMaxCols];
  uint8_t *valid[kMaxCols];
  int64_t *seq;
  int64_t *wm;
};

struct XBuffers {
  uint32_t *owner, *idx, *k1, *v1;  // [batch] partition sort
  void *sort_scratch;
  uint64_t *hist;                    // [kMaxRanks + 1]
  int64_t *info;                     // [6 + G] this rank: max, min, n, has_valid, counts[G], changelog
                                     // room, row clamp (exchange.cpp info_words)
  int64_t *info_all;                 // [G * (6 + G)]
  int64_t *h_info;                   // pinned mirror of info_all
  int64_t *h_room;                   // pinned: this rank's changelog room words, copied into info
  int64_t *wm_local;                 // [batch] per-record stream time before the exchange
  uint64_t *send;                    // [batch * max words]
  uint64_t *recv;                    // [G * batch * max words]
  uint64_t batch;                    // per-rank push capacity
};

// columnar exchange buffers of the fast path
struct XCols {
  uint32_t *key;
  int64_t *ts;
  int64_t *col[kMaxCols];
  uint8_t *valid[kMaxCols];
  int64_t *seq;  // sequenced exchange: the record's global arrival index (null: not sent)
  int64_t *wm;   // sequenced exchange with late records: its stream time (null: not sent)
};

uint64_t x_tiles(uint64_t n);
// xl = log2 of the owner partitions (ranks, or more when a test partitions finer)
void launch_x_hist(hipStream_t s, const Batch &b, int xl, bool unwin, uint32_t *hist, uint64_t *text, DevScalars *sc);
void launch_x_info(hipStream_t s, DevScalars *sc, const uint64_t *bstart, int xl, uint32_t G, uint64_t n,
                   bool has_valid, int64_t *info, const uint64_t *text, uint64_t tiles);
void launch_x_scatter(hipStream_t s, const Batch &b, int xl, bool unwin, bool write_valid, int ncols,
                      const uint32_t *offt, const XCols &send);
// the sequenced exchange's scatter: stable (each owner's records in arrival
// order), with the global sequence (seq_base + index) and, when wm is given,
// each record's stream time; all_ts: records of every ts travel (sessions,
// unwindowed), else only ts >= 0 (time windows: the others have no window)
void launch_x_scatter_seq(hipStream_t s, const Batch &b, int xl, bool all_ts, bool write_valid, int ncols,
                          const uint32_t *offt, const XCols &send, uint64_t seq_base, const int64_t *wm);

void launch_x_minmax(hipStream_t s, const int64_t *tmax, const int64_t *tmin, uint64_t n_tiles, uint64_t n,
                     int has_valid, int64_t *info);
void launch_x_owner(hipStream_t s, const Batch &b, uint32_t G, uint32_t *owner, uint32_t *idx, uint64_t *hist);
void launch_x_recwm(hipStream_t s, const Batch &b, const int64_t *tprefix, int64_t *wm);
void launch_x_pack(hipStream_t s, const Batch &b, const XLayout &L, const uint32_t *sidx, uint64_t m,
                   uint64_t seq_base, const int64_t *wm, uint64_t *send);
void launch_x_unpack(hipStream_t s, const XLayout &L, const uint64_t *recv, uint64_t m, const XStaging &st);

}  // namespace hsg
