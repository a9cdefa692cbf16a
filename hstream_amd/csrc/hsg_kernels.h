// Internal entry points between the orchestration files. Not part of the ABI.
#pragma once

#include <string>

#include "hsg_internal.h"
#include "hsg_ops.h"

namespace hsg {

// op_device.cpp
int stage_batch(OpDevice &d, const hsg_batch *b, Batch &kb, std::string &err, int staged_set = -1);
TwParams make_tw_params(const hsg_op_config &cfg, const PushArgs &a);
void launch_stream_time(OpDevice &d, const hsg_op_config &cfg, const Batch &kb, int64_t wm_in, int64_t adv);
int fetch_scalars(OpDevice &d, std::string &err);
// wait for stream s: poll an event (5 ms), then block
int poll_stream(OpDevice &d, hipStream_t s, std::string &err);
int clear_batch_scalars(OpDevice &d, std::string &err);
int finish_batch(OpDevice &d, int64_t wm_in, uint64_t n, PushResult &r, std::string &err);
int push_local(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, const Batch &kb,
               const int64_t *seq, const int64_t *rec_wm, PushResult &r, std::string &err);

// per-record changelog for time windows (perrecord.cpp / k_perrecord.hip)
int perrecord_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err);
int part_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err);
bool perrecord_part_eligible(const Program &prog, uint64_t wpr);
int perrecord_part_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, std::string &err);
int push_time_perrecord(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a,
                        const Batch &kb, const int64_t *seq, const int64_t *rec_wm, PushResult &r, std::string &err);

// sessions (session.cpp / k_session.hip)
int session_device_init(OpDevice &d, const hsg_op_config &cfg, const Program &prog, uint64_t rows, std::string &err);
int session_device_reset(OpDevice &d, std::string &err);
void session_device_free(OpDevice &d);
int push_session(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, const Batch &kb,
                 const int64_t *seq, PushResult &r, std::string &err);
void launch_session_dump(OpDevice &d, const hsg_op_config &cfg, const Program &prog, OutCols out, uint64_t cap,
                         uint64_t *counter);

// multi-GPU key exchange (exchange.cpp / k_exchange.hip)
int exchange_device_init(OpDevice &d, const hsg_op_config &cfg, uint64_t batch_cap, std::string &err);
void exchange_device_free(OpDevice &d);
int push_sharded(OpDevice &d, const hsg_op_config &cfg, const Program &prog, const PushArgs &a, PushResult &r,
                 std::string &err);

}  // namespace hsg
