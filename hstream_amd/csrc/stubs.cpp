// Temporary: entry points not implemented yet.
#include "hsg_kernels.h"
namespace hsg {
static int ni(std::string &err, const char *w) { err = std::string(w) + ": not implemented yet"; return HSG_E_INVALID; }
int perrecord_device_init(OpDevice &, const hsg_op_config &, const Program &, std::string &) { return HSG_OK; }
int push_time_perrecord(OpDevice &, const hsg_op_config &, const Program &, const PushArgs &, const Batch &,
                        const int64_t *, const int64_t *, PushResult &, std::string &err) { return ni(err, "per-record"); }
int push_time_atomic_sharded(OpDevice &, const hsg_op_config &, const Program &, const PushArgs &, const Batch &,
                             const int64_t *, const int64_t *, PushResult &, std::string &err) { return ni(err, "sharded"); }
int session_device_init(OpDevice &, const hsg_op_config &, const Program &, uint64_t, std::string &err) { return ni(err, "session"); }
int push_session(OpDevice &, const hsg_op_config &, const Program &, const PushArgs &, const Batch &, const int64_t *,
                 PushResult &, std::string &err) { return ni(err, "session"); }
void launch_session_dump(OpDevice &, const hsg_op_config &, const Program &, OutCols, uint64_t, uint64_t *) {}
int exchange_device_init(OpDevice &, const hsg_op_config &, uint64_t, std::string &err) { return ni(err, "exchange"); }
int push_sharded(OpDevice &, const hsg_op_config &, const Program &, const PushArgs &, PushResult &, std::string &err) { return ni(err, "exchange"); }
}
