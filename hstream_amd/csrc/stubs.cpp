// Temporary: multi-GPU entry points not implemented yet.
#include "hsg_kernels.h"
namespace hsg {
static int ni(std::string &err, const char *w) { err = std::string(w) + ": not implemented yet"; return HSG_E_INVALID; }
int exchange_device_init(OpDevice &, const hsg_op_config &, uint64_t, std::string &err) { return ni(err, "exchange"); }
int push_sharded(OpDevice &, const hsg_op_config &, const Program &, const PushArgs &, PushResult &, std::string &err) { return ni(err, "exchange"); }
}
