// k_part_agg instantiations for ops with <= 8 state slots (see hsg_agg.h).
#include "hsg_agg.h"

namespace hsg {

void agg_launch_ms8(hipStream_t s, dim3 g, int W, bool maybe_packed, const Program &prog, const TwParams &p,
                    const PartParams &pp, const TwTable &t, const PartBuffers &pb, DevScalars *sc) {
  agg_launch<8>(s, g, W, maybe_packed, prog, p, pp, t, pb, sc);
}

}  // namespace hsg
