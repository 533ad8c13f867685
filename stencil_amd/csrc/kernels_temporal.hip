// kernels_temporal.hip -- fused two-step (temporal blocking) sweeps.
#include "common.hpp"

namespace stencil {

bool temporal2_supports(const stencil_problem&) { return false; }

int launch_temporal2(const stencil_layout&, const void*, void*, int64_t, int64_t, hipStream_t) {
    return set_error(STENCIL_EUNSUPPORTED, "TEMPORAL2 not built");
}

}  // namespace stencil
