// 2-D instantiations of the LDS-staged implicit-GEMM conv (see conv_impl.h).
#include "conv_impl.h"

namespace esm {

int launch_conv2d(const esm_conv_desc& a, hipStream_t s) {
    using namespace conv;
    if (a.transposed) return launch_geom<false, 4, 2, true>(a, s);
    const int k = a.kh, S = a.stride;
    if (k == 1 && S == 1) return launch_geom<false, 1, 1, false>(a, s);
    if (k == 3 && S == 1) return launch_geom<false, 3, 1, false>(a, s);
    if (k == 3 && S == 2) return launch_geom<false, 3, 2, false>(a, s);
    if (k == 5 && S == 1) return launch_geom<false, 5, 1, false>(a, s);
    set_error("conv2d: unsupported kernel/stride combination");
    return ESM_ERR_UNSUPPORTED;
}

}  // namespace esm
