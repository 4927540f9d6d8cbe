// 3-D instantiations of the LDS-staged implicit-GEMM conv (see conv_impl.h).
#include "conv_impl.h"

namespace esm {

int launch_conv3d(const esm_conv_desc& a, hipStream_t s) {
    using namespace conv;
    if (a.transposed) return launch_geom<true, 4, 2, true>(a, s);
    const int k = a.kh, S = a.stride;
    if (k == 1 && S == 1) return launch_geom<true, 1, 1, false>(a, s);
    if (k == 3 && S == 1) return launch_geom<true, 3, 1, false>(a, s);
    if (k == 3 && S == 2) return launch_geom<true, 3, 2, false>(a, s);
    set_error("conv3d: unsupported kernel/stride combination");
    return ESM_ERR_UNSUPPORTED;
}

}  // namespace esm

#ifdef ESM_CONV_STAMPS
// Diagnostic build only: the 3-D direct kernels' stamps (this translation unit's own copy of
// esm_stamps; the 2-D reader is esm_diag_stamps in conv2d.hip).
extern "C" int esm_diag_stamps3(unsigned long long* host, int max_waves) {
    unsigned int n = 0;
    if (hipDeviceSynchronize() != hipSuccess ||
        hipMemcpyFromSymbol(&n, HIP_SYMBOL(esm::conv::esm_stamp_count), sizeof n) != hipSuccess)
        return -1;
    n = n < static_cast<unsigned>(max_waves) ? n : static_cast<unsigned>(max_waves);
    if (n && hipMemcpyFromSymbol(host, HIP_SYMBOL(esm::conv::esm_stamps), 8ull * n * sizeof(unsigned long long)) != hipSuccess)
        return -1;
    const unsigned int zero = 0;
    if (hipMemcpyToSymbol(HIP_SYMBOL(esm::conv::esm_stamp_count), &zero, sizeof zero) != hipSuccess) return -1;
    return static_cast<int>(n);
}
#endif
