// Probe: does the raw-buffer range check include soffset? (gfx950)
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const float* p, float* o, int n, int soff) {
    __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(p), (short)0, n * 4, 0x00020000);
    o[threadIdx.x] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, threadIdx.x * 4, soff, 0));
}
int main() {
    const int n = 64;
    float h[4 * n];
    for (int i = 0; i < 4 * n; ++i) h[i] = 1.0f + i;
    float *d, *o;
    if (hipMalloc(&d, sizeof h) != hipSuccess || hipMalloc(&o, 64 * 4) != hipSuccess) return 1;
    if (hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) return 1;
    // in range; past num_records but inside the allocation (safe whatever the answer)
    const int soffs[2] = {0, 64 * 4};
    for (int t = 0; t < 2; ++t) {
        float r[64];
        hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d, o, n, soffs[t]);
        if (hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost) != hipSuccess) return 1;
        printf("soffset %d: lane0 %.0f lane63 %.0f\n", soffs[t], r[0], r[63]);
        if (t == 1 && r[0] == 0.f) printf("=> soffset IS range-checked\n");
        if (t == 1 && r[0] != 0.f) printf("=> soffset is NOT range-checked\n");
    }
    return 0;
}
