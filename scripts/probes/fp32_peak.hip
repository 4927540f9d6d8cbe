// Probe: attainable fp32 throughput on gfx950 of (a) v_mfma_f32_16x16x4_f32 with 4 independent
// accumulators per wave and (b) packed VALU FMA (v_pk_fma_f32 on float2), all operands in
// registers.  Prints TFLOP/s for each.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float floatx4 __attribute__((ext_vector_type(4)));
typedef float floatx2 __attribute__((ext_vector_type(2)));

__global__ void __launch_bounds__(256) mfma_loop(float* out, int iters, float x) {
    floatx4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    float a = x + threadIdx.x, b = x - threadIdx.x;
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
        }
    }
    floatx4 s = c0 + c1 + c2 + c3;
    out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y + s.z + s.w;
}

__global__ void __launch_bounds__(256) pkfma_loop(float* out, int iters, float x) {
    floatx2 acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = floatx2{x * j, x + j};
    const floatx2 w = {x * 0.999f, x * 1.001f};
    const floatx2 v = {0.5f + threadIdx.x * 1e-6f, 0.25f};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
        for (int u = 0; u < 16; ++u)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[j] = __builtin_elementwise_fma(acc[j], w, v);
    }
    float s = 0;
#pragma unroll
    for (int j = 0; j < 8; ++j) s += acc[j].x + acc[j].y;
    out[blockIdx.x * 256 + threadIdx.x] = s;
}

int main() {
    const int blocks = 256 * 8, iters = 2000;
    float* out;
    if (hipMalloc(&out, blocks * 256 * sizeof(float)) != hipSuccess) return 1;
    hipEvent_t e0, e1;
    if (hipEventCreate(&e0) != hipSuccess || hipEventCreate(&e1) != hipSuccess) return 1;
    for (int rep = 0; rep < 2; ++rep) {
        float ms = 0;
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(mfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
        hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 1;
        hipEventElapsedTime(&ms, e0, e1);
        const double fl = 2.0 * 16 * 16 * 4 * 16.0 * iters * (blocks * 4.0);  // per wave: 16 mfma/iter
        printf("mfma_f32_16x16x4  %.1f TFLOP/s (%.3f ms)\n", fl / (ms * 1e-3) / 1e12, ms);
        hipEventRecord(e0, 0);
        hipLaunchKernelGGL(pkfma_loop, dim3(blocks), dim3(256), 0, 0, out, iters, 1.0f);
        hipEventRecord(e1, 0);
        if (hipEventSynchronize(e1) != hipSuccess) return 1;
        hipEventElapsedTime(&ms, e0, e1);
        const double fv = 2.0 * 2 * 8 * 16.0 * iters * (blocks * 256.0);
        printf("v_pk_fma_f32      %.1f TFLOP/s (%.3f ms)\n", fv / (ms * 1e-3) / 1e12, ms);
    }
    return 0;
}
