// Microbenchmark: the 1x1 conv 56 -> 16 at 192x624 (ref4x.agg_1.0's A layer), NCHW fp32, in
// variants that isolate the cost of the access pattern, the MFMA chain and the GELU epilogue.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probes/k1_micro scripts/probes/k1_micro.hip
//   ./scripts/probes/k1_micro
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../../esmstereo_amd/csrc/common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr int C = 56, CO = 16, H = 192, W = 624, NG = 14;

__device__ __forceinline__ float ld(__amdgpu_buffer_rsrc_t r, unsigned v, int s) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(v), s, 0));
}

// MODE 0: full (MFMA + GELU + store); 1: MFMA, no GELU; 2: loads only (sum), 3: loads + MFMA, no store
template <int MODE, int R, int CHAINS>
__global__ void __launch_bounds__(256) k1(const float* x, const float* w, float* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n16 = lane & 15, kq = lane >> 4;
    const int x0 = (blockIdx.x * 4 + wave) * 16, y0 = blockIdx.y * R;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, C * H * W * 4, 0x00020000);
    float wv[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) wv[g] = w[(4 * g + kq) * CO + n16];
    unsigned vo[NG];
#pragma unroll
    for (int g = 0; g < NG; ++g) vo[g] = 4u * ((4 * g + kq) * H * W + x0 + n16);
    float bin[R][NG];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int g = 0; g < NG; ++g) bin[r][g] = ld(rs, vo[g], 4 * (y0 + r) * W);
    float sink = 0.f;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        if constexpr (MODE == 2) {
#pragma unroll
            for (int g = 0; g < NG; ++g) sink += bin[r][g];
            continue;
        } else {
            floatx4 acc[CHAINS];
#pragma unroll
            for (int c = 0; c < CHAINS; ++c) acc[c] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int g = 0; g < NG; ++g)
                acc[g % CHAINS] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[g], bin[r][g], acc[g % CHAINS], 0, 0, 0);
#pragma unroll
            for (int c = 1; c < CHAINS; ++c) acc[0] += acc[c];
            if constexpr (MODE == 3) {
                sink += acc[0][0] + acc[0][1] + acc[0][2] + acc[0][3];
                continue;
            }
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = acc[0][j];
                if constexpr (MODE == 0) v = esm::gelu_erf(v);
                out[(4 * kq + j) * H * W + (y0 + r) * W + x0 + n16] = v;
            }
        }
    }
    if (MODE >= 2 && sink == 12345.f) out[0] = sink;
}

// float4 loads of the same bytes (lane = 4 consecutive pixels of one channel), summed: the access
// pattern's floor at 16 B per lane
template <int R>
__global__ void __launch_bounds__(256) k1_f4(const float* x, float* out) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int x0 = (blockIdx.x * 4 + wave) * 16, y0 = blockIdx.y * R;
    float sink = 0.f;
    // 56 channels x 16 px = 224 float4 per row: lane takes (channel c = (lane + 64k) / 4, quad (lane + 64k) % 4)
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const int i = lane + 64 * k;
            if (i < 224) {
                const float4 v = *reinterpret_cast<const float4*>(x + (i >> 2) * H * W + (y0 + r) * W + x0 + 4 * (i & 3));
                sink += v.x + v.y + v.z + v.w;
            }
        }
    if (sink == 12345.f) out[0] = sink;
}

template <typename F>
float timeit(F f, int reps = 200) {
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(a);
    for (int i = 0; i < reps; ++i) f();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    return ms / reps * 1e3f;
}

int main() {
    float *x, *w, *o;
    (void)hipMalloc(&x, 4ull * C * H * W);
    (void)hipMalloc(&w, 4ull * C * CO);
    (void)hipMalloc(&o, 4ull * CO * H * W);
    std::vector<float> hx(static_cast<size_t>(C) * H * W), hw(C * CO);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = std::sin(0.001f * i);
    for (size_t i = 0; i < hw.size(); ++i) hw[i] = std::cos(0.01f * i);
    (void)hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
    const dim3 blk(256);
#define RUN(MODE, R, CH)                                                                                         \
    printf("mode %d R %d chains %d: %7.2f us\n", MODE, R, CH,                                                    \
           timeit([&] { hipLaunchKernelGGL((k1<MODE, R, CH>), dim3(W / 64 + (W % 64 != 0), H / R), blk, 0, 0, x, w, o); }))
    RUN(0, 2, 2); RUN(0, 4, 2); RUN(0, 4, 4); RUN(1, 4, 2); RUN(3, 4, 2); RUN(2, 4, 2); RUN(2, 2, 2); RUN(2, 8, 2);
    printf("float4 loads R 4: %7.2f us\n", timeit([&] { hipLaunchKernelGGL((k1_f4<4>), dim3(W / 64 + 1, H / 4), blk, 0, 0, x, o); }));
    printf("float4 loads R 2: %7.2f us\n", timeit([&] { hipLaunchKernelGGL((k1_f4<2>), dim3(W / 64 + 1, H / 2), blk, 0, 0, x, o); }));
    printf("bytes read %.1f MB, written %.1f MB\n", 4.0 * C * H * W / 1e6, 4.0 * CO * H * W / 1e6);
    return 0;
}
