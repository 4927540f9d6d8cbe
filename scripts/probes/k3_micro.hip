// Microbenchmark: the 3x3 conv 16 -> 16 at 192x624 (ref4x.conv1.1 / agg_1.1), NCHW fp32, register
// weights (the conv_wide.hip form) in variants: rows per wave, row prefetch depth, GELU or not,
// horizontal taps by 3 loads or by DPP row shifts of one load.
//   hipcc -O3 --offload-arch=gfx950 -o scripts/probes/k3_micro scripts/probes/k3_micro.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <vector>

#include "../../esmstereo_amd/csrc/common.h"

typedef float floatx4 __attribute__((ext_vector_type(4)));
constexpr int C = 16, CO = 16, H = 192, W = 624, NG = 4;
constexpr unsigned kOOB = 0x40000000u;

__device__ __forceinline__ float ld(__amdgpu_buffer_rsrc_t r, unsigned v, int s) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(v), s, 0));
}
template <int D>
__device__ __forceinline__ float row_shift(float v) {
    constexpr int ctrl = D > 0 ? (0x100 + D) : (0x110 - D);
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, true));
}

// PF: input rows loaded ahead (1 = next row only; NR = all rows up front); DPP: 1 load + 2 row shifts
template <int R, int PF, bool GELU, bool DPP, int PIPE = 0>
__global__ void __launch_bounds__(256) k3(const float* x, const float* w, float* out) {
    constexpr int NR = R + 2;
    constexpr int VALID = DPP ? 14 : 16;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int n16 = lane & 15, kq = lane >> 4;
    const int x0 = (blockIdx.x * 4 + wave) * VALID - (DPP ? 1 : 0), y0 = blockIdx.y * R;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(x), 0, C * H * W * 4, 0x00020000);
    float wv[9][NG];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int g = 0; g < NG; ++g) wv[t][g] = w[(t * C + 4 * g + kq) * CO + n16];
    const int xo = x0 + n16;
    constexpr int NL = DPP ? 1 : 3;
    unsigned vo[NG][NL];
#pragma unroll
    for (int g = 0; g < NG; ++g)
#pragma unroll
        for (int l = 0; l < NL; ++l) {
            const int xi = DPP ? xo : xo - 1 + l;
            vo[g][l] = (xi >= 0 && xi < W && xo < W) ? 4u * ((4 * g + kq) * H * W + xi) : kOOB;
        }
    auto load_row = [&](float (&d)[NG][NL], int r) {
        const int yi = y0 - 1 + r;
        const int roff = (yi >= 0 && yi < H) ? 4 * yi * W : static_cast<int>(kOOB);
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int l = 0; l < NL; ++l) d[g][l] = ld(rs, vo[g][l], roff);
    };
    floatx4 acc[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = floatx4{0.f, 0.f, 0.f, 0.f};
    constexpr int NB = PF >= NR ? NR : PF + 1;
    float bin[NB][NG][NL];
#pragma unroll
    for (int r = 0; r < NB - 1; ++r) load_row(bin[r], r);
#pragma unroll
    for (int r = 0; r < NR; ++r) {
        if (r + NB - 1 < NR) load_row(bin[(r + NB - 1) % NB], r + NB - 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                float bv;
                if constexpr (DPP) {
                    const float v = bin[r % NB][g][0];
                    bv = dx == 0 ? row_shift<-1>(v) : (dx == 1 ? v : row_shift<1>(v));
                } else {
                    bv = bin[r % NB][g][dx];
                }
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
                    const int ro = r - dy;
                    if (ro < 0 || ro >= R) continue;
                    acc[ro] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[dy * 3 + dx][g], bv, acc[ro], 0, 0, 0);
                }
            }
        // PIPE: the epilogue of the row completed one iteration earlier runs here, after this row's
        // MFMAs were issued (same basic block: the scheduler may fill the MFMA gaps with it)
        const int rf = PIPE ? r - 3 : r - 2;
        if (rf >= 0) {
            const int yo = y0 + rf;
            if (!(yo >= H || xo >= W || xo < 0 || (DPP && (n16 == 0 || n16 == 15)))) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v = acc[rf][j] * 1.01f + 0.01f;
                    if constexpr (GELU) v = esm::gelu_erf(v);
                    out[(4 * kq + j) * H * W + yo * W + xo] = v;
                }
            }
        }
        if constexpr (PIPE == 2) {
#pragma unroll
            for (int i = 0; i < 12; ++i) {
                __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
                __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
            }
        }
    }
    if constexpr (PIPE != 0) {
        const int rf = NR - 3;
        const int yo = y0 + rf;
        if (!(yo >= H || xo >= W || xo < 0)) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = acc[rf][j] * 1.01f + 0.01f;
                if constexpr (GELU) v = esm::gelu_erf(v);
                out[(4 * kq + j) * H * W + yo * W + xo] = v;
            }
        }
    }
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
    (void)hipMalloc(&w, 4ull * 9 * C * CO);
    (void)hipMalloc(&o, 4ull * CO * H * W);
    std::vector<float> hx(static_cast<size_t>(C) * H * W), hw(9 * C * CO);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = std::sin(0.001f * i);
    for (size_t i = 0; i < hw.size(); ++i) hw[i] = 0.1f * std::cos(0.01f * i);
    (void)hipMemcpy(x, hx.data(), hx.size() * 4, hipMemcpyHostToDevice);
    (void)hipMemcpy(w, hw.data(), hw.size() * 4, hipMemcpyHostToDevice);
#define RUN(R, PF, G, D)                                                                                      \
    printf("R %d prefetch %d gelu %d dpp %d: %7.2f us\n", R, PF, G, D, timeit([&] {                            \
               const int valid = D ? 14 : 16;                                                                \
               hipLaunchKernelGGL((k3<R, PF, G, D>), dim3((W + 4 * valid - 1) / (4 * valid), (H + R - 1) / R), \
                                  dim3(256), 0, 0, x, w, o);                                                  \
           }))
    RUN(2, 1, true, false); RUN(4, 2, true, false); RUN(8, 2, true, false); RUN(8, 2, false, false);
#define RUNP(R, PF, P)                                                                                        \
    printf("R %d prefetch %d pipe %d: %7.2f us\n", R, PF, P, timeit([&] {                                     \
               hipLaunchKernelGGL((k3<R, PF, true, false, P>), dim3((W + 63) / 64, (H + R - 1) / R), dim3(256), 0, \
                                  0, x, w, o);                                                                \
           }))
    RUNP(2, 1, 1); RUNP(4, 2, 1); RUNP(8, 2, 1); RUNP(2, 1, 2); RUNP(4, 2, 2); RUNP(8, 2, 2); RUNP(16, 2, 1); RUNP(16, 2, 2);
    return 0;
}
