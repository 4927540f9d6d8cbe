// Disparity regressions on the aggregated cost [B, D, H, W] (fp32, HBM-bound, one thread
// per pixel, loads coalesced along W, D walked sequentially).
//
//  disparity_regression  models/submodule.py:211-216: out = sum_d cost[d] * d  (NO softmax;
//                        products rounded, then summed in d order -> bit-exact with the
//                        reference's `torch.sum(x * arange, 1)`)
//  regression_topk k=2   models/submodule.py:218-225: top-2 of D (value desc, lowest index
//                        first on ties), softmax over the pair, sum of index*prob.
#include "common.h"

// products rounded, then summed (torch.sum(x * arange)): no FMA contraction
#pragma clang fp contract(off)

namespace esm {
namespace {

constexpr int kThreads = 256;
constexpr int kRegChunk = 16;  // cost planes loaded per round trip

__global__ void __launch_bounds__(kThreads) dispreg_kernel(const float* __restrict__ cost, float* __restrict__ out,
                                                           int D, int HW, int npix) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= npix) return;
    const int b = i / HW;
    const int p = i - b * HW;
    const float* c = cost + static_cast<long long>(b) * D * HW + p;
    float acc = 0.f;
    // kRegChunk loads in flight per round trip, then the adds in d order (reference order)
    for (int d0 = 0; d0 < D; d0 += kRegChunk) {
        float v[kRegChunk];
#pragma unroll
        for (int k = 0; k < kRegChunk; ++k) v[k] = d0 + k < D ? c[static_cast<long long>(d0 + k) * HW] : 0.f;
#pragma unroll
        for (int k = 0; k < kRegChunk; ++k)
            if (d0 + k < D) acc = acc + v[k] * static_cast<float>(d0 + k);
    }
    out[i] = acc;
}

// Order of torch.sort(descending=True): NaN ranks above every number; on equal keys the lower
// index stays first (the scan visits d in increasing order and only a strictly earlier key moves).
__device__ __forceinline__ bool desc_before(float v, float w) { return (v != v && w == w) || v > w; }

__global__ void __launch_bounds__(kThreads) topk2_kernel(const float* __restrict__ cost,
                                                         const float* __restrict__ samples, float* __restrict__ out,
                                                         int D, int HW, int npix) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= npix) return;
    const int b = i / HW;
    const int p = i - b * HW;
    const long long base = static_cast<long long>(b) * D * HW + p;
    const float* c = cost + base;
    float v0 = -INFINITY, v1 = -INFINITY;
    int i0 = 0, i1 = 1;
    bool have0 = false, have1 = false;
    for (int d0 = 0; d0 < D; d0 += kRegChunk) {
        float vs[kRegChunk];
#pragma unroll
        for (int k = 0; k < kRegChunk; ++k) vs[k] = d0 + k < D ? c[static_cast<long long>(d0 + k) * HW] : 0.f;
#pragma unroll
        for (int k = 0; k < kRegChunk; ++k) {
            if (d0 + k >= D) break;
            const float v = vs[k];
            const int d = d0 + k;
            if (!have0 || desc_before(v, v0)) {
                if (have0) { v1 = v0; i1 = i0; have1 = true; }
                v0 = v; i0 = d; have0 = true;
            } else if (!have1 || desc_before(v, v1)) {
                v1 = v; i1 = d; have1 = true;
            }
        }
    }
    // softmax over (v0, v1): max is v0
    const float e0 = expf(v0 - v0);
    const float e1 = expf(v1 - v0);
    const float s = e0 + e1;
    const float p0 = e0 / s;
    const float p1 = e1 / s;
    // disparity_samples gathered at the two indices (NULL samples = arange(D), as ESMStereo.py:719-720)
    const float d0 = samples ? samples[base + static_cast<long long>(i0) * HW] : static_cast<float>(i0);
    const float d1 = samples ? samples[base + static_cast<long long>(i1) * HW] : static_cast<float>(i1);
    out[i] = d0 * p0 + d1 * p1;
}

}  // namespace

int launch_regression(int kind, const float* cost, const float* samples, float* out, int B, int D, int H, int W,
                      hipStream_t s) {
    if (!cost || !out) return arg_error("regression: null pointer");
    if (B <= 0 || D <= 0 || H <= 0 || W <= 0) return arg_error("regression: non-positive size");
    const int HW = H * W;
    const int npix = B * HW;
    if (kind == 0) {
        hipLaunchKernelGGL(dispreg_kernel, dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, cost, out, D, HW, npix);
    } else if (kind == 1) {
        if (D < 2) return arg_error("regression_topk: k=2 needs D >= 2");
        hipLaunchKernelGGL(topk2_kernel, dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, cost, samples, out, D, HW,
                           npix);
    } else {
        return arg_error("regression: unknown kind");
    }
    return check_launch("regression");
}

}  // namespace esm

extern "C" {

int esm_disp_regression_f32(const float* cost, float* out, int B, int D, int H, int W, void* stream) {
    return esm::launch_regression(0, cost, nullptr, out, B, D, H, W, esm::as_stream(stream));
}

int esm_topk2_regression_f32(const float* cost, const float* samples, float* out, int B, int D, int H, int W,
                             void* stream) {
    return esm::launch_regression(1, cost, samples, out, B, D, H, W, esm::as_stream(stream));
}

}  // extern "C"
