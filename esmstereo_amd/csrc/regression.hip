// Disparity regressions on the aggregated cost [B, D, H, W] (fp32, HBM-bound, one thread
// per pixel, loads coalesced along W, D walked sequentially).
//
//  disparity_regression  models/submodule.py:211-216: out = sum_d cost[d] * d  (NO softmax;
//                        products rounded, then summed in d order -> bit-exact with the
//                        reference's `torch.sum(x * arange, 1)`)
//  regression_topk       models/submodule.py:218-225: top-k of D (value desc, lowest index
//                        first on ties), softmax over the k costs, sum of sample*prob; k <= 8
//                        as a sorted register list in one pass (k = 2 is the ESMStereo call),
//                        larger k by selection passes.
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

// softmax over the K selected costs (max = the first, torch.softmax's exp(x - max) / sum), then
// the probability-weighted sum of their disparity samples, both sums in rank order
template <int K>
__device__ __forceinline__ float topk_finish(const float (&v)[K], const int (&ix)[K], int n,
                                             const float* __restrict__ samples, long long base, int HW) {
    float e[K];
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < K; ++t) {
        e[t] = t < n ? expf(v[t] - v[0]) : 0.f;
        if (t < n) s = s + e[t];
    }
    float acc = 0.f;
#pragma unroll
    for (int t = 0; t < K; ++t) {
        if (t >= n) break;
        // disparity_samples gathered at the index (NULL samples = arange(D), as ESMStereo.py:719-720)
        const float d = samples ? samples[base + static_cast<long long>(ix[t]) * HW] : static_cast<float>(ix[t]);
        acc = acc + d * (e[t] / s);
    }
    return acc;
}

// regression_topk for K <= 8: a sorted register list, one pass over D (compile-time insertion
// position, no dynamically indexed register array)
template <int K>
__global__ void __launch_bounds__(kThreads) topk_kernel(const float* __restrict__ cost,
                                                        const float* __restrict__ samples, float* __restrict__ out,
                                                        int D, int HW, int npix) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= npix) return;
    const int b = i / HW;
    const int p = i - b * HW;
    const long long base = static_cast<long long>(b) * D * HW + p;
    const float* c = cost + base;
    float v[K];
    int ix[K];
#pragma unroll
    for (int t = 0; t < K; ++t) {
        v[t] = -INFINITY;
        ix[t] = 0;
    }
    int n = 0;
    for (int d0 = 0; d0 < D; d0 += kRegChunk) {
        float vs[kRegChunk];
#pragma unroll
        for (int k = 0; k < kRegChunk; ++k) vs[k] = d0 + k < D ? c[static_cast<long long>(d0 + k) * HW] : 0.f;
#pragma unroll
        for (int k = 0; k < kRegChunk; ++k) {
            if (d0 + k >= D) break;
            const float val = vs[k];
            int pos = 0;  // entries ranked before val (an equal earlier entry keeps its rank)
#pragma unroll
            for (int e = 0; e < K; ++e) pos += (e < n && !desc_before(val, v[e])) ? 1 : 0;
            if (pos < K) {
#pragma unroll
                for (int t = K - 1; t > 0; --t)
                    if (t > pos) {
                        v[t] = v[t - 1];
                        ix[t] = ix[t - 1];
                    }
#pragma unroll
                for (int t = 0; t < K; ++t)
                    if (t == pos) {
                        v[t] = val;
                        ix[t] = d0 + k;
                    }
                n = n < K ? n + 1 : K;
            }
        }
    }
    out[i] = topk_finish<K>(v, ix, n, samples, base, HW);
}

__device__ __forceinline__ bool same_key(float v, float w) { return v == w || (v != v && w != w); }

// regression_topk for any larger k: k selection passes over the column (each finds the next entry
// in (value desc, index asc) order after the previous one), the probabilities' denominator from a
// first round of passes, the weighted sum from a second.  O(k * D) loads per pixel, L2-resident.
__global__ void __launch_bounds__(kThreads) topk_select_kernel(const float* __restrict__ cost,
                                                               const float* __restrict__ samples,
                                                               float* __restrict__ out, int D, int HW, int npix,
                                                               int k) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= npix) return;
    const int b = i / HW;
    const int p = i - b * HW;
    const long long base = static_cast<long long>(b) * D * HW + p;
    const float* c = cost + base;
    float s = 0.f, acc = 0.f, v0 = 0.f;
    for (int round = 0; round < 2; ++round) {
        float pv = 0.f;
        int pi = -1;
        for (int t = 0; t < k; ++t) {
            float bv = 0.f;
            int bi = -1;
            for (int d = 0; d < D; ++d) {
                const float val = c[static_cast<long long>(d) * HW];
                const bool after = pi < 0 || desc_before(pv, val) || (same_key(val, pv) && d > pi);
                if (after && (bi < 0 || desc_before(val, bv))) {
                    bv = val;
                    bi = d;
                }
            }
            pv = bv;
            pi = bi;
            if (t == 0) v0 = bv;
            const float e = expf(bv - v0);
            if (round == 0) {
                s = s + e;
            } else {
                const float dv = samples ? samples[base + static_cast<long long>(bi) * HW] : static_cast<float>(bi);
                acc = acc + dv * (e / s);
            }
        }
    }
    out[i] = acc;
}

template <int K>
void launch_topk_k(const float* cost, const float* samples, float* out, int D, int HW, int npix, hipStream_t s) {
    hipLaunchKernelGGL((topk_kernel<K>), dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, cost, samples, out, D,
                       HW, npix);
}

}  // namespace

// kind 0: disparity_regression; kind 1: regression_topk k = 2 (the ESMStereo call); kind 2 + k:
// regression_topk with k = kind - 2 (k = min(k, D): the reference slices the sorted indices).
int launch_regression(int kind, const float* cost, const float* samples, float* out, int B, int D, int H, int W,
                      hipStream_t s) {
    if (!cost || !out) return arg_error("regression: null pointer");
    if (B <= 0 || D <= 0 || H <= 0 || W <= 0) return arg_error("regression: non-positive size");
    const int HW = H * W;
    const int npix = B * HW;
    if (kind == 0) {
        hipLaunchKernelGGL(dispreg_kernel, dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, cost, out, D, HW, npix);
        return check_launch("regression");
    }
    if (kind < 1) return arg_error("regression: unknown kind");
    int k = kind == 1 ? 2 : kind - 2;
    if (k < 1) return arg_error("regression_topk: k must be >= 1");
    k = k < D ? k : D;
    switch (k) {
        case 1: launch_topk_k<1>(cost, samples, out, D, HW, npix, s); break;
        case 2: launch_topk_k<2>(cost, samples, out, D, HW, npix, s); break;
        case 3: launch_topk_k<3>(cost, samples, out, D, HW, npix, s); break;
        case 4: launch_topk_k<4>(cost, samples, out, D, HW, npix, s); break;
        case 5: launch_topk_k<5>(cost, samples, out, D, HW, npix, s); break;
        case 6: launch_topk_k<6>(cost, samples, out, D, HW, npix, s); break;
        case 7: launch_topk_k<7>(cost, samples, out, D, HW, npix, s); break;
        case 8: launch_topk_k<8>(cost, samples, out, D, HW, npix, s); break;
        default:
            hipLaunchKernelGGL(topk_select_kernel, dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, cost, samples,
                               out, D, HW, npix, k);
    }
    return check_launch("regression_topk");
}

}  // namespace esm

extern "C" {

int esm_disp_regression_f32(const float* cost, float* out, int B, int D, int H, int W, void* stream) {
    return esm::launch_regression(0, cost, nullptr, out, B, D, H, W, esm::as_stream(stream));
}

int esm_topk2_regression_f32(const float* cost, const float* samples, float* out, int B, int D, int H, int W,
                             void* stream) {
    if (D < 2) return esm::arg_error("regression_topk: k=2 needs D >= 2");
    return esm::launch_regression(1, cost, samples, out, B, D, H, W, esm::as_stream(stream));
}

int esm_topk_regression_f32(const float* cost, const float* samples, float* out, int B, int D, int H, int W, int k,
                            void* stream) {
    if (k < 1) return esm::arg_error("regression_topk: k must be >= 1");
    return esm::launch_regression(2 + k, cost, samples, out, B, D, H, W, esm::as_stream(stream));
}

}  // extern "C"
