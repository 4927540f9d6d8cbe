// Cost-volume construction for gfx950 (HBM write-bound kernels).
//
//  gwc      models/submodule.py:143-161  V[b,g,d,y,x] = mean_{c in g} L[c,y,x]*R[c,y,x-d], 0 for x<d
//           (+ `volume * att` of models/ESMStereo.py:711 fused as an epilogue)
//  concat   models/submodule.py:129-140  V[b,c<C,d] = L (all x), V[b,C+c,d,y,x] = R[c,y,x-d] (x>=d)
//  normcorr models/submodule.py:187-200  V[b,0,d] = mean_c (L/(|L|+1e-5)) * (R/(|R|+1e-5))(x-d)
//
// Layout: NCHW in, [B,G,D,H,W] out, fp32.  Each output plane (b,g,d) is H*W contiguous
// floats, and for a pixel p = y*W + x the shifted right pixel is p-d in the SAME flattened
// plane (x >= d keeps it in row y).  So a workgroup owns a flat pixel tile [p0, p0+1024) of
// one (b,g): it keeps its left values in registers, stages the right segment
// [p0-D+1, p0+1024) once in LDS, and streams D planes of float4 stores (one 1 KiB
// coalesced store per wave-instruction).  Products and the pairwise mean are rounded one
// operation at a time (FMA contraction off for this file), so the gwc/concat results are
// bit-exact with the reference's `(a*b).mean()`.
#include "common.h"

// The reference rounds every product and every sum separately; never fuse them into FMAs.
#pragma clang fp contract(off)

namespace esm {
namespace {

constexpr int kThreads = 256;
constexpr int kPix = 4;                       // pixels per thread
constexpr int kTile = kThreads * kPix;         // flat pixels per workgroup
constexpr int kDChunk = 16;                    // disparity planes per workgroup

template <int CPG, bool ATT, bool VEC>
__global__ void __launch_bounds__(kThreads) gwc_kernel(const float* __restrict__ L, const float* __restrict__ R,
                                                       const float* __restrict__ att, float* __restrict__ V, int G,
                                                       int H, int W, int D) {
    __shared__ float rs[CPG][kTile + kDChunk];
    const int HW = H * W;
    const int bg = blockIdx.y;  // b*G + g
    const int b = bg / G;
    const int g = bg - b * G;
    const int p0 = blockIdx.x * kTile;
    const int d0 = blockIdx.z * kDChunk;
    const int dn = min(kDChunk, D - d0);
    const int C = G * CPG;
    const float* lb = L + (static_cast<long long>(b) * C + g * CPG) * HW;
    const float* rb = R + (static_cast<long long>(b) * C + g * CPG) * HW;
    // stage right pixels [p0 - (d0+dn-1), p0 + kTile - d0) for this group's channels
    const int lo = p0 - (d0 + dn - 1);
    const int span = kTile + dn - 1;
    // every load of the thread (right segment, left pixels, att) issued as one batch with clamped
    // addresses, then selected and stored: one memory round trip per workgroup
    constexpr int NR = (kTile + kDChunk - 1 + kThreads - 1) / kThreads;
    float rr[CPG][NR];
#pragma unroll
    for (int c = 0; c < CPG; ++c)
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            const int i = threadIdx.x + k * kThreads;
            const int p = lo + i;
            const bool ok = i < span && p >= 0 && p < HW;
            const float v = rb[static_cast<long long>(c) * HW + (ok ? p : 0)];
            rr[c][k] = ok ? v : 0.f;
        }
    const int pt = p0 + threadIdx.x * kPix;
    float lv[CPG][kPix];
    float av[kPix];
    int xs[kPix];
#pragma unroll
    for (int k = 0; k < kPix; ++k) {
        const int p = pt + k;
        const bool in = p < HW;
        xs[k] = in ? p % W : -1;
#pragma unroll
        for (int c = 0; c < CPG; ++c) {
            const float v = lb[static_cast<long long>(c) * HW + (in ? p : 0)];
            lv[c][k] = in ? v : 0.f;
        }
        if (ATT) {
            const float v = att[static_cast<long long>(bg) * HW + (in ? p : 0)];
            av[k] = in ? v : 1.f;
        } else {
            av[k] = 1.f;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int c = 0; c < CPG; ++c)
#pragma unroll
        for (int k = 0; k < NR; ++k) {
            const int i = threadIdx.x + k * kThreads;
            if (i < span) rs[c][i] = rr[c][k];
        }
    __syncthreads();
    float* vb = V + (static_cast<long long>(bg) * D + d0) * HW;
    const float inv = 1.0f / static_cast<float>(CPG);
    for (int dd = 0; dd < dn; ++dd) {
        const int d = d0 + dd;
        float o[kPix];
#pragma unroll
        for (int k = 0; k < kPix; ++k) {
            const int li = (pt + k - d) - lo;
            float s = lv[0][k] * rs[0][li];
#pragma unroll
            for (int c = 1; c < CPG; ++c) s = s + lv[c][k] * rs[c][li];
            float v = s * inv;
            if (ATT) v = v * av[k];
            o[k] = (xs[k] >= d) ? v : 0.f;
        }
        float* dst = vb + static_cast<long long>(dd) * HW;
        if (VEC && pt + kPix <= HW) {
            *reinterpret_cast<float4*>(dst + pt) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int k = 0; k < kPix; ++k)
                if (pt + k < HW) dst[pt + k] = o[k];
        }
    }
}

template <bool VEC>
__global__ void __launch_bounds__(kThreads) concat_kernel(const float* __restrict__ L, const float* __restrict__ R,
                                                          float* __restrict__ V, int C, int H, int W, int D) {
    __shared__ float rs[kTile + kDChunk];
    const int HW = H * W;
    const int bc = blockIdx.y;  // b*2C + c2
    const int b = bc / (2 * C);
    const int c2 = bc - b * 2 * C;
    const int p0 = blockIdx.x * kTile;
    const int d0 = blockIdx.z * kDChunk;
    const int dn = min(kDChunk, D - d0);
    const int pt = p0 + threadIdx.x * kPix;
    float* vb = V + (static_cast<long long>(bc) * D + d0) * HW;
    if (c2 < C) {  // left half: the same plane for every d (block-uniform branch)
        const float* lb = L + (static_cast<long long>(b) * C + c2) * HW;
        float o[kPix];
#pragma unroll
        for (int k = 0; k < kPix; ++k) o[k] = (pt + k < HW) ? lb[pt + k] : 0.f;
        for (int dd = 0; dd < dn; ++dd) {
            float* dst = vb + static_cast<long long>(dd) * HW;
            if (VEC && pt + kPix <= HW) {
                *reinterpret_cast<float4*>(dst + pt) = make_float4(o[0], o[1], o[2], o[3]);
            } else {
#pragma unroll
                for (int k = 0; k < kPix; ++k)
                    if (pt + k < HW) dst[pt + k] = o[k];
            }
        }
        return;
    }
    const float* rb = R + (static_cast<long long>(b) * C + (c2 - C)) * HW;
    const int lo = p0 - (d0 + dn - 1);
    const int span = kTile + dn - 1;
    for (int i = threadIdx.x; i < span; i += kThreads) {
        const int p = lo + i;
        rs[i] = (p >= 0 && p < HW) ? rb[p] : 0.f;
    }
    int xs[kPix];
#pragma unroll
    for (int k = 0; k < kPix; ++k) xs[k] = (pt + k < HW) ? (pt + k) % W : -1;
    __syncthreads();
    for (int dd = 0; dd < dn; ++dd) {
        const int d = d0 + dd;
        float o[kPix];
#pragma unroll
        for (int k = 0; k < kPix; ++k) o[k] = (xs[k] >= d) ? rs[pt + k - d - lo] : 0.f;
        float* dst = vb + static_cast<long long>(dd) * HW;
        if (VEC && pt + kPix <= HW) {
            *reinterpret_cast<float4*>(dst + pt) = make_float4(o[0], o[1], o[2], o[3]);
        } else {
#pragma unroll
            for (int k = 0; k < kPix; ++k)
                if (pt + k < HW) dst[pt + k] = o[k];
        }
    }
}

// Per-pixel L2 normalisation over channels: out[c] = x[c] / (sqrt(sum x^2) + 1e-5).
__global__ void __launch_bounds__(kThreads) l2norm_kernel(const float* __restrict__ X, float* __restrict__ Y, int C,
                                                          int HW, int npix) {
    const int i = blockIdx.x * kThreads + threadIdx.x;
    if (i >= npix) return;
    const int b = i / HW;
    const int p = i - b * HW;
    const float* xb = X + static_cast<long long>(b) * C * HW + p;
    float* yb = Y + static_cast<long long>(b) * C * HW + p;
    float ss = 0.f;
    for (int c = 0; c < C; ++c) {
        const float v = xb[static_cast<long long>(c) * HW];
        ss = ss + v * v;
    }
    const float n = sqrtf(ss) + 1e-05f;
    for (int c = 0; c < C; ++c) yb[static_cast<long long>(c) * HW] = xb[static_cast<long long>(c) * HW] / n;
}

// Correlation of normalised features: one thread per pixel, kNcD disparities in registers,
// right rows staged in LDS in channel chunks of 16.
constexpr int kNcPix = 256;
constexpr int kNcD = 16;
constexpr int kNcC = 16;

__global__ void __launch_bounds__(kThreads) normcorr_kernel(const float* __restrict__ Ln, const float* __restrict__ Rn,
                                                            float* __restrict__ V, int C, int H, int W, int D) {
    __shared__ float rs[kNcC][kNcPix + kNcD];
    const int HW = H * W;
    const int b = blockIdx.y;
    const int p0 = blockIdx.x * kNcPix;
    const int d0 = blockIdx.z * kNcD;
    const int dn = min(kNcD, D - d0);
    const int p = p0 + threadIdx.x;
    const bool in = p < HW;
    const int x = in ? p % W : -1;
    const int lo = p0 - (d0 + dn - 1);
    const int span = kNcPix + dn - 1;
    float acc[kNcD];
#pragma unroll
    for (int k = 0; k < kNcD; ++k) acc[k] = 0.f;
    const float* lb = Ln + static_cast<long long>(b) * C * HW;
    const float* rb = Rn + static_cast<long long>(b) * C * HW;
    for (int c0 = 0; c0 < C; c0 += kNcC) {
        const int cn = min(kNcC, C - c0);
        __syncthreads();
        for (int i = threadIdx.x; i < cn * span; i += kThreads) {
            const int cc = i / span;
            const int j = i - cc * span;
            const int q = lo + j;
            rs[cc][j] = (q >= 0 && q < HW) ? rb[static_cast<long long>(c0 + cc) * HW + q] : 0.f;
        }
        __syncthreads();
        for (int cc = 0; cc < cn; ++cc) {
            const float lv = in ? lb[static_cast<long long>(c0 + cc) * HW + p] : 0.f;
#pragma unroll
            for (int k = 0; k < kNcD; ++k) {
                if (k < dn) {
                    const int d = d0 + k;
                    const int j = p - d - lo;
                    acc[k] = acc[k] + lv * rs[cc][j];
                }
            }
        }
    }
    if (!in) return;
    float* vb = V + (static_cast<long long>(b) * D + d0) * HW + p;
    const float invC = 1.0f / static_cast<float>(C);
#pragma unroll
    for (int k = 0; k < kNcD; ++k)
        if (k < dn) vb[static_cast<long long>(k) * HW] = (x >= d0 + k) ? acc[k] * invC : 0.f;
}

}  // namespace

int launch_gwc(const float* L, const float* R, const float* att, float* V, int B, int C, int H, int W, int D, int G,
               hipStream_t s) {
    if (!L || !R || !V) return arg_error("gwc: null pointer");
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || D <= 0 || G <= 0) return arg_error("gwc: non-positive size");
    if (C % G) return arg_error("gwc: C must be divisible by num_groups");
    const int cpg = C / G;
    const int HW = H * W;
    dim3 grid(ceil_div(HW, kTile), B * G, ceil_div(D, kDChunk));
    const bool vec = (HW % 4) == 0;
#define ESM_GWC(CP)                                                                                          \
    if (cpg == CP) {                                                                                         \
        if (att) {                                                                                           \
            if (vec) hipLaunchKernelGGL((gwc_kernel<CP, true, true>), grid, dim3(kThreads), 0, s, L, R, att, V, G, H, W, D); \
            else hipLaunchKernelGGL((gwc_kernel<CP, true, false>), grid, dim3(kThreads), 0, s, L, R, att, V, G, H, W, D); \
        } else {                                                                                             \
            if (vec) hipLaunchKernelGGL((gwc_kernel<CP, false, true>), grid, dim3(kThreads), 0, s, L, R, att, V, G, H, W, D); \
            else hipLaunchKernelGGL((gwc_kernel<CP, false, false>), grid, dim3(kThreads), 0, s, L, R, att, V, G, H, W, D); \
        }                                                                                                    \
        return check_launch("gwc");                                                                          \
    }
    ESM_GWC(1)
    ESM_GWC(2)
    ESM_GWC(4)
    ESM_GWC(8)
#undef ESM_GWC
    set_error("gwc: channels per group must be 1, 2, 4 or 8");
    return ESM_ERR_UNSUPPORTED;
}

int launch_concat(const float* L, const float* R, float* V, int B, int C, int H, int W, int D, hipStream_t s) {
    if (!L || !R || !V) return arg_error("concat: null pointer");
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || D <= 0) return arg_error("concat: non-positive size");
    const int HW = H * W;
    dim3 grid(ceil_div(HW, kTile), B * 2 * C, ceil_div(D, kDChunk));
    if (HW % 4 == 0)
        hipLaunchKernelGGL((concat_kernel<true>), grid, dim3(kThreads), 0, s, L, R, V, C, H, W, D);
    else
        hipLaunchKernelGGL((concat_kernel<false>), grid, dim3(kThreads), 0, s, L, R, V, C, H, W, D);
    return check_launch("concat");
}

int launch_normcorr(const float* L, const float* R, float* V, float* work, int B, int C, int H, int W, int D,
                    hipStream_t s) {
    if (!L || !R || !V || !work) return arg_error("normcorr: null pointer");
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || D <= 0) return arg_error("normcorr: non-positive size");
    const int HW = H * W;
    const int npix = B * HW;
    float* Ln = work;
    float* Rn = work + static_cast<long long>(B) * C * HW;
    hipLaunchKernelGGL(l2norm_kernel, dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, L, Ln, C, HW, npix);
    hipLaunchKernelGGL(l2norm_kernel, dim3(ceil_div(npix, kThreads)), dim3(kThreads), 0, s, R, Rn, C, HW, npix);
    dim3 grid(ceil_div(HW, kNcPix), B, ceil_div(D, kNcD));
    hipLaunchKernelGGL(normcorr_kernel, grid, dim3(kThreads), 0, s, Ln, Rn, V, C, H, W, D);
    return check_launch("normcorr");
}

}  // namespace esm

extern "C" {

int esm_gwc_volume_f32(const float* L, const float* R, const float* att, float* V, int B, int C, int H, int W, int D,
                       int G, void* stream) {
    return esm::launch_gwc(L, R, att, V, B, C, H, W, D, G, esm::as_stream(stream));
}

int esm_concat_volume_f32(const float* L, const float* R, float* V, int B, int C, int H, int W, int D, void* stream) {
    return esm::launch_concat(L, R, V, B, C, H, W, D, esm::as_stream(stream));
}

int esm_normcorr_volume_f32(const float* L, const float* R, float* V, float* work, int B, int C, int H, int W, int D,
                            void* stream) {
    return esm::launch_normcorr(L, R, V, work, B, C, H, W, D, esm::as_stream(stream));
}

}  // extern "C"
