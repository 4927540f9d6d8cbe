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

template <int CPG, bool ATT, bool VEC, int DCH = kDChunk>
__global__ void __launch_bounds__(kThreads) gwc_kernel(const float* __restrict__ L, const float* __restrict__ R,
                                                       const float* __restrict__ att, float* __restrict__ V, int G,
                                                       int H, int W, int D) {
    __shared__ float rs[CPG][kTile + DCH];
    const int HW = H * W;
    const int bg = blockIdx.y;  // b*G + g
    const int b = bg / G;
    const int g = bg - b * G;
    const int p0 = blockIdx.x * kTile;
    const int d0 = blockIdx.z * DCH;
    const int dn = min(DCH, D - d0);
    const int C = G * CPG;
    const float* lb = L + (static_cast<long long>(b) * C + g * CPG) * HW;
    const float* rb = R + (static_cast<long long>(b) * C + g * CPG) * HW;
    // stage right pixels [p0 - (d0+dn-1), p0 + kTile - d0) for this group's channels
    const int lo = p0 - (d0 + dn - 1);
    const int span = kTile + dn - 1;
    // every load of the thread (right segment, left pixels, att) issued as one batch with clamped
    // addresses, then selected and stored: one memory round trip per workgroup
    constexpr int NR = (kTile + DCH - 1 + kThreads - 1) / kThreads;
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
            // write-through (sc1) 16-B stores: no dirty volume lines left for the kernel-boundary
            // write-back (conv_direct.h kStoreAux; -0.7 us on the S-K step with the two below)
            typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
            const __amdgpu_buffer_rsrc_t rv = __builtin_amdgcn_make_buffer_rsrc(vb, static_cast<short>(0), 0x7fffffff,
                                                                                0x00020000);
            __builtin_amdgcn_raw_buffer_store_b128(
                u32x4{__float_as_uint(o[0]), __float_as_uint(o[1]), __float_as_uint(o[2]), __float_as_uint(o[3])}, rv,
                static_cast<int>(4 * (static_cast<long long>(dd) * HW + pt)), 0, 16);
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

// Norm-correlation in one launch.  A workgroup owns one row segment [x0, x0+kNcW) of (b, y)
// and a chunk of kNcD disparities.  It stages the left segment and the right segment
// [x0-d0-kNcD+1, x0+kNcW-d0) of all C channels in LDS (every load of the tile in flight at
// once), computes each staged pixel's L2 norm over C (hoisted out of the d loop: the reference
// recomputes it per d), normalises in place, and writes kNcD planes of the row segment.
// The norm is summed in channel order and the eps is added after the sqrt, as
// torch.norm(., 2, 1) + 1e-5 (submodule.py:188-189); the mean is sum_c / C (submodule.py:190).
constexpr int kNcW = 64;   // output pixels per workgroup (one per lane of a wave)
constexpr int kNcD = 16;   // disparities per workgroup (ESMStereo's D is 12-64: little idle work)
constexpr int kNcSpan = kNcW + kNcD - 1;

template <int CT>  // CT: channel capacity of the LDS tile (C <= CT)
__global__ void __launch_bounds__(kThreads) normcorr_kernel(const float* __restrict__ L, const float* __restrict__ R,
                                                            float* __restrict__ V, int C, int H, int W, int D) {
    __shared__ float ls[CT][kNcW + 1];
    __shared__ float rs[CT][kNcSpan + 1];
    const int x0 = blockIdx.x * kNcW;
    const int y = blockIdx.y % H;
    const int b = blockIdx.y / H;
    const int d0 = blockIdx.z * kNcD;
    const int r0 = x0 - d0 - (kNcD - 1);  // right x of rs[.][0]
    const long long HW = static_cast<long long>(H) * W;
    const float* lrow = L + static_cast<long long>(b) * C * HW + static_cast<long long>(y) * W;
    const float* rrow = R + static_cast<long long>(b) * C * HW + static_cast<long long>(y) * W;
    const int t = threadIdx.x;

    // stage: all loads of the tile issued before the first LDS store
    constexpr int NL = (CT * kNcW + kThreads - 1) / kThreads;
    constexpr int NR = (CT * kNcSpan + kThreads - 1) / kThreads;
    float lv[NL], rv[NR];
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int i = t + k * kThreads;
        const int c = i / kNcW, j = i - c * kNcW, x = x0 + j;
        lv[k] = (i < C * kNcW && x < W) ? lrow[c * HW + x] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const int i = t + k * kThreads;
        const int c = i / kNcSpan, j = i - c * kNcSpan, x = r0 + j;
        rv[k] = (i < C * kNcSpan && x >= 0 && x < W) ? rrow[c * HW + x] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < NL; ++k) {
        const int i = t + k * kThreads;
        if (i < C * kNcW) ls[i / kNcW][i % kNcW] = lv[k];
    }
#pragma unroll
    for (int k = 0; k < NR; ++k) {
        const int i = t + k * kThreads;
        if (i < C * kNcSpan) rs[i / kNcSpan][i % kNcSpan] = rv[k];
    }
    __syncthreads();
    // per-pixel norms (one staged pixel per thread), then normalise in place
    float n = 1.f;
    if (t < kNcW + kNcSpan) {
        float ss = 0.f;
        if (t < kNcW) {
#pragma unroll 8
            for (int c = 0; c < C; ++c) ss = ss + ls[c][t] * ls[c][t];
        } else {
#pragma unroll 8
            for (int c = 0; c < C; ++c) ss = ss + rs[c][t - kNcW] * rs[c][t - kNcW];
        }
        n = sqrtf(ss) + 1e-05f;
    }
    __syncthreads();
    if (t < kNcW) {
#pragma unroll 8
        for (int c = 0; c < C; ++c) ls[c][t] = ls[c][t] / n;
    } else if (t < kNcW + kNcSpan) {
#pragma unroll 8
        for (int c = 0; c < C; ++c) rs[c][t - kNcW] = rs[c][t - kNcW] / n;
    }
    __syncthreads();
    // correlation: lane = pixel, wave w takes disparities d0 + w, d0 + w + 4, ...
    const int j = t & (kNcW - 1);
    const int x = x0 + j;
    const int w = t / kNcW;
    constexpr int PER = kNcD / (kThreads / kNcW);
    float acc[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) acc[k] = 0.f;
#pragma unroll 4
    for (int c = 0; c < C; ++c) {
        const float l = ls[c][j];
#pragma unroll
        for (int k = 0; k < PER; ++k) {
            const int dd = w + 4 * k;  // x - (d0 + dd) - r0 = j + kNcD - 1 - dd
            acc[k] = acc[k] + l * rs[c][j + kNcD - 1 - dd];
        }
    }
    if (x >= W) return;
    float* vrow = V + static_cast<long long>(b) * D * HW + static_cast<long long>(y) * W + x;
    const float invC = 1.0f / static_cast<float>(C);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const int d = d0 + w + 4 * k;
        if (d < D) vrow[d * HW] = x >= d ? acc[k] * invC : 0.f;
    }
}

}  // namespace

int launch_gwc(const float* L, const float* R, const float* att, float* V, int B, int C, int H, int W, int D, int G,
               hipStream_t s) {
    if (!L || !R || !V) return arg_error("gwc: null pointer");
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || D <= 0 || G <= 0) return arg_error("gwc: non-positive size");
    if (C % G) return arg_error("gwc: C must be divisible by num_groups");
    const int cpg = C / G;
    const int HW = H * W;
    // small volumes (the S variant at 1/16 resolution: 2 pixel tiles x 32 groups) get 4-plane
    // disparity chunks, i.e. 4x the workgroups; the values are the same (per-voxel arithmetic)
    const bool small = static_cast<long long>(ceil_div(HW, kTile)) * B * G * ceil_div(D, kDChunk) < 512;
    const int dch = small ? 4 : kDChunk;
    dim3 grid(ceil_div(HW, kTile), B * G, ceil_div(D, dch));
    const bool vec = (HW % 4) == 0;
#define ESM_GWC_L(CP, AT, VC)                                                                                      \
    if (small) hipLaunchKernelGGL((gwc_kernel<CP, AT, VC, 4>), grid, dim3(kThreads), 0, s, L, R, att, V, G, H, W, D); \
    else hipLaunchKernelGGL((gwc_kernel<CP, AT, VC>), grid, dim3(kThreads), 0, s, L, R, att, V, G, H, W, D);
#define ESM_GWC(CP)                                                                                          \
    if (cpg == CP) {                                                                                         \
        if (att) {                                                                                           \
            if (vec) { ESM_GWC_L(CP, true, true) } else { ESM_GWC_L(CP, true, false) }                      \
        } else {                                                                                             \
            if (vec) { ESM_GWC_L(CP, false, true) } else { ESM_GWC_L(CP, false, false) }                     \
        }                                                                                                    \
        return check_launch("gwc");                                                                          \
    }
    ESM_GWC(1)
    ESM_GWC(2)
    ESM_GWC(4)
    ESM_GWC(8)
#undef ESM_GWC
#undef ESM_GWC_L
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
    (void)work;  // kept in the ABI; the fused kernel normalises in LDS
    if (!L || !R || !V) return arg_error("normcorr: null pointer");
    if (B <= 0 || C <= 0 || H <= 0 || W <= 0 || D <= 0) return arg_error("normcorr: non-positive size");
    dim3 grid(ceil_div(W, kNcW), B * H, ceil_div(D, kNcD));
    if (C <= 16)
        hipLaunchKernelGGL(normcorr_kernel<16>, grid, dim3(kThreads), 0, s, L, R, V, C, H, W, D);
    else if (C <= 64)
        hipLaunchKernelGGL(normcorr_kernel<64>, grid, dim3(kThreads), 0, s, L, R, V, C, H, W, D);
    else {
        set_error("normcorr: C must be <= 64");
        return ESM_ERR_UNSUPPORTED;
    }
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
