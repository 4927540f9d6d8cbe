// Shared helpers for the gfx950 kernels of esmstereo_amd.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>

#include "../../include/esmstereo_amd.h"

namespace esm {

void set_error(const std::string& msg);

inline int check_launch(const char* what) {
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        set_error(std::string(what) + ": " + hipGetErrorString(e));
        return ESM_ERR_LAUNCH;
    }
    return ESM_OK;
}

inline int arg_error(const std::string& msg) {
    set_error(msg);
    return ESM_ERR_ARG;
}

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline unsigned ceil_div(long long a, long long b) { return static_cast<unsigned>((a + b - 1) / b); }

// erf(x) with the two minimax polynomials of the device library's erff (|x| < 1: odd polynomial
// in x^2; |x| >= 1: 1 - exp(-p(|x|))), both evaluated and selected instead of branched on.  The
// library form branches per value under an exec mask, so the four values a lane finishes in an
// MFMA epilogue run one after the other as serial dependency chains; branch-free, they interleave
// (profiles/r02_pmc_*: ~2600 VALU per wave and 43 % issue stalls in the pair kernel were mostly erf).
__device__ __forceinline__ float erf_bf(float x) {
    const float ax = fabsf(x);
    const float x2 = x * x;
    float s = fmaf(x2, __int_as_float(0xba1345e1), __int_as_float(0x3ba10414));
    s = fmaf(x2, s, __int_as_float(0xbcdac9b8));
    s = fmaf(x2, s, __int_as_float(0x3de703be));
    s = fmaf(x2, s, __int_as_float(0xbec09330));
    s = fmaf(x2, s, __int_as_float(0x3e0375d0));
    const float rs = fmaf(ax, s, ax);
    float l = fmaf(ax, __int_as_float(0x378e98ab), __int_as_float(0xb9c68948));
    l = fmaf(ax, l, __int_as_float(0x3b7cd369));
    l = fmaf(ax, l, __int_as_float(0xbcc618b2));
    l = fmaf(ax, l, __int_as_float(0x3dda74e4));
    l = fmaf(ax, l, __int_as_float(0x3f228afd));
    l = fmaf(ax, l, __int_as_float(0x3e03c728));
    l = fmaf(ax, l, ax);
    // 1 - exp(-l) with the hardware exp2 (v_exp_f32, 1 ulp) instead of the library expf's range reduction:
    // l >= 0.84 here, so exp(-l) <= 0.43 and its rounding moves erf by < 2^-24 relative (the GELU test's
    // 2.5e-7 |x| bound vs fp64 holds); ~10 fewer instructions per GELU in every BasicConv epilogue
#ifdef ESM_GELU_LIBEXP  // A/B builds: the library expf
    const float rl = 1.0f - expf(-l);
#else
    const float rl = 1.0f - __builtin_amdgcn_exp2f(-l * 1.44269504088896341f);
#endif
    return copysignf(ax < 1.0f ? rs : rl, x);
}

// exact-erf GELU as nn.GELU() (models/submodule.py:37): x * 0.5 * (1 + erf(x / sqrt 2))
__device__ __forceinline__ float gelu_erf(float x) {
    return x * 0.5f * (1.0f + erf_bf(x * 0.70710678118654752440f));
}

// f(integral_constant<int, I>) for I = B .. E-1, unrolled at compile time (ring-buffer indices
// inside runtime loops over ring periods)
template <int B, int E, typename F>
__device__ __forceinline__ void static_for(F&& f) {
    if constexpr (B < E) {
        f(std::integral_constant<int, B>{});
        static_for<B + 1, E>(f);
    }
}

struct Blk3 {
    int x, y, z;
};
// Workgroup coordinates.  The dispatcher deals workgroups (x fastest, then y, z) round-robin over the
// 8 XCDs, so neighbouring tiles, which read each other's halo rows, sit in different XCDs' L2s and
// each fetches the shared lines from memory again.  With `slab` (a per-launch flag: conv hint bit 30,
// esm_shuffle_tail_desc.flags bit 0) the order is remapped bijectively so that XCD k runs a contiguous
// range of logical tiles (a slab of rows) and the halo stays in its own L2.  Measured (round 3, S-K):
// memory-side bytes of the full-resolution launches fall from 2.1-2.9x the algorithmic to 1.05-1.13x
// at no cost in their time, while on the small maps of the hourglasses the slab order costs
// 0.1-1 us per launch (+10 us on the step with every launch remapped), so the host sets the flag for
// 2-D maps of >= 64k output pixels only (engine.XCD_SLAB_MIN_PIX).
constexpr int kHintXcd = 1 << 30;
__device__ __forceinline__ Blk3 xcd_block(bool slab) {
    if (!slab) return {static_cast<int>(blockIdx.x), static_cast<int>(blockIdx.y), static_cast<int>(blockIdx.z)};
    const unsigned gx = gridDim.x, gy = gridDim.y;
    const unsigned nwg = gx * gy * gridDim.z;
    const unsigned orig = blockIdx.x + gx * (blockIdx.y + gy * blockIdx.z);
    const unsigned q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    unsigned wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    const int x = static_cast<int>(wg % gx);
    wg /= gx;
    const int y = static_cast<int>(wg % gy);
    return {x, y, static_cast<int>(wg / gy)};
}

// SiLU as nn.SiLU: x / (1 + exp(-x))
__device__ __forceinline__ float silu(float x) { return x / (1.0f + expf(-x)); }

// SiLU with the hardware exp2 / reciprocal (a few ulp): per-pixel chains where the libm forms'
// division and exp sequences dominate the instruction count (smix, shuffle_tail).  The reciprocal is the
// v_rcp_f32 builtin: __fdividef compiles to the full IEEE division sequence (v_div_scale x2, v_rcp, 4 FMAs,
// v_div_fmas, v_div_fixup) without fast-math, 34 such sequences in the 4x head alone (round 5)
__device__ __forceinline__ float silu_fast(float x) {
#ifdef ESM_SILU_DIV  // A/B builds: the division form
    return __fdividef(x, 1.0f + __expf(-x));
#else
    return x * __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.44269504088896341f));
#endif
}

__device__ __forceinline__ float apply_act(float v, int act) {
    switch (act) {
        case ESM_ACT_GELU: return gelu_erf(v);
        case ESM_ACT_SILU: return silu(v);
        case ESM_ACT_RELU: return v > 0.f ? v : 0.f;
        case ESM_ACT_SIGMOID: return 1.0f / (1.0f + expf(-v));
        case ESM_ACT_RELU6: return fminf(fmaxf(v, 0.f), 6.f);
        default: return v;
    }
}

// Activation fixed at compile time (ACT >= 0: one folded case, no per-value switch in an
// epilogue) or chosen at run time (ACT < 0).
template <int ACT>
__device__ __forceinline__ float act_t(float v, int act) {
    if constexpr (ACT < 0) {
        return apply_act(v, act);
    } else {
        return apply_act(v, ACT);
    }
}

// F.interpolate(mode='bilinear', align_corners=False, scale_factor=f) at output (y, x):
// src = (dst + 0.5) / f - 0.5 clamped at 0; neighbour index clamped at the last row/col.
__device__ __forceinline__ float bilinear_at(const float* __restrict__ img, int H, int W, long long sh, int f, int y,
                                             int x) {
    const float sc = 1.0f / static_cast<float>(f);
    float sy = sc * (static_cast<float>(y) + 0.5f) - 0.5f;
    float sx = sc * (static_cast<float>(x) + 0.5f) - 0.5f;
    sy = sy < 0.f ? 0.f : sy;
    sx = sx < 0.f ? 0.f : sx;
    const int y0 = static_cast<int>(sy);
    const int x0 = static_cast<int>(sx);
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0);
    const int x1 = x0 + (x0 < W - 1 ? 1 : 0);
    const float ly1 = sy - static_cast<float>(y0), ly0 = 1.0f - ly1;
    const float lx1 = sx - static_cast<float>(x0), lx0 = 1.0f - lx1;
    const float a = img[y0 * sh + x0], b = img[y0 * sh + x1];
    const float c = img[y1 * sh + x0], d = img[y1 * sh + x1];
    return ly0 * (lx0 * a + lx1 * b) + ly1 * (lx0 * c + lx1 * d);
}

}  // namespace esm
