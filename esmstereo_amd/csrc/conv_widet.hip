// Register-resident-weight ConvTranspose2d(k=4, s=2, p=1): the decoder steps of the refinement
// hourglass (conv3_up / conv2_up of up_refinement, models/ESMStereo.py:210-212 (185-239); BasicConv
// deconv, models/submodule.py:12-38).  ESMStereo-S's ref4x.conv2_up (16 -> 16, 96x312 -> 192x624)
// is the third-largest launch of the S-K step.
//
// Output (2y + qh, 2x + qw) = sum_{th, tw in {0, 1}} sum_c W[(qh, qw)][(th, tw)][c] X[c][y + qh - th][x + qw - tw]
// (the per-parity-class form of conv_impl.h).  A wave owns a 16-column strip of the input grid and
// R input-grid rows, and computes all four parity classes, i.e. a 32-column x 2R-row output tile:
//   * every class's 4 taps x NG channel groups of weights live in VGPRs (16 * NG registers);
//   * input row yi at column shift s in {-1, 0, 1} is ONE buffer_load per group and feeds every
//     (class, tap) that reads it: s = -1 -> (qw 0, tw 1); s = 0 -> (0, 0), (1, 1); s = 1 -> (1, 0), for
//     both qh and both th (output rows yi - qh + th inside the block): 16 MFMAs per group per row;
//   * the two column classes of an output row sit in the same lanes and registers, so the epilogue
//     stores (2x, 2x + 1) as one 8-byte store per lane: 128 contiguous bytes per 16 lanes.
#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

constexpr int kWtThreads = 256;

template <int NG, int MT, int R, int ACT, bool PLAIN>
__global__ void __launch_bounds__(kWtThreads) wtconv_kernel(const esm_conv_desc a) {
    constexpr int NR = R + 2;  // input rows y0 - 1 .. y0 + R
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15, kq = lane >> 4;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int x0 = (bk_.x * 4 + wave) * 16;  // input-grid column of lane 0
    const int y0 = bk_.y * R;
    const int b = bk_.z;

    // ---- weights -> VGPRs: packed w[cls][tap][cin_pad][cout_pad], cls = qh*2 + qw, tap = th*2 + tw
    float wv[4][4][NG][MT];
    {
        const int wcls = 4 * a.cin_pad * a.cout_pad;
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.w), static_cast<short>(0), 4 * 4 * wcls, 0x00020000);
        const unsigned wl = 4u * (kq * a.cout_pad + n16);
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int g = 0; g < NG; ++g)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
                        wv[c][t][g][mt] = buf_load_s(wrs, wl, 4 * (c * wcls + (t * a.cin_pad + 4 * g) * a.cout_pad + 16 * mt));
    }
    float scl[MT][4], shf[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = min(16 * mt + 4 * kq + j, a.Cout - 1);
            scl[mt][j] = a.scale ? a.scale[co] : 1.f;
            shf[mt][j] = a.shift ? a.shift[co] : 0.f;
        }

    // ---- input addressing (one source): lane column x0 + n16 + s
    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0), 4 * ((s0.C - 1) * sc + (a.Hi - 1) * sh + a.Wi),
        0x00020000);
    const int xs = x0 + n16;
    unsigned vo[NG][3];
#pragma unroll
    for (int g = 0; g < NG; ++g) {
        const int c = 4 * g + kq;
#pragma unroll
        for (int s = 0; s < 3; ++s) {
            const int xi = xs + s - 1;
            vo[g][s] = (c < a.Cin && xs < a.Wi && xi >= 0 && xi < a.Wi) ? 4u * (c * sc + xi) : kOOB;
        }
    }
    auto load_row = [&](float (&d)[NG][3], int r) {  // input row y0 - 1 + r
        const int yi = y0 - 1 + r;
        const int roff = (yi >= 0 && yi < a.Hi) ? 4 * yi * sh : static_cast<int>(kOOB);
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int s = 0; s < 3; ++s) d[g][s] = buf_load_s(rs, vo[g][s], roff);
    };

    floatx4 acc[R][2][2][MT];  // [sub-grid row][qh][qw][mt]
#pragma unroll
    for (int y = 0; y < R; ++y)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
            for (int qw = 0; qw < 2; ++qw)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) acc[y][qh][qw][mt] = floatx4{0.f, 0.f, 0.f, 0.f};

    // output through a descriptor over this batch item; lane (kq, n16) stores (2x, 2x + 1) of cout row j
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo), 0x00020000);
    unsigned ovo[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 16 * mt + 4 * kq + j;
            ovo[mt][j] = (co < a.Cout && xs < a.Wi) ? 4u * (co * static_cast<int>(a.oc) + 2 * xs) : kOOB;
        }
    auto finish = [&](int y) {  // sub-grid row y0 + y: output rows 2(y0 + y) + qh
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
            const int oy = 2 * (y0 + y) + qh;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    float v2[2];
#pragma unroll
                    for (int qw = 0; qw < 2; ++qw) {
                        float v = acc[y][qh][qw][mt][j];
                        v = a.scale ? v * scl[mt][j] + shf[mt][j] : v + shf[mt][j];
                        v2[qw] = act_t<ACT>(v, a.act);
                    }
                    if constexpr (PLAIN) {
                        const int orow = oy < a.Ho ? 4 * oy * static_cast<int>(a.oh) : static_cast<int>(kOOB);
                        typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
                        const u32x2 pk2 = {__float_as_uint(v2[0]), __float_as_uint(v2[1])};
                        __builtin_amdgcn_raw_buffer_store_b64(pk2, ro_, static_cast<int>(ovo[mt][j]), orow, kStoreAux);
                    } else {
                        const int co = 16 * mt + 4 * kq + j;
                        if (co >= a.Cout || xs >= a.Wi || oy >= a.Ho) continue;
#pragma unroll
                        for (int qw = 0; qw < 2; ++qw) {
                            float v = v2[qw];
                            const int ox = 2 * xs + qw;
                            if (a.res) v = v + a.res[b * a.rb + co * a.rc + static_cast<long long>(oy) * a.rh + ox];
                            const long long o = b * a.ob + co * a.oc + static_cast<long long>(oy) * a.oh + ox;
                            a.out[o] = v * a.post_scale;
                            if (a.out2) a.out2[o] = v * a.post_scale2;
                        }
                    }
                }
        }
    };

    float bin[2][NG][3];
    load_row(bin[0], 0);
#pragma unroll
    for (int r = 0; r < NR; ++r) {  // input row yi = y0 - 1 + r feeds sub-grid rows y = r - 1 - qh + th
        if (r + 1 < NR) load_row(bin[(r + 1) & 1], r + 1);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < NG; ++g)
#pragma unroll
            for (int s = 0; s < 3; ++s)
#pragma unroll
                for (int tw = 0; tw < 2; ++tw) {
                    const int qw = s - 1 + tw;  // column class reading shift s - 1 through tap tw
                    if (qw < 0 || qw > 1) continue;
#pragma unroll
                    for (int qh = 0; qh < 2; ++qh)
#pragma unroll
                        for (int th = 0; th < 2; ++th) {
                            const int y = r - 1 - qh + th;
                            if (y < 0 || y >= R) continue;
#pragma unroll
                            for (int mt = 0; mt < MT; ++mt)
                                acc[y][qh][qw][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    wv[qh * 2 + qw][th * 2 + tw][g][mt], bin[r & 1][g][s], acc[y][qh][qw][mt], 0, 0, 0);
                        }
                }
        // sub-grid row r - 2 has all its input rows (its last is yi = y + 1)
        if (r - 2 >= 0) finish(r - 2);
    }
}

template <int NG, int MT>
int launch_widet_g(const esm_conv_desc& a, hipStream_t s) {
    const long long units = static_cast<long long>(a.B) * a.Hi * ceil_div(a.Wi, 16);
    // sub-grid rows per wave: keep ~2 waves per SIMD; hint bits 26-27 = 1 / 2 force R = 1 / 2 (tuning)
    const int rsel = (a.hint >> 26) & 3;
    const int R = rsel == 1 ? 1 : (rsel == 2 ? 2 : (units >= 8192 ? 2 : 1));
    const dim3 grid(ceil_div(a.Wi, 64), ceil_div(a.Hi, R), static_cast<unsigned>(a.B));
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("conv(wide-T): grid too large");
    const bool plain = a.act == ESM_ACT_GELU && !a.res && !a.out2 && a.post_scale == 1.f &&
                       static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (R == 2) {
        if (plain) hipLaunchKernelGGL((wtconv_kernel<NG, MT, 2, ESM_ACT_GELU, true>), grid, dim3(kWtThreads), 0, s, a);
        else hipLaunchKernelGGL((wtconv_kernel<NG, MT, 2, -1, false>), grid, dim3(kWtThreads), 0, s, a);
    } else {
        if (plain) hipLaunchKernelGGL((wtconv_kernel<NG, MT, 1, ESM_ACT_GELU, true>), grid, dim3(kWtThreads), 0, s, a);
        else hipLaunchKernelGGL((wtconv_kernel<NG, MT, 1, -1, false>), grid, dim3(kWtThreads), 0, s, a);
    }
    return check_launch("conv(wide-T)");
}

}  // namespace

// 2-D ConvTranspose k4 s2 p1 with one source, Cout <= 32 and weights that fit the register budget
// (16 * channel groups * cout tiles <= 64).
bool widet_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (d3 || !a.transposed || a.kh != 4 || a.stride != 2 || a.nsrc != 1 || a.mul || a.up || a.shuffle > 1) return false;
    const int ng = (a.Cin + 3) / 4, mt = a.Cout > 16 ? 2 : 1;
    return a.Cout <= 32 && ng * mt <= 4 && direct_ok(a);
}

int launch_widet(const esm_conv_desc& a, hipStream_t s) {
    if (!widet_ok(a)) return arg_error("conv: wide-T hint not applicable");
    const int ng = (a.Cin + 3) / 4;
    if (a.Cout > 16) return ng <= 1 ? launch_widet_g<1, 2>(a, s) : launch_widet_g<2, 2>(a, s);
    if (ng <= 1) return launch_widet_g<1, 1>(a, s);
    if (ng <= 2) return launch_widet_g<2, 1>(a, s);
    return launch_widet_g<4, 1>(a, s);
}

}  // namespace conv
}  // namespace esm
