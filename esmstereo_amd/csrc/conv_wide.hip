// Register-resident-weight row-streaming convolution for the full-resolution 2-D layers of the ESM
// upsampler (models/ESMStereo.py:242-509: dmNx, spx_Nx, the refinement hourglass' conv1.1 / agg
// layers at 96x312 .. 192x624 for ESMStereo-S at KITTI): BasicConv (models/submodule.py:12-38),
// stride 1, k1 / k3 (and the 1 -> 16 5x5 disparity heads dmNx.0), Cout <= 32, one input or a
// channel concat of up to 3 (spx_Nx.0, agg_N.0).
//
// A wave owns one 16-pixel column strip and R consecutive output rows (compile time), all couts of
// its tile and the full K.  Everything but the strip / row origin is fixed at compile time:
//   * the layer's weights live in VGPRs for the whole wave (A operands of v_mfma_f32_16x16x4_f32,
//     K*K*NG*MT registers: 36 for 16 -> 16 k3), loaded once: no LDS, no per-MFMA operand read;
//   * per input row and 4-channel group the K horizontally shifted B operands are K buffer_loads
//     (per-lane voffset = channel + shifted column, kOOB-marked outside; the row in soffset, kOOB
//     for a padding row), issued one (R = 2) or two (R >= 4) rows ahead of their MFMAs;
//   * input row r feeds output rows r - dy (dy < K): the row loop is unrolled over the R + K - 1 input
//     rows and only the (input, output) row pairs inside the wave's block are multiplied, so the
//     MFMA count is exactly R * K*K * NG * MT; consecutive MFMAs go to different output rows'
//     accumulators (no dependent-issue stall);
//   * an output row is finished as soon as its last input row is in: BN scale/shift, activation,
//     optional residual, * post_scale (+ second copy), 16 consecutive pixels per store.
// The 4 waves of a workgroup take 4 adjacent strips of the same rows (their halo columns are each
// other's interior: L1 / L2 hits).
#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

constexpr int kWideThreads = 256;

// KS = 2: the K reduction of a strip is split over two waves (channel groups [0, NGW) and [NGW, 2 NGW)),
// so a 192x624 layer runs ~2 waves per SIMD instead of ~1 (one wave alone leaves the MFMA pipe idle
// across its dependency and memory stalls); the two partial row blocks meet in
// LDS once, after the last MFMA, and each wave finishes half of the rows.
// WIN: every source inside one buffer window (conv_direct.h source_window: the plan's arena) -> one
// descriptor, a group's source folded into its voffsets; else a descriptor per source, picked per group.
template <int K, int NG, int MT, int R, int ACT, bool PLAIN, int KS, bool WIN>
__global__ void __launch_bounds__(kWideThreads) wconv_kernel(const esm_conv_desc a, const float* wbase, int wspan,
                                                             int d0, int d1, int d2) {
    constexpr int NR = R + K - 1;  // input rows a wave reads
    constexpr int NGW = (NG + KS - 1) / KS;  // channel groups per wave
    static_assert(KS == 1 || (KS == 2 && R % 2 == 0), "K split: two waves, an even row block");
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15, kq = lane >> 4;
    const int kh = KS == 2 ? (wave & 1) : 0;  // which half of the channel groups
    const int gb = kh * NGW;                  // first channel group of this wave
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int x0 = (bk_.x * (4 / KS) + wave / KS) * 16;
    const int y0 = bk_.y * R;
    const int b = bk_.z;
    const int cob = 0;  // Cout <= 16 * MT: one cout tile

    // ---- weights -> VGPRs: w[tap][cin_pad][cout_pad], lane (kq, n16) = k row 4g + kq, cout n16
    float wv[K * K][NGW][MT];
    {
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.w), static_cast<short>(0), 4 * K * K * a.cin_pad * a.cout_pad, 0x00020000);
        const unsigned wl = 4u * (kq * a.cout_pad + cob + n16);
#pragma unroll
        for (int t = 0; t < K * K; ++t)
#pragma unroll
            for (int g = 0; g < NGW; ++g)
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)  // groups past cin_pad read past the buffer: 0
                    wv[t][g][mt] = buf_load_s(wrs, wl, 4 * ((t * a.cin_pad + 4 * (gb + g)) * a.cout_pad + 16 * mt));
    }
    // BN / bias constants of the lane's couts
    float scl[MT][4], shf[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = min(cob + 16 * mt + 4 * kq + j, a.Cout - 1);
            scl[mt][j] = a.scale ? a.scale[co] : 1.f;
            shf[mt][j] = a.shift ? a.shift[co] : 0.f;
        }

    // ---- input addressing.  WIN: one descriptor over the sources' window, a group's source, batch item
    //      and channel folded into its per-lane voffsets once.  Else one descriptor per source over this
    //      batch item (the sources may lie anywhere: a caller's feature map next to the plan's own
    //      buffers); a concat splits on 4-channel boundaries (direct_ok), so a group's source is
    //      wave-uniform and picked per group by a scalar select
    const int sh = static_cast<int>(a.src[0].sh);
    const int ns = a.nsrc;
    const int lo1 = a.src[0].C, lo2 = a.src[0].C + (ns > 1 ? a.src[1].C : 0);
    auto src_rsrc = [&](const esm_src& q) __attribute__((always_inline)) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(q.ptr + b * q.sb), static_cast<short>(0),
                                                 4 * ((q.C - 1) * static_cast<int>(q.sc) + (a.Hi - 1) * sh + a.Wi),
                                                 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t rs0 = WIN ? __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wbase), static_cast<short>(0),
                                                                               wspan, 0x00020000)
                                           : src_rsrc(a.src[0]);
    const __amdgpu_buffer_rsrc_t rs1 = !WIN && ns > 1 ? src_rsrc(a.src[1]) : rs0;
    const __amdgpu_buffer_rsrc_t rs2 = !WIN && ns > 2 ? src_rsrc(a.src[2]) : rs0;
    const int xo = x0 + n16;
    int gs[NGW];          // source of group g (wave-uniform)
    unsigned vo[NGW][K];  // per-lane byte offset of group g's channel at column shift dx
#pragma unroll
    for (int g = 0; g < NGW; ++g) {
        const int cg = 4 * (gb + g);
        gs[g] = cg < lo1 ? 0 : (cg < lo2 ? 1 : 2);
        const int c = cg + kq;
        const int s = gs[g];
        const int cl = c - (s == 0 ? 0 : (s == 1 ? lo1 : lo2));
        const long long sb = s == 0 ? a.src[0].sb : (s == 1 ? a.src[1].sb : a.src[2].sb);
        const long long sc = s == 0 ? a.src[0].sc : (s == 1 ? a.src[1].sc : a.src[2].sc);
        const int dl = s == 0 ? d0 : (s == 1 ? d1 : d2);
#pragma unroll
        for (int dx = 0; dx < K; ++dx) {
            const int xi = xo - a.pw + dx;
            const bool ok = c < a.Cin && xo < a.Wo && xi >= 0 && xi < a.Wi;
            if constexpr (WIN)
                vo[g][dx] = ok ? static_cast<unsigned>(dl + 4 * (b * sb + cl * sc + xi)) : kOOB;
            else
                vo[g][dx] = ok ? 4u * static_cast<unsigned>(cl * static_cast<int>(sc) + xi) : kOOB;
        }
    }
    auto load_row = [&](float (&dst)[NGW][K], int r) {  // input row y0 - ph + r
        const int yi = y0 - a.ph + r;
        const int roff = (yi >= 0 && yi < a.Hi) ? 4 * yi * sh : static_cast<int>(kOOB);
#pragma unroll
        for (int g = 0; g < NGW; ++g)
#pragma unroll
            for (int dx = 0; dx < K; ++dx)
                dst[g][dx] = buf_load_s(WIN ? rs0 : (gs[g] == 0 ? rs0 : (gs[g] == 1 ? rs1 : rs2)), vo[g][dx], roff);
    };

    floatx4 acc[R][MT];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)  // the partial sum `pre` (one wave of a K split) or 0
            acc[r][mt] = kh == 0 ? pre_tile(a, b, cob + 16 * mt, kq, y0 + r, xo) : floatx4{0.f, 0.f, 0.f, 0.f};

    // output through a buffer descriptor over this batch item: per-lane voffset (cout, column) fixed
    // for the whole wave, the row in soffset; a cout past Cout / column past Wo / row past Ho carries
    // kOOB, so the hardware drops the store (no branches, no 64-bit address arithmetic per store)
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0), 4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
    unsigned ovo[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = cob + 16 * mt + 4 * kq + j;
            ovo[mt][j] = (co < a.Cout && xo < a.Wo) ? 4u * (co * static_cast<int>(a.oc) + xo) : kOOB;
        }
    auto finish = [&](int r) {  // output row y0 + r is complete
        const int yo = y0 + r;
        const int orow = yo < a.Ho ? 4 * yo * static_cast<int>(a.oh) : static_cast<int>(kOOB);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                float v = acc[r][mt][j];
                v = a.scale ? v * scl[mt][j] + shf[mt][j] : v + shf[mt][j];
                v = act_t<ACT>(v, a.act);
                if constexpr (!PLAIN) {
                    const int co = cob + 16 * mt + 4 * kq + j;
                    if (yo >= a.Ho || xo >= a.Wo || co >= a.Cout) continue;
                    if (a.res) v = v + a.res[b * a.rb + co * a.rc + static_cast<long long>(yo) * a.rh + xo];
                    const long long o = b * a.ob + co * a.oc + static_cast<long long>(yo) * a.oh + xo;
                    a.out[o] = v * a.post_scale;
                    if (a.out2) a.out2[o] = v * a.post_scale2;
                } else {
                    store_b32(__float_as_uint(v), ro_, static_cast<int>(ovo[mt][j]), orow);
                }
            }
    };

    // input rows in flight: PF ahead of the row being multiplied (ring of PF + 1 row buffers)
    constexpr int PF = R >= 4 ? 2 : 1;
    constexpr int NB = PF + 1;
    float bin[NB][NGW][K];
#pragma unroll
    for (int r = 0; r < PF; ++r) load_row(bin[r], r);
#pragma unroll
    for (int r = 0; r < NR; ++r) {  // input row r feeds output rows r - dy, dy = K-1 .. 0
        if (r + PF < NR) load_row(bin[(r + PF) % NB], r + PF);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < NGW; ++g)
#pragma unroll
            for (int dx = 0; dx < K; ++dx)
#pragma unroll
                for (int dy = 0; dy < K; ++dy) {
                    const int ro = r - dy;  // output row (block-relative) this tap row feeds
                    if (ro < 0 || ro >= R) continue;
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
                        acc[ro][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[dy * K + dx][g][mt], bin[r % NB][g][dx],
                                                                           acc[ro][mt], 0, 0, 0);
                }
        if (KS == 1 && r - (K - 1) >= 0) finish(r - (K - 1));
    }
    if constexpr (KS == 2) {
        // the partner's partial sums of the rows this wave finishes: wave kh finishes rows
        // [kh R/2, kh R/2 + R/2); it hands the other half over through LDS; sums in the fixed order
        // (groups [0, NGW)) + (groups [NGW, 2 NGW)) on both sides
        constexpr int RH = R / 2;
        __shared__ float xch[4][RH * MT * 4][64];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((r < RH) != (kh == 0)) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int j = 0; j < 4; ++j) xch[wave][((r % RH) * MT + mt) * 4 + j][lane] = acc[r][mt][j];
            }
        }
        __syncthreads();
        const int partner = wave ^ 1;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if ((r < RH) == (kh == 0)) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const float p = xch[partner][((r % RH) * MT + mt) * 4 + j][lane];
                        acc[r][mt][j] = kh == 0 ? acc[r][mt][j] + p : p + acc[r][mt][j];
                    }
                finish(r);
            }
        }
    }
}

template <int K, int NG, int MT>
int launch_wide_r(const esm_conv_desc& a, hipStream_t s) {
    const long long units = static_cast<long long>(a.B) * a.Ho * ceil_div(a.Wo, 16);
    // rows per wave, from a sweep of the 3x3 16 -> 16 layer at 192x624 (scripts/probes/k3_micro.hip):
    // 8 rows (2 rows of loads in flight) 10.3 us, 4 rows 11.7, 2 rows 14.1 -- fewer halo rows and
    // longer MFMA runs beat more waves per SIMD; small maps keep at least ~1 wave per SIMD
    // hint bits 26-27 (tuning, scripts/step_tune.py): 1 / 2 / 3 force R = 2 / 4 / 8
    const int rsel = (a.hint >> 26) & 3;
    const int R = rsel ? (1 << rsel) : (units >= 6144 ? 8 : (units >= 3072 ? 4 : 2));
    // hint bit 28: split each strip's K over two waves (the KS = 2 form, 2 strips per workgroup)
    const bool ks2 = (a.hint & (1 << 28)) && NG >= 2 && R >= 4;
    const dim3 grid(ceil_div(a.Wo, ks2 ? 32 : 64), ceil_div(a.Ho, R), static_cast<unsigned>(a.B));
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("conv(wide): grid too large");
    const float* base = nullptr;
    int span = 0, dl[ESM_MAX_SRC] = {0, 0, 0};
    const bool win = source_window(a, &base, &span, dl);
    // BasicConv (BN + GELU, nothing else: the hot path's common case) compiled with the activation
    // folded in and the branch-free buffer-store epilogue; anything else takes the general epilogue
    const bool gelu = a.act == ESM_ACT_GELU && !a.res && !a.out2 && a.post_scale == 1.f &&
                      static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
#define ESM_WIDE_W(RR, AC, KSP)                                                                                \
    do {                                                                                                        \
        if (win)                                                                                                \
            hipLaunchKernelGGL((wconv_kernel<K, NG, MT, RR, AC, (AC == ESM_ACT_GELU), KSP, true>), grid,         \
                               dim3(kWideThreads), 0, s, a, base, span, dl[0], dl[1], dl[2]);                   \
        else                                                                                                    \
            hipLaunchKernelGGL((wconv_kernel<K, NG, MT, RR, AC, (AC == ESM_ACT_GELU), KSP, false>), grid,        \
                               dim3(kWideThreads), 0, s, a, base, span, 0, 0, 0);                               \
    } while (0)
#define ESM_WIDE(RR, AC) ESM_WIDE_W(RR, AC, 1)
#define ESM_WIDE2(RR, AC) ESM_WIDE_W(RR, AC, 2)
    if constexpr (NG >= 2) {
        if (ks2) {
            if (R == 8) {
                if (gelu) ESM_WIDE2(8, ESM_ACT_GELU);
                else ESM_WIDE2(8, -1);
            } else {
                if (gelu) ESM_WIDE2(4, ESM_ACT_GELU);
                else ESM_WIDE2(4, -1);
            }
            return check_launch("conv(wide, K split)");
        }
    }
    if (R == 8) {
        if (gelu) ESM_WIDE(8, ESM_ACT_GELU);
        else ESM_WIDE(8, -1);
    } else if (R == 4) {
        if (gelu) ESM_WIDE(4, ESM_ACT_GELU);
        else ESM_WIDE(4, -1);
    } else {
        if (gelu) ESM_WIDE(2, ESM_ACT_GELU);
        else ESM_WIDE(2, -1);
    }
#undef ESM_WIDE
#undef ESM_WIDE2
#undef ESM_WIDE_W
    return check_launch("conv(wide)");
}

}  // namespace

// Whether the wide form can run this layer (and its weights fit the register budget).
bool wide_ok(const esm_conv_desc& a) {
    if (a.transposed || a.stride != 1 || a.kd != 1 || a.Di != 1 || a.Do != 1) return false;
    if (a.mul || a.up || a.shuffle > 1 || a.Cout > 32 || !direct_ok(a)) return false;
    for (int i = 0; i < a.nsrc; ++i)  // one soffset per input row for every source
        if (!a.src[i].ptr || a.src[i].sh != a.src[0].sh) return false;
    if (a.kh != a.kw || (a.kh != 1 && a.kh != 3 && a.kh != 5)) return false;
    const int ng = (a.Cin + 3) / 4, mt = a.Cout > 16 ? 2 : 1;
    if (a.kh == 5) return ng <= 2 && mt == 1;  // the 5x5 disparity heads (dmNx.0: 1 -> 16)
    return a.kh == 3 ? (ng * mt <= 10 && (mt == 1 || ng <= 4)) : ng * mt <= 32;
}

int launch_wide(const esm_conv_desc& a, hipStream_t s) {
    if (!wide_ok(a)) return arg_error("conv: wide-form hint not applicable");
    const int ng = (a.Cin + 3) / 4;
    const bool m2 = a.Cout > 16;
    if (a.kh == 5) return ng <= 1 ? launch_wide_r<5, 1, 1>(a, s) : launch_wide_r<5, 2, 1>(a, s);
    if (a.kh == 3) {
        if (!m2) {
            if (ng <= 2) return launch_wide_r<3, 2, 1>(a, s);
            if (ng <= 4) return launch_wide_r<3, 4, 1>(a, s);
            if (ng <= 6) return launch_wide_r<3, 6, 1>(a, s);
            if (ng <= 8) return launch_wide_r<3, 8, 1>(a, s);
            return launch_wide_r<3, 10, 1>(a, s);
        }
        if (ng <= 2) return launch_wide_r<3, 2, 2>(a, s);
        return launch_wide_r<3, 4, 2>(a, s);
    }
    if (!m2) {
        if (ng <= 4) return launch_wide_r<1, 4, 1>(a, s);
        if (ng <= 8) return launch_wide_r<1, 8, 1>(a, s);
        if (ng <= 12) return launch_wide_r<1, 12, 1>(a, s);
        if (ng <= 14) return launch_wide_r<1, 14, 1>(a, s);
        if (ng <= 16) return launch_wide_r<1, 16, 1>(a, s);
        if (ng <= 24) return launch_wide_r<1, 24, 1>(a, s);
        return launch_wide_r<1, 32, 1>(a, s);
    }
    if (ng <= 4) return launch_wide_r<1, 4, 2>(a, s);
    if (ng <= 8) return launch_wide_r<1, 8, 2>(a, s);
    return launch_wide_r<1, 16, 2>(a, s);
}

}  // namespace conv
}  // namespace esm
