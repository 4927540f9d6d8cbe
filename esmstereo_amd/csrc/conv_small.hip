// Lean K-split convolution for the latency-bound layers of the hot path: the low-resolution
// levels of the 3-D aggregation hourglass (models/ESMStereo.py:129-182, 1/32-1/64 of the input at
// S-K: 2x3x10 .. 6x12x39 voxels) and the small 2-D maps of the ESM upsampler's first stage and its
// refinement hourglass (:185-239, 242-509: 12x39 .. 48x156), i.e. BasicConv (models/submodule.py:
// 12-38) where the whole layer is a few dozen output tiles.
//
// Why a third form: at these sizes one wave's lifetime is the kernel's duration, and in the general
// forms it is dominated by instruction issue, not by memory or the matrix pipe: per-op PMC of the S-K
// step (profiles/r02_pmc_sq_ops_SK.txt) shows ~700 VALU + ~700 SALU instructions per wave (runtime
// tap decomposition, grid-index divisions, SGPR spills to VGPR lanes) around 9-54 MFMAs, 15k cycles
// per wave, 43 % of them issuing.  Here everything a wave does is fixed at compile time except the
// channel-group loop:
//   * grid = (16-pixel column segment, sub-grid row, plane x batch x parity class x cout tile); the
//     z split uses host-computed reciprocals (two s_mul_hi), no division sequence;
//   * the K reduction is split over the 4 waves by 4-channel GROUP (wave w takes groups w, w+4, ..),
//     so every wave walks the same compile-time tap list; a group's B operand is one buffer_load per
//     tap: per-lane voffset = channel + column part (kOOB-marked outside, conv_direct.h), wave-uniform
//     soffset = the tap's (plane, row) part (kOOB for a padding row), so borders cost no branches;
//   * A (weights [cls][tap][cin_pad][cout_pad]): per-lane voffset fixed for the whole kernel, the
//     tap / group part in soffset;
//   * the 4 waves' partial tiles meet in LDS and are added in a fixed order (w0 + w1 + w2 + w3:
//     deterministic); then every thread finishes one (cout, pixel) element: BN scale/shift,
//     activation, optional residual, * post_scale (+ the second copy), one coalesced store.
// Plain epilogues only (no `* mul`, bilinear add or PixelShuffle): the launcher falls back otherwise.
#include "conv_up1.h"

namespace esm {
namespace conv {
namespace {

constexpr int kSmallThreads = 256;

// floor(n / d) for n * d < 2^32 from the host-computed m = ceil(2^32 / d) (m = 0 encodes d = 1)
__device__ __forceinline__ int fast_div(int n, unsigned m) {
    return m ? static_cast<int>(__umulhi(static_cast<unsigned>(n), m)) : n;
}

inline unsigned magic_for(int d) {
    return d <= 1 ? 0u : static_cast<unsigned>(((1ull << 32) + static_cast<unsigned long long>(d) - 1) / d);
}

// NW = 4 or 8 waves splitting the K reduction (8: layers with more than 4 channel groups, so that no
// wave walks two groups one after the other; the epilogue runs on the first 256 threads)
// XB > 0 (transposed, MT = 1): the 1x1 BasicConv behind it fused (conv_up1.h; bp: its descriptor, up to XB
// extra 4-channel k-steps): wave 0 finishes the 16 x 16 tile, the conv's output never leaves its registers
template <bool D3, int K, int S, bool TR, int MT, int ACT, bool PLAIN, int NW, int XB>
__device__ __forceinline__ void lconv_body(const esm_conv_desc& a, unsigned m_ds, unsigned m_b, const esm_conv_desc* bp) {
    constexpr int KT = TR ? 2 : K;  // taps per dim (per parity class when transposed)
    constexpr int KDT = D3 ? KT : 1;
    constexpr int TAPS = KDT * KT * KT;
    constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;
    __shared__ __attribute__((aligned(16))) float red[NW * MT * 4 * 64];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n16 = lane & 15, kq = lane >> 4;

    const int Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int x0 = bk_.x * 16;
    const int ys = bk_.y;
    const int zz = bk_.z;
    const int r1 = fast_div(zz, m_ds);
    const int zs = zz - r1 * Ds;
    const int r2 = fast_div(r1, m_b);
    const int b = r1 - r2 * a.B;
    const int cls = TR ? (r2 & (NCLS - 1)) : 0;
    const int cob = (TR ? r2 / NCLS : r2) * 16 * MT;
    const int qd = (TR && D3) ? (cls >> 2) & 1 : 0;
    const int qh = TR ? (cls >> 1) & 1 : 0;
    const int qw = TR ? cls & 1 : 0;

    // epilogue constants of the (cout, pixel) elements this thread finishes, loaded up front
    const int ej = (tid >> 6) & 3;  // accumulator register j of the element
    const int ecol = lane & 15;
    float scl[MT], shf[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int co = min(cob + 16 * mt + 4 * kq + ej, a.Cout - 1);
        scl[mt] = a.scale ? a.scale[co] : 1.f;
        shf[mt] = a.shift ? a.shift[co] : 0.f;
    }

    // fused 1x1: its weights, BN and the extra sources at this lane's output pixel, loaded up front by wave 0
    Up1Ops<(XB > 0 ? XB : 1)> u1;
    float bx1[(XB > 0 ? XB : 1)];
    float s1[4], h1[4];
    if constexpr (XB > 0) {
        static_assert(TR && MT == 1, "fused 1x1: transposed conv, one cout tile");
        if (wave == 0) {
            const esm_conv_desc& bb = *bp;
            up1_weights(u1, bb, a.Cout, lane);
            const Up1Src us = up1_src(bb, b, D3);
            up1_extra(bx1, us, bb, a.Cout, lane, D3 ? 2 * zs + qd : 0, 2 * ys + qh, 2 * (x0 + n16) + qw);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = min(4 * kq + r, a.Cout - 1);
                s1[r] = a.scale[co];
                h1[r] = a.shift[co];
            }
        }
    }

    // per-lane column byte offsets per horizontal tap (kOOB: outside the input or past the map)
    const int xs = x0 + n16;
    unsigned xoff[KT];
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        const int xi = TR ? xs + qw - t : xs * S - a.pw + t;
        xoff[t] = (xs < Ws && xi >= 0 && xi < a.Wi) ? 4u * xi : kOOB;
    }
    // input plane / row of each vertical tap (wave-uniform)
    int zin[KDT], yin[KT];
    bool zok[KDT], yok[KT];
#pragma unroll
    for (int t = 0; t < KDT; ++t) {
        zin[t] = D3 ? (TR ? zs + qd - t : zs * S - a.pd + t) : 0;
        zok[t] = !D3 || (zin[t] >= 0 && zin[t] < a.Di);
    }
#pragma unroll
    for (int t = 0; t < KT; ++t) {
        yin[t] = TR ? ys + qh - t : ys * S - a.ph + t;
        yok[t] = yin[t] >= 0 && yin[t] < a.Hi;
    }

    const int wtap = a.cin_pad * a.cout_pad;  // elements per tap in the packed weights
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w + static_cast<long long>(cls) * TAPS * wtap), static_cast<short>(0), 4 * TAPS * wtap,
        0x00020000);
    const unsigned wl = 4u * (kq * a.cout_pad + cob + n16);

    floatx4 acc[2][MT];
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[c][mt] = floatx4{0.f, 0.f, 0.f, 0.f};
    if constexpr (!TR && !D3) {  // the partial sum `pre` (2-D) starts wave 0's accumulator
        if (wave == 0) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[0][mt] = pre_tile(a, b, cob + 16 * mt, kq, ys, x0 + n16);
        }
    }

    const int G = (a.Cin + 3) >> 2;
    const int lo1 = a.src[0].C, lo2 = a.src[0].C + a.src[1].C;
    for (int g = wave; g < G; g += NW) {
        const int c0 = 4 * g;
        // the group's source (4-channel aligned splits): named-field selects, no runtime index
        const int s = c0 < lo1 ? 0 : (c0 < lo2 ? 1 : 2);
        const int lo = s == 0 ? 0 : (s == 1 ? lo1 : lo2);
        const float* sp = s == 0 ? a.src[0].ptr : (s == 1 ? a.src[1].ptr : a.src[2].ptr);
        const int sC = s == 0 ? a.src[0].C : (s == 1 ? a.src[1].C : a.src[2].C);
        const long long sb = s == 0 ? a.src[0].sb : (s == 1 ? a.src[1].sb : a.src[2].sb);
        const int sc = static_cast<int>(s == 0 ? a.src[0].sc : (s == 1 ? a.src[1].sc : a.src[2].sc));
        const int sd = static_cast<int>(s == 0 ? a.src[0].sd : (s == 1 ? a.src[1].sd : a.src[2].sd));
        const int sh = static_cast<int>(s == 0 ? a.src[0].sh : (s == 1 ? a.src[1].sh : a.src[2].sh));
        const int span = 4 * ((sC - 1) * sc + (D3 ? (a.Di - 1) * sd : 0) + (a.Hi - 1) * sh + a.Wi);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sp + b * sb), static_cast<short>(0), span, 0x00020000);
        const int cl = c0 - lo + kq;
        const unsigned chv = (c0 + kq < a.Cin && cl < sC) ? 4u * cl * sc : kOOB;

        float bv[TAPS], av[TAPS][MT];
#pragma unroll
        for (int dz = 0; dz < KDT; ++dz)
#pragma unroll
            for (int dy = 0; dy < KT; ++dy) {
                const int roff = (zok[dz] && yok[dy]) ? 4 * ((D3 ? zin[dz] * sd : 0) + yin[dy] * sh)
                                                      : static_cast<int>(kOOB);
#pragma unroll
                for (int dx = 0; dx < KT; ++dx) {
                    const int tap = (dz * KT + dy) * KT + dx;
                    bv[tap] = buf_load_s(rs, chv + xoff[dx], roff);
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
                        av[tap][mt] = buf_load_s(wrs, wl, 4 * (tap * wtap + c0 * a.cout_pad + 16 * mt));
                }
            }
        __builtin_amdgcn_sched_barrier(0);  // every load of the group in flight before the first MFMA
#pragma unroll
        for (int tap = 0; tap < TAPS; ++tap)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
                acc[tap & 1][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[tap][mt], bv[tap], acc[tap & 1][mt], 0, 0, 0);
    }

    // the 4 waves' partial tiles -> LDS [wave][mt][j][lane]; fixed-order sum per element
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[((wave * MT + mt) * 4 + j) * 64 + lane] = acc[0][mt][j] + acc[1][mt][j];
    __syncthreads();
    if (NW > 4 && tid >= 256) return;
    // fixed-order sum of the NW partial tiles of element e
    auto reduced = [&](int e) {
        float v = red[e];
#pragma unroll
        for (int w = 1; w < NW; ++w) v = v + red[w * MT * 256 + e];
        return v;
    };

    if constexpr (XB > 0) {
        // wave 0: y = GELU(BN(conv)) in the D layout (lane (n16, kq): channels 4 kq + r), then the 1x1
        if (wave != 0) return;
        const esm_conv_desc& bb = *bp;
        float y[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) y[r] = gelu_erf(reduced(r * 64 + lane) * s1[r] + h1[r]);
        const floatx4 o = up1_finish(u1, y, bx1, D3 ? floatx4{0.f, 0.f, 0.f, 0.f}
                                                    : pre_tile(bb, b, 0, kq, 2 * ys + qh, 2 * (x0 + n16) + qw));
        const int ox = 2 * (x0 + n16) + qw, oy = 2 * ys + qh, oz = D3 ? 2 * zs + qd : 0;
        const bool pok = ox < bb.Wo && oy < bb.Ho && oz < bb.Do;
        const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
            bb.out + b * bb.ob, static_cast<short>(0),
            4 * ((bb.Cout - 1) * static_cast<int>(bb.oc) + (D3 ? (bb.Do - 1) * static_cast<int>(bb.od) : 0) +
                 (bb.Ho - 1) * static_cast<int>(bb.oh) + bb.Wo),
            0x00020000);
        const int orow = 4 * ((D3 ? oz * static_cast<int>(bb.od) : 0) + oy * static_cast<int>(bb.oh));
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int co = 4 * kq + r;
            const unsigned vo = (pok && co < bb.Cout) ? 4u * static_cast<unsigned>(co * static_cast<int>(bb.oc) + ox) : kOOB;
            store_b32(__float_as_uint(o[r]), ro_, static_cast<int>(vo), orow);
        }
        return;
    }

    const int xsub = x0 + ecol;
    const int oz = TR ? 2 * zs + qd : zs;
    const int oy = TR ? 2 * ys + qh : ys;
    const int ox = TR ? 2 * xsub + qw : xsub;
    if constexpr (PLAIN) {
        // buffer store over this batch item: (cout, column) in voffset, (plane, row) in soffset; a cout
        // past Cout or a column past the map carries kOOB and the hardware drops the store
        const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
            a.out + b * a.ob, static_cast<short>(0),
            4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (D3 ? (a.Do - 1) * static_cast<int>(a.od) : 0) +
                 (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
            0x00020000);
        const int orow = 4 * ((D3 ? oz * static_cast<int>(a.od) : 0) + oy * static_cast<int>(a.oh));
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int co = cob + 16 * mt + 4 * kq + ej;
            const int e = (mt * 4 + ej) * 64 + lane;
            float v = reduced(e);
            v = a.scale ? v * scl[mt] + shf[mt] : v + shf[mt];
            v = act_t<ACT>(v, a.act);
            const unsigned vo = (co < a.Cout && xsub < Ws) ? 4u * (co * static_cast<int>(a.oc) + ox) : kOOB;
            store_b32(__float_as_uint(v), ro_, static_cast<int>(vo), orow);
        }
        return;
    }
    if (xsub >= Ws) return;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int co = cob + 16 * mt + 4 * kq + ej;
        if (co >= a.Cout) continue;
        const int e = (mt * 4 + ej) * 64 + lane;
        float v = reduced(e);
        v = a.scale ? v * scl[mt] + shf[mt] : v + shf[mt];
        v = act_t<ACT>(v, a.act);
        if (a.res) v = v + a.res[b * a.rb + co * a.rc + static_cast<long long>(oz) * a.rd + static_cast<long long>(oy) * a.rh + ox];
        const long long o = b * a.ob + co * a.oc + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox;
        a.out[o] = v * a.post_scale;
        if (a.out2) a.out2[o] = v * a.post_scale2;
    }
}

template <bool D3, int K, int S, bool TR, int MT, int ACT, bool PLAIN, int NW = 4>
__global__ void __launch_bounds__(64 * NW) lconv_kernel(const esm_conv_desc a, unsigned m_ds, unsigned m_b) {
    lconv_body<D3, K, S, TR, MT, ACT, PLAIN, NW, 0>(a, m_ds, m_b, nullptr);
}

// ConvTranspose + crop + cat + 1x1 (conv_up1.h)
template <bool D3, int NW, int XB>
__global__ void __launch_bounds__(64 * NW) lconv_up1_kernel(const esm_conv_desc a, unsigned m_ds, unsigned m_b,
                                                           const esm_conv_desc b) {
    lconv_body<D3, 4, 2, true, 1, ESM_ACT_GELU, true, NW, XB>(a, m_ds, m_b, &b);
}

template <bool D3, int K, int S, bool TR>
int launch_small_m(const esm_conv_desc& a, hipStream_t s) {
    constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int MT = a.Cout > 16 ? 2 : 1;
    const long long z = static_cast<long long>(Ds) * a.B * NCLS * ceil_div(a.Cout, 16 * MT);
    if (Hs > 65535 || z > 65535) return arg_error("conv(small): grid too large");
    const dim3 grid(ceil_div(Ws, 16), static_cast<unsigned>(Hs), static_cast<unsigned>(z));
    const unsigned mds = magic_for(Ds), mb = magic_for(a.B);
    // BasicConv (BN + GELU, nothing else) with the activation folded in and the buffer-store epilogue
    const bool gelu = a.act == ESM_ACT_GELU && !a.res && !a.out2 && a.post_scale == 1.f &&
                      static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(D3 ? a.Do : 1) * a.od +
                              static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    // hint bit 29: 8 waves per workgroup (K split 8 ways) for layers with more than 4 channel groups
    const bool w8 = (a.hint & (1 << 29)) && (a.Cin + 3) / 4 > 4;
#define ESM_SMALL(M, AC, PL)                                                                                   \
    do {                                                                                                       \
        if (w8)                                                                                                \
            hipLaunchKernelGGL((lconv_kernel<D3, K, S, TR, M, AC, PL, 8>), grid, dim3(512), 0, s, a, mds, mb); \
        else                                                                                                   \
            hipLaunchKernelGGL((lconv_kernel<D3, K, S, TR, M, AC, PL>), grid, dim3(kSmallThreads), 0, s, a, mds, mb); \
    } while (0)
    if (MT == 1) {
        if (gelu) ESM_SMALL(1, ESM_ACT_GELU, true);
        else ESM_SMALL(1, -1, false);
    } else {
        if (gelu) ESM_SMALL(2, ESM_ACT_GELU, true);
        else ESM_SMALL(2, -1, false);
    }
#undef ESM_SMALL
    return check_launch("conv(small)");
}

template <bool D3, int NW>
int launch_small_up1_x(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s, const dim3& grid, unsigned mds,
                       unsigned mb) {
    const int xb = (b.Cin - a.Cout) >> 2;
    if (xb <= 3) hipLaunchKernelGGL((lconv_up1_kernel<D3, NW, 3>), grid, dim3(64 * NW), 0, s, a, mds, mb, b);
    else if (xb <= 4) hipLaunchKernelGGL((lconv_up1_kernel<D3, NW, 4>), grid, dim3(64 * NW), 0, s, a, mds, mb, b);
    else if (xb <= 8) hipLaunchKernelGGL((lconv_up1_kernel<D3, NW, 8>), grid, dim3(64 * NW), 0, s, a, mds, mb, b);
    else if (xb <= 10) hipLaunchKernelGGL((lconv_up1_kernel<D3, NW, 10>), grid, dim3(64 * NW), 0, s, a, mds, mb, b);
    else hipLaunchKernelGGL((lconv_up1_kernel<D3, NW, 12>), grid, dim3(64 * NW), 0, s, a, mds, mb, b);
    return check_launch("conv(small, transposed + 1x1)");
}

}  // namespace

bool small_ok(const esm_conv_desc& a);

// ConvTranspose k4 s2 (<= 16 couts) + crop + cat + 1x1 (<= 16 couts, <= 48 extra channels) in the lean form
// (conv_up1.h); a and b validated by the caller (launch_convt_1x1)
int launch_small_up1(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    if (!small_ok(a) || !a.transposed) return arg_error("convt_1x1: the lean form cannot run this transposed conv");
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || a.kd == 4;
    const int ncls = d3 ? 8 : 4;
    const int Ds = d3 ? a.Di : 1;
    const long long z = static_cast<long long>(Ds) * a.B * ncls;
    if (a.Hi > 65535 || z > 65535) return arg_error("convt_1x1(small): grid too large");
    const dim3 grid(ceil_div(a.Wi, 16), static_cast<unsigned>(a.Hi), static_cast<unsigned>(z));
    const unsigned mds = magic_for(Ds), mb = magic_for(a.B);
    const bool w8 = (a.hint & (1 << 29)) && (a.Cin + 3) / 4 > 4;
    if (d3) return w8 ? launch_small_up1_x<true, 8>(a, b, s, grid, mds, mb) : launch_small_up1_x<true, 4>(a, b, s, grid, mds, mb);
    return w8 ? launch_small_up1_x<false, 8>(a, b, s, grid, mds, mb) : launch_small_up1_x<false, 4>(a, b, s, grid, mds, mb);
}

// Whether the lean form can run this layer: plain epilogue, 4-channel aligned source splits, spans
// addressable by 32-bit buffer offsets (conv_direct.h direct_ok), a kernel shape it instantiates.
bool small_ok(const esm_conv_desc& a) {
    if (a.mul || a.up || a.shuffle > 1 || !direct_ok(a)) return false;
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (a.transposed) return a.kh == 4 && a.stride == 2;
    if (a.stride != 1 && a.stride != 2) return false;
    if (a.kh == 5) return !d3 && a.stride == 1;
    return a.kh == 1 || a.kh == 3;
}

// Automatic choice (no hint): the small form for every layer it can run whose output is at most
// 2^17 (pixel x 16-cout tile) units.  Fitted to scripts/autotune.py on MI355X (profiles/
// r02_autotune_*.log): it won on every layer of the S / M / L hot paths up to the 96x312 maps and tied
// at 192x624; the wide 3-D stems keep the 16-block form (checked first), single-output-channel
// transposed layers keep their VALU form.
bool small_auto(const esm_conv_desc& a) {
    if (!small_ok(a)) return false;
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (a.transposed && a.Cout == 1) return false;
    const long long px = static_cast<long long>(a.B) * (d3 ? a.Do : 1) * a.Ho * a.Wo;
    const long long units = px * ceil_div(a.Cout, a.Cout > 16 ? 32 : 16);
    return units <= (1LL << 17);
}

int launch_small(const esm_conv_desc& a, hipStream_t s) {
    if (!small_ok(a)) return arg_error("conv: small-form hint not applicable");
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (a.transposed) return d3 ? launch_small_m<true, 4, 2, true>(a, s) : launch_small_m<false, 4, 2, true>(a, s);
    const int k = a.kh, S = a.stride;
    if (d3) {
        if (k == 1 && S == 1) return launch_small_m<true, 1, 1, false>(a, s);
        if (k == 3 && S == 1) return launch_small_m<true, 3, 1, false>(a, s);
        if (k == 3 && S == 2) return launch_small_m<true, 3, 2, false>(a, s);
    } else {
        if (k == 1 && S == 1) return launch_small_m<false, 1, 1, false>(a, s);
        if (k == 3 && S == 1) return launch_small_m<false, 3, 1, false>(a, s);
        if (k == 3 && S == 2) return launch_small_m<false, 3, 2, false>(a, s);
        if (k == 5 && S == 1) return launch_small_m<false, 5, 1, false>(a, s);
    }
    return arg_error("conv(small): unsupported kernel/stride");
}

}  // namespace conv
}  // namespace esm
