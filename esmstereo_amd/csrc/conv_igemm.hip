// Implicit-GEMM convolution (2-D / 3-D, normal and k4-s2-p1 transposed) on fp32 MFMA.
//
// Replaces every conv of the hot path: BasicConv (models/submodule.py:12-38) in the 3-D
// stems (models/ESMStereo.py:610,620,622), the aggregation hourglass (:129-182), the ESM
// upsampler (:185-509) and the plain Conv2d layers of models/shufflemixer.py:124-126.
//
// GEMM view:   C[cout][pixel] = sum_k W[cout][k] * X[k][pixel],  k = (tap, cin)
// MFMA:        v_mfma_f32_16x16x4_f32 (exact f32, one fma per product, k-ordered)
//              A = 16 couts x 4 k (lane l: cout l&15, k l>>4) from the packed weights,
//              B = 4 k x 16 pixels (lane l: k l>>4, pixel l&15) gathered from the input,
//              C = 16 couts x 16 pixels, row (cout) = (l>>4)*4 + j, col (pixel) = l&15,
//              so every store instruction writes 16 consecutive output pixels per cout.
// Tiling:      256-thread workgroup = 4 waves; each wave owns 64 consecutive flattened
//              output pixels (4 n-tiles) of one (batch, depth) plane and 16*MT couts.
// Transposed:  ConvTranspose(k=4, s=2, p=1) is split into its 4 (2-D) / 8 (3-D) output
//              parity classes; inside a class every output sees exactly 2 taps per dim
//              (input i = m + q - t, kernel k = 1 - q + 2t for output o = 2m + q), so the
//              gather stays dense and the MFMA A operand is uniform over the n-tile.
// Fusions:     multi-source K (torch.cat along channels, with crop = smaller logical
//              extent than the source), BN scale/shift, GELU/SiLU/ReLU, broadcast multiply
//              (`* att`), residual add, bilinear-upsample-and-add, final scale and
//              PixelShuffle index remap are all applied in the epilogue.
#include "common.h"

namespace esm {
namespace {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kNT = 4;                       // 16-pixel n-tiles per wave
constexpr int kPixPerBlock = kThreads / 64 * kNT * 16;

template <bool D3, int K, int S, bool TR, int MT>
__global__ void __launch_bounds__(kThreads) conv_kernel(const esm_conv_desc a) {
    constexpr int KD = TR ? (D3 ? 2 : 1) : (D3 ? K : 1);
    constexpr int KH = TR ? 2 : K;
    constexpr int KW = TR ? 2 : K;
    constexpr int TAPS = KD * KH * KW;
    constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;

    const int lane = threadIdx.x & 63;
    const int wave = threadIdx.x >> 6;
    const int n16 = lane & 15;
    const int kq = lane >> 4;

    const int Hs = TR ? a.Hi : a.Ho;
    const int Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int P = Hs * Ws;
    const int b = blockIdx.y / Ds;
    const int zs = blockIdx.y - b * Ds;
    const int cls = TR ? static_cast<int>(blockIdx.z % NCLS) : 0;
    const int cob = static_cast<int>(TR ? blockIdx.z / NCLS : blockIdx.z) * 16 * MT;
    const int qd = (TR && D3) ? (cls >> 2) & 1 : 0;
    const int qh = TR ? (cls >> 1) & 1 : 0;
    const int qw = TR ? cls & 1 : 0;

    int py[kNT], px[kNT];
    bool pv[kNT];
    const int pbase = blockIdx.x * kPixPerBlock + wave * (kNT * 16);
#pragma unroll
    for (int nt = 0; nt < kNT; ++nt) {
        const int p = pbase + nt * 16 + n16;
        pv[nt] = p < P;
        py[nt] = pv[nt] ? p / Ws : 0;
        px[nt] = pv[nt] ? p - py[nt] * Ws : 0;
    }

    floatx4 acc[MT][kNT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < kNT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    const long long wcls = static_cast<long long>(cls) * TAPS * a.cin_pad * a.cout_pad;
#pragma unroll
    for (int td = 0; td < KD; ++td) {
        const int id = D3 ? (TR ? zs + qd - td : zs * S - a.pd + td) : 0;
        if (D3 && (id < 0 || id >= a.Di)) continue;  // block-uniform
#pragma unroll
        for (int th = 0; th < KH; ++th) {
#pragma unroll
            for (int tw = 0; tw < KW; ++tw) {
                const int tap = (td * KH + th) * KW + tw;
                int ih[kNT], iw[kNT];
                bool ok[kNT];
#pragma unroll
                for (int nt = 0; nt < kNT; ++nt) {
                    ih[nt] = TR ? py[nt] + qh - th : py[nt] * S - a.ph + th;
                    iw[nt] = TR ? px[nt] + qw - tw : px[nt] * S - a.pw + tw;
                    ok[nt] = pv[nt] && ih[nt] >= 0 && ih[nt] < a.Hi && iw[nt] >= 0 && iw[nt] < a.Wi;
                }
                const float* wt = a.w + wcls + static_cast<long long>(tap) * a.cin_pad * a.cout_pad + cob + n16;
                int cbase = 0;
                for (int s = 0; s < a.nsrc; ++s) {
                    const esm_src& sr = a.src[s];
                    const float* base = sr.ptr + static_cast<long long>(b) * sr.sb + (D3 ? static_cast<long long>(id) * sr.sd : 0);
                    long long off[kNT];
#pragma unroll
                    for (int nt = 0; nt < kNT; ++nt) off[nt] = static_cast<long long>(ih[nt]) * sr.sh + iw[nt];
                    for (int c0 = 0; c0 < sr.C; c0 += 4) {
                        const int c = c0 + kq;
                        const bool cok = c < sr.C;
                        float bv[kNT];
#pragma unroll
                        for (int nt = 0; nt < kNT; ++nt) {
                            const bool g = ok[nt] && cok;
                            const long long idx = g ? static_cast<long long>(c) * sr.sc + off[nt] : 0;
                            const float v = base[idx];
                            bv[nt] = g ? v : 0.f;
                        }
                        const float* wr = wt + static_cast<long long>(cbase + c) * a.cout_pad;
                        float av[MT];
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt) av[mt] = wr[mt * 16];
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                            for (int nt = 0; nt < kNT; ++nt)
                                acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], bv[nt], acc[mt][nt], 0, 0, 0);
                    }
                    cbase += sr.C;
                }
            }
        }
    }

    // ---------------------------------------------------------------- epilogue
    const int r = a.shuffle > 1 ? a.shuffle : 1;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = cob + mt * 16 + kq * 4 + j;
            if (co >= a.Cout) continue;
            const float scl = a.scale ? a.scale[co] : 1.f;
            const float shf = a.shift ? a.shift[co] : 0.f;
#pragma unroll
            for (int nt = 0; nt < kNT; ++nt) {
                if (!pv[nt]) continue;
                const int oz = TR ? 2 * zs + qd : zs;
                const int oy = TR ? 2 * py[nt] + qh : py[nt];
                const int ox = TR ? 2 * px[nt] + qw : px[nt];
                float v = acc[mt][nt][j];
                v = a.scale ? v * scl + shf : v + shf;
                v = apply_act(v, a.act);
                if (a.mul) v = v * a.mul[b * a.mb + co * a.mc + oy * a.mh + ox];
                if (a.res) v = v + a.res[b * a.rb + co * a.rc + oz * a.rd + oy * a.rh + ox];
                if (a.up) v = bilinear_at(a.up + b * a.ub, a.up_h, a.up_w, a.uh, a.up_f, oy, ox) + v;
                long long o;
                if (r > 1) {
                    const int cs = co / (r * r);
                    const int rem = co - cs * r * r;
                    const int yy = oy * r + rem / r;
                    const int xx = ox * r + (rem - (rem / r) * r);
                    o = b * a.ob + cs * a.oc + static_cast<long long>(yy) * a.oh + xx;
                } else {
                    o = b * a.ob + co * a.oc + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox;
                }
                a.out[o] = v * a.post_scale;
                if (a.out2) a.out2[o] = v * a.post_scale2;
            }
        }
    }
}

template <bool D3, int K, int S, bool TR>
int launch_mt(const esm_conv_desc& a, hipStream_t s) {
    const int MT = a.Cout > 16 ? 2 : 1;
    const int ncls = TR ? (D3 ? 8 : 4) : 1;
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    dim3 grid(ceil_div(static_cast<long long>(Hs) * Ws, kPixPerBlock), a.B * Ds, ceil_div(a.Cout, 16 * MT) * ncls);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("conv: grid too large");
    if (MT == 1)
        hipLaunchKernelGGL((conv_kernel<D3, K, S, TR, 1>), grid, dim3(kThreads), 0, s, a);
    else
        hipLaunchKernelGGL((conv_kernel<D3, K, S, TR, 2>), grid, dim3(kThreads), 0, s, a);
    return check_launch("conv");
}

}  // namespace

int launch_conv(const esm_conv_desc* d, hipStream_t s) {
    if (!d) return arg_error("conv: null descriptor");
    const esm_conv_desc& a = *d;
    if (!a.w || !a.out) return arg_error("conv: null weights/output");
    if (a.nsrc < 1 || a.nsrc > ESM_MAX_SRC) return arg_error("conv: nsrc must be 1..3");
    int cin = 0;
    for (int i = 0; i < a.nsrc; ++i) {
        if (!a.src[i].ptr || a.src[i].C <= 0) return arg_error("conv: bad source");
        if (a.nsrc > 1 && a.src[i].C % 4) return arg_error("conv: concatenated sources need C % 4 == 0");
        cin += a.src[i].C;
    }
    if (cin != a.Cin) return arg_error("conv: Cin != sum of source channels");
    if (a.B <= 0 || a.Cout <= 0) return arg_error("conv: bad B/Cout");
    if (a.cin_pad < ((a.Cin + 3) / 4) * 4) return arg_error("conv: cin_pad too small");
    if (a.cout_pad % 32 || a.cout_pad < a.Cout) return arg_error("conv: cout_pad must be a multiple of 32 >= Cout");
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (a.kh != a.kw) return arg_error("conv: kh must equal kw");
    if (d3 && a.kd != a.kh) return arg_error("conv: 3-D kernels must be cubic");
    if (!d3 && (a.Di != 1 || a.Do != 1)) return arg_error("conv: 2-D conv needs Di = Do = 1");
    if (a.shuffle > 1 && (d3 || a.transposed)) return arg_error("conv: pixel shuffle only for 2-D convs");
    if (a.up && (a.Cout != 1 || d3 || a.up_f <= 0)) return arg_error("conv: bilinear add needs 2-D, Cout == 1");
    if (a.transposed) {
        if (a.kh != 4 || a.stride != 2 || a.ph != 1 || a.pw != 1 || (d3 && a.pd != 1))
            return arg_error("conv: transposed conv supports k=4, s=2, p=1 only");
        if (a.Ho != 2 * a.Hi || a.Wo != 2 * a.Wi || (d3 && a.Do != 2 * a.Di))
            return arg_error("conv: transposed output extent must be 2x the input");
        return d3 ? launch_mt<true, 4, 2, true>(a, s) : launch_mt<false, 4, 2, true>(a, s);
    }
    const int S = a.stride;
    if (S != 1 && S != 2) return arg_error("conv: stride must be 1 or 2");
    if (a.Ho != (a.Hi + 2 * a.ph - a.kh) / S + 1 || a.Wo != (a.Wi + 2 * a.pw - a.kw) / S + 1 ||
        (d3 && a.Do != (a.Di + 2 * a.pd - a.kd) / S + 1))
        return arg_error("conv: output extent inconsistent with kernel/stride/padding");
    if (a.Ho <= 0 || a.Wo <= 0) return arg_error("conv: empty output");
    const int k = a.kh;
    if (d3) {
        if (k == 3 && S == 1) return launch_mt<true, 3, 1, false>(a, s);
        if (k == 3 && S == 2) return launch_mt<true, 3, 2, false>(a, s);
        if (k == 1 && S == 1) return launch_mt<true, 1, 1, false>(a, s);
    } else {
        if (k == 1 && S == 1) return launch_mt<false, 1, 1, false>(a, s);
        if (k == 3 && S == 1) return launch_mt<false, 3, 1, false>(a, s);
        if (k == 3 && S == 2) return launch_mt<false, 3, 2, false>(a, s);
        if (k == 5 && S == 1) return launch_mt<false, 5, 1, false>(a, s);
    }
    set_error("conv: unsupported kernel/stride combination");
    return ESM_ERR_UNSUPPORTED;
}

}  // namespace esm

extern "C" int esm_conv_f32(const esm_conv_desc* desc, void* stream) {
    return esm::launch_conv(desc, esm::as_stream(stream));
}
