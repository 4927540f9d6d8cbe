// LDS-staged implicit-GEMM convolution (2-D / 3-D, normal and k4-s2-p1 transposed) on the
// gfx950 fp32 matrix cores.  Included by conv2d.hip / conv3d.hip, which instantiate it.
//
// Replaces every conv of the hot path: BasicConv (models/submodule.py:12-38) in the 3-D
// stems (models/ESMStereo.py:610,620,622), the aggregation hourglass (:129-182), the ESM
// upsampler (:185-509) and the plain Conv2d layers of models/shufflemixer.py:124-126.
//
// GEMM view  C[cout][pixel] = sum_k W[cout][k] * X[k][pixel],   k = (tap, cin)
// MFMA       v_mfma_f32_16x16x4_f32 (exact f32, one rounding per product, k-ordered):
//            A = 16 couts x 4 k   (lane l: cout l&15, k l>>4)  from the LDS weight slab,
//            B = 4 k x 16 pixels  (lane l: k l>>4, pixel l&15) from the LDS input patch,
//            C = 16 couts x 16 px, row (cout) = (l>>4)*4 + j, col (pixel) = l&15, so every
//            store instruction writes 16 consecutive output pixels per cout.
// Tiling     a 256-thread workgroup (4 waves) owns a TH=4 x TW=16*NT output tile of one
//            (batch, depth) plane and 16*MT couts; wave w computes output row w of the tile.
//            Per input-channel chunk of CC channels the workgroup stages (a) the input patch
//            the tile needs (all taps; zero-padded borders) and (b) the weight slab
//            [tap][CC][16*MT] in LDS with all loads in flight at once, then runs the
//            TAPS x CC/4 MFMA steps fully unrolled from LDS: one global round trip per
//            chunk instead of one per K-step.
// LDS banks  channel planes are padded so lanes 0-15 (k=0) and 16-31 (k=1) of a ds_read_b32
//            hit disjoint banks: plane = 16 (mod 32) at unit pixel stride, odd at stride 2;
//            the 32-wide weight row is padded to 48 floats for the same reason.
// Transposed ConvTranspose(k=4, s=2, p=1) runs per output-parity class (grid z): inside a
//            class every output sees exactly 2 taps per dim (input m + q - t, kernel
//            1 - q + 2t for output 2m + q), so the gather is dense.
// Fusions    multi-source K (torch.cat along channels, crops = smaller logical extent than
//            the source), BN scale/shift, GELU / SiLU / ReLU, broadcast multiply (`* att`),
//            residual add, bilinear-upsample-and-add, final scales, PixelShuffle remap.
#pragma once

#include "common.h"

namespace esm {
namespace conv {

typedef float floatx4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int kTH = 4;  // output rows per workgroup (one per wave)

constexpr int pad_plane(int raw, bool stride2) {
    if (stride2) return raw | 1;
    const int up = (raw + 31) / 32 * 32;
    return (up - 16 >= raw) ? up - 16 : up + 16;
}

template <bool D3, int K, int S, bool TR, int MT, int NT, int CC>
struct Cfg {
    static constexpr int TW = 16 * NT;
    static constexpr int KT = TR ? 2 : K;
    static constexpr int KDT = D3 ? KT : 1;
    static constexpr int TAPS = KDT * KT * KT;
    static constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;
    static constexpr int PZ = KDT;
    static constexpr int PR = TR ? kTH + 1 : (kTH - 1) * S + K;
    static constexpr int PC = TR ? TW + 1 : (TW - 1) * S + K;
    static constexpr int RAW = PZ * PR * PC;
    static constexpr int PLANE = pad_plane(RAW, S == 2 && !TR);
    static constexpr int CO = 16 * MT;
    static constexpr int WROW = MT == 1 ? 16 : 48;
    static constexpr int XS = CC * PLANE;
    static constexpr int WS = TAPS * CC * WROW;
    static_assert((XS + WS) * 4 <= 64 * 1024, "conv tile exceeds the 64 KiB LDS budget (2 workgroups/CU)");
};

template <bool D3, int K, int S, bool TR, int MT, int NT, int CC>
__global__ void __launch_bounds__(kThreads) conv_kernel(const esm_conv_desc a) {
    using C = Cfg<D3, K, S, TR, MT, NT, CC>;
    __shared__ float xs[C::XS];
    __shared__ float wl[C::WS];

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int n16 = lane & 15;
    const int kq = lane >> 4;

    const int Hs = TR ? a.Hi : a.Ho;
    const int Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int tiles_w = (Ws + C::TW - 1) / C::TW;
    const int ty = blockIdx.x / tiles_w;
    const int tx = blockIdx.x - ty * tiles_w;
    const int y0 = ty * kTH;
    const int x0 = tx * C::TW;
    const int b = blockIdx.y / Ds;
    const int zs = blockIdx.y - b * Ds;
    const int cls = TR ? static_cast<int>(blockIdx.z % C::NCLS) : 0;
    const int cob = static_cast<int>(TR ? blockIdx.z / C::NCLS : blockIdx.z) * C::CO;
    const int qd = (TR && D3) ? (cls >> 2) & 1 : 0;
    const int qh = TR ? (cls >> 1) & 1 : 0;
    const int qw = TR ? cls & 1 : 0;

    // patch origin in input coordinates
    const int zo = D3 ? (TR ? zs + qd - 1 : zs * S - a.pd) : 0;
    const int ro = TR ? y0 + qh - 1 : y0 * S - a.ph;
    const int xo = TR ? x0 + qw - 1 : x0 * S - a.pw;

    floatx4 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    const long long wcls = static_cast<long long>(cls) * C::TAPS * a.cin_pad * a.cout_pad;
    const int c_src0 = a.src[0].C;
    const int c_src1 = a.src[1].C;

    for (int c0 = 0; c0 < a.Cin; c0 += CC) {
        __syncthreads();  // the previous chunk's LDS readers are done
        // ---- stage the input patch (zero outside the tensor / past Cin)
        for (int i = tid; i < CC * C::RAW; i += kThreads) {
            const int c = i / C::RAW;
            int rem = i - c * C::RAW;
            const int z = rem / (C::PR * C::PC);
            rem -= z * (C::PR * C::PC);
            const int r = rem / C::PC;
            const int col = rem - r * C::PC;
            const int cg = c0 + c;
            const int id = zo + z, ih = ro + r, iw = xo + col;
            float v = 0.f;
            if (cg < a.Cin && ih >= 0 && ih < a.Hi && iw >= 0 && iw < a.Wi && (!D3 || (id >= 0 && id < a.Di))) {
                const float* p;
                long long off;
                if (cg < c_src0) {
                    p = a.src[0].ptr;
                    off = b * a.src[0].sb + cg * a.src[0].sc + (D3 ? id * a.src[0].sd : 0) + ih * a.src[0].sh;
                } else if (cg - c_src0 < c_src1) {
                    const int cl = cg - c_src0;
                    p = a.src[1].ptr;
                    off = b * a.src[1].sb + cl * a.src[1].sc + (D3 ? id * a.src[1].sd : 0) + ih * a.src[1].sh;
                } else {
                    const int cl = cg - c_src0 - c_src1;
                    p = a.src[2].ptr;
                    off = b * a.src[2].sb + cl * a.src[2].sc + (D3 ? id * a.src[2].sd : 0) + ih * a.src[2].sh;
                }
                v = p[off + iw];
            }
            xs[c * C::PLANE + (z * C::PR + r) * C::PC + col] = v;
        }
        // ---- stage the weight slab [tap][CC][16*MT]
        for (int i = tid; i < C::TAPS * CC * C::CO; i += kThreads) {
            const int tap = i / (CC * C::CO);
            const int rem = i - tap * (CC * C::CO);
            const int c = rem / C::CO;
            const int co = rem - c * C::CO;
            wl[(tap * CC + c) * C::WROW + co] =
                a.w[wcls + (static_cast<long long>(tap) * a.cin_pad + c0 + c) * a.cout_pad + cob + co];
        }
        __syncthreads();
        // ---- MFMA over the chunk, fully unrolled, operands from LDS
#pragma unroll
        for (int tap = 0; tap < C::TAPS; ++tap) {
            const int td = tap / (C::KT * C::KT);
            const int th = (tap / C::KT) % C::KT;
            const int tw = tap % C::KT;
            const int zi = (D3 && TR) ? 1 - td : td;
            const int ri = TR ? wave + 1 - th : wave * S + th;
#pragma unroll
            for (int c4 = 0; c4 < CC / 4; ++c4) {
                const int c = c4 * 4 + kq;
                const float* xrow = xs + c * C::PLANE + (zi * C::PR + ri) * C::PC;
                float bv[NT];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int ci = TR ? nt * 16 + n16 + 1 - tw : (nt * 16 + n16) * S + tw;
                    bv[nt] = xrow[ci];
                }
                float av[MT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) av[mt] = wl[(tap * CC + c) * C::WROW + mt * 16 + n16];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], bv[nt], acc[mt][nt], 0, 0, 0);
            }
        }
    }

    // ---------------------------------------------------------------- epilogue
    const int ys = y0 + wave;  // sub-grid / output row of this wave
    if (ys >= Hs) return;
    const int r = a.shuffle > 1 ? a.shuffle : 1;
    const int oz = TR ? 2 * zs + qd : zs;
    const int oy = TR ? 2 * ys + qh : ys;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = cob + mt * 16 + kq * 4 + j;
            if (co >= a.Cout) continue;
            const float scl = a.scale ? a.scale[co] : 1.f;
            const float shf = a.shift ? a.shift[co] : 0.f;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int xsub = x0 + nt * 16 + n16;
                if (xsub >= Ws) continue;
                const int ox = TR ? 2 * xsub + qw : xsub;
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

// Channel-chunk size per geometry (fits 2 workgroups per CU at the largest NT, MT).
template <bool D3, int K, int S, bool TR>
constexpr int chunk() {
    if (TR) return D3 ? 8 : 16;
    if (D3) return K == 1 ? 16 : 4;
    if (K == 5) return 4;
    return S == 2 ? 8 : 16;
}

template <bool D3, int K, int S, bool TR, int MT, int NT>
int launch_nt(const esm_conv_desc& a, hipStream_t s) {
    constexpr int CC = chunk<D3, K, S, TR>();
    using C = Cfg<D3, K, S, TR, MT, NT, CC>;
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const long long tiles = static_cast<long long>((Ws + C::TW - 1) / C::TW) * ((Hs + kTH - 1) / kTH);
    dim3 grid(static_cast<unsigned>(tiles), a.B * Ds, ceil_div(a.Cout, C::CO) * C::NCLS);
    if (tiles > 0x7fffffffLL || grid.y > 65535u || grid.z > 65535u) return arg_error("conv: grid too large");
    hipLaunchKernelGGL((conv_kernel<D3, K, S, TR, MT, NT, CC>), grid, dim3(kThreads), 0, s, a);
    return check_launch("conv");
}

// Tile width: cover the row with as little waste as possible, then trade width for
// parallelism while the grid is small (tiny problems are latency-bound).
template <bool D3, int K, int S, bool TR>
int launch_geom(const esm_conv_desc& a, hipStream_t s) {
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int MT = a.Cout > 16 ? 2 : 1;
    constexpr int NTMAX = (D3 && K == 3 && S == 2) ? 2 : 4;
    int nt = Ws > 32 ? 4 : (Ws > 16 ? 2 : 1);
    if (nt > NTMAX) nt = NTMAX;
    const long long per = static_cast<long long>(a.B) * Ds * ((Hs + kTH - 1) / kTH) * ceil_div(a.Cout, 16 * MT) *
                          (TR ? (D3 ? 8 : 4) : 1);
    while (nt > 1 && per * ((Ws + 16 * nt - 1) / (16 * nt)) < 512) nt /= 2;
    if (MT == 1) {
        if (nt == 4) return launch_nt<D3, K, S, TR, 1, NTMAX>(a, s);
        if (nt == 2) return launch_nt<D3, K, S, TR, 1, 2>(a, s);
        return launch_nt<D3, K, S, TR, 1, 1>(a, s);
    }
    if (nt == 4) return launch_nt<D3, K, S, TR, 2, NTMAX>(a, s);
    if (nt == 2) return launch_nt<D3, K, S, TR, 2, 2>(a, s);
    return launch_nt<D3, K, S, TR, 2, 1>(a, s);
}

}  // namespace conv
}  // namespace esm
