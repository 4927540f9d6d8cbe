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
// C1 path    single-output-channel layers (tail convs, the refinement heads) would use
//            1/16 of an MFMA tile; they run as a VALU dot product instead, one output pixel
//            per lane, weights broadcast from LDS.
// Tiling     a 256-thread workgroup (4 waves) owns a TH x TW(=16*NT) output tile of one
//            (batch, depth) plane and 16*MT couts.  KS = 1: TH = 4, wave w computes row w.
//            KS = 4 (small, latency-bound layers): TH = 1 and the 4 waves split the taps of
//            the same tile, their partial sums added in LDS in a fixed order at the end
//            (deterministic), which cuts the serial MFMA chain per wave by 4.
// Staging    per input-channel chunk of CC channels the workgroup needs (a) the input patch
//            of the tile (all taps, zero-padded borders) and (b) the weight slab
//            [tap][CC][16*MT].  Every thread issues its share of both as one batch of
//            independent loads into registers (compile-time counts), and the batch for chunk
//            c+1 is issued before the MFMAs of chunk c, so global latency overlaps compute.
//            CC is the largest of 16/8/4 whose tile fits 64 KiB of LDS (2 workgroups/CU).
// LDS banks  channel planes are padded so lanes 0-15 (k=0) and 16-31 (k=1) of a ds_read_b32
//            hit disjoint banks: plane = 16 (mod 32) at unit pixel stride, odd at stride 2;
//            the 32-wide weight row is padded to 48 floats for the same reason.
// Transposed ConvTranspose(k=4, s=2, p=1) runs per output-parity class (grid z): inside a
//            class every output sees exactly 2 taps per dim (input m + q - t, kernel
//            1 - q + 2t for output 2m + q), so the gather is dense.
// Fusions    multi-source K (torch.cat along channels, crops = smaller logical extent than
//            the source), BN scale/shift, GELU / SiLU / ReLU, broadcast multiply (`* att`),
//            residual add, bilinear-upsample-and-add, final scales, PixelShuffle remap (with
//            one 16-byte store per lane for r = 4).
#pragma once

#include "conv_c1.h"
#include "conv_direct.h"
#include "conv_rows.h"
#include "conv_epilogue.h"

namespace esm {
namespace conv {

constexpr int kThreads = 256;
constexpr int kLdsBudget = 64 * 1024;

constexpr int pad_plane(int raw, bool stride2) {
    if (stride2) return raw | 1;
    const int up = (raw + 31) / 32 * 32;
    return (up - 16 >= raw) ? up - 16 : up + 16;
}

template <bool D3, int K, int S, bool TR, int MT, int NT, bool C1, int KS>
struct Geo {
    static constexpr int TH = 4 / KS;
    static constexpr int TW = 16 * NT;
    static constexpr int KT = TR ? 2 : K;
    static constexpr int KDT = D3 ? KT : 1;
    static constexpr int TAPS = KDT * KT * KT;
    static constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;
    static constexpr int PZ = KDT;
    static constexpr int PR = TR ? TH + 1 : (TH - 1) * S + K;
    static constexpr int PC = TR ? TW + 1 : (TW - 1) * S + K;
    static constexpr int RAW = PZ * PR * PC;
    static constexpr int PLANE = pad_plane(RAW, S == 2 && !TR);
    static constexpr int CO = C1 ? 4 : 16 * MT;  // couts staged per workgroup (C1: 1 used)
    static constexpr int WROW = C1 ? 4 : (MT == 1 ? 16 : 48);
    static constexpr int RAW64 = (RAW + 63) / 64 * 64;
    static constexpr int RED = (KS - 1) * TH * 64 * MT * NT * 4;  // K-split partial sums
    static constexpr int lds_bytes(int cc) {
        const int xs = cc * PLANE, ws = TAPS * cc * WROW;
        return 4 * ((xs + ws) > RED ? (xs + ws) : RED);
    }
    static constexpr int nx(int cc) { return (cc * RAW64 + kThreads - 1) / kThreads; }
    // largest channel chunk that fits the LDS budget with a bounded staging register file
    static constexpr int CC = (lds_bytes(16) <= kLdsBudget && nx(16) <= 40) ? 16
                              : (lds_bytes(8) <= kLdsBudget && nx(8) <= 40) ? 8 : 4;
    static constexpr int XS = CC * PLANE;
    static constexpr int WS = TAPS * CC * WROW;
    static constexpr int SMEM = (XS + WS) > RED ? (XS + WS) : RED;
    static constexpr int NX = nx(CC);                                            // patch loads / thread
    static constexpr int NW = (TAPS * CC * CO / 4 + kThreads - 1) / kThreads;  // float4 weight loads / thread
    static constexpr bool OK = SMEM * 4 <= kLdsBudget;  // configurations that do not fit are never launched
    static_assert(XS % 4 == 0, "weight slab must start 16-B aligned");
    static_assert(!C1 || (NT == 4 && KS == 1), "C1 path maps one output pixel per lane (TW = 64)");
};

template <bool D3, int K, int S, bool TR, int MT, int NT, bool C1, int KS>
__global__ void __launch_bounds__(kThreads) conv_kernel(const esm_conv_desc a) {
    using C = Geo<D3, K, S, TR, MT, NT, C1, KS>;
    constexpr int CC = C::CC;
    __shared__ __attribute__((aligned(16))) float smem[C::SMEM];
    float* xs = smem;
    float* wl = smem + C::XS;

    const int tid = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int row = wave / KS;    // output row of the tile this wave computes
    const int kpart = wave % KS;  // tap subset (K-split)
    const int n16 = lane & 15;
    const int kq = lane >> 4;

    const int Hs = TR ? a.Hi : a.Ho;
    const int Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int tiles_w = (Ws + C::TW - 1) / C::TW;
    const int ty = blockIdx.x / tiles_w;
    const int tx = blockIdx.x - ty * tiles_w;
    const int y0 = ty * C::TH;
    const int x0 = tx * C::TW;
    const int b = blockIdx.y / Ds;
    const int zs = blockIdx.y - b * Ds;
    const int cls = TR ? static_cast<int>(blockIdx.z % C::NCLS) : 0;
    const int cob = static_cast<int>(TR ? blockIdx.z / C::NCLS : blockIdx.z) * (C1 ? 1 : C::CO);
    const int qd = (TR && D3) ? (cls >> 2) & 1 : 0;
    const int qh = TR ? (cls >> 1) & 1 : 0;
    const int qw = TR ? cls & 1 : 0;

    // patch origin in input coordinates
    const int zo = D3 ? (TR ? zs + qd - 1 : zs * S - a.pd) : 0;
    const int ro = TR ? y0 + qh - 1 : y0 * S - a.ph;
    const int xo = TR ? x0 + qw - 1 : x0 * S - a.pw;

    const long long wcls = static_cast<long long>(cls) * C::TAPS * a.cin_pad * a.cout_pad;
    const int c_src0 = a.src[0].C;
    const int c_src1 = a.src[1].C;

    float rx[C::NX];
    floatx4 rw[C::NW];

    // ---- issue the global loads of one chunk into registers (all independent, in flight together)
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int k = 0; k < C::NX; ++k) {
            const int i = tid + k * kThreads;
            // channel of this wave-instruction: uniform by construction (RAW64 % 64 == 0)
            const int c = __builtin_amdgcn_readfirstlane(i / C::RAW64);
            const int cg = c0 + c;
            float v = 0.f;
            if (c < CC && cg < a.Cin) {  // wave-uniform: no loads for padding channels
                const int e = i - c * C::RAW64;
                const int z = e / (C::PR * C::PC);
                const int rem = e - z * (C::PR * C::PC);
                const int r = rem / C::PC;
                const int col = rem - r * C::PC;
                const int id = zo + z, ih = ro + r, iw = xo + col;
                const bool ok = e < C::RAW && ih >= 0 && ih < a.Hi && iw >= 0 && iw < a.Wi &&
                                (!D3 || (id >= 0 && id < a.Di));
                // one wave-uniform branch per source, each with its own constant-index kernarg
                // fields (a select between sources becomes a scratch lookup table in hipcc)
#pragma unroll
                for (int s = 0; s < ESM_MAX_SRC; ++s) {
                    const int lo = s == 0 ? 0 : (s == 1 ? c_src0 : c_src0 + c_src1);
                    if (s < a.nsrc && cg >= lo && cg - lo < a.src[s].C) {
                        const esm_src& sr = a.src[s];
                        const float* base = sr.ptr + b * sr.sb + (cg - lo) * sr.sc;
                        const int off = ok ? static_cast<int>((D3 ? id * sr.sd : 0) + ih * sr.sh) + iw : 0;
                        const float t = base[off];
                        v = ok ? t : 0.f;
                    }
                }
            }
            rx[k] = v;
        }
#pragma unroll
        for (int k = 0; k < C::NW; ++k) {
            const int i = tid + k * kThreads;  // float4 index into [tap][CC][CO/4]
            const int tap = i / (CC * C::CO / 4);
            const int rem = i - tap * (CC * C::CO / 4);
            const int c = rem / (C::CO / 4);
            const int q4 = rem - c * (C::CO / 4);
            const bool ok = i < C::TAPS * CC * C::CO / 4;
            const long long g = ok ? wcls + (static_cast<long long>(tap) * a.cin_pad + c0 + c) * a.cout_pad +
                                         (cob & ~3) + 4 * q4
                                   : 0;
            rw[k] = *reinterpret_cast<const floatx4*>(a.w + g);
        }
    };
    auto store_chunk = [&]() {
#pragma unroll
        for (int k = 0; k < C::NX; ++k) {
            const int i = tid + k * kThreads;
            const int c = i / C::RAW64;
            const int e = i - c * C::RAW64;
            if (c < CC && e < C::RAW) xs[c * C::PLANE + e] = rx[k];
        }
#pragma unroll
        for (int k = 0; k < C::NW; ++k) {
            const int i = tid + k * kThreads;
            if (i < C::TAPS * CC * C::CO / 4) {
                const int rowi = i / (C::CO / 4);  // tap*CC + c
                const int q4 = i - rowi * (C::CO / 4);
                *reinterpret_cast<floatx4*>(wl + rowi * C::WROW + 4 * q4) = rw[k];
            }
        }
    };

    floatx4 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
    float acc1 = 0.f;  // C1 path

    // one tap of the current chunk: CC/4 MFMA k-steps (or CC VALU FMAs on the C1 path)
    auto do_tap = [&](int tap) {
        const int td = tap / (C::KT * C::KT);
        const int th = (tap / C::KT) % C::KT;
        const int tw = tap % C::KT;
        const int zi = (D3 && TR) ? 1 - td : td;
        const int ri = TR ? row + 1 - th : row * S + th;
        if constexpr (C1) {
            const int ci = TR ? lane + 1 - tw : lane * S + tw;
#pragma unroll
            for (int c = 0; c < CC; ++c)
                acc1 += wl[(tap * CC + c) * C::WROW + (cob & 3)] * xs[c * C::PLANE + (zi * C::PR + ri) * C::PC + ci];
        } else {
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
    };

    load_chunk(0);
    __builtin_amdgcn_sched_barrier(0);
    for (int c0 = 0; c0 < a.Cin; c0 += CC) {
        __syncthreads();  // every wave is done reading the previous chunk
        store_chunk();
        __syncthreads();
        if (c0 + CC < a.Cin) load_chunk(c0 + CC);  // in flight during this chunk's math
        __builtin_amdgcn_sched_barrier(0);          // ... not sunk below it by the scheduler
        if constexpr (KS == 1) {
            // one row of KT taps per iteration: enough independent LDS reads to cover their latency
            // without hoisting the whole chunk's operands (which would exhaust the VGPRs)
#pragma unroll 1
            for (int tg = 0; tg < C::TAPS / C::KT; ++tg) {
#pragma unroll
                for (int tw = 0; tw < C::KT; ++tw) do_tap(tg * C::KT + tw);
            }
        } else {
#pragma unroll 2
            for (int tap = kpart; tap < C::TAPS; tap += KS) do_tap(tap);
        }
    }

    if constexpr (KS > 1) {  // add the K-split partial sums in a fixed order (deterministic)
        __syncthreads();
        constexpr int E = MT * NT * 4;
        if (kpart > 0) {
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        smem[(((kpart - 1) * C::TH + row) * E + (mt * NT + nt) * 4 + j) * 64 + lane] = acc[mt][nt][j];
        }
        __syncthreads();
        if (kpart > 0) return;
#pragma unroll
        for (int p = 1; p < KS; ++p)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                    for (int j = 0; j < 4; ++j)
                        acc[mt][nt][j] += smem[(((p - 1) * C::TH + row) * E + (mt * NT + nt) * 4 + j) * 64 + lane];
    }

    // ---------------------------------------------------------------- epilogue
    const int ys = y0 + row;  // sub-grid / output row of this wave
    if (ys >= Hs) return;
    const int oz = TR ? 2 * zs + qd : zs;
    const int oy = TR ? 2 * ys + qh : ys;
    if constexpr (C1) {
        const int xsub = x0 + lane;
        if (xsub < Ws) {
            const int ox = TR ? 2 * xsub + qw : xsub;
            conv_put(a, conv_finish(a, acc1, b, cob, oz, oy, ox), b, cob, oz, oy, ox);
        }
        return;
    } else {
        conv_store_tile<MT, NT>(a, acc, b, oz, oy, x0, Ws, TR, qw, cob, lane, conv_epi_const<MT>(a, cob, lane));
    }
}

template <bool D3, int K, int S, bool TR, int MT, int NT, bool C1, int KS>
int launch_cfg(const esm_conv_desc& a, hipStream_t s) {
    using C = Geo<D3, K, S, TR, MT, NT, C1, KS>;
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const long long tiles = static_cast<long long>((Ws + C::TW - 1) / C::TW) * ((Hs + C::TH - 1) / C::TH);
    const unsigned zc = C1 ? static_cast<unsigned>(a.Cout) : ceil_div(a.Cout, C::CO);
    dim3 grid(static_cast<unsigned>(tiles), a.B * Ds, zc * C::NCLS);
    if (tiles > 0x7fffffffLL || grid.y > 65535u || grid.z > 65535u) return arg_error("conv: grid too large");
    hipLaunchKernelGGL((conv_kernel<D3, K, S, TR, MT, NT, C1, KS>), grid, dim3(kThreads), 0, s, a);
    return check_launch("conv");
}

template <bool D3, int K, int S, bool TR, int MT, int KS>
int launch_nt(const esm_conv_desc& a, hipStream_t s, int nt) {
    if constexpr (Geo<D3, K, S, TR, MT, 4, false, KS>::OK)
        if (nt == 4) return launch_cfg<D3, K, S, TR, MT, 4, false, KS>(a, s);
    if constexpr (Geo<D3, K, S, TR, MT, 2, false, KS>::OK)
        if (nt >= 2) return launch_cfg<D3, K, S, TR, MT, 2, false, KS>(a, s);
    static_assert(Geo<D3, K, S, TR, MT, 1, false, KS>::OK, "narrowest conv tile must fit the LDS budget");
    return launch_cfg<D3, K, S, TR, MT, 1, false, KS>(a, s);
}

// Direct form: N tiles (1/2) and K-split (1/4) as requested; rows per workgroup so that the
// grid holds about 2048 waves (4 rows per wave at most, for L1 reuse of the tap rows).
template <bool D3, int K, int S, bool TR, int MT>
int launch_direct_sel(const esm_conv_desc& a, hipStream_t s, int nt, int ks, int rows_per_wave = 0) {
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const long long rows = static_cast<long long>(a.B) * Ds * Hs * ((Ws + 16 * nt - 1) / (16 * nt)) *
                           ceil_div(a.Cout, 16 * MT) * (TR ? (D3 ? 8 : 4) : 1);
    if (ks == 4) {
        return nt == 2 ? launch_direct<D3, K, S, TR, MT, 2, 4>(a, s, 1) : launch_direct<D3, K, S, TR, MT, 1, 4>(a, s, 1);
    }
    const long long per_wave = rows_per_wave > 0 ? rows_per_wave : rows / 2048;
    const int rb = 4 * static_cast<int>(per_wave < 1 ? 1 : (per_wave > 8 ? 8 : per_wave));
    return nt == 2 ? launch_direct<D3, K, S, TR, MT, 2, 1>(a, s, rb) : launch_direct<D3, K, S, TR, MT, 1, 1>(a, s, rb);
}

// Tile choice.  hint (esm_conv_desc.hint) forces one: NT | KS << 4 | C1 << 8 | DIRECT << 9 |
// ROWS << 10 (row-streaming form, conv_rows.h) | rows-per-wave << 12 (direct form) |
// C1T << 16 (VALU single-output-channel transposed form, conv_c1.h).
// Automatic: single-output-channel layers take the VALU path; everything the direct form can
// address takes it (fewest instructions per MFMA, no barriers), K-split when the grid is far
// below one wave per SIMD; the LDS-staged form covers the rest.
template <bool D3, int K, int S, bool TR>
int launch_geom(const esm_conv_desc& a, hipStream_t s) {
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int MT = a.Cout > 16 ? 2 : 1;
    if (a.hint & (1 << 16)) {  // VALU single-output-channel transposed form (conv_c1.h)
        if constexpr (TR) {
            if (convt_c1_ok(a)) return launch_convt_c1<D3>(a, s);
        }
        return arg_error("conv: c1-transposed hint not applicable");
    }
    if (a.hint & ~kHintXcd) {  // explicit tile (tuning sweeps, tests of every variant)
        const int hnt = a.hint & 15, hks = (a.hint >> 4) & 15, hc1 = (a.hint >> 8) & 1, hdir = (a.hint >> 9) & 1;
        const int hrw = (a.hint >> 12) & 15;  // direct form: rows per wave (0 = automatic)
        if ((a.hint >> 10) & 1) {  // row-streaming form
            if constexpr (!TR && S == 1 && (K & 1)) {
                if (MT == 1 ? rows_ok<D3, K, 1>(a) : rows_ok<D3, K, 2>(a))
                    return MT == 1 ? launch_rows<D3, K, 1>(a, s) : launch_rows<D3, K, 2>(a, s);
            }
            return arg_error("conv: row-streaming hint not applicable");
        }
        if ((hnt != 1 && hnt != 2 && hnt != 4) || (hks != 1 && hks != 4)) return arg_error("conv: bad tile hint");
        if (hdir) {
            if (hc1 || hnt == 4 || !direct_ok(a)) return arg_error("conv: direct hint not applicable");
            return MT == 1 ? launch_direct_sel<D3, K, S, TR, 1>(a, s, hnt, hks, hrw)
                           : launch_direct_sel<D3, K, S, TR, 2>(a, s, hnt, hks, hrw);
        }
        if (hc1) {
            if (D3 || a.Cout > 2 || a.shuffle > 1 || hnt != 4 || hks != 1) return arg_error("conv: C1 hint not applicable");
            return launch_cfg<D3, K, S, TR, 1, 4, true, 1>(a, s);
        }
        if (hks == 4) return MT == 1 ? launch_nt<D3, K, S, TR, 1, 4>(a, s, hnt) : launch_nt<D3, K, S, TR, 2, 4>(a, s, hnt);
        return MT == 1 ? launch_nt<D3, K, S, TR, 1, 1>(a, s, hnt) : launch_nt<D3, K, S, TR, 2, 1>(a, s, hnt);
    }
    // single-output-channel transposed layers (the hourglasses' last decoder step): VALU form
    if constexpr (TR) {
        if (convt_c1_ok(a)) return launch_convt_c1<D3>(a, s);
    }
    // row-streaming form for stride-1 layers with horizontal taps to share (1x1 layers measured
    // faster in the direct form)
    if constexpr (!TR && S == 1 && (K & 1) && K >= 3) {
        if (MT == 1 ? rows_ok<D3, K, 1>(a) : rows_ok<D3, K, 2>(a))
            return MT == 1 ? launch_rows<D3, K, 1>(a, s) : launch_rows<D3, K, 2>(a, s);
    }
    // single-output-channel layers the direct form cannot take: VALU path
    if (!D3 && a.Cout <= 2 && Ws >= 64 && a.shuffle <= 1 && !direct_ok(a))
        return launch_cfg<D3, K, S, TR, 1, 4, true, 1>(a, s);
    constexpr int TAPS = (TR ? 2 : K) * (TR ? 2 : K) * (D3 ? (TR ? 2 : K) : 1);
    const long long per = static_cast<long long>(a.B) * Ds * ceil_div(a.Cout, 16 * MT) * (TR ? (D3 ? 8 : 4) : 1);
    const long long rows1 = per * Hs * ((Ws + 15) / 16);  // 16-pixel row segments
    if (direct_ok(a)) {
        // sweep-fitted (profiles/r01_conv_sweep*.txt): two N tiles pay off for concatenated 1x1
        // inputs and for wide-input, narrow-output 3-D layers; tiny grids split the taps
        const int ks = (TAPS >= 8 && rows1 < 256) ? 4 : 1;
        const int nt = (ks == 1 && ((K == 1 && a.nsrc > 1) || (D3 && a.Cin >= 32 && a.Cout <= 16))) ? 2 : 1;
        return MT == 1 ? launch_direct_sel<D3, K, S, TR, 1>(a, s, nt, ks) : launch_direct_sel<D3, K, S, TR, 2>(a, s, nt, ks);
    }
    // LDS-staged form; rules fitted to scripts/conv_sweep.py on MI355X (profiles/r01_conv_sweep.txt)
    const long long b1 = per * ((Hs + 3) / 4) * ((Ws + 15) / 16);
    int nt = 1;
    if (!D3 && a.Cin <= 4 && Ws >= 64) nt = 4;
    else if (b1 >= 8192 && a.cin_pad >= 32) nt = 2;
    const bool ksplit = TAPS >= 8 && b1 < 300;
    if (ksplit) return MT == 1 ? launch_nt<D3, K, S, TR, 1, 4>(a, s, 1) : launch_nt<D3, K, S, TR, 2, 4>(a, s, 1);
    return MT == 1 ? launch_nt<D3, K, S, TR, 1, 1>(a, s, nt) : launch_nt<D3, K, S, TR, 2, 1>(a, s, nt);
}

}  // namespace conv
}  // namespace esm
