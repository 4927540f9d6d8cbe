// Row-streaming implicit-GEMM convolution for stride-1, non-transposed layers (2-D and 3-D)
// on the gfx950 fp32 matrix cores — the form most of the hot path's layers take (3x3 / 3x3x3
// BasicConv bodies, the 1x1 agg / to_feat convs, the 5x5 disparity heads).  Included by
// conv2d.hip / conv3d.hip; launch_geom (conv_impl.h) picks it when it applies.
//
// Reference layers: BasicConv (models/submodule.py:12-38) in models/ESMStereo.py:129-509,
// 610-622 and the convs of models/shufflemixer.py:124-126.
//
// Why: measured per-wave timelines of the direct form (scripts/probes/wave_timeline.py) show a
// wave living ~6.5 us for one 16-pixel row: ~1.3 us of setup, a K loop waiting on 72 loads, and
// only 3 waves per SIMD resident (140 registers).  Here:
//   * B (4 channels x 16 columns) is ONE buffer_load per (tap row, k-step): lanes hold 16
//     consecutive input columns and the K-1 horizontal taps are DPP row shifts of that value
//     (row_shl / row_shr within each 16-lane row), so a tile yields 16-(K-1) output columns
//     and needs no side or edge loads — 3x fewer loads than the direct form for 3x3;
//   * A (weights of the workgroup's 16*MT couts, all taps and channels) is staged in LDS once
//     per workgroup and read per MFMA with a conflict-free ds_read_b32;
//   * each wave walks RW rows (the 4 waves of a workgroup interleave), issuing the next row's B
//     loads before the current row's MFMAs, so load latency overlaps compute and the setup is
//     paid once per wave.
// Out-of-range columns / rows / channels read as zeros through the buffer range check (kOOB
// marks in voffset / soffset, as in conv_direct.h).
#pragma once

#include "conv_direct.h"

namespace esm {
namespace conv {

// v from lane (l & ~15) + ((l & 15) + d) of the same 16-lane row; lanes shifted past the row read 0
template <int D>
__device__ __forceinline__ float row_shift(float v) {
    if constexpr (D == 0) {
        return v;
    } else {
        constexpr int ctrl = D > 0 ? (0x100 + D) : (0x110 - D);  // row_shl:D / row_shr:-D
        return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xf, 0xf, true));
    }
}

template <bool D3, int K, int MT>
struct RGeo {
    static constexpr int KDT = D3 ? K : 1;
    static constexpr int TAPS = KDT * K * K;
    static constexpr int VALID = 16 - (K - 1);  // output columns per 16-lane tile
    static constexpr int A0 = K / 2;            // lane of the tile's first output column = anchor tap
    static constexpr int WROW = MT == 1 ? 16 : 48;  // LDS weight row (48: lanes 16-31 off by 16 banks)
};

// bytes of LDS the weight slab of one workgroup needs
template <bool D3, int K, int MT>
constexpr long long rows_lds_bytes(int cin_pad) {
    return 4LL * RGeo<D3, K, MT>::TAPS * cin_pad * RGeo<D3, K, MT>::WROW;
}

template <bool D3, int K, int MT, int CK>
__global__ void __launch_bounds__(kDirectThreads) rconv_kernel(const esm_conv_desc a) {
    using G = RGeo<D3, K, MT>;
    constexpr int KDT = G::KDT, TAPS = G::TAPS, VALID = G::VALID, A0 = G::A0, WROW = G::WROW;
    constexpr int NB = KDT * K * CK;  // B values of one output row (per tap row and k-step)
    constexpr int NC = MT >= 2 ? 2 : 4;  // independent accumulation chains per tile
    extern __shared__ float wl[];  // [TAPS][cin_pad][WROW]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15;
    const int kq = lane >> 4;
    const int Hs = a.Ho, Ws = a.Wo;
    const int Ds = D3 ? a.Do : 1;
    const int RB = a.hint;  // rows per workgroup (launcher)
    const int tiles_w = (Ws + VALID - 1) / VALID;
    const int tiles_h = (Hs + RB - 1) / RB;
    // XCD-aware tile order (see conv_direct.h)
    const unsigned nwg = gridDim.x, orig = blockIdx.x;
    const unsigned q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    unsigned wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
    const int tx = static_cast<int>(wg % tiles_w);
    wg /= tiles_w;
    const int ty = static_cast<int>(wg % tiles_h);
    wg /= tiles_h;
    const int bz = static_cast<int>(wg % (a.B * Ds));
    const int cob = static_cast<int>(wg / (a.B * Ds)) * 16 * MT;
    const int b = bz / Ds;
    const int zs = bz - b * Ds;
    const int o0 = tx * VALID;          // first output column of the tile
    const int xin0 = o0 - a.pw;         // input column held by lane 0 (output o0 sits at lane A0)

    // ---- the single source (multi-source layers use the direct form)
    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (D3 ? (a.Di - 1) * sd : 0) + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const int xi = xin0 + n16;
    const unsigned xoffb = (xi >= 0 && xi < a.Wi) ? 4u * xi : kOOB;

    const int y_end = min(Hs, ty * RB + RB);
    const int y_first = ty * RB + wave;

    // B loads of one output row (the single channel chunk), into bv[(td*K + th)*CK + k]
    auto load_row = [&](float (&bv)[NB], int ys, int cc) {
        const bool yok = ys < y_end;
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            const int cl = cc + 4 * k + kq;
            const unsigned vo = (cl < a.Cin ? 4u * cl * sc : kOOB) + xoffb;
#pragma unroll
            for (int td = 0; td < KDT; ++td)
#pragma unroll
                for (int th = 0; th < K; ++th) {
                    const int zi = D3 ? zs - a.pd + td : 0;
                    const int yi = ys - a.ph + th;
                    const bool rok = yok && yi >= 0 && yi < a.Hi && (!D3 || (zi >= 0 && zi < a.Di));
                    const int roff = rok ? 4 * ((D3 ? zi * sd : 0) + yi * sh) : static_cast<int>(kOOB);
                    bv[(td * K + th) * CK + k] = buf_load_s(rs, vo, roff);
                }
        }
    };

    // the first row's operands are requested before the weight staging and its barrier, so the
    // two memory round trips overlap
    float bcur[NB];
    load_row(bcur, y_first, 0);
    const EpiConst<MT> ec = conv_epi_const<MT>(a, cob, lane);
    // weights of this workgroup's couts -> LDS (once): cin_pad is 16 on this form (rows_ok), so the
    // count is a compile-time constant and every load is issued before the first LDS store
    {
        constexpr int N4 = TAPS * 16 * (16 * MT / 4);  // float4 count
        constexpr int R4 = (N4 + kDirectThreads - 1) / kDirectThreads;
        floatx4 rw[R4];
#pragma unroll
        for (int k = 0; k < R4; ++k) {
            const int i = min(static_cast<int>(threadIdx.x) + k * kDirectThreads, N4 - 1);  // clamped: no branch
            const int row = i / (4 * MT);  // tap * 16 + c
            const int q4 = i - row * (4 * MT);
            rw[k] = *reinterpret_cast<const floatx4*>(a.w + static_cast<long long>(row) * a.cout_pad + cob + 4 * q4);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < R4; ++k) {
            const int i = threadIdx.x + k * kDirectThreads;
            const int row = i / (4 * MT);
            const int q4 = i - row * (4 * MT);
            if (i < N4) *reinterpret_cast<floatx4*>(wl + row * WROW + 4 * q4) = rw[k];
        }
    }

    __syncthreads();
    for (int ys = y_first; ys < y_end; ys += 4) {
        float bnext[NB];
        load_row(bnext, ys + 4, 0);  // next row's operands in flight during this row's MFMAs
        // keep every load of the next row above this row's MFMAs: left alone the scheduler sinks
        // each load next to its use and the wave pays one memory round trip per load
        __builtin_amdgcn_sched_barrier(0);

        floatx4 accs[NC][MT];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) accs[c][mt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int td = 0; td < KDT; ++td)
#pragma unroll
            for (int th = 0; th < K; ++th)
#pragma unroll
                for (int k = 0; k < CK; ++k) {
                    const float v = bcur[(td * K + th) * CK + k];
#pragma unroll
                    for (int tw = 0; tw < K; ++tw) {
                        float bs;
                        if constexpr (K == 1) bs = v;
                        else if (tw == A0) bs = v;
                        else if (tw == A0 - 1) bs = row_shift<-1>(v);
                        else if (tw == A0 + 1) bs = row_shift<1>(v);
                        else if (tw == A0 - 2) bs = row_shift<-2>(v);
                        else bs = row_shift<2>(v);
                        const int tap = (td * K + th) * K + tw;
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt) {
                            const float av = wl[(tap * a.cin_pad + 4 * k + kq) * WROW + mt * 16 + n16];
                            floatx4& acc = accs[(tap * CK + k) % NC][mt];
                            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bs, acc, 0, 0, 0);
                        }
                    }
                }
        floatx4 acc[MT][1];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            acc[mt][0] = accs[0][mt];
#pragma unroll
            for (int c = 1; c < NC; ++c) acc[mt][0] += accs[c][mt];  // fixed order (deterministic)
        }
        // lane n16 holds output column o0 + n16 - A0 (stored for n16 in [A0, A0 + VALID))
        conv_store_tile<MT, 1>(a, acc, b, zs, ys, o0 - A0, min(Ws, o0 + VALID), false, 0, cob, lane, ec, o0);
#pragma unroll
        for (int i = 0; i < NB; ++i) bcur[i] = bnext[i];
    }
}

template <bool D3, int K, int MT>
int launch_rows(const esm_conv_desc& a, hipStream_t s) {
    using G = RGeo<D3, K, MT>;
    const int Hs = a.Ho, Ws = a.Wo;
    const int Ds = D3 ? a.Do : 1;
    const long long tiles_w = (Ws + G::VALID - 1) / G::VALID;
    const long long rows = static_cast<long long>(a.B) * Ds * Hs * tiles_w * ceil_div(a.Cout, 16 * MT);
    // rows per wave: enough waves to fill the chip (~4 per SIMD), at most 8 rows each
    const long long want = rows / 4096;
    const int rw = static_cast<int>(want < 1 ? 1 : (want > 8 ? 8 : want));
    const int rb = 4 * rw;
    esm_conv_desc d = a;
    d.hint = rb;
    const long long nwg = tiles_w * ((Hs + rb - 1) / rb) * a.B * Ds * ceil_div(a.Cout, 16 * MT);
    if (nwg > 0x7fffffffLL) return arg_error("conv: grid too large");
    const size_t lds = static_cast<size_t>(rows_lds_bytes<D3, K, MT>(a.cin_pad));
    const int ck = a.Cin <= 4 ? 1 : (a.Cin <= 8 ? 2 : 4);
    if (ck == 1)
        hipLaunchKernelGGL((rconv_kernel<D3, K, MT, 1>), dim3(static_cast<unsigned>(nwg)), dim3(kDirectThreads), lds, s, d);
    else if (ck == 2)
        hipLaunchKernelGGL((rconv_kernel<D3, K, MT, 2>), dim3(static_cast<unsigned>(nwg)), dim3(kDirectThreads), lds, s, d);
    else
        hipLaunchKernelGGL((rconv_kernel<D3, K, MT, 4>), dim3(static_cast<unsigned>(nwg)), dim3(kDirectThreads), lds, s, d);
    return check_launch("conv(rows)");
}

// The row-streaming form applies to single-source stride-1 convs with at most 16 input channels
// (one channel chunk: the row pipeline keeps one row's operands live), odd K <= 5, and a
// weight slab that fits 64 KiB of LDS.
template <bool D3, int K, int MT>
bool rows_ok(const esm_conv_desc& a) {
    return !a.transposed && a.stride == 1 && (K & 1) && K <= 5 && a.nsrc == 1 && a.Cin <= 16 &&
           rows_lds_bytes<D3, K, MT>(a.cin_pad) <= 64 * 1024 && direct_ok(a);
}

}  // namespace conv
}  // namespace esm
