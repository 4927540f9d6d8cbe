// Fused ESM upsampling head: Conv2d 1x1 (nf -> nf*r*r, bias) -> PixelShuffle(r) -> SiLU ->
// Conv2d 3x3 (nf -> 1, pad 1, bias), i.e. `upsampling{2,4}` followed by `tail{2x,4x}` of the
// ESM upsamplers (models/ESMStereo.py:264-271,290-296 upsample4; :363-407 upsample8;
// :455-500 upsample16; forward :301-302,311-312 and the like).
//
// The shuffled nf-channel map at r x the input resolution (S at KITTI: 8 x 384 x 1248 fp32,
// 15 MB) is never written: a workgroup owns a TH x 64 tile of the 1-channel output, stages the
// low-resolution input pixels under the tile plus a one-pixel halo and every weight in LDS with
// one batch of loads, builds the shuffled tile + halo in LDS (a thread takes one channel of one
// low-resolution pixel and produces its r*r sub-pixels, so the 1x1 weights are wave-uniform
// LDS broadcasts), then runs the 3x3 conv from LDS, 4 consecutive outputs per thread and one
// 16-byte store.  Arithmetic per element is the unfused order: bias + sum_i w*x, SiLU, then
// bias + sum over (channel, ky, kx) of w*v.
#include "conv_direct.h"

typedef float f2v __attribute__((ext_vector_type(2)));

namespace esm {
namespace {

constexpr int kThreads = 256;

template <int NF, int R, int TH, int kTW>
struct StGeo {
    static constexpr int LRH = TH / R + 2;  // low-res rows under tile + halo
    static constexpr int LRW = kTW / R + 2;
    // nf = 8, r = 4 (ESMStereo-S) builds the shuffled tile with MFMA: each low-res pixel's 4x4
    // sub-pixels land as 4 aligned columns, so its tile spans the whole low-res window (origin X0 - 4)
    // (round 6: nf = 16, r = 2, ESMStereo-L, likewise: each low-res pixel's 2x2 sub-pixels as 2 aligned columns)
    static constexpr bool MF = (NF == 8 && R == 4) || (NF == 16 && R == 2);
    static constexpr int MX0 = MF ? R : 1;  // tile column 0 = output column X0 - MX0
    static constexpr int MH = TH + 2, MW = MF ? LRW * R : kTW + 2, MWP = MF ? MW : MW + 2;  // 16-B aligned rows
    static constexpr int NUP = NF * R * R;
    static constexpr int WN = NUP * NF + NUP + NF * 9 + 1;  // up_w, up_b, tail_w, tail_b
    static constexpr int XN = NF * LRH * LRW;
    static constexpr int PIX = LRH * LRW;
    static constexpr int PIXP = (PIX + 63) / 64 * 64;  // items per channel, padded to whole waves
};

template <int NF, int R, int TH, int kTW>
__global__ void __launch_bounds__(kThreads) shuffle_tail_kernel(const esm_shuffle_tail_desc a) {
    using G = StGeo<NF, R, TH, kTW>;
    constexpr int LRH = G::LRH, LRW = G::LRW, MH = G::MH, MW = G::MW, MWP = G::MWP, PIX = G::PIX, PIXP = G::PIXP;
    constexpr int MX0 = G::MX0;
    constexpr int NUP = G::NUP, WN = G::WN, XN = G::XN;
    constexpr int WR = (WN + kThreads - 1) / kThreads;
    constexpr int XR = (XN + kThreads - 1) / kThreads;
    __shared__ __attribute__((aligned(16))) float wsh[WN];
    __shared__ float lr[NF][LRH][LRW];
    __shared__ __attribute__((aligned(16))) float mid[NF][MH][MWP];

    const int tid = threadIdx.x;
    const int H = a.H, W = a.W, HO = H * R, WO = W * R;
    const Blk3 bk_ = xcd_block((a.flags & 1) != 0);
    const int b = bk_.z;
    const int Y0 = bk_.y * TH, X0 = bk_.x * kTW;
    const int ly0 = Y0 / R - 1, lx0 = X0 / R - 1;  // low-res pixel of lr[.][0][0]
    const float* xb = a.x + b * a.xb;

    // ---- stage (one round trip): weights and the low-res tile
    float rw[WR], rx[XR];
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        const int i = tid + k * kThreads;
        const float* p = i < NUP * NF ? a.up_w : i < NUP * NF + NUP ? a.up_b : i < WN - 1 ? a.tail_w : a.tail_b;
        const int off = i < NUP * NF ? i : i < NUP * NF + NUP ? i - NUP * NF : i < WN - 1 ? i - NUP * NF - NUP : 0;
        // unconditional load (clamped offset) then select: a conditional load makes hipcc branch
        // around it and wait for each one separately
        const float* q = p ? p : a.up_w;
        const float v = q[i < WN && p ? off : 0];
        rw[k] = (i < WN && p) ? v : 0.f;
    }
#pragma unroll
    for (int k = 0; k < XR; ++k) {
        const int i = tid + k * kThreads;
        const int c = i / (LRH * LRW);
        const int rem = i - c * LRH * LRW;
        const int yy = ly0 + rem / LRW, xx = lx0 + rem % LRW;
        const bool ok = i < XN && yy >= 0 && yy < H && xx >= 0 && xx < W;
        const float v = xb[ok ? c * a.xc + yy * a.xh + xx : 0];
        rx[k] = ok ? v : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
    for (int k = 0; k < WR; ++k)
        if (tid + k * kThreads < WN) wsh[tid + k * kThreads] = rw[k];
#pragma unroll
    for (int k = 0; k < XR; ++k)
        if (tid + k * kThreads < XN) (&lr[0][0][0])[tid + k * kThreads] = rx[k];
    __syncthreads();

    // ---- shuffled tile: item = (channel c, low-res pixel), channel-major with each channel's
    //      items padded to whole waves, so c (and every 1x1 weight a wave reads) is wave-uniform
    const float* upw = wsh;
    const float* upb = wsh + NUP * NF;
    const float* tw = wsh + NUP * NF + NUP;
    const float tb = a.tail_b ? wsh[WN - 1] : 0.f;
    if constexpr (G::MF && R == 2) {
        // nf = 16, r = 2 (ESMStereo-L's heads, round 6): the 1x1 as MFMA, M = the 64 up-channels (wave w: tile
        // 16 w .. 16 w + 15 = channels 4w .. 4w + 3 x their 2x2 sub-pixels), N = 16 low-res pixels, K = the 16
        // input channels (4 k-steps).  Lane (g, n) receives up-channels 16 w + 4 g + j, i.e. channel 4 w + g,
        // sub-pixel (j / 2, j % 2) of low-res pixel n: two 8-byte LDS stores.  (The VALU loop it replaces did
        // 64 FMAs per item with wave-uniform LDS weight reads: 110 us of the L-K B = 4 step's 4x head.)
        typedef float f32x2 __attribute__((ext_vector_type(2)));
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int lane = tid & 63, g = lane >> 4, n = lane & 15;
        float av[4], bias[4];
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) av[kk] = upw[(wave * 16 + n) * NF + 4 * kk + g];
#pragma unroll
        for (int j = 0; j < 4; ++j) bias[j] = upb[wave * 16 + 4 * g + j];
        const int c = 4 * wave + g;
        const float* lrf = &lr[0][0][0];
#pragma unroll 1
        for (int nt = 0; nt < (PIX + 15) / 16; ++nt) {
            const int p = nt * 16 + n;
            const bool pin = p < PIX;
            const int py = p / LRW, px = p - (p / LRW) * LRW;
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[kk], lrf[(4 * kk + g) * PIX + (pin ? p : 0)], acc, 0, 0, 0);
            const int X = (lx0 + px) * R;  // sub-pixel column 0
#pragma unroll
            for (int sy = 0; sy < 2; ++sy) {
                const int Y = (ly0 + py) * R + sy;
                const int my = Y - (Y0 - 1);
                const bool yok = Y >= 0 && Y < HO;
                f32x2 o;
#pragma unroll
                for (int sx = 0; sx < 2; ++sx) {
                    const float v = silu_fast(acc[2 * sy + sx] + bias[2 * sy + sx]);
                    o[sx] = (yok && X + sx >= 0 && X + sx < WO) ? v : 0.f;  // zero padding of the 3x3 tail
                }
                if (pin && my >= 0 && my < MH) *reinterpret_cast<f32x2*>(&mid[c][my][px * R]) = o;
            }
        }
    } else if constexpr (G::MF) {
        // 1x1 conv as MFMA: M = the 16 sub-pixels (sy, sx) of one channel c, N = 16 low-res pixels,
        // K = the 8 input channels (2 k-steps).  Lane (g, n) gets sub-pixel row sy = g, columns
        // sx = 0..3 of low-res pixel n: one 16-byte LDS store per lane.  Wave w: channels 2w, 2w+1.
        const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
        const int lane = tid & 63, g = lane >> 4, n = lane & 15;
        float av[2][2], bias[2][4];
#pragma unroll
        for (int ci = 0; ci < 2; ++ci) {
            const int c = 2 * wave + ci;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) av[ci][kk] = upw[(c * 16 + n) * NF + 4 * kk + g];
#pragma unroll
            for (int j = 0; j < 4; ++j) bias[ci][j] = upb[c * 16 + 4 * g + j];
        }
        const float* lrf = &lr[0][0][0];
#pragma unroll 1
        for (int nt = 0; nt < (PIX + 15) / 16; ++nt) {
            const int p = nt * 16 + n;
            const bool pin = p < PIX;
            const int py = p / LRW, px = p - (p / LRW) * LRW;
            float bk[2];
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) bk[kk] = lrf[(4 * kk + g) * PIX + (pin ? p : 0)];
            const int Y = (ly0 + py) * R + g;
            const int my = Y - (Y0 - 1);
            const bool yok = Y >= 0 && Y < HO;
            const int X = (lx0 + px) * R;  // sub-pixel column 0
#pragma unroll
            for (int ci = 0; ci < 2; ++ci) {
                conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ci][0], bk[0], acc, 0, 0, 0);
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ci][1], bk[1], acc, 0, 0, 0);
                conv::floatx4 o;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = silu_fast(acc[j] + bias[ci][j]);
                    o[j] = (yok && X + j >= 0 && X + j < WO) ? v : 0.f;  // zero padding of the 3x3 tail
                }
                if (pin && my >= 0 && my < MH)
                    *reinterpret_cast<conv::floatx4*>(&mid[2 * wave + ci][my][px * R]) = o;
            }
        }
    } else {
    for (int i = tid; i < NF * PIXP; i += kThreads) {
        const int c = __builtin_amdgcn_readfirstlane(i / PIXP);
        const int rem = i - c * PIXP;
        if (rem >= PIX) continue;
        const int py = rem / LRW, px = rem - (rem / LRW) * LRW;
        float xv[NF];
#pragma unroll
        for (int j = 0; j < NF; ++j) xv[j] = lr[j][py][px];
#pragma unroll
        for (int sy = 0; sy < R; ++sy)
#pragma unroll
            for (int sx = 0; sx < R; ++sx) {
                // shuffled output position, in tile coordinates (tile row 0 = output row Y0 - 1)
                const int Y = (ly0 + py) * R + sy, X = (lx0 + px) * R + sx;
                const int my = Y - (Y0 - 1), mx = X - (X0 - MX0);
                if (my < 0 || my >= MH || mx < 0 || mx >= MW) continue;
                float v = 0.f;  // zero padding of the 3x3 conv outside the shuffled map
                if (Y >= 0 && Y < HO && X >= 0 && X < WO) {
                    const float* wr = upw + (c * R * R + sy * R + sx) * NF;  // wave-uniform row
                    float s = 0.f;
#pragma unroll
                    for (int j = 0; j < NF; ++j) s += wr[j] * xv[j];
                    v = silu_fast(s + upb[c * R * R + sy * R + sx]);
                }
                mid[c][my][mx] = v;
            }
    }
    }
    __syncthreads();

    // ---- 3x3 tail: thread (row, QW consecutive columns), QW chosen so the tile's items fill the
    //      workgroup (16 x 32: 2 columns per thread on all 4 waves, not 4 on two of them)
    constexpr int QW = TH * kTW >= 4 * kThreads ? 4 : (TH * kTW >= 2 * kThreads ? 2 : 1);
    constexpr int QPR = kTW / QW;  // items per row
    const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc(a.out + b * a.ob, static_cast<short>(0),
                                                                         0x7fffffff, 0x00020000);
    for (int q = tid; q < TH * QPR; q += kThreads) {
        const int r = q / QPR, g = q - (q / QPR) * QPR;
        const int oy = Y0 + r, ox = X0 + QW * g;
        float acc[QW];
#pragma unroll
        for (int j = 0; j < QW; ++j) acc[j] = 0.f;
#pragma unroll 2
        for (int c = 0; c < NF; ++c) {
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                float v[QW + 2];
#pragma unroll
                for (int j = 0; j < QW + 2; ++j) v[j] = mid[c][r + ky][QW * g + j + MX0 - 1];
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float w = tw[(c * 3 + ky) * 3 + kx];
#pragma unroll
                    for (int j = 0; j < QW; ++j) acc[j] += w * v[j + kx];
                }
            }
        }
        if (oy >= HO) continue;
        const int vo = static_cast<int>(4 * (static_cast<long long>(oy) * a.oh + ox));
        if (ox + QW - 1 < WO && ((reinterpret_cast<uintptr_t>(a.out + b * a.ob) + vo) & (4 * QW - 1)) == 0) {
            // write-through (sc1) vector store (conv_direct.h kStoreAux)
            if constexpr (QW == 4) {
                typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
                __builtin_amdgcn_raw_buffer_store_b128(
                    u32x4{__float_as_uint(acc[0] + tb), __float_as_uint(acc[1] + tb), __float_as_uint(acc[2] + tb),
                          __float_as_uint(acc[3] + tb)},
                    rso, vo, 0, conv::kStoreAux);
            } else if constexpr (QW == 2) {
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(acc[0] + tb), __float_as_uint(acc[1] + tb)},
                                                      rso, vo, 0, conv::kStoreAux);
            } else {
                conv::store_b32(__float_as_uint(acc[0] + tb), rso, vo, 0);
            }
        } else {
            float* o = a.out + b * a.ob + static_cast<long long>(oy) * a.oh + ox;
#pragma unroll
            for (int j = 0; j < QW; ++j)
                if (ox + j < WO) o[j] = acc[j] + tb;
        }
    }
}

// ---------------------------------------------------------------------------------------------
// nf = 8, r = 4 (ESMStereo-S, both heads; the 4x head is the S-K step's largest launch): a workgroup of
// L waves owns L low-resolution rows x 16 low-resolution pixels = a (4L) x 64 output tile.  Wave w
// builds the shuffled map of low-res row w with MFMA (M = the 16 sub-pixels (sy, sx) of one channel,
// N = the 16 low-res pixels, K = the 8 input channels): lane (g, n) receives sub-row g, sub-columns
// 0..3 of pixel n, SiLU'd and stored to LDS as one 16-byte write.  Only the one-pixel ring the 3x3 tail
// needs around the tile (the sub-row above / below, the sub-column left / right) is computed on top,
// on the VALU: 2 (4L + 2) + 2 * 64 values per channel, against the (L + 2) x 18 low-res window's 1.6-1.9x
// of the previous form.  The tail then runs with lane (g, n) of wave w producing the 4 outputs it built
// (row 4w + g, columns 4n .. 4n + 3), reading each (channel, tap row) as one 16-byte + two 4-byte LDS
// reads, and stores them with one 16-byte write-through store.
template <int L>
struct St4Geo {
    static constexpr int NF = 8, R = 4;
    static constexpr int TR = 4 * L, TC = 64;           // output tile
    static constexpr int SR = TR + 2, SC = 72;          // shuffled tile: row 0 = Y0 - 1, col 4 = X0 (cols 3..68 used)
    static constexpr int LH = L + 2, LW = 18;           // low-res window: rows ly0 - 1 .., cols lx0 - 1 ..
    static constexpr int OW_UB = 128 * NF, OW_TW = OW_UB + 128, OW_TB = OW_TW + NF * 9, WN = OW_TB + 1;
    static constexpr int XN = NF * LH * LW;
    static constexpr int HALO = 2 * SC - 2 * 3 /* cols 3..68 on the two ring rows */ + 2 * TR;
};

template <int L>
__global__ void __launch_bounds__(64 * L) shuffle_tail4_kernel(const esm_shuffle_tail_desc a) {
    using G = St4Geo<L>;
    constexpr int NF = G::NF, SR = G::SR, SC = G::SC, LH = G::LH, LW = G::LW, WN = G::WN, XN = G::XN, NT = 64 * L;
    __shared__ __attribute__((aligned(16))) float wsh[WN];
    __shared__ float lr[NF][LH][LW];
    __shared__ __attribute__((aligned(16))) float sh[NF][SR][SC];

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, HO = 4 * H, WO = 4 * W;
    const Blk3 bk_ = xcd_block((a.flags & 1) != 0);
    const int b = bk_.z;
    const int ly0 = bk_.y * L, lx0 = bk_.x * 16;  // first low-res row / pixel of the tile
    const int Y0 = 4 * ly0, X0 = 4 * lx0;
    const float* xb = a.x + b * a.xb;

    // ---- stage (one round trip): every weight and the low-res window
    constexpr int WRN = (WN + NT - 1) / NT, XRN = (XN + NT - 1) / NT;
    float rw[WRN], rx[XRN];
#pragma unroll
    for (int k = 0; k < WRN; ++k) {
        const int i = tid + k * NT;
        const float* p = i < G::OW_UB ? a.up_w : i < G::OW_TW ? a.up_b : i < G::OW_TB ? a.tail_w : a.tail_b;
        const int off = i < G::OW_UB ? i : i < G::OW_TW ? i - G::OW_UB : i < G::OW_TB ? i - G::OW_TW : 0;
        const bool ok = i < WN && p != nullptr;
        const float v = (ok ? p : a.up_w)[ok ? off : 0];
        rw[k] = ok ? v : 0.f;
    }
#pragma unroll
    for (int k = 0; k < XRN; ++k) {
        const int i = tid + k * NT;
        const int c = i / (LH * LW), rem = i - c * (LH * LW);
        const int yy = ly0 - 1 + rem / LW, xx = lx0 - 1 + rem % LW;
        const bool ok = i < XN && yy >= 0 && yy < H && xx >= 0 && xx < W;
        const float v = xb[ok ? c * a.xc + yy * a.xh + xx : 0];
        rx[k] = ok ? v : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
    for (int k = 0; k < WRN; ++k)
        if (tid + k * NT < WN) wsh[tid + k * NT] = rw[k];
#pragma unroll
    for (int k = 0; k < XRN; ++k)
        if (tid + k * NT < XN) (&lr[0][0][0])[tid + k * NT] = rx[k];
    __syncthreads();

    // ---- interior: wave w = low-res row ly0 + w, 8 channels x 2 MFMA k-steps
    {
        const int Y = Y0 + 4 * wave + g;  // lane's output row
        const int Xl = X0 + 4 * n;        // lane's first output column
        float bk[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) bk[kk] = lr[4 * kk + g][wave + 1][n + 1];
#pragma unroll
        for (int c = 0; c < NF; ++c) {
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wsh[(c * 16 + n) * NF + 4 * kk + g], bk[kk], acc, 0, 0, 0);
            conv::floatx4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = silu_fast(acc[j] + wsh[G::OW_UB + c * 16 + 4 * g + j]);
                o[j] = (Y < HO && Xl + j < WO) ? v : 0.f;  // zero padding of the 3x3 tail
            }
            *reinterpret_cast<conv::floatx4*>(&sh[c][1 + 4 * wave + g][4 + 4 * n]) = o;
        }
    }
    // ---- the ring (VALU): ring rows 0 and SR - 1 over cols 3..68, then ring cols 3 and 68 over rows 1..TR
    auto ring_value = [&](int c, int tr, int tc) __attribute__((always_inline)) {
        const int Y = Y0 - 1 + tr, X = X0 - 4 + tc;
        float v = 0.f;
        if (Y >= 0 && Y < HO && X >= 0 && X < WO) {
            const int py = (Y >> 2) - (ly0 - 1), px = (X >> 2) - (lx0 - 1);  // in the low-res window
            const int m = c * 16 + (Y & 3) * 4 + (X & 3);
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < NF; ++k) acc += wsh[m * NF + k] * lr[k][py][px];
            v = silu_fast(acc + wsh[G::OW_UB + m]);
        }
        sh[c][tr][tc] = v;
    };
    constexpr int RROW = SC - 6;  // 66 columns per ring row
    for (int i = tid; i < NF * 2 * RROW; i += NT) {
        const int c = i / (2 * RROW), q = i - c * (2 * RROW);
        const int bot = q >= RROW;
        ring_value(c, bot ? SR - 1 : 0, 3 + q - bot * RROW);
    }
    for (int i = tid; i < NF * 2 * G::TR; i += NT) {
        const int c = i / (2 * G::TR), q = i - c * (2 * G::TR);
        const int right = q >= G::TR;
        ring_value(c, 1 + q - right * G::TR, right ? 68 : 3);
    }
    __syncthreads();

    // ---- 3x3 tail: lane (g, n) of wave w -> output row 4w + g, columns 4n .. 4n + 3
    const int oy = Y0 + 4 * wave + g, ox = X0 + 4 * n;
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    // a lane's own 4 columns are one conflict-free 16-byte read; its neighbours' edge columns come from
    // lanes n -+ 1 by DPP row shifts, except at the strip's ends (n = 0, 15), which read the ring column
    // (every other lane reads the same ring word: a broadcast).  The 4-byte reads at stride 4 words this
    // replaces were 4-way bank conflicts (SQ_LDS_BANK_CONFLICT 1.0 M cycles per launch at S-K)
    const int edge = n == 0 ? 3 : 68;
#pragma unroll 2
    for (int c = 0; c < NF; ++c) {
#pragma unroll
        for (int ky = 0; ky < 3; ++ky) {
            const float* row = &sh[c][4 * wave + g + ky][0];
            float v[6];
            const conv::floatx4 mid4 = *reinterpret_cast<const conv::floatx4*>(row + 4 + 4 * n);
            const float ev = row[edge];
            const float lf = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mid4[3]), 0x111, 0xf, 0xf, false));
            const float rt = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mid4[0]), 0x101, 0xf, 0xf, false));
            v[0] = n == 0 ? ev : lf;   // row_shr:1 -> lane n - 1's column 3
            v[1] = mid4[0];
            v[2] = mid4[1];
            v[3] = mid4[2];
            v[4] = mid4[3];
            v[5] = n == 15 ? ev : rt;  // row_shl:1 -> lane n + 1's column 0
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) {
                const float w = wsh[G::OW_TW + (c * 3 + ky) * 3 + kx];
                // output pairs (0, 1), (2, 3) as packed FMAs (v_pk_fma_f32), per output the same order
                const f2v w2 = {w, w};
                const f2v lo = __builtin_elementwise_fma(w2, f2v{v[kx], v[1 + kx]}, f2v{acc[0], acc[1]});
                const f2v hi = __builtin_elementwise_fma(w2, f2v{v[2 + kx], v[3 + kx]}, f2v{acc[2], acc[3]});
                acc[0] = lo[0];
                acc[1] = lo[1];
                acc[2] = hi[0];
                acc[3] = hi[1];
            }
        }
    }
    const float tb = a.tail_b ? wsh[G::OW_TB] : 0.f;
    if (oy >= HO) return;
    const int vo = static_cast<int>(4 * (static_cast<long long>(oy) * a.oh + ox));
    const __amdgpu_buffer_rsrc_t rso = __builtin_amdgcn_make_buffer_rsrc(a.out + b * a.ob, static_cast<short>(0),
                                                                         0x7fffffff, 0x00020000);
    if (ox + 3 < WO && ((reinterpret_cast<uintptr_t>(a.out + b * a.ob) + vo) & 15) == 0) {
        typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
        __builtin_amdgcn_raw_buffer_store_b128(
            u32x4{__float_as_uint(acc[0] + tb), __float_as_uint(acc[1] + tb), __float_as_uint(acc[2] + tb),
                  __float_as_uint(acc[3] + tb)},
            rso, vo, 0, conv::kStoreAux);
    } else {
        float* o = a.out + b * a.ob + static_cast<long long>(oy) * a.oh + ox;
#pragma unroll
        for (int j = 0; j < 4; ++j)
            if (ox + j < WO) o[j] = acc[j] + tb;
    }
}

template <int L>
int launch_tile4(const esm_shuffle_tail_desc& a, hipStream_t s) {
    const dim3 grid(ceil_div(a.W, 16), ceil_div(a.H, L), a.B);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("shuffle_tail: grid too large");
    hipLaunchKernelGGL((shuffle_tail4_kernel<L>), grid, dim3(64 * L), 0, s, a);
    return check_launch("shuffle_tail");
}

template <int NF, int R, int TH, int TW>
int launch_tile(const esm_shuffle_tail_desc& a, hipStream_t s) {
    dim3 grid(ceil_div(static_cast<long long>(a.W) * R, TW), ceil_div(static_cast<long long>(a.H) * R, TH), a.B);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("shuffle_tail: grid too large");
    hipLaunchKernelGGL((shuffle_tail_kernel<NF, R, TH, TW>), grid, dim3(kThreads), 0, s, a);
    return check_launch("shuffle_tail");
}

// 16 (8 for nf = 16) x 64 output tiles when that gives the chip ~one workgroup per CU, else
// 8 x 32 tiles (4x the workgroups for the coarse stage's small output).
template <int NF, int R>
int launch_nr(const esm_shuffle_tail_desc& a, hipStream_t s) {
    constexpr int TH = NF <= 8 ? 16 : 8;
    const long long big = static_cast<long long>(ceil_div(static_cast<long long>(a.W) * R, 64)) *
                          ceil_div(static_cast<long long>(a.H) * R, TH) * a.B;
    // nf = 8, r = 4 (ESMStereo-S 4x head): 16 x 32 tiles measured faster than 16 x 64 (15.1 vs 16.5 us
    // at 384x1248, 8 x 64: 16.8, 8 x 32: 18.1; in the S-K launch sequence)
    if constexpr (NF == 8 && R == 4) {
        // flags bits 1-2 (esm_shuffle_tail_desc): 0 automatic, 1 the window form below, 2 / 3 the row form
        // with 4 / 8 low-res rows per workgroup.  Automatic (r04 probe, back to back): the 8-row form where
        // it still gives >= 128 workgroups (96x312 in: 8.9 us vs 10.3 for 4 rows, 12.9 window), else the
        // window form (24x78 in: 8.5 vs 10.6 / 8.8)
        const int form = (a.flags >> 1) & 3;
        const long long t8 = static_cast<long long>(ceil_div(a.W * R, 64)) * ceil_div(a.H * R, 32) * a.B;
        if (form == 3 || (form == 0 && t8 >= 128)) return launch_tile4<8>(a, s);
        if (form == 2) return launch_tile4<4>(a, s);
        if (big >= 256) return launch_tile<NF, R, 16, 32>(a, s);
    }
    // nf = 16 (ESMStereo-L heads): 8 x 32 tiles (4x head at 384x1248: 38.9 vs 48.2 us for 8 x 64;
    // 2x head equal)
    if constexpr (NF == 16) return launch_tile<NF, R, 8, 32>(a, s);
    return big >= 256 ? launch_tile<NF, R, TH, 64>(a, s) : launch_tile<NF, R, 8, 32>(a, s);
}

// ---------------------------------------------------------------------------------------------
// shuffle_tail followed by the refinement hourglass's first conv, in one launch:
//   x  = tail(SiLU(PixelShuffle(r)(up(lowres))))              (the 1-channel map, never stored)
//   c1 = GELU(BN(Conv2d(1, C, 3, stride 2, pad 1)(x)))          (up_refinement.conv1[0])
// (models/ESMStereo.py:301-303 / :311-313: `x = self.tail(self.upsampling(x))`, then
// `self.ref(x, ...)` whose first layer is BasicConv(1, C, 3, 2, 1) at :190-191).  A workgroup owns a
// TH2 x 16 tile of c1 (all C channels); it stages the low-resolution window under the tile, builds
// the shuffled map on it with MFMA (M = the r*r sub-pixels of 16/(r*r) channels, N = 16 low-res pixels,
// K = nf), runs the 3x3 tail on the (2*TH2 + 1) x 33 x window, then conv1 from LDS.  The x map (1.9 MB
// at S-K) and its re-read by a separate conv launch disappear.  Arithmetic per element follows the
// two unfused kernels (shuffle_tail_kernel, conv_stem.hip c1in_kernel).
template <int NF, int R, int C, int TH2>
struct ScGeo {
    static constexpr int TW2 = 16;
    static constexpr int RR = R * R;
    static constexpr int NUP = NF * RR;
    static constexpr int LRH = 2 * TH2 / R + 2, LRW = 2 * TW2 / R + 2;  // low-res window
    static constexpr int PIX = LRH * LRW;
    static constexpr int MR = LRH * R, MC = LRW * R + 4;                 // shuffled window (padded row)
    static constexpr int XH = 2 * TH2 + 1, XW = 2 * TW2 + 1, XWP = 36;  // x window
    static constexpr int CPT = 16 / RR;                                  // channels per MFMA M-tile
    static constexpr int NMT = NF / CPT;
    static constexpr int NNT = (PIX + 15) / 16;
    // weights: up_w [NUP][NF], up_b [NUP], tail_w [NF*9], tail_b, c1 w [9][C], scale [C], shift [C]
    static constexpr int OW_UB = NUP * NF, OW_TW = OW_UB + NUP, OW_TB = OW_TW + NF * 9, OW_CW = OW_TB + 1,
                         OW_SC = OW_CW + 9 * C, OW_SH = OW_SC + C, WN = OW_SH + C;
};

template <int NF, int R, int C, int TH2>
__global__ void __launch_bounds__(kThreads) shuffle_conv_kernel(const esm_shuffle_conv_desc a) {
    using G = ScGeo<NF, R, C, TH2>;
    constexpr int TW2 = G::TW2, RR = G::RR, LRW = G::LRW, PIX = G::PIX, MR = G::MR, MC = G::MC;
    constexpr int XH = G::XH, XW = G::XW, XWP = G::XWP, WN = G::WN;
    __shared__ __attribute__((aligned(16))) float wsh[WN];
    __shared__ float lr[NF][PIX];
    __shared__ __attribute__((aligned(16))) float mid[NF][MR][MC];
    __shared__ float xs[XH][XWP];

    const esm_shuffle_tail_desc& t = a.st;
    const int tid = threadIdx.x;
    const int H = t.H, W = t.W, HO = H * R, WO = W * R;
    const int b = blockIdx.z;
    const int y0 = blockIdx.y * TH2, x0 = blockIdx.x * TW2;  // c1 tile origin
    const int ly0 = 2 * y0 / R - 1, lx0 = 2 * x0 / R - 1;    // low-res window origin (mid row 0 = ly0 * R)
    const float* xb = t.x + b * t.xb;

    // ---- stage weights and the low-res window (one round trip)
    constexpr int WR = (WN + kThreads - 1) / kThreads;
    constexpr int LN = NF * PIX;
    constexpr int LR_ = (LN + kThreads - 1) / kThreads;
    float rw[WR], rx[LR_];
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        const int i = tid + k * kThreads;
        const float* p;
        int off;
        if (i < G::OW_UB) { p = t.up_w; off = i; }
        else if (i < G::OW_TW) { p = t.up_b; off = i - G::OW_UB; }
        else if (i < G::OW_TB) { p = t.tail_w; off = i - G::OW_TW; }
        else if (i < G::OW_CW) { p = t.tail_b; off = 0; }
        else if (i < G::OW_SC) { p = a.w; off = (i - G::OW_CW) / C * a.cin_pad * a.cout_pad + (i - G::OW_CW) % C; }
        else if (i < G::OW_SH) { p = a.scale; off = i - G::OW_SC; }
        else { p = a.shift; off = i - G::OW_SH; }
        const bool ok = i < WN && p != nullptr;
        const float v = (ok ? p : t.up_w)[ok ? off : 0];
        rw[k] = ok ? v : (i >= G::OW_SC && i < G::OW_SH ? 1.f : 0.f);
    }
#pragma unroll
    for (int k = 0; k < LR_; ++k) {
        const int i = tid + k * kThreads;
        const int c = i / PIX, rem = i - c * PIX;
        const int yy = ly0 + rem / LRW, xx = lx0 + rem % LRW;
        const bool ok = i < LN && yy >= 0 && yy < H && xx >= 0 && xx < W;
        const float v = xb[ok ? c * t.xc + yy * t.xh + xx : 0];
        rx[k] = ok ? v : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
    for (int k = 0; k < WR; ++k)
        if (tid + k * kThreads < WN) wsh[tid + k * kThreads] = rw[k];
#pragma unroll
    for (int k = 0; k < LR_; ++k)
        if (tid + k * kThreads < LN) (&lr[0][0])[tid + k * kThreads] = rx[k];
    __syncthreads();

    // ---- shuffled window: unit (M-tile mt, N-tile nt); lane (g, n): MFMA rows 4g + j = (channel
    //      mt * CPT + m / RR, sub-pixel m % RR) of low-res pixel nt * 16 + n
    {
        const int wave = tid >> 6, lane = tid & 63, g = lane >> 4, n = lane & 15;
        for (int u = wave; u < G::NMT * G::NNT; u += kThreads / 64) {
            const int mt = u % G::NMT, nt = u / G::NMT;
            const int p = nt * 16 + n;
            const bool pin = p < PIX;
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < NF / 4; ++kk) {
                const float av = wsh[(mt * 16 + n) * NF + 4 * kk + g];  // A[m = n][k]: up_w row (channel, sub-pixel)
                const float bv = lr[4 * kk + g][pin ? p : 0];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc, 0, 0, 0);
            }
            const int py = p / LRW, px = p - (p / LRW) * LRW;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = 4 * g + j;
                const int c = mt * G::CPT + m / RR, sp = m % RR, sy = sp / R, sx = sp % R;
                const int my = py * R + sy, mx = px * R + sx;  // window coordinates
                const int Y = ly0 * R + my, X = lx0 * R + mx;
                const float v = silu_fast(acc[j] + wsh[G::OW_UB + mt * 16 + m]);
                if (pin) mid[c][my][mx] = (Y >= 0 && Y < HO && X >= 0 && X < WO) ? v : 0.f;  // tail zero padding
            }
        }
    }
    __syncthreads();

    // ---- x window (rows 2*y0 - 1 ..., cols 2*x0 - 1 ...): 4 consecutive columns per thread
    {
        constexpr int QPR = (XW + 3) / 4;
        const int XY0 = 2 * y0 - 1, XX0 = 2 * x0 - 1;
        const int oy = XY0 - 1 - ly0 * R, ox = XX0 - 1 - lx0 * R;  // mid window position of x (0, 0)'s tap (0, 0)
        const float tb = wsh[G::OW_TB];
        for (int q = tid; q < XH * QPR; q += kThreads) {
            const int r = q / QPR, g = q - (q / QPR) * QPR;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
            for (int c = 0; c < NF; ++c) {
#pragma unroll
                for (int ky = 0; ky < 3; ++ky) {
                    float v[6];
#pragma unroll
                    for (int j = 0; j < 6; ++j) v[j] = mid[c][oy + r + ky][min(ox + 4 * g + j, MC - 1)];
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) {
                        const float w = wsh[G::OW_TW + (c * 3 + ky) * 3 + kx];
#pragma unroll
                        for (int j = 0; j < 4; ++j) acc[j] += w * v[j + kx];
                    }
                }
            }
            const int Y = XY0 + r;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int X = XX0 + 4 * g + j;
                if (4 * g + j < XW) xs[r][4 * g + j] = (Y >= 0 && Y < HO && X >= 0 && X < WO) ? acc[j] + tb : 0.f;
            }
        }
    }
    __syncthreads();

    // ---- c1 = GELU(BN(conv 3x3 s2 p1 (x))): thread = (pixel, half of the channels)
    {
        constexpr int NPX = TH2 * TW2;
        constexpr int CH = C * NPX / kThreads;  // channels per thread
        const int pxi = tid % NPX, c0 = (tid / NPX) * CH;
        const int yy = pxi / TW2, xx = pxi % TW2;
        const int oy = y0 + yy, ox = x0 + xx;
        float xv[9];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) xv[ky * 3 + kx] = xs[2 * yy + ky][2 * xx + kx];
        const int Ho2 = (HO + 1) / 2, Wo2 = (WO + 1) / 2;
        const bool ok = oy < Ho2 && ox < Wo2;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            a.out + b * a.ob, static_cast<short>(0),
            static_cast<int>(4 * ((C - 1) * a.oc + (Ho2 - 1) * a.oh + Wo2)), 0x00020000);
#pragma unroll
        for (int k = 0; k < CH; ++k) {
            const int co = c0 + k;
            float acc = 0.f;
#pragma unroll
            for (int tp = 0; tp < 9; ++tp) acc += wsh[G::OW_CW + tp * C + co] * xv[tp];
            const float v = gelu_erf(acc * wsh[G::OW_SC + co] + wsh[G::OW_SH + co]);
            const unsigned o = ok ? 4u * static_cast<unsigned>(co * a.oc + static_cast<long long>(oy) * a.oh + ox)
                                  : conv::kOOB;
            conv::store_b32(__float_as_uint(v), ro, static_cast<int>(o), 0);
        }
    }
}

// nf = 8, r = 4, C = 16 on large maps (ESMStereo-S's 4x stage: upsampling4 + tail4x + ref4x.conv1[0]):
// shuffle_tail4_kernel's tile (L low-res rows x 16 low-res pixels -> a (4L) x 64 x tile, its shuffled
// map built by MFMA, the tail on the VALU with DPP neighbour columns) plus the one x row above and the
// one x column left of it that the stride-2 conv needs; x stays in LDS and the conv's (2L) x 32 output
// tile (all 16 channels) is computed from it, one output pixel per thread.  The tail's arithmetic is
// shuffle_tail4_kernel's, the conv's the c1in / shuffle_conv_kernel order (taps outer, BN, exact GELU).
template <int L>
struct Sc4Geo {
    static constexpr int NF = 8, R = 4, C = 16;
    static constexpr int TR = 4 * L;                     // x tile rows (64 columns)
    static constexpr int SR = TR + 3, SC = 72;           // shuffled map: row 0 = Y0 - 2, col 4 = X0 (cols 2..68 used)
    static constexpr int LH = L + 2, LW = 18;            // low-res window: rows ly0 - 1 .., cols lx0 - 1 ..
    static constexpr int XR = TR + 1, XC = 72;           // x: row 0 = Y0 - 1, col 4 = X0 (col 3 = X0 - 1)
    static constexpr int OW_UB = 128 * NF, OW_TW = OW_UB + 128, OW_TB = OW_TW + NF * 9, OW_CW = OW_TB + 1,
                         OW_SC = OW_CW + 9 * C, OW_SH = OW_SC + C, WN = OW_SH + C;
    static constexpr int XN = NF * LH * LW;
    // the pre-conv (PRE): its input window (16 channels x (LH + 2) x (LW + 2), channel stride 240 = 16 mod 32
    // banks), its weights as the MFMA A image [tap][ci 16][co 16] and BN (8 + 8)
    static constexpr int PCH = 16, PR = LH + 2, PW = LW + 2, PCS = PR * PW, PXN = PCH * PCS;
    static constexpr int PWN = 9 * 16 * 16, PBN = 2 * NF;
    static constexpr int PNT = (LH * LW + 15) / 16;  // pre-conv N tiles (16 window pixels each)
};

#ifdef ESM_CONV_STAMPS
// Diagnostic build only: s_memrealtime (100 MHz) of workgroup-thread 0 at each phase boundary of
// shuffle_conv4_kernel, [workgroup][8] (esm_diag_sc4_stamps); never in the product library.
__device__ unsigned long long sc4_stamps[4096 * 8];
#define SC4_STAMP(k)                                                                                     \
    do {                                                                                                 \
        const unsigned wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);             \
        if (threadIdx.x == 0 && wg_ < 4096) sc4_stamps[wg_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define SC4_STAMP(k) (void)0
#endif

template <int L, bool PRE, bool MC1 = false>
__global__ void __launch_bounds__(64 * L) shuffle_conv4_kernel(const esm_shuffle_conv_desc d) {
    using G = Sc4Geo<L>;
    constexpr int NF = G::NF, C = G::C, SR = G::SR, SC = G::SC, LH = G::LH, LW = G::LW, WN = G::WN, XN = G::XN;
    constexpr int TR = G::TR, NT = 64 * L;
    const esm_shuffle_tail_desc& a = d.st;
    __shared__ __attribute__((aligned(16))) float wsh[WN];
    __shared__ float lr[NF][LH][LW];
    __shared__ __attribute__((aligned(16))) float sh[NF][SR][SC];
    __shared__ __attribute__((aligned(16))) float xs[G::XR][G::XC];
    __shared__ float pxs[PRE ? G::PXN : 1];
    __shared__ float pws[PRE ? G::PWN + G::PBN : 1];

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, HO = 4 * H, WO = 4 * W;
    const Blk3 bk_ = xcd_block((a.flags & 1) != 0);
    const int b = bk_.z;
    const int ly0 = bk_.y * L, lx0 = bk_.x * 16;
    const int Y0 = 4 * ly0, X0 = 4 * lx0;
    const float* xb = PRE ? nullptr : a.x + b * a.xb;
    SC4_STAMP(0);

    // ---- stage (one round trip): every weight (head, tail, conv, BN) and the low-res window
    constexpr int WRN = (WN + NT - 1) / NT, XRN = (XN + NT - 1) / NT;
    float rw[WRN], rx[XRN];
#pragma unroll
    for (int k = 0; k < WRN; ++k) {
        const int i = tid + k * NT;
        const float* p;
        int off;
        if (i < G::OW_UB) { p = a.up_w; off = i; }
        else if (i < G::OW_TW) { p = a.up_b; off = i - G::OW_UB; }
        else if (i < G::OW_TB) { p = a.tail_w; off = i - G::OW_TW; }
        else if (i < G::OW_CW) { p = a.tail_b; off = 0; }
        else if (i < G::OW_SC) { p = d.w; off = (i - G::OW_CW) / C * d.cin_pad * d.cout_pad + (i - G::OW_CW) % C; }
        else if (i < G::OW_SH) { p = d.scale; off = i - G::OW_SC; }
        else { p = d.shift; off = i - G::OW_SH; }
        const bool ok = i < WN && p != nullptr;
        const float v = (ok ? p : a.up_w)[ok ? off : 0];
        rw[k] = ok ? v : (i >= G::OW_SC && i < G::OW_SH ? 1.f : 0.f);
    }
    if constexpr (!PRE) {
#pragma unroll
        for (int k = 0; k < XRN; ++k) {
            const int i = tid + k * NT;
            const int c = i / (LH * LW), rem = i - c * (LH * LW);
            const int yy = ly0 - 1 + rem / LW, xx = lx0 - 1 + rem % LW;
            const bool ok = i < XN && yy >= 0 && yy < H && xx >= 0 && xx < W;
            const float v = xb[ok ? c * a.xc + yy * a.xh + xx : 0];
            rx[k] = ok ? v : 0.f;
        }
    }
    // PRE: the pre-conv's input window (rows ly0 - 2 .., cols lx0 - 2 ..; zero outside the image: the
    // conv's padding), weights and BN
    constexpr int PXR = PRE ? (G::PXN + NT - 1) / NT : 1, PWR = PRE ? (G::PWN + G::PBN + NT - 1) / NT : 1;
    float rp[PXR], rq[PWR];
    if constexpr (PRE) {
        const float* pb = d.pre_x + b * d.pb;
#pragma unroll
        for (int k = 0; k < PXR; ++k) {
            const int i = tid + k * NT;
            const int c = i / G::PCS, rem = i - c * G::PCS;
            const int yy = ly0 - 2 + rem / G::PW, xx = lx0 - 2 + rem % G::PW;
            const bool ok = i < G::PXN && c < d.pre_cin && yy >= 0 && yy < H && xx >= 0 && xx < W;
            const float v = pb[ok ? c * d.pc + yy * d.ph + xx : 0];
            rp[k] = ok ? v : 0.f;
        }
#pragma unroll
        for (int k = 0; k < PWR; ++k) {
            const int i = tid + k * NT;
            float v = 0.f;
            if (i < G::PWN) {  // [tap][ci][co] <- packed [tap][cin_pad][cout_pad]
                const int co = i & 15, ci = (i >> 4) & 15, tap = i >> 8;
                const bool ok = ci < d.pre_cin && co < NF;
                const float u = d.pre_w[ok ? (tap * d.pre_cin_pad + ci) * d.pre_cout_pad + co : 0];
                v = ok ? u : 0.f;
            } else if (i < G::PWN + G::PBN) {
                const int j = i - G::PWN;
                const float* q = j < NF ? d.pre_scale : d.pre_shift;
                const float u = (q ? q : d.pre_w)[q ? (j & (NF - 1)) : 0];
                v = q ? u : (j < NF ? 1.f : 0.f);
            }
            rq[k] = v;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < WRN; ++k)
        if (tid + k * NT < WN) wsh[tid + k * NT] = rw[k];
    if constexpr (!PRE) {
#pragma unroll
        for (int k = 0; k < XRN; ++k)
            if (tid + k * NT < XN) (&lr[0][0][0])[tid + k * NT] = rx[k];
    } else {
#pragma unroll
        for (int k = 0; k < PXR; ++k)
            if (tid + k * NT < G::PXN) pxs[tid + k * NT] = rp[k];
#pragma unroll
        for (int k = 0; k < PWR; ++k)
            if (tid + k * NT < G::PWN + G::PBN) pws[tid + k * NT] = rq[k];
        __syncthreads();
        SC4_STAMP(1);
        // x = GELU(BN(conv3x3(pre_x))) on the low-res window (MFMA: M = the nf couts (rows 8..15 zero weights),
        // N = 16 window pixels, K = 16 channels x 9 taps), zero outside the image (the head's window padding)
        for (int nt = wave; nt < G::PNT; nt += NT / 64) {
            const int p = nt * 16 + n;
            const int pp = p < LH * LW ? p : 0;
            const int py = pp / LW, px = pp - (pp / LW) * LW;
            // two accumulation chains (even / odd channel groups): a dependent MFMA waits for its predecessor
            conv::floatx4 acc2[2] = {conv::floatx4{0.f, 0.f, 0.f, 0.f}, conv::floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int dy = tap / 3, dx = tap % 3;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int ci = 4 * ks + g;
                    acc2[ks & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                        pws[(tap * 16 + ci) * 16 + n], pxs[ci * G::PCS + (py + dy) * G::PW + px + dx], acc2[ks & 1], 0, 0, 0);
                }
            }
            const conv::floatx4 acc = acc2[0] + acc2[1];
            const int yy = ly0 - 1 + py, xx = lx0 - 1 + px;
            const bool in = p < LH * LW && yy >= 0 && yy < H && xx >= 0 && xx < W;
            if (g < 2 && p < LH * LW) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = 4 * g + j;
                    const float v = gelu_erf(acc[j] * pws[G::PWN + co] + pws[G::PWN + NF + co]);
                    lr[co][py][px] = in ? v : 0.f;
                }
            }
        }
    }
    __syncthreads();
    SC4_STAMP(2);

    // ---- shuffled interior (MFMA, as shuffle_tail4_kernel), rows 2 .. TR + 1
    {
        const int Y = Y0 + 4 * wave + g, Xl = X0 + 4 * n;
        float bk[2];
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) bk[kk] = lr[4 * kk + g][wave + 1][n + 1];
#pragma unroll
        for (int c = 0; c < NF; ++c) {
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int kk = 0; kk < 2; ++kk)
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(wsh[(c * 16 + n) * NF + 4 * kk + g], bk[kk], acc, 0, 0, 0);
            conv::floatx4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = silu_fast(acc[j] + wsh[G::OW_UB + c * 16 + 4 * g + j]);
                o[j] = (Y < HO && Xl + j < WO) ? v : 0.f;
            }
            *reinterpret_cast<conv::floatx4*>(&sh[c][2 + 4 * wave + g][4 + 4 * n]) = o;
        }
    }
    // ---- the ring (VALU): rows 0, 1 and SR - 1 over cols 2..68, cols 2, 3 and 68 over rows 2..TR + 1
    auto ring_value = [&](int c, int tr, int tc) __attribute__((always_inline)) {
        const int Y = Y0 - 2 + tr, X = X0 - 4 + tc;
        float v = 0.f;
        if (Y >= 0 && Y < HO && X >= 0 && X < WO) {
            const int py = (Y >> 2) - (ly0 - 1), px = (X >> 2) - (lx0 - 1);
            const int m = c * 16 + (Y & 3) * 4 + (X & 3);
            float acc = 0.f;
#pragma unroll
            for (int k = 0; k < NF; ++k) acc += wsh[m * NF + k] * lr[k][py][px];
            v = silu_fast(acc + wsh[G::OW_UB + m]);
        }
        sh[c][tr][tc] = v;
    };
    constexpr int RROW = SC - 5;  // 67 columns per ring row (2..68)
    for (int i = tid; i < NF * 3 * RROW; i += NT) {
        const int c = i / (3 * RROW), q = i - c * (3 * RROW);
        const int k = q / RROW;
        ring_value(c, k == 2 ? SR - 1 : k, 2 + q - k * RROW);
    }
    for (int i = tid; i < NF * 3 * TR; i += NT) {
        const int c = i / (3 * TR), q = i - c * (3 * TR);
        const int k = q / TR;
        ring_value(c, 2 + q - k * TR, k == 0 ? 2 : (k == 1 ? 3 : 68));
    }
    __syncthreads();
    SC4_STAMP(3);

    // ---- tail -> x in LDS: lane (g, n) of wave w -> x row Y0 + 4w + g, columns X0 + 4n .. + 3
    const float tb = a.tail_b ? wsh[G::OW_TB] : 0.f;
    {
        const int oy = Y0 + 4 * wave + g, ox = X0 + 4 * n;
        float acc[4] = {0.f, 0.f, 0.f, 0.f};
        const int edge = n == 0 ? 3 : 68;
#pragma unroll 2
        for (int c = 0; c < NF; ++c) {
#pragma unroll
            for (int ky = 0; ky < 3; ++ky) {
                const float* row = &sh[c][4 * wave + g + 1 + ky][0];
                float v[6];
                const conv::floatx4 mid4 = *reinterpret_cast<const conv::floatx4*>(row + 4 + 4 * n);
                const float ev = row[edge];
                const float lf = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mid4[3]), 0x111, 0xf, 0xf, false));
                const float rt = __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(mid4[0]), 0x101, 0xf, 0xf, false));
                v[0] = n == 0 ? ev : lf;
                v[1] = mid4[0];
                v[2] = mid4[1];
                v[3] = mid4[2];
                v[4] = mid4[3];
                v[5] = n == 15 ? ev : rt;
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) {
                    const float w = wsh[G::OW_TW + (c * 3 + ky) * 3 + kx];
                    const f2v w2 = {w, w};  // packed output pairs, as shuffle_tail4_kernel
                    const f2v lo = __builtin_elementwise_fma(w2, f2v{v[kx], v[1 + kx]}, f2v{acc[0], acc[1]});
                    const f2v hi = __builtin_elementwise_fma(w2, f2v{v[2 + kx], v[3 + kx]}, f2v{acc[2], acc[3]});
                    acc[0] = lo[0];
                    acc[1] = lo[1];
                    acc[2] = hi[0];
                    acc[3] = hi[1];
                }
            }
        }
        conv::floatx4 o;
#pragma unroll
        for (int j = 0; j < 4; ++j) o[j] = (oy < HO && ox + j < WO) ? acc[j] + tb : 0.f;  // the conv's zero padding
        *reinterpret_cast<conv::floatx4*>(&xs[1 + 4 * wave + g][4 + 4 * n]) = o;
    }
    SC4_STAMP(4);
    // the x row above the tile (row 0, cols 3..67) and the column left of it (col 3, rows 1..TR): VALU
    for (int i = tid; i < 65 + TR; i += NT) {
        const int xr = i < 65 ? 0 : 1 + (i - 65), xc = i < 65 ? 3 + i : 3;
        const int Y = Y0 - 1 + xr, X = X0 - 4 + xc;
        float acc = 0.f;
#pragma unroll 2
        for (int c = 0; c < NF; ++c)
#pragma unroll
            for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                for (int kx = 0; kx < 3; ++kx) acc += wsh[G::OW_TW + (c * 3 + ky) * 3 + kx] * sh[c][xr + ky][xc - 1 + kx];
        xs[xr][xc] = (Y >= 0 && Y < HO && X >= 0 && X < WO) ? acc + tb : 0.f;
    }
    __syncthreads();
    SC4_STAMP(5);

    // ---- c1 = GELU(BN(conv 3x3 s2 p1 (x)))
    if constexpr (MC1) {
        // on the matrix cores (round 5): N-tile = 16 output pixels of one row, M = the 16 couts, K = the 9 taps in
        // 3 k-steps (lane (g, n): tap 4s + g of pixel n); C lane (g, n): couts 4g .. 4g + 3.  Phase stamps of the
        // VALU form below: 3.4 of the kernel's 15.6 us; this form 1.2 us (profiles/r05_sc4_stamps.txt)
        const int Ho2 = (HO + 1) / 2, Wo2 = (WO + 1) / 2;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            d.out + b * d.ob, static_cast<short>(0), static_cast<int>(4 * ((C - 1) * d.oc + (Ho2 - 1) * d.oh + Wo2)),
            0x00020000);
        float ca[3], sc[4], shf[4];
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
            const int t = 4 * s3 + g;
            ca[s3] = t < 9 ? wsh[G::OW_CW + t * C + n] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sc[j] = wsh[G::OW_SC + 4 * g + j];
            shf[j] = wsh[G::OW_SH + 4 * g + j];
        }
        for (int nt = wave; nt < 4 * L; nt += L) {
            const int oyl = nt >> 1, oxl = 16 * (nt & 1) + n;
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3) {
                const int t = 4 * s3 + g;
                const int tt = t < 9 ? t : 8;
                const int ky = tt / 3, kx = tt - (tt / 3) * 3;
                const float bv = xs[2 * oyl + ky][3 + 2 * oxl + kx];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[s3], t < 9 ? bv : 0.f, acc, 0, 0, 0);
            }
            const int oy = Y0 / 2 + oyl, ox = X0 / 2 + oxl;
            const bool ok = oy < Ho2 && ox < Wo2;
            const unsigned pix = 4u * static_cast<unsigned>(oy * d.oh + ox);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = 4 * g + j;
                const float v = gelu_erf(acc[j] * sc[j] + shf[j]);
                conv::store_b32(__float_as_uint(v), ro,
                                static_cast<int>(ok ? pix + 4u * static_cast<unsigned>(co * d.oc) : conv::kOOB), 0);
            }
        }
    } else {
        const int yy = tid >> 5, xx = tid & 31;
        const int oy = Y0 / 2 + yy, ox = X0 / 2 + xx;
        float xv[9];
#pragma unroll
        for (int ky = 0; ky < 3; ++ky)
#pragma unroll
            for (int kx = 0; kx < 3; ++kx) xv[ky * 3 + kx] = xs[2 * yy + ky][3 + 2 * xx + kx];
        const int Ho2 = (HO + 1) / 2, Wo2 = (WO + 1) / 2;
        const bool ok = oy < Ho2 && ox < Wo2;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            d.out + b * d.ob, static_cast<short>(0), static_cast<int>(4 * ((C - 1) * d.oc + (Ho2 - 1) * d.oh + Wo2)),
            0x00020000);
        const unsigned pix = 4u * static_cast<unsigned>(oy * d.oh + ox);
#pragma unroll
        for (int co = 0; co < C; ++co) {
            float acc = 0.f;
#pragma unroll
            for (int tp = 0; tp < 9; ++tp) acc += wsh[G::OW_CW + tp * C + co] * xv[tp];
            const float v = gelu_erf(acc * wsh[G::OW_SC + co] + wsh[G::OW_SH + co]);
            conv::store_b32(__float_as_uint(v), ro, static_cast<int>(ok ? pix + 4u * static_cast<unsigned>(co * d.oc) : conv::kOOB), 0);
        }
    }
    SC4_STAMP(6);
#ifdef ESM_CONV_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    SC4_STAMP(7);
#endif
}

// The 4x stage's spx_4x[1] + upsampling4 + tail4x + ref4x.conv1[0] + ref4x.conv1[1] in ONE launch (round 5,
// esm_shuffle_conv_desc.w2): shuffle_conv4_kernel's low-res tile (L rows x 16 pixels) grown by the second conv's
// one-pixel halo, which the low-res window already covers: the shuffled map on the WHOLE (L + 2) x 18 window by MFMA
// (rows Y0 - 4 .. Y0 + 4L + 3, no VALU ring), x on (4L + 5) x 69, the first conv (c1) on its (2L + 2) x 34 tile + halo
// by MFMA into LDS (zero outside the map: the second conv's padding), then the second conv (3x3 16 -> 16, K = 144 in
// 36 k-steps) by MFMA with BN + GELU, stored.  c1 never leaves LDS.  Arithmetic: the pre-conv, shuffled map and tail
// as shuffle_conv4_kernel; the convs in MFMA k-step order (relative 1e-5 vs fp64).
// Round 6: L = 4 rows on 256 threads (4 waves).  The three weight images the MFMA phases read as A operands (the
// pre-conv, upsampling's 1x1, the second conv: 5632 floats) are staged through LDS once and then held in registers
// (each lane's 36 + 2 x (8 / L) + 36 values), so the workgroup needs ~66 KB of LDS and two fit on a CU: 480
// workgroups on 256 CUs at S-K, one workgroup's VALU / LDS phases (shuffle, tail, c1) overlapping the other's
// matrix-core phases (pre-conv, second conv).  L = 8 (512 threads, ~111 KB, one per CU) stays selectable
// (esm_shuffle_tail_desc.flags bit 3) for A/B measurements.
template <int L_, int NW_>
struct Sc7Geo {
    static constexpr int NF = 8, C = 16, L = L_, NW = NW_, NT = 64 * NW;
    // the second conv's A image in LDS for the whole kernel (8 waves on 4 rows: two workgroups per CU need
    // <= 128 VGPRs, so it cannot stay in registers), else in registers
    static constexpr bool W2LDS = NW == 8 && L == 4;
    static constexpr int pad16(int v) { return v + ((16 - v % 32) + 32) % 32; }  // = 16 (mod 32)
    static constexpr int LH = L + 2, LW = 18, LP0 = LH * LW;           // low-res window: rows ly0 - 1 .., cols lx0 - 1 ..
    static constexpr int LP = pad16(LP0);
    static constexpr int LNT = (LP0 + 15) / 16;                         // window N-tiles
    static constexpr int SR = 4 * LH, SC = 72;                          // shuffled map: row 0 = Y0 - 4, col 0 = X0 - 4
    static constexpr int XR = 4 * L + 5, XC = 72;                       // x: row 0 = Y0 - 3, col 0 = X0 - 4
    static constexpr int TQ = 18, TITEMS = XR * TQ;                      // tail items (x row, column quad)
    static constexpr int QR = 2 * L + 2, QW = 34, QWP = 36;             // c1: row 0 = oy0 - 1, col 0 = ox0 - 1
    static constexpr int QS = pad16(QR * QWP);                          // c1 channel stride (16 mod 32)
    static constexpr int QP = QR * QW, QNT = (QP + 15) / 16;            // c1 pixels, N-tiles
    // small per-channel constants, in LDS for the whole kernel
    static constexpr int OW_UB = 0, OW_TW = OW_UB + 16 * NF, OW_TB = OW_TW + NF * 9, OW_CW = (OW_TB + 1 + 3) / 4 * 4,
                         OW_SC = OW_CW + 9 * C, OW_SH = OW_SC + C, OW_PS = OW_SH + C, OW_PH = OW_PS + NF,
                         OW_S2 = OW_PH + NF, OW_H2 = OW_S2 + C, OW_W2 = OW_H2 + C,
                         WN = OW_W2 + (W2LDS ? 9 * C * C : 0);
    // the MFMA A images, staged in `un` behind the pre-conv window, read once into registers
    static constexpr int PR = L + 4, PW = 20, PCS = pad16(PR * PW), PXN = 16 * PCS;  // pre-conv window [16][PCS]
    static constexpr int BW = PXN, BU = 0, BP = BU + 16 * NF * NF, B2 = BP + 9 * 16 * 16, BWN = B2 + 9 * C * C;
    static constexpr int POST = NF * SR * SC + XR * XC;
    static constexpr int UN = POST > BW + BWN ? POST : BW + BWN;
    static_assert(PCS % 32 == 16 && 16 * QS <= NF * SR * SC && NF % NW == 0, "layout");
};

// L low-res rows, NW waves: (4, 8) two workgroups per CU at <= 128 VGPRs (min 4 waves per SIMD), (4, 4) two at
// <= 256, (8, 8) one (its LDS)
template <int L, int NW>
__global__ void __launch_bounds__(64 * NW, L == 4 ? NW / 2 : 2) shuffle_conv11_kernel(const esm_shuffle_conv_desc d) {
    using G = Sc7Geo<L, NW>;
    constexpr int NF = G::NF, C = G::C, NT = G::NT, LW = G::LW, LP = G::LP, LP0 = G::LP0;
    constexpr int SR = G::SR, SC = G::SC, XC = G::XC, WN = G::WN;
    constexpr int CPW = NF / NW;  // shuffled-map channels per wave (phase 3)
    constexpr bool W2LDS = G::W2LDS;
    const esm_shuffle_tail_desc& a = d.st;
    __shared__ __attribute__((aligned(16))) float wsh[WN];
    __shared__ __attribute__((aligned(16))) float lr[NF * LP];
    __shared__ __attribute__((aligned(16))) float un[G::UN];
    float* const sh = un;                    // [NF][SR][SC]
    float* const xs = un + NF * SR * SC;     // [XR][XC]
    float* const pxs = un;                   // [16][PCS]  (until lr is built)
    float* const bw = un + G::BW;            // A images (until read into registers)
    float* const qs = un;                    // c1 [C][QS] (over sh, once x is built)

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int H = a.H, W = a.W, HO = 4 * H, WO = 4 * W;
    const int Ho2 = (HO + 1) / 2, Wo2 = (WO + 1) / 2;
    const Blk3 bk_ = xcd_block((a.flags & 1) != 0);
    const int b = bk_.z;
    const int ly0 = bk_.y * L, lx0 = bk_.x * 16;
    const int Y0 = 4 * ly0, X0 = 4 * lx0, oy0 = Y0 / 2, ox0 = X0 / 2;
    SC4_STAMP(0);

    // ---- 1. stage (one round trip): every weight and the pre-conv window
    constexpr int WRN = (WN + NT - 1) / NT, BRN = (G::BWN + NT - 1) / NT, PXR = (G::PXN + NT - 1) / NT;
    float rw[WRN], rb[BRN], rp[PXR];
#pragma unroll
    for (int k = 0; k < WRN; ++k) {
        const int i = tid + k * NT;
        const float* p;
        int off;
        float dflt = 0.f;
        if (i < G::OW_TW) { p = a.up_b; off = i - G::OW_UB; }
        else if (i < G::OW_TB) { p = a.tail_w; off = i - G::OW_TW; }
        else if (i == G::OW_TB) { p = a.tail_b; off = 0; }
        else if (i < G::OW_CW) { p = nullptr; off = 0; }
        else if (i < G::OW_SC) { p = d.w; off = (i - G::OW_CW) / C * d.cin_pad * d.cout_pad + (i - G::OW_CW) % C; }
        else if (i < G::OW_SH) { p = d.scale; off = i - G::OW_SC; dflt = 1.f; }
        else if (i < G::OW_PS) { p = d.shift; off = i - G::OW_SH; }
        else if (i < G::OW_PH) { p = d.pre_scale; off = i - G::OW_PS; dflt = 1.f; }
        else if (i < G::OW_S2) { p = d.pre_shift; off = i - G::OW_PH; }
        else if (i < G::OW_H2) { p = d.scale2; off = i - G::OW_S2; dflt = 1.f; }
        else if (i < G::OW_W2) { p = d.shift2; off = i - G::OW_H2; }
        else {  // (W2LDS) the second conv's A image [tap][ci][co]
            const int j = i - G::OW_W2, co = j & 15, ci = (j >> 4) & 15, tap = j >> 8;
            p = d.w2;
            off = (tap * d.cin_pad2 + ci) * d.cout_pad2 + co;
        }
        const bool ok = i < WN && p != nullptr;
        const float v = (ok ? p : a.up_w)[ok ? off : 0];
        rw[k] = ok ? v : dflt;
    }
#pragma unroll
    for (int k = 0; k < BRN; ++k) {
        const int i = tid + k * NT;
        const float* p;
        int off;
        bool ok = i < G::BWN;
        if (i < G::BP) {  // upsampling's 1x1 [NF * 16 out][NF in]
            p = a.up_w;
            off = i;
        } else {  // pre-conv / second conv A images [tap][ci][co 16] (pre: co >= nf zero rows)
            const bool two = i >= G::B2;
            const int j = i - (two ? G::B2 : G::BP), co = j & 15, ci = (j >> 4) & 15, tap = j >> 8;
            p = two ? d.w2 : d.pre_w;
            ok = ok && (two || (ci < d.pre_cin && co < NF));
            off = two ? (tap * d.cin_pad2 + ci) * d.cout_pad2 + co : (tap * d.pre_cin_pad + ci) * d.pre_cout_pad + co;
        }
        const float v = (ok ? p : a.up_w)[ok ? off : 0];
        rb[k] = ok ? v : 0.f;
    }
    {
        const float* pb = d.pre_x + b * d.pb;
#pragma unroll
        for (int k = 0; k < PXR; ++k) {
            const int i = tid + k * NT;
            const int c = i / G::PCS, rem = i - c * G::PCS;
            const int yy = ly0 - 2 + rem / G::PW, xx = lx0 - 2 + rem % G::PW;
            const bool ok = i < G::PXN && c < d.pre_cin && rem < G::PR * G::PW && yy >= 0 && yy < H && xx >= 0 && xx < W;
            const float v = pb[ok ? c * d.pc + yy * d.ph + xx : 0];
            rp[k] = ok ? v : 0.f;
        }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < WRN; ++k)
        if (tid + k * NT < WN) wsh[tid + k * NT] = rw[k];
#pragma unroll
    for (int k = 0; k < BRN; ++k)
        if (tid + k * NT < G::BWN) bw[tid + k * NT] = rb[k];
#pragma unroll
    for (int k = 0; k < PXR; ++k)
        if (tid + k * NT < G::PXN) pxs[tid + k * NT] = rp[k];
    __syncthreads();
    // this lane's A operands: lane (g, n) holds row n, k = g of each k-step (W2LDS: the pre-conv's are read from
    // the staged image in phase 2, the second conv's from wsh in phase 6)
    float pa[W2LDS ? 1 : 9][4], ua[CPW][2], wa[W2LDS ? 1 : 9][4];
    if constexpr (!W2LDS) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                pa[tap][ks] = bw[G::BP + (tap * 16 + 4 * ks + g) * 16 + n];
                wa[tap][ks] = bw[G::B2 + (tap * 16 + 4 * ks + g) * 16 + n];
            }
    }
#pragma unroll
    for (int cc = 0; cc < CPW; ++cc)
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) ua[cc][kk] = bw[G::BU + ((wave + NW * cc) * 16 + n) * NF + 4 * kk + g];
    SC4_STAMP(1);

    // ---- 2. pre-conv on the low-res window (shuffle_conv4_kernel's MFMA form); two tiles interleaved per wave
#pragma unroll 2
    for (int nt = wave; nt < G::LNT; nt += NW) {
        const int p = nt * 16 + n;
        const int pp = p < LP0 ? p : 0;
        const int py = pp / LW, px = pp - (pp / LW) * LW;
        conv::floatx4 acc2[2] = {conv::floatx4{0.f, 0.f, 0.f, 0.f}, conv::floatx4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int dy = tap / 3, dx = tap % 3;
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
                const int ci = 4 * ks + g;
                const float av = W2LDS ? bw[G::BP + (tap * 16 + ci) * 16 + n] : pa[W2LDS ? 0 : tap][ks];
                acc2[ks & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, pxs[ci * G::PCS + (py + dy) * G::PW + px + dx],
                                                                    acc2[ks & 1], 0, 0, 0);
            }
        }
        const conv::floatx4 acc = acc2[0] + acc2[1];
        const int yy = ly0 - 1 + py, xx = lx0 - 1 + px;
        const bool in = p < LP0 && yy >= 0 && yy < H && xx >= 0 && xx < W;
        if (g < 2 && p < LP0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = 4 * g + j;
                const float v = gelu_erf(acc[j] * wsh[G::OW_PS + co] + wsh[G::OW_PH + co]);
                lr[co * LP + p] = in ? v : 0.f;
            }
        }
    }
    __syncthreads();  // lr complete; the pre-conv window and the A images (aliased by sh) are dead
    SC4_STAMP(2);

    // ---- 3. shuffled map on the whole window: wave w takes channels w + L cc of every window tile, 16x16x4 MFMA
    //         (4 tiles interleaved: their 2-MFMA chains and SiLUs overlap)
#pragma unroll 4
    for (int wt = 0; wt < G::LNT; ++wt) {
        const int p = wt * 16 + n;
        const int pp = p < LP0 ? p : 0;
        const int py = pp / LW, px = pp - (pp / LW) * LW;
        const float b0 = lr[g * LP + pp], b1 = lr[(4 + g) * LP + pp];
        const int row = 4 * py + g;  // sh row: Y0 - 4 + row
        const int Y = Y0 - 4 + row, X = X0 - 4 + 4 * px;
        const bool yok = Y >= 0 && Y < HO;
#pragma unroll
        for (int cc = 0; cc < CPW; ++cc) {
            const int c = wave + NW * cc;
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cc][0], b0, acc, 0, 0, 0);
            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ua[cc][1], b1, acc, 0, 0, 0);
            conv::floatx4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float v = silu_fast(acc[j] + wsh[G::OW_UB + c * 16 + 4 * g + j]);
                o[j] = (yok && X + j >= 0 && X + j < WO) ? v : 0.f;  // zero padding of the 3x3 tail
            }
            if (p < LP0) *reinterpret_cast<conv::floatx4*>(&sh[(c * SR + row) * SC + 4 * px]) = o;
        }
    }
    __syncthreads();
    SC4_STAMP(3);

    // ---- 4. tail -> x rows Y0 - 3 .. Y0 + 4L + 1, cols X0 - 4 + 4q .. + 3 (q = 0 .. 17; cols X0 - 3 .. X0 + 65 used)
    {
        const float tb = a.tail_b ? wsh[G::OW_TB] : 0.f;
        for (int it = tid; it < G::TITEMS; it += NT) {
            const int r = it / G::TQ, q = it - (it / G::TQ) * G::TQ;
            const int cl = 4 * q - 1 < 0 ? 0 : 4 * q - 1, cr = 4 * q + 4 < SC ? 4 * q + 4 : SC - 1;
            float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
            for (int c = 0; c < NF; ++c) {
#pragma unroll
                for (int ky = 0; ky < 3; ++ky) {
                    const float* row = &sh[(c * SR + r + ky) * SC];
                    const conv::floatx4 m4 = *reinterpret_cast<const conv::floatx4*>(row + 4 * q);
                    const float v[6] = {row[cl], m4[0], m4[1], m4[2], m4[3], row[cr]};
#pragma unroll
                    for (int kx = 0; kx < 3; ++kx) {
                        const float w = wsh[G::OW_TW + (c * 3 + ky) * 3 + kx];
                        const f2v w2 = {w, w};
                        const f2v lo = __builtin_elementwise_fma(w2, f2v{v[kx], v[1 + kx]}, f2v{acc[0], acc[1]});
                        const f2v hi = __builtin_elementwise_fma(w2, f2v{v[2 + kx], v[3 + kx]}, f2v{acc[2], acc[3]});
                        acc[0] = lo[0];
                        acc[1] = lo[1];
                        acc[2] = hi[0];
                        acc[3] = hi[1];
                    }
                }
            }
            const int Y = Y0 - 3 + r;
            conv::floatx4 o;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int X = X0 - 4 + 4 * q + j;
                o[j] = (Y >= 0 && Y < HO && X >= 0 && X < WO) ? acc[j] + tb : 0.f;  // the first conv's zero padding
            }
            *reinterpret_cast<conv::floatx4*>(&xs[r * XC + 4 * q]) = o;
        }
    }
    __syncthreads();
    SC4_STAMP(4);

    // ---- 5. c1 = GELU(BN(conv 3x3 s2 (x))) on rows oy0 - 1 .. oy0 + 2L, cols ox0 - 1 .. ox0 + 32 (in 16-pixel
    //         N-tiles), zero outside the map (the second conv's padding) -> LDS
    {
        float ca[3], sc[4], shf[4];
#pragma unroll
        for (int s3 = 0; s3 < 3; ++s3) {
            const int t = 4 * s3 + g;
            ca[s3] = t < 9 ? wsh[G::OW_CW + t * C + n] : 0.f;
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sc[j] = wsh[G::OW_SC + 4 * g + j];
            shf[j] = wsh[G::OW_SH + 4 * g + j];
        }
#pragma unroll 2
        for (int nt = wave; nt < G::QNT; nt += NW) {
            const int p = nt * 16 + n;
            const int pp = p < G::QP ? p : 0;
            const int qa = pp / G::QW, qb = pp - (pp / G::QW) * G::QW;
            conv::floatx4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int s3 = 0; s3 < 3; ++s3) {
                const int t = 4 * s3 + g;
                const int tt = t < 9 ? t : 8;
                const int ky = tt / 3, kx = tt - (tt / 3) * 3;
                const float bv = xs[(2 * qa + ky) * XC + 2 * qb + kx + 1];
                acc = __builtin_amdgcn_mfma_f32_16x16x4f32(ca[s3], t < 9 ? bv : 0.f, acc, 0, 0, 0);
            }
            const int oy = oy0 - 1 + qa, ox = ox0 - 1 + qb;
            const bool in = p < G::QP && oy >= 0 && oy < Ho2 && ox >= 0 && ox < Wo2;
            if (p < G::QP) {
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = gelu_erf(acc[j] * sc[j] + shf[j]);
                    qs[(4 * g + j) * G::QS + qa * G::QWP + qb] = in ? v : 0.f;
                }
            }
        }
    }
    __syncthreads();
    SC4_STAMP(5);

    // ---- 6. the second conv (3x3 16 -> 16, BN, GELU) on the 2L x 32 output tile: N-tile = 16 pixels of one row,
    //         two tiles per wave iteration on independent accumulators; lane (g, n): k-step (tap, ks) reads channel
    //         4ks + g of pixel n; C lane (g, n): couts 4g .. 4g + 3
    {
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            d.out + b * d.ob, static_cast<short>(0), static_cast<int>(4 * ((C - 1) * d.oc + (Ho2 - 1) * d.oh + Wo2)),
            0x00020000);
        float sc[4], shf[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            sc[j] = wsh[G::OW_S2 + 4 * g + j];
            shf[j] = wsh[G::OW_H2 + 4 * g + j];
        }
        // UT output tiles per wave iteration: independent accumulator chains (4 where the tile count allows)
        constexpr int UT = (4 * L) % (4 * NW) == 0 ? 4 : 2;
        for (int nt = UT * wave; nt < 4 * L; nt += UT * NW) {
            conv::floatx4 acc[UT];
#pragma unroll
            for (int u = 0; u < UT; ++u) acc[u] = conv::floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                const int dy = tap / 3, dx = tap % 3;
#pragma unroll
                for (int ks = 0; ks < 4; ++ks) {
                    const int ci = 4 * ks + g;
#pragma unroll
                    for (int u = 0; u < UT; ++u) {
                        const int t2 = nt + u;
                        const int oyl = t2 >> 1, oxl = 16 * (t2 & 1) + n;
                        const float av = W2LDS ? wsh[G::OW_W2 + (tap * 16 + ci) * 16 + n] : wa[W2LDS ? 0 : tap][ks];
                        acc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                            av, qs[ci * G::QS + (oyl + dy) * G::QWP + oxl + dx], acc[u], 0, 0, 0);
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < UT; ++u) {
                const int t2 = nt + u;
                const int oy = oy0 + (t2 >> 1), ox = ox0 + 16 * (t2 & 1) + n;
                const bool ok = oy < Ho2 && ox < Wo2;
                const unsigned pix = 4u * static_cast<unsigned>(oy * d.oh + ox);
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = 4 * g + j;
                    const float v = gelu_erf(acc[u][j] * sc[j] + shf[j]);
                    conv::store_b32(__float_as_uint(v), ro,
                                    static_cast<int>(ok ? pix + 4u * static_cast<unsigned>(co * d.oc) : conv::kOOB), 0);
                }
            }
        }
    }
    SC4_STAMP(6);
#ifdef ESM_CONV_STAMPS
    __builtin_amdgcn_s_waitcnt(0);
    SC4_STAMP(7);
#endif
}

// flags bits 3-4: 0 = 4 low-res rows on 8 waves (two workgroups per CU; the default), 1 = 8 rows on 8 waves (one per
// CU; the round-5 tile), 2 = 4 rows on 4 waves
int launch_sc11(const esm_shuffle_conv_desc& a, hipStream_t s) {
    const int sel = (a.st.flags >> 3) & 3;
    const dim3 grid(ceil_div(a.st.W, 16), ceil_div(a.st.H, sel == 1 ? 8 : 4), a.st.B);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("shuffle_conv: grid too large");
    if (sel == 1)
        hipLaunchKernelGGL((shuffle_conv11_kernel<8, 8>), grid, dim3(Sc7Geo<8, 8>::NT), 0, s, a);
    else if (sel == 2)
        hipLaunchKernelGGL((shuffle_conv11_kernel<4, 4>), grid, dim3(Sc7Geo<4, 4>::NT), 0, s, a);
    else
        hipLaunchKernelGGL((shuffle_conv11_kernel<4, 8>), grid, dim3(Sc7Geo<4, 8>::NT), 0, s, a);
    return check_launch("shuffle_conv");
}

template <int L, bool MC1 = false>
int launch_sc4(const esm_shuffle_conv_desc& a, hipStream_t s) {
    const dim3 grid(ceil_div(a.st.W, 16), ceil_div(a.st.H, L), a.st.B);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("shuffle_conv: grid too large");
    if (a.pre_x)
        hipLaunchKernelGGL((shuffle_conv4_kernel<L, true, MC1>), grid, dim3(64 * L), 0, s, a);
    else
        hipLaunchKernelGGL((shuffle_conv4_kernel<L, false, MC1>), grid, dim3(64 * L), 0, s, a);
    return check_launch("shuffle_conv");
}

template <int NF, int R, int C>
int launch_sc(const esm_shuffle_conv_desc& a, hipStream_t s) {
    const esm_shuffle_tail_desc& t = a.st;
    const long long Ho2 = (static_cast<long long>(t.H) * R + 1) / 2, Wo2 = (static_cast<long long>(t.W) * R + 1) / 2;
    // 8-row c1 tiles where that leaves the chip ~one workgroup per CU, else 4 rows
    const long long big = ceil_div(Wo2, 16) * ceil_div(Ho2, 8) * t.B;
    if (big >= 256) {
        const dim3 grid(ceil_div(Wo2, 16), ceil_div(Ho2, 8), t.B);
        if (grid.y > 65535u || grid.z > 65535u) return arg_error("shuffle_conv: grid too large");
        hipLaunchKernelGGL((shuffle_conv_kernel<NF, R, C, 8>), grid, dim3(kThreads), 0, s, a);
    } else {
        const dim3 grid(ceil_div(Wo2, 16), ceil_div(Ho2, 4), t.B);
        hipLaunchKernelGGL((shuffle_conv_kernel<NF, R, C, 4>), grid, dim3(kThreads), 0, s, a);
    }
    return check_launch("shuffle_conv");
}

}  // namespace

int launch_shuffle_tail(const esm_shuffle_tail_desc* d, hipStream_t s) {
    if (!d) return arg_error("shuffle_tail: null descriptor");
    const esm_shuffle_tail_desc& a = *d;
    if (!a.x || !a.out || !a.up_w || !a.up_b || !a.tail_w) return arg_error("shuffle_tail: null pointer");
    if (a.B <= 0 || a.H <= 0 || a.W <= 0) return arg_error("shuffle_tail: bad size");
    if (a.xh < a.W || a.xc < static_cast<long long>(a.H) * a.xh || a.oh < static_cast<long long>(a.W) * a.r)
        return arg_error("shuffle_tail: strides inconsistent with the extents");
    if (a.nf == 8 && a.r == 4) return launch_nr<8, 4>(a, s);
    if (a.nf == 8 && a.r == 2) return launch_nr<8, 2>(a, s);
    if (a.nf == 16 && a.r == 2) return launch_nr<16, 2>(a, s);
    if (a.nf == 16 && a.r == 4) return launch_nr<16, 4>(a, s);
    set_error("shuffle_tail: (nf, r) must be one of (8, 2), (8, 4), (16, 2), (16, 4)");
    return ESM_ERR_UNSUPPORTED;
}

int launch_shuffle_conv(const esm_shuffle_conv_desc* d, hipStream_t s) {
    if (!d) return arg_error("shuffle_conv: null descriptor");
    const esm_shuffle_conv_desc& a = *d;
    const esm_shuffle_tail_desc& t = a.st;
    if (!(a.pre_x ? !t.x : t.x != nullptr) || !t.up_w || !t.up_b || !t.tail_w || !a.w || !a.out)
        return arg_error("shuffle_conv: null pointer (or both st.x and pre_x set)");
    if (a.pre_x) {
        if (!(t.nf == 8 && t.r == 4 && a.C == 16) || (t.flags >> 1 & 3) == 1)
            return arg_error("shuffle_conv: the pre-conv needs nf 8, r 4, C 16 and the row form");
        if (!a.pre_w || a.pre_cin < 1 || a.pre_cin > 16 || a.pre_cin_pad < a.pre_cin || a.pre_cout_pad < t.nf)
            return arg_error("shuffle_conv: bad pre-conv weights / channels");
        if (a.ph < t.W || a.pc < static_cast<long long>(t.H) * a.ph) return arg_error("shuffle_conv: pre_x strides");
    }
    if (t.B <= 0 || t.H <= 0 || t.W <= 0) return arg_error("shuffle_conv: bad size");
    if (t.x && (t.xh < t.W || t.xc < static_cast<long long>(t.H) * t.xh)) return arg_error("shuffle_conv: strides inconsistent");
    if (a.cin_pad < 1 || a.cout_pad < a.C) return arg_error("shuffle_conv: bad conv weight padding");
    const long long Ho2 = (static_cast<long long>(t.H) * t.r + 1) / 2, Wo2 = (static_cast<long long>(t.W) * t.r + 1) / 2;
    if (a.oh < Wo2 || a.oc < Ho2 * a.oh || a.ob < a.C * a.oc) return arg_error("shuffle_conv: output strides");
    if (4 * (a.C * a.oc) >= 0x7fffffffLL) return arg_error("shuffle_conv: output too large");
    if (a.w2) {  // the second conv fused (the row form with its pre-conv only)
        if (!(t.nf == 8 && t.r == 4 && a.C == 16) || (t.flags >> 1 & 3) == 1 || !a.pre_x)
            return arg_error("shuffle_conv: the second conv needs nf 8, r 4, C 16, the row form and the pre-conv");
        if (a.cin_pad2 < a.C || a.cout_pad2 < a.C || a.cin_pad2 % 16 || a.cout_pad2 % 32)
            return arg_error("shuffle_conv: bad second-conv weight padding");
        return launch_sc11(a, s);
    }
    if (t.nf == 8 && t.r == 4 && a.C == 16) {
        // st.flags bits 1-2: 0 automatic, 1 the window form, 2 the row form (shuffle_conv4_kernel, 8 low-res
        // rows per workgroup); automatic: the row form where it gives >= 128 workgroups
        const int form = (t.flags >> 1) & 3;
        const long long t8 = static_cast<long long>(ceil_div(t.W, 16)) * ceil_div(t.H, 8) * t.B;
        // automatic: the refinement conv on the matrix cores (S-K step 0.3193 -> 0.3180 ms, three alternations,
        // profiles/r05_sc_form_ab.txt); form 2 keeps it on the VALU
        if (form == 2) return launch_sc4<8, false>(a, s);
        if (a.pre_x || form == 3 || (form == 0 && t8 >= 128)) return launch_sc4<8, true>(a, s);
        return launch_sc<8, 4, 16>(a, s);
    }
    if (t.nf == 8 && t.r == 2 && a.C == 16) return launch_sc<8, 2, 16>(a, s);
    if (t.nf == 16 && t.r == 2 && a.C == 32) return launch_sc<16, 2, 32>(a, s);
    if (t.nf == 16 && t.r == 4 && a.C == 32) return launch_sc<16, 4, 32>(a, s);
    set_error("shuffle_conv: (nf, r, C) must be one of (8, 4, 16), (8, 2, 16), (16, 2, 32), (16, 4, 32)");
    return ESM_ERR_UNSUPPORTED;
}

}  // namespace esm

extern "C" int esm_shuffle_tail_f32(const esm_shuffle_tail_desc* desc, void* stream) {
    return esm::launch_shuffle_tail(desc, esm::as_stream(stream));
}

extern "C" int esm_shuffle_conv_f32(const esm_shuffle_conv_desc* desc, void* stream) {
    return esm::launch_shuffle_conv(desc, esm::as_stream(stream));
}

#ifdef ESM_CONV_STAMPS
// Diagnostic build only: copy n <= 4096 * 8 shuffle_conv4 phase stamps to the host.
extern "C" int esm_diag_sc4_stamps(unsigned long long* host, int n) {
    if (n > 4096 * 8) n = 4096 * 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(esm::sc4_stamps), 8ull * n) == hipSuccess ? n : -1;
}
#endif
