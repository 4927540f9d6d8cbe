// ShuffleMixer per-pixel chain (models/shufflemixer.py):
//   [optional] depthwise KxK `spatial` conv with bias            (SMLayer :103, :110)
//   per stage: t = shuffle(cat(fc2(silu(fc0(LN(t)[:C/2]))), LN(t)[C/2:])) + t
//              LN = BiasFree_LayerNorm over C (mean IS subtracted) :47-62
//              SplitPointMlp :23-37, channel shuffle 'b (g d) -> b (d g)', g = 8
//   [optional] + res                                              (FMBlock `net(x) + x` :130)
// A workgroup owns a 4x16 pixel tile (the coarse 1/16-res map is small: many small workgroups
// spread it over the chip).  All weights (<= 1.4K floats) and, with the depthwise conv, the tile
// plus its (K-1)/2 halo are staged in LDS by one batch of loads at kernel start.  The depthwise
// conv runs on all 256 threads (4 channel groups x 64 pixels, weights as LDS broadcasts); the
// per-pixel LN/MLP chain then runs on one thread per pixel with its C channels in registers.
#include "common.h"

namespace esm {
namespace {

constexpr int kTileH = 4;
constexpr int kTileW = 16;
constexpr int kPix = kTileH * kTileW;  // pixels per workgroup
constexpr int kThreads = 256;          // depthwise: 4 channel groups x 64 pixels; LN/MLP: 64 pixels

template <int C>
struct SmixLayout {
    static constexpr int H2 = C / 2;
    static constexpr int LN = 0, F0W = C, F0B = F0W + C * H2, F2W = F0B + C, F2B = F2W + H2 * C;
    static constexpr int STAGE = F2B + H2;  // floats per stage
};

// One LN -> SplitPointMlp -> shuffle -> residual stage on a pixel's C channels.  The weights come
// either from LDS (smix_kernel) or straight from global memory through wave-uniform addresses
// (fmnet_kernel: the compiler turns them into scalar loads, no LDS read per weight).
template <int C>
__device__ __forceinline__ void mix_stage_w(float (&t)[C], const float* __restrict__ ln_w, const float* __restrict__ fc0_w,
                                            const float* __restrict__ fc0_b, const float* __restrict__ fc2_w,
                                            const float* __restrict__ fc2_b) {
    constexpr int H2 = C / 2;
    constexpr int DD = C / 8;
    float mu = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) mu += t[c];
    mu = mu / static_cast<float>(C);
    float var = 0.f;
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const float dv = t[c] - mu;
        var += dv * dv;
    }
    var = var / static_cast<float>(C);
    // (t - mu) / sqrt(var + eps) as a multiply by the hardware reciprocal square root (1 ulp): the C
    // IEEE divisions of the libm form were most of the per-pixel chain (profiles/r02_pmc_sq_ops_SK.txt)
    const float inv = __builtin_amdgcn_rsqf(var + 1e-5f);
    float n[C];
#pragma unroll
    for (int c = 0; c < C; ++c) n[c] = (t[c] - mu) * inv * ln_w[c];
    float h[C];
#pragma unroll
    for (int j = 0; j < C; ++j) {
        float s = fc0_b[j];
#pragma unroll
        for (int i = 0; i < H2; ++i) s += fc0_w[j * H2 + i] * n[i];
        h[j] = silu_fast(s);
    }
    float cat[C];
#pragma unroll
    for (int i = 0; i < H2; ++i) {
        float s = fc2_b[i];
#pragma unroll
        for (int j = 0; j < C; ++j) s += fc2_w[i * C + j] * h[j];
        cat[i] = s;
    }
#pragma unroll
    for (int i = H2; i < C; ++i) cat[i] = n[i];
    // out[d*8 + g] = cat[g*DD + d]  (einops 'b (g d) h w -> b (d g) h w', g = 8)
    float o[C];
#pragma unroll
    for (int g = 0; g < 8; ++g)
#pragma unroll
        for (int d = 0; d < DD; ++d) o[d * 8 + g] = cat[g * DD + d] + t[d * 8 + g];
#pragma unroll
    for (int c = 0; c < C; ++c) t[c] = o[c];
}

template <int C>
__device__ __forceinline__ void mix_stage(float (&t)[C], const float* __restrict__ w) {
    using Lyt = SmixLayout<C>;
    mix_stage_w<C>(t, w + Lyt::LN, w + Lyt::F0W, w + Lyt::F0B, w + Lyt::F2W, w + Lyt::F2B);
}

template <int C>
__device__ __forceinline__ void mix_stage_g(float (&t)[C], const esm_smix_stage& g) {
    mix_stage_w<C>(t, g.ln_w, g.fc0_w, g.fc0_b, g.fc2_w, g.fc2_b);
}

template <int C, int K>
__global__ void __launch_bounds__(kThreads) smix_kernel(const esm_smix_desc a) {
    using Lyt = SmixLayout<C>;
    constexpr int R = K / 2;
    constexpr int LH = kTileH + 2 * R;
    constexpr int LW = kTileW + 2 * R;
    constexpr int DWO = ESM_SMIX_MAX_STAGES * Lyt::STAGE;
    constexpr int NW = DWO + (K > 1 ? C * K * K + C : 0);
    constexpr int NT = (K > 1) ? C * LH * LW : 1;
    constexpr int NWR = (NW + kThreads - 1) / kThreads;
    constexpr int NTR = (NT + kThreads - 1) / kThreads;
    __shared__ float wsh[NW];
    __shared__ float tile[(K > 1) ? C : 1][(K > 1) ? LH : 1][(K > 1) ? LW + 1 : 1];
    const int tid = threadIdx.x;
    const int H = a.H, W = a.W;
    const int b = blockIdx.z;
    const int y0 = blockIdx.y * kTileH, x0 = blockIdx.x * kTileW;
    const int ty = (tid % kPix) / kTileW, tx = tid % kTileW;  // pixel of the LN/MLP phase (tid < kPix)
    const int y = y0 + ty, x = x0 + tx;
    const long long plane = static_cast<long long>(H) * W;
    const float* xb = a.x + static_cast<long long>(b) * C * plane;

    // ---- one staging phase: every weight (both stages + depthwise) and the pixel tile with halo,
    //      all loads in flight together, then the LDS stores
    // weight element i of the LDS image: stage s (ln | fc0_w | fc0_b | fc2_w | fc2_b), then the
    // depthwise weights and bias; every pointer is a kernel argument, so the select is scalar
    auto weight_at = [&](int i) -> float {
        const float* p = nullptr;
        int off = 0;
#pragma unroll
        for (int st = 0; st < ESM_SMIX_MAX_STAGES; ++st) {
            const esm_smix_stage& g = a.stage[st];
            const int j = i - st * Lyt::STAGE;
            if (st < a.nstages && j >= 0 && j < Lyt::STAGE) {
                p = j < Lyt::F0W ? g.ln_w : j < Lyt::F0B ? g.fc0_w : j < Lyt::F2W ? g.fc0_b : j < Lyt::F2B ? g.fc2_w : g.fc2_b;
                off = j - (j < Lyt::F0W ? Lyt::LN : j < Lyt::F0B ? Lyt::F0W : j < Lyt::F2W ? Lyt::F0B : j < Lyt::F2B ? Lyt::F2W : Lyt::F2B);
            }
        }
        if (K > 1 && i >= DWO) {
            p = i < DWO + C * K * K ? a.dw_w : a.dw_b;
            off = i - (i < DWO + C * K * K ? DWO : DWO + C * K * K);
        }
        const float v = (p ? p : a.x)[p ? off : 0];  // unconditional load, then select
        return p ? v : 0.f;
    };
    float rw[NWR];
#pragma unroll
    for (int k = 0; k < NWR; ++k) {
        const int i = tid + k * kThreads;
        rw[k] = i < NW ? weight_at(i) : 0.f;
    }
    float rt[NTR];
    if constexpr (K > 1) {
#pragma unroll
        for (int k = 0; k < NTR; ++k) {
            const int i = tid + k * kThreads;
            const int c = i / (LH * LW);
            const int rem = i - c * LH * LW;
            const int ly = rem / LW, lx = rem - (rem / LW) * LW;
            const int gy = y0 + ly - R, gx = x0 + lx - R;
            const bool ok = i < NT && gy >= 0 && gy < H && gx >= 0 && gx < W;
            const float v = xb[ok ? c * plane + gy * W + gx : 0];
            rt[k] = ok ? v : 0.f;
        }
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
    for (int k = 0; k < NWR; ++k)
        if (tid + k * kThreads < NW) wsh[tid + k * kThreads] = rw[k];
    if constexpr (K > 1) {
#pragma unroll
        for (int k = 0; k < NTR; ++k) {
            const int i = tid + k * kThreads;
            if (i < NT) {
                const int c = i / (LH * LW);
                const int rem = i - c * LH * LW;
                const int ly = rem / LW, lx = rem - (rem / LW) * LW;
                tile[c][ly][lx] = rt[k];
            }
        }
    }
    __syncthreads();
    float t[C];
    if constexpr (K > 1) {
        // depthwise KxK: thread = (channel group, pixel); the group (C/4 channels) is wave-uniform,
        // so the weights are LDS broadcasts; results meet their pixel's thread through LDS
        __shared__ float dws[C][kPix];
        const int p = tid % kPix, cg = tid / kPix;
        const int py = p / kTileW, px = p - (p / kTileW) * kTileW;
        const float* dww = wsh + DWO;
        const float* dwb = wsh + DWO + C * K * K;
#pragma unroll
        for (int cc = 0; cc < C / 4; ++cc) {
            const int c = cg * (C / 4) + cc;
            float s = 0.f;
#pragma unroll
            for (int ky = 0; ky < K; ++ky)
#pragma unroll
                for (int kx = 0; kx < K; ++kx) s += dww[(c * K + ky) * K + kx] * tile[c][py + ky][px + kx];
            dws[c][p] = s + dwb[c];
        }
        __syncthreads();
        if (tid >= kPix || y >= H || x >= W) return;
#pragma unroll
        for (int c = 0; c < C; ++c) t[c] = dws[c][tid];
    } else {
        if (tid >= kPix || y >= H || x >= W) return;
#pragma unroll
        for (int c = 0; c < C; ++c) t[c] = xb[c * plane + y * W + x];
    }
    for (int s = 0; s < a.nstages; ++s) mix_stage<C>(t, wsh + s * Lyt::STAGE);
    const long long pix = static_cast<long long>(b) * C * plane + static_cast<long long>(y) * W + x;
    if (a.res) {
#pragma unroll
        for (int c = 0; c < C; ++c) t[c] += a.res[pix + c * plane];
    }
#pragma unroll
    for (int c = 0; c < C; ++c) a.out[pix + c * plane] = t[c];
}

template <int C>
int launch_c(const esm_smix_desc& a, hipStream_t s) {
    dim3 grid(ceil_div(a.W, kTileW), ceil_div(a.H, kTileH), a.B);
    if (!a.dw_w) {
        hipLaunchKernelGGL((smix_kernel<C, 1>), grid, dim3(kThreads), 0, s, a);
    } else if (a.dw_k == 7) {
        hipLaunchKernelGGL((smix_kernel<C, 7>), grid, dim3(kThreads), 0, s, a);
    } else if (a.dw_k == 3) {
        hipLaunchKernelGGL((smix_kernel<C, 3>), grid, dim3(kThreads), 0, s, a);
    } else {
        set_error("smix: depthwise kernel must be 3 or 7");
        return ESM_ERR_UNSUPPORTED;
    }
    return check_launch("smix");
}

// The whole `net` of an FMBlock (two SMLayers, models/shufflemixer.py:100-112,129-130) in one
// launch instead of three smix launches (mlp1 | dw0 -> mlp2 -> mlp1 | dw1 -> mlp2, + x), with halo
// recomputation.  A workgroup owns a kFTH x kFTW output tile: it computes t1 on the tile plus a 2R
// halo and t2 on the tile plus an R halo (each zero outside the image: the depthwise convs' zero
// padding), then the output.  Per pixel and channel the operations and their order are those of
// smix_kernel (equal to the three-launch chain up to the compiler's FMA contraction choices).
#ifdef ESM_CONV_STAMPS
// Diagnostic build only: s_memrealtime (100 MHz) of workgroup-thread 0 at each phase boundary of the
// whole-FMBlock kernel, [workgroup][8] (esm_diag_fmnet_stamps); never in the product library.
__device__ unsigned long long fm_stamps[4096 * 8];
#define FM_STAMP(k)                                                                                   \
    do {                                                                                              \
        const unsigned wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);          \
        if (threadIdx.x == 0 && wg_ < 4096) fm_stamps[wg_ * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define FM_STAMP(k) (void)0
#endif
constexpr int kFTW = 16;
// 512 threads: the t1 region is one pass (448 / 480 pixels), the t2 region one pass, the depthwise
// phases half the iterations of a 256-thread workgroup
constexpr int kFThreads = 512;
// output tile of the whole-FMBlock form: 16 wide, 1 or 3 rows.  1 x 16 measured 1.2 us faster per S-K
// step than 2 x 16 (twice the workgroups on a map that fills a quarter of the chip); on maps with
// enough tiles to fill the chip the recompute of the halo dominates (the t1 region of a 1 x 16 tile is
// 450 pixels, 28x the tile; of a 3 x 16 tile 510 pixels, 10.6x), so those take 3 rows
constexpr int kFConvTW = 16;
constexpr int kFConvTallMinTiles = 512;  // 3-row tiles at or above this many (2 per CU)

// CONV: FMBlock.conv fused behind net (shufflemixer.py:124-131): out = conv2(silu(conv0(t3) + b0)) + b2
// + t3, t3 = net(x) + x.  conv0 is 3x3 zero-padded, so t3 is computed on the tile plus a 1-pixel ring
// (zero outside the image) and kept in LDS; the tile is CTH x kFConvTW (the t1 region
// (CTH + 2 + 12) x (16 + 2 + 12) <= 512 pixels is one pass).  HID = conv0's output channels (dim + 16).
// Depthwise K x K (+ bias) of an OH x OW region, reading the [C][SH][SWP] LDS image `src` (row r
// of the region reads source rows r .. r + K - 1), into dst [C][OH * OW].  A wave owns a channel
// (wave-uniform: its K*K weights and bias are scalar loads from global memory) and a lane owns SEG
// consecutive outputs of a row, so each source value read from LDS feeds up to K outputs.  Per output
// the products are summed over ky, then kx, as in smix_kernel.  Lanes of the last segment of a row
// compute (and drop) up to SEG - 1 outputs past OW: src needs SEG + K - 2 floats of slack at its end.
// NTH threads: with more waves than channels, WPC waves share a channel's items
template <int C, int K, int OH, int OW, int SH, int SWP, int SEG, int NTH = kFThreads>
__device__ __forceinline__ void dw_region(const float* src, float* dst, const float* lw, const float* lb, int wave,
                                          int lane) {
    constexpr int NSEG = (OW + SEG - 1) / SEG;
    constexpr int ITEMS = OH * NSEG;
    constexpr int NWAVES = NTH / 64;
    constexpr int WPC = NWAVES > C ? NWAVES / C : 1;
    for (int cw = wave; cw < C * WPC; cw += NWAVES) {
        const int c = cw % C, part = cw / C;
        // the channel's K*K weights from the workgroup's LDS copy into registers (broadcast reads)
        float w[K * K];
#pragma unroll
        for (int i = 0; i < K * K; ++i) w[i] = lw[c * K * K + i];
        const float bias = lb[c];
        for (int it = part * 64 + lane; it < ITEMS; it += 64 * WPC) {
            const int py = it / NSEG, px0 = (it - py * NSEG) * SEG;
            float acc[SEG];
#pragma unroll
            for (int j = 0; j < SEG; ++j) acc[j] = 0.f;
#pragma unroll
            for (int ky = 0; ky < K; ++ky) {
                float row[SEG + K - 1];
                const float* sr = src + (c * SH + py + ky) * SWP + px0;
#pragma unroll
                for (int j = 0; j < SEG + K - 1; ++j) row[j] = sr[j];
#pragma unroll
                for (int kx = 0; kx < K; ++kx)
#pragma unroll
                    for (int j = 0; j < SEG; ++j) acc[j] += w[ky * K + kx] * row[j + kx];
            }
#pragma unroll
            for (int j = 0; j < SEG; ++j)
                if (px0 + j < OW) dst[c * OH * OW + py * OW + px0 + j] = acc[j] + bias;
        }
    }
}

// NTH: threads per workgroup (1024 for the S-K map, 24 x 78 at C = 8: 120 workgroups on 256 CUs, so a
// workgroup can take a whole CU and halve the per-thread depthwise work)
template <int C, int K, bool CONV, int HID, int CTH = 1, int NTH = kFThreads>
__global__ void __launch_bounds__(NTH) fmnet_kernel(const esm_fmnet_desc a) {
    constexpr int R = K / 2;
    constexpr int TH = CONV ? CTH : 4, TW = CONV ? kFConvTW : kFTW;                        // output tile
    constexpr int HC = CONV ? 1 : 0;                                    // t3 ring for conv0
    constexpr int CH = TH + 2 * HC, CW = TW + 2 * HC, CP = CH * CW;    // t3 region
    constexpr int BH = CH + 2 * R, BW = CW + 2 * R, BP = BH * BW;      // t2 region
    constexpr int AH = CH + 4 * R, AW = CW + 4 * R, AP = AH * AW;      // t1 region
    constexpr int AWP = AW + 1, BWP = BW + 1;
    constexpr int SEG = NTH >= 1024 ? 2 : 4;  // 1024 threads: two waves per channel in the depthwise phases
    constexpr int SLACK = SEG + K;                                      // dw_region's over-read
    constexpr int NWAVES = NTH / 64;
    constexpr int NPX = TH * TW;
    static_assert(AP <= NTH, "one t1 pixel per thread");
    static_assert(!CONV || (NPX <= 64 && (C == 8 || HID % NWAVES == 0)), "conv0 / conv2: one pixel per lane");
    // Every weight is staged in LDS once (below) and read there as a wave-uniform broadcast; the LDS
    // otherwise carries the activations of the three regions
    __shared__ float s1[C * AH * AWP + SLACK];  // t1 image, then t2 image ([C][BH][BWP])
    __shared__ float s2[C * BP];                // depthwise results: region B, then region C
    __shared__ float s3[CONV ? C * CP : 1];           // t3 on region C
    __shared__ float sh[CONV ? HID * NPX : 1];        // silu(conv0(t3)) on the tile
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid / 64), lane = tid % 64;
    const int H = a.H, W = a.W;
    const int b = blockIdx.z;
    const int y0 = blockIdx.y * TH, x0 = blockIdx.x * TW;
    const long long plane = static_cast<long long>(H) * W;
    const float* xb = a.x + static_cast<long long>(b) * C * plane;
    FM_STAMP(0);

    // Weights: one vector load per weight and thread slot, all in flight together with the t1 pixel loads.
    using Lyt = SmixLayout<C>;
    constexpr int DW0 = 4 * Lyt::STAGE, DW1 = DW0 + C * K * K + C;
    constexpr int CV0 = DW1 + C * K * K + C;
    constexpr int CV2 = CV0 + (CONV ? HID * C * 9 + HID : 0);
    constexpr int NW = CV2 + (CONV ? C * HID + C : 0);
    constexpr int NWR = (NW + NTH - 1) / NTH;
    // every weight goes to LDS (the warm-up loads below fetch each one once, all in flight together with
    // the t1 pixel loads) and every phase reads its weights there as LDS broadcasts: as scalar loads they
    // were a chain of L2 (or, in the replayed step, memory) round trips per phase -- dw0 1.6, dw1 1.5,
    // conv0 3.5 us of the 12.4-us block at S-K (profiles/r03_fmnet_phases.txt)
    // LDS weights for C = 8 (S / M): at C = 16 (L) their 32 KB would halve the residency of the 3-row-tile
    // form (two workgroups per CU on L-K's 96 x 312 maps), so there the weights stay scalar loads
    constexpr bool LW = C == 8;
    __shared__ float sw[LW ? NW : 1];
    __shared__ float wsink[LW ? 1 : NTH];
    float rw[NWR];
#pragma unroll
    for (int k = 0; k < NWR; ++k) {
        const int i = tid + k * NTH;
        const float* p = nullptr;
        int off = 0;
        if (i < DW0) {
            const esm_smix_stage& g = a.stage[i / Lyt::STAGE];
            const int j = i % Lyt::STAGE;
            p = j < Lyt::F0W ? g.ln_w : j < Lyt::F0B ? g.fc0_w : j < Lyt::F2W ? g.fc0_b : j < Lyt::F2B ? g.fc2_w : g.fc2_b;
            off = j - (j < Lyt::F0W ? Lyt::LN : j < Lyt::F0B ? Lyt::F0W : j < Lyt::F2W ? Lyt::F0B : j < Lyt::F2B ? Lyt::F2W : Lyt::F2B);
        } else if (i < CV0) {
            const int l = i < DW1 ? 0 : 1;
            const int j = i - (l ? DW1 : DW0);
            p = j < C * K * K ? a.dw_w[l] : a.dw_b[l];
            off = j < C * K * K ? j : j - C * K * K;
        } else if (CONV && i < CV2) {
            const int j = i - CV0;
            p = j < HID * C * 9 ? a.conv0_w : a.conv0_b;
            off = j < HID * C * 9 ? j : j - HID * C * 9;
        } else if (CONV && i < NW) {
            const int j = i - CV2;
            p = j < C * HID ? a.conv2_w : a.conv2_b;
            off = j < C * HID ? j : j - C * HID;
        }
        rw[k] = (p ? p : a.x)[p ? off : 0];
    }
    const int q = tid;  // this thread's t1 pixel (region A)
    const int aly = q / AW, alx = q - (q / AW) * AW;
    const int agy = y0 - HC - 2 * R + aly, agx = x0 - HC - 2 * R + alx;
    const bool ain = q < AP && agy >= 0 && agy < H && agx >= 0 && agx < W;
    float t1[C];
#pragma unroll
    for (int c = 0; c < C; ++c) {
        const float v = xb[ain ? c * plane + agy * W + agx : 0];
        t1[c] = ain ? v : 0.f;
    }
    const float* lw_dw0 = sw + DW0;                    // [C][K][K], then bias [C]
    const float* lw_dw1 = sw + DW1;
    const float* lw_cv0 = sw + CV0;                    // conv0_w [HID][C][9], then conv0_b [HID]
    const float* lw_cv2 = sw + CV2;                    // conv2_w [C][HID], then conv2_b [C]
    const float* w_dw0 = LW ? lw_dw0 : a.dw_w[0];
    const float* b_dw0 = LW ? lw_dw0 + C * K * K : a.dw_b[0];
    const float* w_dw1 = LW ? lw_dw1 : a.dw_w[1];
    const float* b_dw1 = LW ? lw_dw1 + C * K * K : a.dw_b[1];
    const float* w_cv2 = LW ? lw_cv2 : a.conv2_w;
    const float* b_cv2 = LW ? lw_cv2 + C * HID : a.conv2_b;
    // the mlp stages: SmixLayout<C> blocks 0..3 at the start of sw (the warm-up's index order)
    // t1 = SMLayer0.mlp1 (x) on region A, its weights as scalar loads: the phase then waits for the pixel
    // loads only, not for the whole weight batch (staging stage 0 in LDS first cost the S-K block 1 us)
    if (q < AP) {
        if (ain) mix_stage_g<C>(t1, a.stage[0]);
#pragma unroll
        for (int c = 0; c < C; ++c) s1[(c * AH + aly) * AWP + alx] = ain ? t1[c] : 0.f;
    }
    if constexpr (LW) {  // the warm-up values -> LDS weights, read from the next phase on
#pragma unroll
        for (int k = 0; k < NWR; ++k) {
            const int i = tid + k * NTH;
            if (i < NW) sw[i] = rw[k];
        }
    } else {  // scalar weights: the vector loads above only warm L2 for them
        float sink = 0.f;
#pragma unroll
        for (int k = 0; k < NWR; ++k) sink += rw[k];
        wsink[tid] = sink;
    }
    __syncthreads();
    FM_STAMP(1);
    // dw0 (t1) on region B
    dw_region<C, K, BH, BW, AH, AWP, SEG, NTH>(s1, s2, w_dw0, b_dw0, wave, lane);
    __syncthreads();
    FM_STAMP(2);
    // t2 = SMLayer1.mlp1 (SMLayer0.mlp2 (dw0)) on region B, into s1
    for (int p = tid; p < BP; p += NTH) {
        const int py = p / BW, px = p - (p / BW) * BW;
        const int gy = y0 - HC - R + py, gx = x0 - HC - R + px;
        const bool in = gy >= 0 && gy < H && gx >= 0 && gx < W;
        float t[C];
#pragma unroll
        for (int c = 0; c < C; ++c) t[c] = s2[c * BP + p];
        if (in) {
            if constexpr (LW) {
                mix_stage<C>(t, sw + Lyt::STAGE);
                mix_stage<C>(t, sw + 2 * Lyt::STAGE);
            } else {
                mix_stage_g<C>(t, a.stage[1]);
                mix_stage_g<C>(t, a.stage[2]);
            }
        }
#pragma unroll
        for (int c = 0; c < C; ++c) s1[(c * BH + py) * BWP + px] = in ? t[c] : 0.f;
    }
    __syncthreads();
    FM_STAMP(3);
    // dw1 (t2) on region C
    dw_region<C, K, CH, CW, BH, BWP, SEG, NTH>(s1, s2, w_dw1, b_dw1, wave, lane);
    __syncthreads();
    FM_STAMP(4);
    // t3 = SMLayer1.mlp2 (dw1) + x on region C
    if constexpr (!CONV) {
        if (tid >= CP) return;
        const int py = tid / CW, px = tid - (tid / CW) * CW;
        const int y = y0 + py, x = x0 + px;
        if (y >= H || x >= W) return;
        float t[C];
#pragma unroll
        for (int c = 0; c < C; ++c) t[c] = s2[c * CP + tid];
        if constexpr (LW) mix_stage<C>(t, sw + 3 * Lyt::STAGE); else mix_stage_g<C>(t, a.stage[3]);
        const long long pix = static_cast<long long>(b) * C * plane + static_cast<long long>(y) * W + x;
#pragma unroll
        for (int c = 0; c < C; ++c) t[c] += a.x[pix + c * plane];
#pragma unroll
        for (int c = 0; c < C; ++c) a.out[pix + c * plane] = t[c];
    } else {
        if (tid < CP) {
            const int py = tid / CW, px = tid - (tid / CW) * CW;
            const int y = y0 - HC + py, x = x0 - HC + px;
            const bool in = y >= 0 && y < H && x >= 0 && x < W;
            float t[C];
#pragma unroll
            for (int c = 0; c < C; ++c) t[c] = s2[c * CP + tid];
            if (in) {
                if constexpr (LW) mix_stage<C>(t, sw + 3 * Lyt::STAGE); else mix_stage_g<C>(t, a.stage[3]);
                const long long pix = static_cast<long long>(y) * W + x;
#pragma unroll
                for (int c = 0; c < C; ++c) t[c] += xb[pix + c * plane];
            }
            // conv0 pads t3 with zeros outside the image
#pragma unroll
            for (int c = 0; c < C; ++c) s3[c * CP + tid] = in ? t[c] : 0.f;
        }
        __syncthreads();
        FM_STAMP(5);
        if constexpr (LW) {
            // h = silu(conv0(t3) + b0) on the tile: one (hidden channel, pixel) output per thread and pass, so
            // every lane works (a wave owning HID / 8 channels of the tile's 16 pixels left 3/4 of its lanes
            // idle: 1.6 us of the S-K block); weights as LDS reads, per output the products summed over c, ky,
            // kx as before
            for (int e = tid; e < HID * NPX; e += NTH) {
                const int hc = e / NPX, pp = e - (e / NPX) * NPX;
                const int py = pp / TW, px = pp - (pp / TW) * TW;
                const float* w0 = lw_cv0 + hc * C * 9;
                float acc = 0.f;
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx) acc += w0[c * 9 + ky * 3 + kx] * s3[(c * CH + py + ky) * CW + px + kx];
                sh[hc * NPX + pp] = silu_fast(acc + lw_cv0[HID * C * 9 + hc]);
            }
        } else {  // C = 16: a wave owns HID / 8 hidden channels (scalar weight loads), a lane one pixel
            constexpr int HPW = HID / NWAVES;
            if (lane < NPX) {
                const int py = lane / TW, px = lane - (lane / TW) * TW;
                float acc[HPW];
#pragma unroll
                for (int j = 0; j < HPW; ++j) acc[j] = 0.f;
                const float* w0 = a.conv0_w + wave * HPW * C * 9;
#pragma unroll
                for (int c = 0; c < C; ++c)
#pragma unroll
                    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
                        for (int kx = 0; kx < 3; ++kx) {
                            const float v = s3[(c * CH + py + ky) * CW + px + kx];
#pragma unroll
                            for (int j = 0; j < HPW; ++j) acc[j] += w0[(j * C + c) * 9 + ky * 3 + kx] * v;
                        }
#pragma unroll
                for (int j = 0; j < HPW; ++j) {
                    const int hc = wave * HPW + j;
                    sh[hc * NPX + lane] = silu_fast(acc[j] + a.conv0_b[hc]);
                }
            }
        }
        __syncthreads();
        FM_STAMP(6);
        // out = conv2(h) + b2 + t3 on the tile: a wave owns C / 8 output channels, a lane one pixel
        if (lane < NPX) {
            const int py = lane / TW, px = lane - (lane / TW) * TW;
            const int y = y0 + py, x = x0 + px;
            if (y < H && x < W) {
#pragma unroll
                for (int c = wave; c < C; c += NWAVES) {
                    const float* w = w_cv2 + c * HID;
                    float sacc = 0.f;
#pragma unroll
                    for (int hc = 0; hc < HID; ++hc) sacc += w[hc] * sh[hc * NPX + lane];
                    const float v = sacc + b_cv2[c] + s3[(c * CH + py + HC) * CW + px + HC];
                    a.out[static_cast<long long>(b) * C * plane + c * plane + static_cast<long long>(y) * W + x] = v;
                }
            }
        }
        __syncthreads();
        FM_STAMP(7);
    }
}

// ---------------------------------------------------------------------------------------------
// The whole FMBlock as TWO launches for large maps (esm_fmnet_desc.work given): the block split at its
// second depthwise conv, so each launch recomputes only a 3-pixel halo (the fused form above recomputes
// the t1 region 10.6x its tile at L-K, whose halo is the whole block's 7 + 1 pixels), and FMBlock.conv on
// the fp32 matrix cores (the fused form ran its 9C x (C+16) and (C+16) x C GEMMs on the VALU from LDS):
//   fm2a: t1 = mlp1_0(x) on tile + 3, dw0 on the tile, d = mlp1_1(mlp2_0(.)) -> work
//   fm2b: dw1(d) on tile + 1, t3 = mlp2_1(.) + x, h = silu(conv0(t3) + b0) (MFMA), out = conv2(h) + b2 + t3
//         (MFMA); t3 stays in LDS.
// Per pixel and channel the per-pixel chain and the depthwise convs run the operations of the fused
// form in its order; the two GEMMs sum over (tap, channel) k-steps in MFMA order (rel. 1e-5 vs the chain).
constexpr int kF2TH = 8, kF2TW = 32;  // output tile: 256 pixels, 4 waves
typedef float f2x4 __attribute__((ext_vector_type(4)));
constexpr int kF2Threads = 256;

// the mlp stage weights (SmixLayout blocks), the depthwise weights and bias: staged in LDS by the
// launch's first loads (index order of fmnet_kernel's warm-up)
template <int C, int NSTAGE>
__device__ __forceinline__ void f2_stage_weights(const esm_fmnet_desc& a, const float* dww, const float* dwb,
                                                 float (&rw)[(NSTAGE * SmixLayout<C>::STAGE + C * 49 + C +
                                                               kF2Threads - 1) / kF2Threads]) {
    using Lyt = SmixLayout<C>;
    constexpr int NW = NSTAGE * Lyt::STAGE + C * 49 + C;
    constexpr int NWR = (NW + kF2Threads - 1) / kF2Threads;
    const int tid = threadIdx.x;
#pragma unroll
    for (int k = 0; k < NWR; ++k) {
        const int i = tid + k * kF2Threads;
        const float* p = nullptr;
        int off = 0;
        // stage s's fields with a compile-time index (a run-time a.stage[i / STAGE] puts the kernarg
        // struct in scratch)
        static_for<0, NSTAGE>([&](auto sc) {
            constexpr int S = decltype(sc)::value;
            const int j = i - S * Lyt::STAGE;
            if (j >= 0 && j < Lyt::STAGE) {
                const esm_smix_stage& g = a.stage[S];
                p = j < Lyt::F0W ? g.ln_w : j < Lyt::F0B ? g.fc0_w : j < Lyt::F2W ? g.fc0_b : j < Lyt::F2B ? g.fc2_w : g.fc2_b;
                off = j - (j < Lyt::F0W ? Lyt::LN : j < Lyt::F0B ? Lyt::F0W : j < Lyt::F2W ? Lyt::F0B : j < Lyt::F2B ? Lyt::F2W : Lyt::F2B);
            }
        });
        if (i >= NSTAGE * Lyt::STAGE && i < NW) {
            const int j = i - NSTAGE * Lyt::STAGE;
            p = j < C * 49 ? dww : dwb;
            off = j < C * 49 ? j : j - C * 49;
        }
        rw[k] = (p ? p : dww)[p ? off : 0];
    }
}

// depthwise 7x7 + bias of an OH x OW region from the [C][SH][SWP] LDS image src (region row r reads source
// rows r .. r + 6) into dst [C][OH][DWS] (row stride DWS >= OW); a wave owns a channel, a lane 4
// consecutive outputs of a row
template <int C, int OH, int OW, int SH, int SWP, int DWS = OW>
__device__ __forceinline__ void f2_dw(const float* src, float* dst, const float* lw, const float* lb, int wave, int lane) {
    constexpr int SEG = 4, NSEG = (OW + SEG - 1) / SEG, ITEMS = OH * NSEG, NWAVES = kF2Threads / 64;
    for (int c = wave; c < C; c += NWAVES) {
        float w[49];
#pragma unroll
        for (int i = 0; i < 49; ++i) w[i] = lw[c * 49 + i];
        const float bias = lb[c];
        for (int it = lane; it < ITEMS; it += 64) {
            const int py = it / NSEG, px0 = (it - py * NSEG) * SEG;
            float acc[SEG];
#pragma unroll
            for (int j = 0; j < SEG; ++j) acc[j] = 0.f;
#pragma unroll
            for (int ky = 0; ky < 7; ++ky) {
                float row[SEG + 6];
                const float* sr = src + (c * SH + py + ky) * SWP + px0;
#pragma unroll
                for (int j = 0; j < SEG + 6; ++j) row[j] = sr[j];
#pragma unroll
                for (int kx = 0; kx < 7; ++kx)
#pragma unroll
                    for (int j = 0; j < SEG; ++j) acc[j] += w[ky * 7 + kx] * row[j + kx];
            }
#pragma unroll
            for (int j = 0; j < SEG; ++j)
                if (px0 + j < OW) dst[(c * OH + py) * DWS + px0 + j] = acc[j] + bias;
        }
    }
}

template <int C>
__global__ void __launch_bounds__(kF2Threads) fm2a_kernel(const esm_fmnet_desc a) {
    using Lyt = SmixLayout<C>;
    constexpr int TH = kF2TH, TW = kF2TW;
    constexpr int AH = TH + 6, AW = TW + 6, AP = AH * AW, AWP = AW + 1 + 6;  // + slack for the 4-wide dw reads
    constexpr int NW = 3 * Lyt::STAGE + C * 49 + C;
    constexpr int NWR = (NW + kF2Threads - 1) / kF2Threads;
    constexpr int NPA = (AP + kF2Threads - 1) / kF2Threads;  // region-A pixels per thread
    __shared__ float sw[NW];
    __shared__ float sa[C * AH * AWP];
    __shared__ float sb[C * TH * TW];
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int H = a.H, W = a.W, b = blockIdx.z;
    const int y0 = blockIdx.y * TH, x0 = blockIdx.x * TW;
    const long long plane = static_cast<long long>(H) * W;
    const float* xb = a.x + static_cast<long long>(b) * C * plane;

    // weights (stages: SMLayer0.mlp1, SMLayer0.mlp2, SMLayer1.mlp1; dw0) and region A's pixels, one batch
    float rw[NWR];
    f2_stage_weights<C, 3>(a, a.dw_w[0], a.dw_b[0], rw);
    float t[NPA][C];
    bool in[NPA];
#pragma unroll
    for (int k = 0; k < NPA; ++k) {
        const int p = tid + k * kF2Threads;
        const int py = p / AW, px = p - (p / AW) * AW;
        const int gy = y0 - 3 + py, gx = x0 - 3 + px;
        in[k] = p < AP && gy >= 0 && gy < H && gx >= 0 && gx < W;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float v = xb[in[k] ? c * plane + gy * W + gx : 0];
            t[k][c] = in[k] ? v : 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < NWR; ++k)
        if (tid + k * kF2Threads < NW) sw[tid + k * kF2Threads] = rw[k];
    __syncthreads();
    // t1 = SMLayer0.mlp1 (x) on region A (zero outside the image: dw0's padding)
#pragma unroll
    for (int k = 0; k < NPA; ++k) {
        const int p = tid + k * kF2Threads;
        if (p >= AP) continue;
        const int py = p / AW, px = p - (p / AW) * AW;
        if (in[k]) mix_stage<C>(t[k], sw);
#pragma unroll
        for (int c = 0; c < C; ++c) sa[(c * AH + py) * AWP + px] = in[k] ? t[k][c] : 0.f;
    }
    __syncthreads();
    f2_dw<C, TH, TW, AH, AWP>(sa, sb, sw + 3 * Lyt::STAGE, sw + 3 * Lyt::STAGE + C * 49, wave, lane);
    __syncthreads();
    // d = SMLayer1.mlp1 (SMLayer0.mlp2 (dw0)) on the tile -> work
    {
        const int py = tid / TW, px = tid - (tid / TW) * TW;
        const int gy = y0 + py, gx = x0 + px;
        if (gy < H && gx < W) {
            float u[C];
#pragma unroll
            for (int c = 0; c < C; ++c) u[c] = sb[(c * TH + py) * TW + px];
            mix_stage<C>(u, sw + Lyt::STAGE);
            mix_stage<C>(u, sw + 2 * Lyt::STAGE);
            float* wb = a.work + static_cast<long long>(b) * C * plane + gy * W + gx;
#pragma unroll
            for (int c = 0; c < C; ++c) wb[c * plane] = u[c];
        }
    }
}

template <int C>
__global__ void __launch_bounds__(kF2Threads) fm2b_kernel(const esm_fmnet_desc a) {
    using Lyt = SmixLayout<C>;
    constexpr int HID = C + 16, HT = 2;                      // hidden channels, their 16-row MFMA tiles
    constexpr int TH = kF2TH, TW = kF2TW;
    constexpr int DH = TH + 8, DW = TW + 8, DP = DH * DW, DWP = DW + 1 + 6;  // d on tile + 4
    constexpr int CH = TH + 2, CW = TW + 2, CP = CH * CW, CWP = CW + 2;      // t3 on tile + 1
    constexpr int NW1 = Lyt::STAGE + C * 49 + C;                             // mlp2_1, dw1
    constexpr int W0 = 9 * C * 32, B0 = 32, W2 = 32 * 16, B2 = 16;           // conv0 [tap][c][32], conv2 [h][16]
    constexpr int NW = NW1 + W0 + B0 + W2 + B2;
    constexpr int NWR = (NW + kF2Threads - 1) / kF2Threads;
    constexpr int NPD = (DP + kF2Threads - 1) / kF2Threads;
    constexpr int NPC = (CP + kF2Threads - 1) / kF2Threads;
    constexpr int SH_ = C * DH * DWP > HID * TH * TW ? C * DH * DWP : HID * TH * TW;
    __shared__ float sw[NW];
    __shared__ float sd[SH_];        // d on region D, then h = silu(conv0 + b0) [HID][TH * TW]
    __shared__ float sc_[C * CH * CWP];  // dw1 on region C, then t3 in place
    const int tid = threadIdx.x;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
    const int g = lane >> 4, n = lane & 15;
    const int H = a.H, W = a.W, b = blockIdx.z;
    const int y0 = blockIdx.y * TH, x0 = blockIdx.x * TW;
    const long long plane = static_cast<long long>(H) * W;
    const float* db = a.work + static_cast<long long>(b) * C * plane;
    const float* xb = a.x + static_cast<long long>(b) * C * plane;

    // weights: mlp2_1 + dw1 (as fm2a), conv0 as the MFMA A image [tap][c][32 hidden] (zero past HID), b0,
    // conv2 as [h][16 out channels] (zero past C), b2
    float rw[NWR];
#pragma unroll
    for (int k = 0; k < NWR; ++k) {
        const int i = tid + k * kF2Threads;
        const float* p = nullptr;
        int off = 0;
        if (i < Lyt::STAGE) {
            const esm_smix_stage& st = a.stage[3];
            const int j = i;
            p = j < Lyt::F0W ? st.ln_w : j < Lyt::F0B ? st.fc0_w : j < Lyt::F2W ? st.fc0_b : j < Lyt::F2B ? st.fc2_w : st.fc2_b;
            off = j - (j < Lyt::F0W ? Lyt::LN : j < Lyt::F0B ? Lyt::F0W : j < Lyt::F2W ? Lyt::F0B : j < Lyt::F2B ? Lyt::F2W : Lyt::F2B);
        } else if (i < NW1) {
            const int j = i - Lyt::STAGE;
            p = j < C * 49 ? a.dw_w[1] : a.dw_b[1];
            off = j < C * 49 ? j : j - C * 49;
        } else if (i < NW1 + W0) {  // conv0_w [HID][C][3][3] -> [tap][c][h]
            const int j = i - NW1;
            const int h = j % 32, c = (j / 32) % C, tap = j / (32 * C);
            if (h < HID) {
                p = a.conv0_w;
                off = (h * C + c) * 9 + tap;
            }
        } else if (i < NW1 + W0 + B0) {
            const int h = i - NW1 - W0;
            if (h < HID) {
                p = a.conv0_b;
                off = h;
            }
        } else if (i < NW1 + W0 + B0 + W2) {  // conv2_w [C][HID] -> [h][16]
            const int j = i - NW1 - W0 - B0;
            const int co = j % 16, h = j / 16;
            if (co < C && h < HID) {
                p = a.conv2_w;
                off = co * HID + h;
            }
        } else if (i < NW) {
            const int co = i - NW1 - W0 - B0 - W2;
            if (co < C) {
                p = a.conv2_b;
                off = co;
            }
        }
        const float v = (p ? p : a.x)[p ? off : 0];
        rw[k] = p ? v : 0.f;
    }
    // d on region D (zero outside the image: dw1's padding); x on region C (t3's residual), in registers
#pragma unroll
    for (int k = 0; k < NPD; ++k) {
        const int p = tid + k * kF2Threads;
        const int py = p / DW, px = p - (p / DW) * DW;
        const int gy = y0 - 4 + py, gx = x0 - 4 + px;
        const bool ok = p < DP && gy >= 0 && gy < H && gx >= 0 && gx < W;
        float v[C];
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float u = db[ok ? c * plane + gy * W + gx : 0];
            v[c] = ok ? u : 0.f;
        }
        if (p < DP) {
#pragma unroll
            for (int c = 0; c < C; ++c) sd[(c * DH + py) * DWP + px] = v[c];
        }
    }
    float xr[NPC][C];
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
        const int p = tid + k * kF2Threads;
        const int py = p / CW, px = p - (p / CW) * CW;
        const int gy = y0 - 1 + py, gx = x0 - 1 + px;
        const bool ok = p < CP && gy >= 0 && gy < H && gx >= 0 && gx < W;
#pragma unroll
        for (int c = 0; c < C; ++c) {
            const float u = xb[ok ? c * plane + gy * W + gx : 0];
            xr[k][c] = ok ? u : 0.f;
        }
    }
#pragma unroll
    for (int k = 0; k < NWR; ++k)
        if (tid + k * kF2Threads < NW) sw[tid + k * kF2Threads] = rw[k];
    __syncthreads();
    // dw1 on region C
    f2_dw<C, CH, CW, DH, DWP, CWP>(sd, sc_, sw + Lyt::STAGE, sw + Lyt::STAGE + C * 49, wave, lane);
    __syncthreads();
    // t3 = SMLayer1.mlp2 (dw1) + x on region C, zero outside the image (conv0's padding), in place
#pragma unroll
    for (int k = 0; k < NPC; ++k) {
        const int p = tid + k * kF2Threads;
        if (p >= CP) continue;
        const int py = p / CW, px = p - (p / CW) * CW;
        const int gy = y0 - 1 + py, gx = x0 - 1 + px;
        const bool ok = gy >= 0 && gy < H && gx >= 0 && gx < W;
        float u[C];
#pragma unroll
        for (int c = 0; c < C; ++c) u[c] = sc_[(c * CH + py) * CWP + px];
        if (ok) mix_stage<C>(u, sw);
#pragma unroll
        for (int c = 0; c < C; ++c) sc_[(c * CH + py) * CWP + px] = ok ? u[c] + xr[k][c] : 0.f;
    }
    __syncthreads();
    // h = silu(conv0(t3) + b0) on the tile (MFMA): wave w owns tile rows 2w, 2w + 1 (N tiles: 16 pixels of
    // a row half), both 16-row hidden tiles; A = conv0 [tap][c][h], B = t3 window rows
    const float* w0 = sw + NW1;
    f2x4 acc[4][HT];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
        for (int mt = 0; mt < HT; ++mt) acc[nt][mt] = f2x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
        const int dy = tap / 3, dx = tap % 3;
#pragma unroll
        for (int ks = 0; ks < C / 4; ++ks) {
            const int c = 4 * ks + g;
            float av[HT];
#pragma unroll
            for (int mt = 0; mt < HT; ++mt) av[mt] = w0[(tap * C + c) * 32 + 16 * mt + n];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const int row = 2 * wave + (nt >> 1), col = 16 * (nt & 1) + n;
                const float bv = sc_[(c * CH + row + dy) * CWP + col + dx];
#pragma unroll
                for (int mt = 0; mt < HT; ++mt)
                    acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], bv, acc[nt][mt], 0, 0, 0);
            }
        }
    }
    __syncthreads();  // every wave is done reading d (sd) before h overwrites it
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int pp = (2 * wave + (nt >> 1)) * TW + 16 * (nt & 1) + n;
#pragma unroll
        for (int mt = 0; mt < HT; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int h = 16 * mt + 4 * g + j;
                if (h < HID) sd[h * (TH * TW) + pp] = silu_fast(acc[nt][mt][j] + w0[W0 + h]);
            }
    }
    __syncthreads();
    // out = conv2(h) + b2 + t3 on the tile (MFMA): A = conv2 [h][16], B = h
    const float* w2 = sw + NW1 + W0 + B0;
    f2x4 o[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) o[nt] = f2x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < HID / 4; ++ks) {
        const int h = 4 * ks + g;
        const float av = w2[h * 16 + n];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const int pp = (2 * wave + (nt >> 1)) * TW + 16 * (nt & 1) + n;
            o[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, sd[h * (TH * TW) + pp], o[nt], 0, 0, 0);
        }
    }
    float* ob = a.out + static_cast<long long>(b) * C * plane;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int row = 2 * wave + (nt >> 1), col = 16 * (nt & 1) + n;
        const int gy = y0 + row, gx = x0 + col;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * g + j;
            if (co < C && gy < H && gx < W)
                ob[co * plane + gy * W + gx] = o[nt][j] + w2[W2 + co] + sc_[(co * CH + row + 1) * CWP + col + 1];
        }
    }
}

}  // namespace

int launch_smix(const esm_smix_desc* d, hipStream_t s) {
    if (!d) return arg_error("smix: null descriptor");
    const esm_smix_desc& a = *d;
    if (!a.x || !a.out) return arg_error("smix: null pointer");
    if (a.B <= 0 || a.H <= 0 || a.W <= 0) return arg_error("smix: bad size");
    if (a.nstages < 0 || a.nstages > ESM_SMIX_MAX_STAGES) return arg_error("smix: nstages must be 0..2");
    if (a.dw_w && !a.dw_b) return arg_error("smix: depthwise conv needs a bias");
    if (a.x == a.out && a.dw_w) return arg_error("smix: depthwise conv cannot run in place");
    for (int i = 0; i < a.nstages; ++i) {
        const esm_smix_stage& st = a.stage[i];
        if (!st.ln_w || !st.fc0_w || !st.fc0_b || !st.fc2_w || !st.fc2_b) return arg_error("smix: null stage weights");
    }
    if (a.C == 8) return launch_c<8>(a, s);
    if (a.C == 16) return launch_c<16>(a, s);
    set_error("smix: C must be 8 or 16");
    return ESM_ERR_UNSUPPORTED;
}

int launch_fmnet(const esm_fmnet_desc* d, hipStream_t s) {
    if (!d) return arg_error("fmnet: null descriptor");
    const esm_fmnet_desc& a = *d;
    if (!a.x || !a.out || !a.dw_w[0] || !a.dw_b[0] || !a.dw_w[1] || !a.dw_b[1]) return arg_error("fmnet: null pointer");
    if (a.x == a.out) return arg_error("fmnet: cannot run in place");
    if (a.B <= 0 || a.H <= 0 || a.W <= 0) return arg_error("fmnet: bad size");
    for (int i = 0; i < 4; ++i) {
        const esm_smix_stage& st = a.stage[i];
        if (!st.ln_w || !st.fc0_w || !st.fc0_b || !st.fc2_w || !st.fc2_b) return arg_error("fmnet: null stage weights");
    }
    if (a.dw_k != 7) {
        set_error("fmnet: depthwise kernel must be 7 (FMBlock kernel_size)");
        return ESM_ERR_UNSUPPORTED;
    }
    const bool conv = a.conv0_w != nullptr;
    if (conv && (!a.conv0_b || !a.conv2_w || !a.conv2_b || a.hid != a.C + 16))
        return arg_error("fmnet: the fused FMBlock.conv needs conv0/conv2 weights and biases, hid = C + 16");
    if (conv && a.work) {  // two launches (large maps): fm2a writes d to work, fm2b the block's output
        if (a.work == a.x || a.work == a.out) return arg_error("fmnet: work must not alias x / out");
        const dim3 grid2(ceil_div(a.W, kF2TW), ceil_div(a.H, kF2TH), a.B);
        if (grid2.y > 65535u || grid2.z > 65535u) return arg_error("fmnet: grid too large");
        if (a.C == 8) {
            hipLaunchKernelGGL((fm2a_kernel<8>), grid2, dim3(kF2Threads), 0, s, a);
            hipLaunchKernelGGL((fm2b_kernel<8>), grid2, dim3(kF2Threads), 0, s, a);
        } else if (a.C == 16) {
            hipLaunchKernelGGL((fm2a_kernel<16>), grid2, dim3(kF2Threads), 0, s, a);
            hipLaunchKernelGGL((fm2b_kernel<16>), grid2, dim3(kF2Threads), 0, s, a);
        } else {
            set_error("fmnet: C must be 8 or 16");
            return ESM_ERR_UNSUPPORTED;
        }
        return check_launch("fmnet(two launches)");
    }
    const bool tall = conv && static_cast<long long>(ceil_div(a.W, kFConvTW)) * ceil_div(a.H, 3) * a.B >= kFConvTallMinTiles;
    const int th = conv ? (tall ? 3 : 1) : 4;
    const dim3 grid(ceil_div(a.W, conv ? kFConvTW : kFTW), ceil_div(a.H, th), a.B);
    if (a.C == 8) {
        if (tall) hipLaunchKernelGGL((fmnet_kernel<8, 7, true, 24, 3>), grid, dim3(kFThreads), 0, s, a);
        else if (conv) hipLaunchKernelGGL((fmnet_kernel<8, 7, true, 24, 1, 1024>), grid, dim3(1024), 0, s, a);
        else hipLaunchKernelGGL((fmnet_kernel<8, 7, false, 1>), grid, dim3(kFThreads), 0, s, a);
    } else if (a.C == 16) {
        if (tall) hipLaunchKernelGGL((fmnet_kernel<16, 7, true, 32, 3>), grid, dim3(kFThreads), 0, s, a);
        else if (conv) hipLaunchKernelGGL((fmnet_kernel<16, 7, true, 32>), grid, dim3(kFThreads), 0, s, a);
        else hipLaunchKernelGGL((fmnet_kernel<16, 7, false, 1>), grid, dim3(kFThreads), 0, s, a);
    } else {
        set_error("fmnet: C must be 8 or 16");
        return ESM_ERR_UNSUPPORTED;
    }
    return check_launch("fmnet");
}

}  // namespace esm

extern "C" int esm_fmnet_f32(const esm_fmnet_desc* desc, void* stream) {
    return esm::launch_fmnet(desc, esm::as_stream(stream));
}

#ifdef ESM_CONV_STAMPS
// Diagnostic build only: copy n <= 4096 * 8 fmnet phase stamps to the host.
extern "C" int esm_diag_fmnet_stamps(unsigned long long* host, int n) {
    if (n > 4096 * 8) n = 4096 * 8;
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(esm::fm_stamps), 8ull * n) == hipSuccess ? n : -1;
}
#endif

extern "C" int esm_smix_f32(const esm_smix_desc* desc, void* stream) {
    return esm::launch_smix(desc, esm::as_stream(stream));
}
