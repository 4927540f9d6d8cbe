// Register-resident-weight plane-streaming 3-D convolution (3x3x3, stride 1, padding 1, Cout <= 16):
// the 3-D stems of the hot path, group_stem (32 -> 8), corr_stem (1 -> 8) and agg (8 -> 8)
// (models/ESMStereo.py:610,620,622, used at :703-715; BasicConv, models/submodule.py:12-38), which at
// ESMStereo-L KITTI are a fifth of the whole step.
//
// The 3-D analogue of conv_wide.hip.  A workgroup owns one 16-pixel column strip of one output row y
// and a block of Z output planes; its 4 waves split the work KSW ways over 4-channel groups (wave
// w takes groups w % KSW, w % KSW + KSW, ...) and 4 / KSW ways over sub-blocks of the planes.  A wave
// keeps its groups' 27-tap weights in VGPRs and streams input planes: plane zi's 9 in-plane taps are
// 9 buffer_loads per group (3 rows x 3 column shifts, kOOB-marked borders), and each feeds the MFMAs
// of the three output planes zi + 1, zi, zi - 1 (tap plane dz = 0, 1, 2), so a loaded operand is
// used three times and consecutive MFMAs go to different planes' accumulators.  The loop over input
// planes is unrolled (compile-time Z) and only (input, output) plane pairs inside the block are
// multiplied.  With <= 8 couts the 16 MFMA rows carry two output planes (a plane pair), so no row
// is padding.  The waves' partial tiles meet in LDS at the end and are added in a fixed order
// (deterministic); every thread then finishes its (plane, cout, pixel) elements.
#include <cstdlib>

#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

// KSW x ZS waves per workgroup: KSW ways over channel groups, ZS plane sub-blocks
template <int KSW, int NGW, int ZW, int ACT, bool PLAIN, bool PZ, int ZS = 4 / KSW>
__global__ void __launch_bounds__(64 * KSW * ZS) wconv3_kernel(const esm_conv_desc a) {
    constexpr int kW3Threads = 64 * KSW * ZS;
    constexpr int NZ = ZW + 2;         // input planes a wave streams
    constexpr int ZB = ZW * ZS;        // output planes per workgroup
    // PZ (<= 8 couts): the 16 MFMA rows hold 8 couts x 2 output planes (a plane pair 2q, 2q + 1), so
    // no row is padding.  Input plane z0 - 1 + p reaches pair q through relative plane r = p - 2q in
    // 0..3: rows 0-7 use tap plane dz = r (if <= 2), rows 8-15 dz = r - 1 (if >= 0); 4 weight sets
    constexpr int NA = PZ ? ZW / 2 : ZW;  // accumulators (pairs or planes)
    static_assert(!PZ || ZW % 2 == 0, "plane pairs need an even plane block");
    __shared__ __attribute__((aligned(16))) float red[KSW * ZS][NA][4][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15, kq = lane >> 4;
    const int kpart = wave % KSW, zpart = wave / KSW;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int x0 = bk_.x * 16;
    const int y = bk_.y;
    const int nzb = (a.Do + ZB - 1) / ZB;
    const int b = bk_.z / nzb;
    const int z0 = (bk_.z - b * nzb) * ZB + zpart * ZW;  // this wave's first output plane

    // ---- weights of the wave's groups -> VGPRs: w[tap][cin_pad][cout_pad], tap = (dz*3 + dy)*3 + dx
    constexpr int NWS = PZ ? 4 : 3;  // weight sets: tap planes dz (or the pair-relative planes r)
    float wv[NGW][NWS][9];
    {
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.w), static_cast<short>(0), 4 * 27 * a.cin_pad * a.cout_pad, 0x00020000);
        const unsigned wl = 4u * (kq * a.cout_pad + (PZ ? (n16 & 7) : n16));
#pragma unroll
        for (int i = 0; i < NGW; ++i) {
            const int g = kpart + i * KSW;
#pragma unroll
            for (int r = 0; r < NWS; ++r)
#pragma unroll
                for (int t = 0; t < 9; ++t) {
                    int dz = r;
                    if constexpr (PZ) dz = n16 < 8 ? r : r - 1;  // per-lane: rows 8-15 lag one plane
                    const bool ok = dz >= 0 && dz <= 2;
                    const float v = buf_load_s(wrs, ok ? wl : kOOB, 4 * (((ok ? dz : 0) * 9 + t) * a.cin_pad + 4 * g) * a.cout_pad);
                    wv[i][r][t] = v;  // past cin_pad or an invalid plane: out of range -> 0
                }
        }
    }
    // ---- input addressing (one source)
    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (a.Di - 1) * sd + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const int xo = x0 + n16;
    unsigned vo[NGW][3];  // group i's channel at column shift dx
#pragma unroll
    for (int i = 0; i < NGW; ++i) {
        const int c = 4 * (kpart + i * KSW) + kq;
#pragma unroll
        for (int dx = 0; dx < 3; ++dx) {
            const int xi = xo - 1 + dx;
            vo[i][dx] = (c < a.Cin && xo < a.Wo && xi >= 0 && xi < a.Wi) ? 4u * (c * sc + xi) : kOOB;
        }
    }
    // plane / row offsets are unsigned: two kOOB marks add to 2^31 without signed overflow, and the
    // sum is cast once at the soffset operand (past the end of the buffer either way)
    unsigned roff[3];  // rows y - 1 .. y + 1 (kOOB outside)
#pragma unroll
    for (int dy = 0; dy < 3; ++dy) {
        const int yi = y - 1 + dy;
        roff[dy] = (yi >= 0 && yi < a.Hi) ? 4u * yi * sh : kOOB;
    }
    auto load_plane = [&](float (&d)[NGW][9], int zi) {
        const unsigned poff = (zi >= 0 && zi < a.Di) ? 4u * zi * sd : kOOB;
#pragma unroll
        for (int i = 0; i < NGW; ++i)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    d[i][dy * 3 + dx] = buf_load_s(rs, vo[i][dx], static_cast<int>(poff + roff[dy]));
    };

    floatx4 acc[NA];
#pragma unroll
    for (int z = 0; z < NA; ++z) acc[z] = floatx4{0.f, 0.f, 0.f, 0.f};
    float bin[2][NGW][9];
    load_plane(bin[0], z0 - 1);
#pragma unroll
    for (int p = 0; p < NZ; ++p) {  // input plane z0 - 1 + p
        if (p + 1 < NZ) load_plane(bin[(p + 1) & 1], z0 + p);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int i = 0; i < NGW; ++i)
#pragma unroll
            for (int t9 = 0; t9 < 9; ++t9)
#pragma unroll
                for (int k = 0; k < (PZ ? 2 : 3); ++k) {
                    if constexpr (PZ) {  // pairs q with r = p - 2q in 0..3
                        const int q = p / 2 - k;
                        const int r = p - 2 * q;
                        if (q < 0 || q >= NA || r > 3) continue;
                        acc[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[i][r][t9], bin[p & 1][i][t9], acc[q], 0, 0, 0);
                    } else {  // output planes p - dz
                        const int zo = p - k;
                        if (zo < 0 || zo >= ZW) continue;
                        acc[zo] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[i][k][t9], bin[p & 1][i][t9], acc[zo], 0, 0, 0);
                    }
                }
    }

    // ---- K-split partial sums: LDS [wave][acc][j][lane], fixed-order sum over the KSW parts
#pragma unroll
    for (int z = 0; z < NA; ++z)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[wave][z][j][lane] = acc[z][j];
    __syncthreads();
    // elements (plane sub-block zp, accumulator z, j, lane) over the 256 threads, lane fastest
    constexpr int NEL = ZS * NA * 4 * 64;                      // elements (zp, z, j, lane)
    constexpr int NE = (NEL + kW3Threads - 1) / kW3Threads;  // elements per thread
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) + (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
    const int zbase = (bk_.z - b * nzb) * ZB;
#pragma unroll
    for (int e = 0; e < NE; ++e) {
        const int idx = e * kW3Threads + static_cast<int>(threadIdx.x);  // over (zp, z, j, lane)
        if (NEL % kW3Threads != 0 && idx >= NEL) break;
        const int l = idx & 63, j = (idx >> 6) & 3, zz = idx >> 8;       // zz = zp * NA + z (= e)
        const int zp = zz / NA, z = zz - zp * NA;
        float v = red[zp * KSW][z][j][l];
#pragma unroll
        for (int k = 1; k < KSW; ++k) v += red[zp * KSW + k][z][j][l];
        const int row = 4 * (l >> 4) + j;                      // MFMA row of the element
        const int co = PZ ? (row & 7) : row;
        const int zo = zbase + zp * ZW + (PZ ? 2 * z + (row >> 3) : z);
        const int px = x0 + (l & 15);
        const float sc_ = a.scale ? a.scale[min(co, a.Cout - 1)] : 1.f;
        const float sh_ = a.shift ? a.shift[min(co, a.Cout - 1)] : 0.f;
        v = a.scale ? v * sc_ + sh_ : v + sh_;
        v = act_t<ACT>(v, a.act);
        if constexpr (PLAIN) {
            const unsigned o = (co < a.Cout && px < a.Wo && zo < a.Do)
                                   ? 4u * (co * static_cast<int>(a.oc) + zo * static_cast<int>(a.od) + y * static_cast<int>(a.oh) + px)
                                   : kOOB;
            store_b32(__float_as_uint(v), ro_, static_cast<int>(o), 0);
        } else {
            if (co >= a.Cout || px >= a.Wo || zo >= a.Do) continue;
            if (a.mul) v = v * a.mul[b * a.mb + co * a.mc + static_cast<long long>(y) * a.mh + px];
            if (a.res) v = v + a.res[b * a.rb + co * a.rc + static_cast<long long>(zo) * a.rd + static_cast<long long>(y) * a.rh + px];
            const long long o = b * a.ob + co * a.oc + static_cast<long long>(zo) * a.od + static_cast<long long>(y) * a.oh + px;
            a.out[o] = v * a.post_scale;
            if (a.out2) a.out2[o] = v * a.post_scale2;
        }
    }
}

// Row-streaming variant for the small volumes (S-K group_stem: 32 -> 8 on 12x24x78), where the plane-pair
// form above with one output row per workgroup re-fetched every weight once per workgroup and every input
// row three times from L2: 720 workgroups x 8 waves x (36 weight + 36 input loads) ~ 106 MB of L2 -> CU
// traffic for 3.7 MB of algorithmic bytes.  Here a workgroup owns RB consecutive output rows of its
// 16-column strip and plane pair: each wave (one 4-channel group) loads its 36 weight operands once and
// streams input rows through a 4-row register ring (load row y + 2 while the MFMAs of row y run), so per
// output row it loads 12 input operands instead of 36.  Per wave and output row the MFMAs run in the
// same order as wconv3_kernel<8, 1, 2, ..> (input plane, then tap), and the 8 waves' partial tiles are
// added in the same fixed order: results are bit-identical to that form.
template <int KSW, int RB, int ACT, bool PLAIN>
__global__ void __launch_bounds__(64 * KSW) wconv3r_kernel(const esm_conv_desc a) {
    constexpr int NT = 64 * KSW;
    __shared__ __attribute__((aligned(16))) float red[KSW][RB][4][64];
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15, kq = lane >> 4;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int x0 = bk_.x * 16;
    const int y0 = bk_.y * RB;
    const int nzb = (a.Do + 1) / 2;
    const int b = bk_.z / nzb;
    const int z0 = (bk_.z - b * nzb) * 2;  // the plane pair z0, z0 + 1

    // weights of group `wave` for the 4 pair-relative input planes (rows 8-15 of the MFMA lag one plane)
    float wv[4][9];
    {
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.w), static_cast<short>(0), 4 * 27 * a.cin_pad * a.cout_pad, 0x00020000);
        const unsigned wl = 4u * (kq * a.cout_pad + (n16 & 7));
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int t = 0; t < 9; ++t) {
                const int dz = n16 < 8 ? r : r - 1;
                const bool ok = dz >= 0 && dz <= 2;
                wv[r][t] = buf_load_s(wrs, ok ? wl : kOOB, 4 * (((ok ? dz : 0) * 9 + t) * a.cin_pad + 4 * wave) * a.cout_pad);
            }
    }
    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (a.Di - 1) * sd + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const int xo = x0 + n16;
    const int c = 4 * wave + kq;
    unsigned vo[3];
#pragma unroll
    for (int dx = 0; dx < 3; ++dx) {
        const int xi = xo - 1 + dx;
        vo[dx] = (c < a.Cin && xo < a.Wo && xi >= 0 && xi < a.Wi) ? 4u * (c * sc + xi) : kOOB;
    }
    unsigned poff[4];  // input planes z0 - 1 .. z0 + 2 (kOOB outside; unsigned as in wconv3_kernel)
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int zi = z0 - 1 + p;
        poff[p] = (zi >= 0 && zi < a.Di) ? 4u * zi * sd : kOOB;
    }
    // ring of input rows: row yi = y0 - 1 + k lives in slot k % 4
    float ring[4][4][3];  // [slot][plane][dx]
    auto load_row = [&](float (&d)[4][3], int k) {
        const int yi = y0 - 1 + k;
        const unsigned ro = (yi >= 0 && yi < a.Hi) ? 4u * yi * sh : kOOB;
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) d[p][dx] = buf_load_s(rs, vo[dx], static_cast<int>(poff[p] + ro));
    };
    load_row(ring[0], 0);
    load_row(ring[1], 1);
    floatx4 acc[RB];
#pragma unroll
    for (int r = 0; r < RB; ++r) {
        acc[r] = floatx4{0.f, 0.f, 0.f, 0.f};
        load_row(ring[(r + 2) & 3], r + 2);  // output row y0 + r needs input rows r .. r + 2 (ring index)
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int p = 0; p < 4; ++p)
#pragma unroll
            for (int dy = 0; dy < 3; ++dy)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx)
                    acc[r] = __builtin_amdgcn_mfma_f32_16x16x4f32(wv[p][dy * 3 + dx], ring[(r + dy) & 3][p][dx], acc[r], 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int j = 0; j < 4; ++j) red[wave][r][j][lane] = acc[r][j];
    __syncthreads();
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) + (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
    constexpr int NEL = RB * 4 * 64;  // elements (r, j, lane)
#pragma unroll
    for (int e = 0; e < (NEL + NT - 1) / NT; ++e) {
        const int idx = e * NT + static_cast<int>(threadIdx.x);
        if (NEL % NT != 0 && idx >= NEL) break;
        const int l = idx & 63, j = (idx >> 6) & 3, r = idx >> 8;
        float v = red[0][r][j][l];
#pragma unroll
        for (int k = 1; k < KSW; ++k) v += red[k][r][j][l];
        const int row = 4 * (l >> 4) + j;
        const int co = row & 7;
        const int zo = z0 + (row >> 3);
        const int y = y0 + r;
        const int px = x0 + (l & 15);
        const float sc_ = a.scale ? a.scale[min(co, a.Cout - 1)] : 1.f;
        const float sh_ = a.shift ? a.shift[min(co, a.Cout - 1)] : 0.f;
        v = a.scale ? v * sc_ + sh_ : v + sh_;
        v = act_t<ACT>(v, a.act);
        if constexpr (PLAIN) {
            const unsigned o = (co < a.Cout && px < a.Wo && zo < a.Do && y < a.Ho)
                                   ? 4u * (co * static_cast<int>(a.oc) + zo * static_cast<int>(a.od) + y * static_cast<int>(a.oh) + px)
                                   : kOOB;
            store_b32(__float_as_uint(v), ro_, static_cast<int>(o), 0);
        } else {
            if (co >= a.Cout || px >= a.Wo || zo >= a.Do || y >= a.Ho) continue;
            if (a.mul) v = v * a.mul[b * a.mb + co * a.mc + static_cast<long long>(y) * a.mh + px];
            if (a.res) v = v + a.res[b * a.rb + co * a.rc + static_cast<long long>(zo) * a.rd + static_cast<long long>(y) * a.rh + px];
            const long long o = b * a.ob + co * a.oc + static_cast<long long>(zo) * a.od + static_cast<long long>(y) * a.oh + px;
            a.out[o] = v * a.post_scale;
            if (a.out2) a.out2[o] = v * a.post_scale2;
        }
    }
}

// output rows per workgroup of the row-streaming variant (A/B: ESM_W3_ROWS=1 disables it, read only with
// ESM_AB=1 so that a caller's environment never selects an untested form).  Measured at S-K
// (scripts/gpu_r03_w3rows.sh, two rotations): RB 1 / 2 / 3 / 4 -> group_stem in the replayed step 13.6 /
// 13.4 / 10.1 / 11.5-12.2 us.  Neither two accumulators per row nor the same form for the 8 -> 8 `agg`
// (2 waves) measured faster; both were removed.
static const int kW3Rows = [] {
    const char* ab = getenv("ESM_AB");
    const char* e = ab && ab[0] == '1' && ab[1] == 0 ? getenv("ESM_W3_ROWS") : nullptr;
    return e ? atoi(e) : 3;
}();
template <int KSW, int RB>
int launch_w3r(const esm_conv_desc& a, hipStream_t s) {
    const long long z = static_cast<long long>(a.B) * ((a.Do + 1) / 2);
    if (z > 65535) return arg_error("conv(wide3r): grid too large");
    const dim3 grid(ceil_div(a.Wo, 16), ceil_div(a.Ho, RB), static_cast<unsigned>(z));
    const bool plain = a.act == ESM_ACT_GELU && !a.res && !a.out2 && !a.mul && a.post_scale == 1.f &&
                       static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Do) * a.od +
                               static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (plain)
        hipLaunchKernelGGL((wconv3r_kernel<KSW, RB, ESM_ACT_GELU, true>), grid, dim3(64 * KSW), 0, s, a);
    else
        hipLaunchKernelGGL((wconv3r_kernel<KSW, RB, -1, false>), grid, dim3(64 * KSW), 0, s, a);
    return check_launch("conv(wide3r)");
}

template <int KSW, int NGW, int ZW, int ZS = 4 / KSW>
int launch_w3(const esm_conv_desc& a, hipStream_t s) {
    constexpr int ZB = ZW * ZS;
    constexpr int kW3Threads = 64 * KSW * ZS;
    const long long z = static_cast<long long>(a.B) * ((a.Do + ZB - 1) / ZB);
    if (a.Ho > 65535 || z > 65535) return arg_error("conv(wide3): grid too large");
    const dim3 grid(ceil_div(a.Wo, 16), static_cast<unsigned>(a.Ho), static_cast<unsigned>(z));
    const bool plain = a.act == ESM_ACT_GELU && !a.res && !a.out2 && !a.mul && a.post_scale == 1.f &&
                       static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Do) * a.od +
                               static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (a.Cout <= 8) {  // plane pairs: no padding MFMA rows
        if (plain)
            hipLaunchKernelGGL((wconv3_kernel<KSW, NGW, ZW, ESM_ACT_GELU, true, true, ZS>), grid, dim3(kW3Threads), 0, s, a);
        else
            hipLaunchKernelGGL((wconv3_kernel<KSW, NGW, ZW, -1, false, true, ZS>), grid, dim3(kW3Threads), 0, s, a);
    } else {
        if (plain)
            hipLaunchKernelGGL((wconv3_kernel<KSW, NGW, ZW, ESM_ACT_GELU, true, false, ZS>), grid, dim3(kW3Threads), 0, s, a);
        else
            hipLaunchKernelGGL((wconv3_kernel<KSW, NGW, ZW, -1, false, false, ZS>), grid, dim3(kW3Threads), 0, s, a);
    }
    return check_launch("conv(wide3)");
}

}  // namespace

// 3x3x3 stride-1 padding-1 3-D convs with <= 16 couts over one source (plain or `* mul` / residual
// epilogues), input channels up to 32.
bool wide3_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (!d3 || a.transposed || a.stride != 1 || a.kd != 3 || a.kh != 3 || a.kw != 3) return false;
    if (a.pd != 1 || a.ph != 1 || a.pw != 1 || a.nsrc != 1 || a.Cout > 16 || a.Cin > 32 || a.up || a.shuffle > 1)
        return false;
    return direct_ok(a);
}

#ifdef ESM_W3_NOSPLIT8
constexpr bool kW3Split8 = false;  // A/B builds
#else
constexpr bool kW3Split8 = true;
#endif

int launch_wide3(const esm_conv_desc& a, hipStream_t s) {
    if (!wide3_ok(a)) return arg_error("conv: wide3-form hint not applicable");
    const int ng = (a.Cin + 3) / 4;
    // plane blocks: 4 planes per wave where the grid stays wide, else 2
    const long long rows = static_cast<long long>(a.B) * a.Ho * ceil_div(a.Wo, 16);
    const long long vox = rows * a.Do;
    if (ng > 4) {  // 5..8 groups: 4 waves split K, 2 groups each; more planes per wave on big volumes
        if (vox >= 16LL * 65536) return launch_w3<4, 2, 8>(a, s);
        if (vox >= 4LL * 16384) return launch_w3<4, 2, 4>(a, s);
        // small volumes (S-K group_stem): 8 waves, one group each, halving each wave's load -> MFMA chain;
        // <= 8 couts: RB output rows per workgroup streamed through a register ring (ESM_W3_ROWS, 1 = off)
        if (a.Cout <= 8 && ng <= 8 && kW3Rows > 1) {
            if (kW3Rows == 2) return launch_w3r<8, 2>(a, s);
            if (kW3Rows == 3) return launch_w3r<8, 3>(a, s);
            return launch_w3r<8, 4>(a, s);
        }
        return kW3Split8 ? launch_w3<8, 1, 2, 1>(a, s) : launch_w3<4, 2, 2>(a, s);
    }
    if (ng > 2) return launch_w3<4, 1, 2>(a, s);  // 3..4 groups: one each
    if (ng == 2) return rows * a.Do >= 4LL * 16384 ? launch_w3<2, 1, 4>(a, s) : launch_w3<2, 1, 2>(a, s);
    return rows * a.Do >= 4LL * 16384 ? launch_w3<1, 1, 4>(a, s) : launch_w3<1, 1, 2>(a, s);
}

}  // namespace conv
}  // namespace esm
