// Row-block LDS-staged 3x3x3 convolution for the narrow 3-D stems (stride 1, padding 1, <= 8 output
// channels, 4..32 input channels in whole 4-channel groups): group_stem (32 -> 8) and agg (8 -> 8)
// of models/ESMStereo.py:620,622 (used at :711-715; BasicConv, models/submodule.py:12-38).
//
// Why: the plane-streaming form (conv_wide3.hip) gives every workgroup ONE output row, so each input
// row is fetched by the three workgroups whose 3x3 windows cover it, and those sit on different XCDs
// (memory-side bytes 6.6x the algorithmic for group_stem at S-K, profiles/r02_pmc_traffic_SK_final.txt).
// Here a workgroup owns a 16-column strip of R output rows and one output plane PAIR; it stages the
// whole input window it needs -- all channels x 4 planes x (R + 2) rows x 18 columns -- and the
// weights in LDS once, so the halo rows are read once per R rows and never re-fetched per tap.
//
// MFMA mapping (v_mfma_f32_16x16x4_f32): the 16 rows are 8 couts x 2 output planes (z0, z0 + 1), the
// 16 columns the strip's pixels, k = 4 input channels.  Input plane z0 - 1 + p (p = 0..3) reaches
// plane z0 through tap plane dz = p and plane z0 + 1 through dz = p - 1, so one MFMA per (p, dy, dx,
// channel group) serves both planes (rows 0-7 / 8-15 read the two taps' weights; an out-of-range tap
// reads zero).  B: lane l reads channel 4g + l/16 at column (l & 15) + dx of the staged row; the
// channel stride in LDS is = 16 (mod 64) words, so the wave's 64 reads hit 64 distinct banks.
// A: lane l reads W[dz][dy][dx][4g + l/16][l & 7]; the dz stride is = 32 (mod 64), so the two plane
// halves do not collide.  Waves: R rows x KSW ways over the channel groups; the KSW partial tiles
// meet in LDS and are added in a fixed order (deterministic).
#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

template <int CIN>
struct R3Layout {
    static constexpr int wdz() {  // dz stride of the weight slab, = 32 (mod 64) words
        return 72 * CIN + ((32 - (72 * CIN) % 64) + 64) % 64;
    }
};

template <int KC, int R, int KSW, int ACT, bool PLAIN>
__global__ void __launch_bounds__(64 * R * KSW) rconv3_kernel(const esm_conv_desc a) {
    constexpr int CIN = 4 * KC;
    constexpr int RR = R + 2;                 // staged rows
    constexpr int PLANE = RR * 18;            // words per staged (channel, plane)
    constexpr int CS0 = 4 * PLANE;            // words per staged channel (4 planes)
    constexpr int CS = CS0 + ((16 - CS0 % 64) + 64) % 64;  // padded to = 16 (mod 64)
    constexpr int WDZ = R3Layout<CIN>::wdz();
    constexpr int NG = (KC + KSW - 1) / KSW;  // channel groups per wave
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* xin = lds;                 // [CIN][4][RR][18] (channel stride CS)
    float* wl = lds + CIN * CS;       // [3][WDZ]: [dz][(dy*3+dx)*CIN + c][8 couts]
    float* red = wl + 3 * WDZ;        // [KSW-1][R][4][64] partial tiles

    const int tid = static_cast<int>(threadIdx.x);
    const int lane = tid & 63;
    (void)tid;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int kpart = wave % KSW, r = wave / KSW;
    const int x0 = static_cast<int>(blockIdx.x) * 16;
    const int y0 = static_cast<int>(blockIdx.y) * R;
    const int npair = (a.Do + 1) / 2;
    const int b = static_cast<int>(blockIdx.z) / npair;
    const int z0 = (static_cast<int>(blockIdx.z) - b * npair) * 2;

    // ---- stage the input window (channels x planes z0-1..z0+2 x rows y0-1..y0+R x columns x0-1..x0+16)
    //      and the weights with the MFMA lane layout, so a load's address is a per-lane voffset fixed for
    //      the kernel (channel k = lane / 16, column lane % 16) plus a wave-uniform soffset (channel group,
    //      plane, row): scalar arithmetic per load instead of a per-element index decomposition.
    constexpr int NW = R * KSW;
    const int n = lane & 15, kq = lane >> 4;
    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (a.Di - 1) * sd + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const int xin_ = x0 + n;                                       // interior column
    const int xh = n == 0 ? x0 - 1 : x0 + 16;                      // halo column (lanes n = 0, 1)
    const unsigned vin = xin_ < a.Wi ? 4u * (kq * sc + xin_) : kOOB;
    const unsigned vh = (n < 2 && xh >= 0 && xh < a.Wi) ? 4u * (kq * sc + xh) : kOOB;
    constexpr int NU = KC * 4 * RR;                                // (channel group, plane, row) units
    constexpr int NUW = (NU + NW - 1) / NW;
    float vi[NUW], vhv[NUW];
#pragma unroll
    for (int j = 0; j < NUW; ++j) {
        const int u = wave + j * NW;                               // wave-uniform
        const int cg = u / (4 * RR), p = (u / RR) % 4, row = u % RR;
        const int zi = z0 - 1 + p, yi = y0 - 1 + row;
        const bool ok = u < NU && zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi;
        const int so = ok ? 4 * (4 * cg * sc + zi * sd + yi * sh) : static_cast<int>(kOOB);
        vi[j] = buf_load_s(rs, vin, so);
        vhv[j] = buf_load_s(rs, vh, so);
    }
    // weights: packed w[tap][cin_pad][cout_pad], tap = (dz*3 + dy)*3 + dx -> wl[dz][(t*CIN + c)*8 + co];
    // a load covers 8 channels x 8 couts (lane = channel * 8 + cout)
    constexpr int NG8 = (CIN + 7) / 8;
    constexpr int NWU = 27 * NG8;
    constexpr int NWW = (NWU + NW - 1) / NW;
    const int wcl = lane >> 3, wco = lane & 7;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w), static_cast<short>(0), 4 * 27 * a.cin_pad * a.cout_pad, 0x00020000);
    float wv[NWW];
#pragma unroll
    for (int j = 0; j < NWW; ++j) {
        const int u = wave + j * NW;
        const int tap = u / NG8, g8 = u % NG8;
        const bool ok = u < NWU && g8 * 8 + wcl < a.Cin && wco < a.Cout;
        wv[j] = buf_load_s(wrs, ok ? 4u * (wcl * a.cout_pad + wco) : kOOB, 4 * (tap * a.cin_pad + g8 * 8) * a.cout_pad);
    }
#pragma unroll
    for (int j = 0; j < NUW; ++j) {
        const int u = wave + j * NW;
        if (u < NU) {
            const int cg = u / (4 * RR), pr = u % (4 * RR);  // pr = p * RR + row
            float* dst = xin + (4 * cg + kq) * CS + pr * 18;
            dst[n + 1] = vi[j];
            if (n < 2) dst[n == 0 ? 0 : 17] = vhv[j];
        }
    }
#pragma unroll
    for (int j = 0; j < NWW; ++j) {
        const int u = wave + j * NW;
        const int tap = u / NG8, g8 = u % NG8;
        if (u < NWU && g8 * 8 + wcl < CIN) wl[(tap / 9) * WDZ + ((tap % 9) * CIN + g8 * 8 + wcl) * 8 + wco] = wv[j];
    }
    __syncthreads();

    // ---- MFMAs: this wave's output row y0 + r, channel groups kpart, kpart + KSW, ...
    const int co = lane & 7, hi = (lane >> 3) & 1;
    floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
    const float* xb = xin + kq * CS + r * 18 + n;
    const float* wb = wl + kq * 8 + co;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int dz = p - hi;                       // this lane's tap plane
        // an out-of-range tap plane multiplies a clamped (valid) weight by 0: an unconditional LDS read,
        // so the reads are not split by exec-mask branches and can run ahead of the MFMAs
        const float wm = (dz >= 0 && dz <= 2) ? 1.f : 0.f;
        const float* wp = wb + (dz < 0 ? 0 : (dz > 2 ? 2 : dz)) * WDZ;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
            const int dy = t / 3, dx = t % 3;
#pragma unroll
            for (int gi = 0; gi < NG; ++gi) {
                const int g = kpart + gi * KSW;
                if (g >= KC) break;
                const float av = wp[(t * CIN + 4 * g) * 8] * wm;
                const float bv = xb[4 * g * CS + p * PLANE + dy * 18 + dx];
                // two accumulation chains, alternating per MFMA (a single dependent chain stalls)
                acc[(t * NG + gi) & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[(t * NG + gi) & 1], 0, 0, 0);
            }
        }
    }
    floatx4 sum;
#pragma unroll
    for (int j = 0; j < 4; ++j) sum[j] = acc[0][j] + acc[1][j];

    // ---- K-split partial tiles: waves kpart > 0 park theirs in LDS, kpart 0 adds them in order
    if constexpr (KSW > 1) {
        __syncthreads();  // every wave is done reading xin / wl (red aliases nothing, but keep order simple)
        if (kpart > 0) {
#pragma unroll
            for (int j = 0; j < 4; ++j) red[(((kpart - 1) * R + r) * 4 + j) * 64 + lane] = sum[j];
        }
        __syncthreads();
        if (kpart > 0) return;
#pragma unroll
        for (int k = 1; k < KSW; ++k)
#pragma unroll
            for (int j = 0; j < 4; ++j) sum[j] += red[(((k - 1) * R + r) * 4 + j) * 64 + lane];
    }

    // ---- epilogue: lane (kq, n) holds MFMA rows 4*kq + j: cout (row & 7) of plane z0 + (row >> 3)
    const int y = y0 + r, px = x0 + n;
    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) + (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = 4 * kq + j;
        const int c = row & 7, zo = z0 + (row >> 3);
        const bool ok = c < a.Cout && zo < a.Do && y < a.Ho && px < a.Wo;
        const int cc = c < a.Cout ? c : a.Cout - 1;
        float v2 = a.scale ? sum[j] * a.scale[cc] + (a.shift ? a.shift[cc] : 0.f) : sum[j] + (a.shift ? a.shift[cc] : 0.f);
        v2 = act_t<ACT>(v2, a.act);
        if constexpr (PLAIN) {
            const unsigned o = ok ? 4u * (c * static_cast<int>(a.oc) + zo * static_cast<int>(a.od) + y * static_cast<int>(a.oh) + px)
                                  : kOOB;
            store_b32(__float_as_uint(v2), ro, static_cast<int>(o), 0);
        } else {
            if (!ok) continue;
            if (a.mul) v2 = v2 * a.mul[b * a.mb + c * a.mc + static_cast<long long>(y) * a.mh + px];
            if (a.res) v2 = v2 + a.res[b * a.rb + c * a.rc + static_cast<long long>(zo) * a.rd + static_cast<long long>(y) * a.rh + px];
            const long long o = b * a.ob + c * a.oc + static_cast<long long>(zo) * a.od + static_cast<long long>(y) * a.oh + px;
            a.out[o] = v2 * a.post_scale;
            if (a.out2) a.out2[o] = v2 * a.post_scale2;
        }
    }
}

template <int KC, int R, int KSW>
int launch_r3(const esm_conv_desc& a, hipStream_t s) {
    constexpr int CIN = 4 * KC;
    constexpr int PLANE = (R + 2) * 18;
    constexpr int CS0 = 4 * PLANE;
    constexpr int CS = CS0 + ((16 - CS0 % 64) + 64) % 64;
    const size_t lds = sizeof(float) * (static_cast<size_t>(CIN) * CS + 3 * R3Layout<CIN>::wdz() +
                                        static_cast<size_t>(KSW > 1 ? KSW - 1 : 0) * R * 4 * 64);
    const long long z = static_cast<long long>(a.B) * ((a.Do + 1) / 2);
    if (z > 65535) return arg_error("conv(rows3): grid too large");
    const dim3 grid(ceil_div(a.Wo, 16), ceil_div(a.Ho, R), static_cast<unsigned>(z));
    const bool plain = a.act == ESM_ACT_GELU && !a.res && !a.out2 && !a.mul && a.post_scale == 1.f &&
                       static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Do) * a.od +
                               static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (plain)
        hipLaunchKernelGGL((rconv3_kernel<KC, R, KSW, ESM_ACT_GELU, true>), grid, dim3(64 * R * KSW), lds, s, a);
    else
        hipLaunchKernelGGL((rconv3_kernel<KC, R, KSW, -1, false>), grid, dim3(64 * R * KSW), lds, s, a);
    return check_launch("conv(rows3)");
}

template <int KC>
int launch_r3_kc(const esm_conv_desc& a, hipStream_t s) {
    // rows per workgroup and K-split ways: small volumes split K 4 ways over 2 rows (more waves per
    // output, ~3 per SIMD at S-K); large ones take 4 rows x 2 ways (halo rows read once per 4 rows)
    const long long tiles = static_cast<long long>(a.B) * ceil_div(a.Wo, 16) * a.Ho * ((a.Do + 1) / 2);
    if constexpr (KC >= 4) {
        if (tiles <= 8192) return launch_r3<KC, 2, 4>(a, s);
        return launch_r3<KC, 4, 2>(a, s);
    } else {
        if (tiles <= 8192) return launch_r3<KC, 2, KC>(a, s);
        return launch_r3<KC, 4, 1>(a, s);
    }
}

}  // namespace

// 3x3x3 stride-1 padding-1 3-D convs with <= 8 couts over one source of 4..32 channels (whole
// 4-channel groups), plain or `* mul` / residual / out2 epilogues.
bool rows3_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (!d3 || a.transposed || a.stride != 1 || a.kd != 3 || a.kh != 3 || a.kw != 3) return false;
    if (a.pd != 1 || a.ph != 1 || a.pw != 1 || a.nsrc != 1 || a.Cout > 8 || a.up || a.shuffle > 1) return false;
    if (a.Cin < 4 || a.Cin > 32 || a.Cin % 4) return false;
    if (a.Do != a.Di || a.Ho != a.Hi || a.Wo != a.Wi) return false;
    return direct_ok(a);
}

int launch_rows3(const esm_conv_desc& a, hipStream_t s) {
    if (!rows3_ok(a)) return arg_error("conv: rows3-form hint not applicable");
    switch (a.Cin / 4) {
        case 1: return launch_r3_kc<1>(a, s);
        case 2: return launch_r3_kc<2>(a, s);
        case 3: return launch_r3_kc<3>(a, s);
        case 4: return launch_r3_kc<4>(a, s);
        case 5: return launch_r3_kc<5>(a, s);
        case 6: return launch_r3_kc<6>(a, s);
        case 7: return launch_r3_kc<7>(a, s);
        default: return launch_r3_kc<8>(a, s);
    }
}

}  // namespace conv
}  // namespace esm
