// Two consecutive 2-D BasicConvs in one launch, both through LDS (halo recomputation):
//   y = actB(BN_B(convB(actA(BN_A(convA(cat(sources)))))))
// convA: k 1/3/5, stride 1/2, any padding, <= 48 input channels (64 for 1x1) over up to 3 sources, 16 outputs;
// convB: k 1/3, stride 1, 16 inputs, <= 16 outputs.  The pairs of the ESM upsampler stages and the
// refinement hourglasses (models/ESMStereo.py:185-239, 247-259 and twins): dm<t>.0 -> dm<t>.1,
// dm<t>.2 -> dm<t>.3, spx_<t>.0 -> spx_<t>.1, conv2.0 -> conv2.1, conv3.0 -> conv3.1.
//
// Why: on the 1/16..1/4-resolution maps of ESMStereo-S each of these convs is a latency floor
// (~4.5 us per launch, ~2 us of it serial memory round trips: profiles/r02_pmc_sq_ops_SK_b.txt).
// Here one round trip stages everything a workgroup needs -- the input window of its tile (+ the
// halo both convs need), both weight slabs, both BN affines -- into LDS; convA runs on the tile +
// convB's halo into LDS (zero outside A's extent: convB's zero padding), convB runs from LDS and
// stores.  The intermediate map never touches memory, and the launch between the two is gone.
//
// MFMA mapping (v_mfma_f32_16x16x4_f32): M = 16 output channels, N = 16 pixels of one tile row,
// k = 4 input channels.  A workgroup owns TH output rows x (16 - KB + 1) output columns; convA
// computes TH + KB - 1 rows x 16 columns.  4 waves: rows round-robin in both phases.
#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

constexpr int kP2Threads = 256;
// a.hint bit 29 on convA: its single input channel is disparity_regression of the cost volume in src[0]
// (src[0].C = D planes), also stored to a.out (see pair2_ok)
constexpr int kHintPairReg = 1 << 29;

// disparity_regression at one pixel, as regression.hip dispreg_kernel: products rounded, then summed in
// d order (torch.sum(x * arange)): the same bits as the separate launch
__device__ __forceinline__ float regress_px(const float* __restrict__ cp, int D, int sc) {
#pragma clang fp contract(off)
    float acc = 0.f;
    for (int d0 = 0; d0 < D; d0 += 16) {
        float v[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] = d0 + k < D ? cp[(d0 + k) * sc] : 0.f;
#pragma unroll
        for (int k = 0; k < 16; ++k)
            if (d0 + k < D) acc = acc + v[k] * static_cast<float>(d0 + k);
    }
    return acc;
}

template <int KA, int SA, int KB, int TH>
struct P2Geo {
    static constexpr int NA = TH + KB - 1;        // convA rows per tile
    static constexpr int IR = (NA - 1) * SA + KA;   // staged input rows
    static constexpr int IC = 15 * SA + KA;         // staged input columns
    static constexpr int ICP = IC;
    static constexpr int ICS0 = IR * ICP;
    static constexpr int ICS = ICS0 + ((16 - ICS0 % 64) + 64) % 64;  // channel stride = 16 (mod 64)
    static constexpr int AR = 18;                                   // convA row in LDS (16 + dx overrun)
    static constexpr int ACS0 = NA * AR;
    static constexpr int ACS = ACS0 + ((16 - ACS0 % 64) + 64) % 64;
};

template <int KA, int SA, int KB, int TH, int CINMAX, bool REG>
__global__ void __launch_bounds__(kP2Threads) pair2_kernel(const esm_conv_desc a, const esm_conv_desc bd) {
    using G = P2Geo<KA, SA, KB, TH>;
    constexpr int NA = G::NA, IR = G::IR, IC = G::IC, ICP = G::ICP, ICS = G::ICS, AR = G::AR, ACS = G::ACS;
    constexpr int TA = KA * KA, TB = KB * KB;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* in = lds;                          // [CINMAX][IR][ICP] (channel stride ICS)
    float* wa = in + CINMAX * ICS;            // [TA][CINMAX][16]
    float* wb = wa + TA * CINMAX * 16;        // [TB][16][16]
    float* at = wb + TB * 256;                // [16][NA][AR] (channel stride ACS)
    float* ep = at + 16 * ACS;                // scaleA, shiftA, scaleB, shiftB [16] each

    const int tid = static_cast<int>(threadIdx.x);
    const int lane = tid & 63, wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int n = lane & 15, kq = lane >> 4;
    constexpr int VB = 16 - KB + 1;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int b = bk_.z;
    const int yb0 = bk_.y * TH, xb0 = bk_.x * VB;
    const int pb = bd.ph;
    const int ya0 = yb0 - pb, xa0 = xb0 - pb;                 // convA tile origin
    const int yi0 = ya0 * SA - a.ph, xi0 = xa0 * SA - a.pw;   // staged input origin
    const int cin = a.Cin;

    // ---- stage: input window (zero outside the input and past Cin), weights, BN affines.  The sources'
    //      pointers / strides are read once as wave-uniform values and selected per element in
    //      registers (indexing a.src[] by a per-lane value would re-load them from the kernarg
    //      segment for every element).
    const int ns = a.nsrc;
    const float* sp0 = a.src[0].ptr + b * a.src[0].sb;
    const float* sp1 = ns > 1 ? a.src[1].ptr + b * a.src[1].sb : sp0;
    const float* sp2 = ns > 2 ? a.src[2].ptr + b * a.src[2].sb : sp0;
    const int c0 = a.src[0].C, c01 = c0 + (ns > 1 ? a.src[1].C : 0);
    const int sc0 = static_cast<int>(a.src[0].sc), sh0 = static_cast<int>(a.src[0].sh);
    const int sc1 = ns > 1 ? static_cast<int>(a.src[1].sc) : sc0, sh1 = ns > 1 ? static_cast<int>(a.src[1].sh) : sh0;
    const int sc2 = ns > 2 ? static_cast<int>(a.src[2].sc) : sc0, sh2 = ns > 2 ? static_cast<int>(a.src[2].sh) : sh0;
    constexpr int NIN = CINMAX * IR * IC;
    constexpr int PI = (NIN + kP2Threads - 1) / kP2Threads;
    float vi[PI];
    if constexpr (!REG) {
#pragma unroll
        for (int i = 0; i < PI; ++i) {
            const int e = i * kP2Threads + tid;
            const int q = e % IC, r = (e / IC) % IR, c = e / (IC * IR);
            const int yi = yi0 + r, xi = xi0 + q;
            const bool s1 = c >= c0, s2 = c >= c01;
            const float* base = s2 ? sp2 : (s1 ? sp1 : sp0);
            const int cl = c - (s2 ? c01 : (s1 ? c0 : 0));
            const int scs = s2 ? sc2 : (s1 ? sc1 : sc0), shs = s2 ? sh2 : (s1 ? sh1 : sh0);
            const bool ok = e < NIN && c < cin && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
            const float v = base[ok ? cl * scs + yi * shs + xi : 0];
            vi[i] = ok ? v : 0.f;
        }
    }
    constexpr int NWA = TA * CINMAX * 16;
    constexpr int PWA = (NWA + kP2Threads - 1) / kP2Threads;
    float vwa[PWA];
#pragma unroll
    for (int i = 0; i < PWA; ++i) {
        const int e = i * kP2Threads + tid;
        const int co = e & 15, c = (e >> 4) % CINMAX, tap = e / (16 * CINMAX);
        const bool ok = e < NWA && c < cin && co < a.Cout;
        const float v = a.w[ok ? (static_cast<long long>(tap) * a.cin_pad + c) * a.cout_pad + co : 0];
        vwa[i] = ok ? v : 0.f;
    }
    constexpr int NWB = TB * 256;
    constexpr int PWB = NWB / kP2Threads;
    float vwb[PWB];
#pragma unroll
    for (int i = 0; i < PWB; ++i) {
        const int e = i * kP2Threads + tid;
        const int co = e & 15, c = (e >> 4) & 15, tap = e >> 8;
        const bool ok = c < bd.Cin && co < bd.Cout;
        const float v = bd.w[ok ? (static_cast<long long>(tap) * bd.cin_pad + c) * bd.cout_pad + co : 0];
        vwb[i] = ok ? v : 0.f;
    }
    float vep = 0.f;
    if (tid < 64) {  // scaleA, shiftA, scaleB, shiftB: wave-uniform pointers, selected per lane
        const int k = tid >> 4, c = tid & 15;
        const float* p = k == 0 ? a.scale : (k == 1 ? a.shift : (k == 2 ? bd.scale : bd.shift));
        const int cn = k < 2 ? a.Cout : bd.Cout;
        const bool ok = p != nullptr && c < cn;
        const float v = (ok ? p : a.w)[ok ? c : 0];
        vep = ok ? v : ((k & 1) ? 0.f : 1.f);
    }
    if constexpr (REG) {
        // after the weight loads (the regression's adds and the map's store wait for the cost planes, the
        // weights' loads need not); channel 0 only (Cin 1), the other staged channels zero.  The map is
        // written once per pixel by the tile that owns it: rows [yb0, yb0 + TH) and columns [xb0, xb0 + VB),
        // the edge tiles extended to the map's edges (their windows cover them: launch_p2)
#pragma unroll
        for (int i = 0; i < PI; ++i) {
            const int e = i * kP2Threads + tid;
            const int q = e % IC, r = (e / IC) % IR, c = e / (IC * IR);
            const int yi = yi0 + r, xi = xi0 + q;
            vi[i] = 0.f;
            if (e < NIN && c == 0 && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi) {
                const float v = regress_px(sp0 + yi * sh0 + xi, a.src[0].C, sc0);
                vi[i] = v;
                const bool own_y = (bk_.y == 0 || yi >= yb0) && (bk_.y == static_cast<int>(gridDim.y) - 1 || yi < yb0 + TH);
                const bool own_x = (bk_.x == 0 || xi >= xb0) && (bk_.x == static_cast<int>(gridDim.x) - 1 || xi < xb0 + VB);
                if (own_y && own_x) a.out[b * a.ob + yi * a.oh + xi] = v;
            }
        }
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
    for (int i = 0; i < PI; ++i) {
        const int e = i * kP2Threads + tid;
        if (e < NIN) in[(e / (IC * IR)) * ICS + ((e / IC) % IR) * ICP + e % IC] = vi[i];
    }
#pragma unroll
    for (int i = 0; i < PWA; ++i) {
        const int e = i * kP2Threads + tid;
        if (e < NWA) wa[e] = vwa[i];
    }
#pragma unroll
    for (int i = 0; i < PWB; ++i) wb[i * kP2Threads + tid] = vwb[i];
    if (tid < 64) ep[tid] = vep;
    __syncthreads();

    // ---- convA on the tile + halo: row i of the tile = convA output row ya0 + i
    for (int i = wave; i < NA; i += kP2Threads / 64) {
        floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
        const float* ib = in + kq * ICS + i * SA * ICP + n * SA;
        const float* wp = wa + kq * 16 + n;
        const int kca = (cin + 3) >> 2;
        // accumulator indices stay compile-time (a runtime index turns every MFMA into a select chain
        // over the accumulators): two chains alternate by tap, or by channel group for 1x1 convA
        if constexpr (TA > 1) {
            if (cin == 1) {
                // one input channel (the dm<t>.0 heads): the taps fill k, 4 per MFMA (7 MFMAs per row for 5x5,
                // not 25 with 3 zero channels each); lane group kq takes tap 4 kc + kq
                const float* ib0 = in + i * SA * ICP + n * SA;
#pragma unroll
                for (int kc = 0; kc < (TA + 3) / 4; ++kc) {
                    const int t = 4 * kc + kq;
                    const bool tv = t < TA;
                    const int tt = tv ? t : 0;
                    const float bv = ib0[(tt / KA) * ICP + tt % KA];
                    const float av = wa[tt * CINMAX * 16 + n];
                    acc[kc & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(tv ? av : 0.f, tv ? bv : 0.f, acc[kc & 1], 0, 0, 0);
                }
            } else {
                for (int kc = 0; kc < kca; ++kc) {
#pragma unroll
                    for (int t = 0; t < TA; ++t) {
                        const int ky = t / KA, kx = t % KA;
                        const float bv = ib[4 * kc * ICS + ky * ICP + kx];
                        const float av = wp[(t * CINMAX + 4 * kc) * 16];
                        acc[t & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[t & 1], 0, 0, 0);
                    }
                }
            }
        } else {
            for (int kc = 0; kc < kca; kc += 2) {
                acc[0] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[4 * kc * 16], ib[4 * kc * ICS], acc[0], 0, 0, 0);
                if (kc + 1 < kca)
                    acc[1] = __builtin_amdgcn_mfma_f32_16x16x4f32(wp[4 * (kc + 1) * 16], ib[4 * (kc + 1) * ICS], acc[1],
                                                                  0, 0, 0);
            }
        }
        const int ya = ya0 + i, xa = xa0 + n;
        const bool inside = ya >= 0 && ya < a.Ho && xa >= 0 && xa < a.Wo;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * kq + j;
            const float v = act_t<ESM_ACT_GELU>((acc[0][j] + acc[1][j]) * ep[co] + ep[16 + co], 0);
            at[co * ACS + i * AR + n] = inside ? v : 0.f;
        }
    }
    __syncthreads();

    // ---- convB from LDS: output row yb0 + t, columns xb0 .. xb0 + VB - 1
    for (int t = wave; t < TH; t += kP2Threads / 64) {
        floatx4 acc[2] = {floatx4{0.f, 0.f, 0.f, 0.f}, floatx4{0.f, 0.f, 0.f, 0.f}};
        const float* ab = at + kq * ACS + t * AR + n;
        const float* wp = wb + kq * 16 + n;
#pragma unroll
        for (int kc = 0; kc < 4; ++kc)
#pragma unroll
            for (int tp = 0; tp < TB; ++tp) {
                const int dy = tp / KB, dx = tp % KB;
                const float bv = ab[4 * kc * ACS + dy * AR + dx];
                const float av = wp[(tp * 16 + 4 * kc) * 16];
                acc[tp & 1] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv, acc[tp & 1], 0, 0, 0);
            }
        const int yb = yb0 + t, xb = xb0 + n;
        const bool ok = yb < bd.Ho && xb < bd.Wo && n < VB;
        const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
            bd.out + b * bd.ob, static_cast<short>(0),
            4 * ((bd.Cout - 1) * static_cast<int>(bd.oc) + (bd.Ho - 1) * static_cast<int>(bd.oh) + bd.Wo), 0x00020000);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = 4 * kq + j;
            const float v = act_t<ESM_ACT_GELU>((acc[0][j] + acc[1][j]) * ep[32 + co] + ep[48 + co], 0);
            const unsigned o = (ok && co < bd.Cout) ? 4u * (co * static_cast<int>(bd.oc) + yb * static_cast<int>(bd.oh) + xb)
                                                    : kOOB;
            store_b32(__float_as_uint(v), ro, static_cast<int>(o), 0);
        }
    }
}

template <int KA, int SA, int KB, int TH, int CINMAX, bool REG = false>
int launch_p2(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    using G = P2Geo<KA, SA, KB, TH>;
    const size_t lds = sizeof(float) * (static_cast<size_t>(CINMAX) * G::ICS + KA * KA * CINMAX * 16 + KB * KB * 256 +
                                        16 * G::ACS + 64);
    constexpr int VB = 16 - KB + 1;
    const dim3 grid(ceil_div(b.Wo, VB), ceil_div(b.Ho, TH), a.B);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("conv pair: grid too large");
    if constexpr (REG) {
        // every pixel of the regressed map inside the window of the tile that stores it
        const int pr = b.ph + a.ph, pc = b.pw + a.pw;
        if (pr < 0 || pc < 0 || TH > G::IR - pr || VB > G::IC - pc ||
            (static_cast<int>(grid.y) - 1) * TH - pr + G::IR < a.Hi || (static_cast<int>(grid.x) - 1) * VB - pc + G::IC < a.Wi)
            return arg_error("conv pair: regressed map not covered by the tiles");
    }
    hipLaunchKernelGGL((pair2_kernel<KA, SA, KB, TH, CINMAX, REG>), grid, dim3(kP2Threads), lds, s, a, b);
    return check_launch("conv pair");
}

template <int KA, int SA, int KB>
int launch_p2_k(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    // 2-row tiles on small maps (more workgroups), 4-row tiles where that still gives >= 256
    const long long tiles4 = static_cast<long long>(ceil_div(b.Wo, 16 - KB + 1)) * ceil_div(b.Ho, 4) * a.B;
    // b.hint bits 26-27: tile rows 2 / 4 / 8 (8: <= 16 input channels), 0 automatic
    const int thsel = (b.hint >> 26) & 3;
    const bool small = thsel ? thsel == 1 : tiles4 < 256;
    const bool tall = thsel == 3 && a.Cin <= 16;
    if constexpr (KA == 5 && KB == 3) {
        if (a.hint & kHintPairReg) {
            if (tall) return launch_p2<KA, SA, KB, 8, 4, true>(a, b, s);
            return small ? launch_p2<KA, SA, KB, 2, 4, true>(a, b, s) : launch_p2<KA, SA, KB, 4, 4, true>(a, b, s);
        }
    }
    if (tall) return a.Cin <= 4 ? launch_p2<KA, SA, KB, 8, 4>(a, b, s) : launch_p2<KA, SA, KB, 8, 16>(a, b, s);
    if (a.Cin <= 4) return small ? launch_p2<KA, SA, KB, 2, 4>(a, b, s) : launch_p2<KA, SA, KB, 4, 4>(a, b, s);
    if (a.Cin <= 16) return small ? launch_p2<KA, SA, KB, 2, 16>(a, b, s) : launch_p2<KA, SA, KB, 4, 16>(a, b, s);
    if (a.Cin <= 32) return small ? launch_p2<KA, SA, KB, 2, 32>(a, b, s) : launch_p2<KA, SA, KB, 4, 32>(a, b, s);
    if constexpr (KA == 1) {
        if (a.Cin > 48) return small ? launch_p2<KA, SA, KB, 2, 64>(a, b, s) : launch_p2<KA, SA, KB, 4, 64>(a, b, s);
    }
    return small ? launch_p2<KA, SA, KB, 2, 48>(a, b, s) : launch_p2<KA, SA, KB, 4, 48>(a, b, s);
}

}  // namespace

// convA: 2-D, not transposed, k 1/3/5 (stride 1) or 3 (stride 2), <= 48 input channels (64 for k 1; 1..3 sources),
// 16 outputs, BN + GELU, plain output (only convB's output is stored); convB: 2-D k1/k3 stride 1 over
// convA's 16 channels, <= 16 outputs, BN + GELU, plain epilogue.  With hint bit 29 on convA (5x5, one
// input channel, convB 3x3): src[0] is a [B, D, H, W] cost volume (C = D) and convA's input map is its
// disparity_regression (models/submodule.py:211-216), computed per staged pixel and stored once to
// a.out ([B, 1, H, W], strides ob / oh) -- the regression launch of the hot path folded into the
// upsampler's first pair.
bool pair2_ok(const esm_conv_desc& a, const esm_conv_desc& b) {
    const bool a3 = a.kd > 1 || a.Di > 1 || a.Do > 1, b3 = b.kd > 1 || b.Di > 1 || b.Do > 1;
    if (a3 || b3 || a.transposed || b.transposed || a.shuffle > 1 || b.shuffle > 1) return false;
    if (a.Cout != 16 || a.Cin < 1 || a.Cin > (a.kh == 1 ? 64 : 48) || b.Cin != 16 || b.Cout < 1 || b.Cout > 16)
        return false;
    if (!((a.kh == 3 && (a.stride == 1 || a.stride == 2)) || ((a.kh == 1 || a.kh == 5) && a.stride == 1))) return false;
    if (a.ph != a.pw || b.ph != b.pw || b.stride != 1 || (b.kh != 1 && b.kh != 3)) return false;
    if (a.act != ESM_ACT_GELU || b.act != ESM_ACT_GELU) return false;
    if (a.mul || a.res || a.up || a.out2 || a.post_scale != 1.f) return false;
    if (b.mul || b.res || b.up || b.out2 || b.post_scale != 1.f || !b.out) return false;
    if (b.Hi != a.Ho || b.Wi != a.Wo || b.B != a.B) return false;
    if (b.Ho != b.Hi + 2 * b.ph - b.kh + 1 || b.Wo != b.Wi + 2 * b.pw - b.kw + 1) return false;
    if (a.nsrc > 1)
        for (int i = 0; i < a.nsrc; ++i)
            if (a.src[i].C % 4) return false;
    if (a.hint & kHintPairReg) {  // convA 5x5 1 -> 16 over the regressed map, convB 3x3 (the dm<t>.0 + .1 head)
        if (a.kh != 5 || b.kh != 3 || a.Cin != 1 || a.nsrc != 1 || a.src[0].C < 1 || !a.out || a.out == b.out)
            return false;
        if (static_cast<long long>(a.src[0].C) * a.src[0].sc >= (1LL << 31) || a.src[0].sh >= (1 << 28)) return false;
    }
    const long long last = (b.Cout - 1) * b.oc + (b.Ho - 1) * b.oh + b.Wo;
    return 4 * last < static_cast<long long>(kOOB) && b.oc < (1 << 28) && b.oh < (1 << 28);
}

int launch_pair2(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    if (!pair2_ok(a, b)) return arg_error("conv pair: unsupported pair");
    if (a.kh == 5) return b.kh == 3 ? launch_p2_k<5, 1, 3>(a, b, s) : launch_p2_k<5, 1, 1>(a, b, s);
    if (a.kh == 1) return b.kh == 3 ? launch_p2_k<1, 1, 3>(a, b, s) : launch_p2_k<1, 1, 1>(a, b, s);
    if (a.stride == 2) return b.kh == 3 ? launch_p2_k<3, 2, 3>(a, b, s) : launch_p2_k<3, 2, 1>(a, b, s);
    return b.kh == 3 ? launch_p2_k<3, 1, 3>(a, b, s) : launch_p2_k<3, 1, 1>(a, b, s);
}

}  // namespace conv
}  // namespace esm

extern "C" int esm_conv_pair2_f32(const esm_conv_desc* a, const esm_conv_desc* b, void* stream) {
    if (!a || !b) return esm::arg_error("conv pair: null descriptor");
    return esm::conv::launch_pair2(*a, *b, esm::as_stream(stream));
}
