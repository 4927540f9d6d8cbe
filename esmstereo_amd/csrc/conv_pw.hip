// Pointwise (1x1 / 1x1x1, stride 1, no padding) BasicConv over a channel concat of up to 3 sources, as a
// streaming kernel for the large maps / volumes of ESMStereo-L / -M (round 6): the hourglass's agg_0.0 /
// agg_1.0 (models/ESMStereo.py:169-175, 1x1x1 over torch.cat of the decoder output and the skip) and
// up_refinement's agg_0[0] / agg_1[0] (models/ESMStereo.py:221-234, 1x1 over the cat with the image
// features).  At L-K B = 4 these layers moved 2.5-4x their algorithmic bytes' time through the LDS-tiled
// form (profiles/r06_ops_LK4.txt), which stages every input element through LDS for a single use.  A 1x1
// is a GEMM W[Cout x Cin] * X[Cin x pixels] at ~12 flop / byte, near the fp32 MFMA / HBM ridge (~20), so the
// form streams X straight into MFMA operands:
//   * a wave owns 64 consecutive pixels of the flattened (D, H, W) extent as four 16-column MFMA tiles
//     t = 0..3 with column n <-> pixel 4n + t: lane (q, n) reads channel 4k + q, pixels 4n .. 4n + 3 as
//     ONE 16-byte load per k-step (a wave-instruction covers 4 channels x 64 pixels, 256-byte rows), and
//     after the epilogue holds 4 consecutive pixels of each of its couts: 16-byte stores;
//   * the weights (<= 192 x 48) sit in LDS once per workgroup, sized to Cin (row stride = 16 mod 32 banks:
//     conflict-free ds_read_b32 of the A operand, one per cout tile and k-step, shared by the 4 column tiles);
//   * per source, k-steps go in batches of 4, double-buffered: batch i + 1's loads (4 KB per wave) are in
//     flight while batch i's 16 MT MFMAs run;
//   * small launches with 3 cout tiles put one tile per workgroup (grid z) for occupancy.
// (Round 6 measured two alternatives slower at L-K B = 4: no double buffering, 63 /
//     56 us for ref4x.agg_1.0 / agg_1.0; A operands loaded from global per k-step with one flat k loop over
//     the sources, ~79 us: the per-k-step source select put the buffer descriptor in vector registers, i.e.
//     a waterfall loop around every load.)
// Each output is one fixed-order sum (channel order, 4 per MFMA): deterministic, within fp32 reassociation
// of the other forms (tests: 1e-5 relative).  Plain BasicConv epilogue (BN + activation) only.
#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

constexpr int kPwThreads = 256;
constexpr int kPwMaxCin = 192;

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int MT, int ACT>
__global__ void __launch_bounds__(kPwThreads) pw_kernel(const esm_conv_desc a, int P, int ngroups) {
    constexpr int WCS = MT % 2 ? MT * 16 : MT * 16 + 16;        // weight row stride, = 16 mod 32
    extern __shared__ __attribute__((aligned(16))) float ws[];  // [round_up(Cin, 4)][WCS] (launcher's size)

    const int tid = threadIdx.x;
    const int lane = tid & 63, q = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int b = blockIdx.y;
    const int m0 = blockIdx.z * MT * 16;  // first cout of this workgroup (cout-split launches: one tile per z)

    // weights: row = input channel (zero past Cin, up to the next multiple of 4), column = output channel
    const int cin4 = (a.Cin + 3) & ~3;
    for (int e = tid; e < cin4 * MT * 16; e += kPwThreads) {
        const int c = e / (MT * 16), m = e - c * (MT * 16);
        ws[c * WCS + m] = (c < a.Cin && m0 + m < a.cout_pad) ? a.w[static_cast<long long>(c) * a.cout_pad + m0 + m] : 0.f;
    }
    float scl[MT][4], shf[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cc = min(m0 + 16 * mt + 4 * q + r, a.Cout - 1);
            scl[mt][r] = a.scale ? a.scale[cc] : 1.f;
            shf[mt][r] = a.shift ? a.shift[cc] : 0.f;
        }
    __syncthreads();

    const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0), 4 * ((a.Cout - 1) * static_cast<int>(a.oc) + P), 0x00020000);

    for (int gi = blockIdx.x * 4 + wave; gi < ngroups; gi += gridDim.x * 4) {
        const int pp = gi * 64 + 4 * n;  // this lane's first pixel (P % 4 == 0: all four valid or none)
        const bool pok = pp < P;
        floatx4 acc[4][MT];
#pragma unroll
        for (int t = 0; t < 4; ++t)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[t][mt] = floatx4{0.f, 0.f, 0.f, 0.f};

        int c0 = 0;  // first (global) channel of the source
#pragma unroll
        for (int j = 0; j < ESM_MAX_SRC; ++j) {
            if (j >= a.nsrc) break;
            const esm_src& sj = a.src[j];  // (compile-time index: the descriptor stays in scalar registers)
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float*>(sj.ptr + b * sj.sb), static_cast<short>(0),
                4 * ((sj.C - 1) * static_cast<int>(sj.sc) + P), 0x00020000);
            const int sc = static_cast<int>(sj.sc);
            const unsigned vo = pok ? 4u * static_cast<unsigned>(q * sc + pp) : kOOB;
            const int ns = sj.C >> 2;
            // batch i = k-steps 4i .. 4i + 3 (the last one partial: cnt = its k-steps, a wave-uniform count)
            auto load_b = [&](u32x4 (&bv)[4], int i) __attribute__((always_inline)) {
                const int cnt = min(4, ns - 4 * i);
#pragma unroll
                for (int u = 0; u < 4; ++u)  // (past the source: range-checked zeros, which no MFMA reads)
                    bv[u] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(u < cnt ? vo : kOOB),
                                                                  16 * (4 * i + u) * sc, 0);
            };
            auto mfma_b = [&](const u32x4 (&bv)[4], int i) __attribute__((always_inline)) {
                const int cnt = min(4, ns - 4 * i);
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    if (u >= cnt) break;
                    const float* wr = &ws[(c0 + 4 * (4 * i + u) + q) * WCS + n];
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt) {
                        const float av = wr[16 * mt];
#pragma unroll
                        for (int t = 0; t < 4; ++t)
                            acc[t][mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, __uint_as_float(bv[u][t]), acc[t][mt],
                                                                              0, 0, 0);
                    }
                }
            };
            // double-buffered: batch i + 1's loads (up to 4 KB per wave) in flight during batch i's MFMAs
            const int nb = (ns + 3) >> 2;
            u32x4 b0[4], b1[4];
            load_b(b0, 0);
            int i = 0;
            for (; i + 2 <= nb; i += 2) {
                load_b(b1, i + 1);
                mfma_b(b0, i);
                if (i + 2 < nb) load_b(b0, i + 2);
                mfma_b(b1, i + 1);
            }
            if (i < nb) mfma_b(b0, i);
            c0 += sj.C;
        }

        // epilogue: lane (n, q) holds couts m0 + 16 mt + 4 q + r at pixels 4n + t (t = 0..3): one 16-byte store each
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = m0 + 16 * mt + 4 * q + r;
                u32x4 o;
#pragma unroll
                for (int t = 0; t < 4; ++t) {
                    float v = acc[t][mt][r];
                    v = a.scale ? v * scl[mt][r] + shf[mt][r] : v + shf[mt][r];
                    o[t] = __float_as_uint(act_t<ACT>(v, a.act));
                }
                const unsigned ov = (pok && co < a.Cout) ? 4u * static_cast<unsigned>(co * static_cast<int>(a.oc) + pp) : kOOB;
                __builtin_amdgcn_raw_buffer_store_b128(o, ro, static_cast<int>(ov), 0, kStoreAux);
            }
    }
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15) == 0; }

}  // namespace

// 1x1 (x1) stride 1 pad 0, plain BasicConv epilogue, <= 48 couts, <= 192 input channels in 4-channel
// aligned sources; every source and the output dense over the flattened (D, H, W) extent with 16-byte
// aligned channel / batch strides, and every span within 32-bit buffer offsets.
bool pw_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (a.transposed || a.kh != 1 || a.kw != 1 || (d3 && a.kd != 1) || a.stride != 1 || a.ph || a.pw || a.pd) return false;
    if (a.mul || a.res || a.out2 || a.up || a.pre || a.shuffle > 1 || a.post_scale != 1.f) return false;
    if (a.Cout > 48 || a.Cin > kPwMaxCin || a.cout_pad < 16 * ((a.Cout + 15) / 16)) return false;
    const long long P = static_cast<long long>(a.Di) * a.Hi * a.Wi;
    if (P % 4 || a.Do != a.Di || a.Ho != a.Hi || a.Wo != a.Wi) return false;
    if (!aligned16(a.out) || a.ob % 4 || a.oc % 4 || a.oh != a.Wo || (d3 && a.od != static_cast<long long>(a.Ho) * a.Wo))
        return false;
    if (4 * ((a.Cout - 1) * a.oc + P) >= static_cast<long long>(kOOB)) return false;
    for (int k = 0; k < a.nsrc; ++k) {
        const esm_src& s = a.src[k];
        if (s.C % 4 || !aligned16(s.ptr) || s.sb % 4 || s.sc % 4 || s.sh != a.Wi ||
            (d3 && s.sd != static_cast<long long>(a.Hi) * a.Wi))
            return false;
        if (4 * ((s.C - 1) * s.sc + P) >= static_cast<long long>(kOOB)) return false;
    }
    return true;
}

// automatic choice: the large maps / volumes (>= 2^16 pixels per launch)
bool pw_auto(const esm_conv_desc& a) {
    return pw_ok(a) && static_cast<long long>(a.B) * a.Di * a.Hi * a.Wi >= (1LL << 16);
}

int launch_pw(const esm_conv_desc& a, hipStream_t s) {
    if (!pw_ok(a)) return arg_error("conv: pointwise-form hint not applicable");
    const int P = a.Di * a.Hi * a.Wi;
    const int ngroups = (P + 63) / 64;
    const long long total = static_cast<long long>(ngroups) * a.B;
    const int tiles = (a.Cout + 15) / 16;
    // launches of fewer than 4096 pixel groups with 3 cout tiles (agg_0.0 at L-K B = 4: 1404 groups, 40 couts; 23.6 ->
    // 20.8 us): one cout tile per workgroup (grid z), tiles x the waves; else every tile in one wave, the B operands
    // loaded once (2 tiles split measured slower: ref4x.agg_0.0, 112 -> 32 at 96 x 312, 24.7 -> 30.0 us)
    const bool split = total < 4096 && tiles > 2;
    // one pixel group per wave up to 2^14 groups (latency hiding by occupancy), then up to 8 per wave
    const int per_wave = static_cast<int>(std::max<long long>(1, std::min<long long>(8, total / 16384)));
    const int gx = std::max(1, (ngroups + 4 * per_wave - 1) / (4 * per_wave));
    if (a.B > 65535) return arg_error("conv(pointwise): batch too large");
    const dim3 grid(gx, a.B, split ? tiles : 1);
    const int mt = split ? 1 : tiles;
    const bool gelu = a.act == ESM_ACT_GELU;
    const size_t lds = 4u * static_cast<size_t>((a.Cin + 3) & ~3) * (mt % 2 ? mt * 16 : mt * 16 + 16);
#define ESM_PW(M)                                                                                             \
    do {                                                                                                      \
        if (gelu)                                                                                             \
            hipLaunchKernelGGL((pw_kernel<M, ESM_ACT_GELU>), grid, dim3(kPwThreads), lds, s, a, P, ngroups);  \
        else                                                                                                  \
            hipLaunchKernelGGL((pw_kernel<M, -1>), grid, dim3(kPwThreads), lds, s, a, P, ngroups);            \
    } while (0)
    if (mt == 1) ESM_PW(1);
    else if (mt == 2) ESM_PW(2);
    else ESM_PW(3);
#undef ESM_PW
    return check_launch("conv(pointwise)");
}

}  // namespace conv
}  // namespace esm
