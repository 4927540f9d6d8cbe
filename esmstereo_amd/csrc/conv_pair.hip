// Two stride-1 2-D convolutions fused into one launch: B(act_B(bn_B(conv_B(act_A(bn_A(conv_A(x)))))))
// [+ res], with the intermediate never leaving the chip.  The pairs of the hot path it replaces:
//   agg_0 / agg_1 of up_refinement       conv1x1 over a channel concat -> conv3x3   (models/ESMStereo.py:214-218, 228-235)
//   spx_2x / spx_4x of the upsamplers    conv3x3 over a concat -> conv3x3 (+BN+GELU) (:256-259, 283-286, and twins)
//   dmNx.1 -> dmNx.2                     conv3x3 -> conv3x3                           (:250-253)
//   FMBlock.conv                         conv3x3 (+SiLU) -> conv1x1 (+ residual)      (models/shufflemixer.py:124-131)
//
// Row streaming on the fp32 matrix cores (the form of conv_rows.h, chained): a wave owns one
// 16-column tile and walks RW consecutive output rows.  Per step it computes ONE new row of A's
// output for all of A's channels (MFMA, B operand = input row loads shifted across the 16-lane
// rows by DPP for the horizontal taps), applies A's epilogue and zero padding, and keeps the last
// KB such rows in registers.  The MFMA accumulator layout of A's output (lane (g, n) holds
// channels 4g + j of pixel n in register j) is exactly a B-operand k-step of the next MFMA when
// B's k order is permuted to (j, g): no lane movement and no LDS for the intermediate.  B's
// horizontal taps are DPP shifts of those registers again.  Each A row is computed once per wave
// and reused by KB output rows.  A 16-lane tile yields 16 - 2*(KA/2 + KB/2) valid columns.
// Weights of both layers are staged in LDS once per workgroup (one batch of loads).
#include "conv_rows.h"

namespace esm {
namespace conv {
namespace {

constexpr int kPairThreads = 256;

template <int MA>
constexpr int pair_wrow() { return MA == 1 ? 16 : 48; }  // LDS weight row (48: k rows g, g+1 16 banks apart)

template <int KA, int KB, int MA, int MB, int NKA>
struct PGeo {
    static constexpr int A0 = KA / 2, B0 = KB / 2, HALO = A0 + B0, VALID = 16 - 2 * HALO;
    static constexpr int TAPA = KA * KA, TAPB = KB * KB;
    static constexpr int CINA = 4 * NKA, CM = 16 * MA;
    static constexpr int WRA = pair_wrow<MA>(), WRB = pair_wrow<MB>();
    static constexpr int LDSA = TAPA * CINA * WRA, LDSB = TAPB * CM * WRB;
    static constexpr int BYTES = 4 * (LDSA + LDSB);
};

__device__ __forceinline__ float pair_act(float v, int act) { return apply_act(v, act); }

template <int KA, int KB, int MA, int MB, int NKA>
__global__ void __launch_bounds__(kPairThreads) pair_kernel(const esm_conv_desc a, const esm_conv_desc bd, int RW) {
    using G = PGeo<KA, KB, MA, MB, NKA>;
    constexpr int A0 = G::A0, B0 = G::B0, HALO = G::HALO, VALID = G::VALID;
    constexpr int TAPA = G::TAPA, TAPB = G::TAPB, CINA = G::CINA, CM = G::CM, WRA = G::WRA, WRB = G::WRB;
    extern __shared__ __attribute__((aligned(16))) float lds[];
    float* wa = lds;              // [TAPA][CINA][WRA]: A weights, couts 0..CM-1
    float* wb = lds + G::LDSA;    // [TAPB][CM][WRB]:   B weights, couts 0..16MB-1

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15, kq = lane >> 4;
    const int H = bd.Ho, W = bd.Wo;
    const int tiles_w = (W + VALID - 1) / VALID;
    const int rows_wg = 4 * RW;
    const int tiles_h = (H + rows_wg - 1) / rows_wg;
    // XCD-aware tile order (conv_direct.h)
    const unsigned nwg = gridDim.x, orig = blockIdx.x;
    const unsigned q = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    unsigned wg = (xcd < r8 ? xcd * (q + 1) : r8 * (q + 1) + (xcd - r8) * q) + orig / 8;
    const int tx = static_cast<int>(wg % tiles_w);
    wg /= tiles_w;
    const int ty = static_cast<int>(wg % tiles_h);
    const int b = static_cast<int>(wg / tiles_h);
    const int T = tx * VALID - HALO;  // image column held by lane 0 (every stage)
    const int col = T + n16;
    const bool col_ok = col >= 0 && col < W;
    const unsigned xoff = col_ok ? 4u * col : kOOB;

    // ---- A's input: up to 3 channel-concatenated sources; k-step kk reads channels 4kk..4kk+3
    //      (all in one source: the launcher requires 4-channel-aligned splits)
    const int lo1 = a.src[0].C, lo2 = a.src[0].C + a.src[1].C;
    // one descriptor per source, each from constant-index kernel-argument fields (a runtime index
    // into a.src[] or into an array of descriptors becomes a scratch lookup table in hipcc)
    auto mk = [&](const esm_src& sr) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sr.ptr + b * sr.sb), static_cast<short>(0),
                                                 4 * ((sr.C - 1) * static_cast<int>(sr.sc) +
                                                      (a.Hi - 1) * static_cast<int>(sr.sh) + a.Wi),
                                                 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t rs0 = mk(a.src[0]);
    const __amdgpu_buffer_rsrc_t rs1 = a.nsrc > 1 ? mk(a.src[1]) : rs0;
    const __amdgpu_buffer_rsrc_t rs2 = a.nsrc > 2 ? mk(a.src[2]) : rs0;
    const int sh0 = static_cast<int>(a.src[0].sh);
    const int sh1 = a.nsrc > 1 ? static_cast<int>(a.src[1].sh) : sh0;
    const int sh2 = a.nsrc > 2 ? static_cast<int>(a.src[2].sh) : sh0;
    const int sc0 = static_cast<int>(a.src[0].sc), sc1 = static_cast<int>(a.src[1].sc), sc2 = static_cast<int>(a.src[2].sc);
    unsigned vk[NKA];  // per-lane channel + column byte offset of k-step kk (kOOB past Cin)
#pragma unroll
    for (int kk = 0; kk < NKA; ++kk) {
        const int c0 = 4 * kk;
        const int lo = c0 < lo1 ? 0 : (c0 < lo2 ? lo1 : lo2);
        const int sc = c0 < lo1 ? sc0 : (c0 < lo2 ? sc1 : sc2);
        const int cl = c0 + kq - lo;
        vk[kk] = (c0 < a.Cin && c0 + kq < a.Cin) ? 4u * cl * sc + xoff : kOOB;
    }
    float bin[KA][NKA];
    auto load_a_row = [&](float (&dst)[KA][NKA], int ya) {
#pragma unroll
        for (int th = 0; th < KA; ++th) {
            const int yi = ya - A0 + th;
            const bool rok = yi >= 0 && yi < a.Hi;
#pragma unroll
            for (int kk = 0; kk < NKA; ++kk) {
                const int c0 = 4 * kk;  // the k-step's source: wave-uniform selects of named descriptors
                const __amdgpu_buffer_rsrc_t r = c0 < lo1 ? rs0 : (c0 < lo2 ? rs1 : rs2);
                const int sh = c0 < lo1 ? sh0 : (c0 < lo2 ? sh1 : sh2);
                const int roff = rok ? 4 * yi * sh : static_cast<int>(kOOB);
                dst[th][kk] = buf_load_s(r, vk[kk], roff);
            }
        }
    };

    const int yb0 = ty * rows_wg + wave * RW;  // first output row of this wave
    load_a_row(bin, yb0 - B0);

    // ---- both layers' weights -> LDS, one batch of loads (counts are compile-time constants)
    {
        constexpr int NA4 = TAPA * CINA * (CM / 4), NB4 = TAPB * CM * (4 * MB);
        constexpr int RA = (NA4 + kPairThreads - 1) / kPairThreads, RB = (NB4 + kPairThreads - 1) / kPairThreads;
        floatx4 ra[RA], rb[RB];
#pragma unroll
        for (int k = 0; k < RA; ++k) {
            const int i = min(static_cast<int>(threadIdx.x) + k * kPairThreads, NA4 - 1);
            const int row = i / (CM / 4), q4 = i - row * (CM / 4);  // row = tap * CINA + c
            const int tap = row / CINA, c = row - tap * CINA;
            const floatx4 v = *reinterpret_cast<const floatx4*>(
                a.w + (static_cast<long long>(tap) * a.cin_pad + min(c, a.cin_pad - 1)) * a.cout_pad + 4 * q4);
            ra[k] = c < a.cin_pad ? v : floatx4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = min(static_cast<int>(threadIdx.x) + k * kPairThreads, NB4 - 1);
            const int row = i / (4 * MB), q4 = i - row * (4 * MB);  // row = tap * CM + c
            const int tap = row / CM, c = row - tap * CM;
            const floatx4 v = *reinterpret_cast<const floatx4*>(
                bd.w + (static_cast<long long>(tap) * bd.cin_pad + min(c, bd.cin_pad - 1)) * bd.cout_pad + 4 * q4);
            rb[k] = c < bd.cin_pad ? v : floatx4{0.f, 0.f, 0.f, 0.f};
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < RA; ++k) {
            const int i = threadIdx.x + k * kPairThreads;
            const int row = i / (CM / 4), q4 = i - row * (CM / 4);
            if (i < NA4) *reinterpret_cast<floatx4*>(wa + row * WRA + 4 * q4) = ra[k];
        }
#pragma unroll
        for (int k = 0; k < RB; ++k) {
            const int i = threadIdx.x + k * kPairThreads;
            const int row = i / (4 * MB), q4 = i - row * (4 * MB);
            if (i < NB4) *reinterpret_cast<floatx4*>(wb + row * WRB + 4 * q4) = rb[k];
        }
    }
    // per-lane epilogue constants: A's channels 16ma + 4kq + j, B's couts 16mb + 4kq + j
    float sA[MA][4], hA[MA][4], sB[MB][4], hB[MB][4];
#pragma unroll
    for (int m = 0; m < MA; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int ch = min(16 * m + 4 * kq + j, a.Cout - 1);
            sA[m][j] = a.scale ? a.scale[ch] : 1.f;
            hA[m][j] = a.shift ? a.shift[ch] : 0.f;
        }
#pragma unroll
    for (int m = 0; m < MB; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = min(16 * m + 4 * kq + j, bd.Cout - 1);
            sB[m][j] = bd.scale ? bd.scale[co] : 1.f;
            hB[m][j] = bd.shift ? bd.shift[co] : 0.f;
        }
    __syncthreads();
    if (yb0 >= H) return;  // past the bottom (after the workgroup's only barrier)

    // rolling window of A's output rows (w[KB-1] newest)
    floatx4 win[KB][MA];
#pragma unroll
    for (int t = 0; t < KB; ++t)
#pragma unroll
        for (int m = 0; m < MA; ++m) win[t][m] = floatx4{0.f, 0.f, 0.f, 0.f};
    const int yb_end = min(H, yb0 + RW);
    const int steps = RW + KB - 1;
    for (int it = 0; it < steps; ++it) {
        const int ya = yb0 - B0 + it;
        float bnx[KA][NKA];
        load_a_row(bnx, ya + 1);          // next A row's operands, in flight during this step
        __builtin_amdgcn_sched_barrier(0);
        // ---- A row ya: MA x (16 channels x 16 pixels), two accumulation chains
        floatx4 acA[2][MA];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int m = 0; m < MA; ++m) acA[c][m] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int th = 0; th < KA; ++th)
#pragma unroll
            for (int kk = 0; kk < NKA; ++kk) {
                const float v = bin[th][kk];
#pragma unroll
                for (int tw = 0; tw < KA; ++tw) {
                    float bs;
                    if constexpr (KA == 1) bs = v;
                    else if (tw == 0) bs = row_shift<-1>(v);
                    else if (tw == 1) bs = v;
                    else bs = row_shift<1>(v);
                    const int tap = th * KA + tw;
#pragma unroll
                    for (int m = 0; m < MA; ++m) {
                        const float av = wa[(tap * CINA + 4 * kk + kq) * WRA + 16 * m + n16];
                        floatx4& acc = acA[(tap * NKA + kk) & 1][m];
                        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bs, acc, 0, 0, 0);
                    }
                }
            }
        const bool row_ok = ya >= 0 && ya < H;
#pragma unroll
        for (int t = 0; t + 1 < KB; ++t)
#pragma unroll
            for (int m = 0; m < MA; ++m) win[t][m] = win[t + 1][m];
#pragma unroll
        for (int m = 0; m < MA; ++m)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = 16 * m + 4 * kq + j;
                const float s = acA[0][m][j] + acA[1][m][j];
                const float v = pair_act(a.scale ? s * sA[m][j] + hA[m][j] : s + hA[m][j], a.act);
                win[KB - 1][m][j] = (row_ok && col_ok && ch < a.Cout) ? v : 0.f;  // B's zero padding
            }
#pragma unroll
        for (int th = 0; th < KA; ++th)
#pragma unroll
            for (int kk = 0; kk < NKA; ++kk) bin[th][kk] = bnx[th][kk];
        if (it < KB - 1) continue;
        const int yb = ya - B0;
        if (yb >= yb_end) continue;
        // ---- B row yb: k-step (m, j) = A channels 16m + 4g + j on lane group g
        floatx4 acB[2][MB];
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int m = 0; m < MB; ++m) acB[c][m] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int th = 0; th < KB; ++th)
#pragma unroll
            for (int ma = 0; ma < MA; ++ma)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const float v = win[th][ma][j];
#pragma unroll
                    for (int tw = 0; tw < KB; ++tw) {
                        float bs;
                        if constexpr (KB == 1) bs = v;
                        else if (tw == 0) bs = row_shift<-1>(v);
                        else if (tw == 1) bs = v;
                        else bs = row_shift<1>(v);
                        const int tap = th * KB + tw;
#pragma unroll
                        for (int mb = 0; mb < MB; ++mb) {
                            const float av = wb[(tap * CM + 16 * ma + 4 * kq + j) * WRB + 16 * mb + n16];
                            floatx4& acc = acB[(tap * 4 + j) & 1][mb];
                            acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bs, acc, 0, 0, 0);
                        }
                    }
                }
        if (n16 < HALO || n16 >= 16 - HALO || !col_ok) continue;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = 16 * mb + 4 * kq + j;
                if (co >= bd.Cout) continue;
                const float s = acB[0][mb][j] + acB[1][mb][j];
                float v = pair_act(bd.scale ? s * sB[mb][j] + hB[mb][j] : s + hB[mb][j], bd.act);
                if (bd.res) v = v + bd.res[b * bd.rb + co * bd.rc + static_cast<long long>(yb) * bd.rh + col];
                bd.out[b * bd.ob + co * bd.oc + static_cast<long long>(yb) * bd.oh + col] = v * bd.post_scale;
            }
    }
}

template <int KA, int KB, int MA, int MB, int NKA>
int launch_pair_t(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    using G = PGeo<KA, KB, MA, MB, NKA>;
    if (G::BYTES > 64 * 1024) return ESM_ERR_UNSUPPORTED;
    const int H = b.Ho, W = b.Wo;
    const long long tiles_w = (W + G::VALID - 1) / G::VALID;
    const long long rows = static_cast<long long>(a.B) * H * tiles_w;
    // rows per wave (each A row is computed once and reused by KB output rows; the first KB-1 are
    // the wave's warm-up).  Swept on MI355X in the S-K launch sequence: the 192x624 agg_1 pair is
    // fastest at 3 (31.1 us vs 35.9 at 4, 37.5 at 2), the 24x78 FMBlock pairs at 1 (10.4 vs 12.6 at 2),
    // and in the L sequence the 96x312 FMBlock pairs at 1 too (15.9 vs 18.8 us at 2)
    const int rw = rows >= 6144 ? 3 : 1;
    const long long nwg = tiles_w * ((H + 4 * rw - 1) / (4 * rw)) * a.B;
    if (nwg > 0x7fffffffLL) return arg_error("conv pair: grid too large");
    hipLaunchKernelGGL((pair_kernel<KA, KB, MA, MB, NKA>), dim3(static_cast<unsigned>(nwg)), dim3(kPairThreads),
                       G::BYTES, s, a, b, rw);
    return check_launch("conv pair");
}

template <int KA, int KB, int MA, int MB>
int launch_pair_nk(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    const int nk = (a.Cin + 3) / 4;
    if constexpr (KA == 1) {
        if (nk <= 8) return launch_pair_t<KA, KB, MA, MB, 8>(a, b, s);
        if (nk <= 16) return launch_pair_t<KA, KB, MA, MB, 16>(a, b, s);
        if (nk <= 24) return launch_pair_t<KA, KB, MA, MB, 24>(a, b, s);
    } else {
        if (nk <= 2) return launch_pair_t<KA, KB, MA, MB, 2>(a, b, s);
        if (nk <= 4) return launch_pair_t<KA, KB, MA, MB, 4>(a, b, s);
        if (nk <= 8) return launch_pair_t<KA, KB, MA, MB, 8>(a, b, s);
        if (nk <= 12) return launch_pair_t<KA, KB, MA, MB, 12>(a, b, s);
    }
    return ESM_ERR_UNSUPPORTED;
}

template <int KA, int KB>
int launch_pair_m(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    const int ma = a.Cout > 16 ? 2 : 1, mb = b.Cout > 16 ? 2 : 1;
    if (ma == 1 && mb == 1) return launch_pair_nk<KA, KB, 1, 1>(a, b, s);
    if (ma == 2 && mb == 1) return launch_pair_nk<KA, KB, 2, 1>(a, b, s);
    if (ma == 1 && mb == 2) return launch_pair_nk<KA, KB, 1, 2>(a, b, s);
    return launch_pair_nk<KA, KB, 2, 2>(a, b, s);
}

bool plain_2d(const esm_conv_desc& d) {
    return !d.transposed && d.stride == 1 && d.kd == 1 && d.Di == 1 && d.Do == 1 && d.kh == d.kw &&
           (d.kh == 1 || d.kh == 3) && d.ph == d.kh / 2 && d.pw == d.kw / 2 && d.Ho == d.Hi && d.Wo == d.Wi &&
           d.shuffle <= 1 && !d.mul && !d.up && !d.out2;
}

}  // namespace

int launch_conv_pair(const esm_conv_desc* pa, const esm_conv_desc* pb, hipStream_t s) {
    if (!pa || !pb) return arg_error("conv pair: null descriptor");
    const esm_conv_desc& a = *pa;
    const esm_conv_desc& b = *pb;
    if (!plain_2d(a) || !plain_2d(b) || a.res)
        return arg_error("conv pair: both layers must be stride-1 2-D k1/k3 same-padding convs without extra epilogues");
    if (a.nsrc < 1 || a.nsrc > ESM_MAX_SRC || !a.w || !b.w || !b.out) return arg_error("conv pair: bad descriptor");
    int cin = 0;
    for (int i = 0; i < a.nsrc; ++i) {
        const esm_src& r = a.src[i];
        if (!r.ptr || r.C <= 0 || (a.nsrc > 1 && (r.C & 3))) return arg_error("conv pair: sources must split on 4 channels");
        const long long last = (r.C - 1) * r.sc + (a.Hi - 1) * r.sh + a.Wi;
        if (4 * last >= kOOB || r.sc > (1 << 28) || r.sh > (1 << 28)) return arg_error("conv pair: source too large");
        cin += r.C;
    }
    if (cin != a.Cin || a.B != b.B || b.Cin != a.Cout || b.Hi != a.Ho || b.Wi != a.Wo || a.Cout > 32 || b.Cout > 32 ||
        a.Cin > 96)
        return arg_error("conv pair: inconsistent shapes");
    int rc = ESM_ERR_UNSUPPORTED;
    if (a.kh == 1 && b.kh == 3) rc = launch_pair_m<1, 3>(a, b, s);
    else if (a.kh == 3 && b.kh == 3) rc = launch_pair_m<3, 3>(a, b, s);
    else if (a.kh == 3 && b.kh == 1) rc = launch_pair_m<3, 1>(a, b, s);
    if (rc == ESM_ERR_UNSUPPORTED) set_error("conv pair: no fused form for this pair (run the two convs separately)");
    return rc;
}

}  // namespace conv
}  // namespace esm

extern "C" int esm_conv_pair_f32(const esm_conv_desc* a, const esm_conv_desc* b, void* stream) {
    return esm::conv::launch_conv_pair(a, b, esm::as_stream(stream));
}
