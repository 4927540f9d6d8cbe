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

// ---------------------------------------------------------------------------------------------
// Lean 1x1 -> 3x3 pair (the full-resolution agg_1 of up_refinement, models/ESMStereo.py:228-235:
// conv1x1 over the [u2, c1, left_f2x] concat -> BN -> GELU -> conv3x3 -> BN -> GELU).  The same
// algorithm as pair_kernel above, with the instruction overhead that bound it (profiles/
// r02_pmc_sq_ops_SK.txt: ~2600 VALU + ~1800 SALU per wave, SGPR spills, one LDS weight read per
// MFMA) removed:
//   * both layers' weights live in VGPRs for the whole wave (NKA*MA + 9*4*MA*MB registers);
//   * the concat sources are addressed through ONE buffer descriptor based at the lowest source
//     (the launcher checks that every source's whole batch span lies in a window addressable with
//     the kOOB marking): a k-step's source is folded into its per-lane voffset once, so a row's
//     loads share one descriptor and one soffset (no per-k-step source selection);
//   * the R output rows of a wave are compile-time: the row loop is unrolled, only the R + 2 A rows
//     the block needs are computed, and each A row is DPP-shifted once into the three horizontal
//     taps' operands, reused by the three B rows it feeds;
//   * the next A row's loads are in flight during the current row's MFMAs (loading all R + 2 rows up
//     front measured slower: 38 vs 29 us at 192x624, the registers halve the waves per SIMD).
template <int NKA, int MA, int MB, int R, int ACT>
__global__ void __launch_bounds__(kPairThreads) lpair_kernel(const esm_conv_desc a, const esm_conv_desc bd,
                                                             const float* wbase, int wspan, int d0, int d1, int d2) {
    constexpr int HALO = 1, VALID = 14, NRA = R + 2;
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n16 = lane & 15, kq = lane >> 4;
    const int H = bd.Ho, W = bd.Wo;
    const int tx = blockIdx.x * 4 + wave;
    const int y0 = blockIdx.y * R;
    const int b = blockIdx.z;
    const int col = tx * VALID - HALO + n16;  // image column of this lane (A and B tiles alike)
    const bool col_ok = col >= 0 && col < W;

    // ---- weights -> VGPRs.  A: k-step g, lane (kq, n16) = channel 4g + kq, A-cout 16ma + n16.
    //      B: k-step (ma, j) = A channels 16ma + 4kq + j on lane group kq, B-cout 16mb + n16.
    float wa[NKA][MA], wb[9][MA][4][MB];
    {
        const __amdgpu_buffer_rsrc_t ra = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(a.w), static_cast<short>(0), 4 * a.cin_pad * a.cout_pad, 0x00020000);
        const __amdgpu_buffer_rsrc_t rb = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<float*>(bd.w), static_cast<short>(0), 4 * 9 * bd.cin_pad * bd.cout_pad, 0x00020000);
#pragma unroll
        for (int g = 0; g < NKA; ++g)
#pragma unroll
            for (int m = 0; m < MA; ++m)
                wa[g][m] = buf_load_s(ra, 4u * ((4 * g + kq) * a.cout_pad + 16 * m + n16), 0);
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
            for (int m = 0; m < MA; ++m)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int mb = 0; mb < MB; ++mb)
                        wb[t][m][j][mb] = buf_load_s(
                            rb, 4u * ((t * bd.cin_pad + 16 * m + 4 * kq + j) * bd.cout_pad + 16 * mb + n16), 0);
    }
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

    // ---- A's input: per-lane byte offset of k-step g from the window base (kOOB outside)
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wbase), static_cast<short>(0), wspan, 0x00020000);
    const int lo1 = a.src[0].C, lo2 = a.src[0].C + a.src[1].C;
    unsigned vk[NKA];
#pragma unroll
    for (int g = 0; g < NKA; ++g) {
        const int c = 4 * g + kq;
        const int s = c < lo1 ? 0 : (c < lo2 ? 1 : 2);
        const int cl = c - (s == 0 ? 0 : (s == 1 ? lo1 : lo2));
        const long long sb = s == 0 ? a.src[0].sb : (s == 1 ? a.src[1].sb : a.src[2].sb);
        const long long sc = s == 0 ? a.src[0].sc : (s == 1 ? a.src[1].sc : a.src[2].sc);
        const int dl = s == 0 ? d0 : (s == 1 ? d1 : d2);
        vk[g] = (c < a.Cin && col_ok) ? static_cast<unsigned>(dl + 4 * (b * sb + cl * sc + col)) : kOOB;
    }
    const int sh = static_cast<int>(a.src[0].sh);  // every source: the same row stride (launcher)
    auto load_a = [&](float (&dst)[NKA], int ya) {
        const int roff = (ya >= 0 && ya < H) ? 4 * ya * sh : static_cast<int>(kOOB);
#pragma unroll
        for (int g = 0; g < NKA; ++g) dst[g] = buf_load_s(rs, vk[g], roff);
    };

    floatx4 acc[R][MB];
#pragma unroll
    for (int r = 0; r < R; ++r)
#pragma unroll
        for (int m = 0; m < MB; ++m) acc[r][m] = floatx4{0.f, 0.f, 0.f, 0.f};
    const bool store_lane = n16 >= HALO && n16 < 16 - HALO && col_ok;

    // software pipeline, one A row ahead: iteration ia issues the loads of A row ia + 2 and the MFMAs of
    // A row ia + 1 before the epilogue (VALU) of A row ia, so the matrix pipe has independent work
    // while the wave evaluates GELU (the per-wave phases were serial: PMC showed 43-50 % issue stalls)
    float bin[3][NKA];
    floatx4 aA[2][2][MA];  // [A row parity][accumulation chain][m]
    auto a_mfma = [&](int ia) {
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
            for (int m = 0; m < MA; ++m) aA[ia & 1][c][m] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int g = 0; g < NKA; ++g)
#pragma unroll
            for (int m = 0; m < MA; ++m)
                aA[ia & 1][g & 1][m] =
                    __builtin_amdgcn_mfma_f32_16x16x4f32(wa[g][m], bin[ia % 3][g], aA[ia & 1][g & 1][m], 0, 0, 0);
    };
    load_a(bin[0], y0 - 1);
    load_a(bin[1], y0);
    a_mfma(0);
#pragma unroll
    for (int ia = 0; ia < NRA; ++ia) {  // A row y0 - 1 + ia feeds B rows ia - dy (dy = 0..2)
        if (ia + 2 < NRA) load_a(bin[(ia + 2) % 3], y0 + ia + 1);
        __builtin_amdgcn_sched_barrier(0);
        if (ia + 1 < NRA) a_mfma(ia + 1);
        // A's epilogue; zero outside the image (B's zero padding) and past A's couts
        const int ya = y0 - 1 + ia;
        const bool row_ok = ya >= 0 && ya < H;
        float v3[3][MA][4];  // the three horizontal taps' B operands (columns n - 1, n, n + 1)
#pragma unroll
        for (int m = 0; m < MA; ++m)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int ch = 16 * m + 4 * kq + j;
                const float sum = aA[ia & 1][0][m][j] + aA[ia & 1][1][m][j];
                const float v = act_t<ACT>(a.scale ? sum * sA[m][j] + hA[m][j] : sum + hA[m][j], a.act);
                const float z = (row_ok && col_ok && ch < a.Cout) ? v : 0.f;
                v3[0][m][j] = row_shift<-1>(z);
                v3[1][m][j] = z;
                v3[2][m][j] = row_shift<1>(z);
            }
#pragma unroll
        for (int dy = 0; dy < 3; ++dy) {
            const int ro = ia - dy;  // B row (block-relative) fed by this A row through tap row dy
            if (ro < 0 || ro >= R) continue;
#pragma unroll
            for (int m = 0; m < MA; ++m)
#pragma unroll
                for (int j = 0; j < 4; ++j)
#pragma unroll
                    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
                        for (int mb = 0; mb < MB; ++mb)
                            acc[ro][mb] = __builtin_amdgcn_mfma_f32_16x16x4f32(wb[dy * 3 + dx][m][j][mb], v3[dx][m][j],
                                                                               acc[ro][mb], 0, 0, 0);
        }
        const int rf = ia - 2;  // B row complete after its last A row
        if (rf < 0) continue;
        const int yb = y0 + rf;
        if (yb >= H || !store_lane) continue;
#pragma unroll
        for (int mb = 0; mb < MB; ++mb)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = 16 * mb + 4 * kq + j;
                if (co >= bd.Cout) continue;
                const float s = acc[rf][mb][j];
                float v = act_t<ACT>(bd.scale ? s * sB[mb][j] + hB[mb][j] : s + hB[mb][j], bd.act);
                if (bd.res) v = v + bd.res[b * bd.rb + co * bd.rc + static_cast<long long>(yb) * bd.rh + col];
                bd.out[b * bd.ob + co * bd.oc + static_cast<long long>(yb) * bd.oh + col] = v * bd.post_scale;
            }
    }
}

// Lean 1x1 -> 3x3 form, when its preconditions hold: returns ESM_ERR_UNSUPPORTED (no launch) otherwise.
template <int MA, int MB>
int launch_lpair_m(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s, const float* base, int span,
                   const int (&dl)[3], int nk, int R) {
    const int H = b.Ho, W = b.Wo;
    const dim3 grid(ceil_div(ceil_div(W, 14), 4), ceil_div(H, R), static_cast<unsigned>(a.B));
    if (grid.y > 65535u || grid.z > 65535u) return ESM_ERR_UNSUPPORTED;
    // both BasicConvs of the hot path end in GELU: that case compiled with the activation folded in
    const bool gg = a.act == ESM_ACT_GELU && b.act == ESM_ACT_GELU;
#define ESM_LPAIR(NK, RR)                                                                                          \
    do {                                                                                                          \
        if (gg)                                                                                                   \
            hipLaunchKernelGGL((lpair_kernel<NK, MA, MB, RR, ESM_ACT_GELU>), grid, dim3(kPairThreads), 0, s, a, b, \
                               base, span, dl[0], dl[1], dl[2]);                                                  \
        else                                                                                                      \
            hipLaunchKernelGGL((lpair_kernel<NK, MA, MB, RR, -1>), grid, dim3(kPairThreads), 0, s, a, b, base,     \
                               span, dl[0], dl[1], dl[2]);                                                        \
    } while (0)
    if (nk <= 4) { if (R == 4) ESM_LPAIR(4, 4); else ESM_LPAIR(4, 2); }
    else if (nk <= 8) { if (R == 4) ESM_LPAIR(8, 4); else ESM_LPAIR(8, 2); }
    else if (nk <= 16) { if (R == 4) ESM_LPAIR(16, 4); else ESM_LPAIR(16, 2); }
    else if (nk <= 24 && MA == 1) ESM_LPAIR(24, 2);  // 4 rows: 264 registers, one wave per SIMD
    else return ESM_ERR_UNSUPPORTED;
#undef ESM_LPAIR
    return check_launch("conv pair (lean)");
}

int launch_lpair(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    if (a.kh != 1 || b.kh != 3 || b.res || b.out2) return ESM_ERR_UNSUPPORTED;
    // one descriptor over every source's whole batch span (conv_direct.h source_window)
    const float* base = nullptr;
    int span = 0, dl[ESM_MAX_SRC];
    if (!source_window(a, &base, &span, dl)) return ESM_ERR_UNSUPPORTED;
    const int nk = (a.Cin + 3) / 4;
    const long long units = static_cast<long long>(a.B) * b.Ho * ceil_div(b.Wo, 14);
    const int R = units >= 4LL * 2048 ? 4 : 2;  // rows per wave: ~2+ waves per SIMD either way
    const int ma = a.Cout > 16 ? 2 : 1, mb = b.Cout > 16 ? 2 : 1;
    if (ma == 1 && mb == 1) return launch_lpair_m<1, 1>(a, b, s, base, span, dl, nk, R);
    if (ma == 1 && mb == 2) return launch_lpair_m<1, 2>(a, b, s, base, span, dl, nk, R);
    return ESM_ERR_UNSUPPORTED;
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
    // the lean 1x1 -> 3x3 form unless a.hint asks for the LDS-weight kernel (bit 23: A/B, tests)
    if (a.kh == 1 && b.kh == 3 && !(a.hint & (1 << 23))) rc = launch_lpair(a, b, s);
    if (rc != ESM_ERR_UNSUPPORTED) return rc;
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
