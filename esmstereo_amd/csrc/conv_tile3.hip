// LDS-tiled implicit-GEMM 3-D convolution for the large volumes of ESMStereo-L / -M (BasicConv 3-D,
// models/submodule.py:12-38, in the stems and the aggregation hourglass, models/ESMStereo.py:129-182,
// 610-622): 3x3x3 stride 1 / 2 padding 1 and 1x1x1, where at KITTI size and above each layer is a dense
// GEMM of M = Cout (8..72), N = voxels (10^5..10^7), K = 27 Cin (216..1944) and the MFMA pipe, not
// latency, bounds the launch.  The register-operand forms (conv_direct.h, conv_stem.hip, conv_wide3.hip)
// fetch every MFMA operand from L1/L2 per wave; here a workgroup stages its input window and the
// weights of one 4-channel k-step in LDS (global loads for the next k-step in flight while the MFMAs of
// this one run: double-buffered LDS, one barrier per k-step) and every MFMA operand is a conflict-free
// ds_read_b32:
//   * GEMM orientation (v_mfma_f32_16x16x4_f32): A = weights (16 couts x 4 channels), B = input (4
//     channels x 16 output columns), D = 16 couts x 16 columns -> each store instruction writes 16
//     consecutive x of one cout;
//   * a wave owns 16 columns x NT rows of one output plane and MT cout tiles; for each (dz, dx) tap pair
//     it reads the NT + 2 (stride 2: 2 NT + 1) input rows once and feeds them to the three dy taps;
//   * <= 8 couts (the stems: group_stem 32 -> 8, agg 8 -> 8): the 16 MFMA rows carry 8 couts of two
//     output planes (PZ); input plane 2q + p (p = 0..3) reaches the pair q through the composite weight
//     A_p[(h, co)][ci] = W[dz = p - h][ci][co] (zero outside 0..2), staged in LDS once per k-step, so a
//     pair costs 36 MFMAs per k-step instead of the 54 of two half-empty tiles;
//   * bank-conflict-free reads: the input image's channel stride is = 16 (stride 1) or = 1 (stride 2)
//     mod 32 banks, the weight rows' stride = 16 mod 32 (MI355X_MICROARCH.md LDS table, ds_read_b32);
//   * partial sums never leave the wave: the K loop runs over every channel chunk in order, so each
//     output is one fixed-order sum (deterministic, independent of the tiling).
// Epilogue as the other forms: folded BN scale / shift, activation, optional * mul, + res, * post_scale
// and the second copy, write-through (sc1) buffer stores.
#include "conv_up1.h"

namespace esm {
namespace conv {
namespace {

constexpr int kT3Threads = 256;
constexpr bool kT3Dma = true;  // buffer-to-LDS staging where a form has it (hint bit 28 turns it off per launch)

// D2: a 2-D conv (one plane, kd = 1): the same pipeline with the depth dimension of extent 1
// DMA (round 6): the input window is staged by buffer_load ... lds (global -> LDS, no staging registers): per
// channel NCH chunks of 64 consecutive window elements, one wave-instruction each, so a channel's LDS stride is
// NCH * 64 + CMOD (the chunk tail lanes write zeros into the padding)
template <int S, int K, int NT, int WZ, bool PZ, int MT, bool D2 = false, bool DMA = false>
struct T3Geo {
    static constexpr int WY = 4 / WZ;                     // waves along y
    static constexpr int ZB = PZ ? 2 * WZ : WZ;           // output planes per workgroup
    static constexpr int YB = WY * NT;                    // output rows per workgroup
    static constexpr int KD = D2 ? 1 : K;                 // depth taps
    static constexpr int IZ = D2 ? 1 : (ZB - 1) * S + K, IY = (YB - 1) * S + K, IX = 15 * S + K;  // input window
    static constexpr int PLANE = IY * IX;
    static constexpr int CS0 = IZ * PLANE;
    static constexpr int CMOD = S == 1 ? 16 : 1;          // channel stride mod 32 (bank offset of lanes 16..31)
    static constexpr int NCH = (CS0 + 63) / 64;
    static constexpr int CS = DMA ? NCH * 64 + CMOD : CS0 + ((CMOD - CS0 % 32) % 32 + 32) % 32;
    static constexpr int XE = 4 * CS0;                    // staged input elements per k-step
    static constexpr int XL = 4 * CS;                     // LDS floats per input buffer
    static constexpr int TAPS = KD * K * K;
    static constexpr int WCS = PZ ? 16 : (MT % 2 ? MT * 16 : MT * 16 + 16);  // weight row stride (= 16 mod 32)
    static constexpr int WE = PZ ? 4 * 9 * 4 * 16 : TAPS * 4 * MT * 16;      // staged weight elements
    static constexpr int WL = PZ ? WE : TAPS * 4 * WCS;                      // LDS floats per weight buffer
    static constexpr int XR = (XE + kT3Threads - 1) / kT3Threads;
    static constexpr int WR = (WE + kT3Threads - 1) / kT3Threads;
    static constexpr int NR = (NT - 1) * S + K;           // input rows a wave reads per (dz, dx)
};

// NS: input sources (a channel concat of up to 3, 4-channel aligned splits; 1x1x1 only): every k-step
// lies inside one source, whose descriptor and offsets are selected per k-step (wave-uniform)
// WREG (plane pairs and the stride-2 MT form, round 6): each lane loads its (composite-)weight A operands
// straight into registers (36, or 27 MT, per k-step, reloaded for the next k-step right after their last MFMA)
// instead of the workgroup staging them in LDS: 18 KB less LDS per workgroup (agg at L-K: 2 -> 4 workgroups per
// CU), no weight stores
template <int S, int K, int MT, int NT, int WZ, bool PZ, int ACT, bool PLAIN, int NS = 1, bool D2 = false, bool WREG = false,
          bool DMA = false>
__global__ void __launch_bounds__(kT3Threads, (WREG && !PZ && MT <= 2) ? 4 : 1) tconv3_kernel(const esm_conv_desc a, int ncg) {
    using G = T3Geo<S, K, NT, WZ, PZ, MT, D2, DMA>;
    static_assert(!DMA || (WREG && NS == 1), "DMA staging: register weights, one source");
    static_assert(!WREG || PZ || (K == 3 && !D2 && NS == 1), "register weights: plane pairs or 3x3x3 MT");
    constexpr int NWA = PZ ? 36 : G::TAPS * MT;  // register A operands per k-step (WREG)
    constexpr int IY = G::IY, IX = G::IX, PLANE = G::PLANE, CS = G::CS, WCS = G::WCS;
    constexpr int XR = DMA ? 1 : G::XR, WR = WREG ? 1 : G::WR, NR = G::NR;
    // (two arrays, not one [2][..]: with DMA staging the waitcnt pass can then tell the buffer being filled from
    // the one being read)
    __shared__ __attribute__((aligned(16))) float xs0[G::XL];
    __shared__ __attribute__((aligned(16))) float xs1[G::XL];
    auto xsb = [&](int buf) __attribute__((always_inline)) { return buf ? xs1 : xs0; };
    __shared__ __attribute__((aligned(16))) float ws[WREG ? 1 : 2][WREG ? 1 : G::WL];

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int zw = wave % WZ, yw = wave / WZ;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int xo0 = bk_.x * 16, yo0 = bk_.y * G::YB;
    const int nzb = (a.Do + G::ZB - 1) / G::ZB;
    const int zz = bk_.z;
    const int mg = zz % ncg;
    const int r1 = zz / ncg;
    const int b = r1 / nzb;
    const int zo0 = (r1 - b * nzb) * G::ZB;
    const int zi0 = D2 ? 0 : zo0 * S - a.pd, yi0 = yo0 * S - a.ph, xi0 = xo0 * S - a.pw;

    // the sources as opaque wave-uniform scalars: selecting between fields of a.src[0..2] by the k-step's
    // source lets the optimizer fold the select into a run-time index of the kernarg struct, which it then
    // copies to scratch; read through readfirstlane, the fields cannot be merged
    auto u32 = [](int v) __attribute__((always_inline)) { return __builtin_amdgcn_readfirstlane(v); };
    auto u64 = [&](long long v) __attribute__((always_inline)) {
        const unsigned long long w = static_cast<unsigned long long>(v);
        return static_cast<long long>((static_cast<unsigned long long>(static_cast<unsigned>(u32(static_cast<int>(w >> 32))))
                                       << 32) |
                                      static_cast<unsigned>(u32(static_cast<int>(w & 0xffffffffu))));
    };
    auto uptr = [&](const float* ptr) __attribute__((always_inline)) {
        return reinterpret_cast<const float*>(u64(static_cast<long long>(reinterpret_cast<uintptr_t>(ptr))));
    };
    const float* p0 = a.src[0].ptr;
    const float* p1 = NS > 1 ? uptr(a.src[1].ptr) : p0;
    const float* p2 = NS > 2 ? uptr(a.src[2].ptr) : p0;
    const int C0 = a.src[0].C, C1 = NS > 1 ? u32(a.src[1].C) : 0, C2 = NS > 2 ? u32(a.src[2].C) : 0;
    const int sc0 = static_cast<int>(a.src[0].sc), sd0 = static_cast<int>(a.src[0].sd), sh0 = static_cast<int>(a.src[0].sh);
    const int sc1 = NS > 1 ? u32(static_cast<int>(a.src[1].sc)) : sc0, sd1 = NS > 1 ? u32(static_cast<int>(a.src[1].sd)) : sd0,
              sh1 = NS > 1 ? u32(static_cast<int>(a.src[1].sh)) : sh0;
    const int sc2 = NS > 2 ? u32(static_cast<int>(a.src[2].sc)) : sc0, sd2 = NS > 2 ? u32(static_cast<int>(a.src[2].sd)) : sd0,
              sh2 = NS > 2 ? u32(static_cast<int>(a.src[2].sh)) : sh0;
    const long long sb0 = a.src[0].sb, sb1 = NS > 1 ? u64(a.src[1].sb) : sb0, sb2 = NS > 2 ? u64(a.src[2].sb) : sb0;
    auto rsrc = [&](const float* ptr, long long sb, int C, int sc, int sd, int sh) __attribute__((always_inline)) {
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(ptr + b * sb), static_cast<short>(0),
                                                 4 * ((C - 1) * sc + (a.Di - 1) * sd + (a.Hi - 1) * sh + a.Wi),
                                                 0x00020000);
    };
    const __amdgpu_buffer_rsrc_t rs0 = rsrc(p0, sb0, C0, sc0, sd0, sh0);
    const int lo1 = C0, lo2 = C0 + C1;  // first channel of sources 1 and 2
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w), static_cast<short>(0), 4 * G::TAPS * a.cin_pad * a.cout_pad, 0x00020000);

    // ---- per-thread staging slots (the same window for every k-step; the k-step's channel offset goes
    //      into the wave-uniform soffset)
    // slot k's element e = tid + 256 k: channel e / CS0, LDS index e + channel * (CS - CS0) (recomputed
    // from e where used: only the global offset is kept in a register)
    unsigned xoff[NS][XR];
#pragma unroll
    for (int k = 0; k < (DMA ? 0 : XR); ++k) {
        const int e = tid + k * kT3Threads;
        const int ix = e % IX, iy = (e / IX) % IY, iz = (e / PLANE) % G::IZ, ci = e / G::CS0;
        const int zi = zi0 + iz, yi = yi0 + iy, xi = xi0 + ix;
        const bool ok = e < G::XE && zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
#pragma unroll
        for (int q = 0; q < NS; ++q) {
            const int scq = q == 0 ? sc0 : (q == 1 ? sc1 : sc2), sdq = q == 0 ? sd0 : (q == 1 ? sd1 : sd2);
            const int shq = q == 0 ? sh0 : (q == 1 ? sh1 : sh2);
            xoff[q][k] = ok ? 4u * static_cast<unsigned>(ci * scq + zi * sdq + yi * shq + xi) : kOOB;
        }
    }
    unsigned woff[WR];
    int wdst[WR];
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        const int e = tid + k * kT3Threads;
        bool ok = e < G::WE;
        unsigned off = 0;
        int dst = -1;
        if constexpr (PZ) {  // e = ((p * 9 + t9) * 4 + ci) * 16 + m
            const int m = e & 15, ci = (e >> 4) & 3, t9 = (e >> 6) % 9, p = (e >> 6) / 9;
            const int dz = p - (m >> 3), co = m & 7;
            ok = ok && dz >= 0 && dz <= 2 && co < a.Cout;
            off = 4u * static_cast<unsigned>(((dz * 9 + t9) * a.cin_pad + ci) * a.cout_pad + co);
            dst = e < G::WE ? e : -1;
        } else {  // e = (tap * 4 + ci) * (MT * 16) + m
            const int m = e % (MT * 16), ci = (e / (MT * 16)) & 3, tap = e / (MT * 64);
            const int co = mg * MT * 16 + m;
            ok = ok && co < a.cout_pad;
            off = 4u * static_cast<unsigned>((tap * a.cin_pad + ci) * a.cout_pad + co);
            dst = e < G::WE ? (tap * 4 + ci) * WCS + m : -1;
        }
        woff[k] = ok ? off : kOOB;
        wdst[k] = dst;
    }
    float xv[XR], wv[WR];
    // DMA: wave w issues the chunks i = w + 4 k (k < NCH) of the 4 x NCH per k-step: channel i / NCH, window elements
    // 64 (i % NCH) + lane (past the window: zeros into the channel's padding)
    constexpr int NCH = G::NCH;
    unsigned doff[DMA ? NCH : 1];
    if constexpr (DMA) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const int i = wave + 4 * k, c = i / NCH, e = (i - c * NCH) * 64 + lane;
            const int ix = e % IX, iy = (e / IX) % IY, iz = e / PLANE;
            const int zi = zi0 + iz, yi = yi0 + iy, xi = xi0 + ix;
            const bool ok = e < G::CS0 && zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
            doff[k] = ok ? 4u * static_cast<unsigned>(c * sc0 + zi * sd0 + yi * sh0 + xi) : kOOB;
        }
    }
    auto stage_dma = [&](int c0, int buf) __attribute__((always_inline)) {
        if constexpr (DMA) {
#pragma unroll
            for (int k = 0; k < NCH; ++k) {
                const int i = wave + 4 * k, c = i / NCH;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs0, (__attribute__((address_space(3))) void*)(xsb(buf) + c * CS + (i - c * NCH) * 64), 4,
                    c0 + c < a.Cin ? doff[k] : kOOB, 4 * c0 * sc0, 0, 0);
            }
        }
    };
    // DMA: the LDS writes of the buffer-to-LDS loads land before the barrier that publishes them
    auto dma_wait = [&]() __attribute__((always_inline)) {
        if constexpr (DMA) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0)
    };
    // the k-step's loads from source Q (compile-time: every array index stays constant; a run-time select
    // between xoff[0][k] and xoff[1][k] becomes a dynamic index of a private array, i.e. scratch)
    auto load_src = [&](auto qc, int c0) __attribute__((always_inline)) {
        constexpr int Q = decltype(qc)::value;
        const __amdgpu_buffer_rsrc_t rq =
            Q == 0 ? rs0 : (Q == 1 ? rsrc(p1, sb1, C1, sc1, sd1, sh1) : rsrc(p2, sb2, C2, sc2, sd2, sh2));
        const int cq = c0 - (Q == 0 ? 0 : (Q == 1 ? lo1 : lo2));
        const int scq = Q == 0 ? sc0 : (Q == 1 ? sc1 : sc2);
#pragma unroll
        for (int k = 0; k < (DMA ? 0 : XR); ++k) {
            const int ci = (tid + k * kT3Threads) / G::CS0;
            xv[k] = buf_load_s(rq, c0 + ci < a.Cin ? xoff[Q][k] : kOOB, 4 * cq * scq);
        }
    };
    auto stage_load = [&](int c0) __attribute__((always_inline)) {
        // the k-step's source (4-channel aligned splits: channels c0 .. c0 + 3 lie in one); uniform branch
        if (NS == 1 || c0 < lo1) {
            load_src(std::integral_constant<int, 0>{}, c0);
        } else if (NS == 2 || c0 < lo2) {
            load_src(std::integral_constant<int, (NS > 1 ? 1 : 0)>{}, c0);
        } else {
            load_src(std::integral_constant<int, (NS > 2 ? 2 : 0)>{}, c0);
        }
        if constexpr (!WREG) {
#pragma unroll
            for (int k = 0; k < WR; ++k) wv[k] = buf_load_s(wrs, woff[k], 4 * c0 * a.cout_pad);
        }
    };
    auto stage_store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < (DMA ? 0 : XR); ++k) {
            const int e = tid + k * kT3Threads;
            if (e < G::XE) xsb(buf)[e + (e / G::CS0) * (CS - G::CS0)] = xv[k];
        }
        if constexpr (!WREG) {
#pragma unroll
            for (int k = 0; k < WR; ++k)
                if (wdst[k] >= 0) ws[buf][wdst[k]] = wv[k];
        }
    };
    // WREG: lane (g, n)'s A operand of (input plane p, tap t9) at the k-step of channel c0 is
    // W[dz = p - n / 8][t9][c0 + g][n % 8] (zero outside dz 0..2 or past Cout); the MT form (round 6, the stride-2
    // downsamplers): operand (tap, mt) is W[tap][c0 + g][mg MT 16 + 16 mt + n], 27 MT registers
    constexpr int NWP = PZ ? 4 : MT;
    unsigned wpo[NWP];
    float wa[WREG ? NWA : 1];
    if constexpr (WREG) {
#pragma unroll
        for (int p = 0; p < NWP; ++p) {
            if constexpr (PZ) {
                const int dz = p - (n >> 3), co = n & 7;
                wpo[p] = (dz >= 0 && dz <= 2 && co < a.Cout)
                             ? 4u * static_cast<unsigned>((dz * 9 * a.cin_pad + g) * a.cout_pad + co)
                             : kOOB;
            } else {
                const int co = mg * MT * 16 + p * 16 + n;
                wpo[p] = co < a.cout_pad ? 4u * static_cast<unsigned>(g * a.cout_pad + co) : kOOB;
            }
        }
    }
    auto wreg_load = [&](int i, int c0) __attribute__((always_inline)) {
        if constexpr (WREG && PZ) wa[i] = buf_load_s(wrs, wpo[i / 9], 4 * ((i % 9) * a.cin_pad + c0) * a.cout_pad);
        if constexpr (WREG && !PZ) wa[i] = buf_load_s(wrs, wpo[i % MT], 4 * ((i / MT) * a.cin_pad + c0) * a.cout_pad);
    };

    // epilogue constants, loaded while the first k-step streams in (the register-weight MT form: in the
    // epilogue, 16 registers it needs for the weights)
    constexpr int NCO = PZ ? 1 : MT;
    constexpr bool LATE_BN = WREG && !PZ;
    float scl[NCO][4], shf[NCO][4];
    auto load_bn = [&]() __attribute__((always_inline)) {
#pragma unroll
        for (int mt = 0; mt < NCO; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = PZ ? ((4 * g + j) & 7) : mg * MT * 16 + mt * 16 + 4 * g + j;
                const int cc = min(co, a.Cout - 1);
                scl[mt][j] = a.scale ? a.scale[cc] : 1.f;
                shf[mt][j] = a.shift ? a.shift[cc] : 0.f;
            }
    };
    if constexpr (!LATE_BN) load_bn();

    floatx4 acc[NT][NCO];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
        for (int mt = 0; mt < NCO; ++mt)  // 2-D: the partial sum `pre` (or 0) starts the accumulator
            acc[nt][mt] = (D2 && !PZ) ? pre_tile(a, b, mg * MT * 16 + mt * 16, g, yo0 + yw * NT + nt, xo0 + n)
                                      : floatx4{0.f, 0.f, 0.f, 0.f};

    const int nchunk = (a.Cin + 3) >> 2;
    stage_load(0);
    if constexpr (WREG) {
#pragma unroll
        for (int i = 0; i < NWA; ++i) wreg_load(i, 0);
    }
    stage_dma(0, 0);
    stage_store(0);
    dma_wait();
    __syncthreads();
    for (int ch = 0; ch < nchunk; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < nchunk) {  // next k-step's loads in flight during the MFMAs
            stage_load(4 * (ch + 1));
            stage_dma(4 * (ch + 1), buf ^ 1);
        }
        const float* xw = xsb(buf) + g * CS + (yw * NT * S) * IX + n * S;
        if constexpr (PZ) {
            const float* wp = &ws[WREG ? 0 : buf][g * 16 + n];
#pragma unroll
            for (int p = 0; p < 4; ++p)
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    float br[NR];
#pragma unroll
                    for (int r = 0; r < NR; ++r) br[r] = xw[(2 * zw + p) * PLANE + r * IX + dx];
#pragma unroll
                    for (int dy = 0; dy < 3; ++dy) {
                        const float av = WREG ? wa[WREG ? p * 9 + dy * 3 + dx : 0] : wp[((p * 9 + dy * 3 + dx) * 4) * 16];
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
                            acc[nt][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, br[nt + dy], acc[nt][0], 0, 0, 0);
                        // (a k-step past the last one reads weights no MFMA uses; the range check bounds it)
                        wreg_load(p * 9 + dy * 3 + dx, 4 * (ch + 1));
                    }
                }
        } else {
            const float* wp = &ws[WREG ? 0 : buf][g * WCS + n];
#pragma unroll
            for (int dz = 0; dz < G::KD; ++dz)
#pragma unroll
                for (int dx = 0; dx < K; ++dx) {
                    float br[NR];
#pragma unroll
                    for (int r = 0; r < NR; ++r) br[r] = xw[(zw * S + dz) * PLANE + r * IX + dx];
#pragma unroll
                    for (int dy = 0; dy < K; ++dy) {
                        const int tap = (dz * K + dy) * K + dx;
                        float av[MT];
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            av[mt] = WREG ? wa[WREG ? tap * MT + mt : 0] : wp[tap * 4 * WCS + mt * 16];
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                            for (int mt = 0; mt < MT; ++mt)
                                acc[nt][mt] =
                                    __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], br[nt * S + dy], acc[nt][mt], 0, 0, 0);
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt) wreg_load(tap * MT + mt, 4 * (ch + 1));
                    }
                }
        }
        if (ch + 1 < nchunk) stage_store(buf ^ 1);
        dma_wait();
        __syncthreads();
    }

    // ---- epilogue: lane (g, n) holds rows 4g + j of each tile, column n
    if constexpr (LATE_BN) load_bn();
    const int x = xo0 + n;
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) +
             (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int y = yo0 + yw * NT + nt;
#pragma unroll
        for (int mt = 0; mt < NCO; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = 4 * g + j;
                const int co = PZ ? (m & 7) : mg * MT * 16 + mt * 16 + m;
                const int z = PZ ? zo0 + 2 * zw + (m >> 3) : zo0 + zw;
                const bool ok = co < a.Cout && z < a.Do && y < a.Ho && x < a.Wo;
                float v = acc[nt][mt][j];
                v = a.scale ? v * scl[mt][j] + shf[mt][j] : v + shf[mt][j];
                v = act_t<ACT>(v, a.act);
                if constexpr (PLAIN) {
                    const unsigned o = ok ? 4u * static_cast<unsigned>(co * static_cast<int>(a.oc) +
                                                                       z * static_cast<int>(a.od) +
                                                                       y * static_cast<int>(a.oh) + x)
                                          : kOOB;
                    store_b32(__float_as_uint(v), ro_, static_cast<int>(o), 0);
                } else {
                    if (!ok) continue;
                    if (a.mul) v = v * a.mul[b * a.mb + co * a.mc + static_cast<long long>(y) * a.mh + x];
                    if (a.res)
                        v = v + a.res[b * a.rb + co * a.rc + static_cast<long long>(z) * a.rd +
                                      static_cast<long long>(y) * a.rh + x];
                    const long long o = b * a.ob + co * a.oc + static_cast<long long>(z) * a.od +
                                        static_cast<long long>(y) * a.oh + x;
                    a.out[o] = v * a.post_scale;
                    if (a.out2) a.out2[o] = v * a.post_scale2;
                }
            }
    }
}

// Cout = 16 MF + 8 (24, 40: the L hourglass's conv1.1 / agg_1.1 / conv2.1 / agg_0.1, 3x3x3 stride 1), round 6.
// The MT form pads such a layer to 16 (MF + 1) MFMA rows, a quarter (24) or a sixth (40) of the matrix work on
// zero weights.  Here a wave owns a PLANE PAIR: the first 16 MF couts run as full tiles for each of the two
// planes, and the last 8 couts of both planes share one 16-row tile through the plane-pair composite weights
// A_p[(h, co)][ci] = W[p - h][ci][co] over the four input planes p (conv_tile3 PZ; 6 of its 8 half-blocks
// carry weights): 90 instead of 108 MFMAs per plane pair, row and k-step at 24 couts, 144 instead of 162 at 40.
// Each input plane's rows are read from LDS once for both.  The composite A operands sit in registers (36 per
// lane, reloaded for the next k-step after their last use, as WREG), the full tiles' weights are staged in LDS.
// Per output the products and their order (dz, dx, dy within a k-step, k-steps in channel order) are the MT
// form's, so the result is bit-identical to it.  Plain BasicConv epilogue only (BN + GELU).
// WZ: waves along z (plane pairs per workgroup; 4 / WZ waves along y): 2 where Do is not a multiple of 8 (the
// 12-plane conv2.1 / agg_0.1 at L-K: 16 planes computed for 12 with 4)
// DMA: the input window staged global -> LDS directly (as T3Geo's DMA)
template <int MF, int NT, int WZ = 4, bool DMA = false>
struct HzGeo {
    static constexpr int WY = 4 / WZ, ZB = 2 * WZ, YB = WY * NT;
    static constexpr int IZ = ZB + 2, IY = YB + 2, IX = 18, PLANE = IY * IX, CS0 = IZ * PLANE;
    static constexpr int NCH = (CS0 + 63) / 64;
    static constexpr int CS = DMA ? NCH * 64 + 16 : CS0 + ((16 - CS0 % 32) % 32 + 32) % 32;  // = 16 mod 32 banks
    static constexpr int XE = 4 * CS0, XL = 4 * CS, XR = (XE + kT3Threads - 1) / kT3Threads;
    static constexpr int WCS = MF % 2 ? 16 * MF : 16 * MF + 16;      // weight row stride = 16 mod 32
    static constexpr int WE = 27 * 4 * 16 * MF, WL = 27 * 4 * WCS, WR = (WE + kT3Threads - 1) / kT3Threads;
    static constexpr int NR = NT + 2;
};

template <int MF, int NT, int WZ, bool DMA>
__global__ void __launch_bounds__(kT3Threads, 2) tconv3hz_kernel(const esm_conv_desc a) {
    using G = HzGeo<MF, NT, WZ, DMA>;
    constexpr int IX = G::IX, PLANE = G::PLANE, CS = G::CS, WCS = G::WCS, WR = G::WR, NR = G::NR;
    constexpr int XR = DMA ? 1 : G::XR, NCH = G::NCH;
    __shared__ __attribute__((aligned(16))) float xs0[G::XL];
    __shared__ __attribute__((aligned(16))) float xs1[G::XL];
    auto xsb = [&](int buf) __attribute__((always_inline)) { return buf ? xs1 : xs0; };
    __shared__ __attribute__((aligned(16))) float ws[2][G::WL];

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int zw = wave % WZ, yw = wave / WZ;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int xo0 = bk_.x * 16, yo0 = bk_.y * G::YB;
    const int nzb = (a.Do + G::ZB - 1) / G::ZB;
    const int b = bk_.z / nzb;
    const int zo0 = (bk_.z - b * nzb) * G::ZB;
    const int zi0 = zo0 - 1, yi0 = yo0 - 1, xi0 = xo0 - 1;

    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (a.Di - 1) * sd + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w), static_cast<short>(0), 4 * 27 * a.cin_pad * a.cout_pad, 0x00020000);

    unsigned xoff[XR];
#pragma unroll
    for (int k = 0; k < (DMA ? 0 : XR); ++k) {
        const int e = tid + k * kT3Threads;
        const int ix = e % IX, iy = (e / IX) % G::IY, iz = (e / PLANE) % G::IZ, ci = e / G::CS0;
        const int zi = zi0 + iz, yi = yi0 + iy, xi = xi0 + ix;
        const bool ok = e < G::XE && zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
        xoff[k] = ok ? 4u * static_cast<unsigned>(ci * sc + zi * sd + yi * sh + xi) : kOOB;
    }
    unsigned woff[WR];
    int wdst[WR];
#pragma unroll
    for (int k = 0; k < WR; ++k) {  // the full tiles' weights: e = (tap * 4 + ci) * 16 MF + m
        const int e = tid + k * kT3Threads;
        const int m = e % (16 * MF), ci = (e / (16 * MF)) & 3, tap = e / (64 * MF);
        woff[k] = e < G::WE ? 4u * static_cast<unsigned>((tap * a.cin_pad + ci) * a.cout_pad + m) : kOOB;
        wdst[k] = e < G::WE ? (tap * 4 + ci) * WCS + m : -1;
    }
    // the last 8 couts' composite A operand of (input plane p, tap t9): lane (g, n) holds W[p - n / 8][t9][c0 + g][16 MF + n % 8]
    unsigned wpo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int dz = p - (n >> 3), co = 16 * MF + (n & 7);
        wpo[p] = (dz >= 0 && dz <= 2 && co < a.Cout) ? 4u * static_cast<unsigned>((dz * 9 * a.cin_pad + g) * a.cout_pad + co)
                                                     : kOOB;
    }
    float wa[36];
    auto wreg_load = [&](int i, int c0) __attribute__((always_inline)) {
        wa[i] = buf_load_s(wrs, wpo[i / 9], 4 * ((i % 9) * a.cin_pad + c0) * a.cout_pad);
    };
    unsigned doff[DMA ? NCH : 1];  // DMA: wave w's chunks i = w + 4 k: channel i / NCH, elements 64 (i % NCH) + lane
    if constexpr (DMA) {
#pragma unroll
        for (int k = 0; k < NCH; ++k) {
            const int i = wave + 4 * k, c = i / NCH, e = (i - c * NCH) * 64 + lane;
            const int ix = e % IX, iy = (e / IX) % G::IY, iz = e / PLANE;
            const int zi = zi0 + iz, yi = yi0 + iy, xi = xi0 + ix;
            const bool ok = e < G::CS0 && zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
            doff[k] = ok ? 4u * static_cast<unsigned>(c * sc + zi * sd + yi * sh + xi) : kOOB;
        }
    }
    auto stage_dma = [&](int c0, int buf) __attribute__((always_inline)) {
        if constexpr (DMA) {
#pragma unroll
            for (int k = 0; k < NCH; ++k) {
                const int i = wave + 4 * k, c = i / NCH;
                __builtin_amdgcn_raw_ptr_buffer_load_lds(
                    rs, (__attribute__((address_space(3))) void*)(xsb(buf) + c * CS + (i - c * NCH) * 64), 4,
                    c0 + c < a.Cin ? doff[k] : kOOB, 4 * c0 * sc, 0, 0);
            }
        }
    };
    auto dma_wait = [&]() __attribute__((always_inline)) {
        if constexpr (DMA) __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the DMA's LDS writes landed
    };
    float xv[XR], wv[WR];
    auto stage_load = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < (DMA ? 0 : XR); ++k) {
            const int ci = (tid + k * kT3Threads) / G::CS0;
            xv[k] = buf_load_s(rs, c0 + ci < a.Cin ? xoff[k] : kOOB, 4 * c0 * sc);
        }
#pragma unroll
        for (int k = 0; k < WR; ++k) wv[k] = buf_load_s(wrs, woff[k], 4 * c0 * a.cout_pad);
    };
    auto stage_store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < (DMA ? 0 : XR); ++k) {
            const int e = tid + k * kT3Threads;
            if (e < G::XE) xsb(buf)[e + (e / G::CS0) * (CS - G::CS0)] = xv[k];
        }
#pragma unroll
        for (int k = 0; k < WR; ++k)
            if (wdst[k] >= 0) ws[buf][wdst[k]] = wv[k];
    };
    floatx4 accf[2][NT][MF], acch[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        acch[nt] = floatx4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int pz = 0; pz < 2; ++pz)
#pragma unroll
            for (int mf = 0; mf < MF; ++mf) accf[pz][nt][mf] = floatx4{0.f, 0.f, 0.f, 0.f};
    }

    const int nchunk = (a.Cin + 3) >> 2;
    stage_load(0);
    stage_dma(0, 0);
#pragma unroll
    for (int i = 0; i < 36; ++i) wreg_load(i, 0);
    stage_store(0);
    dma_wait();
    __syncthreads();
    for (int ch = 0; ch < nchunk; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < nchunk) {  // next k-step's loads in flight during the MFMAs
            stage_load(4 * (ch + 1));
            stage_dma(4 * (ch + 1), buf ^ 1);
        }
        const float* xw = xsb(buf) + g * CS + yw * NT * IX + n;
        const float* wp = &ws[buf][g * WCS + n];
#pragma unroll
        for (int q = 0; q < 4; ++q)
#pragma unroll
            for (int dx = 0; dx < 3; ++dx) {
                float br[NR];
#pragma unroll
                for (int r = 0; r < NR; ++r) br[r] = xw[(2 * zw + q) * PLANE + r * IX + dx];
#pragma unroll
                for (int dy = 0; dy < 3; ++dy) {
#pragma unroll
                    for (int pz = 0; pz < 2; ++pz) {  // full tiles of output plane pz: dz = q - pz
                        const int dz = q - pz;
                        if (dz < 0 || dz > 2) continue;
                        float av[MF];
#pragma unroll
                        for (int mf = 0; mf < MF; ++mf) av[mf] = wp[((dz * 3 + dy) * 3 + dx) * 4 * WCS + mf * 16];
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                            for (int mf = 0; mf < MF; ++mf)
                                accf[pz][nt][mf] =
                                    __builtin_amdgcn_mfma_f32_16x16x4f32(av[mf], br[nt + dy], accf[pz][nt][mf], 0, 0, 0);
                    }
                    const int i = q * 9 + dy * 3 + dx;
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acch[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(wa[i], br[nt + dy], acch[nt], 0, 0, 0);
                    wreg_load(i, 4 * (ch + 1));  // (past the last k-step: weights no MFMA uses, range-checked)
                }
            }
        if (ch + 1 < nchunk) stage_store(buf ^ 1);
        dma_wait();
        __syncthreads();
    }

    // ---- epilogue (BN + GELU, buffer stores): lane (g, n) holds rows 4g + j of each tile, column n; the BN
    //      constants are loaded here (one round trip at the end) rather than held through the K loop
    float scl[MF + 1][4], shf[MF + 1][4];
#pragma unroll
    for (int mf = 0; mf <= MF; ++mf)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = mf < MF ? mf * 16 + 4 * g + j : 16 * MF + ((4 * g + j) & 7);
            scl[mf][j] = a.scale[co];
            shf[mf][j] = a.shift[co];
        }
    const int x = xo0 + n;
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) +
             (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
    auto store = [&](float v, int co, int z, int y) __attribute__((always_inline)) {
        const bool ok = co < a.Cout && z < a.Do && y < a.Ho && x < a.Wo;
        const unsigned o = ok ? 4u * static_cast<unsigned>(co * static_cast<int>(a.oc) + z * static_cast<int>(a.od) +
                                                           y * static_cast<int>(a.oh) + x)
                              : kOOB;
        store_b32(__float_as_uint(v), ro_, static_cast<int>(o), 0);
    };
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int y = yo0 + yw * NT + nt;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
#pragma unroll
            for (int pz = 0; pz < 2; ++pz)
#pragma unroll
                for (int mf = 0; mf < MF; ++mf) {
                    float v = accf[pz][nt][mf][j];  // (the MT form's epilogue expression: the same rounding)
                    v = a.scale ? v * scl[mf][j] + shf[mf][j] : v + shf[mf][j];
                    store(act_t<ESM_ACT_GELU>(v, a.act), mf * 16 + 4 * g + j, zo0 + 2 * zw + pz, y);
                }
            const int m = 4 * g + j;
            float v = acch[nt][j];
            v = a.scale ? v * scl[MF][j] + shf[MF][j] : v + shf[MF][j];
            store(act_t<ESM_ACT_GELU>(v, a.act), 16 * MF + (m & 7), zo0 + 2 * zw + (m >> 3), y);
        }
    }
}

template <int MF, int NT, int WZ = 4>
int launch_hz(const esm_conv_desc& a, hipStream_t s) {
    using G = HzGeo<MF, NT, WZ>;
    // the input window by DMA for the 40-cout layers (conv2.1 / agg_0.1 at L-K B = 4: 101.7 -> 99.7 us in the graph),
    // through registers for 24 couts (conv1.1: 229.4 vs 232.1 us with DMA; scripts/probes/op_hint_probe.py); hint bit
    // 28 flips the choice (A/B)
    const bool dma = ((a.hint >> 28) & 1) ? MF != 2 : (MF == 2 && kT3Dma);
    const long long z = static_cast<long long>(a.B) * ((a.Do + G::ZB - 1) / G::ZB);
    const long long gy = ceil_div(a.Ho, G::YB);
    if (z > 65535 || gy > 65535) return arg_error("conv(tile3 hz): grid too large");
    const dim3 grid(ceil_div(a.Wo, 16), static_cast<unsigned>(gy), static_cast<unsigned>(z));
    if (dma)
        hipLaunchKernelGGL((tconv3hz_kernel<MF, NT, WZ, true>), grid, dim3(kT3Threads), 0, s, a);
    else
        hipLaunchKernelGGL((tconv3hz_kernel<MF, NT, WZ, false>), grid, dim3(kT3Threads), 0, s, a);
    return check_launch("conv(tile3 hz)");
}

// ConvTranspose3d k4 s2 p1 (the hourglass decoder steps conv3_up 72 -> 40 and conv2_up 40 -> 24,
// models/ESMStereo.py:137-138,163-168), same LDS pipeline.  Output 2m + q per dim takes input m + q - t
// with kernel index 1 - q + 2t (t = 0, 1): for one parity class it is a 2x2x2 conv over the input grid,
// and every class of an m-tile reads the same (ZB+2) x (YB+2) x 18 input window, at window offset
// d = 1 + q - t.  A workgroup owns one (qd, qh) class pair of an m-tile; each wave computes both qw
// classes (window columns dx = 0..2 feed qw = 0 through tw = 1 - dx and qw = 1 through tw = 2 - dx), so
// a lane holds the two adjacent output columns 2m, 2m + 1 and stores them as one 8-byte write.
// D2: ConvTranspose2d k4 s2 p1 (the refinement hourglasses' conv3_up / conv2_up): one qh class per
// workgroup, the 4 waves along y (NT rows each), 4 taps per class
// XB > 0 (MT = 1, ncg = 1): the 1x1 BasicConv behind it fused (conv_up1.h; bp: its descriptor, up to XB extra
// 4-channel k-steps): each wave finishes its tiles through the 1x1, the conv's output never leaves registers
template <int MT, int NT, int ACT, bool PLAIN, bool D2, int XB, bool PAIR = false>
__device__ __forceinline__ void tconvt3_body(const esm_conv_desc& a, int ncg, const esm_conv_desc* bp) {
    constexpr int ZB = D2 ? 1 : 4, YB = D2 ? 4 * NT : NT;
    constexpr int NTAP = D2 ? 4 : 8;  // taps per class
    constexpr int IZ = D2 ? 1 : ZB + 2, IY = YB + 2, IX = 18, PLANE = IY * IX, CS0 = IZ * PLANE;
    constexpr int CS = CS0 + ((16 - CS0 % 32) % 32 + 32) % 32;
    constexpr int XE = 4 * CS0, XL = 4 * CS;
    constexpr int WCS = MT % 2 ? MT * 16 : MT * 16 + 16;
    constexpr int WE = 2 * NTAP * 4 * MT * 16, WL = 2 * NTAP * 4 * WCS;  // [qw][tap][ci 4][m]
    constexpr int XR = (XE + kT3Threads - 1) / kT3Threads, WR = (WE + kT3Threads - 1) / kT3Threads;
    __shared__ __attribute__((aligned(16))) float xs[2][XL];
    __shared__ __attribute__((aligned(16))) float ws[2][WL];

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int zw = D2 ? 0 : wave, yw = D2 ? wave : 0;
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int xm0 = bk_.x * 16, ym0 = bk_.y * YB;
    const int nzb = (a.Di + ZB - 1) / ZB;
    int zz = bk_.z;
    const int cp = D2 ? (zz & 1) : (zz & 3);  // (qd, qh) class pair (2-D: qh)
    zz >>= D2 ? 1 : 2;
    const int mg = zz % ncg;
    const int r1 = zz / ncg;
    const int b = r1 / nzb;
    const int zm0 = (r1 - b * nzb) * ZB;
    const int qd = D2 ? 0 : cp >> 1, qh = cp & 1;
    const int zi0 = D2 ? 0 : zm0 - 1, yi0 = ym0 - 1, xi0 = xm0 - 1;

    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (a.Di - 1) * sd + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w), static_cast<short>(0), 4 * NTAP * NTAP * a.cin_pad * a.cout_pad,
        0x00020000);

    unsigned xoff[XR];
#pragma unroll
    for (int k = 0; k < XR; ++k) {
        const int e = tid + k * kT3Threads;
        const int ix = e % IX, iy = (e / IX) % IY, iz = (e / PLANE) % IZ, ci = e / CS0;
        const int zi = zi0 + iz, yi = yi0 + iy, xi = xi0 + ix;
        const bool ok = e < XE && zi >= 0 && zi < a.Di && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
        xoff[k] = ok ? 4u * static_cast<unsigned>(ci * sc + zi * sd + yi * sh + xi) : kOOB;
    }
    // weights: packed w[cls][tap][cin_pad][cout_pad], cls = (qd, qh, qw) bits, tap = (td, th, tw) bits
    unsigned woff[WR];
    int wdst[WR];
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        const int e = tid + k * kT3Threads;  // e = ((qw * 8 + tap) * 4 + ci) * (MT * 16) + m
        const int m = e % (MT * 16), ci = (e / (MT * 16)) & 3, tq = e / (MT * 64);  // tq = qw * NTAP + tap
        const int cls = (cp << 1) | (tq / NTAP), tap = tq % NTAP;
        const int co = mg * MT * 16 + m;
        const bool ok = e < WE && co < a.cout_pad;
        woff[k] = ok ? 4u * static_cast<unsigned>(((cls * NTAP + tap) * a.cin_pad + ci) * a.cout_pad + co) : kOOB;
        wdst[k] = e < WE ? (tq * 4 + ci) * WCS + m : -1;
    }
    float xv[XR], wv[WR];
    auto stage_load = [&](int c0) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < XR; ++k) {
            const int ci = (tid + k * kT3Threads) / CS0;
            xv[k] = buf_load_s(rs, c0 + ci < a.Cin ? xoff[k] : kOOB, 4 * c0 * sc);
        }
#pragma unroll
        for (int k = 0; k < WR; ++k) wv[k] = buf_load_s(wrs, woff[k], 4 * c0 * a.cout_pad);
    };
    auto stage_store = [&](int buf) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < XR; ++k) {
            const int e = tid + k * kT3Threads;
            if (e < XE) xs[buf][e + (e / CS0) * (CS - CS0)] = xv[k];
        }
#pragma unroll
        for (int k = 0; k < WR; ++k)
            if (wdst[k] >= 0) ws[buf][wdst[k]] = wv[k];
    };
    float scl[MT][4], shf[MT][4];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int cc = min(mg * MT * 16 + mt * 16 + 4 * g + j, a.Cout - 1);
            scl[mt][j] = a.scale ? a.scale[cc] : 1.f;
            shf[mt][j] = a.shift ? a.shift[cc] : 0.f;
        }
    // fused 1x1: weights, BN and the extra sources at this lane's output pixels, in flight during the K loop
    Up1Ops<(XB > 0 ? XB : 1)> u1;
    float bx1[2][NT][(XB > 0 ? XB : 1)];
    if constexpr (XB > 0 && MT == 1) {  // (two tiles: loaded in the epilogue, the K loop needs the registers)
        const esm_conv_desc& bb = *bp;
        up1_weights(u1, bb, a.Cout, lane);
        const Up1Src us = up1_src(bb, b, !D2);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int oz = D2 ? 0 : 2 * (zm0 + zw) + qd, oy = 2 * (ym0 + yw * NT + nt) + qh, ox = 2 * (xm0 + n);
            if constexpr (PAIR) {
                up1_extra2(bx1[0][nt], bx1[1][nt], us, bb, a.Cout, lane, oz, oy, ox);
            } else {
#pragma unroll
                for (int qw = 0; qw < 2; ++qw) up1_extra(bx1[qw][nt], us, bb, a.Cout, lane, oz, oy, ox + qw);
            }
        }
    }
    floatx4 acc[2][NT][MT];
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) acc[q][nt][mt] = floatx4{0.f, 0.f, 0.f, 0.f};

    const int nchunk = (a.Cin + 3) >> 2;
    stage_load(0);
    stage_store(0);
    __syncthreads();
    for (int ch = 0; ch < nchunk; ++ch) {
        const int buf = ch & 1;
        if (ch + 1 < nchunk) stage_load(4 * (ch + 1));
        const float* xw = &xs[buf][g * CS + n];
        const float* wp = &ws[buf][g * WCS + n];
#pragma unroll
        for (int td = 0; td < (D2 ? 1 : 2); ++td) {
            const int dz = D2 ? 0 : 1 + qd - td;  // window plane offset (wave-uniform)
#pragma unroll
            for (int th = 0; th < 2; ++th) {
                const int dy = 1 + qh - th;
                const float* xr = xw + (zw + dz) * PLANE + (yw * NT + dy) * IX;
#pragma unroll
                for (int dx = 0; dx < 3; ++dx) {
                    float br[NT];
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) br[nt] = xr[nt * IX + dx];
#pragma unroll
                    for (int qw = 0; qw < 2; ++qw) {
                        const int tw = 1 + qw - dx;
                        if (tw < 0 || tw > 1) continue;
                        const int tq = qw * NTAP + (D2 ? th * 2 + tw : td * 4 + th * 2 + tw);
                        float av[MT];
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt) av[mt] = wp[tq * 4 * WCS + mt * 16];
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                            for (int mt = 0; mt < MT; ++mt)
                                acc[qw][nt][mt] =
                                    __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], br[nt], acc[qw][nt][mt], 0, 0, 0);
                    }
                }
            }
        }
        if (ch + 1 < nchunk) stage_store(buf ^ 1);
        __syncthreads();
    }

    // ---- epilogue: lane (g, n) holds output columns 2m, 2m + 1 (m = xm0 + n) of rows 4g + j
    const int x = 2 * (xm0 + n);
    const int z = D2 ? 0 : 2 * (zm0 + zw) + qd;
    static_assert(XB == 0 || MT <= 2, "fused 1x1: one or two cout tiles");
    if constexpr (XB > 0 && MT == 2) {
        // two tiles (round 6, conv_up1.h Up1Ops2): the 1x1's operands and the extra sources, loaded here
        const esm_conv_desc& bb = *bp;
        Up1Ops2<XB> u2;
        up1_weights2(u2, bb, a.Cout, lane);
        const Up1Src us = up1_src(bb, b, !D2);
        const __amdgpu_buffer_rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(
            bb.out + b * bb.ob, static_cast<short>(0),
            4 * ((bb.Cout - 1) * static_cast<int>(bb.oc) + (D2 ? 0 : (bb.Do - 1) * static_cast<int>(bb.od)) +
                 (bb.Ho - 1) * static_cast<int>(bb.oh) + bb.Wo),
            0x00020000);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int y = 2 * (ym0 + yw * NT + nt) + qh;
            const int orow = 4 * ((D2 ? 0 : z * static_cast<int>(bb.od)) + y * static_cast<int>(bb.oh));
            const bool rok = y < bb.Ho && z < bb.Do;
            float bx[2][XB];
            if constexpr (PAIR) {
                up1_extra2(bx[0], bx[1], us, bb, a.Cout, lane, z, y, x);
            } else {
#pragma unroll
                for (int qw = 0; qw < 2; ++qw) up1_extra(bx[qw], us, bb, a.Cout, lane, z, y, x + qw);
            }
            floatx4 o[2][2];  // [qw][mb]
#pragma unroll
            for (int qw = 0; qw < 2; ++qw) {
                float yv[2][4];
#pragma unroll
                for (int mt = 0; mt < 2; ++mt)
#pragma unroll
                    for (int j = 0; j < 4; ++j) yv[mt][j] = gelu_erf(acc[qw][nt][mt][j] * scl[mt][j] + shf[mt][j]);
                up1_finish2(o[qw], u2, yv, bx[qw]);
            }
#pragma unroll
            for (int mb = 0; mb < 2; ++mb)
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = 16 * mb + 4 * g + j;
                    if constexpr (PAIR) {
                        typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                        const unsigned vo = (rok && x < bb.Wo && co < bb.Cout)
                                                ? 4u * static_cast<unsigned>(co * static_cast<int>(bb.oc) + x) : kOOB;
                        __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(o[0][mb][j]), __float_as_uint(o[1][mb][j])},
                                                              rb_, static_cast<int>(vo), rok ? orow : 0, kStoreAux);
                    } else {
#pragma unroll
                        for (int qw = 0; qw < 2; ++qw) {
                            const unsigned vo = (rok && x + qw < bb.Wo && co < bb.Cout)
                                                    ? 4u * static_cast<unsigned>(co * static_cast<int>(bb.oc) + x + qw) : kOOB;
                            store_b32(__float_as_uint(o[qw][mb][j]), rb_, static_cast<int>(vo), rok ? orow : 0);
                        }
                    }
                }
        }
        return;
    }
    if constexpr (XB > 0 && MT == 1) {
        const esm_conv_desc& bb = *bp;
        const __amdgpu_buffer_rsrc_t rb_ = __builtin_amdgcn_make_buffer_rsrc(
            bb.out + b * bb.ob, static_cast<short>(0),
            4 * ((bb.Cout - 1) * static_cast<int>(bb.oc) + (D2 ? 0 : (bb.Do - 1) * static_cast<int>(bb.od)) +
                 (bb.Ho - 1) * static_cast<int>(bb.oh) + bb.Wo),
            0x00020000);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int y = 2 * (ym0 + yw * NT + nt) + qh;
            const int orow = 4 * ((D2 ? 0 : z * static_cast<int>(bb.od)) + y * static_cast<int>(bb.oh));
            const bool rok = y < bb.Ho && z < bb.Do;
            floatx4 o[2];
#pragma unroll
            for (int qw = 0; qw < 2; ++qw) {
                float yv[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) yv[j] = gelu_erf(acc[qw][nt][0][j] * scl[0][j] + shf[0][j]);
                o[qw] = up1_finish(u1, yv, bx1[qw][nt], D2 ? pre_tile(bb, b, 0, g, y, x + qw) : floatx4{0.f, 0.f, 0.f, 0.f});
            }
            if constexpr (PAIR) {  // 8-byte pair stores (b's output rows 8-byte aligned, even width: launcher)
                typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                const bool pok = rok && x < bb.Wo;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    const int co = 4 * g + j;
                    const unsigned vo =
                        (pok && co < bb.Cout) ? 4u * static_cast<unsigned>(co * static_cast<int>(bb.oc) + x) : kOOB;
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(o[0][j]), __float_as_uint(o[1][j])}, rb_,
                                                          static_cast<int>(vo), rok ? orow : 0, kStoreAux);
                }
            } else {
#pragma unroll
                for (int qw = 0; qw < 2; ++qw) {
                    const bool pok = rok && x + qw < bb.Wo;
#pragma unroll
                    for (int j = 0; j < 4; ++j) {
                        const int co = 4 * g + j;
                        const unsigned vo = (pok && co < bb.Cout)
                                                ? 4u * static_cast<unsigned>(co * static_cast<int>(bb.oc) + x + qw)
                                                : kOOB;
                        store_b32(__float_as_uint(o[qw][j]), rb_, static_cast<int>(vo), rok ? orow : 0);
                    }
                }
            }
        }
        return;
    }
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) +
             (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int y = 2 * (ym0 + yw * NT + nt) + qh;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int co = mg * MT * 16 + mt * 16 + 4 * g + j;
                const bool ok = co < a.Cout && z < a.Do && y < a.Ho && x < a.Wo;
                float v[2];
#pragma unroll
                for (int qw = 0; qw < 2; ++qw) {
                    float t = acc[qw][nt][mt][j];
                    t = a.scale ? t * scl[mt][j] + shf[mt][j] : t + shf[mt][j];
                    v[qw] = act_t<ACT>(t, a.act);
                }
                if constexpr (PLAIN) {
                    const unsigned o = ok ? 4u * static_cast<unsigned>(co * static_cast<int>(a.oc) +
                                                                       z * static_cast<int>(a.od) +
                                                                       y * static_cast<int>(a.oh) + x)
                                          : kOOB;
                    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
                    __builtin_amdgcn_raw_buffer_store_b64(u32x2{__float_as_uint(v[0]), __float_as_uint(v[1])}, ro_,
                                                          static_cast<int>(o), 0, kStoreAux);
                } else {
                    if (!ok) continue;
#pragma unroll
                    for (int qw = 0; qw < 2; ++qw) {
                        float t = v[qw];
                        if (a.res)
                            t = t + a.res[b * a.rb + co * a.rc + static_cast<long long>(z) * a.rd +
                                          static_cast<long long>(y) * a.rh + x + qw];
                        const long long o = b * a.ob + co * a.oc + static_cast<long long>(z) * a.od +
                                            static_cast<long long>(y) * a.oh + x + qw;
                        a.out[o] = t * a.post_scale;
                        if (a.out2) a.out2[o] = t * a.post_scale2;
                    }
                }
            }
    }
}

template <int MT, int NT, int ACT, bool PLAIN, bool D2 = false>
__global__ void __launch_bounds__(kT3Threads) tconvt3_kernel(const esm_conv_desc a, int ncg) {
    tconvt3_body<MT, NT, ACT, PLAIN, D2, 0>(a, ncg, nullptr);
}

// ConvTranspose + crop + cat + 1x1 (conv_up1.h); PAIR: 8-byte extra-source loads and output stores; MT: cout tiles of
// both convs (2: 17-32 couts, round 6)
template <int MT, int NT, bool D2, int XB, bool PAIR>
__global__ void __launch_bounds__(kT3Threads) tconvt3_up1_kernel(const esm_conv_desc a, const esm_conv_desc b) {
    tconvt3_body<MT, NT, ESM_ACT_GELU, true, D2, XB, PAIR>(a, 1, &b);
}

template <int NT, bool D2, int MT = 1>
int launch_tt3_up1(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    const long long z = D2 ? static_cast<long long>(a.B) * 2 : static_cast<long long>(a.B) * ((a.Di + 3) / 4) * 4;
    const long long gy = ceil_div(a.Hi, D2 ? 4 * NT : NT);
    if (z > 65535 || gy > 65535) return arg_error("convt_1x1(tile): grid too large");
    const dim3 grid(ceil_div(a.Wi, 16), static_cast<unsigned>(gy), static_cast<unsigned>(z));
    const int xb = (b.Cin - a.Cout) >> 2;
    // pairs: b's output rows / channels / batch items 8-byte aligned and every extra source likewise
    const bool pair = up1_pairs_ok(b) && !(b.Wo & 1) && !(reinterpret_cast<uintptr_t>(b.out) & 7) && !(b.ob & 1) &&
                      !(b.oc & 1) && !(b.oh & 1) && !(b.od & 1);
#define ESM_UP1(X)                                                                                   \
    do {                                                                                             \
        if (pair)                                                                                    \
            hipLaunchKernelGGL((tconvt3_up1_kernel<MT, NT, D2, X, true>), grid, dim3(kT3Threads), 0, s, a, b); \
        else                                                                                         \
            hipLaunchKernelGGL((tconvt3_up1_kernel<MT, NT, D2, X, false>), grid, dim3(kT3Threads), 0, s, a, b); \
    } while (0)
    if constexpr (MT == 2) {  // (<= 32 extra channels: conv_up1.hip)
        if (xb <= 4) ESM_UP1(4);
        else if (xb <= 6) ESM_UP1(6);
        else ESM_UP1(8);
    } else {
        if (xb <= 4) ESM_UP1(4);
        else if (xb <= 8) ESM_UP1(8);
        else if (xb <= 10) ESM_UP1(10);
        else ESM_UP1(12);
    }
#undef ESM_UP1
    return check_launch("conv(tile3 transposed + 1x1)");
}

template <int MT, int NT, bool D2 = false>
int launch_tt3(const esm_conv_desc& a, hipStream_t s, int ncg) {
    const long long z = D2 ? static_cast<long long>(a.B) * ncg * 2 : static_cast<long long>(a.B) * ((a.Di + 3) / 4) * ncg * 4;
    const long long gy = ceil_div(a.Hi, D2 ? 4 * NT : NT);
    if (z > 65535 || gy > 65535) return arg_error("conv(tile3 transposed): grid too large");
    const dim3 grid(ceil_div(a.Wi, 16), static_cast<unsigned>(gy), static_cast<unsigned>(z));
    // the plain form stores 8-byte pairs: 8-byte aligned rows
    const bool plain = a.act == ESM_ACT_GELU && !a.res && !a.out2 && !a.mul && a.post_scale == 1.f &&
                       (a.oh % 2) == 0 && (a.od % 2) == 0 && (a.oc % 2) == 0 &&
                       (reinterpret_cast<uintptr_t>(a.out) & 7) == 0 &&
                       static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Do) * a.od +
                               static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (plain)
        hipLaunchKernelGGL((tconvt3_kernel<MT, NT, ESM_ACT_GELU, true, D2>), grid, dim3(kT3Threads), 0, s, a, ncg);
    else
        hipLaunchKernelGGL((tconvt3_kernel<MT, NT, -1, false, D2>), grid, dim3(kT3Threads), 0, s, a, ncg);
    return check_launch("conv(tile3 transposed)");
}

template <int NT, bool D2 = false>
int launch_tt3_mt(const esm_conv_desc& a, hipStream_t s) {
    const int tiles = (a.Cout + 15) / 16;
    if (tiles == 1) return launch_tt3<1, NT, D2>(a, s, 1);
    if (tiles == 2) return launch_tt3<2, NT, D2>(a, s, 1);
    if (tiles == 3) return launch_tt3<3, NT, D2>(a, s, 1);
    if (tiles <= 4) return launch_tt3<2, NT, D2>(a, s, 2);
    if (tiles <= 6) return launch_tt3<3, NT, D2>(a, s, 2);
    return arg_error("conv(tile3 transposed): at most 96 output channels");
}

template <int S, int K, int MT, int NT, int WZ, bool PZ, int NS = 1, bool D2 = false, bool WREG = false, bool DMA = false>
int launch_t3(const esm_conv_desc& a, hipStream_t s, int ncg) {
    using G = T3Geo<S, K, NT, WZ, PZ, MT, D2, DMA>;
    const long long z = static_cast<long long>(a.B) * ((a.Do + G::ZB - 1) / G::ZB) * ncg;
    const long long gy = ceil_div(a.Ho, G::YB);
    if (z > 65535 || gy > 65535) return arg_error("conv(tile3): grid too large");
    const dim3 grid(ceil_div(a.Wo, 16), static_cast<unsigned>(gy), static_cast<unsigned>(z));
    const bool plain = a.act == ESM_ACT_GELU && !a.res && !a.out2 && !a.mul && a.post_scale == 1.f &&
                       static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Do) * a.od +
                               static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (plain)
        hipLaunchKernelGGL((tconv3_kernel<S, K, MT, NT, WZ, PZ, ESM_ACT_GELU, true, NS, D2, WREG, DMA>), grid, dim3(kT3Threads),
                           0, s, a, ncg);
    else
        hipLaunchKernelGGL((tconv3_kernel<S, K, MT, NT, WZ, PZ, -1, false, NS, D2, WREG, DMA>), grid, dim3(kT3Threads), 0, s,
                           a, ncg);
    return check_launch("conv(tile3)");
}

// cout tiles per workgroup (MT) and cout groups (ncg) for Cout: MT * 16 * ncg >= Cout
template <int S, int K, int NT, int WZ, int NS = 1, bool D2 = false>
int launch_t3_mt(const esm_conv_desc& a, hipStream_t s) {
    const int tiles = (a.Cout + 15) / 16;
    if (tiles <= 3) {
        if (tiles == 1) return launch_t3<S, K, 1, NT, WZ, false, NS, D2>(a, s, 1);
        if (tiles == 2) return launch_t3<S, K, 2, NT, WZ, false, NS, D2>(a, s, 1);
        return launch_t3<S, K, 3, NT, WZ, false, NS, D2>(a, s, 1);
    }
    // 4+ tiles (72 couts: 5): two cout groups of ceil(tiles / 2) tiles
    if (tiles <= 4) return launch_t3<S, K, 2, NT, WZ, false, NS, D2>(a, s, 2);
    if (tiles <= 6) return launch_t3<S, K, 3, NT, WZ, false, NS, D2>(a, s, 2);
    return arg_error("conv(tile3): at most 96 output channels");
}

// stride 2, register weights: one cout group of 1..3 tiles
template <int NT, int WZ, bool DMA = false>
int launch_t3_mtw(const esm_conv_desc& a, hipStream_t s) {
    const int tiles = (a.Cout + 15) / 16;
    if (tiles == 1) return launch_t3<2, 3, 1, NT, WZ, false, 1, false, true, DMA>(a, s, 1);
    return launch_t3<2, 3, 2, NT, WZ, false, 1, false, true, DMA>(a, s, 1);
}

// 1x1x1 over 1..3 sources
template <int NT>
int launch_t3_k1(const esm_conv_desc& a, hipStream_t s) {
    if (a.nsrc == 1) return launch_t3_mt<1, 1, NT, 4, 1>(a, s);
    if (a.nsrc == 2) return launch_t3_mt<1, 1, NT, 4, 2>(a, s);
    return launch_t3_mt<1, 1, NT, 4, 3>(a, s);
}

// 2-D: 4 waves along y (NT rows each), 1..3 sources
template <int S, int K, int NT>
int launch_t2_ns(const esm_conv_desc& a, hipStream_t s) {
    if (a.nsrc == 1) return launch_t3_mt<S, K, NT, 1, 1, true>(a, s);
    if (a.nsrc == 2) return launch_t3_mt<S, K, NT, 1, 2, true>(a, s);
    return launch_t3_mt<S, K, NT, 1, 3, true>(a, s);
}

template <int S, int K>
int launch_t2_nt(const esm_conv_desc& a, hipStream_t s) {
    const int rsel = (a.hint >> 26) & 3;
    if (rsel == 1) return launch_t2_ns<S, K, 1>(a, s);
    if (rsel == 3) return launch_t2_ns<S, K, 4>(a, s);
    if (rsel == 2) return launch_t2_ns<S, K, 2>(a, s);
    const long long px = static_cast<long long>(a.B) * a.Ho * a.Wo;
    return px >= (1LL << 18) ? launch_t2_ns<S, K, 4>(a, s) : launch_t2_ns<S, K, 2>(a, s);
}

}  // namespace

// 2-D (the upsamplers' large maps at ESMStereo-L / -M): k3 stride 1 / 2 or k1 stride 1, any padding, 1..3
// sources, <= 96 couts
bool tile2_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (!d3 && a.transposed)  // ConvTranspose2d k4 s2 p1, one source, >= 2 couts (one output: convt_c1)
        return a.kh == 4 && a.stride == 2 && a.nsrc == 1 && !a.up && !a.mul && a.shuffle <= 1 && a.Cout > 1 &&
               a.Cout <= 96 && a.cout_pad >= 16 * ((a.Cout + 15) / 16) && direct_ok(a);
    if (d3 || a.transposed || a.up || a.shuffle > 1 || a.Cout > 96) return false;
    if (!((a.kh == 3 && (a.stride == 1 || a.stride == 2)) || (a.kh == 1 && a.stride == 1))) return false;
    if (a.cout_pad < 16 * ((a.Cout + 15) / 16)) return false;
    return direct_ok(a);
}

bool tile2_auto(const esm_conv_desc& a) {
    if (!tile2_ok(a) || a.Cin < 4) return false;  // one input channel: the VALU form (conv_stem.hip c1in)
    const long long units = static_cast<long long>(a.B) * a.Ho * a.Wo * ((a.Cout + 15) / 16);
    return units >= (1LL << 19);
}

int launch_tile2(const esm_conv_desc& a, hipStream_t s) {
    if (!tile2_ok(a)) return arg_error("conv: tile2-form hint not applicable");
    if (a.transposed) {
        const int rsel = (a.hint >> 26) & 3;
        if (rsel == 1) return launch_tt3_mt<1, true>(a, s);
        if (rsel == 3) return launch_tt3_mt<4, true>(a, s);
        return launch_tt3_mt<2, true>(a, s);
    }
    if (a.kh == 1) return launch_t2_nt<1, 1>(a, s);
    if (a.stride == 2) return launch_t2_nt<2, 3>(a, s);
    return launch_t2_nt<1, 3>(a, s);
}

bool tile2_ok(const esm_conv_desc& a);
bool tile3_ok(const esm_conv_desc& a);

// ConvTranspose k4 s2 (<= 16 couts) + crop + cat + 1x1 (<= 16 couts, <= 48 extra channels) in the LDS-tiled
// form (conv_up1.h); a and b validated by the caller (launch_convt_1x1).  Rows per wave from a's hint bits
// 26-27 (1 / 2; default 2)
int launch_tile_up1(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    const bool d3 = a.kd == 4;
    if (!(d3 ? tile3_ok(a) : tile2_ok(a))) return arg_error("convt_1x1: the tiled form cannot run this transposed conv");
    const int rsel = (a.hint >> 26) & 3;
    if (a.Cout > 16 || b.Cout > 16) {  // two cout tiles (3-D only: conv_up1.hip)
        if (!d3) return arg_error("convt_1x1: two cout tiles for the 3-D form only");
        return rsel == 1 ? launch_tt3_up1<1, false, 2>(a, b, s) : launch_tt3_up1<2, false, 2>(a, b, s);
    }
    if (d3) return rsel == 1 ? launch_tt3_up1<1, false>(a, b, s) : launch_tt3_up1<2, false>(a, b, s);
    return rsel == 1 ? launch_tt3_up1<1, true>(a, b, s) : launch_tt3_up1<2, true>(a, b, s);
}

// 3-D, one source, 3x3x3 stride 1 / 2 padding 1 or 1x1x1 stride 1 padding 0, <= 96 couts, spans within
// 32-bit buffer offsets.
bool tile3_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (a.transposed)  // ConvTranspose3d k4 s2 p1, one source, >= 2 couts (one output: convt_c1)
        return d3 && a.kd == 4 && a.kh == 4 && a.stride == 2 && a.nsrc == 1 && !a.up && !a.mul && a.Cout > 1 &&
               a.Cout <= 96 && a.cout_pad >= 16 * ((a.Cout + 15) / 16) && direct_ok(a);
    if (!d3 || a.up || a.shuffle > 1 || a.Cout > 96) return false;
    const bool k3 = a.kd == 3 && a.kh == 3 && a.kw == 3 && a.pd == 1 && a.ph == 1 && a.pw == 1 &&
                    (a.stride == 1 || a.stride == 2);
    const bool k1 = a.kd == 1 && a.kh == 1 && a.kw == 1 && a.pd == 0 && a.ph == 0 && a.pw == 0 && a.stride == 1;
    if (!k3 && !k1) return false;
    if (a.nsrc != 1 && !k1) return false;  // channel concats: 1x1x1 only (the hourglass's agg_0.0 / agg_1.0)
    if (a.cout_pad < 16 * ((a.Cout + 15) / 16)) return false;
    return direct_ok(a);
}

// Automatic choice: the MFMA-bound volumes (>= 2^16 output voxels per launch), where the register-operand
// forms sit at 0.15-0.41 of the fp32 MFMA peak (profiles/r03_ops_LK4.txt; r04 probe at L-K B = 4:
// conv2.0 232 -> 86 us, conv2.1 298 -> 100 us at 89,856 voxels).  The latency-bound small volumes of S / M
// keep their forms.
bool tile3_auto(const esm_conv_desc& a) {
    if (!tile3_ok(a)) return false;
    const long long vox = static_cast<long long>(a.B) * a.Do * a.Ho * a.Wo;
    return vox >= (1LL << 16);
}

// hint bits 26-27 with TILE3 (bit 23): rows per wave 1 / 2 / 4 (0 = automatic)
int launch_tile3(const esm_conv_desc& a, hipStream_t s) {
    if (!tile3_ok(a)) return arg_error("conv: tile3-form hint not applicable");
    const int rsel = (a.hint >> 26) & 3;
    const long long vox = static_cast<long long>(a.B) * a.Do * a.Ho * a.Wo;
    if (a.transposed) {
        if (rsel == 1) return launch_tt3_mt<1>(a, s);
        if (rsel == 3) return launch_tt3_mt<4>(a, s);
        return launch_tt3_mt<2>(a, s);
    }
    if (a.kh == 1) {
        if (rsel == 1) return launch_t3_k1<1>(a, s);
        if (rsel == 2 || (rsel == 0 && vox < (1LL << 19))) return launch_t3_k1<2>(a, s);
        return launch_t3_k1<4>(a, s);
    }
    if (a.stride == 2) {  // one row per wave unless asked (r04 probe, L-K B = 4: conv1.0 274 -> 226 us, conv2.0 92 -> 86)
        // round 6: the weights as register operands (<= 3 cout tiles per workgroup, one source); hint bit 29: LDS
        if (!((a.hint >> 29) & 1) && a.nsrc == 1 && a.Cout <= 32) {  // (3 tiles: 150 VGPRs, conv2.0 84 -> 88 us)
            // the input window staged global -> LDS directly (bit 28: through registers, A/B)
            // (4 rows: the DMA window's channel padding would exceed 64 KB of LDS; measured at L-K B = 4 in the
            // graph, scripts/probes/op_hint_probe.py: conv1.0 168.6 us with it at 2 rows, 161.2 without)
            const bool dma = !((a.hint >> 28) & 1) && kT3Dma;
            if (rsel == 2) return dma ? launch_t3_mtw<2, 2, true>(a, s) : launch_t3_mtw<2, 2>(a, s);
            if (rsel == 3) return launch_t3_mtw<4, 2>(a, s);
            return dma ? launch_t3_mtw<1, 2, true>(a, s) : launch_t3_mtw<1, 2>(a, s);
        }
        if (rsel == 2) return launch_t3_mt<2, 3, 2, 2>(a, s);
        if (rsel == 3) return launch_t3_mt<2, 3, 4, 2>(a, s);
        return launch_t3_mt<2, 3, 1, 2>(a, s);
    }
    if (a.Cout <= 8) {  // plane pairs; hint bit 29: weights staged in LDS (round 5), else in registers (round 6)
        const bool lw = (a.hint >> 29) & 1;
        // register weights: the input window staged global -> LDS directly (round 6), bit 28: through registers
        const bool dma = !((a.hint >> 28) & 1) && kT3Dma;
        if (rsel == 1)
            return lw ? launch_t3<1, 3, 1, 1, 4, true>(a, s, 1)
                      : (dma ? launch_t3<1, 3, 1, 1, 4, true, 1, false, true, true>(a, s, 1)
                             : launch_t3<1, 3, 1, 1, 4, true, 1, false, true>(a, s, 1));
        if (rsel == 2 || (rsel == 0 && vox < (1LL << 20)))
            return lw ? launch_t3<1, 3, 1, 2, 4, true>(a, s, 1)
                      : (dma ? launch_t3<1, 3, 1, 2, 4, true, 1, false, true, true>(a, s, 1)
                             : launch_t3<1, 3, 1, 2, 4, true, 1, false, true>(a, s, 1));
        return lw ? launch_t3<1, 3, 1, 4, 4, true>(a, s, 1)
                  : (dma ? launch_t3<1, 3, 1, 4, 4, true, 1, false, true, true>(a, s, 1)
                         : launch_t3<1, 3, 1, 4, 4, true, 1, false, true>(a, s, 1));
    }
    // 24 / 40 couts, plain BasicConv: the plane-pair hybrid (hint bit 29: the padded MT form, A/B); rows per wave
    // 2 / 4 for rsel 1 / 2-3, automatic 4 (2 on small volumes)
    const bool plain = a.act == ESM_ACT_GELU && a.scale && a.shift && !a.res && !a.out2 && !a.mul && a.post_scale == 1.f &&
                       a.nsrc == 1 && static_cast<long long>(a.Cout) * a.oc + static_cast<long long>(a.Do) * a.od +
                                              static_cast<long long>(a.Ho) * a.oh < (kOOB >> 2);
    if (plain && !((a.hint >> 29) & 1) && (a.Cout == 24 || a.Cout == 40)) {
        const int nt = rsel == 1 ? 2 : rsel >= 2 ? 4 : (vox < (1LL << 19) ? 2 : 4);
        const bool z2 = (a.Do % 8) != 0 && (a.Do % 4) == 0;  // 2 plane pairs x 2 row groups: no idle planes
        if (a.Cout == 24) {
            if (z2) return nt == 2 ? launch_hz<1, 2, 2>(a, s) : launch_hz<1, 4, 2>(a, s);
            return nt == 2 ? launch_hz<1, 2>(a, s) : launch_hz<1, 4>(a, s);  // (8 rows spill)
        }
        return z2 ? launch_hz<2, 2, 2>(a, s) : launch_hz<2, 2>(a, s);  // 40 couts: 2 rows (4, 8 exceed the registers)
    }
    // depth not a multiple of 4 (conv3.1 at L-K: 6 planes): 2 planes x 2 row groups per workgroup, no idle planes
    const bool z2 = (a.Do % 4) != 0 && (a.Do % 2) == 0;
    if (rsel == 1) return z2 ? launch_t3_mt<1, 3, 1, 2>(a, s) : launch_t3_mt<1, 3, 1, 4>(a, s);
    if (rsel == 2 || (rsel == 0 && vox < (1LL << 19)))
        return z2 ? launch_t3_mt<1, 3, 2, 2>(a, s) : launch_t3_mt<1, 3, 2, 4>(a, s);
    if (z2 && rsel == 3 && !(a.hint & (1 << 28))) return launch_t3_mt<1, 3, 4, 2>(a, s);
    // 8 rows per wave on the largest volumes (L-K B = 4 aggregation_out.conv1.1, 24 -> 24 on 24x48x156: 277 vs 301
    // us for 4 rows, r04 probe); hint bit 28 with rows 4 asks for it explicitly
    if ((rsel == 3 && (a.hint & (1 << 28))) || rsel == 0) return launch_t3_mt<1, 3, 8, 4>(a, s);
    return launch_t3_mt<1, 3, 4, 4>(a, s);
}

}  // namespace conv
}  // namespace esm
