// The group-wise correlation volume and its first 3-D conv in one launch (ESMStereo-L / -M):
//
//   V[b,g,d,y,x] = mean_{c in g} L[c,y,x] * R[c,y,x-d]  (0 for x < d)   models/submodule.py:143-161
//   group_stem(V) = GELU(BN(conv3d 3x3x3 G -> 8, pad 1))               models/ESMStereo.py:610-611, 703-704
//
// The unfused path writes V (L-K: 184 MB per pair) and the stem reads it back through its LDS-tiled
// form (conv_tile3.hip, plane pairs).  Here the stem's staging step builds each k-step's volume window
// (4 groups x 10 disparity planes x (NT + 2) rows x 18 columns) from the feature windows instead: the
// workgroup loads the 4 * CPG left-feature channels of the window (18 columns) and the right-feature
// channels over the 27 columns the 10 shifts reach into LDS, and every thread forms its volume elements
// from there, products and the pairwise sum rounded one operation at a time exactly as the gwc kernel
// (volumes.hip) does, so the staged window, and with it every MFMA operand, equals the unfused path's.
// The MFMA schedule is the plane-pair schedule of tconv3_kernel<.., PZ> (the 16 rows of the 16x16x4
// tile carry 8 couts x 2 output planes, composite weights per input plane) with the same accumulation
// order and epilogue: the output is bit-identical to gwc_volume + group_stem.
//
// Pipeline (one barrier per k-step): iteration ch issues the global loads of k-step ch + 2's feature
// windows and ch + 1's weights, runs ch's MFMAs from LDS, then builds ch + 1's volume window from the
// feature windows staged one iteration earlier and stores the loads it issued.
#include "conv_direct.h"

namespace esm {
namespace conv {
namespace {

constexpr int kGsThreads = 256;

template <int NT, int CPG>
struct GsGeo {
    static constexpr int ZB = 8, YB = NT;                 // output planes / rows per workgroup (4 waves along z)
    static constexpr int IZ = ZB + 2, IY = YB + 2, IX = 18;  // volume window
    static constexpr int PLANE = IY * IX, CS0 = IZ * PLANE;
    static constexpr int CS = CS0 + ((16 - CS0 % 32) % 32 + 32) % 32;  // channel stride = 16 mod 32 banks
    static constexpr int XE = 4 * CS0, XL = 4 * CS, XR = (XE + kGsThreads - 1) / kGsThreads;
    static constexpr int WE = 4 * 9 * 4 * 16, WR = (WE + kGsThreads - 1) / kGsThreads;  // composite weights
    static constexpr int FC = 4 * CPG;                    // feature channels per k-step
    static constexpr int RX = IX + IZ - 1;                // right-feature columns the IZ shifts reach
    static constexpr int LW = IY * IX, RW = IY * RX;      // per-channel window sizes
    static constexpr int LE = FC * LW, RE = FC * RW, FE = LE + RE;
    static constexpr int LR = (LE + kGsThreads - 1) / kGsThreads, RR = (RE + kGsThreads - 1) / kGsThreads;
    static_assert(FE < (1 << 15), "packed LDS indices are 15 bits");
};

// WREG (round 6): every lane loads its composite-weight A operands of a k-step straight into registers
// (36 per lane, one k-step ahead, from L1 / L2: the 27 x 32 x 8 stem weights), so the weights take no LDS and
// three workgroups fit on a CU (52.6 KB instead of 71 KB at NT = 4); else they are staged in LDS per k-step
template <int NT, int CPG, int ACT, bool PLAIN, bool WREG>
__global__ void __launch_bounds__(kGsThreads, WREG ? 3 : 2) gwc_stem_kernel(const esm_conv_desc a, const float* __restrict__ Lf,
                                                                            const float* __restrict__ Rf, int C) {
    using G = GsGeo<NT, CPG>;
    constexpr int IY = G::IY, IX = G::IX, PLANE = G::PLANE, CS = G::CS, CS0 = G::CS0;
    constexpr int WR = G::WR, LR = G::LR, RR = G::RR, NR = NT + 2;
    __shared__ __attribute__((aligned(16))) float xs[2][G::XL];
    __shared__ __attribute__((aligned(16))) float ws[WREG ? 1 : 2][WREG ? 1 : G::WE];
    __shared__ float fs[2][G::FE];  // [left: FC][IY][IX] then [right: FC][IY][RX]

    const int tid = threadIdx.x;
    const int lane = tid & 63, g = lane >> 4, n = lane & 15;
    const int zw = __builtin_amdgcn_readfirstlane(tid >> 6);
    const Blk3 bk_ = xcd_block((a.hint & kHintXcd) != 0);
    const int xo0 = bk_.x * 16, yo0 = bk_.y * G::YB;
    const int nzb = (a.Do + G::ZB - 1) / G::ZB;
    const int b = bk_.z / nzb;
    const int zo0 = (bk_.z - b * nzb) * G::ZB;
    const int zi0 = zo0 - 1, yi0 = yo0 - 1, xi0 = xo0 - 1;
    const int D = a.Di, H = a.Hi, W = a.Wi;

    // feature windows: [b] of a contiguous [B, C, H, W] tensor; the k-step's channel base goes in soffset
    const int HW = H * W;
    const unsigned frange = 4u * static_cast<unsigned>(C * HW);
    const __amdgpu_buffer_rsrc_t rl = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(Lf + static_cast<long long>(b) * C * HW), static_cast<short>(0), frange, 0x00020000);
    const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(Rf + static_cast<long long>(b) * C * HW), static_cast<short>(0), frange, 0x00020000);
    unsigned loff[LR], roff[RR];
#pragma unroll
    for (int k = 0; k < LR; ++k) {
        const int f = tid + k * kGsThreads;
        const int c = f / G::LW, r = f % G::LW, iy = r / IX, ix = r % IX;
        const int y = yi0 + iy, x = xi0 + ix;
        const bool ok = f < G::LE && y >= 0 && y < H && x >= 0 && x < W;
        loff[k] = ok ? 4u * static_cast<unsigned>(c * HW + y * W + x) : kOOB;
    }
#pragma unroll
    for (int k = 0; k < RR; ++k) {
        const int f = tid + k * kGsThreads;
        const int c = f / G::RW, r = f % G::RW, iy = r / G::RX, rx = r % G::RX;
        const int y = yi0 + iy, x = xi0 - (zi0 + G::IZ - 1) + rx;
        const bool ok = f < G::RE && y >= 0 && y < H && x >= 0 && x < W;
        roff[k] = ok ? 4u * static_cast<unsigned>(c * HW + y * W + x) : kOOB;
    }
    // the volume window is built by columns: a thread owns window columns (ci, iy, ix) and forms all IZ
    // disparity planes of each from one left value per channel and IZ consecutive right values (the
    // shifts), NRND columns per thread (a thread past the last column repeats its first one: the same
    // values to the same addresses).  cl / cr: LDS indices of the left value / the right value of plane
    // 0 (channel CPG ci); cx: xs index of plane 0; vm: the elements that exist (bit r * IZ + iz:
    // disparity plane inside [0, D), pixel inside the map, x >= d), the rest are the conv's zero padding
    constexpr int IZ = G::IZ, NCOL = 4 * IY * IX, NRND = (NCOL + kGsThreads - 1) / kGsThreads;
    static_assert(NCOL >= kGsThreads && NRND * IZ <= 32, "column plan");
    unsigned cl[NRND], cr[NRND], cx[NRND], vm = 0;
#pragma unroll
    for (int r = 0; r < NRND; ++r) {
        int col = tid + r * kGsThreads;
        col = col < NCOL ? col : tid;
        const int ci = col / (IY * IX), iy = (col / IX) % IY, ix = col % IX;
        cl[r] = static_cast<unsigned>(CPG * ci * G::LW + iy * IX + ix);
        cr[r] = static_cast<unsigned>(G::LE + CPG * ci * G::RW + iy * G::RX + ix + IZ - 1);
        cx[r] = static_cast<unsigned>(ci * CS + iy * IX + ix);
        const int y = yi0 + iy, x = xi0 + ix;
#pragma unroll
        for (int iz = 0; iz < IZ; ++iz) {
            const int d = zi0 + iz;
            const bool ok = d >= 0 && d < D && y >= 0 && y < H && x < W && x >= d;
            vm |= (ok ? 1u : 0u) << (r * IZ + iz);
        }
    }
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w), static_cast<short>(0), 4 * 27 * a.cin_pad * a.cout_pad, 0x00020000);
    unsigned woff[WR];
#pragma unroll
    for (int k = 0; k < WR; ++k) {  // e = ((p * 9 + t9) * 4 + ci) * 16 + m: input plane p of the pair's window
        const int e = tid + k * kGsThreads;
        const int m = e & 15, ci = (e >> 4) & 3, t9 = (e >> 6) % 9, p = (e >> 6) / 9;
        const int dz = p - (m >> 3), co = m & 7;
        const bool ok = e < G::WE && dz >= 0 && dz <= 2 && co < a.Cout;
        woff[k] = ok ? 4u * static_cast<unsigned>(((dz * 9 + t9) * a.cin_pad + ci) * a.cout_pad + co) : kOOB;
    }

    // WREG: lane (g, n)'s A operand of (input plane p, tap t9) at k-step ch is W[dz = p - n / 8][t9][4 ch + g][n % 8]
    // (zero outside dz 0..2 or past Cout): per-lane offset of plane p, the tap and k-step in soffset
    unsigned wpo[4];
#pragma unroll
    for (int p = 0; p < 4; ++p) {
        const int dz = p - (n >> 3), co = n & 7;
        wpo[p] = (dz >= 0 && dz <= 2 && co < a.Cout) ? 4u * static_cast<unsigned>((dz * 9 * a.cin_pad + g) * a.cout_pad + co)
                                                     : kOOB;
    }
    // one register per (p, t9): reloaded with the next k-step's value right after its last MFMA of this k-step
    // (a k-step past the last one reads weights no MFMA uses; the buffer range check keeps it inside the slab)
    float wa[WREG ? 36 : 1];
    auto wreg_load = [&](int i, int ch) __attribute__((always_inline)) {
        if constexpr (WREG) wa[i] = buf_load_s(wrs, wpo[i / 9], 4 * ((i % 9) * a.cin_pad + 4 * ch) * a.cout_pad);
    };

    float lv[LR], rv[RR], wv[WREG ? 1 : WR];
    auto fload = [&](int ch) __attribute__((always_inline)) {
        const int so = 4 * G::FC * ch * HW;
#pragma unroll
        for (int k = 0; k < LR; ++k) lv[k] = buf_load_s(rl, loff[k], so);
#pragma unroll
        for (int k = 0; k < RR; ++k) rv[k] = buf_load_s(rr, roff[k], so);
    };
    auto fstore = [&](int fb) __attribute__((always_inline)) {
#pragma unroll
        for (int k = 0; k < LR; ++k) {
            const int f = tid + k * kGsThreads;
            if (f < G::LE) fs[fb][f] = lv[k];
        }
#pragma unroll
        for (int k = 0; k < RR; ++k) {
            const int f = tid + k * kGsThreads;
            if (f < G::RE) fs[fb][G::LE + f] = rv[k];
        }
    };
    auto wload = [&](int ch) __attribute__((always_inline)) {
        if constexpr (!WREG) {
#pragma unroll
            for (int k = 0; k < WR; ++k) wv[k] = buf_load_s(wrs, woff[k], 4 * 4 * ch * a.cout_pad);
        }
    };
    auto wstore = [&](int buf) __attribute__((always_inline)) {
        if constexpr (!WREG) {
#pragma unroll
            for (int k = 0; k < WR; ++k) {
                const int e = tid + k * kGsThreads;
                if (e < G::WE) ws[buf][e] = wv[k];
            }
        }
    };
    // two planes (iz, iz + 1) of one column of a k-step's window from the staged feature windows
    // (volumes.hip gwc_kernel's arithmetic: products and the pairwise sum rounded one operation at a time)
    float lft[NRND][CPG];
    auto load_left = [&](int fb) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < NRND; ++r)
#pragma unroll
            for (int c = 0; c < CPG; ++c) lft[r][c] = fs[fb][cl[r] + c * G::LW];
    };
    // the two planes as packed fp32 (v_pk_mul_f32 / v_pk_add_f32: per plane the same operations, so the same bits)
    typedef float f2 __attribute__((ext_vector_type(2)));
    auto volume_pair = [&](int u, int fb, int buf) __attribute__((always_inline)) {
        const int r = u / (IZ / 2), iz = 2 * (u % (IZ / 2));
        const float inv = 1.0f / static_cast<float>(CPG);
        f2 sv;
        {
#pragma clang fp contract(off)
            sv = f2{lft[r][0], lft[r][0]} * f2{fs[fb][cr[r] - iz], fs[fb][cr[r] - iz - 1]};
#pragma unroll
            for (int c = 1; c < CPG; ++c)
                sv = sv + f2{lft[r][c], lft[r][c]} * f2{fs[fb][cr[r] + c * G::RW - iz], fs[fb][cr[r] + c * G::RW - iz - 1]};
            sv = sv * f2{inv, inv};
        }
        xs[buf][cx[r] + iz * PLANE] = (vm >> (r * IZ + iz)) & 1u ? sv[0] : 0.f;
        xs[buf][cx[r] + (iz + 1) * PLANE] = (vm >> (r * IZ + iz + 1)) & 1u ? sv[1] : 0.f;
    };
    constexpr int NU = NRND * IZ / 2;  // plane pairs per thread and k-step

    float scl[4], shf[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int cc = min((4 * g + j) & 7, a.Cout - 1);
        scl[j] = a.scale ? a.scale[cc] : 1.f;
        shf[j] = a.shift ? a.shift[cc] : 0.f;
    }
    floatx4 acc[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[nt] = floatx4{0.f, 0.f, 0.f, 0.f};

    // k-steps past the last one load zeros (range-checked offsets past the buffers) and build windows no
    // MFMA reads, so the loop body has no branch between its MFMAs and the next window's work
    const int nchunk = a.Cin >> 2;
    fload(0);
    wload(0);
    if constexpr (WREG) {
#pragma unroll
        for (int i = 0; i < 36; ++i) wreg_load(i, 0);
    }
    fstore(0);
    wstore(0);
    fload(1);
    __syncthreads();
    load_left(0);
#pragma unroll
    for (int u = 0; u < NU; ++u) volume_pair(u, 0, 0);
    fstore(1);
    __syncthreads();
    for (int ch = 0; ch < nchunk; ++ch) {
        const int buf = ch & 1;
        fload(ch + 2);
        wload(ch + 1);
        // keep the loads here: left to itself the scheduler sinks them below the MFMAs, next to the LDS
        // stores that wait for them, and every k-step then waits out a full memory latency
        __builtin_amdgcn_sched_barrier(0);
        const float* xw = &xs[buf][g * CS + n];
        const float* wp = &ws[WREG ? 0 : buf][g * 16 + n];
        load_left((ch + 1) & 1);
#pragma unroll
        for (int it = 0; it < 12; ++it) {
            const int p = it / 3, dx = it % 3;
            float br[NR];
#pragma unroll
            for (int r = 0; r < NR; ++r) br[r] = xw[(2 * zw + p) * PLANE + r * IX + dx];
#pragma unroll
            for (int dy = 0; dy < 3; ++dy) {
                const float av = WREG ? wa[WREG ? p * 9 + dy * 3 + dx : 0] : wp[((p * 9 + dy * 3 + dx) * 4) * 16];
#pragma unroll
                for (int nt = 0; nt < NT; ++nt)
                    acc[nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, br[nt + dy], acc[nt], 0, 0, 0);
                wreg_load(p * 9 + dy * 3 + dx, ch + 1);
            }
            // k-step ch + 1's volume window, spread over the MFMA stream
#pragma unroll
            for (int u = it; u < NU; u += 12) volume_pair(u, (ch + 1) & 1, buf ^ 1);
        }
        wstore(buf ^ 1);
        fstore(ch & 1);
        __syncthreads();
    }

    // epilogue (tconv3_kernel's, plane pairs): lane (g, n) holds rows m = 4g + j = (plane 2 zw + m / 8, cout m % 8)
    const int x = xo0 + n;
    const __amdgpu_buffer_rsrc_t ro_ = __builtin_amdgcn_make_buffer_rsrc(
        a.out + b * a.ob, static_cast<short>(0),
        4 * ((a.Cout - 1) * static_cast<int>(a.oc) + (a.Do - 1) * static_cast<int>(a.od) +
             (a.Ho - 1) * static_cast<int>(a.oh) + a.Wo),
        0x00020000);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
        const int y = yo0 + nt;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int m = 4 * g + j;
            const int co = m & 7;
            const int z = zo0 + 2 * zw + (m >> 3);
            const bool ok = co < a.Cout && z < a.Do && y < a.Ho && x < a.Wo;
            float v = acc[nt][j];
            v = a.scale ? v * scl[j] + shf[j] : v + shf[j];
            v = act_t<ACT>(v, a.act);
            if constexpr (PLAIN) {
                const unsigned o = ok ? 4u * static_cast<unsigned>(co * static_cast<int>(a.oc) + z * static_cast<int>(a.od) +
                                                                   y * static_cast<int>(a.oh) + x)
                                      : kOOB;
                store_b32(__float_as_uint(v), ro_, static_cast<int>(o), 0);
            } else {
                if (!ok) continue;
                const long long o = b * a.ob + co * a.oc + static_cast<long long>(z) * a.od +
                                    static_cast<long long>(y) * a.oh + x;
                a.out[o] = v * a.post_scale;
            }
        }
    }
}

template <int NT, int CPG, bool WREG>
int launch_gs(const esm_conv_desc& a, const float* L, const float* R, int C, hipStream_t s) {
    using G = GsGeo<NT, CPG>;
    const long long z = static_cast<long long>(a.B) * ((a.Do + G::ZB - 1) / G::ZB);
    const long long gy = ceil_div(a.Ho, G::YB);
    if (z > 65535 || gy > 65535) return arg_error("gwc_stem: grid too large");
    const dim3 grid(ceil_div(a.Wo, 16), static_cast<unsigned>(gy), static_cast<unsigned>(z));
    const bool plain = a.act == ESM_ACT_GELU && a.post_scale == 1.f;
    if (plain)
        hipLaunchKernelGGL((gwc_stem_kernel<NT, CPG, ESM_ACT_GELU, true, WREG>), grid, dim3(kGsThreads), 0, s, a, L, R, C);
    else
        hipLaunchKernelGGL((gwc_stem_kernel<NT, CPG, -1, false, WREG>), grid, dim3(kGsThreads), 0, s, a, L, R, C);
    return check_launch("gwc_stem");
}

}  // namespace

// Which stems the fused form takes: a 3x3x3 stride-1 pad-1 BasicConv over the whole G-group volume of
// contiguous [B, C, H, W] features, C = 2 G, G a multiple of 4, <= 8 couts, no extra epilogue operands.
int gwc_stem_check(const esm_conv_desc& a, const float* L, const float* R, int C, int G) {
    if (!L || !R || !a.w || !a.out) return arg_error("gwc_stem: null features / weights / output");
    if (G <= 0 || G % 4 || C != 2 * G) return arg_error("gwc_stem: needs C = 2 G and G a multiple of 4");
    if (a.Cin != G || a.Cout < 1 || a.Cout > 8) return arg_error("gwc_stem: the stem must map G -> <= 8 channels");
    if (a.transposed || a.kd != 3 || a.kh != 3 || a.kw != 3 || a.stride != 1 || a.pd != 1 || a.ph != 1 || a.pw != 1)
        return arg_error("gwc_stem: the stem must be a 3x3x3 stride-1 pad-1 conv");
    if (a.B <= 0 || a.Di <= 0 || a.Hi <= 0 || a.Wi <= 0 || a.Do != a.Di || a.Ho != a.Hi || a.Wo != a.Wi)
        return arg_error("gwc_stem: bad volume extent");
    if (a.mul || a.res || a.up || a.out2 || a.shuffle > 1) return arg_error("gwc_stem: no mul / res / up / out2 / shuffle");
    if (a.cin_pad % 16 || a.cin_pad < a.Cin || a.cout_pad % 32 || a.cout_pad < a.Cout)
        return arg_error("gwc_stem: bad weight padding");
    const long long fspan = 4LL * C * a.Hi * a.Wi;
    const long long ospan = 4LL * ((a.Cout - 1) * a.oc + (a.Do - 1) * a.od + (a.Ho - 1) * a.oh + a.Wo);
    const long long wspan = 4LL * 27 * a.cin_pad * a.cout_pad;
    if (fspan >= kOOB || ospan >= kOOB || wspan >= kOOB || a.oc < 0 || a.od < 0 || a.oh < 0)
        return arg_error("gwc_stem: spans beyond the 32-bit buffer offsets");
    return ESM_OK;
}

int launch_gwc_stem(const esm_conv_desc& a, const float* L, const float* R, int C, int G, hipStream_t s) {
    const int rc = gwc_stem_check(a, L, R, C, G);
    if (rc != ESM_OK) return rc;
    // rows per wave as the tiled stem's automatic choice (conv_tile3.hip launch_tile3, plane pairs)
    const long long vox = static_cast<long long>(a.B) * a.Do * a.Ho * a.Wo;
    const int rsel = (a.hint >> 26) & 3;
    // hint bit 28: the LDS-staged weights (round 5); default: weights in registers (round 6)
    const bool lds_w = (a.hint >> 28) & 1;
    if (rsel == 2 || (rsel == 0 && vox < (1LL << 20)))
        return lds_w ? launch_gs<2, 2, false>(a, L, R, C, s) : launch_gs<2, 2, true>(a, L, R, C, s);
    return lds_w ? launch_gs<4, 2, false>(a, L, R, C, s) : launch_gs<4, 2, true>(a, L, R, C, s);
}

}  // namespace conv
}  // namespace esm

extern "C" int esm_gwc_stem_f32(const esm_conv_desc* stem, const float* L, const float* R, int C, int G, void* stream) {
    if (!stem) return esm::arg_error("gwc_stem: null descriptor");
    return esm::conv::launch_gwc_stem(*stem, L, R, C, G, esm::as_stream(stream));
}
