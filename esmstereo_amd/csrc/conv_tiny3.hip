// Two consecutive 3x3x3 BasicConv3d on a tiny volume in one launch (round 6): the bottom of the aggregation
// hourglass, conv3 = BasicConv(stride 2) -> BasicConv(stride 1) (models/ESMStereo.py:139-141, 160-161), whose
// output at S-K is 2 x 3 x 10 = 60 voxels.  As two launches each is a latency chain of its own (6.7 + 6.9 us in the
// S-K graph, profiles/r06_ops_SK.txt); here
//   * every workgroup computes convA's whole output (<= 128 voxels, <= 32 couts) into LDS with the 16 waves
//     splitting its (cout tile, voxel tile) pairs and K (tap-major k-steps), partial sums added in LDS in a fixed
//     order, BN + GELU applied -- the input volume is read from global / L2 (every workgroup reads it);
//   * workgroup g then computes convB's (cout tile, voxel tile) number g from that LDS volume, its 16 waves splitting
//     K, and stores it.  convA's output never leaves LDS.
// MFMA operands: A = weights (packed w[tap][cin_pad][cout_pad], lane (i, q) holds W[tap][c0 + q][16 mt + i]),
// B = 4 channels x 16 voxels (lane (q, n): channel c0 + q of output voxel 16 nt + n's tap-shifted input, 0 outside
// the volume).  Each output is one fixed-order sum: deterministic; fp32 reassociation of the other forms' order
// (tests: 1e-5 relative).
#include "conv_direct.h"

namespace esm {

int conv_check(const esm_conv_desc& a);  // conv.hip

namespace conv {
namespace {

constexpr int kTyWaves = 16;
constexpr int kTyThreads = 64 * kTyWaves;
constexpr int kTyMaxVox = 128;  // convA / convB output voxels (8 voxel tiles)
constexpr int kTyMaxCout = 32;  // two cout tiles per conv

struct TyConv {  // one conv's geometry as the kernel walks it
    int Di, Hi, Wi, Do, Ho, Wo, S, Cin, ck;  // ck: 4-channel k-steps per tap
};

__device__ __forceinline__ TyConv ty_geo(const esm_conv_desc& d) {
    return TyConv{d.Di, d.Hi, d.Wi, d.Do, d.Ho, d.Wo, d.stride, d.Cin, (d.Cin + 3) >> 2};
}

// the partial sum of one (cout tile mt, voxel tile nt) over k-steps [k0, k1) (k = tap * ck + chunk); IN(ok, c, z, y, x)
// returns input channel c at (z, y, x), or 0 where !ok (an unconditional load then a select: a conditional load
// would make the compiler branch around it and wait for each one) -- global for convA, LDS for convB.  Batches of 8
// k-steps issue their operand loads together.
template <typename In>
__device__ __forceinline__ floatx4 ty_tile(const esm_conv_desc& d, const TyConv& g, int mt, int nt, int k0, int k1,
                                           int lane, In in) {
    const int q = lane >> 4, n = lane & 15;
    const int v = nt * 16 + n;
    const int vo = g.Do * g.Ho * g.Wo;
    const bool vok = v < vo;
    const int oz = vok ? v / (g.Ho * g.Wo) : 0, oy = vok ? (v / g.Wo) % g.Ho : 0, ox = vok ? v % g.Wo : 0;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(d.w), static_cast<short>(0),
                                                                         4 * 27 * d.cin_pad * d.cout_pad, 0x00020000);
    const unsigned wl = 4u * static_cast<unsigned>(q * d.cout_pad + 16 * mt + n);
    floatx4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k = k0; k < k1; k += 8) {
        float av[8], bv[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
            const int kk = k + u;
            const int tap = kk / g.ck, c0 = 4 * (kk - tap * g.ck);
            const int dz = tap / 9, dy = (tap / 3) % 3, dx = tap % 3;
            const int iz = oz * g.S - 1 + dz, iy = oy * g.S - 1 + dy, ix = ox * g.S - 1 + dx;
            const bool ok = kk < k1 && vok && c0 + q < g.Cin && iz >= 0 && iz < g.Di && iy >= 0 && iy < g.Hi && ix >= 0 &&
                            ix < g.Wi;
            bv[u] = in(ok, c0 + q, iz, iy, ix);
            av[u] = buf_load_s(wrs, kk < k1 ? wl : kOOB, 4 * (tap * d.cin_pad + c0) * d.cout_pad);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(av[u], bv[u], acc, 0, 0, 0);
    }
    return acc;
}

__global__ void __launch_bounds__(kTyThreads) tiny3_pair_kernel(const esm_conv_desc a, const esm_conv_desc b) {
    __shared__ float ya[kTyMaxCout * kTyMaxVox];           // convA's output [co][voxel]
    __shared__ float red[kTyWaves][256];                    // partial tiles (lane-major D layout)
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int bi = blockIdx.y;
    const TyConv ga = ty_geo(a), gb = ty_geo(b);
    const int va = ga.Do * ga.Ho * ga.Wo, vb = gb.Do * gb.Ho * gb.Wo;
    const int mta = (a.Cout + 15) >> 4, nta = (va + 15) >> 4, ta = mta * nta;
    const int ksa = max(1, kTyWaves / ta);  // K slices per convA tile (ta x ksa <= 16 work items)
    const int kka = 27 * ga.ck;

    // ---- convA: item w = (tile w % ta, K slice w / ta)
    const esm_src& s0 = a.src[0];
    const float* xb = s0.ptr + bi * s0.sb;
    auto in_a = [&](bool ok, int c, int z, int y, int x) __attribute__((always_inline)) {
        const float v = xb[ok ? c * s0.sc + z * s0.sd + y * s0.sh + x : 0];
        return ok ? v : 0.f;
    };
    if (wave < ta * ksa) {
        const int t = wave % ta, ks = wave / ta;
        const floatx4 acc = ty_tile(a, ga, t / nta, t % nta, kka * ks / ksa, kka * (ks + 1) / ksa, lane, in_a);
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wave][r * 64 + lane] = acc[r];
    }
    __syncthreads();
    // reduce in K-slice order, BN + GELU, into ya (zero past Cout / the volume: convB's padding reads)
    for (int e = tid; e < ta * 256; e += kTyThreads) {
        const int t = e >> 8, r = (e >> 6) & 3, l = e & 63;
        float v = 0.f;
        for (int ks = 0; ks < ksa; ++ks) v += red[ks * ta + t][r * 64 + l];
        const int co = 16 * (t / nta) + 4 * (l >> 4) + r, vox = 16 * (t % nta) + (l & 15);
        if (co < a.Cout && vox < va) {
            v = a.scale ? v * a.scale[co] + a.shift[co] : v + a.shift[co];
            ya[co * kTyMaxVox + vox] = act_t<ESM_ACT_GELU>(v, a.act);
        }
    }
    __syncthreads();

    // ---- convB: this workgroup's tile, K split over the 16 waves
    const int ntb = (vb + 15) >> 4;
    const int t = blockIdx.x, mt = t / ntb, nt = t % ntb;
    const int kkb = 27 * gb.ck;
    auto in_b = [&](bool ok, int c, int z, int y, int x) __attribute__((always_inline)) {
        const float v = ya[ok ? c * kTyMaxVox + (z * gb.Hi + y) * gb.Wi + x : 0];
        return ok ? v : 0.f;
    };
    const floatx4 acc = ty_tile(b, gb, mt, nt, kkb * wave / kTyWaves, kkb * (wave + 1) / kTyWaves, lane, in_b);
#pragma unroll
    for (int r = 0; r < 4; ++r) red[wave][r * 64 + lane] = acc[r];
    __syncthreads();
    if (tid < 256) {
        const int r = tid >> 6, l = tid & 63;
        float v = 0.f;
        for (int w = 0; w < kTyWaves; ++w) v += red[w][r * 64 + l];
        const int co = 16 * mt + 4 * (l >> 4) + r, vox = 16 * nt + (l & 15);
        if (co < b.Cout && vox < vb) {
            v = b.scale ? v * b.scale[co] + b.shift[co] : v + b.shift[co];
            const int z = vox / (gb.Ho * gb.Wo), y = (vox / gb.Wo) % gb.Ho, x = vox % gb.Wo;
            b.out[bi * b.ob + co * b.oc + z * b.od + y * b.oh + x] = act_t<ESM_ACT_GELU>(v, b.act);
        }
    }
}

}  // namespace

// convA: 3x3x3 stride 1 / 2 pad 1, one source, <= 32 couts, <= 128 output voxels; convB: 3x3x3 stride 1 pad 1 over
// convA's output, <= 32 couts; both plain BasicConvs (BN + GELU)
bool tiny3_ok(const esm_conv_desc& a, const esm_conv_desc& b) {
    auto k3 = [](const esm_conv_desc& d) {
        return !d.transposed && d.kd == 3 && d.kh == 3 && d.kw == 3 && d.pd == 1 && d.ph == 1 && d.pw == 1 && d.nsrc == 1 &&
               d.act == ESM_ACT_GELU && !d.mul && !d.res && !d.up && !d.out2 && !d.pre && d.post_scale == 1.f && d.shift;
    };
    if (!k3(a) || !k3(b) || (a.stride != 1 && a.stride != 2) || b.stride != 1) return false;
    if (a.Cout > kTyMaxCout || b.Cout > kTyMaxCout || b.Cin != a.Cout || b.B != a.B || !b.out) return false;
    if (b.Di != a.Do || b.Hi != a.Ho || b.Wi != a.Wo || b.Do != b.Di || b.Ho != b.Hi || b.Wo != b.Wi) return false;
    return static_cast<long long>(a.Do) * a.Ho * a.Wo <= kTyMaxVox;
}

int launch_tiny3(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    esm_conv_desc ac = a;
    if (!ac.out) ac.out = b.out;  // convA's output is never written; conv_check wants a pointer
    int rc = conv_check(ac);
    if (rc == ESM_OK) rc = conv_check(b);
    if (rc != ESM_OK) return rc;
    if (!tiny3_ok(a, b)) return arg_error("conv pair (3-D): unsupported pair");
    const int vb = b.Do * b.Ho * b.Wo;
    const dim3 grid(((b.Cout + 15) >> 4) * ((vb + 15) >> 4), a.B);
    if (a.B > 65535) return arg_error("conv pair (3-D): batch too large");
    hipLaunchKernelGGL(tiny3_pair_kernel, grid, dim3(kTyThreads), 0, s, a, b);
    return check_launch("conv pair (3-D)");
}

}  // namespace conv
}  // namespace esm
