// Narrow-output 3x3(x3) convolutions on the 16-block fp32 MFMA (v_mfma_f32_4x4x1_16b_f32).
//
// Reference layers: the 3-D stems BasicConv(32->8) `group_stem`, BasicConv(1->8) `corr_stem`,
// BasicConv(8->8) `agg` (models/ESMStereo.py:610-622, used at :703-715) and, by shape, every other
// stride-1 3x3(x3) BasicConv with 8 or 12 output channels (models/submodule.py:12-38).
//
// Why a third MFMA form: with 8 couts the 16x16x4 tile of the direct / row-streaming forms
// computes 16 output rows of which 8 are padding, so half of every MFMA is wasted; the stems are
// the largest layers of the L hot path (group_stem alone ~20 GFLOP at KITTI size).  The 16-block
// 4x4x1 MFMA takes the same 8 cycles per 512 FLOP as the 16x16x4 takes per 2048 (full f32 rate,
// MI355X_MICROARCH.md §Matrix cores), and its 4-row blocks fit 8 / 12 couts exactly.
//
// Mapping (one wave):
//   lane l = 16*r + n: r = output row of the wave's 4-row group, n = column in a 16-lane tile;
//   block b = l/4 of the MFMA holds lanes 4b..4b+3.  A_b[i][0] (lane 4b+i) = W[co_g + i][k] — the
//   same weights in every block; B_b[0][j] (lane 4b+j) = X[k][pixel of lane 4b+j]; so D_b[i][j]
//   (VGPR i, lane 4b+j) = output channel co_g + i at the pixel of lane l = 4b + j.
//   B: one buffer_load per (channel, tap plane, tap row) brings 16 consecutive input columns per
//   row; the 3 horizontal taps are DPP row shifts (conv_rows.h row_shift), so a 16-lane tile
//   yields 14 output columns and needs no edge loads; out-of-range rows / columns / channels read
//   zero through the buffer range check (kOOB marks, conv_direct.h).
//   A: the workgroup's weights are staged once in LDS as [ci][tap][i][g] (g = cout group), so the
//   CG couts a lane needs for one k are one broadcast ds_read_b64 / b128 (4 distinct addresses).
// Workgroup = 4 waves = 4 consecutive output planes (3-D) or 4 row groups (2-D) of one 14-column
// tile.  Channel chunks of CK are double-buffered: the next chunk's loads are issued before the
// current chunk's MFMAs.  Accumulation order over k is fixed (deterministic).
#include "conv_rows.h"

namespace esm {
namespace conv {
namespace {

__device__ __forceinline__ floatx4 mfma4(float a, float b, floatx4 c) {
    return __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
}

// KS: the 4 waves split the input-channel chunks of ONE 4-row tile (grids far below one
// workgroup per CU) and add their partial sums in LDS in a fixed order.
// NW: waves per workgroup, 4 or 8 (3-D only: 8 consecutive planes share one staged weight slab, for
// slabs so large that the LDS would otherwise hold two 4-wave workgroups per CU).
template <bool D3, int CG, int CK, bool KS, int NW = 4>
__global__ void __launch_bounds__(64 * NW) sconv_kernel(const esm_conv_desc a) {
    static_assert(NW == 4 || (NW == 8 && D3 && !KS), "8-wave workgroups: 3-D, no K split");
    constexpr int NT = 64 * NW;
    constexpr int K = 3;
    constexpr int KDT = D3 ? 3 : 1;
    constexpr int TAPS = KDT * 9;
    constexpr int CGP = CG == 3 ? 4 : CG;  // LDS entry width (even: float2 / float4 reads)
    constexpr int VALID = 14;
    constexpr int NB = CK * KDT * K;        // B values of one chunk
    extern __shared__ float wl[];           // [cin_stage][TAPS][4][CGP]

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
    const int n = lane & 15;
    const int r = lane >> 4;
    const int q = lane & 3;
    const int Ho = a.Ho, Wo = a.Wo, Do = D3 ? a.Do : 1;
    const int tiles_w = (Wo + VALID - 1) / VALID;
    // 3-D: a workgroup = 4 planes x 4 rows; 2-D: 16 rows (4 groups of 4)
    const int tiles_h = (D3 || KS) ? (Ho + 3) / 4 : (Ho + 15) / 16;
    const int tiles_z = D3 ? (KS ? Do : (Do + NW - 1) / NW) : 1;
    // XCD-aware order (conv_direct.h): each XCD takes a contiguous range of tiles
    const unsigned nwg = gridDim.x, orig = blockIdx.x;
    const unsigned q8 = nwg / 8, r8 = nwg % 8, xcd = orig % 8;
    unsigned wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + orig / 8;
    const int tx = static_cast<int>(wg % tiles_w);
    wg /= tiles_w;
    const int ty = static_cast<int>(wg % tiles_h);
    wg /= tiles_h;
    const int tz = static_cast<int>(wg % tiles_z);
    const int b = static_cast<int>(wg / tiles_z);
    if (b >= a.B) return;  // whole workgroup, before any barrier: a grid larger than the tile count stays in bounds
    const int oz = D3 ? (KS ? tz : tz * NW + wave) : 0;
    const int oy = (D3 || KS) ? ty * 4 + r : ty * 16 + wave * 4 + r;  // this lane's output row
    const int o0 = tx * VALID;
    const int xi = o0 - 1 + n;  // input column held by this lane (pad 1)

    const esm_src& s0 = a.src[0];
    const int sc = static_cast<int>(s0.sc), sd = static_cast<int>(s0.sd), sh = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc + (D3 ? (a.Di - 1) * sd : 0) + (a.Hi - 1) * sh + a.Wi), 0x00020000);
    const bool zok = oz < Do;
    // per (tap plane, tap row): row part of this lane's offset (kOOB when the row is padding)
    unsigned roff[KDT][K];
#pragma unroll
    for (int td = 0; td < KDT; ++td)
#pragma unroll
        for (int th = 0; th < K; ++th) {
            const int zi = oz - 1 + td, yi = oy - 1 + th;
            const bool ok = zok && yi >= 0 && yi < a.Hi && (!D3 || (zi >= 0 && zi < a.Di)) && xi >= 0 && xi < a.Wi;
            roff[td][th] = ok ? 4u * ((D3 ? zi * sd : 0) + yi * sh + xi) : kOOB;
        }

    auto load_chunk = [&](float (&bv)[NB], int cc) {
#pragma unroll
        for (int k = 0; k < CK; ++k) {
            const unsigned co = cc + k < a.Cin ? 4u * (cc + k) * sc : kOOB;
#pragma unroll
            for (int td = 0; td < KDT; ++td)
#pragma unroll
                for (int th = 0; th < K; ++th) bv[(k * KDT + td) * K + th] = buf_load_s(rs, roff[td][th] + co, 0);
        }
    };

    constexpr int CSTEP = KS ? 4 * CK : CK;  // channel step of one wave
    const int c_first = KS ? wave * CK : 0;
    float bcur[NB];
    load_chunk(bcur, c_first);
    // weights -> LDS: wl[((ci * TAPS + tap) * 4 + i) * CGP + g] = w[tap][ci][4g + i]
    const int cst = (a.Cin + CK - 1) / CK * CK;  // staged channels (whole chunks; past Cin: zeros)
    {
        const int total = cst * TAPS * 4 * CGP;
        for (int e0 = 0; e0 < total; e0 += NT * 8) {
            float v[8];
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * NT + static_cast<int>(threadIdx.x);
                const int g = e % CGP, i = (e / CGP) & 3, rest = e / (4 * CGP);
                const int tap = rest % TAPS, ci = rest / TAPS;
                const int co = 4 * g + i;
                v[u] = (e < total && g < CG && ci < a.Cin && co < a.Cout)
                           ? a.w[(static_cast<long long>(tap) * a.cin_pad + ci) * a.cout_pad + co]
                           : 0.f;
            }
#pragma unroll
            for (int u = 0; u < 8; ++u) {
                const int e = e0 + u * NT + static_cast<int>(threadIdx.x);
                if (e < total) wl[e] = v[u];
            }
        }
    }
    __syncthreads();

    // independent accumulation chains: a 4x4x1 MFMA issues every 8 cycles but its result is ready
    // later (PMC: 58% of group_stem's wave cycles were issue stalls with 2 chains), so consecutive
    // MFMAs of one group go to different chains
    constexpr int NCH = CG <= 3 ? 4 : 2;
    floatx4 acc[NCH][CG];
#pragma unroll
    for (int c = 0; c < NCH; ++c)
#pragma unroll
        for (int g = 0; g < CG; ++g) acc[c][g] = floatx4{0.f, 0.f, 0.f, 0.f};

    for (int cc = c_first; cc < cst; cc += CSTEP) {
        float bnext[NB];
        if (cc + CSTEP < cst) load_chunk(bnext, cc + CSTEP);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int k = 0; k < CK; ++k)
#pragma unroll
            for (int td = 0; td < KDT; ++td)
#pragma unroll
                for (int th = 0; th < K; ++th) {
                    const float v = bcur[(k * KDT + td) * K + th];
#pragma unroll
                    for (int tw = 0; tw < K; ++tw) {
                        const float bs = tw == 0 ? row_shift<-1>(v) : (tw == 1 ? v : row_shift<1>(v));
                        const int tap = (td * K + th) * K + tw;
                        const float* wp = wl + (((cc + k) * TAPS + tap) * 4 + q) * CGP;
                        float av[CGP];
                        if constexpr (CGP % 4 == 0) {
#pragma unroll
                            for (int j = 0; j < CGP / 4; ++j) {
                                const float4 w4 = *reinterpret_cast<const float4*>(wp + 4 * j);
                                av[4 * j] = w4.x;
                                av[4 * j + 1] = w4.y;
                                av[4 * j + 2] = w4.z;
                                av[4 * j + 3] = w4.w;
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < CGP / 2; ++j) {
                                const float2 w2 = *reinterpret_cast<const float2*>(wp + 2 * j);
                                av[2 * j] = w2.x;
                                av[2 * j + 1] = w2.y;
                            }
                        }
                        // chain by tap only: the accumulation order is independent of the chunk size
                        const int ch = ((td * K + th) * K + tw) % NCH;
#pragma unroll
                        for (int g = 0; g < CG; ++g) acc[ch][g] = mfma4(av[g], bs, acc[ch][g]);
                    }
                }
        if (cc + CSTEP < cst) {
#pragma unroll
            for (int i = 0; i < NB; ++i) bcur[i] = bnext[i];
        }
    }

    float sum[CG][4];
#pragma unroll
    for (int g = 0; g < CG; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float t = acc[0][g][i];
#pragma unroll
            for (int c = 1; c < NCH; ++c) t += acc[c][g][i];  // fixed order (deterministic)
            sum[g][i] = t;
        }
    if constexpr (KS) {  // fixed-order reduction of the 4 waves' partial sums
        __shared__ float red[3][CG * 4][64];
        if (wave > 0) {
#pragma unroll
            for (int g = 0; g < CG; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) red[wave - 1][g * 4 + i][lane] = sum[g][i];
        }
        __syncthreads();
        if (wave > 0) return;
#pragma unroll
        for (int w = 0; w < 3; ++w)
#pragma unroll
            for (int g = 0; g < CG; ++g)
#pragma unroll
                for (int i = 0; i < 4; ++i) sum[g][i] += red[w][g * 4 + i][lane];
    }
    // epilogue: lane (r, n) holds output column o0 + n - 1 of row oy (plane oz), couts 4g + i
    const int ox = o0 + n - 1;
    if (!zok || oy >= Ho || n < 1 || n > VALID || ox >= Wo) return;
    const bool plain = !a.mul && !a.res && !a.up && !a.out2;
    const long long rowb = b * a.ob + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox;
#pragma unroll
    for (int g = 0; g < CG; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int co = 4 * g + i;
            if (co >= a.Cout) continue;
            const float s = sum[g][i];
            if (plain) {
                // BN scale / shift loaded here, not before the K loop: 2 * CG * 4 registers less
                // through the loop (wave-uniform: scalar loads)
                const float shf = a.shift ? a.shift[co] : 0.f;
                const float v = a.scale ? s * a.scale[co] + shf : s + shf;
                a.out[rowb + co * a.oc] = apply_act(v, a.act) * a.post_scale;
            } else {
                conv_put(a, conv_finish(a, s, b, co, oz, oy, ox), b, co, oz, oy, ox);
            }
        }
}

#ifdef ESM_STEM_NW4
constexpr bool kStemNW8 = false;  // A/B builds
#else
constexpr bool kStemNW8 = true;
#endif

template <bool D3, int CG, bool KS, int NW = 4>
int launch_sconv_ks(const esm_conv_desc& a, hipStream_t s, int ck, long long nwg) {
    constexpr int TAPS = D3 ? 27 : 9;
    constexpr int CGP = CG == 3 ? 4 : CG;
    const int cst = (a.Cin + ck - 1) / ck * ck;
    const size_t lds = static_cast<size_t>(cst) * TAPS * 4 * CGP * sizeof(float);
    if (nwg > 0x7fffffffLL) return arg_error("conv: grid too large");
    const dim3 grid(static_cast<unsigned>(nwg));
    if (ck == 1)
        hipLaunchKernelGGL((sconv_kernel<D3, CG, 1, KS, NW>), grid, dim3(64 * NW), lds, s, a);
    else if (ck == 2)
        hipLaunchKernelGGL((sconv_kernel<D3, CG, 2, KS, NW>), grid, dim3(64 * NW), lds, s, a);
    else
        hipLaunchKernelGGL((sconv_kernel<D3, CG, 4, KS, NW>), grid, dim3(64 * NW), lds, s, a);
    return check_launch("conv(stem)");
}

// Grid / channel-chunk choice: small grids split the channel chunks over the 4 waves (4x the
// workgroups) when there are at least 4 chunks.
template <bool D3, int CG>
int launch_sconv(const esm_conv_desc& a, hipStream_t s) {
    const long long tiles_w = (a.Wo + 13) / 14;
    const long long plain = tiles_w * (D3 ? (a.Ho + 3) / 4 * ((a.Do + 3) / 4) : (a.Ho + 15) / 16) * a.B;
    const int ck_ks = a.Cin >= 16 ? 4 : (a.Cin >= 8 ? 2 : 1);
    if (plain < 512 && (a.Cin + ck_ks - 1) / ck_ks >= 4) {
        const long long nwg = tiles_w * ((a.Ho + 3) / 4) * (D3 ? a.Do : 1) * a.B;
        return launch_sconv_ks<D3, CG, true>(a, s, ck_ks, nwg);
    }
    const int ck = a.Cin <= 1 ? 1 : (a.Cin <= 2 ? 2 : 4);  // the chunk size does not change the order
    if constexpr (D3 && CG >= 6) {
        // a weight slab over 40 KB leaves room for two 4-wave workgroups per CU (2 waves per SIMD):
        // 8 planes per workgroup share it instead (4 waves per SIMD; 2-channel chunks keep the
        // double-buffered operands within the 128 registers that allows)
        const long long slab = static_cast<long long>((a.Cin + 1) / 2 * 2) * 27 * 4 * CG * 4;
        const long long nwg8 = tiles_w * ((a.Ho + 3) / 4) * ((a.Do + 7) / 8) * a.B;
        if (kStemNW8 && slab > 40 * 1024 && nwg8 >= 256) return launch_sconv_ks<D3, CG, false, 8>(a, s, 2, nwg8);
    }
    return launch_sconv_ks<D3, CG, false>(a, s, ck, plain);
}

}  // namespace

// Single-input-channel 2-D convs on the VALU: the refinement heads' first layer (BasicConv(1, C,
// 3, s2, p1), models/ESMStereo.py:190-191) and the disparity feature heads dmNx.0 (BasicConv(1, C,
// 5, p0), :247-248 and twins).  An MFMA tile pads the single channel to a 4-deep k-step (75% of
// every MFMA wasted) and these layers are bandwidth-sized (K*K MACs per output), so one thread per
// output pixel does all couts: K*K loads, K*K*Cout FMAs (weights as LDS broadcasts), Cout
// coalesced stores.
namespace {
constexpr int kC1inTW = 64, kC1inTH = 4;

template <int K, int S, int CO>
__global__ void __launch_bounds__(256) c1in_kernel(const esm_conv_desc a) {
    __shared__ float ws[K * K * CO + 2 * CO];
    const int tid = threadIdx.x;
    for (int i = tid; i < K * K * CO; i += 256) {
        const int tap = i / CO, co = i - (i / CO) * CO;
        ws[i] = co < a.Cout ? a.w[static_cast<long long>(tap) * a.cin_pad * a.cout_pad + co] : 0.f;
    }
    if (tid < CO) {
        const int co = min(tid, a.Cout - 1);
        ws[K * K * CO + tid] = a.scale ? a.scale[co] : 1.f;
        ws[K * K * CO + CO + tid] = a.shift ? a.shift[co] : 0.f;
    }
    const int b = blockIdx.z;
    const int ox = blockIdx.x * kC1inTW + (tid & (kC1inTW - 1));
    const int oy = blockIdx.y * kC1inTH + tid / kC1inTW;
    const esm_src& s0 = a.src[0];
    const float* xb = s0.ptr + b * s0.sb;
    float xv[K * K];
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
        for (int kx = 0; kx < K; ++kx) {
            const int yi = oy * S - a.ph + ky, xi = ox * S - a.pw + kx;
            const bool ok = oy < a.Ho && ox < a.Wo && yi >= 0 && yi < a.Hi && xi >= 0 && xi < a.Wi;
            const float v = xb[ok ? static_cast<long long>(yi) * s0.sh + xi : 0];
            xv[ky * K + kx] = ok ? v : 0.f;
        }
    __syncthreads();
    if (oy >= a.Ho || ox >= a.Wo) return;
    const long long o = b * a.ob + static_cast<long long>(oy) * a.oh + ox;
#pragma unroll 4
    for (int co = 0; co < CO; ++co) {
        if (co >= a.Cout) break;
        float acc = 0.f;
#pragma unroll
        for (int t = 0; t < K * K; ++t) acc += ws[t * CO + co] * xv[t];
        const float v = a.scale ? acc * ws[K * K * CO + co] + ws[K * K * CO + CO + co] : acc + ws[K * K * CO + CO + co];
        // write-through (sc1) store (conv_direct.h kStoreAux): the 7.7 MB first refinement map at
        // S-K leaves no dirty lines for the boundary write-back (-1.6 us on the step)
        __hip_atomic_store(&a.out[o + co * a.oc], apply_act(v, a.act) * a.post_scale, __ATOMIC_RELAXED,
                           __HIP_MEMORY_SCOPE_AGENT);
    }
}

template <int K, int S>
int launch_c1in_k(const esm_conv_desc& a, hipStream_t s) {
    const dim3 grid(ceil_div(a.Wo, kC1inTW), ceil_div(a.Ho, kC1inTH), a.B);
    if (a.Cout <= 16)
        hipLaunchKernelGGL((c1in_kernel<K, S, 16>), grid, dim3(256), 0, s, a);
    else
        hipLaunchKernelGGL((c1in_kernel<K, S, 32>), grid, dim3(256), 0, s, a);
    return check_launch("conv(1-channel input)");
}
}  // namespace

bool c1in_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    return !d3 && !a.transposed && a.Cin == 1 && a.nsrc == 1 && a.Cout <= 32 && a.shuffle <= 1 && !a.mul && !a.res &&
           !a.up && !a.out2 && ((a.kh == 3 && (a.stride == 1 || a.stride == 2)) || (a.kh == 5 && a.stride == 1)) &&
           a.src[0].ptr != nullptr;
}

int launch_c1in(const esm_conv_desc& a, hipStream_t s) {
    if (!c1in_ok(a)) return arg_error("conv: 1-channel-input form not applicable");
    if (a.kh == 5) return launch_c1in_k<5, 1>(a, s);
    return a.stride == 2 ? launch_c1in_k<3, 2>(a, s) : launch_c1in_k<3, 1>(a, s);
}

// Layers this form takes: stride-1 3x3(x3) convs with "same" padding, one source, 8, 12, 16,
// 24 or 32 output channels, no pixel shuffle, a weight slab that fits 64 KiB of LDS.
bool stem_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (a.transposed || a.stride != 1 || a.kh != 3 || a.kw != 3 || (d3 && a.kd != 3)) return false;
    if (a.ph != 1 || a.pw != 1 || (d3 && a.pd != 1) || a.nsrc != 1 || a.shuffle > 1) return false;
    if (a.Cout != 8 && a.Cout != 12 && a.Cout != 16 && a.Cout != 24 && a.Cout != 32) return false;
    const int cgp = a.Cout == 12 ? 4 : a.Cout / 4;
    const long long lds = static_cast<long long>((a.Cin + 3) / 4 * 4) * (d3 ? 27 : 9) * 4 * cgp * 4;
    return lds <= 64 * 1024 && direct_ok(a);
}

template <bool D3>
int launch_stem_d(const esm_conv_desc& a, hipStream_t s) {
    switch (a.Cout) {
        case 8: return launch_sconv<D3, 2>(a, s);
        case 12: return launch_sconv<D3, 3>(a, s);
        case 16: return launch_sconv<D3, 4>(a, s);
        case 24: return launch_sconv<D3, 6>(a, s);
        default: return launch_sconv<D3, 8>(a, s);
    }
}

int launch_stem(const esm_conv_desc& a, hipStream_t s) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    if (!stem_ok(a)) return arg_error("conv: stem form not applicable");
    return d3 ? launch_stem_d<true>(a, s) : launch_stem_d<false>(a, s);
}

// Automatic choice, from scripts/probes/stem_sweep.py on MI355X (profiles/r01_stem_sweep.txt):
// 3-D 8-cout stems at every size; otherwise only large maps (>= 64k output voxels), where the
// per-workgroup weight staging is amortised: 12 / 24 couts (the 16x16 tile pads them) and 16 / 32
// couts over >= 32 input channels (more B reuse per load than the direct form).
bool stem_auto(const esm_conv_desc& a) {
    if (!stem_ok(a)) return false;
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    const long long vox = static_cast<long long>(a.B) * (d3 ? a.Do : 1) * a.Ho * a.Wo;
    if (a.Cout == 8 && d3) return true;
    if (vox < 65536) return false;
    return a.Cout == 8 || a.Cout == 12 || a.Cout == 24 || ((a.Cout == 16 || a.Cout == 32) && a.Cin >= 32);
}

}  // namespace conv
}  // namespace esm
