// Direct-load implicit-GEMM convolution on the gfx950 fp32 matrix cores (no LDS staging).
// Included by conv2d.hip / conv3d.hip next to the LDS-staged kernel of conv_impl.h; the launcher
// picks between them (conv_impl.h launch_geom).
//
// Replaces the same reference layers as conv_impl.h: BasicConv (models/submodule.py:12-38) and
// the plain convs of models/ESMStereo.py:129-509 / models/shufflemixer.py:124-126.
//
// Why a second form: the hot path's convs are small (8-72 channels, B = 1) and a launch is a
// latency chain, not a throughput problem.  Staging a patch through LDS costs every wave a
// load -> barrier -> store -> barrier round trip plus the patch index arithmetic (measured:
// ~1100 VALU + ~1200 SALU instructions per wave for 36 MFMAs, profiles/r01_pmc_conv_sq.txt).
// Here each MFMA operand is one buffer_load straight from L1/L2:
//   B (4 input channels x 16 pixels): lane l reads channel c0 + (l>>4) at pixel (l&15) of the
//     tap's shifted row -> four 64-byte row segments per wave-instruction (coalesced); the
//     byte offset is split into a per-lane voffset (channel + column part, precomputed per
//     chunk) and a wave-uniform soffset (row part), so a load costs no VALU; a part that falls
//     outside the tensor is marked with kOOB, which pushes voffset + soffset past the buffer's
//     range (gfx950 checks the sum: scripts/probes/buffer_oob.hip) so the hardware returns 0
//     (zero padding, padding channels and the tile's right edge need no branches);
//   A (16 couts x 4 k) from the packed weights [cls][tap][cin_pad][cout_pad] (L1-resident).
// A wave owns a 16*NT-pixel x 16*MT-cout output row segment; the 4 waves of a workgroup take
// adjacent rows (their tap rows overlap in L1) and walk RB/4 rows each.  KS = 4 (grids far
// below one wave per SIMD): the 4 waves split the taps of one row and add their partial sums
// in LDS in a fixed order (deterministic).
#pragma once

#include "conv_epilogue.h"

namespace esm {
namespace conv {

// Store cache policy of the buffer-store epilogues: write-through (sc1).  With default-policy
// stores the output's dirty lines are written back at the kernel boundary, on the critical path of
// the launch chain (bytes / ~6 TB/s, MI355X_MICROARCH.md price list "boundary"); written through they
// leave L2 while the kernel runs.  Measured on the S-K step, three rotations on one box (scripts/
// gpu_ab_multi.sh): 382.1 -> 377.0 us.  A per-store runtime choice (sc1 above a size threshold)
// measured 388-390 us: the select splits every store into two branches, so the policy is a constant.
constexpr int kStoreAux = 16;
__device__ __forceinline__ void store_b32(unsigned v, __amdgpu_buffer_rsrc_t r, int vo, int so) {
    __builtin_amdgcn_raw_buffer_store_b32(v, r, vo, so, kStoreAux);
}

constexpr int kDirectThreads = 256;

#ifdef ESM_CONV_STAMPS
// Diagnostic build only (python -m esmstereo_amd.build --diag): per-wave timeline stamps.
__device__ unsigned long long esm_stamps[1 << 20];
__device__ unsigned int esm_stamp_count;
#define ESM_STAMP(v) (v) = __builtin_amdgcn_s_memtime()
#else
#define ESM_STAMP(v) (void)0
#endif
constexpr unsigned kOOB = 0x40000000u;  // offset marker: past the end of every buffer (spans < 1 GiB);
                                        // two marks sum to 2^31, still out of range, no wrap

// voff: per-lane byte offset (carries the kOOB marks; range-checked); soff: wave-uniform part
__device__ __forceinline__ float buf_load_s(__amdgpu_buffer_rsrc_t r, unsigned voff, int soff) {
    return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, static_cast<int>(voff), soff, 0));
}

// The partial conv sum esm_conv_desc.pre (2-D, [B, Cout, Ho, Wo]) at the D-layout elements of lane (n, q) of the
// 16-cout tile from cout c0: rows c0 + 4q + j, output row y, column x -- the accumulator's starting value (0
// past Cout / the map, or without `pre`).
__device__ __forceinline__ floatx4 pre_tile(const esm_conv_desc& a, int b, int c0, int q, int y, int x) {
    floatx4 v = {0.f, 0.f, 0.f, 0.f};
    if (!a.pre || y >= a.Ho || x >= a.Wo) return v;
    const float* p = a.pre + b * a.prb + static_cast<long long>(y) * a.prh + x;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int co = c0 + 4 * q + j;
        if (co < a.Cout) v[j] = p[co * a.prc];
    }
    return v;
}

template <bool D3, int K, int S, bool TR, int MT, int NT, int KS, int CK, bool MS>
__global__ void __launch_bounds__(kDirectThreads) dconv_kernel(const esm_conv_desc a) {
    constexpr int KT = TR ? 2 : K;  // taps per dim (per parity class for transposed)
    constexpr int KDT = D3 ? KT : 1;
    constexpr int TAPS = KDT * KT * KT;
    constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;
    constexpr int TW = 16 * NT;
    constexpr int NC = MT * NT >= 4 ? 1 : 4 / (MT * NT);  // accumulation chains per tile

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(static_cast<int>(threadIdx.x >> 6));
#ifdef ESM_CONV_STAMPS
    unsigned long long st_real = __builtin_amdgcn_s_memrealtime(), st0, st1 = 0, st2 = 0, st3 = 0;
    ESM_STAMP(st0);
#endif
    const int n16 = lane & 15;
    const int kq = lane >> 4;

    const int Hs = TR ? a.Hi : a.Ho;
    const int Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    const int RB = a.hint;  // rows per workgroup (set by the launcher)
    const int tiles_w = (Ws + TW - 1) / TW;
    const int tiles_h = (Hs + RB - 1) / RB;
    // XCD-aware order: workgroups are dealt round-robin to the 8 XCDs (id % 8 share one); remap
    // (bijectively) so each XCD takes a contiguous range of tiles, i.e. a contiguous slab of
    // rows / planes, and the halo rows its neighbours read stay in its own L2
    const unsigned nwg = gridDim.x, orig = blockIdx.x;
    const unsigned q = nwg / 8, r = nwg % 8, xcd = orig % 8;
    unsigned wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
    const int tx = static_cast<int>(wg % tiles_w);
    wg /= tiles_w;
    const int ty = static_cast<int>(wg % tiles_h);
    wg /= tiles_h;
    const int bz = static_cast<int>(wg % (a.B * Ds));  // (batch, plane)
    const int zc = static_cast<int>(wg / (a.B * Ds));  // (cout tile, parity class)
    const int x0 = tx * TW;
    const int b = bz / Ds;
    const int zs = bz - b * Ds;
    const int cls = TR ? zc % NCLS : 0;
    const int cob = (TR ? zc / NCLS : zc) * 16 * MT;
    const int qd = (TR && D3) ? (cls >> 2) & 1 : 0;
    const int qh = TR ? (cls >> 1) & 1 : 0;
    const int qw = TR ? cls & 1 : 0;

    // column part of the B offsets, per kernel column tap and N tile (bytes, kOOB outside)
    unsigned xoff[KT][NT];
#pragma unroll
    for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int xs = x0 + nt * 16 + n16;
            const int xi = TR ? xs + qw - t : xs * S - a.pw + t;
            xoff[t][nt] = (xs < Ws && xi >= 0 && xi < a.Wi) ? 4u * xi : kOOB;
        }

    // source spans / channel ranges (kernel arguments: uniform)
    const int c_lo1 = a.src[0].C, c_lo2 = a.src[0].C + a.src[1].C;
    // weights of this parity class through a buffer descriptor: uniform part in soffset
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(a.w + static_cast<long long>(cls) * TAPS * a.cin_pad * a.cout_pad),
        static_cast<short>(0), 4 * TAPS * a.cin_pad * a.cout_pad, 0x00020000);
    const unsigned wlane = 4u * (kq * a.cout_pad + cob + n16);

    // single source (MS = false): its descriptor and strides are fixed for the whole kernel
    const esm_src& s0 = a.src[0];
    const int sc0 = static_cast<int>(s0.sc), sd0 = static_cast<int>(s0.sd), sh0 = static_cast<int>(s0.sh);
    const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<float*>(s0.ptr + b * s0.sb), static_cast<short>(0),
        4 * ((s0.C - 1) * sc0 + (D3 ? (a.Di - 1) * sd0 : 0) + (a.Hi - 1) * sh0 + a.Wi), 0x00020000);

    const EpiConst<MT> ec = conv_epi_const<MT>(a, cob, lane);
    const int y_end = min(Hs, ty * RB + RB);
#ifdef ESM_CONV_STAMPS
    ESM_STAMP(st1);
#endif
    for (int ys = ty * RB + (KS == 1 ? wave : 0); ys < y_end; ys += (KS == 1 ? 4 : 1)) {
        // NC independent accumulation chains per output tile: a v_mfma_f32_16x16x4_f32 issues every
        // 32 cycles but its result feeds the next one only ~40+ cycles later, and few waves per
        // SIMD are in their MFMA phase at once, so one chain per wave leaves the pipe mostly idle
        floatx4 accs[NC][MT][NT];
#pragma unroll
        for (int c = 0; c < NC; ++c)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) accs[c][mt][nt] = floatx4{0.f, 0.f, 0.f, 0.f};
        floatx4 (&acc)[MT][NT] = accs[0];

        // one 16-channel chunk per iteration: per plane of taps (td), every A and B load of the
        // chunk is issued before the first MFMA (no branch in between: channels past Cin read 0
        // through kOOB and meet zero weights, cin_pad being a multiple of 16)
        for (int cc = 0; cc < a.Cin; cc += 16) {
            unsigned vb[CK][KT][NT];  // per-lane B offsets: channel part + column part (kOOB-marked)
            unsigned chk[CK];
            __amdgpu_buffer_rsrc_t rs[CK];
            int sdk[CK], shk[CK];
#pragma unroll
            for (int k = 0; k < CK; ++k) {
                const int c0 = cc + 4 * k;
                if constexpr (!MS) {
                    rs[k] = rs0;
                    sdk[k] = sd0;
                    shk[k] = sh0;
                    const int cl = c0 + kq;
                    chk[k] = cl < a.Cin ? 4u * cl * sc0 : kOOB;
#pragma unroll
                    for (int t = 0; t < KT; ++t)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt) vb[k][t][nt] = chk[k] + xoff[t][nt];
                    continue;
                }
                // the k-step's 4 channels lie in one source (launcher: C_s % 4 == 0 when nsrc > 1)
                const int s = c0 < c_lo1 ? 0 : (c0 < c_lo2 ? 1 : 2);
                const int lo = s == 0 ? 0 : (s == 1 ? c_lo1 : c_lo2);
                const float* sp = s == 0 ? a.src[0].ptr : (s == 1 ? a.src[1].ptr : a.src[2].ptr);
                const int sC = s == 0 ? a.src[0].C : (s == 1 ? a.src[1].C : a.src[2].C);
                const long long sb = s == 0 ? a.src[0].sb : (s == 1 ? a.src[1].sb : a.src[2].sb);
                const int sc = static_cast<int>(s == 0 ? a.src[0].sc : (s == 1 ? a.src[1].sc : a.src[2].sc));
                sdk[k] = static_cast<int>(s == 0 ? a.src[0].sd : (s == 1 ? a.src[1].sd : a.src[2].sd));
                shk[k] = static_cast<int>(s == 0 ? a.src[0].sh : (s == 1 ? a.src[1].sh : a.src[2].sh));
                const int span = 4 * ((sC - 1) * sc + (D3 ? (a.Di - 1) * sdk[k] : 0) + (a.Hi - 1) * shk[k] + a.Wi);
                rs[k] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sp + b * sb), static_cast<short>(0), span,
                                                          0x00020000);
                const int cl = c0 - lo + kq;
                const unsigned choff = (c0 < a.Cin && cl < sC) ? 4u * cl * sc : kOOB;
                chk[k] = choff;
#pragma unroll
                for (int t = 0; t < KT; ++t)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) vb[k][t][nt] = choff + xoff[t][nt];
            }
            const int wchunk = 4 * cc * a.cout_pad;  // byte offset of the chunk's first k row

            if constexpr (KS == 1) {
#pragma unroll 1
                for (int td = 0; td < KDT; ++td) {
                    constexpr int PT = KT * KT;  // taps of one plane
                    float bv[PT][CK][NT];
                    float av[PT][CK][MT];
                    const int zi = D3 ? (TR ? zs + qd - td : zs * S - a.pd + td) : 0;
#pragma unroll
                    for (int th = 0; th < KT; ++th) {
                        const int yi = TR ? ys + qh - th : ys * S - a.ph + th;
                        const bool rok = yi >= 0 && yi < a.Hi && (!D3 || (zi >= 0 && zi < a.Di));
#pragma unroll
                        for (int k = 0; k < CK; ++k) {
                            // an out-of-range row carries kOOB in soffset (gfx950 range-checks
                            // voffset + soffset: scripts/probes/buffer_oob.hip) -> zeros
                            const int roff = rok ? 4 * ((D3 ? zi * sdk[k] : 0) + yi * shk[k]) : static_cast<int>(kOOB);
#pragma unroll
                            for (int tw = 0; tw < KT; ++tw)
#pragma unroll
                                for (int nt = 0; nt < NT; ++nt)
                                    bv[th * KT + tw][k][nt] = buf_load_s(rs[k], vb[k][tw][nt], roff);
                        }
                    }
#pragma unroll
                    for (int t = 0; t < PT; ++t)
#pragma unroll
                        for (int k = 0; k < CK; ++k)
#pragma unroll
                            for (int mt = 0; mt < MT; ++mt)
                                av[t][k][mt] = buf_load_s(wrs, wlane, wchunk + 4 * (((td * PT + t) * a.cin_pad + 4 * k) * a.cout_pad + mt * 16));
                    // every load above the first MFMA: left alone the scheduler sinks each load next
                    // to its use and the wave pays one memory round trip per load (scripts/isa_waits.py)
                    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                    for (int t = 0; t < PT; ++t)
#pragma unroll
                        for (int k = 0; k < CK; ++k)
#pragma unroll
                            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                                for (int nt = 0; nt < NT; ++nt)
                                    accs[(t * CK + k) % NC][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                        av[t][k][mt], bv[t][k][nt], accs[(t * CK + k) % NC][mt][nt], 0, 0, 0);
                }
            } else {
                // K-split: wave w takes taps w, w + 4, ...  The tap loop is unrolled at compile time and
                // every load of the wave's taps is issued before the first MFMA (one memory round trip
                // per chunk); a tap past TAPS reads zeros (kOOB row) against zero weights (past the
                // weight buffer's range)
                constexpr int TPW = (TAPS + KS - 1) / KS;
                float bv[TPW][CK][NT], av[TPW][CK][MT];
#pragma unroll
                for (int tt = 0; tt < TPW; ++tt) {
                    const int tap = wave + tt * KS;
                    const int td = tap / (KT * KT), th = (tap / KT) % KT, tw = tap % KT;
                    const int zi = D3 ? (TR ? zs + qd - td : zs * S - a.pd + td) : 0;
                    const int yi = TR ? ys + qh - th : ys * S - a.ph + th;
                    const bool rok = tap < TAPS && yi >= 0 && yi < a.Hi && (!D3 || (zi >= 0 && zi < a.Di));
                    unsigned xo[NT];
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt) {
                        const int xs = x0 + nt * 16 + n16;
                        const int xi = TR ? xs + qw - tw : xs * S - a.pw + tw;
                        xo[nt] = (xs < Ws && xi >= 0 && xi < a.Wi) ? 4u * xi : kOOB;
                    }
#pragma unroll
                    for (int k = 0; k < CK; ++k) {
                        const int roff = rok ? 4 * ((D3 ? zi * sdk[k] : 0) + yi * shk[k]) : static_cast<int>(kOOB);
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt) bv[tt][k][nt] = buf_load_s(rs[k], chk[k] + xo[nt], roff);
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
                            av[tt][k][mt] = buf_load_s(wrs, wlane, wchunk + 4 * ((tap * a.cin_pad + 4 * k) * a.cout_pad + mt * 16));
                    }
                }
                __builtin_amdgcn_sched_barrier(0);  // all loads issued before the first MFMA
#pragma unroll
                for (int tt = 0; tt < TPW; ++tt)
#pragma unroll
                    for (int k = 0; k < CK; ++k)
#pragma unroll
                        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                            for (int nt = 0; nt < NT; ++nt)
                                accs[(tt * CK + k) % NC][mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    av[tt][k][mt], bv[tt][k][nt], accs[(tt * CK + k) % NC][mt][nt], 0, 0, 0);
            }
        }

#ifdef ESM_CONV_STAMPS
        if (!st2) ESM_STAMP(st2);
#endif
#pragma unroll
        for (int c = 1; c < NC; ++c)  // fixed order (deterministic)
#pragma unroll
            for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) acc[mt][nt] += accs[c][mt][nt];

        if constexpr (KS > 1) {  // fixed-order reduction of the waves' partial sums
            __shared__ float red[(KS - 1) * MT * NT * 4 * 64];
            __syncthreads();
            if (wave > 0) {
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            red[(((wave - 1) * MT + mt) * NT * 4 + nt * 4 + j) * 64 + lane] = acc[mt][nt][j];
            }
            __syncthreads();
            if (wave == 0) {
#pragma unroll
                for (int p = 1; p < KS; ++p)
#pragma unroll
                    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
                            for (int j = 0; j < 4; ++j)
                                acc[mt][nt][j] += red[(((p - 1) * MT + mt) * NT * 4 + nt * 4 + j) * 64 + lane];
            }
            if (wave > 0) continue;
        }
        const int oz = TR ? 2 * zs + qd : zs;
        const int oy = TR ? 2 * ys + qh : ys;
        conv_store_tile<MT, NT>(a, acc, b, oz, oy, x0, Ws, TR, qw, cob, lane, ec);
    }
#ifdef ESM_CONV_STAMPS
    ESM_STAMP(st3);
    if (lane == 0) {
        const unsigned i = blockIdx.x * 4 + wave;  // no atomics: they would serialise the waves
        if (blockIdx.x == 0 && wave == 0) esm_stamp_count = gridDim.x * 4;
        if (i < (1u << 20) / 8) {
            unsigned long long* o = esm_stamps + 8 * i;
            o[0] = st_real;
            o[1] = st0;
            o[2] = st1;
            o[3] = st2;
            o[4] = st3;
            o[5] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID
            o[6] = __builtin_amdgcn_s_memrealtime();
            o[7] = blockIdx.x;
        }
    }
#endif
}

// Whether the direct form can run this layer: every multi-source split on a 4-channel
// boundary, and each source's per-batch span addressable by a 32-bit buffer offset.
// whether a form without `pre` support may run this desc
inline bool no_pre(const esm_conv_desc& a) { return a.pre == nullptr; }

inline bool direct_ok(const esm_conv_desc& a) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    for (int s = 0; s < a.nsrc; ++s) {
        const esm_src& r = a.src[s];
        if (a.nsrc > 1 && (r.C & 3)) return false;
        const long long last = (r.C - 1) * r.sc + (d3 ? (a.Di - 1) * r.sd : 0) + (a.Hi - 1) * r.sh + a.Wi;
        if (4 * last >= kOOB || r.sc > (1 << 28) || r.sh > (1 << 28) || r.sd > (1 << 28)) return false;
    }
    return true;
}

// One buffer window over every source of a (channel-concatenated) conv input: base = the lowest
// source, dl[s] = source s's byte offset from it, span = bytes to the end of the last one (all batch
// items).  A kernel then addresses every source through ONE descriptor, folding a k-step's source
// into its per-lane voffset once (conv_wide.hip's windowed form, measured 0.5-2.4 us faster per S-K
// launch than a descriptor per source).  False when the sources do not fit a window the kOOB marks
// lie beyond (valid offsets < kOOB; two marks sum to 2^31, no wrap) or differ in row stride (one
// soffset per input row for all of them): the kernel then takes a descriptor per source.
inline bool source_window(const esm_conv_desc& a, const float** base, int* span, int (&dl)[ESM_MAX_SRC]) {
    uintptr_t lo = UINTPTR_MAX, hi = 0;
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1;
    for (int i = 0; i < a.nsrc; ++i) {
        const esm_src& r = a.src[i];
        if (r.sh != a.src[0].sh || (d3 && r.sd != a.src[0].sd) || !r.ptr) return false;
        const uintptr_t p = reinterpret_cast<uintptr_t>(r.ptr);
        const long long last = (a.B - 1) * r.sb + (r.C - 1) * r.sc + (d3 ? (a.Di - 1) * r.sd : 0) + (a.Hi - 1) * r.sh + a.Wi;
        if (last < 0 || r.sb < 0 || r.sc < 0) return false;
        const uintptr_t e = p + 4 * static_cast<uintptr_t>(last);
        lo = p < lo ? p : lo;
        hi = e > hi ? e : hi;
    }
    if (hi - lo >= kOOB) return false;
    for (int i = 0; i < ESM_MAX_SRC; ++i) dl[i] = i < a.nsrc ? static_cast<int>(reinterpret_cast<uintptr_t>(a.src[i].ptr) - lo) : 0;
    *base = reinterpret_cast<const float*>(lo);
    *span = static_cast<int>(hi - lo);
    return true;
}

template <bool D3, int K, int S, bool TR, int MT, int NT, int KS>
int launch_direct(const esm_conv_desc& a, hipStream_t s, int rb) {
    constexpr int NCLS = TR ? (D3 ? 8 : 4) : 1;
    const int Hs = TR ? a.Hi : a.Ho, Ws = TR ? a.Wi : a.Wo;
    const int Ds = D3 ? (TR ? a.Di : a.Do) : 1;
    esm_conv_desc d = a;
    d.hint = rb;
    const long long tiles = static_cast<long long>((Ws + 16 * NT - 1) / (16 * NT)) * ((Hs + rb - 1) / rb) * a.B * Ds *
                            ceil_div(a.Cout, 16 * MT) * NCLS;
    if (tiles > 0x7fffffffLL) return arg_error("conv: grid too large");
    dim3 grid(static_cast<unsigned>(tiles));
    // k-steps per 16-channel chunk: narrow inputs (the disparity map, 8-channel features) skip the
    // all-zero k-steps of their padding
    // (multi-source convs are never that narrow); one source takes the MS = false form
    if (a.nsrc > 1)
        hipLaunchKernelGGL((dconv_kernel<D3, K, S, TR, MT, NT, KS, 4, true>), grid, dim3(kDirectThreads), 0, s, d);
    else if (a.Cin <= 4)
        hipLaunchKernelGGL((dconv_kernel<D3, K, S, TR, MT, NT, KS, 1, false>), grid, dim3(kDirectThreads), 0, s, d);
    else if (a.Cin <= 8)
        hipLaunchKernelGGL((dconv_kernel<D3, K, S, TR, MT, NT, KS, 2, false>), grid, dim3(kDirectThreads), 0, s, d);
    else
        hipLaunchKernelGGL((dconv_kernel<D3, K, S, TR, MT, NT, KS, 4, false>), grid, dim3(kDirectThreads), 0, s, d);
    return check_launch("conv(direct)");
}

}  // namespace conv
}  // namespace esm
