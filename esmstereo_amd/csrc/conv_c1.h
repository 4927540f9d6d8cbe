// Single-output-channel ConvTranspose (k=4, s=2, p=1), 2-D and 3-D, on the VALU.  Included by
// conv2d.hip / conv3d.hip; conv_impl.h launch_geom routes every Cout == 1 transposed layer here.
//
// Reference layers: the last decoder step of both hourglasses, `conv1_up` of up_refinement
// (models/ESMStereo.py:211-212, ConvTranspose2d C -> 1, its output added to the bilinear-upsampled
// previous disparity at :307,316 and scaled by 4 at :735-745) and of aggregation
// (:149-150, ConvTranspose3d -> 1 cost plane per disparity).
//
// Why not the MFMA forms: with one output channel a 16x16 MFMA tile uses 1/16 of its rows, and
// a per-parity-class grid re-reads every input pixel for each of the 4 (8) classes.  Here a
// workgroup owns a 16 x (16*QW) output tile of one output plane (all parity classes), stages
// the weights and, channel chunk by channel chunk, the CC x 10 x (8*QW+2) input tile it needs
// (x2 planes in 3-D) in LDS, the next chunk's loads in flight during the current chunk's FMAs; every thread computes QW consecutive output
// columns of one row.  The 4 waves take rows of one parity each (rows 2i + p), so a wave's
// weights are LDS broadcasts, laid out [qz][qy][c][qx][tap] for two 16-byte reads per channel;
// input rows are 8-byte aligned for 64-bit reads.  QW = 4 stores one 16-byte vector per thread.
//
// Gather (per dim): output 2m + q takes input m + q - t with kernel index 1 - q + 2t, t = 0, 1
// (the packed weight layout w[cls][tap][cin_pad][cout_pad] of engine.pack_weight: cls = parity
// bits (qd, qh, qw), tap = (td, th, tw)).  Accumulation order per output: plane tap, channel,
// row tap, column tap.
#pragma once

#include "conv_direct.h"
#include "conv_epilogue.h"

namespace esm {
namespace conv {

constexpr int kC1Threads = 256;
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int kC1TH = 16;  // output rows per tile

// Per-thread staging plan of an input tile [NP planes][CC channels][IR rows][IC columns] (element i of
// the tile = thread tid + 256 k): the buffer offset of its element at channel c0 = 0 (kOOB outside the
// input or past the tile), its channel within the chunk and its LDS index, computed once; a chunk of
// channels c0.. is then one buffer_load per element with the channel in the wave-uniform soffset and
// one LDS store (no per-element index arithmetic per chunk: the index math was ~4x the FMAs).
template <int XR, int XN, int NP, int CC, int IR, int IC, int ICP>
struct C1Stage {
    unsigned voff[XR];
    int crel[XR];
    int sidx[XR];
    __device__ __forceinline__ C1Stage(const esm_conv_desc& a, int tid, int iz0, int iy0, int ix0) {
        const esm_src& sr = a.src[0];
#pragma unroll
        for (int k = 0; k < XR; ++k) {
            const int i = tid + k * kC1Threads;
            const int col = i % IC;
            const int row = (i / IC) % IR;
            const int c = (i / (IC * IR)) % CC;
            const int p = i / (IC * IR * CC);
            const int iy = iy0 + row, ix = ix0 + col, iz = iz0 + p;
            const bool ok = i < XN && iy >= 0 && iy < a.Hi && ix >= 0 && ix < a.Wi && (NP == 1 || (iz >= 0 && iz < a.Di));
            voff[k] = ok ? 4u * static_cast<unsigned>(c * sr.sc + (NP > 1 ? iz * sr.sd : 0) + iy * sr.sh + ix) : kOOB;
            crel[k] = i < XN ? c : 1 << 30;
            sidx[k] = ((p * CC + c) * IR + row) * ICP + col;
        }
    }
    // channel chunk c0 of the tile into registers (every load in flight together)
    __device__ __forceinline__ void load(float (&rx)[XR], __amdgpu_buffer_rsrc_t rs, int sc, int c0, int cin) const {
#pragma unroll
        for (int k = 0; k < XR; ++k) rx[k] = buf_load_s(rs, crel[k] < cin - c0 ? voff[k] : kOOB, 4 * c0 * sc);
    }
    __device__ __forceinline__ void store(float* xs, const float (&rx)[XR]) const {
#pragma unroll
        for (int k = 0; k < XR; ++k)
            if (k * kC1Threads + static_cast<int>(threadIdx.x) < XN) xs[sidx[k]] = rx[k];
    }
    // without a branch: the lanes past the tile write to xs[dummy] (a word nothing reads)
    __device__ __forceinline__ void store_all(float* xs, const float (&rx)[XR], int dummy) const {
#pragma unroll
        for (int k = 0; k < XR; ++k) xs[(k + 1) * kC1Threads <= XN || crel[k] < (1 << 30) ? sidx[k] : dummy] = rx[k];
    }
};

// buffer descriptor over one batch item of the single source (range = its last element + 1)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t c1_src_rsrc(const esm_conv_desc& a, int b, bool d3) {
    const esm_src& sr = a.src[0];
    const long long span = (a.Cin - 1) * sr.sc + (d3 ? (a.Di - 1) * sr.sd : 0) + (a.Hi - 1) * sr.sh + a.Wi;
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(sr.ptr + b * sr.sb), static_cast<short>(0),
                                             static_cast<int>(4 * span), 0x00020000);
}

// 2-D: the input tile of all channels (<= 32) and the weights staged with one batch of loads.
template <bool D3, int CP, int QW>
__global__ void __launch_bounds__(kC1Threads) convt_c1_batch_kernel(const esm_conv_desc a) {
    constexpr int TW = 16 * QW;               // output columns per tile
    constexpr int IR = kC1TH / 2 + 2;         // input rows of the tile
    constexpr int IC = TW / 2 + 2;            // input columns of the tile
    constexpr int ICP = (IC + 3) / 4 * 4;     // padded LDS row (16-B aligned rows)
    constexpr int NP = D3 ? 2 : 1;            // input planes per output plane
    constexpr int NQZ = D3 ? 2 : 1;
    constexpr int XN = NP * CP * IR * IC;     // staged input elements
    constexpr int XR = (XN + kC1Threads - 1) / kC1Threads;
    constexpr int WN = NQZ * 2 * CP * 2 * 4 * NP;  // staged weights [qz][qy][c][qx][tz][ty][tx]
    constexpr int WR = (WN + kC1Threads - 1) / kC1Threads;
    constexpr int TAPS = D3 ? 8 : 4;
    __shared__ __attribute__((aligned(16))) float xs[NP][CP][IR][ICP];
    __shared__ __attribute__((aligned(16))) float ws[NQZ][2][CP][2][NP][4];

    const int tid = threadIdx.x;
    const int Ho = a.Ho, Wo = a.Wo, Do = D3 ? a.Do : 1;
    const Blk3 bk = xcd_block((a.hint & kHintXcd) != 0);
    const int Y0 = bk.y * kC1TH, X0 = bk.x * TW;
    const int b = bk.z / Do;
    const int oz = bk.z - b * Do;
    const int qz = D3 ? (oz & 1) : 0;
    const int iz0 = D3 ? (oz >> 1) + qz - 1 : 0;  // input plane of plane tap t = 1 (t = 0: iz0 + 1)
    const int iy0 = Y0 / 2 - 1, ix0 = X0 / 2 - 1;  // input row / column of tile index 0
    // the thread's outputs (row oy, columns ox0 ..): their epilogue operands -- BN scale / shift and the
    // 4 bilinear taps of `up` per column (the refinement's conv1_up adds the upsampled previous
    // disparity) -- are loaded with the staging batch below, not after the FMAs (one round trip less)
    const int oy = Y0 + 2 * (((tid >> 6) >> 1) * 4 + (tid & 63) / 16) + ((tid >> 6) & 1);
    const int ox0 = X0 + QW * ((tid & 63) % 16);
    const float ep_s = a.scale ? a.scale[0] : 1.f, ep_h = a.shift ? a.shift[0] : 0.f;
    constexpr int NU = D3 ? 1 : QW;
    float upv[NU][4], ulx[NU], uly = 0.f;
    if (!D3 && a.up) {
        const float* img = a.up + b * a.ub;
        const float sc = 1.0f / static_cast<float>(a.up_f);
        const int y = oy < Ho ? oy : Ho - 1;
        float sy = sc * (static_cast<float>(y) + 0.5f) - 0.5f;
        sy = sy < 0.f ? 0.f : sy;
        const int y0 = static_cast<int>(sy), y1 = y0 + (y0 < a.up_h - 1 ? 1 : 0);
        uly = sy - static_cast<float>(y0);
#pragma unroll
        for (int j = 0; j < NU; ++j) {
            const int x = ox0 + j < Wo ? ox0 + j : Wo - 1;
            float sx = sc * (static_cast<float>(x) + 0.5f) - 0.5f;
            sx = sx < 0.f ? 0.f : sx;
            const int x0 = static_cast<int>(sx), x1 = x0 + (x0 < a.up_w - 1 ? 1 : 0);
            ulx[j] = sx - static_cast<float>(x0);
            upv[j][0] = img[y0 * a.uh + x0];
            upv[j][1] = img[y0 * a.uh + x1];
            upv[j][2] = img[y1 * a.uh + x0];
            upv[j][3] = img[y1 * a.uh + x1];
        }
    }
    // conv_finish with the prefetched operands (bilinear_at's arithmetic, common.h)
    auto finish = [&](float v, int j) __attribute__((always_inline)) {
        v = a.scale ? v * ep_s + ep_h : v + ep_h;
        v = apply_act(v, a.act);
        if (a.mul) v = v * a.mul[b * a.mb + oy * a.mh + ox0 + j];
        if (a.res) v = v + a.res[b * a.rb + oz * a.rd + oy * a.rh + ox0 + j];
        if (!D3 && a.up) {
            const float ly1 = uly, ly0 = 1.0f - ly1, lx1 = ulx[j], lx0 = 1.0f - lx1;
            v = ly0 * (lx0 * upv[j][0] + lx1 * upv[j][1]) + ly1 * (lx0 * upv[j][2] + lx1 * upv[j][3]) + v;
        }
        return v;
    };
    // ---- stage: every load of the thread in flight together, then the LDS stores
    const C1Stage<XR, XN, NP, CP, IR, IC, ICP> stg(a, tid, iz0, iy0, ix0);
    float rx[XR], rw[WR];
    stg.load(rx, c1_src_rsrc(a, b, D3), static_cast<int>(a.src[0].sc), 0, a.Cin);
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        // LDS index (qz, qy, c, qx, tz, ty, tx) <- packed w[cls = (qz,qy,qx)][tap = (tz,ty,tx)][c][0]
        const int i = tid + k * kC1Threads;
        const int tyx = i & 3;
        const int tz = (i >> 2) % NP;
        const int qx = (i / (4 * NP)) & 1;
        const int c = (i / (8 * NP)) % CP;
        const int qy = (i / (8 * NP * CP)) & 1;
        const int qzz = i / (16 * NP * CP);
        const int cls = D3 ? (qzz << 2 | qy << 1 | qx) : (qy << 1 | qx);
        const int tap = D3 ? (tz << 2 | tyx) : tyx;
        const bool ok = i < WN && c < a.cin_pad;
        const float v = a.w[ok ? ((static_cast<long long>(cls) * TAPS + tap) * a.cin_pad + c) * a.cout_pad : 0];
        rw[k] = ok ? v : 0.f;
    }
    __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
    stg.store(&xs[0][0][0][0], rx);
#pragma unroll
    for (int k = 0; k < WR; ++k) {
        const int i = tid + k * kC1Threads;
        if (i < WN) (&ws[0][0][0][0][0][0])[i] = rw[k];
    }
    __syncthreads();

    // ---- thread: output row Y0 + r (wave w: rows of parity w & 1), columns X0 + QW*g ...
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int qy = wave & 1;
    const int g = lane % 16;
    const int r = 2 * ((wave >> 1) * 4 + lane / 16) + qy;
    const int lr = r / 2 + 1 + qy;  // tile row of input m + q (row tap t = 0); t = 1 is lr - 1
    const int lc = QW / 2 * g;      // first tile column the thread reads (QW = 1: see below)
    constexpr int NV = QW / 2 + 2;  // tile columns per row the thread reads
    f32x2 acc2[QW / 2];
#pragma unroll
    for (int j = 0; j < QW / 2; ++j) acc2[j] = f32x2{0.f, 0.f};
#pragma unroll
    for (int tz = 0; tz < NP; ++tz) {
        const int p = D3 ? 1 - tz : 0;  // plane tap t = tz sits at tile plane 1 - t
#pragma unroll 4
        for (int c = 0; c < CP; ++c) {
            float v[2][NV];
#pragma unroll
            for (int ty = 0; ty < 2; ++ty)
#pragma unroll
                for (int j = 0; j < NV; ++j) v[ty][j] = xs[p][c][lr - ty][lc + j];
            // output columns j = 2 jp (qx = 0) and 2 jp + 1 (qx = 1) as one packed pair (v_pk_fma_f32): per
            // element the same product and sum order as one column at a time.  Input m + qx - tx of output
            // column QW*g + j sits at tile column lc + 1 + (j >> 1) + qx - tx
#pragma unroll
            for (int jp = 0; jp < QW / 2; ++jp)
#pragma unroll
                for (int ty = 0; ty < 2; ++ty)
#pragma unroll
                    for (int tx = 0; tx < 2; ++tx) {
                        const f32x2 w2 = {ws[qz][qy][c][0][tz][ty * 2 + tx], ws[qz][qy][c][1][tz][ty * 2 + tx]};
                        const f32x2 v2 = {v[ty][1 + jp - tx], v[ty][2 + jp - tx]};
                        acc2[jp] = __builtin_elementwise_fma(w2, v2, acc2[jp]);
                    }
        }
    }
    float acc[QW];
#pragma unroll
    for (int j = 0; j < QW; ++j) acc[j] = acc2[j >> 1][j & 1];
    if (oy >= Ho) return;
    const long long o = b * a.ob + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox0;
    if constexpr (QW == 4) {
        const bool plain = !a.mul && !a.res && !a.out2;
        if (plain && ox0 + 3 < Wo && ((o | a.oh) & 3) == 0 && (reinterpret_cast<uintptr_t>(a.out) & 15) == 0) {
            floatx4 v4;
            v4.x = finish(acc[0], 0) * a.post_scale;
            v4.y = finish(acc[1], 1) * a.post_scale;
            v4.z = finish(acc[2], 2) * a.post_scale;
            v4.w = finish(acc[3], 3) * a.post_scale;
            *reinterpret_cast<floatx4*>(a.out + o) = v4;
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < QW; ++j)
        if (ox0 + j < Wo) conv_put(a, finish(acc[j], j), b, 0, oz, oy, ox0 + j);
}

// 3-D: channel chunks of CC, the next chunk's loads in flight during the current one's FMAs.
template <bool D3, int CC, int QW>
__global__ void __launch_bounds__(kC1Threads) convt_c1_kernel(const esm_conv_desc a) {
    constexpr int TW = 16 * QW;               // output columns per tile
    constexpr int IR = kC1TH / 2 + 2;         // input rows of the tile
    constexpr int IC = TW / 2 + 2;            // input columns of the tile
    constexpr int ICP = (IC + 3) / 4 * 4;     // padded LDS row (16-B aligned rows)
    constexpr int NP = D3 ? 2 : 1;            // input planes per output plane
    constexpr int NQZ = D3 ? 2 : 1;
    constexpr int CPM = D3 ? 32 : CC;         // channel capacity of the weight table (2-D: one chunk)
    constexpr int XN = NP * CC * IR * IC;     // staged input elements of one channel chunk
    constexpr int XR = (XN + kC1Threads - 1) / kC1Threads;
    constexpr int WN = NQZ * 2 * CPM * 2 * 4 * NP;  // staged weights [qz][qy][c][qx][tz][ty][tx]
    constexpr int WR = (WN + kC1Threads - 1) / kC1Threads;
    constexpr int TAPS = D3 ? 8 : 4;
    __shared__ __attribute__((aligned(16))) float xs[NP][CC][IR][ICP];
    __shared__ __attribute__((aligned(16))) float ws[NQZ][2][CPM][2][NP][4];

    const int tid = threadIdx.x;
    const int Ho = a.Ho, Wo = a.Wo, Do = D3 ? a.Do : 1;
    const Blk3 bk = xcd_block((a.hint & kHintXcd) != 0);
    const int Y0 = bk.y * kC1TH, X0 = bk.x * TW;
    const int b = bk.z / Do;
    const int oz = bk.z - b * Do;
    const int qz = D3 ? (oz & 1) : 0;
    const int iz0 = D3 ? (oz >> 1) + qz - 1 : 0;  // input plane of plane tap t = 1 (t = 0: iz0 + 1)
    const int iy0 = Y0 / 2 - 1, ix0 = X0 / 2 - 1;  // input row / column of tile index 0
    const int nch = (a.Cin + CC - 1) / CC;
    const int sc = static_cast<int>(a.src[0].sc);
    const __amdgpu_buffer_rsrc_t rs = c1_src_rsrc(a, b, D3);
    const C1Stage<XR, XN, NP, CC, IR, IC, ICP> stg(a, tid, iz0, iy0, ix0);
    float rx[XR];
    stg.load(rx, rs, sc, 0, a.Cin);
    {
        float rw[WR];
#pragma unroll
        for (int k = 0; k < WR; ++k) {
            // LDS index (qz, qy, c, qx, tz, ty, tx) <- packed w[cls = (qz,qy,qx)][tap = (tz,ty,tx)][c][0]
            const int i = tid + k * kC1Threads;
            const int tyx = i & 3;
            const int tz = (i >> 2) % NP;
            const int qx = (i / (4 * NP)) & 1;
            const int c = (i / (8 * NP)) % CPM;
            const int qy = (i / (8 * NP * CPM)) & 1;
            const int qzz = i / (16 * NP * CPM);
            const int cls = D3 ? (qzz << 2 | qy << 1 | qx) : (qy << 1 | qx);
            const int tap = D3 ? (tz << 2 | tyx) : tyx;
            const bool ok = i < WN && c < a.Cin;
            const float v = a.w[ok ? ((static_cast<long long>(cls) * TAPS + tap) * a.cin_pad + c) * a.cout_pad : 0];
            rw[k] = ok ? v : 0.f;
        }
        __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
        for (int k = 0; k < WR; ++k) {
            const int i = tid + k * kC1Threads;
            if (i < WN) (&ws[0][0][0][0][0][0])[i] = rw[k];
        }
    }

    // ---- thread: output row Y0 + r (wave w: rows of parity w & 1), columns X0 + QW*g ...
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
    const int lane = tid & 63;
    const int qy = wave & 1;
    const int g = lane % 16;
    const int r = 2 * ((wave >> 1) * 4 + lane / 16) + qy;
    const int oy = Y0 + r;
    const int lr = r / 2 + 1 + qy;  // tile row of input m + q (row tap t = 0); t = 1 is lr - 1
    const int lc = QW / 2 * g;      // first tile column the thread reads (QW = 1: see below)
    constexpr int NV = QW / 2 + 2;  // tile columns per row the thread reads
    f32x2 acc2[QW / 2];
#pragma unroll
    for (int j = 0; j < QW / 2; ++j) acc2[j] = f32x2{0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
        if (ch) __syncthreads();  // the previous chunk's reads of xs are done
        stg.store(&xs[0][0][0][0], rx);
        __syncthreads();
        if (ch + 1 < nch) stg.load(rx, rs, sc, (ch + 1) * CC, a.Cin);  // next chunk in flight during this one's FMAs
#pragma unroll
        for (int tz = 0; tz < NP; ++tz) {
            const int p = D3 ? 1 - tz : 0;  // plane tap t = tz sits at tile plane 1 - t
#pragma unroll 4
            for (int c = 0; c < CC; ++c) {
                const int cw = ch * CC + c;
                float v[2][NV];
#pragma unroll
                for (int ty = 0; ty < 2; ++ty)
#pragma unroll
                    for (int j = 0; j < NV; ++j) v[ty][j] = xs[p][c][lr - ty][lc + j];
                // the packed column pairs of convt_c1_batch_kernel
#pragma unroll
                for (int jp = 0; jp < QW / 2; ++jp)
#pragma unroll
                    for (int ty = 0; ty < 2; ++ty)
#pragma unroll
                        for (int tx = 0; tx < 2; ++tx) {
                            const f32x2 w2 = {ws[qz][qy][cw][0][tz][ty * 2 + tx], ws[qz][qy][cw][1][tz][ty * 2 + tx]};
                            const f32x2 v2 = {v[ty][1 + jp - tx], v[ty][2 + jp - tx]};
                            acc2[jp] = __builtin_elementwise_fma(w2, v2, acc2[jp]);
                        }
            }
        }
    }
    float acc[QW];
#pragma unroll
    for (int j = 0; j < QW; ++j) acc[j] = acc2[j >> 1][j & 1];
    if (oy >= Ho) return;
    const int ox0 = X0 + QW * g;
    const long long o = b * a.ob + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox0;
    if constexpr (QW == 4) {
        const bool plain = !a.mul && !a.res && !a.out2;
        if (plain && ox0 + 3 < Wo && ((o | a.oh) & 3) == 0 && (reinterpret_cast<uintptr_t>(a.out) & 15) == 0) {
            floatx4 v4;
            v4.x = conv_finish(a, acc[0], b, 0, oz, oy, ox0 + 0) * a.post_scale;
            v4.y = conv_finish(a, acc[1], b, 0, oz, oy, ox0 + 1) * a.post_scale;
            v4.z = conv_finish(a, acc[2], b, 0, oz, oy, ox0 + 2) * a.post_scale;
            v4.w = conv_finish(a, acc[3], b, 0, oz, oy, ox0 + 3) * a.post_scale;
            *reinterpret_cast<floatx4*>(a.out + o) = v4;
            return;
        }
    }
#pragma unroll
    for (int j = 0; j < QW; ++j)
        if (ox0 + j < Wo) conv_put(a, conv_finish(a, acc[j], b, 0, oz, oy, ox0 + j), b, 0, oz, oy, ox0 + j);
}

// 3-D, register-blocked over the parity classes: a thread owns MX = 4 consecutive input-grid
// positions m (along x) of one input-grid row and plane and computes all 8 parity classes of each, the
// 2 x 2 x 8 output block (2m + q per dim).  Every class of m reads input m + p, p = q - t in {-1, 0, 1}
// per dim, so per channel the thread reads each of the 3 x 3 input rows around its positions once (6
// values: one 16-byte and one 8-byte LDS read) and does 256 FMAs with them and 64 wave-uniform weights
// (16-byte LDS reads; the per-class form above: 16 FMAs per 8 reads), as 128 v_pk_fma_f32 over the x-parity pairs.  A workgroup (16 x 16 threads)
// owns a 16-row x 64-column input-grid tile of one plane: it stages the 3 planes x 18 rows x 68 columns
// the tile reads, one channel per chunk, double-buffered (one barrier per chunk, the next chunk's loads
// in flight during this one's FMAs), and every weight of the layer once, as [c][qz][qy][tz][ty][qx][tx].
// Each (qz, qy) class pair of a thread is 8 consecutive output columns: two 16-byte stores.
// Accumulation order per output: channel, plane tap, row tap, column tap.
constexpr int kC2TY = 16, kC2TX = 16, kC2MX = 4;

template <bool D3>  // (3-D only; a template so that both conv2d.hip and conv3d.hip may include it)
__global__ void __launch_bounds__(kC1Threads) convt_c1v2_kernel(const esm_conv_desc a) {
    static_assert(D3, "the register-blocked ConvT form is 3-D");
    constexpr int MXW = kC2TX * kC2MX;            // input-grid columns per tile (64)
    constexpr int IR = kC2TY + 2, IC = MXW + 4;   // staged rows / columns (m0 - 1 .. m0 + 66)
    constexpr int NP = 3, CC = 1;
    constexpr int XN = NP * CC * IR * IC;
    constexpr int XR = (XN + kC1Threads - 1) / kC1Threads;
    constexpr int WCAP = 32 * 64;
    constexpr int XS = NP * IR * IC + 4;          // one staged chunk + the staging's dummy word (XS - 1)
    __shared__ __attribute__((aligned(16))) float xs[2][XS];
    __shared__ __attribute__((aligned(16))) float ws[WCAP];

    const int tid = threadIdx.x;
    const int Di = a.Di, Hi = a.Hi, Wi = a.Wi;
    const Blk3 bk = xcd_block((a.hint & kHintXcd) != 0);
    const int my0 = bk.y * kC2TY, mx0 = bk.x * MXW;
    const int b = bk.z / Di;
    const int mz = bk.z - b * Di;
    const int sc = static_cast<int>(a.src[0].sc);
    const __amdgpu_buffer_rsrc_t rs = c1_src_rsrc(a, b, true);
    const C1Stage<XR, XN, NP, CC, IR, IC, IC> stg(a, tid, mz - 1, my0 - 1, mx0 - 1);
    const int nch = a.Cin;
    float rx[XR];
    stg.load(rx, rs, sc, 0, a.Cin);
    {
        constexpr int WR = WCAP / kC1Threads;
        float rw[WR];
#pragma unroll
        for (int k = 0; k < WR; ++k) {  // ws[c][qz][qy][tz][ty][tx][qx] <- packed w[cls = (qz,qy,qx)][tap = (tz,ty,tx)][c][0]
            const int i = tid + k * kC1Threads;
            const int qx = i & 1, tx = (i >> 1) & 1, ty = (i >> 2) & 1, tz = (i >> 3) & 1, qy = (i >> 4) & 1,
                      qz = (i >> 5) & 1, c = i >> 6;
            const int cls = qz << 2 | qy << 1 | qx, tap = tz << 2 | ty << 1 | tx;
            const bool ok = c < a.Cin;
            const float v = a.w[ok ? ((static_cast<long long>(cls) * 8 + tap) * a.cin_pad + c) * a.cout_pad : 0];
            rw[k] = ok ? v : 0.f;
        }
        __builtin_amdgcn_sched_barrier(0);  // every load issued before the first LDS store
#pragma unroll
        for (int k = 0; k < WR; ++k) ws[tid + k * kC1Threads] = rw[k];
    }
    stg.store_all(&xs[0][0], rx, XS - 1);
    __syncthreads();

    const int ty = tid / kC2TX, tx = tid % kC2TX;
    // acc[qz][qy][j] = the qx pair of outputs (2 mz + qz, 2 (my0 + ty) + qy, 2 (mx0 + 4 tx + j) + {0, 1}), one
    // v_pk_fma_f32 per (j, tx): (w[qx = 0][tx], w[qx = 1][tx]) x (x[m_j - tx], x[m_j + 1 - tx])
    f32x2 acc[2][2][kC2MX];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
            for (int j = 0; j < kC2MX; ++j) acc[i][k][j] = f32x2{0.f, 0.f};
    for (int ch = 0; ch < nch; ++ch) {
        const int buf = ch & 1;
        // unconditional: past the last channel the loads return zeros into a buffer nothing reads, and the
        // loop body stays one block (a conditional store let the FMAs sink below it, behind its waits)
        stg.load(rx, rs, sc, ch + 1, a.Cin);
        __builtin_amdgcn_sched_barrier(0);  // the next chunk's loads stay ahead of this chunk's FMAs
        const float* wc = ws + ch * 64;
#pragma unroll
        for (int pz = 0; pz < 3; ++pz)
#pragma unroll
            for (int py = 0; py < 3; ++py) {
                // input row m_y + py - 1 of plane m_z + pz - 1, columns m0 - 1 .. m0 + 4 (m0 = mx0 + 4 tx)
                const float* row = &xs[buf][(pz * IR + ty + py) * IC + kC2MX * tx];
                // the column pairs the packed FMAs take, each in an aligned register pair: x[m0 - 1 + 2i, + 1]
                // (16- and 8-byte reads) and x[m0 + 2i, + 1] (the same row one column on, 4-byte aligned)
                const floatx4 r4 = *reinterpret_cast<const floatx4*>(row);
                const f32x2 e0 = {r4[0], r4[1]}, e1 = {r4[2], r4[3]};
                const f32x2 e2 = *reinterpret_cast<const f32x2*>(row + 4);
                f32x2 o0, o1;
                o0.x = row[1];
                o0.y = row[2];
                o1.x = row[3];
                o1.y = row[4];
                // pair for (j, tx): columns m_j - tx, m_j + 1 - tx, i.e. from x[m0 - 1 + (j + 1 - tx)]
                const f32x2 pr[5] = {e0, o0, e1, o1, e2};  // pr[k] starts at column m0 - 1 + k
#pragma unroll
                for (int qz = 0; qz < 2; ++qz) {
                    const int tz = qz - pz + 1;  // input plane m + q - t
                    if (tz < 0 || tz > 1) continue;
#pragma unroll
                    for (int qy = 0; qy < 2; ++qy) {
                        const int tyy = qy - py + 1;
                        if (tyy < 0 || tyy > 1) continue;
                        const floatx4 w4 = *reinterpret_cast<const floatx4*>(wc + (((qz * 2 + qy) * 2 + tz) * 2 + tyy) * 4);
#pragma unroll
                        for (int txx = 0; txx < 2; ++txx) {
                            const f32x2 w2 = {w4[2 * txx], w4[2 * txx + 1]};  // (qx = 0, qx = 1) at this tx
#pragma unroll
                            for (int j = 0; j < kC2MX; ++j)  // inputs m_j + qx - tx: pair pr[j + 1 - tx]
                                acc[qz][qy][j] = __builtin_elementwise_fma(w2, pr[j + 1 - txx], acc[qz][qy][j]);
                        }
                    }
                }
                // one input row (and its weights) live at a time: left to itself the scheduler issues every
                // LDS read of the channel first (118 values live, 216 VGPRs)
                __builtin_amdgcn_sched_barrier(0);
            }
        // and the next chunk's LDS stores after this chunk's FMAs (moved above them, their waits for the
        // global loads put a full memory latency before the FMAs of every chunk)
        __builtin_amdgcn_sched_barrier(0);
        stg.store_all(&xs[buf ^ 1][0], rx, XS - 1);
        __syncthreads();
    }

    const int my = my0 + ty, m0 = mx0 + kC2MX * tx;
    if (my >= Hi || m0 >= Wi) return;
    const bool plain = !a.mul && !a.res && !a.out2;
    const bool vec = plain && m0 + kC2MX <= Wi && (a.oh & 3) == 0 && (a.od & 3) == 0 && (a.ob & 3) == 0 &&
                     (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;
    const float ep_s = a.scale ? a.scale[0] : 1.f, ep_h = a.shift ? a.shift[0] : 0.f;
#pragma unroll
    for (int qz = 0; qz < 2; ++qz)
#pragma unroll
        for (int qy = 0; qy < 2; ++qy) {
            const int oz = 2 * mz + qz, oy = 2 * my + qy, ox0 = 2 * m0;
            const long long o = b * a.ob + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox0;
            if (vec) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    floatx4 v4;
#pragma unroll
                    for (int e = 0; e < 4; ++e) {
                        float t = acc[qz][qy][2 * h + (e >> 1)][e & 1];
                        t = a.scale ? t * ep_s + ep_h : t + ep_h;
                        v4[e] = apply_act(t, a.act) * a.post_scale;
                    }
                    *reinterpret_cast<floatx4*>(a.out + o + 4 * h) = v4;
                }
            } else {
#pragma unroll
                for (int e = 0; e < 2 * kC2MX; ++e)
                    if (m0 + (e >> 1) < Wi)
                        conv_put(a, conv_finish(a, acc[qz][qy][e >> 1][e & 1], b, 0, oz, oy, ox0 + e), b, 0, oz, oy,
                                 ox0 + e);
            }
        }
}

// Whether the VALU form takes this layer: transposed k4 s2 p1, one output channel, one source,
// at most 32 input channels.
inline bool convt_c1_ok(const esm_conv_desc& a) {
    return a.transposed && a.Cout == 1 && a.nsrc == 1 && a.Cin <= 32 && a.shuffle <= 1;
}

template <bool D3, int QW>
int launch_convt_c1_q(const esm_conv_desc& a, hipStream_t s) {
    const int Do = D3 ? a.Do : 1;
    dim3 grid(ceil_div(a.Wo, 16 * QW), ceil_div(a.Ho, kC1TH), static_cast<unsigned>(a.B) * Do);
    if (grid.y > 65535u || grid.z > 65535u) return arg_error("conv: grid too large");
    // 3-D: channel chunks of 8 (two input planes per output plane); 2-D: every channel in one
    // batch (the chunked kernel with one chunk measured 1.8 us slower at S-K ref4x.conv1_up)
    if constexpr (D3)
        hipLaunchKernelGGL((convt_c1_kernel<D3, 8, QW>), grid, dim3(kC1Threads), 0, s, a);
    else if (a.Cin <= 16)
        hipLaunchKernelGGL((convt_c1_batch_kernel<D3, 16, QW>), grid, dim3(kC1Threads), 0, s, a);
    else
        hipLaunchKernelGGL((convt_c1_batch_kernel<D3, 32, QW>), grid, dim3(kC1Threads), 0, s, a);
    return check_launch("conv(c1 transposed)");
}

// 64-column tiles (one 16-B store per thread) when they give the chip at least ~one workgroup
// per CU, else 32-column tiles (twice the workgroups for the small hourglass outputs).
template <bool D3>
int launch_convt_c1(const esm_conv_desc& a, hipStream_t s) {
    // 3-D: the register-blocked form unless bits 26-27 of the hint ask for the per-class form (A/B)
    if constexpr (D3) {
        if (((a.hint >> 26) & 3) != 1) {
            const dim3 grid(ceil_div(a.Wi, kC2TX * kC2MX), ceil_div(a.Hi, kC2TY), static_cast<unsigned>(a.B) * a.Di);
            if (grid.y > 65535u || grid.z > 65535u) return arg_error("conv: grid too large");
            hipLaunchKernelGGL((convt_c1v2_kernel<true>), grid, dim3(kC1Threads), 0, s, a);
            return check_launch("conv(c1 transposed, blocked)");
        }
    }
    const long long wg64 = static_cast<long long>(ceil_div(a.Wo, 64)) * ceil_div(a.Ho, kC1TH) * a.B * (D3 ? a.Do : 1);
    return wg64 >= 256 ? launch_convt_c1_q<D3, 4>(a, s) : launch_convt_c1_q<D3, 2>(a, s);
}

}  // namespace conv
}  // namespace esm
