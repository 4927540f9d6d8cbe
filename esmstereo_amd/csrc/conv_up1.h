// The hourglasses' decoder step and the 1x1 BasicConv after it in one launch (models/ESMStereo.py:
// 163-175, 221-234): conv3_up / conv2_up (ConvTranspose k4 s2 p1 + BN + GELU), the crop to the skip
// connection's extent, torch.cat with the skip (and, in up_refinement, the image features) and agg_0[0] /
// agg_1[0] (1x1 + BN + GELU).  The transposed conv's output never leaves the registers: its accumulator
// tile (D layout of v_mfma_f32_16x16x4_f32, lane (n, q) holds channels 4q + r of pixel n, r = 0..3) is
// directly the B operand of the 1x1 when the 1x1's k-step r takes the channels {4q + r : q = 0..3}; the
// k-steps over the extra sources take 4 consecutive channels as usual.  Every product is one MFMA
// product and the accumulation order is fixed, so results are deterministic (they differ from the
// two-launch path by fp32 reassociation of the 1x1's sum only; tests hold them to 1e-5 relative).
#pragma once

#include "conv_direct.h"

namespace esm {
namespace conv {

// Operands of the fused 1x1 that do not depend on the transposed conv, for one wave's 16-pixel
// segment: the weights (A: lane (i, q) holds W[out i][k = channel of lane group q]), the output BN,
// and the extra sources' values at this lane's pixel (B).  XB: extra k-steps (4 channels each) the
// instantiation holds; the launcher checks (b.Cin - a.Cout) / 4 <= XB.
template <int XB>
struct Up1Ops {
    float wy[4];
    float wx[XB];
    float s2[4], h2[4];
};

// Weights and BN of the 1x1 (b): k-step r over the transposed conv's Cy channels, k-step cb over the
// extra channels Cy + 4 cb + q.  Loads past Cy / Cin / Cout read 0 (kOOB) and meet zero operands.
template <int XB>
__device__ __forceinline__ void up1_weights(Up1Ops<XB>& u, const esm_conv_desc& b, int Cy, int lane) {
    const int i = lane & 15, q = lane >> 4;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b.w), static_cast<short>(0),
                                                                         4 * b.cin_pad * b.cout_pad, 0x00020000);
    const bool iok = i < b.Cout;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int c = 4 * q + r;
        u.wy[r] = buf_load_s(wrs, (iok && c < Cy) ? 4u * static_cast<unsigned>(c * b.cout_pad + i) : kOOB, 0);
    }
#pragma unroll
    for (int cb = 0; cb < XB; ++cb) {
        const int c = Cy + 4 * cb + q;
        u.wx[cb] = buf_load_s(wrs, (iok && c < b.Cin) ? 4u * static_cast<unsigned>(c * b.cout_pad + i) : kOOB, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {  // (BN present: up1_check)
        const int co = min(4 * q + r, b.Cout - 1);
        u.s2[r] = b.scale[co];
        u.h2[r] = b.shift[co];
    }
}

// The extra sources (b.src[1], b.src[2]; 4-channel aligned split) of batch item bi as buffer resources.
struct Up1Src {
    __amdgpu_buffer_rsrc_t r1, r2;
    int C1, sc1, sd1, sh1, sc2, sd2, sh2;
};

__device__ __forceinline__ Up1Src up1_src(const esm_conv_desc& b, int bi, bool d3) {
    Up1Src s;
    auto rsrc = [&](const esm_src& t) __attribute__((always_inline)) {
        const long long last = (t.C - 1) * t.sc + (d3 ? (b.Di - 1) * t.sd : 0) + (b.Hi - 1) * t.sh + b.Wi;
        return __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(t.ptr + bi * t.sb), static_cast<short>(0),
                                                 static_cast<int>(4 * last), 0x00020000);
    };
    s.r1 = rsrc(b.src[1]);
    s.r2 = b.nsrc > 2 ? rsrc(b.src[2]) : s.r1;
    s.C1 = b.src[1].C;
    s.sc1 = static_cast<int>(b.src[1].sc), s.sd1 = static_cast<int>(b.src[1].sd), s.sh1 = static_cast<int>(b.src[1].sh);
    s.sc2 = b.nsrc > 2 ? static_cast<int>(b.src[2].sc) : s.sc1;
    s.sd2 = b.nsrc > 2 ? static_cast<int>(b.src[2].sd) : s.sd1;
    s.sh2 = b.nsrc > 2 ? static_cast<int>(b.src[2].sh) : s.sh1;
    return s;
}

// B operands of the extra k-steps at output voxel (oz, oy, ox) (per lane; outside b's extent: 0).
template <int XB>
__device__ __forceinline__ void up1_extra(float (&bx)[XB], const Up1Src& s, const esm_conv_desc& b, int Cy, int lane,
                                          int oz, int oy, int ox) {
    const int q = lane >> 4;
    const int Cx = b.Cin - Cy;
    const bool pok = ox < b.Wi && oy < b.Hi && oz < b.Di;
#pragma unroll
    for (int cb = 0; cb < XB; ++cb) {
        const int c = 4 * cb + q;
        const bool second = 4 * cb >= s.C1;  // wave-uniform: the split is 4-channel aligned
        const int cl = second ? c - s.C1 : c;
        const int off = second ? cl * s.sc2 + oz * s.sd2 + oy * s.sh2 + ox : cl * s.sc1 + oz * s.sd1 + oy * s.sh1 + ox;
        const unsigned vo = (pok && c < Cx) ? 4u * static_cast<unsigned>(off) : kOOB;
        bx[cb] = buf_load_s(second ? s.r2 : s.r1, vo, 0);
    }
}

// The same for the output column pair (ox, ox + 1), ox even, as one 8-byte load per k-step (the launcher checks
// that every extra source's rows / channels / batch items start 8-byte aligned and b's width is even).
template <int XB>
__device__ __forceinline__ void up1_extra2(float (&b0)[XB], float (&b1)[XB], const Up1Src& s, const esm_conv_desc& b,
                                           int Cy, int lane, int oz, int oy, int ox) {
    typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
    const int q = lane >> 4;
    const int Cx = b.Cin - Cy;
    const bool pok = ox < b.Wi && oy < b.Hi && oz < b.Di;
#pragma unroll
    for (int cb = 0; cb < XB; ++cb) {
        const int c = 4 * cb + q;
        const bool second = 4 * cb >= s.C1;
        const int cl = second ? c - s.C1 : c;
        const int off = second ? cl * s.sc2 + oz * s.sd2 + oy * s.sh2 + ox : cl * s.sc1 + oz * s.sd1 + oy * s.sh1 + ox;
        const unsigned vo = (pok && c < Cx) ? 4u * static_cast<unsigned>(off) : kOOB;
        const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(second ? s.r2 : s.r1, static_cast<int>(vo), 0, 0);
        b0[cb] = __uint_as_float(v[0]);
        b1[cb] = __uint_as_float(v[1]);
    }
}

// whether up1_extra2 applies: every extra source 8-byte aligned at every (batch, channel, plane, row) start
inline bool up1_pairs_ok(const esm_conv_desc& b) {
    if (b.Wi & 1) return false;
    for (int s = 1; s < b.nsrc; ++s) {
        const esm_src& r = b.src[s];
        if ((reinterpret_cast<uintptr_t>(r.ptr) & 7) || (r.sb & 1) || (r.sc & 1) || (r.sh & 1) || (r.sd & 1)) return false;
    }
    return true;
}

// out[r] = GELU(BN_b(sum_k W[4q + r][k] x[k][pixel n])) for lane (n, q): y[r] holds the transposed conv's
// channel 4q + r (after its BN + GELU), bx the extra channels.  The XB k-steps run unconditionally: those past the
// layer's extra channels meet zero weights and zero inputs (kOOB loads), so no branch splits the MFMA chain.
template <int XB>
__device__ __forceinline__ floatx4 up1_finish(const Up1Ops<XB>& u, const float (&y)[4], const float (&bx)[XB],
                                              floatx4 d /* the 1x1's partial sum `pre`, or 0 */) {
#pragma unroll
    for (int r = 0; r < 4; ++r) d = __builtin_amdgcn_mfma_f32_16x16x4f32(u.wy[r], y[r], d, 0, 0, 0);
#pragma unroll
    for (int cb = 0; cb < XB; ++cb) d = __builtin_amdgcn_mfma_f32_16x16x4f32(u.wx[cb], bx[cb], d, 0, 0, 0);
    floatx4 o;
#pragma unroll
    for (int r = 0; r < 4; ++r) o[r] = gelu_erf(d[r] * u.s2[r] + u.h2[r]);
    return o;
}

// Two cout tiles on both sides (round 6: the L hourglass's conv2_up 40 -> 24 + agg_1.0 48 -> 24): the transposed
// conv's channels 16 mt + 4q + r (tile mt, accumulator row r) feed the 1x1's k-step (mt, r); the 1x1's outputs run
// as two tiles mb.  A operands wy[mb][mt][r] = W_b[16 mb + i][16 mt + 4 q + r], wx[mb][cb] = W_b[16 mb + i][Cy + 4 cb + q].
template <int XB>
struct Up1Ops2 {
    float wy[2][2][4];
    float wx[2][XB];
    float s2[2][4], h2[2][4];
};

template <int XB>
__device__ __forceinline__ void up1_weights2(Up1Ops2<XB>& u, const esm_conv_desc& b, int Cy, int lane) {
    const int i = lane & 15, q = lane >> 4;
    const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(b.w), static_cast<short>(0),
                                                                         4 * b.cin_pad * b.cout_pad, 0x00020000);
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        const int co = 16 * mb + i;
        const bool iok = co < b.Cout;
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int c = 16 * mt + 4 * q + r;
                u.wy[mb][mt][r] = buf_load_s(wrs, (iok && c < Cy) ? 4u * static_cast<unsigned>(c * b.cout_pad + co) : kOOB, 0);
            }
#pragma unroll
        for (int cb = 0; cb < XB; ++cb) {
            const int c = Cy + 4 * cb + q;
            u.wx[mb][cb] = buf_load_s(wrs, (iok && c < b.Cin) ? 4u * static_cast<unsigned>(c * b.cout_pad + co) : kOOB, 0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int cc = min(16 * mb + 4 * q + r, b.Cout - 1);
            u.s2[mb][r] = b.scale[cc];
            u.h2[mb][r] = b.shift[cc];
        }
    }
}

// o[mb][r] = GELU(BN_b(sum_k W[16 mb + 4q + r][k] x[k][pixel n])) for lane (n, q); y[mt][r]: the transposed conv's
// channel 16 mt + 4q + r after its BN + GELU
template <int XB>
__device__ __forceinline__ void up1_finish2(floatx4 (&o)[2], const Up1Ops2<XB>& u, const float (&y)[2][4],
                                            const float (&bx)[XB]) {
#pragma unroll
    for (int mb = 0; mb < 2; ++mb) {
        floatx4 d = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int mt = 0; mt < 2; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) d = __builtin_amdgcn_mfma_f32_16x16x4f32(u.wy[mb][mt][r], y[mt][r], d, 0, 0, 0);
#pragma unroll
        for (int cb = 0; cb < XB; ++cb) d = __builtin_amdgcn_mfma_f32_16x16x4f32(u.wx[mb][cb], bx[cb], d, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[mb][r] = gelu_erf(d[r] * u.s2[mb][r] + u.h2[mb][r]);
    }
}

// Host-side validation of a (transposed conv) + b (1x1 over [a's cropped output, extra sources]); xb_max:
// the extra k-steps the chosen kernel holds.  ESM_OK or ESM_ERR_ARG with the message set.
inline int up1_check(const esm_conv_desc& a, const esm_conv_desc& b, int xb_max, int cout_max = 16) {
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (!a.transposed || a.kh != 4 || a.stride != 2 || a.nsrc != 1) return arg_error("convt_1x1: a must be a k4 s2 transposed conv");
    if (a.act != ESM_ACT_GELU || !a.scale || !a.shift || a.mul || a.res || a.up || a.out2 || a.post_scale != 1.f)
        return arg_error("convt_1x1: a must be a BasicConv (BN + GELU, plain epilogue)");
    if (a.Cout < 1 || a.Cout > cout_max || (a.Cout & 3))
        return arg_error("convt_1x1: a.Cout must be a multiple of 4, <= 16 (<= 32: the tiled form, 3-D, <= 32 extra channels)");
    if (b.transposed || b.kh != 1 || b.kw != 1 || b.kd != 1 || b.stride != 1 || b.ph || b.pw || b.pd)
        return arg_error("convt_1x1: b must be a 1x1 stride-1 conv");
    if (b.act != ESM_ACT_GELU || !b.out || !b.scale || !b.shift || b.mul || b.res || b.up || b.out2 ||
        b.post_scale != 1.f || b.shuffle > 1)
        return arg_error("convt_1x1: b must be a BasicConv (BN + GELU, plain epilogue)");
    if (b.pre && d3) return arg_error("convt_1x1: a partial sum (pre) for the 2-D form only");
    if (b.nsrc < 2 || b.src[0].C != a.Cout || b.Cout < 1 || b.Cout > cout_max || b.B != a.B)
        return arg_error("convt_1x1: b.src[0] must be a's output, b.Cout <= 16 (<= 32: the tiled form)");
    if (b.Hi > a.Ho || b.Wi > a.Wo || b.Di > a.Do || b.Ho != b.Hi || b.Wo != b.Wi || b.Do != b.Di ||
        (d3 ? (b.Di < 1) : (b.Di != 1)))
        return arg_error("convt_1x1: b's extent must be a crop of a's output");
    const int cx = b.Cin - a.Cout;
    for (int s = 1; s < b.nsrc; ++s) {
        const esm_src& r = b.src[s];
        if (!r.ptr || r.C <= 0 || (r.C & 3)) return arg_error("convt_1x1: extra sources need 4-channel multiples");
        const long long last = (r.C - 1) * r.sc + (d3 ? (b.Di - 1) * r.sd : 0) + (b.Hi - 1) * r.sh + b.Wi;
        if (4 * last >= kOOB || r.sc > (1 << 28) || r.sh > (1 << 28) || r.sd > (1 << 28) || r.sc < 0 || r.sh < 0)
            return arg_error("convt_1x1: extra source span beyond 32-bit buffer offsets");
    }
    if (cx < 4 || cx > 4 * xb_max) return arg_error("convt_1x1: too many extra channels for the fused form");
    if (b.cin_pad < b.Cin || b.cout_pad < b.Cout) return arg_error("convt_1x1: bad packed 1x1 weights");
    return ESM_OK;
}

}  // namespace conv
}  // namespace esm
