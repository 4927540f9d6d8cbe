// Fused conv epilogue shared by the LDS-staged (conv_impl.h) and direct-load (conv_direct.h)
// implicit-GEMM kernels: BN scale/shift, activation, `* mul`, `+ res`, `+ bilinear(up)`,
// `* post_scale` (+ second copy), PixelShuffle remap.  Reference order: BasicConv
// (models/submodule.py:33-38), `* att` (models/ESMStereo.py:703), residual adds
// (models/shufflemixer.py:130-131), upsample + add (models/ESMStereo.py:307,316),
// PixelShuffle + SiLU (models/ESMStereo.py:265-268), `* 4` (:735-745).
#pragma once

#include "common.h"

namespace esm {
namespace conv {

typedef float floatx4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float conv_finish(const esm_conv_desc& a, float v, int b, int co, int oz, int oy, int ox) {
    const float scl = a.scale ? a.scale[co] : 1.f;
    const float shf = a.shift ? a.shift[co] : 0.f;
    v = a.scale ? v * scl + shf : v + shf;
    v = apply_act(v, a.act);
    if (a.mul) v = v * a.mul[b * a.mb + co * a.mc + oy * a.mh + ox];
    if (a.res) v = v + a.res[b * a.rb + co * a.rc + oz * a.rd + oy * a.rh + ox];
    if (a.up) v = bilinear_at(a.up + b * a.ub, a.up_h, a.up_w, a.uh, a.up_f, oy, ox) + v;
    return v;
}

__device__ __forceinline__ void conv_put(const esm_conv_desc& a, float v, int b, int co, int oz, int oy, int ox) {
    const long long o = b * a.ob + co * a.oc + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh + ox;
    a.out[o] = v * a.post_scale;
    if (a.out2) a.out2[o] = v * a.post_scale2;
}

// Per-lane BN scale / shift of the 4 couts a lane holds in each M tile (loaded once per
// workgroup: a lane's couts do not change across its rows).
template <int MT>
struct EpiConst {
    float scl[MT][4];
    float shf[MT][4];
};

template <int MT>
__device__ __forceinline__ EpiConst<MT> conv_epi_const(const esm_conv_desc& a, int cob, int lane) {
    EpiConst<MT> e;
    const int kq = lane >> 4;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int co = min(cob + mt * 16 + kq * 4 + j, a.Cout - 1);
            e.scl[mt][j] = a.scale ? a.scale[co] : 1.f;
            e.shf[mt][j] = a.shift ? a.shift[co] : 0.f;
        }
    return e;
}

// Store one wave's MFMA tile: lane l holds couts cob + mt*16 + (l>>4)*4 + j of sub-grid pixel
// xs0 + nt*16 + (l&15).  Transposed convs map sub-grid x to output 2x + qw.
// Only sub-grid columns in [xmin, Ws) are stored (xmin > xs0: tiles whose edge lanes are halo).
template <int MT, int NT>
__device__ __forceinline__ void conv_store_tile(const esm_conv_desc& a, const floatx4 (&acc)[MT][NT], int b, int oz,
                                                int oy, int xs0, int Ws, bool tr, int qw, int cob, int lane,
                                                const EpiConst<MT>& ec, int xmin = 0) {
    const int n16 = lane & 15, kq = lane >> 4;
    const int r = a.shuffle > 1 ? a.shuffle : 1;
    if (r == 1 && !a.mul && !a.res && !a.up && !a.out2) {
        // plain BN + activation + scale: one base address per (tile, lane), stepped by the cout stride
        const long long rowb = b * a.ob + static_cast<long long>(oz) * a.od + static_cast<long long>(oy) * a.oh;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int cq = cob + mt * 16 + kq * 4;
#pragma unroll
            for (int nt = 0; nt < NT; ++nt) {
                const int xsub = xs0 + nt * 16 + n16;
                if (xsub >= Ws || xsub < xmin) continue;
                const int ox = tr ? 2 * xsub + qw : xsub;
                float* o = a.out + rowb + cq * a.oc + ox;
#pragma unroll
                for (int j = 0; j < 4; ++j) {
                    if (cq + j >= a.Cout) break;
                    float v = a.scale ? acc[mt][nt][j] * ec.scl[mt][j] + ec.shf[mt][j] : acc[mt][nt][j] + ec.shf[mt][j];
                    o[j * a.oc] = apply_act(v, a.act) * a.post_scale;
                }
            }
        }
        return;
    }
    const bool vec4 = r == 4 && !a.out2 && ((a.ob | a.oc | a.oh) & 3) == 0 &&
                      (reinterpret_cast<uintptr_t>(a.out) & 15) == 0;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int cq = cob + mt * 16 + kq * 4;  // first of this lane's 4 couts
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
            const int xsub = xs0 + nt * 16 + n16;
            if (xsub >= Ws || xsub < xmin) continue;
            const int ox = tr ? 2 * xsub + qw : xsub;
            if (vec4 && cq + 3 < a.Cout) {
                // PixelShuffle(4): couts cq..cq+3 are dx = 0..3 of one (channel, dy) -> one 16-B store
                floatx4 v4;
                v4.x = conv_finish(a, acc[mt][nt][0], b, cq + 0, oz, oy, ox) * a.post_scale;
                v4.y = conv_finish(a, acc[mt][nt][1], b, cq + 1, oz, oy, ox) * a.post_scale;
                v4.z = conv_finish(a, acc[mt][nt][2], b, cq + 2, oz, oy, ox) * a.post_scale;
                v4.w = conv_finish(a, acc[mt][nt][3], b, cq + 3, oz, oy, ox) * a.post_scale;
                const int cs = cq / 16, dy = (cq / 4) & 3;
                const long long o = b * a.ob + cs * a.oc + static_cast<long long>(oy * 4 + dy) * a.oh + ox * 4;
                *reinterpret_cast<floatx4*>(a.out + o) = v4;
                continue;
            }
            // rolled: one copy of the (long) general epilogue body instead of four live at once
#pragma unroll 1
            for (int j = 0; j < 4; ++j) {
                const int co = cq + j;
                if (co >= a.Cout) continue;
                const float v = conv_finish(a, acc[mt][nt][j], b, co, oz, oy, ox);
                if (r > 1) {
                    const int cs = co / (r * r);
                    const int rem = co - cs * r * r;
                    const int yy = oy * r + rem / r;
                    const int xx = ox * r + (rem - (rem / r) * r);
                    const long long o = b * a.ob + cs * a.oc + static_cast<long long>(yy) * a.oh + xx;
                    a.out[o] = v * a.post_scale;
                    if (a.out2) a.out2[o] = v * a.post_scale2;
                } else {
                    conv_put(a, v, b, co, oz, oy, ox);
                }
            }
        }
    }
}

}  // namespace conv
}  // namespace esm
