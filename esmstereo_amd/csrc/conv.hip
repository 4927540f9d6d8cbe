// esm_conv_f32: descriptor validation (host side, before anything touches the GPU) and
// dispatch to the 2-D / 3-D implicit-GEMM instantiations (conv2d.hip, conv3d.hip).
#include "common.h"

namespace esm {

int launch_conv2d(const esm_conv_desc& a, hipStream_t s);
int launch_conv3d(const esm_conv_desc& a, hipStream_t s);
namespace conv {
bool stem_ok(const esm_conv_desc& a);                    // conv_stem.hip
bool stem_auto(const esm_conv_desc& a);                  // conv_stem.hip
int launch_stem(const esm_conv_desc& a, hipStream_t s);  // conv_stem.hip
bool c1in_ok(const esm_conv_desc& a);                    // conv_stem.hip
int launch_c1in(const esm_conv_desc& a, hipStream_t s);  // conv_stem.hip
bool small_ok(const esm_conv_desc& a);                   // conv_small.hip
bool small_auto(const esm_conv_desc& a);                 // conv_small.hip
int launch_small(const esm_conv_desc& a, hipStream_t s);  // conv_small.hip
bool wide_ok(const esm_conv_desc& a);                    // conv_wide.hip
int launch_wide(const esm_conv_desc& a, hipStream_t s);  // conv_wide.hip
bool wide3_ok(const esm_conv_desc& a);                    // conv_wide3.hip
int launch_wide3(const esm_conv_desc& a, hipStream_t s);  // conv_wide3.hip
bool widet_ok(const esm_conv_desc& a);                    // conv_widet.hip
int launch_widet(const esm_conv_desc& a, hipStream_t s);  // conv_widet.hip
bool tile3_auto(const esm_conv_desc& a);                 // conv_tile3.hip
int launch_tile3(const esm_conv_desc& a, hipStream_t s);  // conv_tile3.hip
bool tile2_auto(const esm_conv_desc& a);                 // conv_tile3.hip
bool tile2_ok(const esm_conv_desc& a);                   // conv_tile3.hip
int launch_tile2(const esm_conv_desc& a, hipStream_t s);  // conv_tile3.hip
bool pw_ok(const esm_conv_desc& a);                       // conv_pw.hip
bool pw_auto(const esm_conv_desc& a);                     // conv_pw.hip
int launch_pw(const esm_conv_desc& a, hipStream_t s);     // conv_pw.hip
}  // namespace conv

constexpr int kHintStem = 1 << 17;    // force the 16-block narrow-output form (conv_stem.hip)
constexpr int kHintNoStem = 1 << 18;  // automatic choice among the other forms
constexpr int kHintC1in = 1 << 20;     // force the VALU single-input-channel form (conv_stem.hip)
constexpr int kHintSmall = 1 << 21;    // lean K-split form for latency-bound layers (conv_small.hip)
constexpr int kHintWide = 1 << 22;     // register-weight row-streaming form, 2-D s1 (conv_wide.hip)
constexpr int kHintWide3 = 1 << 24;    // register-weight plane-streaming 3x3x3 form, <= 16 couts (conv_wide3.hip)
constexpr int kHintWideT = 1 << 25;    // register-weight ConvTranspose2d k4s2 form, all 4 classes per wave (conv_widet.hip)
constexpr int kHintTile3 = 1 << 23;    // LDS-tiled implicit-GEMM 3-D form for the large volumes (conv_tile3.hip)
constexpr int kHintNoTile = 1 << 19;   // automatic choice, without the LDS-tiled forms (A/B measurements)

// Descriptor validation shared by every entry point that takes an esm_conv_desc (launch_conv, the
// chain of chain.hip); ESM_OK or ESM_ERR_ARG with the message set.
int conv_check(const esm_conv_desc& a) {
    if (!a.w || !a.out) return arg_error("conv: null weights/output");
    if (a.nsrc < 1 || a.nsrc > ESM_MAX_SRC) return arg_error("conv: nsrc must be 1..3");
    int cin = 0;
    for (int i = 0; i < ESM_MAX_SRC; ++i) {
        if (i < a.nsrc) {
            if (!a.src[i].ptr || a.src[i].C <= 0) return arg_error("conv: bad source");
            cin += a.src[i].C;
        } else if (a.src[i].C != 0) {
            return arg_error("conv: unused source slots must have C = 0");
        }
    }
    if (cin != a.Cin) return arg_error("conv: Cin != sum of source channels");
    if (a.B <= 0 || a.Cout <= 0) return arg_error("conv: bad B/Cout");
    if (a.cin_pad % 16 || a.cin_pad < a.Cin) return arg_error("conv: cin_pad must be a multiple of 16 >= Cin");
    if (a.cout_pad % 32 || a.cout_pad < a.Cout) return arg_error("conv: cout_pad must be a multiple of 32 >= Cout");
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    if (a.kh != a.kw) return arg_error("conv: kh must equal kw");
    if (d3 && a.kd != a.kh) return arg_error("conv: 3-D kernels must be cubic");
    if (!d3 && (a.Di != 1 || a.Do != 1)) return arg_error("conv: 2-D conv needs Di = Do = 1");
    if (a.shuffle > 1 && (d3 || a.transposed)) return arg_error("conv: pixel shuffle only for 2-D convs");
    if (a.up && (a.Cout != 1 || d3 || a.up_f <= 0)) return arg_error("conv: bilinear add needs 2-D, Cout == 1");
    if (a.Hi <= 0 || a.Wi <= 0 || a.Di <= 0) return arg_error("conv: empty input");
    if (a.pre && (d3 || a.transposed || a.shuffle > 1 || a.up || a.prh < a.Wo || a.prc < 0 || a.prb < 0))
        return arg_error("conv: a partial sum (pre) only for 2-D, non-transposed, unshuffled convs");
    if (a.transposed) {
        if (a.kh != 4 || a.stride != 2 || a.ph != 1 || a.pw != 1 || (d3 && a.pd != 1))
            return arg_error("conv: transposed conv supports k=4, s=2, p=1 only");
        if (a.Ho != 2 * a.Hi || a.Wo != 2 * a.Wi || (d3 && a.Do != 2 * a.Di))
            return arg_error("conv: transposed output extent must be 2x the input");
        return ESM_OK;
    }
    const int S = a.stride;
    if (S != 1 && S != 2) return arg_error("conv: stride must be 1 or 2");
    if (a.Ho != (a.Hi + 2 * a.ph - a.kh) / S + 1 || a.Wo != (a.Wi + 2 * a.pw - a.kw) / S + 1 ||
        (d3 && a.Do != (a.Di + 2 * a.pd - a.kd) / S + 1))
        return arg_error("conv: output extent inconsistent with kernel/stride/padding");
    if (a.Ho <= 0 || a.Wo <= 0 || a.Do <= 0) return arg_error("conv: empty output");
    return ESM_OK;
}

int launch_conv(const esm_conv_desc* d, hipStream_t s) {
    if (!d) return arg_error("conv: null descriptor");
    const esm_conv_desc& a = *d;
    const int rc = conv_check(a);
    if (rc != ESM_OK) return rc;
    const bool d3 = a.kd > 1 || a.Di > 1 || a.Do > 1 || (a.transposed && a.kd == 4);
    const int form = a.hint & ~(kHintXcd | kHintNoTile);  // the form / tile bits (bit 30 only orders the tiles)
    const bool tile_auto = form == 0 && !(a.hint & kHintNoTile);
    if (a.pre) {  // the forms that start their accumulators from a partial sum (round 6)
        if ((a.hint & kHintWide) && conv::wide_ok(a)) return conv::launch_wide(a, s);
        if (((a.hint & kHintTile3) || (tile_auto && conv::tile2_auto(a))) && conv::tile2_ok(a)) return conv::launch_tile2(a, s);
        if (conv::small_ok(a)) return conv::launch_small(a, s);
        if (conv::wide_ok(a)) return conv::launch_wide(a, s);
        return arg_error("conv: a partial sum (pre) needs the lean, register-weight or tiled 2-D form");
    }
    if (a.transposed) {
        if (a.hint & kHintWideT) return conv::launch_widet(a, s);
        if (a.hint & kHintTile3) return d3 ? conv::launch_tile3(a, s) : conv::launch_tile2(a, s);
        // large maps (L at B = 4: ref4x.conv2_up 103 -> 61 us, r04 probe): the LDS-tiled form
        if (tile_auto && (d3 ? conv::tile3_auto(a) : conv::tile2_auto(a))) return d3 ? conv::launch_tile3(a, s) : conv::launch_tile2(a, s);
        if ((a.hint & kHintSmall) || (form == 0 && conv::small_auto(a))) return conv::launch_small(a, s);
        return d3 ? launch_conv3d(a, s) : launch_conv2d(a, s);
    }
    // 1x1 on the large maps / volumes: the pointwise streaming form (round 6); TILE3 | bit 29 forces it, TILE3
    // alone the LDS-tiled k1 form (A/B)
    if (((a.hint & kHintTile3) && (a.hint & (1 << 29))) || (tile_auto && conv::pw_auto(a))) {
        if (conv::pw_ok(a)) return conv::launch_pw(a, s);
    }
    if (a.hint & kHintSmall) return conv::launch_small(a, s);
    if (a.hint & kHintWide) {
        // a tuned choice for a layer the wide form cannot take after all (concat sources with different
        // row strides, e.g. a cropped view): the automatic rules instead
        if (conv::wide_ok(a)) return conv::launch_wide(a, s);
        esm_conv_desc d = a;
        d.hint &= kHintXcd;
        return launch_conv(&d, s);
    }
    if (a.hint & kHintWide3) return conv::launch_wide3(a, s);
    if (a.hint & kHintTile3) return d3 ? conv::launch_tile3(a, s) : conv::launch_tile2(a, s);
    // the MFMA-bound 3-D volumes / 2-D maps of ESMStereo-L / -M: the LDS-tiled form
    if (tile_auto && (d3 ? conv::tile3_auto(a) : conv::tile2_auto(a))) return d3 ? conv::launch_tile3(a, s) : conv::launch_tile2(a, s);
    if (a.hint & kHintStem) return conv::launch_stem(a, s);
    if (a.hint & kHintC1in) return conv::launch_c1in(a, s);
    // one input channel, 2-D, large map: the VALU form (an MFMA k-step would be 3/4 padding).
    // Measured (scripts/probes/c1in_sweep.py, profiles/r01_c1in_sweep.txt): 1->16 k3s2 at 192x624
    // output 8.6 us; on small maps the MFMA direct form wins (4.8 vs 11.6 us at 24x78)
    if (form == 0 && conv::c1in_ok(a) && static_cast<long long>(a.B) * a.Ho * a.Wo >= 65536)
        return conv::launch_c1in(a, s);
    if (a.hint & kHintNoStem) {
        esm_conv_desc d = a;
        d.hint &= ~kHintNoStem;
        return d3 ? launch_conv3d(d, s) : launch_conv2d(d, s);
    }
    // 8 / 12 / 24 output channels, 3x3(x3) stride 1: the 16-block MFMA form wastes no tile rows
    if (form == 0 && conv::stem_auto(a)) return conv::launch_stem(a, s);
    // latency-bound layers (most of the hot path): the lean K-split form (conv_small.hip)
    if (form == 0 && conv::small_auto(a)) return conv::launch_small(a, s);
    return d3 ? launch_conv3d(a, s) : launch_conv2d(a, s);
}

}  // namespace esm

extern "C" int esm_conv_f32(const esm_conv_desc* desc, void* stream) {
    return esm::launch_conv(desc, esm::as_stream(stream));
}
