// esm_convt_1x1_f32: a ConvTranspose BasicConv and the 1x1 BasicConv over [its cropped output, skip / image
// features] in one launch (conv_up1.h; models/ESMStereo.py:163-175 agg_0 / agg_1 after conv3_up / conv2_up,
// 221-234 in up_refinement).  Host validation, then the form of the transposed conv: the LDS-tiled form
// (conv_tile3.hip) where a's hint asks for it (bit 23) or where the lean form does not take the layer,
// else the lean K-split form (conv_small.hip).
#include "conv_up1.h"

namespace esm {

int conv_check(const esm_conv_desc& a);  // conv.hip

namespace conv {
bool small_auto(const esm_conv_desc& a);                                              // conv_small.hip
int launch_small_up1(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s);  // conv_small.hip
int launch_tile_up1(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s);   // conv_tile3.hip

constexpr int kUp1MaxXB = 12;  // extra 4-channel k-steps the fused kernels instantiate (<= 48 channels)

int up1_validate(const esm_conv_desc& a, const esm_conv_desc& b) {
    esm_conv_desc ac = a;
    if (!ac.out) ac.out = b.out;  // a's output is never written; conv_check wants a pointer
    int rc = conv_check(ac);
    if (rc == ESM_OK) rc = conv_check(b);
    if (rc != ESM_OK) return rc;
    // 17-32 couts on either side: the two-tile tiled form only (3-D, <= 32 extra channels)
    const bool wide = a.Cout > 16 || b.Cout > 16;
    const bool d3 = a.kd == 4;
    if (wide && (!d3 || b.Cin - a.Cout > 32))
        return arg_error("convt_1x1: more than 16 couts only for the 3-D tiled form with <= 32 extra channels");
    return up1_check(a, b, wide ? 8 : kUp1MaxXB, wide ? 32 : 16);
}

int launch_convt_1x1(const esm_conv_desc& a, const esm_conv_desc& b, hipStream_t s) {
    const int rc = up1_validate(a, b);
    if (rc != ESM_OK) return rc;
    const bool wide = a.Cout > 16 || b.Cout > 16;
    const bool tile = wide || (a.hint & (1 << 23)) || (!(a.hint & (1 << 21)) && !small_auto(a));
    return tile ? launch_tile_up1(a, b, s) : launch_small_up1(a, b, s);
}

}  // namespace conv
}  // namespace esm

extern "C" int esm_convt_1x1_f32(const esm_conv_desc* a, const esm_conv_desc* b, void* stream) {
    if (!a || !b) return esm::arg_error("convt_1x1: null descriptor");
    return esm::conv::launch_convt_1x1(*a, *b, esm::as_stream(stream));
}
