/*
 * esmstereo_amd — C ABI of the MI355X (gfx950) ESMStereo hot path.
 *
 * Every entry point takes caller-owned DEVICE pointers (fp32, contiguous unless a stride
 * is given), plain sizes and a HIP stream handle passed as `void*` (a `hipStream_t`; NULL =
 * the default stream).  Kernels never allocate or free; launches are stream-ordered and the
 * library keeps no global mutable state apart from a thread-local last-error string.
 * Return value: ESM_OK (0) or a negative ESM_ERR_* code; esm_last_error() says why.
 *
 * Each function replaces one reference interface (file:line in /root/reference):
 *   esm_gwc_volume_f32        models/submodule.py:151-161 build_gwc_volume (+ the S-variant
 *                             `volume * att` at models/ESMStereo.py:711 when att != NULL)
 *   esm_concat_volume_f32     models/submodule.py:129-140 build_concat_volume
 *   esm_normcorr_volume_f32   models/submodule.py:187-200 build_norm_correlation_volume
 *   esm_disp_regression_f32   models/submodule.py:211-216 disparity_regression
 *   esm_topk2_regression_f32  models/submodule.py:218-225 regression_topk(cost, arange, k=2)
 *   esm_topk_regression_f32   models/submodule.py:218-225 regression_topk(cost, samples, k), any k
 *   esm_conv_f32              models/submodule.py:12-38 BasicConv (Conv2d/3d, ConvTranspose2d/3d,
 *                             eval BatchNorm, GELU) and the plain convs of models/ESMStereo.py:
 *                             129-509 with their fused neighbours (crop+cat :172,177,230,234;
 *                             PixelShuffle+SiLU :265-268; bilinear-upsample + add :307,316;
 *                             `* att` :703; residual adds of models/shufflemixer.py:130-131)
 *   esm_fmnet_f32             models/shufflemixer.py:100-112,129-130 FMBlock.net (two SMLayers) + x
 *   esm_smix_f32              models/shufflemixer.py:23-112 LayerNorm('BiasFree') +
 *                             SplitPointMlp + channel shuffle + residual, optionally preceded
 *                             by the depthwise 7x7 `spatial` conv
 *   esm_shuffle_tail_f32      models/ESMStereo.py:264-271,290-302,311-312 (and the upsample8 /
 *                             upsample16 twins): `upsampling` (Conv2d 1x1 nf -> nf*r*r + bias,
 *                             PixelShuffle(r), SiLU) followed by `tail` (Conv2d 3x3 nf -> 1 +
 *                             bias) as one kernel; the shuffled map is never materialised
 *   esm_shuffle_conv_f32      the same head followed by up_refinement.conv1[0] (models/ESMStereo.py:
 *                             190-191, the refinement's first BasicConv(1, C, 3, 2, 1)) in one kernel
 *   esm_conf_f32              the per-pixel stages of the confidence head LAFNet_ESM /
 *                             conf_upsample (models/ESMStereo_confidence.py:511-744) between its
 *                             convs (which run through esm_conv_f32): cost features, attention,
 *                             the scale-driven 3x grid_sample, the softmax-weighted x4 upsample
 *   esm_plan_*                the orchestration of models/ESMStereo.py:700-745 as a native
 *                             launch list, optionally replayed as one hipGraph
 *   esm_preprocess_u8         the input side: pad to /32 + ToTensor +
 *                             Normalize of test_kitti.py:93-106 (pad before normalising) or
 *                             datasets/kitti_dataset.py:151-170 (pad after), datasets/data_io.py:7-16
 *   esm_node_filter_u16       the ROS node's post-processing (kitti_publisher_cuda_node.cpp:385-403):
 *                             crop, medianBlur 5x5, valid mask, x256 -> uint16
 *   esm_disp_to_u16           the output side: crop of the padded disparity (test_kitti.py:115,
 *                             save_disp.py:81) + np.round(d * 256).astype(np.uint16) (save_disp.py:85)
 */
#ifndef ESMSTEREO_AMD_H
#define ESMSTEREO_AMD_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ESM_OK 0
#define ESM_ERR_ARG (-1)
#define ESM_ERR_LAUNCH (-2)
#define ESM_ERR_UNSUPPORTED (-3)
#define ESM_ERR_RUNTIME (-4)

#define ESM_ACT_NONE 0
#define ESM_ACT_GELU 1 /* exact erf GELU, nn.GELU() */
#define ESM_ACT_SILU 2
#define ESM_ACT_RELU 3
#define ESM_ACT_SIGMOID 4 /* 1 / (1 + exp(-x)), torch.sigmoid */
#define ESM_ACT_RELU6 5   /* min(max(x, 0), 6), nn.ReLU6 (the MobileNetV2 backbone) */

#define ESM_MAX_SRC 3

/* One channel-slice source of a (possibly concatenated, possibly cropped) conv input.
 * Element strides; the innermost (W) stride is 1.  For 2-D tensors sd is ignored. */
typedef struct {
    const float* ptr;
    int32_t C;
    int32_t reserved;
    int64_t sb, sc, sd, sh;
} esm_src;

/* Implicit-GEMM convolution on NC(D)HW fp32, fp32 MFMA.
 * 2-D convs use kd = 1, Di = Do = 1.
 * Transposed convs are supported for kernel 4, stride 2, padding 1 (the only form the
 * reference uses); out extent = 2 x in extent.
 * weights: packed by esm_conv_pack_* conventions (see esmstereo_amd/engine.py):
 *   normal:     w[tap][cin_pad][cout_pad], tap = (kd_i*kh + kh_i)*kw + kw_i
 *   transposed: w[cls][tap][cin_pad][cout_pad], cls = parity class of the output voxel
 * Epilogue order: v = acc*scale[c] + shift[c] (scale NULL -> 1, shift NULL -> 0);
 *   v = act(v); v *= mul[b,c,y,x] (broadcast over d); v += res[b,c,d,y,x];
 *   v = bilinear_up(up)[b,0,y,x] + v; store v * post_scale (through a PixelShuffle of
 *   factor `shuffle` when > 1) and, when out2 != NULL, v * post_scale2 to out2. */
typedef struct {
    esm_src src[ESM_MAX_SRC];
    int32_t nsrc;
    int32_t B, Cin;
    int32_t Di, Hi, Wi;
    int32_t Do, Ho, Wo;
    int32_t kd, kh, kw;
    int32_t stride;
    int32_t transposed;
    int32_t pd, ph, pw;
    int32_t Cout;
    int32_t cin_pad, cout_pad;
    const float* w;
    const float* scale;
    const float* shift;
    int32_t act;
    int32_t shuffle;
    const float* mul;
    int64_t mb, mc, mh;
    const float* res;
    int64_t rb, rc, rd, rh;
    float* out;
    int64_t ob, oc, od, oh;
    const float* up;
    int32_t up_h, up_w, up_f;
    int32_t hint; /* 0 = automatic tile choice; else NT | KS << 4 | C1 << 8 | DIRECT << 9 | ROWS << 10 |
                     rows-per-wave << 12 | C1T << 16 | STEM << 17 (16-block 4x4x1 MFMA form for
                     3x3(x3) s1 convs with 8/12/16/24/32 couts) | NO_STEM << 18 (automatic, without it) |
                     C1IN << 20: force the VALU form for 2-D convs with one input channel
                     (tuning sweeps / tests; see conv_impl.h launch_geom) |
                     SMALL << 21: the lean K-split form for latency-bound layers (conv_small.hip;
                     plain epilogues: no mul / up / shuffle) |
                     NO_TILE << 19: the automatic choice without the LDS-tiled forms (A/B measurements) |
                     WIDE << 22: register-resident-weight row-streaming form (conv_wide.hip; 2-D, stride 1,
                     k1 / k3 / k5, concat sources with one row stride, Cout <= 32) |
                     TILE3 << 23: LDS-tiled implicit-GEMM form (conv_tile3.hip; 3-D k3 s1 / s2 p1, k1 s1 over up
                     to 3 sources and ConvTranspose3d k4 s2; 2-D k3 s1 / s2, k1 s1 and ConvTranspose2d k4 s2;
                     <= 96 couts; bits 26-27: rows per wave 1 / 2 / 4, 0 automatic; chosen automatically
                     for 3-D volumes of >= 2^16 output voxels and 2-D maps of >= 2^19 pixel x cout-tiles) |
                     WIDE3 << 24: register-weight plane-streaming form for 3x3x3 s1 p1 3-D convs with <= 16 couts
                     and <= 32 input channels (conv_wide3.hip; plain, `* mul` and residual epilogues) |
                     WIDET << 25: register-weight ConvTranspose2d k4 s2 form computing all 4 parity classes per
                     wave (conv_widet.hip; one source, 16 * channel groups * cout tiles <= 64).
                     Bits 26-27 with WIDE / WIDET: rows per wave (1 / 2 / 3 = 2 / 4 / 8 rows, WIDET 1 / 2
                     sub-grid rows); 0 = the automatic choice.  Bit 28 with WIDE: each strip's channel groups
                     split over two waves (partial rows summed once through LDS; R >= 4).  Bit 29 with SMALL:
                     8 waves per workgroup splitting K (layers with more than 4 channel groups); bit 29 on
                     the first desc of esm_conv_pair2_f32: regression source (see there).
                     With TILE3 (round 6): bit 29 on a 1x1 = the pointwise streaming form (conv_pw.hip, chosen
                     automatically for dense 1x1 BasicConvs over >= 2^16 pixels), on a 3x3x3 layer = its
                     LDS-staged-weight / padded-MT variant (A/B); bit 28 on the register-weight 3-D forms flips
                     the buffer-to-LDS (DMA) staging of the input window.
                     Bit 30 (any value of the other bits, including 0 = automatic): XCD-slab tile order for
                     the small / wide / wide3 / wideT / pair / single-output ConvT forms: each XCD runs a
                     contiguous band of tiles, so halo rows are fetched once per band instead of once per
                     XCD (memory-side bytes ~1.1x the algorithmic instead of 2-3x on full-size maps). */
    int64_t ub, uh;
    float post_scale;
    float post_scale2;
    float* out2; /* nullable: second copy of the result (same strides as out), x post_scale2 / post_scale */
    /* nullable (round 6): a partial conv sum over other input channels, [B, Cout, Ho, Wo] (2-D, element strides
     * prb / prc / prh, W contiguous), added before the BN scale/shift: acc = pre + sum over this conv's sources.
     * The upsampler stages' concat convs (models/ESMStereo.py:488, 501) split this way: the image-feature part
     * runs on the plan's side branch (esm_plan_set_branch) while the disparity chain runs.  Lean, register-
     * weight and LDS-tiled 2-D forms (and esm_convt_1x1_f32's second desc); ESM_ERR_ARG elsewhere. */
    const float* pre;
    int64_t prb, prc, prh;
} esm_conv_desc;

/* ShuffleMixer per-pixel chain on a [B, C, H, W] tensor, C in {8, 16}:
 *   t = dw ? (depthwise KxK conv of x with bias) : x          (SMLayer.spatial)
 *   for s in stages: t = shuffle(cat(fc2(silu(fc0(LN_s(t)[:C/2]))), LN_s(t)[C/2:])) + t
 *   if res: t += res
 * (SMLayer.forward, shufflemixer.py:108-112; FMBlock `net(x) + x`, :130). */
#define ESM_SMIX_MAX_STAGES 2
typedef struct {
    const float* ln_w;  /* [C] */
    const float* fc0_w; /* [C][C/2] */
    const float* fc0_b; /* [C] */
    const float* fc2_w; /* [C/2][C] */
    const float* fc2_b; /* [C/2] */
} esm_smix_stage;

typedef struct {
    const float* x;
    float* out;
    const float* res; /* nullable */
    const float* dw_w; /* [C][K][K], nullable (no depthwise) */
    const float* dw_b; /* [C] */
    int32_t dw_k;
    int32_t nstages;
    esm_smix_stage stage[ESM_SMIX_MAX_STAGES];
    int32_t B, C, H, W;
} esm_smix_desc;

/* The whole `net` of an FMBlock (two SMLayers, models/shufflemixer.py:100-112,129-130) in one launch:
 * out = SMLayer1(SMLayer0(x)) + x, where SMLayer(t) = mlp2(dw(mlp1(t))) with mlp = the per-pixel
 * LN -> SplitPointMlp -> shuffle -> residual chain of esm_smix_desc.  stage[] = SMLayer0.mlp1,
 * SMLayer0.mlp2, SMLayer1.mlp1, SMLayer1.mlp2; dw_w/dw_b[l] = SMLayer l's depthwise K x K conv
 * (K = 7); C in {8, 16}.  The three esm_smix_f32 launches it replaces, in one (same operations). */
typedef struct {
    const float* x;
    float* out;
    const float* dw_w[2];
    const float* dw_b[2];
    int32_t dw_k;
    int32_t reserved;
    esm_smix_stage stage[4];
    int32_t B, C, H, W;
    /* optional, conv0_w != NULL: FMBlock.conv fused behind net (shufflemixer.py:124-131), out =
     * conv2(silu(conv0(t) + conv0_b)) + conv2_b + t with t = net(x) + x; conv0_w [hid][C][3][3] (zero
     * padding 1), conv0_w/b [hid], conv2_w [C][hid], conv2_b [C]; hid = C + 16 */
    const float* conv0_w;
    const float* conv0_b;
    const float* conv2_w;
    const float* conv2_b;
    int32_t hid;
    int32_t reserved2;
    /* optional, with conv0_w: a [B, C, H, W] scratch buffer; when given, the block runs as two launches
     * split at the second depthwise conv (halo 3 each side instead of the whole block's 7) with FMBlock.conv
     * on the matrix cores: the form for large maps (ESMStereo-L at KITTI size and up) */
    float* work;
} esm_fmnet_desc;

/* Fused `tail(upsampling(x))` of the ESM upsamplers: out[b,0] = tail_b + conv3x3(tail_w,
 * silu(pixel_shuffle(conv1x1(up_w, x) + up_b, r))), zero padding 1.  (nf, r) in
 * {(8,2), (8,4), (16,2), (16,4)}.  x: [B, nf, H, W] with strides xb, xc, xh (innermost 1);
 * out: [B, 1, r*H, r*W] with strides ob, oh.  tail_b may be NULL (no bias). */
typedef struct {
    const float* x;
    int64_t xb, xc, xh;
    const float* up_w;   /* [nf*r*r][nf] */
    const float* up_b;   /* [nf*r*r] */
    const float* tail_w; /* [nf][3][3] */
    const float* tail_b; /* [1] or NULL */
    float* out;
    int64_t ob, oh;
    int32_t B, nf, H, W, r;
    int32_t flags; /* bit 0: XCD-slab tile order (each XCD runs a contiguous band of output rows; see
                      esm_conv_desc.hint bit 30); bits 1-2, (nf, r) = (8, 4) only: 0 automatic, 1 the
                      low-res-window form, 2 / 3 the MFMA row form with 4 / 8 low-res rows per workgroup */
} esm_shuffle_tail_desc;

/* `tail(upsampling(x))` (as esm_shuffle_tail_desc, st.out unused) followed by the refinement
 * hourglass's first layer BasicConv(1, C, 3, stride 2, pad 1) + folded BN + exact GELU
 * (up_refinement.conv1[0], models/ESMStereo.py:190-191), in one launch; the 1-channel map between
 * them is never stored.  w: packed conv weights [9][cin_pad][cout_pad] (cin 1); scale/shift: the
 * folded BN (scale NULL = 1); out: [B, C, ceil(r*H/2), ceil(r*W/2)] with strides ob, oc, oh.
 * (nf, r, C) in {(8, 4, 16), (8, 2, 16), (16, 2, 32), (16, 4, 32)}.  st.flags bit 0: XCD-slab tile order;
 * bits 1-2, (8, 4, 16) only: 0 automatic, 1 the low-res-window form, 2 the MFMA row form (8 low-res rows
 * per workgroup), 3 the same row form with the refinement conv on the matrix cores. */
typedef struct {
    esm_shuffle_tail_desc st;
    const float* w;
    const float* scale;
    const float* shift;
    float* out;
    int64_t ob, oc, oh;
    int32_t C, cin_pad, cout_pad, reserved;
    /* Optional pre-conv (nf 8, r 4, C 16 row form only): with pre_x set, the head's input x is not read from
     * st.x (which must be NULL) but computed in the launch as GELU(BN(Conv2d(pre_cin, nf, 3, 1, 1)(pre_x)))
     * -- the upsampler stage's spx_<t>[1] (models/ESMStereo.py:247-259) -- from pre_x [B, pre_cin, H, W]
     * (strides pb, pc, ph; pre_cin <= 16), packed weights pre_w [9][pre_cin_pad][pre_cout_pad] and the
     * folded BN pre_scale / pre_shift (pre_scale NULL = 1). */
    const float* pre_x;
    int64_t pb, pc, ph;
    const float* pre_w;
    const float* pre_scale;
    const float* pre_shift;
    int32_t pre_cin, pre_cin_pad, pre_cout_pad, pre_reserved;
    /* Optional second conv (nf 8, r 4, C 16 row form with pre_x only): with w2 set, the refinement's
     * conv1[1] (BasicConv(C, C, 3, 1, 1): folded BN scale2 / shift2 (scale2 NULL = 1) + exact GELU, packed
     * w2 [9][cin_pad2][cout_pad2]) runs in the same launch on the first conv's map, which is never stored:
     * `out` receives conv1[1]'s output (same shape and strides). */
    const float* w2;
    const float* scale2;
    const float* shift2;
    int32_t cin_pad2, cout_pad2;
} esm_shuffle_conv_desc;

/* Depthwise KxK conv (groups = C, no bias) + folded BN (out = act(conv * scale[c] + shift[c]); scale NULL = 1,
 * shift NULL = 0): timm's conv_dw + bn of the backbone blocks (models/ESMStereo.py:40-77).  x: [B, C, H, W]
 * (strides xb, xc, xh; innermost 1), w: [C][K][K], out: [B, C, Ho, Wo] (strides ob, oc, oh), zero padding
 * `pad`, (K, stride) in {(3, 1), (3, 2), (5, 1), (5, 2)}, act one of ESM_ACT_*. */
typedef struct {
    const float* x;
    int64_t xb, xc, xh;
    const float* w;
    const float* scale;
    const float* shift;
    float* out;
    int64_t ob, oc, oh;
    int32_t B, C, H, W, K, stride, pad, act, Ho, Wo;
} esm_dwconv_desc;

const char* esm_last_error(void);
int esm_version(void);
/* sizeof of the ABI structs, for binding checks: 0 esm_src, 1 esm_conv_desc,
 * 2 esm_smix_stage, 3 esm_smix_desc, 4 esm_shuffle_tail_desc, 5 esm_fmnet_desc, 6 esm_conf_desc,
 * 8 esm_shuffle_conv_desc, 9 esm_dwconv_desc;
 * -1 for an unknown id. */
int esm_struct_size(int which);

int esm_gwc_volume_f32(const float* L, const float* R, const float* att, float* V, int B, int C, int H, int W,
                       int D, int G, void* stream);
/* The gwc volume and the first 3-D conv over it in one launch (ESMStereo-L / -M: build_gwc_volume,
 * models/submodule.py:151-161, then group_stem, models/ESMStereo.py:610-611 / 703-704): `stem` describes the
 * conv as esm_conv_f32 would take it over the [B, G, D, H, W] volume (Cin = G, Di x Hi x Wi = D x H x W,
 * 3x3x3 stride 1 pad 1, <= 8 outputs; its src[] is ignored and no volume is written); L / R are contiguous
 * [B, C, H, W] features with C = 2 G, G a multiple of 4.  Bit-identical to esm_gwc_volume_f32 followed by
 * esm_conv_f32 with the LDS-tiled form (hint bit 23); bits 26-27 of stem->hint: rows per wave 2 / 4. */
int esm_gwc_stem_f32(const esm_conv_desc* stem, const float* L, const float* R, int C, int G, void* stream);
int esm_concat_volume_f32(const float* L, const float* R, float* V, int B, int C, int H, int W, int D,
                          void* stream);
/* work: unused since the single-launch kernel (normalises in LDS); may be NULL.  C <= 64. */
int esm_normcorr_volume_f32(const float* L, const float* R, float* V, float* work, int B, int C, int H, int W,
                            int D, void* stream);
int esm_disp_regression_f32(const float* cost, float* out, int B, int D, int H, int W, void* stream);
/* samples: [B, D, H, W] disparity_samples, or NULL for arange(D) (the ESMStereo call). */
int esm_topk2_regression_f32(const float* cost, const float* samples, float* out, int B, int D, int H, int W,
                             void* stream);
/* regression_topk for any k >= 1 (models/submodule.py:218-225): the reference slices the sorted
 * indices, so k > D selects all D.  Ties rank the lower index first; NaN ranks first. */
int esm_topk_regression_f32(const float* cost, const float* samples, float* out, int B, int D, int H, int W, int k,
                            void* stream);
int esm_conv_f32(const esm_conv_desc* desc, void* stream);
int esm_smix_f32(const esm_smix_desc* desc, void* stream);
int esm_fmnet_f32(const esm_fmnet_desc* desc, void* stream);
int esm_shuffle_tail_f32(const esm_shuffle_tail_desc* desc, void* stream);
int esm_shuffle_conv_f32(const esm_shuffle_conv_desc* desc, void* stream);
/* Two consecutive 2-D BasicConvs in one launch (the intermediate map stays in LDS; halo recomputed):
 * out_b = GELU(BN_b(conv_b(GELU(BN_a(conv_a(cat(a->src))))))).  a: k 1/3/5 stride 1 or k 3 stride 2,
 * 16 outputs, <= 48 input channels (64 for k 1) over 1..3 sources (4-channel multiples when several);
 * a->out is not written.  b: k 1 or 3, stride 1, 16 inputs (its src[] is ignored: the input is a's
 * output), <= 16 outputs, plain epilogue.  ESM_ERR_ARG for a pair outside that set.
 * Regression source (a->hint bit 29; a: 5x5, Cin 1, one source; b: 3x3): a->src[0] is a [B, D, H, W]
 * cost volume (src[0].C = D, H x W = a's input extent) and a's input map is its disparity_regression
 * sum_d cost[d] * d (models/submodule.py:211-216, the bits of esm_disp_regression_f32), which is also
 * stored to a->out ([B, 1, H, W], strides ob / oh): the regression launch folded into the upsampler's
 * first pair (models/ESMStereo.py:735-745).  b->hint bits 26-27: tile rows 2 / 4 / 8 (8 only with <= 16
 * input channels; other bits of b->hint are ignored), 0 = automatic (4 rows where that gives >= 256 tiles).
 * (models/ESMStereo.py:185-259: the refinement hourglasses' conv2 / conv3 pairs and the upsampler
 * stages' dm<t> / spx_<t> pairs.) */
int esm_conv_pair2_f32(const esm_conv_desc* a, const esm_conv_desc* b, void* stream);
/* A ConvTranspose BasicConv and the 1x1 BasicConv over [its output cropped to b's extent, further sources]
 * in one launch; replaces the decoder steps of models/ESMStereo.py:163-175 (aggregation: conv3_up ->
 * cat(crop, conv2) -> agg_0[0], conv2_up -> cat(crop, conv1) -> agg_1[0]) and :221-234 (up_refinement, with
 * left_f1x / left_f2x as the third source).  out_b = GELU(BN_b(conv1x1_b(cat(crop(GELU(BN_a(convT_a(a->src)))),
 * b->src[1..])))).  a: k4 s2 p1, one source, 4 / 8 / 12 / 16 outputs, BN + GELU, plain epilogue; a->out is
 * not written (may be NULL).  b: 1x1 stride 1, b->src[0].C = a->Cout (its ptr is not read; b's input extent
 * is the crop, at most a's output extent), b->src[1..2]: 4-channel multiples, at most 48 channels together;
 * <= 16 outputs, BN + GELU, plain epilogue.  a->hint picks the transposed conv's form (bit 23: LDS-tiled,
 * bits 26-27 rows per wave 1 / 2; bit 21: lean), 0 = automatic.  ESM_ERR_ARG outside that set. */
int esm_convt_1x1_f32(const esm_conv_desc* a, const esm_conv_desc* b, void* stream);
/* Confidence-head stages (models/ESMStereo_confidence.py), fp32 NCHW, contiguous:
 *   ESM_CONF_COST_FEATURES  x[0] = cost [B,D,H,W] (D >= 7) -> out [B,7,H,W]: the 7 largest of
 *                           softmax(-100 * cost / sqrt(sum_d cost^2 + 1e-6)) over D, descending (:647-654)
 *   ESM_CONF_ATTEND         x[0..2] = cost_x, disp_x, imag_x [B,C,H,W], x[3] = logits [B,3,H,W] ->
 *                           out [B,3C,H,W] = cat(x_k * softmax_k(logits)) (:679-689)
 *   ESM_CONF_ENLARGE        x[0] = feat [B,C,H,W], x[1] = scale [B,1,H,W] -> out [B,9C,H,W]: the 3x
 *                           enlarged grid_sample(feat, grid(scale), bilinear, align_corners, zeros) of
 *                           :691-714, stored space-to-depth (channel c*9 + 3i + j = sample (3y+i, 3x+j)),
 *                           so embed_conv2 (k3 s3) runs as a 1x1 conv over 9C channels
 *   ESM_CONF_COMBINE        x[0] = logits [B,9,4H,4W], x[1] = init [B,1,H,W] -> out [B,1,4H,4W] =
 *                           sum_k softmax_k(logits) * unfold3x3(init)[k] at (Y/4, X/4) (:538-543)
 *   ESM_CONF_SIGMOID        x[0] [B*C*H*W] -> out, torch.sigmoid (:744) */
#define ESM_CONF_COST_FEATURES 1
#define ESM_CONF_ATTEND 2
#define ESM_CONF_ENLARGE 3
#define ESM_CONF_COMBINE 4
#define ESM_CONF_SIGMOID 5
typedef struct {
    int32_t op;
    int32_t B, C, D, H, W;
    const float* x[4];
    float* out;
} esm_conf_desc;
int esm_conf_f32(const esm_conf_desc* desc, void* stream);
/* The backbone's depthwise conv + BN + activation (esm_dwconv_desc; replaces MIOpen's grouped conv + BatchNorm +
 * activation of timm's blocks, backbone side of models/ESMStereo.py:640-697). */
int esm_dwconv_f32(const esm_dwconv_desc* desc, void* stream);

/* img: [B, H, W, 3] uint8 RGB (PIL order); out: [B, 3, Hp, Wp] fp32.  The image lands at rows
 * [top, top+H), columns [left, left+W); pad_normalized = 1 fills the rest with normalised zeros
 * (test_kitti.py: top = Hp-H, left = Wp-W), 0 with 0.0 (kitti_dataset.py: top = Hp-H, left = 0). */
int esm_preprocess_u8(const uint8_t* img, float* out, int B, int H, int W, int Hp, int Wp, int top, int left,
                      int pad_normalized, void* stream);
/* disp: [B, Hp, Wp] fp32; out: [B, h, w] uint16 = round_half_even(disp[b, top+y, left+x] * 256). */
int esm_disp_to_u16(const float* disp, uint16_t* out, int B, int Hp, int Wp, int top, int left, int h, int w,
                    void* stream);

/* The ROS node's post-processing (kitti_publisher/src/kitti_publisher_cuda_node.cpp:385-403) on the
 * device: disp [B, Hp, Wp] fp32 -> window (top, left, h, w) -> 5x5 median (cv::medianBlur, replicate
 * border inside the window) -> 0 outside (0, max_disp) -> out [B, h, w] uint16 =
 * saturate_cast<ushort>(rint(d * 256)); `filtered` (may be NULL) receives the masked median [B, h, w]. */
int esm_node_filter_u16(const float* disp, uint16_t* out, float* filtered, int B, int Hp, int Wp, int top, int left,
                        int h, int w, float max_disp, void* stream);

/* ---- native launch plan (the hot path as one replayable unit) ---- */
typedef struct esm_plan esm_plan;
esm_plan* esm_plan_create(void);
void esm_plan_destroy(esm_plan* plan);
int esm_plan_add_conv(esm_plan* plan, const esm_conv_desc* desc);
int esm_plan_add_smix(esm_plan* plan, const esm_smix_desc* desc);
int esm_plan_add_fmnet(esm_plan* plan, const esm_fmnet_desc* desc);
int esm_plan_add_shuffle_tail(esm_plan* plan, const esm_shuffle_tail_desc* desc);
int esm_plan_add_shuffle_conv(esm_plan* plan, const esm_shuffle_conv_desc* desc);
int esm_plan_add_conv_pair2(esm_plan* plan, const esm_conv_desc* a, const esm_conv_desc* b);
int esm_plan_add_convt_1x1(esm_plan* plan, const esm_conv_desc* a, const esm_conv_desc* b);
/* Fork-join (round 6).  Op `index` runs on the plan's second stream (branch 1) instead of the main chain
 * (branch 0): forked from the start of every run / graph replay, so it overlaps the main chain.  A side op
 * may read only buffers no main op writes before the join and write only buffers no main op reads before it.
 * esm_plan_set_join(index, 1): main op `index` first waits for every side op listed before it (the join);
 * side ops not joined by any op are joined at the end of the plan.  Both return the previous value. */
int esm_plan_set_branch(esm_plan* plan, int index, int branch);
int esm_plan_set_join(esm_plan* plan, int index, int join);
int esm_plan_add_gwc(esm_plan* plan, const float* L, const float* R, const float* att, float* V, int B, int C,
                     int H, int W, int D, int G);
int esm_plan_add_gwc_stem(esm_plan* plan, const esm_conv_desc* stem, const float* L, const float* R, int C, int G);
int esm_plan_add_concat(esm_plan* plan, const float* L, const float* R, float* V, int B, int C, int H, int W,
                        int D);
int esm_plan_add_normcorr(esm_plan* plan, const float* L, const float* R, float* V, float* work, int B, int C,
                          int H, int W, int D);
/* kind 0 = disparity_regression, 1 = regression_topk k=2, 2 + k = regression_topk with that k */
int esm_plan_add_regression(esm_plan* plan, int kind, const float* cost, float* out, int B, int D, int H, int W);
int esm_plan_add_conf(esm_plan* plan, const esm_conf_desc* desc);
int esm_plan_num_ops(const esm_plan* plan);
/* 0 = unknown, 1 = conv, 2 = smix, 3 = gwc, 4 = concat, 5 = normcorr, 6 = regression,
 * 7 = shuffle_tail, 9 = fmnet, 10 = conf, 12 = shuffle_conv, 13 = conv_pair2, 14 = gwc_stem (8 and 11
 * were retired fused forms) */
int esm_plan_op_kind(const esm_plan* plan, int index);
/* Replace the tile hint of conv op `index` (see esm_conv_desc.hint); returns the previous hint
 * (>= 0) or an error.  Bit 30 (tile order) is kept as the op was added, and is not part of the
 * returned value.  Drops a built graph (rebuild with esm_plan_graph_build). */
int esm_plan_set_conv_hint(esm_plan* plan, int index, int hint);
/* Diagnostics: launch op `index` `repeat` times per replay (0..8; 0 drops it, so the step time
 * minus the dropped step time is the op's marginal cost in the chain, gaps included).  Returns the
 * previous count; drops a built graph.  Results of a plan with a dropped op are not meaningful. */
int esm_plan_set_repeat(esm_plan* plan, int index, int repeat);
int esm_plan_run(esm_plan* plan, void* stream);
/* Launch op `index` alone, `reps` times back to back on `stream` (timing one kernel of the
 * path with a single hipEvent pair around the batch; the op's buffers are the plan's own). */
int esm_plan_run_op(esm_plan* plan, int index, int reps, void* stream);
/* Capture the launch list into a hipGraph (instantiated once; replays are cheap).  graph_launch
 * builds the graph first when there is none (never built, or dropped by a hint / repeat / probe change
 * or a rebind that changed an op's kernel). */
int esm_plan_graph_build(esm_plan* plan, void* stream);
int esm_plan_graph_launch(esm_plan* plan, void* stream);
/* Zero-copy input binding: every pointer of every op that lies in [old_base[k], old_base[k] + bytes[k])
 * moves to the same offset in new_base[k], k < n (the caller's tensors are read where they lie, the
 * reference forward's behaviour, models/ESMStereo.py:700-745).  With a built graph, the nodes of the
 * ops that changed are updated in place (after the previous replay has finished); when an op's
 * kernel choice changes with its pointers, the graph is dropped and rebuilt by the next launch.
 * Returns the number of pointer fields moved, or an error: ESM_ERR_ARG when two old ranges overlap
 * (which range a pointer belongs to would be ambiguous; bind aliased inputs through copies).  When
 * waiting for the previous replay fails, the ops are already moved and the graph is dropped (rebuilt
 * from the moved ops by the next launch). */
int esm_plan_rebind(esm_plan* plan, int n, const void* const* old_base, const uint64_t* bytes,
                    const void* const* new_base);
/* 1 while the last graph replay of the plan may still be running on the device (a rebind would then
 * wait for it), 0 when it has finished or the plan was never launched as a graph; < 0 on error. */
int esm_plan_busy(esm_plan* plan);
/* Probe: record a hipEvent pair around op `index` on every run/replay (ring of `ring`
 * pairs, ring <= 4096).  esm_plan_probe_read returns the elapsed ms of the completed
 * runs since the last read (caller synchronises first); returns the count written. */
int esm_plan_set_probe(esm_plan* plan, int index, int ring);
int esm_plan_probe_read(esm_plan* plan, float* ms, int max);

#ifdef __cplusplus
}
#endif

#endif /* ESMSTEREO_AMD_H */
