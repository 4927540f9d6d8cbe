"""CPU oracle for the ESMStereo hot path — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker / the timed CPU baseline.  The product path
(``esmstereo_amd``) never imports it and has no CPU fallback.

This is a from-scratch, functional restatement (plain PyTorch fp32 on the CPU, weights
passed as a state dict with the reference's key names) of the reference algorithm:

* cost volumes ............ ``models/submodule.py:129-200``
* regressions ............. ``models/submodule.py:211-225``
* BasicConv ............... ``models/submodule.py:12-38``
* aggregation hourglass ... ``models/ESMStereo.py:129-182``
* up_refinement ........... ``models/ESMStereo.py:185-239``
* ShuffleMixer FMBlock .... ``models/shufflemixer.py:23-132``
* upsample4/8/16 .......... ``models/ESMStereo.py:242-509``
* hot-path orchestration .. ``models/ESMStereo.py:700-745``

Pinning: ``tests/test_oracle_golden.py`` checks every function here against golden
vectors produced by running the reference itself (``tests/golden/make_golden.py``).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

SD = Dict[str, torch.Tensor]

# ----------------------------------------------------------------------------- volumes


def gwc_volume(L: torch.Tensor, R: torch.Tensor, D: int, G: int) -> torch.Tensor:
    """``build_gwc_volume`` (submodule.py:151-161): V[b,g,d,y,x] = mean_{c in g} L*R(x-d), 0 for x<d."""
    B, C, H, W = L.shape
    assert C % G == 0
    V = L.new_zeros(B, G, D, H, W)
    for d in range(min(D, W)):  # planes d >= W stay zero (the reference slices are empty there)
        prod = L[..., d:] * R[..., : W - d]
        V[:, :, d, :, d:] = prod.view(B, G, C // G, H, W - d).mean(dim=2)
    return V


def concat_volume(L: torch.Tensor, R: torch.Tensor, D: int) -> torch.Tensor:
    """``build_concat_volume`` (submodule.py:129-140): left copied for every x, right shifted."""
    B, C, H, W = L.shape
    V = L.new_zeros(B, 2 * C, D, H, W)
    V[:, :C] = L.unsqueeze(2)
    for d in range(min(D, W)):
        V[:, C:, d, :, d:] = R[..., : W - d]
    return V


def normcorr_volume(L: torch.Tensor, R: torch.Tensor, D: int) -> torch.Tensor:
    """``build_norm_correlation_volume`` (submodule.py:187-200); eps added after the sqrt."""
    B, C, H, W = L.shape
    Ln = L / (torch.norm(L, 2, 1, True) + 1e-05)
    Rn = R / (torch.norm(R, 2, 1, True) + 1e-05)
    V = L.new_zeros(B, 1, D, H, W)
    for d in range(min(D, W)):
        V[:, :, d, :, d:] = torch.mean(Ln[..., d:] * Rn[..., : W - d], dim=1, keepdim=True)
    return V


def disparity_regression(cost: torch.Tensor, D: int) -> torch.Tensor:
    """``disparity_regression`` (submodule.py:211-216): sum_d cost[d]*d, no softmax."""
    assert cost.dim() == 4
    d = torch.arange(0, D, dtype=cost.dtype, device=cost.device).view(1, D, 1, 1)
    return torch.sum(cost * d, 1, keepdim=False)


def regression_topk2(cost: torch.Tensor) -> torch.Tensor:
    """``regression_topk(cost, arange, 2)`` (submodule.py:218-225).

    Top-2 over D (value descending; ties -> lowest index, the build's documented order since
    ``torch.sort`` is unstable), softmax over the two values, weighted sum of the indices.
    """
    _, ind = torch.sort(cost, dim=1, descending=True, stable=True)
    idx = ind[:, :2]
    val = torch.gather(cost, 1, idx)
    prob = F.softmax(val, 1)
    return torch.sum(idx.to(cost.dtype) * prob, dim=1, keepdim=True)


def regression_topk(cost: torch.Tensor, disparity_samples, k: int) -> torch.Tensor:
    """``regression_topk(cost, disparity_samples, k)`` (submodule.py:218-225) for any k: the sorted
    indices sliced ``[:, :k]`` (Python slicing: k > D keeps all D), the gathered costs' softmax, the
    probability-weighted sum of the gathered samples (``None``: arange(D)).  Ties -> lowest index
    (stable sort; the reference's ``cost.sort`` is unstable, so tie order is this build's)."""
    _, ind = torch.sort(cost, dim=1, descending=True, stable=True)
    idx = ind[:, :k]
    if disparity_samples is None:
        samples = idx.to(cost.dtype)
    else:
        samples = torch.gather(disparity_samples, 1, idx)  # no broadcasting: gather's own failure class
    prob = F.softmax(torch.gather(cost, 1, idx), 1)
    return torch.sum(samples * prob, dim=1, keepdim=True)


# ----------------------------------------------------------------------------- BasicConv


def basic_conv(sd: SD, p: str, x: torch.Tensor, *, k, s=1, pad=0, deconv=False, bn=True, act="gelu") -> torch.Tensor:
    """``BasicConv`` (submodule.py:12-38): conv (bias=False) -> eval BatchNorm -> exact GELU."""
    w = sd[p + "conv.weight"]
    nd = w.dim() - 2
    if deconv:
        fn = F.conv_transpose3d if nd == 3 else F.conv_transpose2d
    else:
        fn = F.conv3d if nd == 3 else F.conv2d
    x = fn(x, w, None, s, pad)
    if bn:
        x = F.batch_norm(x, sd[p + "bn.running_mean"], sd[p + "bn.running_var"], sd[p + "bn.weight"],
                         sd[p + "bn.bias"], False, 0.0, 1e-5)
    if act == "gelu":
        x = F.gelu(x)
    return x


def conv(sd: SD, p: str, x: torch.Tensor, pad: int) -> torch.Tensor:
    """Plain ``nn.Conv2d`` with optional bias."""
    return F.conv2d(x, sd[p + "weight"], sd.get(p + "bias"), 1, pad)


def bn_gelu(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    x = F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                     False, 0.0, 1e-5)
    return F.gelu(x)


# ----------------------------------------------------------------------------- 3D hourglass


def aggregation(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """``aggregation.forward`` (ESMStereo.py:165-182)."""
    bc = lambda q, t, **kw: basic_conv(sd, p + q, t, **kw)  # noqa: E731
    c1 = bc("conv1.1.", bc("conv1.0.", x, k=3, s=2, pad=1), k=3, pad=1)
    c2 = bc("conv2.1.", bc("conv2.0.", c1, k=3, s=2, pad=1), k=3, pad=1)
    c3 = bc("conv3.1.", bc("conv3.0.", c2, k=3, s=2, pad=1), k=3, pad=1)
    u3 = bc("conv3_up.", c3, k=4, s=2, pad=1, deconv=True)
    c2 = torch.cat((u3[:, :, : c2.shape[2], : c2.shape[3], : c2.shape[4]], c2), 1)
    c2 = bc("agg_0.1.", bc("agg_0.0.", c2, k=1), k=3, pad=1)
    u2 = bc("conv2_up.", c2, k=4, s=2, pad=1, deconv=True)
    c1 = torch.cat((u2[:, :, : c1.shape[2], : c1.shape[3], : c1.shape[4]], c1), 1)
    c1 = bc("agg_1.1.", bc("agg_1.0.", c1, k=1), k=3, pad=1)
    return bc("conv1_up.", c1, k=4, s=2, pad=1, deconv=True, bn=False, act=None)


# ----------------------------------------------------------------------------- upsampler


def up_refinement(sd: SD, p: str, disp: torch.Tensor, f1: torch.Tensor, f2: torch.Tensor) -> torch.Tensor:
    """``up_refinement.forward`` (ESMStereo.py:221-239); the :234 concat does not crop."""
    bc = lambda q, t, **kw: basic_conv(sd, p + q, t, **kw)  # noqa: E731
    c1 = bc("conv1.1.", bc("conv1.0.", disp, k=3, s=2, pad=1), k=3, pad=1)
    c2 = bc("conv2.1.", bc("conv2.0.", c1, k=3, s=2, pad=1), k=3, pad=1)
    c3 = bc("conv3.1.", bc("conv3.0.", c2, k=3, s=2, pad=1), k=3, pad=1)
    u3 = bc("conv3_up.", c3, k=4, s=2, pad=1, deconv=True)
    c2 = torch.cat((u3[:, : c2.shape[1], : c2.shape[2], : c2.shape[3]], c2, f1), 1)
    c2 = bc("agg_0.1.", bc("agg_0.0.", c2, k=1), k=3, pad=1)
    u2 = bc("conv2_up.", c2, k=4, s=2, pad=1, deconv=True)
    c1 = torch.cat((u2, c1, f2), 1)
    c1 = bc("agg_1.1.", bc("agg_1.0.", c1, k=1), k=3, pad=1)
    return bc("conv1_up.", c1, k=4, s=2, pad=1, deconv=True, bn=False, act=None)


def layernorm_c(x: torch.Tensor, w: torch.Tensor) -> torch.Tensor:
    """``LayerNorm('BiasFree')`` (shufflemixer.py:47-62,83-93): per-pixel over C, mean IS subtracted."""
    t = x.permute(0, 2, 3, 1)
    mu = t.mean(-1, keepdim=True)
    var = t.var(-1, keepdim=True, unbiased=False)
    t = (t - mu) / torch.sqrt(var + 1e-5) * w
    return t.permute(0, 3, 1, 2)


def split_point_mlp(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """``SplitPointMlp`` (shufflemixer.py:23-37): MLP on the first half, then shuffle (g d)->(d g), g=8."""
    C = x.shape[1]
    x1, x2 = x[:, : C // 2], x[:, C // 2:]
    x1 = F.conv2d(F.silu(F.conv2d(x1, sd[p + "fc.0.weight"], sd[p + "fc.0.bias"])), sd[p + "fc.2.weight"],
                  sd[p + "fc.2.bias"])
    y = torch.cat([x1, x2], 1)
    B, _, H, W = y.shape
    return y.view(B, 8, C // 8, H, W).transpose(1, 2).reshape(B, C, H, W)


def sm_layer(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """``SMLayer.forward`` (shufflemixer.py:108-112)."""
    x = split_point_mlp(sd, p + "mlp1.", layernorm_c(x, sd[p + "norm1.body.weight"])) + x
    C = x.shape[1]
    x = F.conv2d(x, sd[p + "spatial.weight"], sd[p + "spatial.bias"], 1, sd[p + "spatial.weight"].shape[-1] // 2,
                 1, C)
    x = split_point_mlp(sd, p + "mlp2.", layernorm_c(x, sd[p + "norm2.body.weight"])) + x
    return x


def fm_block(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """``FMBlock.forward`` (shufflemixer.py:129-132)."""
    x = sm_layer(sd, p + "net.1.", sm_layer(sd, p + "net.0.", x)) + x
    y = F.conv2d(x, sd[p + "conv.0.weight"], sd[p + "conv.0.bias"], 1, 1)
    y = F.conv2d(F.silu(y), sd[p + "conv.2.weight"], sd[p + "conv.2.bias"])
    return y + x


def _dm(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """``dm{2,4,8}x`` disparity-feature stacks: k5 p1, k3 p1, k3 p1, k1 p1 (ESMStereo.py:250-253)."""
    x = basic_conv(sd, p + "0.", x, k=5, pad=1)
    x = basic_conv(sd, p + "1.", x, k=3, pad=1)
    x = basic_conv(sd, p + "2.", x, k=3, pad=1)
    return basic_conv(sd, p + "3.", x, k=1, pad=1)


def _spx(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    """``spx_*``: BasicConv k3 -> Conv2d k3 (no bias) -> BN -> GELU (ESMStereo.py:255-258)."""
    x = basic_conv(sd, p + "0.", x, k=3, pad=1)
    x = F.conv2d(x, sd[p + "1.weight"], None, 1, 1)
    return bn_gelu(sd, p + "2.", x)


def _shuffle_up(sd: SD, p: str, x: torch.Tensor, r: int) -> torch.Tensor:
    """``upsampling*``: 1x1 conv (bias) -> PixelShuffle(r) -> SiLU (ESMStereo.py:265-268)."""
    return F.silu(F.pixel_shuffle(conv(sd, p + "0.", x, 0), r))


def _bilinear(x: torch.Tensor, f: int) -> torch.Tensor:
    return F.interpolate(x, scale_factor=f, mode="bilinear", align_corners=False)


def upsample4(sd: SD, p: str, f1: torch.Tensor, f2: torch.Tensor, f4: torch.Tensor, init: torch.Tensor):
    """``upsample4.forward`` (ESMStereo.py:296-318), ESMStereo-L."""
    x = _spx(sd, p + "spx_2x.", torch.cat((_dm(sd, p + "dm2x.", init), f2), 1))
    x = F.conv2d(x, sd[p + "to_feat.weight"], None, 1, 1)
    x = fm_block(sd, p + "blocks.1.", fm_block(sd, p + "blocks.0.", x))
    x2 = conv(sd, p + "tail2x.", _shuffle_up(sd, p + "upsampling2.", x, 2), 1)
    x2 = up_refinement(sd, p + "ref2x.", x2, f1, f2)
    up2 = _bilinear(init, 2) + x2
    c4 = _spx(sd, p + "spx_4x.", torch.cat((_dm(sd, p + "dm4x.", up2), f4), 1))
    x4 = conv(sd, p + "tail4x.", _shuffle_up(sd, p + "upsampling4.", c4, 2), 1)
    x4 = up_refinement(sd, p + "ref4x.", x4, f2, f4)
    return [_bilinear(up2, 2) + x4, up2]


def upsample8(sd: SD, p: str, f2: torch.Tensor, f4: torch.Tensor, f8: torch.Tensor, s2: torch.Tensor,
              init: torch.Tensor):
    """``upsample8.forward`` (ESMStereo.py:396-428), ESMStereo-M."""
    x = _spx(sd, p + "spx_2x.", torch.cat((_dm(sd, p + "dm2x.", init), f4), 1))
    x = F.conv2d(x, sd[p + "to_feat.weight"], None, 1, 1)
    x = fm_block(sd, p + "blocks.1.", fm_block(sd, p + "blocks.0.", x))
    x2 = conv(sd, p + "tail2x.", _shuffle_up(sd, p + "upsampling2.", x, 2), 1)
    x2 = up_refinement(sd, p + "ref2x.", x2, f2, f4)
    up2 = _bilinear(init, 2) + x2
    c4 = _spx(sd, p + "spx_4x.", torch.cat((_dm(sd, p + "dm4x.", up2), f8), 1))
    x4 = conv(sd, p + "tail4x.", _shuffle_up(sd, p + "upsampling4.", c4, 2), 1)
    x4 = up_refinement(sd, p + "ref4x.", x4, f4, f8)
    up4 = _bilinear(up2, 2) + x4
    c8 = _spx(sd, p + "spx_8x.", torch.cat((_dm(sd, p + "dm8x.", up4), s2), 1))
    x8 = conv(sd, p + "tail8x.", _shuffle_up(sd, p + "upsampling8.", c8, 2), 1)
    x8 = up_refinement(sd, p + "ref8x.", x8, f8, s2)
    return [_bilinear(up4, 2) + x8, up4, up2]


def upsample16(sd: SD, p: str, f1: torch.Tensor, f2: torch.Tensor, f4: torch.Tensor, f8: torch.Tensor,
               init: torch.Tensor):
    """``upsample16.forward`` (ESMStereo.py:484-509), ESMStereo-S (two x4 stages)."""
    x = _spx(sd, p + "spx_2x.", torch.cat((_dm(sd, p + "dm2x.", init), f2), 1))
    x = F.conv2d(x, sd[p + "to_feat.weight"], None, 1, 1)
    x = fm_block(sd, p + "blocks.1.", fm_block(sd, p + "blocks.0.", x))
    x2 = conv(sd, p + "tail2x.", _shuffle_up(sd, p + "upsampling2.", x, 4), 1)
    x2 = up_refinement(sd, p + "ref2x.", x2, f2, f1)
    up2 = _bilinear(init, 4) + x2
    c4 = _spx(sd, p + "spx_4x.", torch.cat((_dm(sd, p + "dm4x.", up2), f4), 1))
    x4 = conv(sd, p + "tail4x.", _shuffle_up(sd, p + "upsampling4.", c4, 4), 1)
    x4 = up_refinement(sd, p + "ref4x.", x4, f4, f8)
    return [_bilinear(up2, 4) + x4, up2]


# ----------------------------------------------------------------------------- hot path


def hot_path(sd: SD, cv_scale: int, maxdisp: int, gwc: bool, ml: torch.Tensor, mr: torch.Tensor,
             att: Optional[torch.Tensor], up: List[torch.Tensor]) -> Dict[str, torch.Tensor]:
    """``ESMStereo.forward`` lines 700-745 from matching features to disparities.

    Returns the intermediates the golden fixtures hold: volume, stem, agg, cost, init_pred,
    disp_0.. (each disp already ``squeeze(1)*4``, eval output = ``disp_0``).
    """
    D = maxdisp // cv_scale
    out: Dict[str, torch.Tensor] = {}
    if gwc:
        vol = gwc_volume(ml, mr, D, 32)
        out["volume"] = vol
        if cv_scale == 16:
            vol = vol * att.unsqueeze(2)
        vol = basic_conv(sd, "group_stem.", vol, k=3, pad=1)
    else:
        vol = normcorr_volume(ml, mr, D)
        out["volume"] = vol
        vol = basic_conv(sd, "corr_stem.", vol, k=3, pad=1)
        if cv_scale == 16:
            vol = vol * att.unsqueeze(2)
    out["stem"] = vol
    vol = basic_conv(sd, "agg.", vol, k=3, pad=1)
    out["agg"] = vol
    cost = aggregation(sd, "aggregation_out.", vol)
    out["cost"] = cost
    c = cost.squeeze(1)
    if c.shape[1] != D:
        raise RuntimeError(f"aggregated depth {c.shape[1]} != D={D} (D must be even, SURVEY.md §0.4)")
    if cv_scale == 4:
        init = regression_topk2(c)
        disps = upsample4(sd, "upsample_module.", up[0], up[1], up[2], init)
    elif cv_scale == 8:
        init = disparity_regression(c, D).unsqueeze(1)
        disps = upsample8(sd, "upsample_module.", up[0], up[1], up[2], up[3], init)
    else:
        init = disparity_regression(c, D).unsqueeze(1)
        disps = upsample16(sd, "upsample_module.", up[0], up[1], up[2], up[3], init)
    out["init_pred"] = init
    for i, d in enumerate(disps):
        out[f"disp_{i}"] = d.squeeze(1) * 4
    return out
