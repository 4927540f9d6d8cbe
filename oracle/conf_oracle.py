"""CPU oracle for the ESMStereo confidence head — TEST INFRASTRUCTURE, NOT PRODUCT CODE.

Only ``tests/`` may import this module, as the checker.  The product path
(``esmstereo_amd.confidence``) never imports it and has no CPU fallback.

A from-scratch functional restatement (plain PyTorch fp32 on the CPU, weights passed as a state
dict with the reference's key names) of ``models/ESMStereo_confidence.py``:

* ``conf_upsample.forward`` ..... ``:511-548``
* ``LAFNet_ESM.forward`` ........ ``:551-744`` (``L2normalize`` ``:647-651``)

Pinning: ``tests/test_conf_oracle.py`` checks it against golden vectors produced by running the
reference module itself (``tests/golden/make_golden_conf.py``).
"""
from __future__ import annotations

from typing import Dict

import numpy as np
import torch
import torch.nn.functional as F

from .esm_oracle import basic_conv

SD = Dict[str, torch.Tensor]


def _bn(sd: SD, p: str, x: torch.Tensor) -> torch.Tensor:
    return F.batch_norm(x, sd[p + "running_mean"], sd[p + "running_var"], sd[p + "weight"], sd[p + "bias"],
                        False, 0.0, 1e-5)


def _cbr(sd: SD, conv: str, bn: str, x: torch.Tensor, pad: int, relu: bool = True, stride: int = 1) -> torch.Tensor:
    """``F.relu(bn(conv(x)))`` of LAFNet_ESM (conv with bias, eval BatchNorm)."""
    x = _bn(sd, bn + ".", F.conv2d(x, sd[conv + ".weight"], sd[conv + ".bias"], stride, pad))
    return F.relu(x) if relu else x


def cost_features(cost: torch.Tensor) -> torch.Tensor:
    """``topk(softmax(-L2normalize(cost) * 100), 7)`` values (:647-654)."""
    norm = (cost ** 2).sum(dim=1, keepdim=True) + 1e-6
    x = F.softmax(-(cost / norm ** 0.5) * 100, dim=1)
    return torch.topk(x, k=7, dim=1).values


def enlarge_grid(scale: torch.Tensor) -> torch.Tensor:
    """The 3x-enlarged sampling grid of :689-712 (x offsets scaled by 2/(w-1), y offsets not)."""
    b, _, h, w = scale.shape
    gw, gh = np.meshgrid(np.linspace(-1, 1, w), np.linspace(-1, 1, h))
    gh = torch.tensor(gh, dtype=torch.float).repeat(b, 1, 1, 1)
    gw = torch.tensor(gw, dtype=torch.float).repeat(b, 1, 1, 1)
    grid = torch.cat((gw, gh), 1).permute(0, 2, 3, 1)
    st = scale.permute(0, 2, 3, 1)
    step_y = 2 / (w - 1)
    g = torch.zeros(b, 3 * h, 3 * w, 2)
    for i, oy in enumerate((-1, 0, 1)):
        for j, ox in enumerate((-1, 0, 1)):
            g[:, i::3, j::3, :] = grid + torch.cat((ox * step_y * st, oy * st), 3)
    return g


def conf_upsample(sd: SD, p: str, feat: torch.Tensor, init_conf: torch.Tensor) -> torch.Tensor:
    """``conf_upsample.forward`` (:532-548): x4 confidence through softmax-weighted 3x3 neighbours."""
    x = basic_conv(sd, p + "cm.0.", init_conf, k=5, pad=1)
    x = basic_conv(sd, p + "cm.1.", x, k=3, pad=1)
    x = basic_conv(sd, p + "cm.2.", x, k=3, pad=1)
    x = basic_conv(sd, p + "cm.3.", x, k=1, pad=1)
    x = basic_conv(sd, p + "conf_spx_4.0.", torch.cat((x, feat), 1), k=3, pad=1)
    x = F.relu(_bn(sd, p + "conf_spx_4.2.", F.conv2d(x, sd[p + "conf_spx_4.1.weight"], None, 1, 1)))
    x = F.conv_transpose2d(x, sd[p + "conf_spx.weight"], sd[p + "conf_spx.bias"], 4, 0)
    sfm = F.softmax(x, 1)
    b, _, h, w = init_conf.shape
    unf = F.unfold(init_conf, 3, 1, 1).reshape(b, -1, h, w)
    unf = F.interpolate(unf, (h * 4, w * 4), mode="nearest").reshape(b, 9, h * 4, w * 4)
    conf1 = (unf * sfm).sum(1).unsqueeze(1)
    c = basic_conv(sd, p + "conv1.", conf1, k=3, pad=1)
    c = basic_conv(sd, p + "conv2.", c, k=3, s=2, pad=1)
    c = basic_conv(sd, p + "conv1_up.", c, k=4, s=2, pad=1, deconv=True)
    return c + conf1


def lafnet(sd: SD, p: str, cost, disp, imag, left_f1x, left_f2x, C: int = 16, keep=None) -> torch.Tensor:
    """``LAFNet_ESM.forward`` (:653-744) -> sigmoid confidence at 16x the cost resolution."""
    x = cost_features(cost)
    x = _cbr(sd, p + "cost_conv1", p + "cost_bn1", x, 1)
    x = _cbr(sd, p + "cost_conv2", p + "cost_bn2", x, 1)
    cost_x = _cbr(sd, p + "cost_conv3", p + "cost_bn3", x, 0)
    x = _cbr(sd, p + "disp_conv1", p + "disp_bn1", disp, 1)
    x = _cbr(sd, p + "disp_conv2", p + "disp_bn2", x, 1)
    disp_x = _cbr(sd, p + "disp_conv3", p + "disp_bn3", x, 0)
    x = _cbr(sd, p + "imag_conv1", p + "imag_bn1", imag, 1)
    x = _cbr(sd, p + "imag_conv2", p + "imag_bn2", x, 1)
    imag_x = _cbr(sd, p + "imag_conv3", p + "imag_bn3", x, 0)
    att = []
    for n, src in (("cost", cost_x), ("disp", disp_x), ("imag", imag_x)):
        x = _cbr(sd, p + f"{n}_att_conv1", p + f"{n}_att_bn1", src, 1)
        att.append(_cbr(sd, p + f"{n}_att_conv2", p + f"{n}_att_bn2", x, 0, relu=False))
    a = F.softmax(torch.cat(att, 1), 1)
    x = torch.cat((cost_x * a[:, 0:1], disp_x * a[:, 1:2], imag_x * a[:, 2:3]), 1)
    feat = _cbr(sd, p + "embed_conv1", p + "embed_bn1", x, 1)
    x = _cbr(sd, p + "scale_conv1", p + "scale_bn1", feat, 1)
    x = _cbr(sd, p + "scale_conv2", p + "scale_bn2", x, 1)
    scale = 2 * torch.sigmoid(_cbr(sd, p + "scale_conv3", p + "scale_bn3", x, 0, relu=False))
    feat_enlarge = F.grid_sample(feat, enlarge_grid(scale), align_corners=True)
    feat = _cbr(sd, p + "embed_conv2", p + "embed_bn2", feat_enlarge, 0, stride=3)
    b, _, h, w = disp.shape
    out = torch.zeros(b, 1, h, w) + 0.5
    for it in (1, 2, 3):
        x = torch.cat((feat, out), 1)
        x = _cbr(sd, p + "fusion_conv1", p + f"fusion_bn1_iter{it}", x, 1)
        x = _cbr(sd, p + "fusion_conv2", p + f"fusion_bn2_iter{it}", x, 1)
        out = _cbr(sd, p + "fusion_conv3", p + f"fusion_bn3_iter{it}", x, 0)
        if keep is not None:
            keep[f"fusion_{it}"] = out
    out4 = conf_upsample(sd, p + "conf_up4.", left_f1x, out)
    out1 = conf_upsample(sd, p + "conf_up1.", left_f2x, out4)
    if keep is not None:
        keep.update(out4=out4, out1=out1, scale=scale)
    return torch.sigmoid(out1)
