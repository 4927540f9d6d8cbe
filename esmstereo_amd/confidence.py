"""The confidence head of ESMStereo-S (reference ``models/ESMStereo_confidence.py``).

``LAFNet_ESM`` (``:551-744``) and ``conf_upsample`` (``:511-548``) with the reference's class names,
constructor arguments and state-dict keys; ``ESMStereo_confidence`` (``:746-974``) is
:class:`esmstereo_amd.model.ESMStereo` plus ``confidence_net``, with ``forward(left, right) ->
[disp * 4, confidence]`` (``:974``).  Every step runs on the HIP library:

* each ``Conv2d + BatchNorm2d (+ ReLU)`` pair is one ``esm_conv_f32`` launch (bias folded into the
  BN shift, ReLU / sigmoid in the epilogue, ``2 * sigmoid`` as sigmoid + ``post_scale``);
* the three attention logits land in one ``[B, 3, h, w]`` buffer (channel-slice outputs);
* ``embed_conv2`` (k3 s3 p0 over the 3x-enlarged map) is a 1x1 conv over the 9C channels the
  enlarge stage writes space-to-depth, so the enlarged image and its grid are never formed;
* ``conf_spx`` (ConvTranspose2d k4 s4 p0, no overlap) is a 1x1 conv to 16 x 9 channels stored
  through the PixelShuffle(4) epilogue;
* the element-wise stages (cost features, attention, grid_sample, softmax-weighted x4 upsample,
  final sigmoid) are ``esm_conf_f32`` launches (csrc/confidence.hip).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ._lib import (ACT_NONE, ACT_RELU, ACT_SIGMOID, CONF_ATTEND, CONF_COMBINE, CONF_COST_FEATURES, CONF_ENLARGE,
                   CONF_SIGMOID)
from .blocks import BasicConv
from .engine import Ctx, pack_conv, param_token, require_device, run_conv

__all__ = ["conf_upsample", "LAFNet_ESM"]


def _as_conv2d(weight: torch.Tensor, bias) -> nn.Conv2d:
    """A 1x1 nn.Conv2d holding ``weight`` [Cout, Cin, 1, 1] (for pack_conv)."""
    m = nn.Conv2d(int(weight.shape[1]), int(weight.shape[0]), 1, bias=bias is not None).to(weight.device)
    m.weight.data = weight.detach().float().contiguous()
    if bias is not None:
        m.bias.data = bias.detach().float().contiguous()
    return m


class conf_upsample(nn.Module):
    """x4 confidence upsampling (reference ``ESMStereo_confidence.py:511-548``)."""

    def __init__(self, C: int, fc: int) -> None:
        super().__init__()
        self.conv1 = BasicConv(1, C, is_3d=False, bn=True, gelu=True, kernel_size=3, padding=1, stride=1, dilation=1)
        self.conv2 = BasicConv(C, C, is_3d=False, bn=True, gelu=True, kernel_size=3, padding=1, stride=2, dilation=1)
        self.conv1_up = BasicConv(C, 1, deconv=True, is_3d=False, bn=True, gelu=True, kernel_size=4, padding=1, stride=2)
        self.cm = nn.Sequential(BasicConv(1, C, is_3d=False, kernel_size=5, padding=1, stride=1),
                                BasicConv(C, C, is_3d=False, kernel_size=3, padding=1, stride=1),
                                BasicConv(C, C, is_3d=False, kernel_size=3, padding=1, stride=1),
                                BasicConv(C, C, is_3d=False, kernel_size=1, padding=1, stride=1))
        self.conf_spx_4 = nn.Sequential(BasicConv(C + fc, C, kernel_size=3, stride=1, padding=1),
                                        nn.Conv2d(C, C, 3, 1, 1, bias=False), nn.BatchNorm2d(C), nn.ReLU())
        self.conf_spx = nn.ConvTranspose2d(C, 9, kernel_size=4, stride=4, padding=0)
        self._esm = None

    def _packed(self):
        tok = param_token(self.conf_spx_4[1], self.conf_spx_4[2], self.conf_spx)
        if self._esm is None or self._esm[0] != tok:
            wt, bt = self.conf_spx.weight, self.conf_spx.bias  # [C, 9, 4, 4]: out (c9, 4y+i, 4x+j)
            w1 = wt.detach().permute(1, 2, 3, 0).reshape(-1, wt.shape[0], 1, 1)  # row c9*16 + 4i + j
            b1 = bt.detach().repeat_interleave(16) if bt is not None else None
            self._esm = (tok, {"spx4_1": pack_conv(self.conf_spx_4[1], self.conf_spx_4[2], ACT_RELU),
                               "spx": pack_conv(_as_conv2d(w1, b1), None, ACT_NONE)})
        return self._esm[1]

    def emit(self, ctx: Ctx, feat: torch.Tensor, init_conf: torch.Tensor) -> torch.Tensor:
        p = self._packed()
        me = getattr(self, "_esm_name", "conf_upsample")
        B, _, h, w = (int(v) for v in init_conf.shape)
        x = init_conf
        for m in self.cm:  # k5 p1, k3 p1, k3 p1, k1 p1: back to h x w
            x = m.emit(ctx, [x])
        x = self.conf_spx_4[0].emit(ctx, [x, feat])
        x = run_conv(ctx, p["spx4_1"], [x], tag=f"{me}.conf_spx_4.1")
        logits = run_conv(ctx, p["spx"], [x], shuffle=4, tag=f"{me}.conf_spx")  # [B, 9, 4h, 4w]
        conf1 = ctx.empty(B, 1, 4 * h, 4 * w)
        ctx.conf(CONF_COMBINE, [logits, init_conf], conf1, B, 0, 0, h, w, name=f"{me}.softmax+unfold")
        c = self.conv1.emit(ctx, [conf1])
        c = self.conv2.emit(ctx, [c])
        return self.conv1_up.emit(ctx, [c], res=conf1)

    def forward(self, left_f1x: torch.Tensor, init_conf: torch.Tensor) -> torch.Tensor:
        require_device(init_conf, "init_conf")
        return self.emit(Ctx(init_conf.device), left_f1x.contiguous(), init_conf.contiguous())


class LAFNet_ESM(nn.Module):
    """Confidence network (reference ``ESMStereo_confidence.py:551-744``)."""

    def __init__(self, C: int) -> None:
        super().__init__()
        self.C = C
        self.softmax = nn.Softmax(dim=1)
        for n, cin in (("cost", 7), ("disp", 1), ("imag", 64)):
            setattr(self, f"{n}_conv1", nn.Conv2d(cin, C, kernel_size=3, padding=1))
            setattr(self, f"{n}_bn1", nn.BatchNorm2d(C))
            setattr(self, f"{n}_conv2", nn.Conv2d(C, C, kernel_size=3, padding=1))
            setattr(self, f"{n}_bn2", nn.BatchNorm2d(C))
            setattr(self, f"{n}_conv3", nn.Conv2d(C, C, kernel_size=1, padding=0))
            setattr(self, f"{n}_bn3", nn.BatchNorm2d(C))
        for n in ("cost", "disp", "imag"):
            setattr(self, f"{n}_att_conv1", nn.Conv2d(C, C, kernel_size=3, padding=1))
            setattr(self, f"{n}_att_bn1", nn.BatchNorm2d(C))
            setattr(self, f"{n}_att_conv2", nn.Conv2d(C, 1, kernel_size=1, padding=0))
            setattr(self, f"{n}_att_bn2", nn.BatchNorm2d(1))
        self.softmax_att = nn.Softmax(dim=1)
        self.scale_conv1 = nn.Conv2d(C, C, kernel_size=3, padding=1)
        self.scale_bn1 = nn.BatchNorm2d(C)
        self.scale_conv2 = nn.Conv2d(C, C, kernel_size=3, padding=1)
        self.scale_bn2 = nn.BatchNorm2d(C)
        self.scale_conv3 = nn.Conv2d(C, 1, kernel_size=1, padding=0)
        self.scale_bn3 = nn.BatchNorm2d(1)
        self.embed_conv1 = nn.Conv2d(3 * C, C, kernel_size=3, padding=1)
        self.embed_bn1 = nn.BatchNorm2d(C)
        self.embed_conv2 = nn.Conv2d(C, C, kernel_size=3, padding=0, stride=3)
        self.embed_bn2 = nn.BatchNorm2d(C)
        # one conv per fusion layer, one BatchNorm per (layer, iteration), in the reference's order
        for i, (cin, cout, k) in enumerate(((C + 1, C, 3), (C, C, 3), (C, 1, 1)), start=1):
            setattr(self, f"fusion_conv{i}", nn.Conv2d(cin, cout, kernel_size=k, padding=k // 2))
            for it in (1, 2, 3):
                setattr(self, f"fusion_bn{i}_iter{it}", nn.BatchNorm2d(cout))
        self.sigmoid = nn.Sigmoid()
        self.conf_up4 = conf_upsample(C, 96)
        self.conf_up1 = conf_upsample(C, 24)
        for m in self.modules():  # the reference init (:630-637)
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)
        nn.init.constant_(self.scale_bn3.weight, 0)
        nn.init.constant_(self.scale_bn3.bias, 0)
        self._esm = None

    def _packed(self):
        own = [m for n, m in self.named_children() if not n.startswith("conf_up")]
        tok = param_token(*own)
        if self._esm is None or self._esm[0] != tok:
            g = lambda n: getattr(self, n)  # noqa: E731
            p = {}
            for n in ("cost", "disp", "imag"):
                for i in (1, 2, 3):
                    p[f"{n}{i}"] = pack_conv(g(f"{n}_conv{i}"), g(f"{n}_bn{i}"), ACT_RELU)
                p[f"{n}_att1"] = pack_conv(g(f"{n}_att_conv1"), g(f"{n}_att_bn1"), ACT_RELU)
                p[f"{n}_att2"] = pack_conv(g(f"{n}_att_conv2"), g(f"{n}_att_bn2"), ACT_NONE)
            p["embed1"] = pack_conv(self.embed_conv1, self.embed_bn1, ACT_RELU)
            p["scale1"] = pack_conv(self.scale_conv1, self.scale_bn1, ACT_RELU)
            p["scale2"] = pack_conv(self.scale_conv2, self.scale_bn2, ACT_RELU)
            p["scale3"] = pack_conv(self.scale_conv3, self.scale_bn3, ACT_SIGMOID)
            # k3 s3 p0 over the enlarged map == 1x1 over its space-to-depth channels c*9 + 3*ky + kx
            w2 = self.embed_conv2.weight.detach()
            p["embed2"] = pack_conv(_as_conv2d(w2.reshape(w2.shape[0], -1, 1, 1), self.embed_conv2.bias), self.embed_bn2,
                                    ACT_RELU)
            for it in (1, 2, 3):
                p[f"fus1_{it}"] = pack_conv(self.fusion_conv1, g(f"fusion_bn1_iter{it}"), ACT_RELU)
                p[f"fus2_{it}"] = pack_conv(self.fusion_conv2, g(f"fusion_bn2_iter{it}"), ACT_RELU)
                p[f"fus3_{it}"] = pack_conv(self.fusion_conv3, g(f"fusion_bn3_iter{it}"), ACT_RELU)
            self._esm = (tok, p)
        return self._esm[1]

    def emit(self, ctx: Ctx, cost: torch.Tensor, disp: torch.Tensor, imag: torch.Tensor, left_f1x: torch.Tensor,
             left_f2x: torch.Tensor) -> torch.Tensor:
        """The forward of :653-744 as library launches; returns the sigmoid confidence [B, 1, 16h, 16w]."""
        p = self._packed()
        me = getattr(self, "_esm_name", "confidence_net")
        C = self.C
        B, D, h, w = (int(v) for v in cost.shape)
        e = ctx.empty
        cf = e(B, 7, h, w)
        ctx.conf(CONF_COST_FEATURES, [cost], cf, B, 0, D, h, w, name=f"{me}.cost_topk7")
        feats = {}
        for n, src in (("cost", cf), ("disp", disp), ("imag", imag)):
            x = src
            for i in (1, 2, 3):
                x = run_conv(ctx, p[f"{n}{i}"], [x], tag=f"{me}.{n}_conv{i}")
            feats[n] = x
        logits = e(B, 3, h, w)
        for k, n in enumerate(("cost", "disp", "imag")):
            x = run_conv(ctx, p[f"{n}_att1"], [feats[n]], tag=f"{me}.{n}_att_conv1")
            run_conv(ctx, p[f"{n}_att2"], [x], out=logits[:, k:k + 1], tag=f"{me}.{n}_att_conv2")
        att = e(B, 3 * C, h, w)
        ctx.conf(CONF_ATTEND, [feats["cost"], feats["disp"], feats["imag"], logits], att, B, C, 0, h, w,
                 name=f"{me}.attention")
        feat = run_conv(ctx, p["embed1"], [att], tag=f"{me}.embed_conv1")
        x = run_conv(ctx, p["scale1"], [feat], tag=f"{me}.scale_conv1")
        x = run_conv(ctx, p["scale2"], [x], tag=f"{me}.scale_conv2")
        scale = run_conv(ctx, p["scale3"], [x], post_scale=2.0, tag=f"{me}.scale_conv3")
        big = e(B, 9 * C, h, w)
        ctx.conf(CONF_ENLARGE, [feat, scale], big, B, C, 0, h, w, name=f"{me}.grid_sample")
        feat = run_conv(ctx, p["embed2"], [big], tag=f"{me}.embed_conv2")
        out = e(B, 1, h, w)
        out.fill_(0.5)  # the constant first `out` (:718); written once, never by a launch
        for it in (1, 2, 3):
            x = run_conv(ctx, p[f"fus1_{it}"], [feat, out], tag=f"{me}.fusion_conv1.iter{it}")
            x = run_conv(ctx, p[f"fus2_{it}"], [x], tag=f"{me}.fusion_conv2.iter{it}")
            out = run_conv(ctx, p[f"fus3_{it}"], [x], tag=f"{me}.fusion_conv3.iter{it}")
        out4 = self.conf_up4.emit(ctx, left_f1x, out)
        out1 = self.conf_up1.emit(ctx, left_f2x, out4)
        conf = e(B, 1, 16 * h, 16 * w)
        ctx.conf(CONF_SIGMOID, [out1], conf, B, 1, 0, 16 * h, 16 * w, name=f"{me}.sigmoid")
        return conf

    def forward(self, cost, disp, imag, left_f1x, left_f2x, device=None) -> torch.Tensor:
        """Reference signature (:653); ``device`` is accepted and unused (inputs carry theirs)."""
        for t in (cost, disp, imag, left_f1x, left_f2x):
            require_device(t, "confidence input")
        with torch.no_grad():
            return self.emit(Ctx(cost.device), *(t.contiguous() for t in (cost, disp, imag, left_f1x, left_f2x)))
