"""Feature pyramid of the drop-in ``ESMStereo`` module.

The reference backbone (``models/ESMStereo.py:40-77``) is a timm ``features_only`` model,
``efficientnet_b2`` or ``mobilenetv2_100``, created with ``pretrained=True``, whose
``conv_stem``, ``bn1`` and ``blocks[0:1] / [1:2] / [2:3] / [3:5] / [5:6]`` are re-wrapped as
``conv_stem``, ``bn1``, ``act1 = ReLU6`` and ``block0 .. block4`` (``layers = [1, 2, 3, 5, 6]``,
``:47,55,62-66``).  timm is not installed here and its pretrained weights need the network, so
:class:`Feature` rebuilds the same module tree in plain PyTorch (MIOpen convolutions; the
backbone is not on the HIP hot path):

* the state-dict keys and shapes are timm's, so a reference checkpoint's ``module.feature.*``
  tensors load into it (``feature.conv_stem.weight``, ``feature.bn1.running_var``,
  ``feature.block0.0.0.conv_dw.weight``, ``feature.block3.1.2.se.conv_reduce.bias``, ...);
* the block internals follow timm's published EfficientNet / MobileNetV2 definitions
  (``DepthwiseSeparableConv``, ``InvertedResidual``, ``SqueezeExcite``, ``BatchNormAct2d``,
  symmetric ``get_padding`` padding, ``make_divisible`` channel rounding, ``ceil`` depth
  scaling), restated from the architecture strings below.

Parity against timm itself is UNPINNED (timm is absent, nothing in the reference holds backbone
outputs).  What is pinned (``tests/test_backbone.py``): the channel ladder and strides the
reference hard-codes (``:48,57``), and the published parameter counts of the two networks
(mobilenetv2_100 3,504,872 and efficientnet_b2 9,109,994 with their heads) reproduced by the
full seven-stage stacks built here.

:class:`StubFeature` is the five-conv placeholder of round 1.  The committed golden vectors
were generated with it standing in for the reference ``Feature`` (``tests/golden/make_golden.py``),
so the golden tests construct ``ESMStereo(..., feature_cls=StubFeature)``; nothing else uses it.
"""
from __future__ import annotations

import math
from typing import List, Optional, Tuple

import torch
import torch.nn as nn

BACKBONE_CHANS = {
    "efficientnet_b2": [16, 24, 48, 120, 208],
    "mobilenetv2_100": [16, 24, 32, 96, 160],
}

# timm architecture strings: (block type, repeats, kernel, stride, expansion, out channels, se ratio)
# efficientnet_b2 = _gen_efficientnet(channel_multiplier=1.1, depth_multiplier=1.2), act swish;
# mobilenetv2_100 = _gen_mobilenet_v2(1.0), act relu6, no SE.
_ARCH = {
    "efficientnet_b2": dict(
        stages=[("ds", 1, 3, 1, 1, 16, 0.25), ("ir", 2, 3, 2, 6, 24, 0.25), ("ir", 2, 5, 2, 6, 40, 0.25),
                ("ir", 3, 3, 2, 6, 80, 0.25), ("ir", 3, 5, 1, 6, 112, 0.25), ("ir", 4, 5, 2, 6, 192, 0.25),
                ("ir", 1, 3, 1, 6, 320, 0.25)],
        width=1.1, depth=1.2, stem=32, act="silu", head=1280),
    "mobilenetv2_100": dict(
        stages=[("ds", 1, 3, 1, 1, 16, 0.0), ("ir", 2, 3, 2, 6, 24, 0.0), ("ir", 3, 3, 2, 6, 32, 0.0),
                ("ir", 4, 3, 2, 6, 64, 0.0), ("ir", 3, 3, 1, 6, 96, 0.0), ("ir", 3, 3, 2, 6, 160, 0.0),
                ("ir", 1, 3, 1, 6, 320, 0.0)],
        width=1.0, depth=1.0, stem=32, act="relu6", head=1280),
}
_LAYERS = [1, 2, 3, 5, 6]  # models/ESMStereo.py:47,56


def make_divisible(v: float, divisor: int = 8, min_value: int = None, round_limit: float = 0.9) -> int:
    """timm ``make_divisible``: round to the divisor, never more than 10 % below ``v``."""
    min_value = min_value or divisor
    new_v = max(min_value, int(v + divisor / 2) // divisor * divisor)
    if new_v < round_limit * v:
        new_v += divisor
    return new_v


def get_padding(kernel_size: int, stride: int = 1, dilation: int = 1) -> int:
    """timm symmetric padding for ``pad_type=''``."""
    return ((stride - 1) + dilation * (kernel_size - 1)) // 2


def _act(kind: str) -> nn.Module:
    return nn.SiLU(inplace=True) if kind == "silu" else nn.ReLU6(inplace=True)


class BatchNormAct2d(nn.BatchNorm2d):
    """timm ``BatchNormAct2d``: BatchNorm2d (same parameters and buffers) + optional activation."""

    def __init__(self, num_features: int, act: str = "silu", apply_act: bool = True) -> None:
        super().__init__(num_features)
        self.drop = nn.Identity()
        self.act = _act(act) if apply_act else nn.Identity()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.act(self.drop(super().forward(x)))


class SqueezeExcite(nn.Module):
    """timm ``_efficientnet_blocks.SqueezeExcite``: mean over H, W -> 1x1 reduce -> act -> 1x1 expand
    -> sigmoid gate."""

    def __init__(self, in_chs: int, rd_channels: int, act: str) -> None:
        super().__init__()
        self.conv_reduce = nn.Conv2d(in_chs, rd_channels, 1, bias=True)
        self.act1 = _act(act)
        self.conv_expand = nn.Conv2d(rd_channels, in_chs, 1, bias=True)
        self.gate = nn.Sigmoid()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        s = x.mean((2, 3), keepdim=True)
        return x * self.gate(self.conv_expand(self.act1(self.conv_reduce(s))))


class DepthwiseSeparableConv(nn.Module):
    """timm ``DepthwiseSeparableConv`` ('ds'): dw conv -> BN+act -> SE -> pw conv -> BN (no act);
    residual when stride 1 and in == out."""

    def __init__(self, in_chs: int, out_chs: int, k: int, stride: int, se_ratio: float, act: str) -> None:
        super().__init__()
        self.has_skip = stride == 1 and in_chs == out_chs
        self.conv_dw = nn.Conv2d(in_chs, in_chs, k, stride, get_padding(k, stride), groups=in_chs, bias=False)
        self.bn1 = BatchNormAct2d(in_chs, act)
        self.aa = nn.Identity()
        self.se = SqueezeExcite(in_chs, round(in_chs * se_ratio), act) if se_ratio > 0 else nn.Identity()
        self.conv_pw = nn.Conv2d(in_chs, out_chs, 1, bias=False)
        self.bn2 = BatchNormAct2d(out_chs, act, apply_act=False)
        self.drop_path = nn.Identity()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.bn2(self.conv_pw(self.se(self.aa(self.bn1(self.conv_dw(x))))))
        return self.drop_path(y) + x if self.has_skip else y


class InvertedResidual(nn.Module):
    """timm ``InvertedResidual`` ('ir'): pw expand -> BN+act -> dw conv -> BN+act -> SE -> pw linear
    -> BN (no act); residual when stride 1 and in == out.  SE channels from the block input
    (``se_from_exp=False``: rd = round(mid * se_ratio / exp))."""

    def __init__(self, in_chs: int, out_chs: int, k: int, stride: int, exp: float, se_ratio: float, act: str) -> None:
        super().__init__()
        mid = make_divisible(in_chs * exp)
        self.has_skip = stride == 1 and in_chs == out_chs
        self.conv_pw = nn.Conv2d(in_chs, mid, 1, bias=False)
        self.bn1 = BatchNormAct2d(mid, act)
        self.conv_dw = nn.Conv2d(mid, mid, k, stride, get_padding(k, stride), groups=mid, bias=False)
        self.bn2 = BatchNormAct2d(mid, act)
        self.aa = nn.Identity()
        self.se = SqueezeExcite(mid, round(mid * se_ratio / exp), act) if se_ratio > 0 else nn.Identity()
        self.conv_pwl = nn.Conv2d(mid, out_chs, 1, bias=False)
        self.bn3 = BatchNormAct2d(out_chs, act, apply_act=False)
        self.drop_path = nn.Identity()

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        y = self.bn2(self.conv_dw(self.bn1(self.conv_pw(x))))
        y = self.bn3(self.conv_pwl(self.se(self.aa(y))))
        return self.drop_path(y) + x if self.has_skip else y


def build_stages(backbone: str) -> Tuple[int, str, List[nn.Sequential]]:
    """(stem channels, activation, the seven timm stages) of ``backbone``."""
    if backbone not in _ARCH:
        raise ValueError(f"unknown backbone {backbone!r}; expected one of {sorted(_ARCH)}")
    a = _ARCH[backbone]
    stem = make_divisible(a["stem"] * a["width"])
    cin = stem
    stages = []
    for kind, reps, k, s, exp, c, se in a["stages"]:
        cout = make_divisible(c * a["width"])
        n = max(1, math.ceil(reps * a["depth"]))  # depth_trunc='ceil', one block definition per stage
        blocks = []
        for i in range(n):
            stride = s if i == 0 else 1
            if kind == "ds":
                blocks.append(DepthwiseSeparableConv(cin, cout, k, stride, se, a["act"]))
            else:
                blocks.append(InvertedResidual(cin, cout, k, stride, exp, se, a["act"]))
            cin = cout
        stages.append(nn.Sequential(*blocks))
    return stem, a["act"], stages


def _he_init(module: nn.Module) -> None:
    for m in module.modules():
        if isinstance(m, nn.Conv2d):
            fan_out = m.kernel_size[0] * m.kernel_size[1] * m.out_channels // m.groups
            m.weight.data.normal_(0, math.sqrt(2.0 / fan_out))
            if m.bias is not None:
                m.bias.data.zero_()
        elif isinstance(m, nn.BatchNorm2d):
            m.weight.data.fill_(1.0)
            m.bias.data.zero_()


class Feature(nn.Module):
    """Reference ``Feature`` (models/ESMStereo.py:40-77) with timm's module tree and key names.

    Random (He) initialisation: the reference's ``pretrained=True`` weights are not fetchable
    offline; a reference checkpoint supplies them through ``load_state_dict``."""

    def __init__(self, backbone: str) -> None:
        super().__init__()
        self.backbone = backbone
        stem, act, stages = build_stages(backbone)
        self.chans = list(BACKBONE_CHANS[backbone])
        self.conv_stem = nn.Conv2d(3, stem, 3, 2, get_padding(3, 2), bias=False)
        self.bn1 = BatchNormAct2d(stem, act)
        self.act1 = nn.ReLU6()
        bounds = [0] + _LAYERS
        for i in range(5):
            setattr(self, f"block{i}", nn.Sequential(*stages[bounds[i]:bounds[i + 1]]))
        _he_init(self)

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        if fast_path_ok(self, x):
            return fast_features(self, x)
        x = self.act1(self.bn1(self.conv_stem(x)))
        x2 = self.block0(x)
        x4 = self.block1(x2)
        x8 = self.block2(x4)
        x16 = self.block3(x8)
        x32 = self.block4(x16)
        return [x2, x4, x8, x16, x32]


def full_param_count(backbone: str, num_classes: int = 1000) -> int:
    """Parameters of the whole timm classification network (stem, seven stages, conv_head +
    bn2, classifier): checks the stage definitions against the published totals."""
    stem, _, stages = build_stages(backbone)
    head = make_divisible(_ARCH[backbone]["head"] * _ARCH[backbone]["width"])
    last = stages[-1][-1]
    cout = last.conv_pwl.out_channels if isinstance(last, InvertedResidual) else last.conv_pw.out_channels
    n = 3 * stem * 9 + 2 * stem
    n += sum(p.numel() for s in stages for p in s.parameters())
    n += cout * head + 2 * head + head * num_classes + num_classes
    return n


class StubFeature(nn.Module):
    """Round-1 placeholder: five stride-2 ``conv3x3 -> BN -> ReLU6`` stages with the reference
    channel ladder.  Only the golden-vector tests use it (see the module docstring)."""

    def __init__(self, backbone: str) -> None:
        super().__init__()
        if backbone not in BACKBONE_CHANS:
            raise ValueError(f"unknown backbone {backbone!r}; expected one of {sorted(BACKBONE_CHANS)}")
        self.backbone = backbone
        self.chans = list(BACKBONE_CHANS[backbone])
        stages = []
        cin = 3
        for cout in self.chans:
            stages.append(nn.Sequential(
                nn.Conv2d(cin, cout, 3, 2, 1, bias=False),
                nn.BatchNorm2d(cout),
                nn.ReLU6(),
            ))
            cin = cout
        self.stages = nn.ModuleList(stages)

    def forward(self, x: torch.Tensor) -> List[torch.Tensor]:
        feats = []
        for stage in self.stages:
            x = stage(x)
            feats.append(x)
        return feats


# ----------------------------------------------------------------------------- HIP inference path
# The same blocks in eval mode with no autograd, launched on the HIP kernels of this package instead of MIOpen
# (round 5): every dense conv (the stem, the 1x1 expand / project convs) through esm_conv_f32 with its
# BatchNorm folded and the activation / residual in the epilogue, every depthwise conv through esm_dwconv_f32
# with its BatchNorm and activation.  On PyTorch-ROCm these were MIOpen's naive grouped-conv kernel
# (~55 us a launch at 192 x 624) plus separate BatchNorm and clamp kernels: 2.5 ms of the S-K forward's
# backbone side.  SqueezeExcite (EfficientNet only) stays in torch ops on its [B, C, 1, 1] vectors.
# Results agree with the modules' own forward to fp32 rounding (tests/test_gpu_backbone.py).


def fast_path_ok(mod: nn.Module, x: torch.Tensor) -> bool:
    return (not mod.training and x.is_cuda and x.dtype == torch.float32 and not torch.is_grad_enabled()
            and x.dim() == 4)


def _act_code(act: nn.Module) -> int:
    from .engine import ACT_NONE, ACT_RELU, ACT_RELU6, ACT_SILU
    if isinstance(act, nn.ReLU6):
        return ACT_RELU6
    if isinstance(act, nn.SiLU):
        return ACT_SILU
    if isinstance(act, nn.ReLU):
        return ACT_RELU
    if isinstance(act, nn.Identity):
        return ACT_NONE
    raise ValueError(f"backbone fast path: unsupported activation {act}")


def _conv_bn(ctx, owner: nn.Module, name: str, conv: nn.Conv2d, bn: nn.Module, x: torch.Tensor,
             res: Optional[torch.Tensor] = None) -> torch.Tensor:
    """conv (groups 1) -> BN(+act) as one esm_conv_f32 launch (BN folded into the epilogue)."""
    from .engine import cached_pack, pack_conv, run_conv
    act = _act_code(bn.act) if isinstance(bn, BatchNormAct2d) else 0
    pc = cached_pack(owner, name, (conv, bn), lambda: pack_conv(conv, bn, act), act)
    return run_conv(ctx, pc, [x], res=res, tag=name)


def _dw_bn(ctx, owner: nn.Module, conv: nn.Conv2d, bn: "BatchNormAct2d", x: torch.Tensor) -> torch.Tensor:
    """depthwise conv -> BN + act as one esm_dwconv_f32 launch."""
    from .engine import bn_affine, cached_pack, run_dwconv
    k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    if conv.groups != conv.in_channels or conv.out_channels != conv.in_channels or conv.bias is not None:
        raise ValueError("backbone fast path: expected a bias-free depthwise conv")

    def build():
        sc, sh = bn_affine(bn)
        return conv.weight.detach().float().reshape(conv.out_channels, k * k).contiguous(), sc, sh

    w, sc, sh = cached_pack(owner, "dw", (conv, bn), build)
    return run_dwconv(ctx, x, w, sc, sh, k, s, p, _act_code(bn.act), tag="dw")


def _se(se: nn.Module, x: torch.Tensor) -> torch.Tensor:
    if isinstance(se, nn.Identity):
        return x
    return se(x)


def fast_features(feat: "Feature", x: torch.Tensor) -> List[torch.Tensor]:
    """Feature.forward (models/ESMStereo.py:68-77) on the HIP kernels, eval mode."""
    from .engine import Ctx
    ctx = Ctx(x.device)
    y = _conv_bn(ctx, feat, "stem", feat.conv_stem, feat.bn1, x)
    if not isinstance(feat.bn1.act, nn.ReLU6):  # act1 = ReLU6 behind the model's own activation
        y = y.clamp_(0.0, 6.0)
    outs = []
    for i in range(5):
        for blk in getattr(feat, f"block{i}"):
            for b in (blk if isinstance(blk, nn.Sequential) else [blk]):
                inp = y
                if isinstance(b, DepthwiseSeparableConv):
                    y = _se(b.se, _dw_bn(ctx, b, b.conv_dw, b.bn1, y))
                    y = _conv_bn(ctx, b, "pw", b.conv_pw, b.bn2, y, res=inp if b.has_skip else None)
                elif isinstance(b, InvertedResidual):
                    y = _conv_bn(ctx, b, "pw", b.conv_pw, b.bn1, y)
                    y = _se(b.se, _dw_bn(ctx, b, b.conv_dw, b.bn2, y))
                    y = _conv_bn(ctx, b, "pwl", b.conv_pwl, b.bn3, y, res=inp if b.has_skip else None)
                else:
                    y = b(y)
        outs.append(y)
    return outs
