"""ShuffleMixer blocks used by the ESM upsampler (reference ``models/shufflemixer.py``).

Parameter names match the reference state dict (``net.0.norm1.body.weight``,
``net.0.mlp1.fc.0.weight``, ``net.0.spatial.weight``, ``conv.0.weight`` ...).  The forward
of an ``FMBlock`` is four HIP launches:

1. ``smix``:  t1 = mlp1(LN1(x)) + x                                  (SMLayer 0, first half)
2. ``smix``:  t2 = dw7(t1) -> mlp2(LN2(.)) + . -> SMLayer 1's mlp1(LN1(.)) + .
3. ``smix``:  t3 = dw7(t2) -> mlp2(LN2(.)) + . ; t3 += x               (``net(x) + x``)
4. ``conv``:  y = conv1x1(SiLU(conv3x3(t3) + b)) + b + t3          (``conv(x) + x``)

For C in {8, 16} with the reference's 7x7 depthwise kernel (every ESMStereo upsampler) all four
are ONE launch (``esm_fmnet_f32``: halo recomputation, the hidden maps never leave the chip).
"""
from __future__ import annotations

import numbers
from typing import List

import torch
import torch.nn as nn

from .engine import ACT_NONE, ACT_SILU, Ctx, SmixStage, pack_conv, param_token, run_conv, run_fmnet, run_smix

__all__ = ["BiasFree_LayerNorm", "LayerNorm", "SplitPointMlp", "SMLayer", "FMBlock"]


class BiasFree_LayerNorm(nn.Module):
    """Per-pixel LayerNorm over channels with a weight and no bias; the mean IS subtracted
    (reference shufflemixer.py:47-62)."""

    def __init__(self, normalized_shape) -> None:
        super().__init__()
        if isinstance(normalized_shape, numbers.Integral):
            normalized_shape = (normalized_shape,)
        self.normalized_shape = torch.Size(normalized_shape)
        assert len(self.normalized_shape) == 1
        self.weight = nn.Parameter(torch.ones(self.normalized_shape))


class LayerNorm(nn.Module):
    """Wrapper holding ``body`` (reference shufflemixer.py:83-93); only 'BiasFree' is used by ESMStereo."""

    def __init__(self, dim: int, LayerNorm_type: str = "BiasFree") -> None:
        super().__init__()
        if LayerNorm_type != "BiasFree":
            raise NotImplementedError("ESMStereo uses the BiasFree LayerNorm only")
        self.body = BiasFree_LayerNorm(dim)


class SplitPointMlp(nn.Module):
    """1x1 MLP on the first half of the channels, then the (g d)->(d g) shuffle, g = 8
    (reference shufflemixer.py:23-37)."""

    def __init__(self, dim: int, mlp_ratio: int = 2) -> None:
        super().__init__()
        hidden = int(dim // 2 * mlp_ratio)
        self.fc = nn.Sequential(nn.Conv2d(dim // 2, hidden, 1, 1, 0), nn.SiLU(inplace=True),
                                nn.Conv2d(hidden, dim // 2, 1, 1, 0))


def _stage(norm: LayerNorm, mlp: SplitPointMlp) -> SmixStage:
    f0, f2 = mlp.fc[0], mlp.fc[2]
    C = norm.body.weight.numel()
    if f0.weight.shape[0] != C:
        raise NotImplementedError("smix kernel assumes mlp_ratio = 2 (hidden = C)")
    return SmixStage(norm.body.weight.detach().float().contiguous(), f0.weight.detach().float().reshape(C, C // 2).contiguous(),
                     f0.bias.detach().float().contiguous(), f2.weight.detach().float().reshape(C // 2, C).contiguous(),
                     f2.bias.detach().float().contiguous())


class SMLayer(nn.Module):
    """Shuffle mixing layer (reference shufflemixer.py:97-112)."""

    def __init__(self, dim: int, kernel_size: int, mlp_ratio: int = 2) -> None:
        super().__init__()
        self.norm1 = LayerNorm(dim)
        self.norm2 = LayerNorm(dim)
        self.spatial = nn.Conv2d(dim, dim, kernel_size, 1, kernel_size // 2, groups=dim)
        self.mlp1 = SplitPointMlp(dim, mlp_ratio)
        self.mlp2 = SplitPointMlp(dim, mlp_ratio)

    def stages(self):
        return _stage(self.norm1, self.mlp1), _stage(self.norm2, self.mlp2)

    def dw(self):
        return self.spatial.weight.detach().float().contiguous(), self.spatial.bias.detach().float().contiguous()

    def emit(self, ctx: Ctx, x: torch.Tensor) -> torch.Tensor:
        s1, s2 = self.stages()
        t = run_smix(ctx, x, [s1])
        return run_smix(ctx, t, [s2], dw=self.dw())

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.emit(Ctx(x.device), x.contiguous())


class FMBlock(nn.Module):
    """Feature mixing block (reference shufflemixer.py:116-132)."""

    def __init__(self, dim: int, kernel_size: int, mlp_ratio: int = 2) -> None:
        super().__init__()
        self.net = nn.Sequential(SMLayer(dim, kernel_size, mlp_ratio), SMLayer(dim, kernel_size, mlp_ratio))
        self.conv = nn.Sequential(nn.Conv2d(dim, dim + 16, 3, 1, 1), nn.SiLU(inplace=True),
                                  nn.Conv2d(dim + 16, dim, 1, 1, 0))
        self._esm = None

    def _packed(self):
        tok = param_token(*self.modules())
        if self._esm is None or self._esm[0] != tok:
            l0, l1 = self.net[0], self.net[1]
            a1, a2 = l0.stages()
            b1, b2 = l1.stages()
            c0, c2 = self.conv[0], self.conv[2]
            cw = None
            if c0.bias is not None and c2.bias is not None and c0.out_channels == c0.in_channels + 16:
                cw = tuple(t.detach().float().contiguous() for t in (c0.weight, c0.bias, c2.weight, c2.bias))
            self._esm = (tok, dict(a1=a1, a2=a2, b1=b1, b2=b2, dw0=l0.dw(), dw1=l1.dw(), cw=cw,
                                   c0=pack_conv(c0, act=ACT_SILU), c2=pack_conv(c2, act=ACT_NONE)))
        return self._esm[1]

    def emit(self, ctx: Ctx, x: torch.Tensor) -> torch.Tensor:
        p = self._packed()
        me = getattr(self, "_esm_name", "FMBlock")
        if int(x.shape[1]) in (8, 16) and int(p["dw0"][0].shape[-1]) == 7:
            if p["cw"] is not None:
                # the whole block (net + x, then conv + residual) as one launch
                return run_fmnet(ctx, x, [p["a1"], p["a2"], p["b1"], p["b2"]], p["dw0"], p["dw1"], conv=p["cw"],
                                 tag=f"{me}")
            # the two SMLayers + x as one launch (the same operations as the three below)
            t3 = run_fmnet(ctx, x, [p["a1"], p["a2"], p["b1"], p["b2"]], p["dw0"], p["dw1"], tag=f"{me}.net")
        else:
            t1 = run_smix(ctx, x, [p["a1"]], tag=f"{me}.net.0.mlp1")
            t2 = run_smix(ctx, t1, [p["a2"], p["b1"]], dw=p["dw0"], tag=f"{me}.net.0.spatial+mlp2+net.1.mlp1")
            t3 = run_smix(ctx, t2, [p["b2"]], dw=p["dw1"], res=x, tag=f"{me}.net.1.spatial+mlp2+res")
        # conv.0 (3x3 + SiLU), then conv.2 (1x1) + residual
        h = run_conv(ctx, p["c0"], [t3], tag=f"{me}.conv.0")
        return run_conv(ctx, p["c2"], [h], res=t3, tag=f"{me}.conv.2")

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.emit(Ctx(x.device), x.contiguous())


def fm_blocks_emit(ctx: Ctx, blocks: List[FMBlock], x: torch.Tensor) -> torch.Tensor:
    for b in blocks:
        x = b.emit(ctx, x)
    return x
