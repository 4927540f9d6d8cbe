"""Op-level drop-ins for the free functions of the reference ``models/submodule.py``.

Same names, argument meaning and failure class as the reference (``maxdisp`` here is
already the volume depth D, as at the call sites ``models/ESMStereo.py:701,708``); every
computation runs in a HIP kernel of ``libesmstereo_amd.so``.  Device tensors only.
"""
from __future__ import annotations

import torch

from .engine import Ctx, require_device

__all__ = ["build_gwc_volume", "build_concat_volume", "build_norm_correlation_volume", "disparity_regression",
           "regression_topk"]


def _feat_pair(refimg_fea: torch.Tensor, targetimg_fea: torch.Tensor):
    require_device(refimg_fea, "refimg_fea")
    require_device(targetimg_fea, "targetimg_fea")
    if refimg_fea.dim() != 4 or refimg_fea.shape != targetimg_fea.shape:
        raise RuntimeError(f"feature shapes must be equal [B,C,H,W]: {tuple(refimg_fea.shape)} vs "
                           f"{tuple(targetimg_fea.shape)}")
    return refimg_fea.contiguous(), targetimg_fea.contiguous()


def build_gwc_volume(refimg_fea: torch.Tensor, targetimg_fea: torch.Tensor, maxdisp: int, num_groups: int,
                     att: torch.Tensor = None) -> torch.Tensor:
    """``build_gwc_volume`` (submodule.py:151-161) -> [B, G, maxdisp, H, W].

    ``att`` ([B, G, H, W] or [B, G, 1, H, W]) optionally fuses the ESMStereo-S
    ``volume * att`` of ESMStereo.py:711 into the same kernel.
    """
    L, R = _feat_pair(refimg_fea, targetimg_fea)
    B, C, H, W = (int(v) for v in L.shape)
    assert C % num_groups == 0  # the reference asserts (submodule.py:145)
    V = torch.empty(B, num_groups, maxdisp, H, W, device=L.device, dtype=torch.float32)
    if maxdisp == 0 or V.numel() == 0:
        return V.zero_()
    if att is not None:
        require_device(att, "att")
        att = att.reshape(B, num_groups, H, W).contiguous()
    Ctx(L.device).gwc(L, R, att, V, B, C, H, W, int(maxdisp), int(num_groups))
    return V


def build_concat_volume(refimg_fea: torch.Tensor, targetimg_fea: torch.Tensor, maxdisp: int) -> torch.Tensor:
    """``build_concat_volume`` (submodule.py:129-140) -> [B, 2C, maxdisp, H, W]."""
    L, R = _feat_pair(refimg_fea, targetimg_fea)
    B, C, H, W = (int(v) for v in L.shape)
    V = torch.empty(B, 2 * C, maxdisp, H, W, device=L.device, dtype=torch.float32)
    if maxdisp == 0 or V.numel() == 0:
        return V.zero_()
    Ctx(L.device).concat(L, R, V, B, C, H, W, int(maxdisp))
    return V


def build_norm_correlation_volume(refimg_fea: torch.Tensor, targetimg_fea: torch.Tensor, maxdisp: int) -> torch.Tensor:
    """``build_norm_correlation_volume`` (submodule.py:191-200) -> [B, 1, maxdisp, H, W]."""
    L, R = _feat_pair(refimg_fea, targetimg_fea)
    B, C, H, W = (int(v) for v in L.shape)
    V = torch.empty(B, 1, maxdisp, H, W, device=L.device, dtype=torch.float32)
    if maxdisp == 0 or V.numel() == 0:
        return V.zero_()
    work = torch.empty(2, B, C, H, W, device=L.device, dtype=torch.float32)
    Ctx(L.device).normcorr(L, R, V, work, B, C, H, W, int(maxdisp))
    return V


def disparity_regression(x: torch.Tensor, maxdisp: int) -> torch.Tensor:
    """``disparity_regression`` (submodule.py:211-216): sum_d x[:, d] * d -> [B, H, W] (no softmax)."""
    assert len(x.shape) == 4
    require_device(x, "disparity_regression input")
    B, D, H, W = (int(v) for v in x.shape)
    if D != maxdisp:
        raise RuntimeError(f"The size of tensor a ({D}) must match the size of tensor b ({maxdisp}) at "
                           "non-singleton dimension 1")
    x = x.contiguous()
    out = torch.empty(B, H, W, device=x.device, dtype=torch.float32)
    Ctx(x.device).regression(0, x, out, B, D, H, W)
    return out


def _gather_samples(s: torch.Tensor, B: int, D: int, H: int, W: int) -> torch.Tensor:
    """The block of ``disparity_samples`` the reference's ``torch.gather(disparity_samples, 1, pool_ind)``
    (submodule.py:223) reads, with gather's failure class: no broadcasting (a 4-D tensor at least
    [B, ., H, W] in the non-gathered dims, else ``RuntimeError: Size does not match at dimension ...``),
    and every selected index must lie inside dim 1 (an index past it raises ``index ... is out of bounds``;
    here whenever dim 1 is shorter than D, since any of the D planes may be selected)."""
    require_device(s, "disparity_samples")
    if s.dim() != 4:
        raise RuntimeError("Index tensor must have the same number of dimensions as input tensor "
                           f"(disparity_samples {tuple(s.shape)}, index [B, k, H, W])")
    for d, n in ((0, B), (2, H), (3, W)):
        if int(s.shape[d]) < n:
            raise RuntimeError(f"Size does not match at dimension {d} expected index [{B}, k, {H}, {W}] to be "
                               f"smaller than self {list(s.shape)} apart from dimension 1")
    if int(s.shape[1]) < D:
        raise RuntimeError(f"index {D - 1} is out of bounds for dimension 1 with size {int(s.shape[1])}")
    return s[:B, :D, :H, :W].contiguous()


def regression_topk(cost: torch.Tensor, disparity_samples: torch.Tensor, k: int) -> torch.Tensor:
    """``regression_topk`` (submodule.py:218-225) -> [B, 1, H, W]: the top-k costs over D (value
    descending; ties -> lowest index, NaN first), softmax over them, the probability-weighted sum of
    ``disparity_samples`` at their indices (``None``: arange(D)).  The reference slices the sorted
    indices (``ind[:, :k]``), so k follows Python slicing: k > D takes all D, k <= -D or k = 0 none
    (a zero map)."""
    require_device(cost, "regression_topk cost")
    if cost.dim() != 4:
        raise RuntimeError(f"regression_topk: expected a [B, D, H, W] cost, got shape {tuple(cost.shape)}")
    B, D, H, W = (int(v) for v in cost.shape)
    ke = len(range(D)[:int(k)])
    out = torch.empty(B, 1, H, W, device=cost.device, dtype=torch.float32)
    if ke == 0 or out.numel() == 0:
        return out.zero_()
    cost = cost.contiguous()
    samples = None
    if disparity_samples is not None:
        samples = _gather_samples(disparity_samples, B, D, H, W)
    Ctx(cost.device).regression(1, cost, out, B, D, H, W, samples=samples, k=ke)
    return out
