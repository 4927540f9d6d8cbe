"""Shared test helpers: deterministic weights from a spec, synthetic stereo inputs.

Weights are drawn from ``numpy.random.default_rng(seed)`` (PCG64, stable across numpy
versions) in state-dict order, so golden fixtures only carry inputs, outputs, the
key/shape/kind spec and the seed.  BatchNorm running statistics are
randomised so BN folding is exercised.
"""
from __future__ import annotations

import json
import math
import os
import re
from typing import Dict, List, Sequence, Tuple

import numpy as np
import torch
import torch.nn as nn

GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

SpecEntry = Tuple[str, List[int], str]


def module_spec(model: nn.Module) -> List[SpecEntry]:
    """(key, shape, kind) for every state-dict entry, in state-dict order.

    ``kind`` selects the init distribution: conv / deconv / bias / bn_weight / bn_bias /
    bn_mean / bn_var / bn_count / ln_weight.
    """
    kinds: Dict[str, str] = {}
    for mname, mod in model.named_modules():
        prefix = mname + "." if mname else ""
        cls = type(mod).__name__
        if isinstance(mod, (nn.ConvTranspose2d, nn.ConvTranspose3d)):
            kinds[prefix + "weight"] = "deconv"
            kinds[prefix + "bias"] = "bias"
        elif isinstance(mod, (nn.Conv2d, nn.Conv3d)):
            kinds[prefix + "weight"] = "conv"
            kinds[prefix + "bias"] = "bias"
        elif isinstance(mod, (nn.BatchNorm2d, nn.BatchNorm3d)):
            kinds[prefix + "weight"] = "bn_weight"
            kinds[prefix + "bias"] = "bn_bias"
            kinds[prefix + "running_mean"] = "bn_mean"
            kinds[prefix + "running_var"] = "bn_var"
            kinds[prefix + "num_batches_tracked"] = "bn_count"
        elif cls.endswith("LayerNorm") and hasattr(mod, "weight") and isinstance(mod.weight, nn.Parameter):
            kinds[prefix + "weight"] = "ln_weight"
            if getattr(mod, "bias", None) is not None:
                kinds[prefix + "bias"] = "bn_bias"
    spec = []
    for k, v in model.state_dict().items():
        if k not in kinds:
            raise KeyError(f"no init kind for state-dict key {k}")
        kind = kinds[k]
        if kind == "deconv" and REFINE_HEAD.match(k):
            kind = "deconv_head"
        elif kind == "deconv" and COST_HEAD.match(k):
            kind = "deconv_cost_head"
        spec.append((k, list(v.shape), kind))
    return spec


# The residual heads of the ESM refinement stages (``upsample_module.ref*.conv1_up``) are drawn
# at 0.1x He scale, so the synthetic network adds small corrections to the upsampled
# disparity as a trained one does; at full He scale each x2/x4 stage multiplies the disparity
# magnitude and random-weight outputs reach 1e3-1e4 px, where "EPE <= 1e-3 px" would measure
# fp32 rounding at an unrealistic scale rather than parity.
REFINE_HEAD = re.compile(r"(^|\.)upsample_module\.ref\d+x\.conv1_up\.conv\.weight$")
# The aggregated-cost head (``aggregation_out.conv1_up``) at 0.25x: disparity_regression has no
# softmax, so at full scale sum_d cost[d]*d of a random net leaves [0, D);
# 0.25x keeps the initial disparity in the range a trained model produces.
COST_HEAD = re.compile(r"(^|\.)aggregation_out\.conv1_up\.conv\.weight$")
HEAD_GAIN = {"deconv_head": 0.1, "deconv_cost_head": 0.25}


def seeded_state(spec: Sequence[SpecEntry], seed: int) -> Dict[str, torch.Tensor]:
    rng = np.random.default_rng(seed)
    out: Dict[str, torch.Tensor] = {}
    for key, shape, kind in spec:
        shape = tuple(shape)
        n = int(np.prod(shape)) if shape else 1
        if kind == "conv":
            fan = int(np.prod(shape[1:]))
            a = rng.standard_normal(n) * math.sqrt(2.0 / fan)
        elif kind.startswith("deconv"):
            nd = len(shape) - 2
            fan = max(1, shape[0] * int(np.prod(shape[2:])) // (2 ** nd))
            a = rng.standard_normal(n) * math.sqrt(2.0 / fan) * HEAD_GAIN.get(kind, 1.0)
        elif kind == "bias" or kind == "bn_bias" or kind == "bn_mean":
            a = rng.uniform(-0.1, 0.1, n)
        elif kind == "bn_weight" or kind == "ln_weight":
            a = rng.uniform(0.8, 1.2, n)
        elif kind == "bn_var":
            a = rng.uniform(0.5, 1.5, n)
        elif kind == "bn_count":
            out[key] = torch.zeros(shape, dtype=torch.long)
            continue
        else:
            raise ValueError(kind)
        out[key] = torch.from_numpy(a.astype(np.float32).reshape(shape))
    return out


def load_spec(name: str) -> List[SpecEntry]:
    with open(os.path.join(GOLDEN_DIR, name)) as f:
        return [tuple(e) for e in json.load(f)]


def load_golden(name: str) -> Dict[str, np.ndarray]:
    with np.load(os.path.join(GOLDEN_DIR, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def stereo_pair(B: int, H: int, W: int, seed: int, max_shift: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Smooth random texture (sum of sinusoids, ImageNet-normalised range) and a
    right view shifted by a planar disparity field."""
    rng = np.random.default_rng(seed)
    yy, xx = np.meshgrid(np.arange(H, dtype=np.float64), np.arange(W + max_shift, dtype=np.float64), indexing="ij")
    left_full = np.zeros((B, 3, H, W + max_shift))
    for b in range(B):
        for c in range(3):
            acc = np.zeros_like(xx)
            for _ in range(8):
                fx, fy = rng.uniform(0.02, 0.35, 2)
                ph = rng.uniform(0, 2 * np.pi)
                acc += np.sin(fx * xx + fy * yy + ph)
            left_full[b, c] = acc / 2.0
    left = left_full[..., max_shift:]
    right = np.empty_like(left)
    disp = (np.linspace(0.1, 0.9, H)[:, None] * max_shift).astype(np.int64)  # planar in y
    for y in range(H):
        d = int(disp[y, 0])
        right[:, :, y, :] = left_full[:, :, y, max_shift - d: max_shift - d + W]
    right += rng.standard_normal(right.shape) * 0.05
    return (torch.from_numpy(left.astype(np.float32)), torch.from_numpy(right.astype(np.float32)))


def feature_pair(B: int, C: int, h: int, w: int, seed: int, D: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """Matching-feature pair whose correlation peaks at a per-row disparity < D."""
    rng = np.random.default_rng(seed)
    full = rng.standard_normal((B, C, h, w + D)).astype(np.float32)
    left = full[..., D:].copy()
    right = np.empty_like(left)
    for y in range(h):
        d = (3 * y + 1) % D
        right[:, :, y, :] = full[:, :, y, D - d: D - d + w]
    right += 0.1 * rng.standard_normal(right.shape).astype(np.float32)
    return torch.from_numpy(left), torch.from_numpy(right)


# ----------------------------------------------------------------------------- full-size fixtures
# Hot-path inputs at a BASELINE configuration, generated from a seed with numpy only (PCG64
# normals, then fixed-order float64 additions), so the GPU box regenerates them bit for bit (each
# fixture stores the SHA-256 of the bytes it was made from).  SURVEY.md §8(d) input: a smooth
# texture for the matching features with the right view shifted by a planar disparity field, so
# the cost volume is peaked; the upsampler features are smooth random maps.

# (channels, stride) of the upsampler feature inputs per cv_scale (models/ESMStereo.py:722,726,733)
UP_LAYOUT = {4: [(96, 8), (48, 4), (32, 2)], 8: [(240, 16), (96, 8), (24, 4), (32, 2)],
             16: [(32, 8), (32, 16), (24, 4), (24, 2)]}


def smooth_field(rng: np.random.Generator, shape: Sequence[int], k: int = 2) -> np.ndarray:
    """Normals box-blurred over the last two axes ((2k+1)^2 window), unit-ish scale, float32."""
    *lead, h, w = shape
    a = rng.standard_normal(tuple(lead) + (h + 2 * k, w + 2 * k))
    acc = np.zeros(tuple(lead) + (h + 2 * k, w), dtype=np.float64)
    for i in range(2 * k + 1):
        acc += a[..., i:i + w]
    out = np.zeros(tuple(lead) + (h, w), dtype=np.float64)
    for i in range(2 * k + 1):
        out += acc[..., i:i + h, :]
    return (out / (2 * k + 1)).astype(np.float32)


def fullsize_inputs(cv_scale: int, B: int, H: int, W: int, maxdisp: int, seed: int, att: bool):
    """(match_left, match_right, att or None, [upsampler features]) as float32 numpy arrays."""
    rng = np.random.default_rng(seed)
    h, w = H // cv_scale, W // cv_scale
    D = maxdisp // cv_scale
    tex = smooth_field(rng, (B, 64, h, w + D))
    ml = np.ascontiguousarray(tex[..., D:])
    mr = np.empty_like(ml)
    for y in range(h):  # right[x] = left texture at x - d(y), d planar in y within [0.1, 0.8] D
        d = int((0.1 + 0.7 * y / max(1, h - 1)) * D)
        mr[:, :, y, :] = tex[:, :, y, D - d: D - d + w]
    mr += (0.05 * rng.standard_normal(mr.shape)).astype(np.float32)
    a = (0.5 + rng.random((B, 32, h, w))).astype(np.float32) if att else None
    up = [smooth_field(rng, (B, c, H // s, W // s), 1) for c, s in UP_LAYOUT[cv_scale]]
    return ml, mr, a, up


def digest(*arrays) -> str:
    import hashlib
    hs = hashlib.sha256()
    for x in arrays:
        if x is not None:
            hs.update(np.ascontiguousarray(x).tobytes())
    return hs.hexdigest()
