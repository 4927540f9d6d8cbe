"""Placeholder feature pyramid for the drop-in ``ESMStereo`` module.

The reference backbone is a timm ``efficientnet_b2`` / ``mobilenetv2_100``
``features_only`` model with ``pretrained=True`` (reference
``models/ESMStereo.py:40-77``).  timm is not installed here and pretrained weights
need network access, so the backbone is OUT OF SCOPE for this build (SURVEY.md
§2, §8(f) rank 1).  This stand-in keeps the reference's *interface*:

* attribute ``chans`` with the real channel ladder of each backbone
  (``ESMStereo.py:48,57``), and
* ``forward(x) -> [x2, x4, x8, x16, x32]`` at strides 2..32
  (``ESMStereo.py:68-77``),

so every downstream layer (FeatUp, stems, matching descriptor, the hot path)
sees tensors of exactly the reference's shapes.  It runs on PyTorch/MIOpen; it is
not part of the HIP hot path and its parameters do not follow timm's key names.
"""
from __future__ import annotations

from typing import List

import torch
import torch.nn as nn

BACKBONE_CHANS = {
    "efficientnet_b2": [16, 24, 48, 120, 208],
    "mobilenetv2_100": [16, 24, 32, 96, 160],
}


class StubFeature(nn.Module):
    """Five stride-2 ``conv3x3 -> BN -> ReLU6`` stages with the reference channel ladder."""

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
