"""The timm-layout backbone (esmstereo_amd/backbone.py; reference
models/ESMStereo.py:40-77).  Parity against timm's own outputs is UNPINNED (timm is absent and
the reference holds no backbone vectors); pinned here: the channel ladder and strides the
reference hard-codes (:48,57), timm's key layout, and the published parameter counts of
mobilenetv2_100 (3,504,872) and efficientnet_b2 (9,109,994), which the seven-stage stacks
reproduce only if every stage's blocks, expansions, kernels and SE widths are right."""
import json
import os

import pytest
import torch

import esmstereo_amd as E
from esmstereo_amd.backbone import Feature, InvertedResidual, full_param_count
from helpers import GOLDEN_DIR, load_spec, module_spec


@pytest.mark.parametrize("backbone,count", [("mobilenetv2_100", 3_504_872), ("efficientnet_b2", 9_109_994)])
def test_published_parameter_counts(backbone, count):
    assert full_param_count(backbone) == count


@pytest.mark.parametrize("backbone,chans", [("mobilenetv2_100", [16, 24, 32, 96, 160]),
                                            ("efficientnet_b2", [16, 24, 48, 120, 208])])
def test_pyramid_channels_and_strides(backbone, chans):
    f = Feature(backbone).eval()
    assert f.chans == chans
    with torch.no_grad():
        outs = f(torch.randn(2, 3, 64, 96))
    assert [tuple(o.shape) for o in outs] == [(2, c, 64 >> (i + 1), 96 >> (i + 1)) for i, c in enumerate(chans)]


def test_timm_key_layout():
    sd = Feature("efficientnet_b2").state_dict()
    # stem + bn1 (BatchNormAct2d keeps BatchNorm2d's buffers), block0 = blocks[0:1] (two ds blocks with SE),
    # block3 = blocks[3:5] (stage 3 and stage 4), block4 = blocks[5:6]
    for k, shape in [("conv_stem.weight", (32, 3, 3, 3)), ("bn1.running_var", (32,)),
                     ("block0.0.0.conv_dw.weight", (32, 1, 3, 3)), ("block0.0.0.se.conv_reduce.weight", (8, 32, 1, 1)),
                     ("block0.0.1.conv_pw.weight", (16, 16, 1, 1)), ("block1.0.0.conv_pw.weight", (96, 16, 1, 1)),
                     ("block2.0.2.conv_dw.weight", (288, 1, 5, 5)), ("block3.0.3.conv_pwl.weight", (88, 528, 1, 1)),
                     ("block3.1.0.se.conv_expand.bias", (528,)), ("block3.1.3.conv_pwl.weight", (120, 720, 1, 1)),
                     ("block4.0.4.bn3.num_batches_tracked", ())]:
        assert tuple(sd[k].shape) == shape, k
    assert not any(k.startswith("block5") for k in sd)
    m = Feature("mobilenetv2_100").state_dict()
    assert tuple(m["block0.0.0.conv_pw.weight"].shape) == (16, 32, 1, 1) and not any(".se." in k for k in m)
    assert tuple(m["block3.1.2.conv_pwl.weight"].shape) == (96, 576, 1, 1)
    assert isinstance(Feature("mobilenetv2_100").block4[0][2], InvertedResidual)


@pytest.mark.parametrize("var,cv", [(v, c) for v in "SML" for c in ("gwc", "nc")])
def test_non_backbone_keys_match_reference(var, cv):
    """Everything outside feature.* keeps the reference's names and shapes (specs dumped from the
    reference modules by tests/golden/make_golden.py)."""
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        m = json.load(f)[f"hot_{var}_{cv}.npz"]
    model = E.ESMStereo(m["maxdisp"], cv == "gwc", cv == "nc", m["backbone"], m["cv_scale"])
    strip = lambda spec: [e for e in spec if not e[0].startswith("feature.")]  # noqa: E731
    assert strip(module_spec(model)) == strip([tuple(e) for e in load_spec(m["spec"])])
