"""Pin the confidence-head oracle (oracle/conf_oracle.py) to golden vectors produced by running
the reference ``LAFNet_ESM`` itself (tests/golden/make_golden_conf.py)."""
import json
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN_DIR, load_golden, load_spec, seeded_state
from oracle import conf_oracle as CO

with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
    MANIFEST = json.load(f)
CONF = sorted(k for k in MANIFEST if k.startswith("conf_"))


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def rel_err(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


@pytest.mark.parametrize("name", CONF)
def test_conf_oracle_golden(name):
    m = MANIFEST[name]
    g = load_golden(name)
    sd = seeded_state(load_spec(m["spec"]), m["seed"])
    keep = {}
    with torch.no_grad():
        out = CO.lafnet(sd, "", _t(g["cost"]), _t(g["disp"]), _t(g["imag"]), _t(g["left_f1x"]), _t(g["left_f2x"]),
                        keep=keep)
    # the same torch ops in the same order as the reference: agreement to fp32 rounding
    assert rel_err(keep["out4"], g["out4"]) < 1e-5
    assert rel_err(keep["out1"], g["out1"]) < 1e-5
    assert rel_err(out, g["conf"]) < 1e-5


def test_cost_features_topk_sorted():
    g = torch.Generator().manual_seed(3)
    cost = torch.randn(2, 12, 4, 5, generator=g)
    f = CO.cost_features(cost)
    assert f.shape == (2, 7, 4, 5)
    assert bool((f[:, :-1] >= f[:, 1:]).all())


def test_lafnet_state_dict_matches_reference_spec():
    """esmstereo_amd.LAFNet_ESM has the reference module's state-dict keys and shapes, in order
    (checkpoints of models/ESMStereo_confidence.py load unchanged)."""
    import esmstereo_amd as E
    spec = load_spec("spec_conf.json")
    sd = E.LAFNet_ESM(16).state_dict()
    assert [(k, list(v.shape)) for k, v in sd.items()] == [(k, s) for k, s, _ in spec]


def test_confidence_model_keys():
    import esmstereo_amd as E
    from esmstereo_amd.backbone import StubFeature
    base = E.ESMStereo(192, True, False, "mobilenetv2_100", 16, feature_cls=StubFeature).state_dict()
    conf = E.ESMStereo_confidence(192, True, False, "mobilenetv2_100", 16, feature_cls=StubFeature).state_dict()
    extra = [k for k in conf if k not in base]
    assert all(k.startswith("confidence_net.") for k in extra) and set(base) <= set(conf)
    assert len(extra) == len(load_spec("spec_conf.json"))
    assert "ESMStereo_confidence" in E.__models__
