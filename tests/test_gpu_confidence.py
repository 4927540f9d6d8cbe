"""Confidence head (reference models/ESMStereo_confidence.py:511-974) on the GPU.

* each esm_conf_f32 stage against its oracle restatement (oracle/conf_oracle.py) at seeded sizes;
* LAFNet_ESM on the reference's own golden vectors (tests/golden/make_golden_conf.py);
* ESMStereo_confidence.forward: the head emitted into the hot path's plan reads the aggregated cost,
  init_pred and match_left in place; checked against the oracle chain (esm_oracle.hot_path ->
  conf_oracle.lafnet) on the same features.

Tolerances: the head sharpens its input (softmax(-100 x / ||x||) over the disparity axis), so the
fp32 rounding of differently ordered sums grows to ~1e-5 in the confidence; the bounds below are
absolute on sigmoid outputs in [0, 1].
"""
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import GOLDEN_DIR, load_golden, load_spec, seeded_state, stereo_pair

pytestmark = pytest.mark.gpu

import esmstereo_amd as E  # noqa: E402
from esmstereo_amd._lib import (CONF_ATTEND, CONF_COMBINE, CONF_COST_FEATURES, CONF_ENLARGE,  # noqa: E402
                                CONF_SIGMOID)
from esmstereo_amd.backbone import StubFeature  # noqa: E402
from esmstereo_amd.engine import Ctx  # noqa: E402
from oracle import conf_oracle as CO  # noqa: E402
from oracle import esm_oracle as O  # noqa: E402

DEV = torch.device("cuda")
with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
    MANIFEST = json.load(f)
CONF = sorted(k for k in MANIFEST if k.startswith("conf_"))


def cu(a):
    return torch.as_tensor(np.ascontiguousarray(a)).to(DEV)


def maxabs(a, b):
    return float((torch.as_tensor(a).double().cpu() - torch.as_tensor(b).double().cpu()).abs().max())


def _stage(op, xs, out_shape, B, C, D, H, W):
    out = torch.empty(out_shape, device=DEV)
    Ctx(DEV).conf(op, [x if x is None else x.contiguous() for x in xs], out, B, C, D, H, W)
    torch.cuda.synchronize()
    return out.cpu()


@pytest.mark.parametrize("B,D,H,W", [(1, 12, 6, 10), (2, 24, 5, 37), (1, 48, 3, 4)])
def test_cost_features_vs_oracle(B, D, H, W):
    g = torch.Generator().manual_seed(D + H)
    cost = torch.randn(B, D, H, W, generator=g)
    got = _stage(CONF_COST_FEATURES, [cost.to(DEV)], (B, 7, H, W), B, 0, D, H, W)
    assert maxabs(got, CO.cost_features(cost)) < 2e-6


def test_attend_vs_oracle():
    g = torch.Generator().manual_seed(5)
    B, C, H, W = 2, 16, 7, 19
    xs = [torch.randn(B, C, H, W, generator=g) for _ in range(3)]
    lg = torch.randn(B, 3, H, W, generator=g)
    got = _stage(CONF_ATTEND, [x.to(DEV) for x in xs] + [lg.to(DEV)], (B, 3 * C, H, W), B, C, 0, H, W)
    a = F.softmax(lg, 1)
    ref = torch.cat([xs[k] * a[:, k:k + 1] for k in range(3)], 1)
    assert maxabs(got, ref) < 1e-6


@pytest.mark.parametrize("B,C,H,W", [(1, 16, 6, 10), (2, 5, 9, 31)])
def test_enlarge_vs_grid_sample(B, C, H, W):
    g = torch.Generator().manual_seed(C)
    feat = torch.randn(B, C, H, W, generator=g)
    scale = 2 * torch.sigmoid(3 * torch.randn(B, 1, H, W, generator=g))  # 0..2, as the head's scale
    got = _stage(CONF_ENLARGE, [feat.to(DEV), scale.to(DEV)], (B, 9 * C, H, W), B, C, 0, H, W)
    big = F.grid_sample(feat, CO.enlarge_grid(scale), align_corners=True)  # [B, C, 3H, 3W]
    s2d = big.view(B, C, H, 3, W, 3).permute(0, 1, 3, 5, 2, 4).reshape(B, 9 * C, H, W)
    assert maxabs(got, s2d) < 2e-5  # the 4-term bilinear sum: contraction and order differ from torch CPU


def test_combine_vs_unfold():
    g = torch.Generator().manual_seed(9)
    B, H, W = 2, 5, 11
    lg = torch.randn(B, 9, 4 * H, 4 * W, generator=g)
    init = torch.randn(B, 1, H, W, generator=g)
    got = _stage(CONF_COMBINE, [lg.to(DEV), init.to(DEV)], (B, 1, 4 * H, 4 * W), B, 0, 0, H, W)
    unf = F.unfold(init, 3, 1, 1).reshape(B, -1, H, W)
    unf = F.interpolate(unf, (4 * H, 4 * W), mode="nearest").reshape(B, 9, 4 * H, 4 * W)
    ref = (unf * F.softmax(lg, 1)).sum(1).unsqueeze(1)
    assert maxabs(got, ref) < 2e-6


def test_sigmoid_and_bad_descriptor():
    x = torch.linspace(-30, 30, 1000)
    got = _stage(CONF_SIGMOID, [x.view(1, 1, 1, 1000).to(DEV)], (1, 1, 1, 1000), 1, 1, 0, 1, 1000)
    assert maxabs(got.view(-1), torch.sigmoid(x)) < 1e-7
    with pytest.raises(E.EsmError):  # D outside 7..64: refused before any launch
        _stage(CONF_COST_FEATURES, [torch.zeros(1, 5, 2, 2, device=DEV)], (1, 7, 2, 2), 1, 0, 5, 2, 2)


def _head(name):
    m = MANIFEST[name]
    net = E.LAFNet_ESM(16)
    net.load_state_dict(seeded_state(load_spec(m["spec"]), m["seed"]))
    return net.eval().to(DEV), m


@pytest.mark.parametrize("name", CONF)
def test_lafnet_golden(name):
    net, m = _head(name)
    g = load_golden(name)
    with torch.no_grad():
        out = net(cu(g["cost"]), cu(g["disp"]), cu(g["imag"]), cu(g["left_f1x"]), cu(g["left_f2x"]), DEV)
    assert out.shape == g["conf"].shape
    err = maxabs(out, g["conf"])
    print(name, "max |conf - reference|", err)
    assert err < 5e-5


@pytest.mark.parametrize("name", CONF)
def test_conf_upsample_stage_golden(name):
    """conf_up4 alone, from the reference's own init_conf-equivalent: the oracle fusion output."""
    net, m = _head(name)
    g = load_golden(name)
    sd = {k: v for k, v in net.state_dict().items()}
    sd = {k: v.cpu() for k, v in sd.items()}
    keep = {}
    with torch.no_grad():
        CO.lafnet(sd, "", *(torch.as_tensor(g[k]) for k in ("cost", "disp", "imag", "left_f1x", "left_f2x")),
                  keep=keep)
        init = keep["fusion_3"]
        out4 = net.conf_up4(cu(g["left_f1x"]), init.to(DEV))
    assert maxabs(out4, g["out4"]) < 5e-5


def test_confidence_model_forward():
    m = MANIFEST["hot_S_gwc.npz"]
    maxdisp = 192  # topk(7) over D = maxdisp / 16 needs D >= 7 (the fixture's maxdisp 64 gives D = 4)
    model = E.ESMStereo_confidence(maxdisp, True, False, m["backbone"], m["cv_scale"], feature_cls=StubFeature)
    spec = load_spec(m["spec"])
    sd = seeded_state(spec, m["seed"])
    conf_sd = seeded_state(load_spec("spec_conf.json"), 77)
    sd.update({"confidence_net." + k: v for k, v in conf_sd.items()})
    model.load_state_dict(sd)
    model = model.eval().to(DEV)
    left, right = (t.to(DEV) for t in stereo_pair(1, 128, 320, 5, max_shift=40))
    with torch.no_grad():
        disp, conf = model(left, right)
        ml, mr, att, up = model.prefix(left, right)
        plain = E.ESMStereo.forward(model, left, right, False)[0]
    B, H, W = disp.shape
    assert conf.shape == (B, H, W)
    assert torch.equal(disp, plain)  # the head does not disturb the disparity path
    # oracle chain on the same (device-computed) features
    cpu = lambda t: t.detach().float().cpu()  # noqa: E731
    sd_cpu = {k: v.float() for k, v in sd.items() if v.is_floating_point()}
    with torch.no_grad():
        inter = O.hot_path(sd_cpu, 16, maxdisp, True, cpu(ml), cpu(mr), cpu(att), [cpu(u) for u in up[:4]])
        ref = CO.lafnet(sd_cpu, "confidence_net.", inter["cost"].squeeze(1), inter["init_pred"], cpu(ml), cpu(up[4]),
                        cpu(up[2]))
    err = maxabs(conf, ref.squeeze(1))
    print("confidence model: max |conf - oracle|", err)
    assert err < 1e-3
    # an in-place edit of a confidence_net weight must reach the compiled plan: the
    # head's packed weights are part of the plan-cache key
    with torch.no_grad():
        last = list(model.confidence_net.parameters())[-1]  # the head's last layer: a smooth change
        last.add_(0.05)
        disp2, conf2 = model(left, right)
        sd2 = {k: v.detach().float().cpu() for k, v in model.state_dict().items() if v.is_floating_point()}
        ref2 = CO.lafnet(sd2, "confidence_net.", inter["cost"].squeeze(1), inter["init_pred"], cpu(ml), cpu(up[4]),
                         cpu(up[2]))
    assert torch.equal(disp2, disp)
    assert not torch.equal(conf2, conf)
    assert maxabs(conf2, ref2.squeeze(1)) < 1e-3


def test_confidence_small_maxdisp_raises():
    """D = maxdisp / 16 < 7: the reference's topk(k=7) raises; so does the head, before any launch."""
    m = MANIFEST["hot_S_gwc.npz"]
    model = E.ESMStereo_confidence(64, True, False, m["backbone"], 16, feature_cls=StubFeature).eval().to(DEV)
    x = torch.zeros(1, 3, 64, 128, device=DEV)
    with pytest.raises(RuntimeError):
        model(x, x)


def test_confidence_requires_cv16():
    model = E.ESMStereo_confidence(192, True, False, "efficientnet_b2", 4, feature_cls=StubFeature).eval().to(DEV)
    x = torch.zeros(1, 3, 64, 128, device=DEV)
    with pytest.raises(UnboundLocalError):
        model(x, x)
