"""Checkpoint compatibility: the reference's checkpoints are
``torch.save({'model': DataParallel(model).state_dict(), ...})`` and every caller loads them with
the key-filtered partial update of test_kitti.py:56-60 (same in save_disp.py / test_mid.py).

CPU:
* a file in that format round-trips into the drop-in module (names, shapes, values), with the
  timm-layout backbone (``module.feature.conv_stem.weight``, ``module.feature.block3.1.*`` ...)
  included, so a reference checkpoint's backbone tensors are not dropped by the key filter;
* a checkpoint whose backbone keys do not match (here: the round-1 stub layout) loads the hot
  path but warns that the backbone keeps its random weights (no silent mis-load).
GPU: loading a second checkpoint into a model that already ran invalidates the packed,
BN-folded weights and the compiled launch plan (outputs follow the new weights)."""
import warnings

import pytest
import torch

import esmstereo_amd as E
from esmstereo_amd.backbone import StubFeature
from helpers import load_golden, load_spec, seeded_state


def _reference_style_load(model, path):
    """test_kitti.py:56-60, verbatim in behaviour."""
    state_dict = torch.load(path, weights_only=True)
    model_dict = model.state_dict()
    pre_dict = {k: v for k, v in state_dict["model"].items() if k in model_dict}
    model_dict.update(pre_dict)
    model.load_state_dict(model_dict)
    return pre_dict


def _randomise(model, seed):
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for v in model.state_dict().values():
            if v.is_floating_point():
                v.copy_(torch.rand(v.shape, generator=g) + 0.5)


@pytest.mark.parametrize("var,backbone,cvs", [("L", "efficientnet_b2", 4), ("S", "mobilenetv2_100", 16)])
def test_reference_format_checkpoint_round_trip(tmp_path, var, backbone, cvs):
    src = E.ESMStereo(192, True, False, backbone, cvs)
    _randomise(src, 7)
    path = tmp_path / f"esmstereo_{var}.ckpt"
    ckpt = {"epoch": 3, "model": torch.nn.DataParallel(src).state_dict(), "optimizer": {}}
    ckpt["model"]["module.auxiliary_head.weight"] = torch.zeros(3)  # not in the model: filtered out
    torch.save(ckpt, path)

    dst = torch.nn.DataParallel(E.ESMStereo(192, True, False, backbone, cvs))
    with warnings.catch_warnings():
        warnings.simplefilter("error")  # every backbone tensor loads: no random-backbone warning
        loaded = _reference_style_load(dst, path)
    assert "module.auxiliary_head.weight" not in loaded
    want = src.state_dict()
    assert set(loaded) == {"module." + k for k in want}
    assert any(k.startswith("module.feature.block4.") for k in loaded)
    got = dst.module.state_dict()
    for k, v in want.items():
        assert torch.equal(got[k], v), k


def test_stub_layout_checkpoint_into_stub_model(tmp_path):
    sd = seeded_state(load_spec("spec_L_gwc.json"), 7)
    src = E.ESMStereo(192, True, False, "efficientnet_b2", 4, feature_cls=StubFeature)
    src.load_state_dict(sd)
    path = tmp_path / "stub.ckpt"
    torch.save({"model": torch.nn.DataParallel(src).state_dict()}, path)
    dst = torch.nn.DataParallel(E.ESMStereo(192, True, False, "efficientnet_b2", 4, feature_cls=StubFeature))
    loaded = _reference_style_load(dst, path)
    assert set(loaded) == {"module." + k for k in sd}


def test_backbone_key_mismatch_warns(tmp_path):
    """A checkpoint of another backbone layout: the callers' key filter drops every feature.*
    tensor; the model says so instead of running a random backbone silently."""
    sd = seeded_state(load_spec("spec_L_gwc.json"), 7)
    path = tmp_path / "other_layout.ckpt"
    torch.save({"model": {"module." + k: v for k, v in sd.items()}}, path)
    dst = torch.nn.DataParallel(E.ESMStereo(192, True, False, "efficientnet_b2", 4))
    with pytest.warns(RuntimeWarning, match="backbone"):
        loaded = _reference_style_load(dst, path)
    assert loaded and not any(k.startswith("module.feature.") for k in loaded)
    assert torch.equal(dst.module.aggregation_out.conv1[0].conv.weight, sd["aggregation_out.conv1.0.conv.weight"])


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a ROCm GPU")
def test_reload_invalidates_packed_weights_and_plan(tmp_path):
    from oracle import esm_oracle as O

    dev = torch.device("cuda")
    g = load_golden("hot_S_gwc.npz")
    t = lambda k: torch.from_numpy(g[k])  # noqa: E731
    up = [t(f"up_{i}") for i in range(4)]
    args = (t("match_left").to(dev), t("match_right").to(dev), t("att").to(dev), [u.to(dev) for u in up])
    dp = torch.nn.DataParallel(E.ESMStereo(64, True, False, "mobilenetv2_100", 16, feature_cls=StubFeature),
                               device_ids=[0]).to(dev).eval()
    outs = []
    for seed in (11, 12):
        sd = seeded_state(load_spec("spec_S_gwc.json"), seed)
        path = tmp_path / f"s{seed}.ckpt"
        torch.save({"model": {"module." + k: v for k, v in sd.items()}}, path)
        _reference_style_load(dp, path)
        with torch.no_grad():
            out = dp.module.hot_path(*args)[0].cpu()
            ref = O.hot_path(sd, 16, 64, True, t("match_left"), t("match_right"), t("att"), up)["disp_0"]
        assert float((out - ref).abs().mean()) <= 1e-3, seed
        outs.append(out)
    assert not torch.equal(outs[0], outs[1])


def test_plan_key_sees_replaced_and_edited_parameters():
    """The compiled-plan cache key (ESMStereo._hot_param_token) changes when a hot-path weight is
    edited in place AND when a hot-path Parameter object is replaced; a backbone edit
    (out of the hot path) leaves it alone."""
    m = E.ESMStereo(64, True, False, "mobilenetv2_100", 16, feature_cls=StubFeature)
    t0 = m._hot_param_token()
    conv = m.aggregation_out.conv1[0].conv
    with torch.no_grad():
        conv.weight.add_(1.0)
    t1 = m._hot_param_token()
    assert t1 != t0
    conv.weight = torch.nn.Parameter(conv.weight.detach().clone())
    t2 = m._hot_param_token()
    assert t2 != t1
    with torch.no_grad():
        for p in m.feature.parameters():
            p.add_(1.0)
    assert m._hot_param_token() == t2


def test_confidence_head_weights_key_the_plan():
    """ESMStereo_confidence emits LAFNet_ESM into the hot path's plan, so its weights are part of the
    plan key: an in-place edit of a confidence_net weight invalidates the compiled plan."""
    m = E.ESMStereo_confidence(64, True, False, "mobilenetv2_100", 16, feature_cls=StubFeature)
    t0 = m._hot_param_token()
    w = next(m.confidence_net.parameters())
    with torch.no_grad():
        w.mul_(2.0)
    assert m._hot_param_token() != t0
