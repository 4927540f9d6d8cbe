"""Checkpoint compatibility: the reference's checkpoints are
``torch.save({'model': DataParallel(model).state_dict(), ...})`` and every caller loads them with
the key-filtered partial update of test_kitti.py:56-60 (same in save_disp.py / test_mid.py).
CPU: a file in that format round-trips into the drop-in module (names, shapes, values).
GPU: loading a second checkpoint into a model that already ran invalidates the packed,
BN-folded weights and the compiled launch plan (outputs follow the new weights)."""
import pytest
import torch

import esmstereo_amd as E
from helpers import load_golden, load_spec, seeded_state


def _reference_style_load(model, path):
    """test_kitti.py:56-60, verbatim in behaviour."""
    state_dict = torch.load(path, weights_only=True)
    model_dict = model.state_dict()
    pre_dict = {k: v for k, v in state_dict["model"].items() if k in model_dict}
    model_dict.update(pre_dict)
    model.load_state_dict(model_dict)
    return pre_dict


def test_reference_format_checkpoint_round_trip(tmp_path):
    sd = seeded_state(load_spec("spec_L_gwc.json"), 7)
    src = E.ESMStereo(192, True, False, "efficientnet_b2", 4)
    src.load_state_dict(sd)
    path = tmp_path / "esmstereo_L.ckpt"
    ckpt = {"epoch": 3, "model": torch.nn.DataParallel(src).state_dict(), "optimizer": {}}
    ckpt["model"]["module.auxiliary_head.weight"] = torch.zeros(3)  # not in the model: filtered out
    torch.save(ckpt, path)

    dst = torch.nn.DataParallel(E.ESMStereo(192, True, False, "efficientnet_b2", 4))
    loaded = _reference_style_load(dst, path)
    assert "module.auxiliary_head.weight" not in loaded
    assert set(loaded) == {"module." + k for k in sd}
    got = dst.module.state_dict()
    for k, v in sd.items():
        assert torch.equal(got[k], v), k


@pytest.mark.gpu
@pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a ROCm GPU")
def test_reload_invalidates_packed_weights_and_plan(tmp_path):
    from oracle import esm_oracle as O

    dev = torch.device("cuda")
    g = load_golden("hot_S_gwc.npz")
    t = lambda k: torch.from_numpy(g[k])  # noqa: E731
    up = [t(f"up_{i}") for i in range(4)]
    args = (t("match_left").to(dev), t("match_right").to(dev), t("att").to(dev), [u.to(dev) for u in up])
    dp = torch.nn.DataParallel(E.ESMStereo(64, True, False, "mobilenetv2_100", 16), device_ids=[0]).to(dev).eval()
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
