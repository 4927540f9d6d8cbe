"""Pin the CPU oracle (oracle/esm_oracle.py) to golden vectors produced by the reference.

The goldens come from running /root/reference's own modules (tests/golden/make_golden.py).
Every hot-path intermediate must agree; the op-level functions must be bit-exact except
where the reference's reduction order is not reproducible (norm-corr: 1e-6 relative).
"""
import json
import os

import numpy as np
import pytest
import torch

from helpers import GOLDEN_DIR, load_golden, load_spec, seeded_state
from oracle import esm_oracle as O

with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
    MANIFEST = json.load(f)
HOT = sorted(k for k in MANIFEST if k.startswith("hot_"))


def _t(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def rel_err(a, b):
    a = torch.as_tensor(a, dtype=torch.float64)
    b = torch.as_tensor(b, dtype=torch.float64)
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def test_ops_golden():
    g = load_golden("ops.npz")
    assert torch.equal(O.gwc_volume(_t(g["gwc_L"]), _t(g["gwc_R"]), 8, 32), _t(g["gwc_out"]))
    assert torch.equal(O.gwc_volume(_t(g["gwc_L"]), _t(g["gwc_R"]), 8, 32) * _t(g["gwc_att"]), _t(g["gwc_att_out"]))
    assert torch.equal(O.concat_volume(_t(g["concat_L"]), _t(g["concat_R"]), 6), _t(g["concat_out"]))
    assert rel_err(O.normcorr_volume(_t(g["nc_L"]), _t(g["nc_R"]), 7), g["nc_out"]) < 1e-6
    assert torch.equal(O.disparity_regression(_t(g["reg_cost"]), 12), _t(g["reg_out"]))
    assert rel_err(O.regression_topk2(_t(g["topk_cost"])), g["topk_out"]) < 1e-6


@pytest.mark.parametrize("name", HOT)
def test_hot_path_golden(name):
    m = MANIFEST[name]
    g = load_golden(name)
    sd = seeded_state(load_spec(m["spec"]), m["seed"])
    up = [_t(g[f"up_{i}"]) for i in range(4) if f"up_{i}" in g]
    att = _t(g["att"]) if "att" in g else None
    with torch.no_grad():
        out = O.hot_path(sd, m["cv_scale"], m["maxdisp"], m["cv"] == "gwc", _t(g["match_left"]),
                         _t(g["match_right"]), att, up)
    for k in ["volume", "stem", "agg", "cost", "init_pred"] + [f"disp_{i}" for i in range(m["n_train_outputs"])]:
        assert out[k].shape == g[k].shape, k
        assert rel_err(out[k], g[k]) < 1e-5, (k, rel_err(out[k], g[k]))


def test_expected_raises_recorded():
    r = MANIFEST["raises"]
    assert r["S_oddD"].startswith("RuntimeError")
    assert r["L_oddD"].startswith("RuntimeError")
    assert r["S_hw_not_32"].startswith("RuntimeError")


FULL = sorted(k for k in MANIFEST if k.startswith("full_"))


@pytest.mark.parametrize("name", FULL)
def test_oracle_fullsize_vs_reference(name):
    """The oracle at BASELINE KITTI size (S-K gwc, L-K gwc, L-K nc) against the reference's own
    summaries of the same seeded inputs (tests/golden/make_golden.py --fullsize): cost samples / sum
    / L2 <= 1e-5 relative; disparities EPE <= 1e-3 (L: flip-masked, tests/parity.py)."""
    from parity import check_fullsize, fullsize_case

    torch.set_num_threads(min(8, os.cpu_count() or 1))
    m, g, (ml, mr, att, up) = fullsize_case(name)
    sd = seeded_state(load_spec(m["spec"]), m["weight_seed"])
    with torch.no_grad():
        out = O.hot_path(sd, m["cv_scale"], m["maxdisp"], m["cv"] == "gwc", _t(ml), _t(mr),
                         None if att is None else _t(att), [_t(u) for u in up])
    rep = check_fullsize(name, m, g, out["cost"][:, 0], out["init_pred"], out["disp_0"])
    print(name, rep)


def test_oracle_regression_topk_any_k_vs_reference():
    """oracle.regression_topk for k != 2 against the reference's own regression_topk outputs
    (tests/golden/topk_k.npz, tie-free costs; make_golden_topk.py), k > D included."""
    g = load_golden("topk_k.npz")
    for k in g["ks"].tolist():
        c, s = torch.from_numpy(g[f"cost_{k}"]), torch.from_numpy(g[f"samples_{k}"])
        got = O.regression_topk(c, s, k)
        assert torch.allclose(got, torch.from_numpy(g[f"out_{k}"]), rtol=1e-6, atol=1e-6), k
    c = torch.randn(2, 12, 3, 5)
    assert torch.equal(O.regression_topk(c, None, 2), O.regression_topk2(c))
