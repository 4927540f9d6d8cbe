"""Generate the golden vectors that pin the oracle (and through it the HIP path).

Run in the build container only (it imports the reference from /root/reference):

    python tests/golden/make_golden.py               # fixture-size vectors (rewrites the manifest)
    python tests/golden/make_golden.py --fullsize    # + full-size summaries (BASELINE KITTI size)
    python tests/golden/make_golden.py --fullsize --only L_gwc_SF8,M_gwc_K   # just these cases

What it does (SURVEY.md §8(c) recipe):
* imports ``models/submodule.py``, ``models/shufflemixer.py`` and ``models/ESMStereo.py``
  from /root/reference through a synthetic package, with inert ``cv2``/``timm`` modules
  (``timm.create_model`` is never called because the module-global ``Feature`` is swapped
  for ``esmstereo_amd.backbone.StubFeature`` before construction);
* builds reference ``ESMStereo`` S/M/L models, draws every state-dict entry from a seeded
  PCG64 generator (``tests/helpers.py:seeded_state``), runs the reference forward
  (``ESMStereo.py:638-745``) and also the hot-path section (``:700-745``) step by step,
  saving its inputs, intermediates and outputs;
* runs the five op-level functions of ``models/submodule.py`` on small seeded inputs.

Only data is written (``.npz`` arrays, ``.json`` specs); no reference source travels.
"""
from __future__ import annotations

import importlib.util
import json
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from helpers import feature_pair, module_spec, seeded_state, stereo_pair  # noqa: E402
from esmstereo_amd.backbone import StubFeature  # noqa: E402

REF = "/root/reference"


def load_reference():
    for n in ("cv2", "timm"):
        sys.modules.setdefault(n, types.ModuleType(n))
    pkg = types.ModuleType("refmodels")
    pkg.__path__ = [REF + "/models"]
    sys.modules["refmodels"] = pkg

    def load(sub):
        spec = importlib.util.spec_from_file_location(f"refmodels.{sub}", f"{REF}/models/{sub}.py")
        m = importlib.util.module_from_spec(spec)
        sys.modules[spec.name] = m
        spec.loader.exec_module(m)
        return m

    sm = load("submodule")
    load("shufflemixer")
    es = load("ESMStereo")
    es.Feature = StubFeature  # module global used by ESMStereo.__init__ (ESMStereo.py:521)
    return sm, es


VARIANTS = {
    # name: (backbone, cv_scale)
    "S": ("mobilenetv2_100", 16),
    "M": ("efficientnet_b2", 8),
    "L": ("efficientnet_b2", 4),
}

CASES = [
    # (variant, cv, B, H, W, maxdisp, seed)
    ("S", "gwc", 2, 64, 128, 64, 11),
    ("S", "nc", 1, 64, 128, 64, 12),
    ("M", "gwc", 1, 64, 128, 64, 13),
    ("M", "nc", 1, 64, 128, 64, 14),
    ("L", "gwc", 1, 64, 128, 48, 15),
    ("L", "nc", 1, 64, 128, 48, 16),
]


def prefix(model, left, right):
    """Reference ESMStereo.forward lines 640-697 (backbone side), returning hot-path inputs."""
    fl = model.feature(left)
    fr = model.feature(right)
    vs = model.vol_size
    if vs in (4, 8):
        fl, fr = model.feature_up(fl, fr)
    stem_2x = model.stem_2(left)
    stem_2y = model.stem_2(right)
    stem_4x = model.stem_4(stem_2x)
    stem_4y = model.stem_4(stem_2y)
    att = None
    if vs == 4:
        ml = torch.cat((fl[0], stem_4x), 1)
        mr = torch.cat((fr[0], stem_4y), 1)
    elif vs == 8:
        stem_8x = model.stem_8(stem_4x)
        stem_8y = model.stem_8(stem_4y)
        ml = torch.cat((fl[1], stem_8x), 1)
        mr = torch.cat((fr[1], stem_8y), 1)
    else:
        stem_8x = model.stem_8(stem_4x)
        stem_8y = model.stem_8(stem_4y)
        stem_16x = model.stem_16(stem_8x)
        stem_16y = model.stem_16(stem_8y)
        ml = torch.cat((fl[3], stem_16x), 1)
        mr = torch.cat((fr[3], stem_16y), 1)
        att = model.semantic(fl[3])  # [B, 32|8, h, w]; the reference unsqueezes at :697
    ml = model.desc(model.conv(ml))
    mr = model.desc(model.conv(mr))
    if vs == 4:
        up = [fl[1], fl[0], stem_2x]
    elif vs == 8:
        up = [fl[2], fl[1], fl[0], stem_2x]
    else:
        up = [fl[2], model.conv_f2(fl[3]), fl[1], model.conv_f0(fl[0])]
    return ml, mr, att, up


def hot_path(sm, model, ml, mr, att, up):
    """Reference ESMStereo.forward lines 700-745 step by step, keeping intermediates."""
    D = model.maxdisp // model.vol_size
    vs = model.vol_size
    inter = {}
    if model.norm_correlation:
        volume = sm.build_norm_correlation_volume(ml, mr, D)
        inter["volume"] = volume
        volume = model.corr_stem(volume) * att.unsqueeze(2) if vs == 16 else model.corr_stem(volume)
    if model.gwc:
        volume = sm.build_gwc_volume(ml, mr, D, model.num_groups)
        inter["volume"] = volume
        volume = model.group_stem(volume * att.unsqueeze(2)) if vs == 16 else model.group_stem(volume)
    inter["stem"] = volume
    volume = model.agg(volume)
    inter["agg"] = volume
    cost = model.aggregation_out(volume)
    inter["cost"] = cost
    if vs == 4:
        ds = torch.arange(0, D, dtype=cost.dtype).view(1, D, 1, 1).repeat(cost.shape[0], 1, cost.shape[3], cost.shape[4])
        init = sm.regression_topk(cost.squeeze(1), ds, 2)
        outs = model.upsample_module(up[0], up[1], up[2], init)
    elif vs == 8:
        init = sm.disparity_regression(cost.squeeze(1), D).unsqueeze(1)
        outs = model.upsample_module(up[0], up[1], up[2], up[3], init)
    else:
        init = sm.disparity_regression(cost.squeeze(1), D).unsqueeze(1)
        outs = model.upsample_module(up[0], up[1], up[2], up[3], init)
    inter["init_pred"] = init
    for i, o in enumerate(outs):
        inter[f"disp_{i}"] = o.squeeze(1) * 4
    return inter


# Full-size configurations pinned to the reference itself: the hot path of
# ESMStereo.forward (:700-745) on seeded feature inputs (tests/helpers.py fullsize_inputs) at the
# BASELINE KITTI size.  Summaries only (the volumes are 3-184 MB): cost sum / L2 / 64 sampled
# voxels, per-pixel top-3 of the aggregated cost (the regression_topk flip analysis), init_pred
# in full, disp_0 sum / L2 and every 4th row and column.
FULL_CASES = [
    # (tag, variant, cv, B, H, W, maxdisp, weight seed, input seed)
    ("S_gwc_K", "S", "gwc", 1, 384, 1248, 192, 11, 101),
    ("L_gwc_K", "L", "gwc", 1, 384, 1248, 192, 15, 102),
    ("L_nc_K", "L", "nc", 1, 384, 1248, 192, 16, 103),
    # round 4: the other BASELINE configurations (configs[2] SceneFlow B=8 padded to 544x960, configs[4]
    # Middlebury padded to 1504x1024 md256) and ESMStereo-M at KITTI size
    ("L_gwc_SF8", "L", "gwc", 8, 544, 960, 192, 15, 201),
    ("L_gwc_Mid", "L", "gwc", 1, 1024, 1504, 256, 15, 401),
    ("M_gwc_K", "M", "gwc", 1, 384, 1248, 192, 13, 104),
]


def make_fullsize(sm, es):
    from helpers import digest, fullsize_inputs

    man = {}
    only = sys.argv[sys.argv.index("--only") + 1].split(",") if "--only" in sys.argv else None
    for tag, var, cv, B, H, W, maxdisp, wseed, iseed in FULL_CASES:
        if only and tag not in only:
            continue
        backbone, cv_scale = VARIANTS[var]
        model = es.ESMStereo(maxdisp, cv == "gwc", cv == "nc", backbone, cv_scale).eval()
        spec = module_spec(model)
        model.load_state_dict(seeded_state(spec, wseed))
        ml, mr, att, up = fullsize_inputs(cv_scale, B, H, W, maxdisp, iseed, att=cv_scale == 16)
        T = lambda a: None if a is None else torch.from_numpy(a)  # noqa: E731
        with torch.no_grad():
            inter = hot_path(sm, model, T(ml), T(mr), T(att), [T(u) for u in up])
        cost = inter["cost"][:, 0]  # [B, D, h, w]
        flat = cost.reshape(-1)
        rng = np.random.default_rng(iseed + 1000)
        idx = np.sort(rng.choice(flat.numel(), 64, replace=False)).astype(np.int64)
        sv, si = torch.sort(cost.double(), dim=1, descending=True, stable=True)
        d0 = inter["disp_0"]
        arrays = dict(
            cost_sum=np.float64(cost.double().sum()), cost_l2=np.float64(cost.double().norm()),
            cost_absmax=np.float64(cost.abs().max()), cost_idx=idx, cost_val=flat[idx].numpy(),
            top3_idx=si[:, :3].numpy().astype(np.int16), top3_val=sv[:, :3].numpy(),
            init_pred=inter["init_pred"].numpy(),
            disp0_sum=np.float64(d0.double().sum()), disp0_l2=np.float64(d0.double().norm()),
            disp0_sub=d0[:, ::4, ::4].numpy())
        np.savez_compressed(os.path.join(HERE, f"full_{tag}.npz"), **arrays)
        man[f"full_{tag}.npz"] = dict(variant=var, cv=cv, backbone=backbone, cv_scale=cv_scale, B=B, H=H, W=W,
                                      maxdisp=maxdisp, weight_seed=wseed, input_seed=iseed,
                                      spec=f"spec_{var}_{cv}.json", input_sha256=digest(ml, mr, att, *up),
                                      disp0_shape=list(d0.shape))
        print(tag, {k: getattr(v, "shape", ()) for k, v in arrays.items()})
    return man


def main():
    torch.set_num_threads(8)
    if "--fullsize" in sys.argv:  # add the full-size fixtures to an existing manifest
        sm, es = load_reference()
        with open(os.path.join(HERE, "manifest.json")) as f:
            manifest = json.load(f)
        manifest.update(make_fullsize(sm, es))
        with open(os.path.join(HERE, "manifest.json"), "w") as f:
            json.dump(manifest, f, indent=1)
        return
    sm, es = load_reference()
    manifest = {}
    for (var, cv, B, H, W, maxdisp, seed) in CASES:
        backbone, cv_scale = VARIANTS[var]
        gwc, nc = cv == "gwc", cv == "nc"
        model = es.ESMStereo(maxdisp, gwc, nc, backbone, cv_scale).eval()
        spec = module_spec(model)
        model.load_state_dict(seeded_state(spec, seed))
        spec_name = f"spec_{var}_{cv}.json"
        with open(os.path.join(HERE, spec_name), "w") as f:
            json.dump(spec, f)
        left, right = stereo_pair(B, H, W, seed, max_shift=maxdisp // 2)
        with torch.no_grad():
            full_eval = model(left, right, False)
            full_train = model(left, right, True)
            ml, mr, att, up = prefix(model, left, right)
            inter = hot_path(sm, model, ml, mr, att, up)
        # the step-by-step hot path must reproduce the reference forward exactly
        assert torch.equal(inter["disp_0"], full_eval[0]), "hot-path replay diverged from forward"
        for i, t in enumerate(full_train):
            assert torch.equal(inter[f"disp_{i}"], t)
        arrays = {"left": left, "right": right, "match_left": ml, "match_right": mr}
        if att is not None:
            arrays["att"] = att
        for i, u in enumerate(up):
            arrays[f"up_{i}"] = u
        arrays.update(inter)
        name = f"hot_{var}_{cv}.npz"
        np.savez_compressed(os.path.join(HERE, name), **{k: v.detach().numpy() for k, v in arrays.items()})
        manifest[name] = dict(variant=var, cv=cv, backbone=backbone, cv_scale=cv_scale, B=B, H=H, W=W,
                              maxdisp=maxdisp, seed=seed, spec=spec_name, n_train_outputs=len(full_train))
        print(name, {k: tuple(v.shape) for k, v in arrays.items()})

    # expected-raise cases
    raises = {}
    for tag, (var, cv, H, W, maxdisp) in {
        "S_oddD": ("S", "gwc", 128, 256, 48),
        "L_oddD": ("L", "gwc", 64, 128, 52),
        "S_hw_not_32": ("S", "gwc", 80, 128, 64),
    }.items():
        backbone, cv_scale = VARIANTS[var]
        model = es.ESMStereo(maxdisp, cv == "gwc", cv == "nc", backbone, cv_scale).eval()
        left, right = stereo_pair(1, H, W, 1, max_shift=8)
        try:
            with torch.no_grad():
                model(left, right, False)
            raises[tag] = None
        except Exception as e:  # noqa: BLE001 - we record what the reference raises
            raises[tag] = f"{type(e).__name__}: {e}"
        print(tag, raises[tag])
    manifest["raises"] = raises

    # op-level functions (models/submodule.py)
    ops = {}
    g = torch.Generator().manual_seed(7)
    l, r = feature_pair(2, 64, 5, 24, 21, 8)
    ops["gwc_L"], ops["gwc_R"] = l, r
    ops["gwc_out"] = sm.build_gwc_volume(l, r, 8, 32)
    att = torch.randn(2, 32, 1, 5, 24, generator=g)
    ops["gwc_att"] = att
    ops["gwc_att_out"] = sm.build_gwc_volume(l, r, 8, 32) * att
    l2, r2 = feature_pair(2, 16, 3, 20, 22, 6)
    ops["concat_L"], ops["concat_R"] = l2, r2
    ops["concat_out"] = sm.build_concat_volume(l2, r2, 6)
    l3, r3 = feature_pair(2, 64, 4, 20, 23, 7)
    ops["nc_L"], ops["nc_R"] = l3, r3
    ops["nc_out"] = sm.build_norm_correlation_volume(l3, r3, 7)
    cost = torch.randn(2, 12, 5, 9, generator=g)
    ops["reg_cost"] = cost
    ops["reg_out"] = sm.disparity_regression(cost, 12)
    tcost = torch.randn(2, 12, 5, 9, generator=g)
    tcost[0, 3, 0, 0] = tcost[0, :, 0, 0].max() + 1.0  # clear winner
    ds = torch.arange(0, 12, dtype=tcost.dtype).view(1, 12, 1, 1).repeat(2, 1, 5, 9)
    ops["topk_cost"] = tcost
    ops["topk_out"] = sm.regression_topk(tcost, ds, 2)
    np.savez_compressed(os.path.join(HERE, "ops.npz"), **{k: v.numpy() for k, v in ops.items()})
    manifest["ops.npz"] = {"gwc": [2, 64, 5, 24, 8, 32], "concat": [2, 16, 3, 20, 6], "nc": [2, 64, 4, 20, 7],
                           "reg": [2, 12, 5, 9], "topk": [2, 12, 5, 9]}
    with open(os.path.join(HERE, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)


if __name__ == "__main__":
    main()
