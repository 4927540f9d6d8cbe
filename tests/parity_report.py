"""Stage-by-stage parity report of the HIP hot path against the CPU oracle (GPU box tool).

    python tests/parity_report.py --variant S --cv gwc --height 384 --width 1248 --maxdisp 192

Runs each hot-path stage through the eager HIP modules on the oracle's own inputs for that
stage (so errors do not compound across stages), then the whole compiled plan end to end,
and prints relative max errors, EPE and, for ESMStereo-L, the top-2 flip count.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)

import esmstereo_amd as E  # noqa: E402
from esmstereo_amd.backbone import StubFeature  # noqa: E402
from helpers import load_spec, seeded_state  # noqa: E402
from oracle import esm_oracle as O  # noqa: E402

VARIANTS = {"S": ("mobilenetv2_100", 16), "M": ("efficientnet_b2", 8), "L": ("efficientnet_b2", 4)}


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="S")
    ap.add_argument("--cv", default="gwc")
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=1248)
    ap.add_argument("--maxdisp", type=int, default=192)
    ap.add_argument("--seed", type=int, default=11)
    args = ap.parse_args()
    dev = torch.device("cuda")
    bb, cvs = VARIANTS[args.variant]
    model = E.ESMStereo(args.maxdisp, args.cv == "gwc", args.cv == "nc", bb, cvs, feature_cls=StubFeature)
    sd = seeded_state(load_spec(f"spec_{args.variant}_{args.cv}.json"), args.seed)
    model.load_state_dict(sd)
    model.eval().to(dev)
    torch.manual_seed(0)
    left = torch.randn(1, 3, args.height, args.width, device=dev)
    right = torch.roll(left, -7, -1) + 0.05 * torch.randn_like(left)
    with torch.no_grad():
        ml, mr, att, up = model.prefix(left, right)
    cpu = lambda t: None if t is None else t.detach().cpu()  # noqa: E731
    with torch.no_grad():
        ref = O.hot_path(sd, cvs, args.maxdisp, args.cv == "gwc", cpu(ml), cpu(mr), cpu(att), [cpu(u) for u in up])
    rep = {}
    D = args.maxdisp // cvs
    g = lambda t: t.to(dev)  # noqa: E731
    with torch.no_grad():
        if args.cv == "gwc":
            V = E.build_gwc_volume(ml, mr, D, 32)
            rep["volume_rel"] = rel(V, ref["volume"])
            stem_in = g(ref["volume"] * att.cpu().unsqueeze(2)) if cvs == 16 else g(ref["volume"])
            rep["stem_rel"] = rel(model.group_stem(stem_in), ref["stem"])
        else:
            V = E.build_norm_correlation_volume(ml, mr, D)
            rep["volume_rel"] = rel(V, ref["volume"])
        rep["agg_rel"] = rel(model.agg(g(ref["stem"])), ref["agg"])
        cost = model.aggregation_out(g(ref["agg"]))
        rep["cost_rel"] = rel(cost, ref["cost"])
        c = ref["cost"].squeeze(1)
        if cvs == 4:
            init = E.regression_topk(g(c), None, 2)
            top = lambda x: torch.sort(torch.sort(x.double(), dim=1, descending=True, stable=True)[1][:, :2], 1)[0]  # noqa
            rep["top2_flips"] = int((top(cost.squeeze(1).cpu()) != top(c)).any(1).sum())
            rep["lowres_pixels"] = int(c[:, 0].numel())
        else:
            init = E.disparity_regression(g(c), D).unsqueeze(1)
        rep["init_rel"] = rel(init, ref["init_pred"])
        outs = model.upsample_module(*[g(cpu(u)) for u in up], g(ref["init_pred"]))
        rep["upsampler_rel"] = rel(outs[0] * 4, ref["disp_0"].unsqueeze(1))
        rep["upsampler_epe"] = float((outs[0].cpu() * 4 - ref["disp_0"].unsqueeze(1)).abs().mean())
        full = model.hot_path(ml, mr, att, up, False)[0]
        rep["hot_path_rel"] = rel(full, ref["disp_0"])
        rep["hot_path_epe"] = float((full.cpu() - ref["disp_0"]).abs().mean())
        rep["disp_mean_abs"] = float(ref["disp_0"].abs().mean())
        rep["disp_max_abs"] = float(ref["disp_0"].abs().max())
    print(json.dumps(rep, indent=1))


if __name__ == "__main__":
    main()
