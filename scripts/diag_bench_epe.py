"""Where does the bench input's EPE vs the oracle come from?  Stage-by-stage comparison of the HIP
hot path and oracle/esm_oracle.py on bench.py's own synthetic input (diagnostic, GPU).

    python scripts/diag_bench_epe.py [--config 1]
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import torch  # noqa: E402

import bench  # noqa: E402
import esmstereo_amd as E  # noqa: E402
from oracle import esm_oracle as O  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=1)
    args = ap.parse_args()
    cfg = bench.CONFIGS[args.config]
    dev = torch.device("cuda", 0)
    backbone, cvs = bench.VARIANTS[cfg["variant"]]
    model = E.ESMStereo(cfg["maxdisp"], cfg["cv"] == "gwc", cfg["cv"] == "nc", backbone, cvs)
    bench.seeded_init(model, 1234)
    bench.load_seeded_weights(model, cfg["variant"], cfg["cv"])
    model = model.eval().to(dev)
    B = cfg.get("batch") or 1
    left, right = bench.synthetic_pair(1, cfg["height"], cfg["width"], cfg["maxdisp"], 100, dev)
    with torch.no_grad():
        ml, mr, att, up = model.prefix(left, right)
    for n, t in [("ml", ml), ("mr", mr), ("att", att)] + [(f"up{i}", u) for i, u in enumerate(up)]:
        if t is not None:
            print(f"{n:4s} {tuple(t.shape)} mean|x| {t.abs().mean().item():.4g} max|x| {t.abs().max().item():.4g}")
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    c = lambda t: None if t is None else t.cpu()  # noqa: E731
    with torch.no_grad():
        ref = O.hot_path(sd, cvs, cfg["maxdisp"], cfg["cv"] == "gwc", c(ml), c(mr), c(att), [c(u) for u in up])
        got = model.hot_path(ml, mr, att, up)[0].cpu()
        D = cfg["maxdisp"] // cvs
        V = E.build_gwc_volume(ml, mr, D, 32, att=att) if cfg["cv"] == "gwc" else E.build_norm_correlation_volume(ml, mr, D)
        vol = model.group_stem(V) if cfg["cv"] == "gwc" else model.corr_stem(V)
        cost = model.aggregation_out(model.agg(vol))[:, 0]
        init = E.disparity_regression(cost, D).unsqueeze(1) if cvs != 4 else E.regression_topk(cost, None, 2)
    for k, v in ref.items():
        if torch.is_tensor(v):
            print(f"oracle {k:12s} {tuple(v.shape)} mean|x| {v.abs().mean().item():.4g}")
    if "cost" in ref:
        rc = ref["cost"].squeeze(1)
        print("cost rel", ((cost.cpu() - rc).norm() / rc.norm()).item(), "max abs", (cost.cpu() - rc).abs().max().item())
    for key in ("init_pred", "init", "pred0"):
        if key in ref:
            print(key, "EPE", (init.cpu().reshape(ref[key].shape) - ref[key]).abs().mean().item())
    d = (got - ref["disp_0"]).abs()
    print("disp_0 EPE", d.mean().item(), "max", d.max().item(), "ref mean|d|", ref["disp_0"].abs().mean().item())
    # upsampler alone on the oracle's init: isolates the upsampler
    if "init_pred" in ref or "init" in ref:
        ri = ref.get("init_pred", ref.get("init"))
        print("oracle keys", sorted(k for k in ref if torch.is_tensor(ref[k])))
        print("init magnitude", ri.abs().mean().item())


if __name__ == "__main__":
    main()
