"""Pick the conv form of every backbone-side conv (round 5: the timm blocks' 1x1 expand / project convs, the
stem, the stems' and descriptor's convs, all on esm_conv_f32) by timing each candidate hint at the layer's real
shape, and add the winners to the tuned-hint table under engine.conv_key (keys already there, the hot path's
in-graph choices, are left alone).

    ESM_AB=1 ESM_NO_TUNED=1 python scripts/tune_backbone.py --out gpurun_out/tuned_hints.json [--variants S,M,L]

Each candidate runs `reps` times back to back between one hipEvent pair on fresh random inputs of the layer's
shape; a hint replaces the automatic choice when it is faster by more than --margin (relative).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

os.environ.setdefault("ESM_AB", "1")
os.environ.setdefault("ESM_NO_TUNED", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "scripts")]

import torch  # noqa: E402

import bench  # noqa: E402
from autotune import CANDIDATES  # noqa: E402


def record(model, left, right):
    """(PackedConv, source shapes, residual shape or None, tag) of every conv the backbone side launches."""
    import esmstereo_amd.blocks as blocks
    import esmstereo_amd.engine as engine
    import esmstereo_amd.model as model_mod
    seen = []
    orig = engine.run_conv

    def rec(ctx, pc, srcs, out=None, **kw):
        seen.append((pc, [tuple(t.shape) for t in srcs], tuple(kw["res"].shape) if kw.get("res") is not None else None,
                     kw.get("tag", "conv")))
        return orig(ctx, pc, srcs, out, **kw)

    engine.run_conv, model_mod.run_conv, blocks.run_conv = rec, rec, rec
    try:
        with torch.no_grad():
            model.prefix(left, right)
    finally:
        engine.run_conv, model_mod.run_conv, blocks.run_conv = orig, orig, orig
    return seen


def time_hint(E, pc, shapes, res_shape, hint, dev, reps=20):
    """Device time per launch: ``reps`` launches captured into one CUDA graph (no host work between them),
    the graph replayed 3 times between one hipEvent pair."""
    srcs = [torch.randn(s, device=dev) for s in shapes]
    res = None
    if res_shape is not None:
        res = torch.randn(res_shape, device=dev)
    try:
        E.engine.run_conv(E.engine.Ctx(dev), pc, srcs, res=res, hint=hint)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        side = torch.cuda.Stream(dev)
        with torch.cuda.stream(side), torch.cuda.graph(g):
            ctx = E.engine.Ctx(dev)
            for _ in range(reps):
                E.engine.run_conv(ctx, pc, srcs, res=res, hint=hint)
    except Exception:
        torch.cuda.synchronize()
        return None
    g.replay()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(3):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    del g
    return a.elapsed_time(b) / (3 * reps) * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="S")
    ap.add_argument("--out", default="gpurun_out/tuned_hints.json")
    ap.add_argument("--margin", type=float, default=0.05)
    args = ap.parse_args()
    bench._load_package()
    E = bench.E
    dev = torch.device("cuda", 0)
    table = json.load(open(args.out)) if os.path.exists(args.out) else {"hints": {}}
    added = {}
    for var in args.variants.split(","):
        backbone, cvs = bench.VARIANTS[var]
        model = E.ESMStereo(192, True, False, backbone, cvs)
        bench.seeded_init(model, 1234)
        model = model.eval().to(dev)
        left, right = bench.synthetic_pair(1, 384, 1248, 192, 7, dev)
        for pc, shapes, res_shape, tag in record(model, left, right):
            srcs = [torch.empty(s, device="meta") for s in shapes]
            with E.engine.Ctx(dev, dry=True) as dry:
                _, _, meta = E.engine._conv_desc(dry, pc, srcs, res=None if res_shape is None else
                                                 torch.empty(res_shape, device="meta"))
            key = meta["key"]
            if key in table["hints"] or key in added:
                continue
            t0 = time_hint(E, pc, shapes, res_shape, 0, dev)
            best, bt = 0, t0
            for h in CANDIDATES[1:]:
                t = time_hint(E, pc, shapes, res_shape, h, dev)
                if t is not None and t < bt:
                    best, bt = h, t
            if best and bt < t0 * (1 - args.margin):
                added[key] = best
            print(f"{var} {tag:28s} {meta['shape']:48s} auto {t0:7.2f} us  best {hex(best):>10s} {bt:7.2f} us", flush=True)
    table["hints"].update(added)
    with open(args.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print(f"added {len(added)} backbone keys to {args.out}")


if __name__ == "__main__":
    main()
