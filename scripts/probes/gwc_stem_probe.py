"""Time the cost-volume head of ESMStereo-L in isolation: gwc_volume + the tiled group_stem (two launches)
vs the fused gwc_stem launch, per rows-per-wave variant (hint bits 26-27), at the L-K per-rank slice.

    python scripts/probes/gwc_stem_probe.py [--B 4] [--reps 20]

Each variant runs `reps` times back to back between one hipEvent pair (inputs rotate over a ring of 3
feature pairs so no launch finds the previous one's inputs in the L2).  Prints us per launch.
"""
import argparse
import os
import sys

os.environ.setdefault("ESM_AB", "1")
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))

import torch  # noqa: E402

from esmstereo_amd.engine import Ctx, pack_conv, run_conv, run_gwc_stem, ACT_GELU  # noqa: E402


def timed(fn, reps):
    fn(0)
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for i in range(reps):
        fn(i)
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--B", type=int, default=4)
    ap.add_argument("--D", type=int, default=48)
    ap.add_argument("--H", type=int, default=96)
    ap.add_argument("--W", type=int, default=312)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--G", type=int, default=32)
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    B, D, H, W, G = args.B, args.D, args.H, args.W, args.G
    torch.manual_seed(0)
    conv = torch.nn.Conv3d(G, 8, 3, 1, 1, bias=False)
    bn = torch.nn.BatchNorm3d(8).eval()
    p = pack_conv(conv.to(dev), bn.to(dev), ACT_GELU)
    feats = [(torch.randn(B, 2 * G, H, W, device=dev), torch.randn(B, 2 * G, H, W, device=dev)) for _ in range(3)]
    V = torch.empty(B, G, D, H, W, device=dev)
    ctx = Ctx(dev)
    res = {}
    res["gwc"] = timed(lambda i: ctx.gwc(feats[i % 3][0], feats[i % 3][1], None, V, B, 2 * G, H, W, D, G), args.reps)
    if args.B * D * H * W < (1 << 18):  # small volumes: the forms the S chain picks from
        for h, nm in ((1 << 24, "stem wide3"), (0, "stem auto")):
            res[nm] = timed(lambda i: run_conv(ctx, p, [V], hint=h), args.reps)
    for rs in (2, 3):
        res[f"stem tile3 rows{2 if rs == 2 else 4}"] = timed(
            lambda i: run_conv(ctx, p, [V], hint=(1 << 23) | (rs << 26)), args.reps)
        res[f"gwc_stem rows{2 if rs == 2 else 4}"] = timed(
            lambda i: run_gwc_stem(ctx, p, feats[i % 3][0], feats[i % 3][1], G, D, hint=rs << 26), args.reps)
    for k, v in res.items():
        print(f"B{B} D{D} {H}x{W}  {k:22s} {v:9.2f} us", flush=True)


if __name__ == "__main__":
    main()
