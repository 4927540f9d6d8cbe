"""Time one conv layer over a range of output heights (same width/channels) to separate the
fixed cost of a launch from its per-row throughput cost.

    python scripts/probes/conv_scaling.py [--hint 0x211] [--cin 16 --cout 16 --w 624]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from esmstereo_amd.engine import ACT_GELU, ACT_NONE, Ctx, pack_conv, run_conv  # noqa: E402


def time_conv(pc, x, hint, reps=20, iters=5):
    ctx = Ctx(x.device, plan=True)
    out = None
    for _ in range(reps):
        out = run_conv(ctx, pc, [x], out=out, hint=hint)
    ctx.launch()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        ctx.launch()
    b.record()
    torch.cuda.synchronize()
    ctx.close()
    return a.elapsed_time(b) * 1e3 / (reps * iters)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cin", type=int, default=16)
    ap.add_argument("--cout", type=int, default=16)
    ap.add_argument("--w", type=int, default=624)
    ap.add_argument("--k", type=int, default=3)
    ap.add_argument("--hints", default="0,0x211,0x12")
    ap.add_argument("--act", default="gelu")
    args = ap.parse_args()
    dev = torch.device("cuda")
    conv = torch.nn.Conv2d(args.cin, args.cout, args.k, 1, args.k // 2, bias=False).to(dev)
    bn = torch.nn.BatchNorm2d(args.cout).eval().to(dev)
    act = ACT_GELU if args.act == "gelu" else ACT_NONE
    pc = pack_conv(conv, bn if act != ACT_NONE else None, act)
    hints = [int(h, 16) for h in args.hints.split(",")]
    print(f"conv {args.k}x{args.k} {args.cin}->{args.cout} W={args.w} act={args.act}; us per launch by H:")
    for H in (4, 12, 24, 48, 96, 192, 384):
        x = torch.randn(1, args.cin, H, args.w, device=dev)
        row = "  ".join(f"{h:#06x}:{time_conv(pc, x, h):7.2f}" for h in hints)
        print(f"H={H:4d}  {row}", flush=True)


if __name__ == "__main__":
    main()
