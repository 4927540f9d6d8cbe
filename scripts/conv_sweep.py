"""Time the implicit-GEMM conv tile variants on the hot path's dominant layer shapes.

    python scripts/conv_sweep.py [--reps 40] [--iters 10]

Each (layer, tile hint) runs as a hipGraph of `reps` back-to-back launches of the same conv,
timed with hipEvents over `iters` replays, so the per-launch number is device time without
host launch gaps.  hint = NT | KS << 4 | C1 << 8 (0 = the library's automatic choice).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from esmstereo_amd.engine import ACT_GELU, ACT_NONE, ACT_SILU, Ctx, pack_conv, run_conv  # noqa: E402

# name, nd, cin list (sources), cout, k, s, transposed, spatial in (D,H,W), act, shuffle
LAYERS = [
    ("ref4x.conv1.1 2d k3 16->16 192x624", 2, [16], 16, 3, 1, False, (1, 192, 624), ACT_GELU, 1),
    ("tail4x 2d k3 8->1 384x1248", 2, [8], 1, 3, 1, False, (1, 384, 1248), ACT_NONE, 1),
    ("ref4x.conv1_up T2d 16->1 192x624", 2, [16], 1, 4, 2, True, (1, 192, 624), ACT_NONE, 1),
    ("ref4x.conv1.0 2d k3s2 1->16 384x1248", 2, [1], 16, 3, 2, False, (1, 384, 1248), ACT_GELU, 1),
    ("ref4x.agg_1.0 2d k1 16+16+24->16 192x624", 2, [16, 16, 24], 16, 1, 1, False, (1, 192, 624), ACT_GELU, 1),
    ("spx_4x.0 2d k3 16+24->16 96x312", 2, [16, 24], 16, 3, 1, False, (1, 96, 312), ACT_GELU, 1),
    ("upsampling4 2d k1 8->128 96x312 PS4", 2, [8], 128, 1, 1, False, (1, 96, 312), ACT_SILU, 4),
    ("ref4x.conv2_up T2d 16->16 96x312", 2, [16], 16, 4, 2, True, (1, 96, 312), ACT_GELU, 1),
    ("group_stem 3d k3 32->8 12x24x78", 3, [32], 8, 3, 1, False, (12, 24, 78), ACT_GELU, 1),
    ("agg 3d k3 8->8 12x24x78", 3, [8], 8, 3, 1, False, (12, 24, 78), ACT_GELU, 1),
    ("conv1.0 3d k3s2 8->12 12x24x78", 3, [8], 12, 3, 2, False, (12, 24, 78), ACT_GELU, 1),
    ("conv3.1 3d k3 24->24 2x3x10", 3, [24], 24, 3, 1, False, (2, 3, 10), ACT_GELU, 1),
    ("conv3.0 3d k3s2 16->24 3x6x20", 3, [16], 24, 3, 2, False, (3, 6, 20), ACT_GELU, 1),
    ("L group_stem 3d k3 32->8 48x96x312", 3, [32], 8, 3, 1, False, (48, 96, 312), ACT_GELU, 1),
    ("L conv1.1 3d k3 24->24 24x48x156", 3, [24], 24, 3, 1, False, (24, 48, 156), ACT_GELU, 1),
    ("L dm4x.1 2d k3 32->32 192x624", 2, [32], 32, 3, 1, False, (1, 192, 624), ACT_GELU, 1),
]

HINTS = [0, 0x11, 0x12, 0x14, 0x41, 0x42, 0x44, 0x114, 0x211, 0x212, 0x241, 0x242]


def make(nd, cins, cout, k, s, tr, act, dev):
    cin = sum(cins)
    if tr:
        conv = (torch.nn.ConvTranspose3d if nd == 3 else torch.nn.ConvTranspose2d)(cin, cout, 4, 2, 1, bias=False)
    else:
        conv = (torch.nn.Conv3d if nd == 3 else torch.nn.Conv2d)(cin, cout, k, s, (k - 1) // 2, bias=False)
    bn = (torch.nn.BatchNorm3d if nd == 3 else torch.nn.BatchNorm2d)(cout).eval()
    conv, bn = conv.to(dev), bn.to(dev)
    return pack_conv(conv, bn if act != ACT_NONE else None, act)


def time_variant(pc, srcs, hint, shuffle, reps, iters, dev):
    ctx = Ctx(dev, plan=True)
    try:
        out = None
        for _ in range(reps):
            out = run_conv(ctx, pc, srcs, out=out, hint=hint, shuffle=shuffle)
        ctx.launch()
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            ctx.launch()
        b.record()
        torch.cuda.synchronize()
        return a.elapsed_time(b) * 1e3 / (iters * reps)
    except Exception as e:  # noqa: BLE001 - a variant may be inapplicable
        return f"n/a ({str(e)[:60]})"
    finally:
        ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=40)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only", default="", help="comma-separated substrings of layer names")
    ap.add_argument("--hints", default="", help="comma-separated hex hints (default: all)")
    args = ap.parse_args()
    hints = [int(h, 16) for h in args.hints.split(",")] if args.hints else HINTS
    dev = torch.device("cuda")
    res = {}
    for name, nd, cins, cout, k, s, tr, (D, H, W), act, shuffle in LAYERS:
        if args.only and not any(o in name for o in args.only.split(",")):
            continue
        pc = make(nd, cins, cout, k, s, tr, act, dev)
        srcs = [torch.randn((1, c, D, H, W) if nd == 3 else (1, c, H, W), device=dev) for c in cins]
        row = {}
        for h in hints:
            t = time_variant(pc, srcs, h, shuffle, args.reps, args.iters, dev)
            row[h] = t
        res[name] = row
        best = min((v, h) for h, v in row.items() if isinstance(v, float))
        cells = "  ".join(f"{h:#05x}:{v:7.2f}" if isinstance(v, float) else f"{h:#05x}:  n/a  " for h, v in row.items())
        print(f"{name:42s} best {best[0]:7.2f} us (hint {best[1]:#05x}) | {cells}", flush=True)
    print(json.dumps({k: {str(h): v for h, v in r.items()} for k, r in res.items()}))


if __name__ == "__main__":
    main()
