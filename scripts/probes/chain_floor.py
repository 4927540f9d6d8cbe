"""Per-launch cost of small hot-path kernels inside a hipGraph chain, next to the launch floor.

Each case is captured 20 times back to back in one graph (stream-ordered, so every launch waits
for the previous one, as in the hot path) and replayed; printed is graph time / launches.
    python scripts/probes/chain_floor.py [name filter ...]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from esmstereo_amd import engine as EN  # noqa: E402


def timed(make, reps=20, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn = make()
        fn()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    torch.cuda.synchronize()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * iters)


def conv_case(dev, nd, cin, cout, k, stride, shape, hint=0):
    def make():
        ctx = EN.Ctx(dev)
        conv = (torch.nn.Conv3d if nd == 3 else torch.nn.Conv2d)(cin, cout, k, stride, k // 2, bias=False).to(dev)
        bn = (torch.nn.BatchNorm3d if nd == 3 else torch.nn.BatchNorm2d)(cout).eval().to(dev)
        pc = EN.pack_conv(conv, bn, EN.ACT_GELU)
        x = torch.randn(1, cin, *shape, device=dev)
        out = EN.run_conv(ctx, pc, [x], hint=hint)
        return lambda: EN.run_conv(ctx, pc, [x], out=out, hint=hint)
    return make


def main():
    dev = torch.device("cuda")

    def add1():
        one = torch.zeros(1, device=dev)
        return lambda: one.add_(1)

    def add_plane():
        x = torch.zeros(12 * 24 * 78, device=dev)
        return lambda: x.add_(1)

    def regression():
        ctx = EN.Ctx(dev)
        cost = torch.randn(1, 12, 24, 78, device=dev)
        out = torch.empty(1, 24, 78, device=dev)
        return lambda: ctx.regression(0, cost, out, 1, 12, 24, 78)

    def gwc():
        ctx = EN.Ctx(dev)
        L = torch.randn(1, 64, 24, 78, device=dev)
        R = torch.randn(1, 64, 24, 78, device=dev)
        V = torch.empty(1, 32, 12, 24, 78, device=dev)
        return lambda: ctx.gwc(L, R, None, V, 1, 64, 24, 78, 12, 32)

    def normcorr():
        ctx = EN.Ctx(dev)
        L = torch.randn(1, 64, 24, 78, device=dev)
        R = torch.randn(1, 64, 24, 78, device=dev)
        V = torch.empty(1, 1, 12, 24, 78, device=dev)
        w = torch.empty(1, device=dev)
        return lambda: ctx.normcorr(L, R, V, w, 1, 64, 24, 78, 12)

    cases = [("torch add 1 elt", add1), ("torch add 22k elts", add_plane), ("disparity_regression S-K", regression),
             ("gwc S-K", gwc), ("normcorr S-K", normcorr),
             ("conv2d 16->16 k3 12x39", conv_case(dev, 2, 16, 16, 3, 1, (12, 39))),
             ("conv2d 16->16 k3 24x78", conv_case(dev, 2, 16, 16, 3, 1, (24, 78))),
             ("conv2d 16->16 k3 96x312", conv_case(dev, 2, 16, 16, 3, 1, (96, 312))),
             ("conv2d 16->16 k3 192x624", conv_case(dev, 2, 16, 16, 3, 1, (192, 624))),
             ("conv2d 16->16 k1 24x78", conv_case(dev, 2, 16, 16, 1, 1, (24, 78))),
             ("conv3d 24->24 k3 2x3x10", conv_case(dev, 3, 24, 24, 3, 1, (2, 3, 10))),
             ("conv3d 16->16 k3 3x6x20", conv_case(dev, 3, 16, 16, 3, 1, (3, 6, 20))),
             ("conv3d 12->12 k3 6x12x39", conv_case(dev, 3, 12, 12, 3, 1, (6, 12, 39))),
             ("conv3d 8->8 k3 12x24x78", conv_case(dev, 3, 8, 8, 3, 1, (12, 24, 78))),
             ("conv3d 32->8 k3 12x24x78", conv_case(dev, 3, 32, 8, 3, 1, (12, 24, 78))),
             ("conv3d 32->8 k3 48x96x312", conv_case(dev, 3, 32, 8, 3, 1, (48, 96, 312))),
             ("conv3d 8->8 k3 48x96x312", conv_case(dev, 3, 8, 8, 3, 1, (48, 96, 312)))]
    only = sys.argv[1:]
    for name, make in cases:
        if only and not any(o in name for o in only):
            continue
        print(f"{name:32s} {timed(make):8.2f} us / launch", flush=True)


if __name__ == "__main__":
    main()
