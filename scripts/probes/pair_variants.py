"""Time the 1x1 -> 3x3 pair (ref4x.agg_1 shape: 16+16+24 -> 16 -> 16 at 192x624) in variants: lean vs LDS
kernel, GELU vs no activation (what the epilogue costs), and against the two single convs.

    python scripts/probes/pair_variants.py
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch  # noqa: E402

from esmstereo_amd.engine import ACT_GELU, ACT_NONE, Ctx, _conv_desc, pack_conv, run_conv  # noqa: E402


def timed(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3


def main():
    dev = torch.device("cuda")
    H, W, cins = 192, 624, (16, 16, 24)
    pool = torch.randn(sum(cins) * H * W + 1024, device=dev)
    xs, off = [], 256
    for c in cins:
        xs.append(pool[off:off + c * H * W].view(1, c, H, W))
        off += c * H * W
    torch.manual_seed(0)
    ca = torch.nn.Conv2d(sum(cins), 16, 1, bias=False).to(dev)
    cb = torch.nn.Conv2d(16, 16, 3, 1, 1, bias=False).to(dev)
    ba = torch.nn.BatchNorm2d(16).eval().to(dev)
    bb = torch.nn.BatchNorm2d(16).eval().to(dev)
    for act in (ACT_GELU, ACT_NONE):
        pa, pb = pack_conv(ca, ba, act), pack_conv(cb, bb, act)
        for hint in (0, 1 << 23):
            ctx = Ctx(dev)
            da, _, _ = _conv_desc(ctx, pa, xs, alloc_out=False)
            da.hint = hint
            db, out, _ = _conv_desc(ctx, pb, [], virtual_in=(1, 16, H, W))
            t = timed(lambda: ctx.pair(da, db))
            print(f"pair {'lean' if hint == 0 else 'lds '} act={'gelu' if act == ACT_GELU else 'none'}: {t:7.2f} us")
        mid = torch.empty(1, 16, H, W, device=dev)
        for h1, h2 in ((0, 0), (1 << 22, 1 << 22), (1 << 21, 1 << 21)):
            t1 = timed(lambda: run_conv(Ctx(dev), pa, xs, out=mid, hint=h1))
            t2 = timed(lambda: run_conv(Ctx(dev), pb, [mid], hint=h2))
            print(f"  two convs hints {hex(h1)}/{hex(h2)} act={act}: {t1:7.2f} + {t2:7.2f} us")


if __name__ == "__main__":
    main()
