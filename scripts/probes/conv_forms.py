"""Back-to-back launch time of the automatic conv form vs the LDS-tiled form (hint bit 23, rows per wave in
bits 26-27) at the hot paths' layer shapes.  Diagnostic only (isolated kernels, warm L2): the step tuner
decides by step time."""
import sys

import torch

sys.path.insert(0, ".")
from esmstereo_amd.engine import ACT_GELU, Ctx, pack_conv, run_conv  # noqa: E402

dev = torch.device("cuda")
T3 = 1 << 23
NOTILE = 1 << 19  # conv.hip kHintNoTile: the automatic rules without the tiled forms
CASES = [  # name, nd, cins, cout, k, s, p, spatial, B
    ("S group_stem", 3, (32,), 8, 3, 1, 1, (12, 24, 78), 1),
    ("S agg", 3, (8,), 8, 3, 1, 1, (12, 24, 78), 1),
    ("L group_stem B4", 3, (32,), 8, 3, 1, 1, (48, 96, 312), 4),
    ("L conv1.1 B4", 3, (24,), 24, 3, 1, 1, (24, 48, 156), 4),
    ("L agg B4", 3, (8,), 8, 3, 1, 1, (48, 96, 312), 4),
    ("S ref4x.conv1.1", 2, (16,), 16, 3, 1, 1, (192, 624), 1),
    ("S ref4x.agg_1.0", 2, (16, 16, 24), 16, 1, 1, 0, (192, 624), 1),
    ("S ref4x.conv2.0", 2, (16,), 16, 3, 2, 1, (192, 624), 1),
    ("S ref4x.conv2.1", 2, (16,), 16, 3, 1, 1, (96, 312), 1),
    ("S spx_4x.0", 2, (16, 24), 16, 3, 1, 1, (96, 312), 1),
    ("S spx_4x.1", 2, (16,), 8, 3, 1, 1, (96, 312), 1),
    ("L spx_4x.0 B4", 2, (32, 32), 32, 3, 1, 1, (192, 624), 4),
    ("L ref4x.agg_1.0 B4", 2, (32, 32, 32), 32, 1, 1, 0, (192, 624), 4),
    ("L agg_1.0 B4", 3, (24, 24), 24, 1, 1, 0, (24, 48, 156), 4),
    ("L conv1.0 B4", 3, (8,), 24, 3, 2, 1, (48, 96, 312), 4),
    ("L conv2.0 B4", 3, (24,), 40, 3, 2, 1, (24, 48, 156), 4),
    ("L conv2.1 B4", 3, (40,), 40, 3, 1, 1, (12, 24, 78), 4),
    ("L conv3.1 B4", 3, (72,), 72, 3, 1, 1, (6, 12, 39), 4),
    ("S ref4x.conv2_up", 2, (16,), 16, 4, 2, 1, (96, 312), 1),
    ("L ref4x.conv2_up B4", 2, (32,), 32, 4, 2, 1, (96, 312), 4),
    ("L conv2_up B4", 3, (40,), 24, 4, 2, 1, (12, 24, 78), 4),
]


def timed(fn, reps=50):
    for _ in range(5):
        fn()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


for name, nd, cins, cout, k, s, p, sp, B in CASES:
    torch.manual_seed(0)
    if k == 4:
        Conv = torch.nn.ConvTranspose3d if nd == 3 else torch.nn.ConvTranspose2d
    else:
        Conv = torch.nn.Conv3d if nd == 3 else torch.nn.Conv2d
    BN = torch.nn.BatchNorm3d if nd == 3 else torch.nn.BatchNorm2d
    conv = Conv(sum(cins), cout, k, s, p, bias=False).to(dev)
    bn = BN(cout).to(dev).eval()
    pc = pack_conv(conv, bn, ACT_GELU)
    xs = [torch.randn(B, c, *sp, device=dev) for c in cins]
    ctx = Ctx(dev)
    out = run_conv(ctx, pc, xs)
    res = {}
    forms = [("auto", 0), ("no tile", NOTILE), ("tile r1", T3 | 1 << 26), ("tile r2", T3 | 2 << 26),
             ("tile r4", T3 | 3 << 26)]
    if nd == 3 and k == 3 and s == 1:
        forms.append(("tile r8", T3 | 3 << 26 | 1 << 28))
    if len(sys.argv) > 1 and not any(f in name for f in sys.argv[1:]):
        continue
    for label, hint in forms:
        try:
            y = run_conv(ctx, pc, xs, hint=hint)
            err = float((y - out).abs().max() / out.abs().max())
            res[label] = (timed(lambda: run_conv(ctx, pc, xs, out=y, hint=hint)), err)
        except Exception as e:  # noqa: BLE001 - a form that does not apply
            res[label] = (float("nan"), str(e)[:40])
    print(f"{name:22s} " + "  ".join(f"{k}: {v[0]:8.2f} us" for k, v in res.items()), flush=True)
