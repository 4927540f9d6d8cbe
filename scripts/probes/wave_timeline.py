"""Per-wave timeline of one direct-conv launch (diagnostic build only).

    python esmstereo_amd/build.py --diag
    ESM_LIB=esmstereo_amd/_build_diag/libesmstereo_amd.so python scripts/probes/wave_timeline.py [--h 192]

Each wave of the 2-D / 3-D direct kernel records s_memrealtime (100 MHz, chip-wide) at entry and
exit and s_memtime (shader clock) at entry, after setup, after its first K loop and at exit.
Prints the kernel span, the phases of a wave, and how many waves were resident over time.
"""
import argparse
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
if "ESM_LIB" not in os.environ:
    raise SystemExit("set ESM_LIB to the diagnostic build (python esmstereo_amd/build.py --diag)")
from esmstereo_amd import _lib  # noqa: E402
from esmstereo_amd.engine import ACT_GELU, Ctx, pack_conv, run_conv  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--h", type=int, default=192)
    ap.add_argument("--w", type=int, default=624)
    ap.add_argument("--cin", type=int, default=16)
    ap.add_argument("--cout", type=int, default=16)
    ap.add_argument("--hint", default="0")
    ap.add_argument("--nd", type=int, default=2)
    ap.add_argument("--d", type=int, default=1, help="depth (3-D)")
    ap.add_argument("--stride", type=int, default=1)
    args = ap.parse_args()
    fn = _lib.lib.esm_diag_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    dev = torch.device("cuda")
    C, BN = (torch.nn.Conv3d, torch.nn.BatchNorm3d) if args.nd == 3 else (torch.nn.Conv2d, torch.nn.BatchNorm2d)
    conv = C(args.cin, args.cout, 3, args.stride, 1, bias=False).to(dev)
    bn = BN(args.cout).eval().to(dev)
    pc = pack_conv(conv, bn, ACT_GELU)
    shape = (args.d, args.h, args.w) if args.nd == 3 else (args.h, args.w)
    x = torch.randn(1, args.cin, *shape, device=dev)
    out = None
    maxw = (1 << 20) // 8
    buf = np.zeros(8 * maxw, dtype=np.uint64)
    for it in range(3):
        out = run_conv(Ctx(dev), pc, [x], out=out, hint=int(args.hint, 16))
        torch.cuda.synchronize()
        n = fn(buf.ctypes.data, maxw)
    st = buf[: 8 * n].reshape(n, 8).astype(np.int64)
    real0, t0, t1, t2, t3, hwid, real1 = st[:, 0], st[:, 1], st[:, 2], st[:, 3], st[:, 4], st[:, 5], st[:, 6]
    span = (real1.max() - real0.min()) * 10 / 1000
    print(f"waves {n}; kernel span (first entry -> last exit) {span:.2f} us")
    lat = (real1 - real0) * 10 / 1000
    print(f"wave lifetime (realtime) us: p10 {np.percentile(lat, 10):.2f} p50 {np.median(lat):.2f} "
          f"p90 {np.percentile(lat, 90):.2f} max {lat.max():.2f}")
    for name, d in (("setup", t1 - t0), ("first K loop", t2 - t1), ("rest (epilogue, more rows)", t3 - t2),
                    ("total", t3 - t0)):
        print(f"  {name:28s} cycles p50 {np.median(d):8.0f}  p90 {np.percentile(d, 90):8.0f}")
    start = (real0 - real0.min()) * 10 / 1000
    end = (real1 - real0.min()) * 10 / 1000
    print(f"wave entry times us: p10 {np.percentile(start, 10):.2f} p50 {np.median(start):.2f} "
          f"p90 {np.percentile(start, 90):.2f} last {start.max():.2f}")
    grid = np.arange(0, span + 0.5, 0.5)
    res = [int(((start <= g) & (end > g)).sum()) for g in grid]
    print("resident waves every 0.5 us:", res)
    cu = (hwid >> 8) & 15
    se = (hwid >> 13) & 7
    print("distinct (se, cu) slots used:", len(set(zip(se.tolist(), cu.tolist()))))


if __name__ == "__main__":
    main()
