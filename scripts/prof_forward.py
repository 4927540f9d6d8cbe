"""The public forward end to end (bench.py forward_e2e's workload: ESMStereo-S, random-init backbone, one
384x1248 pair) for a rocprofv3 kernel trace, then a per-kernel table of the forward's device time:

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fwd -o fwd -- python3 scripts/prof_forward.py
    python3 scripts/prof_forward.py --table gpurun_out/prof_fwd
"""
import csv
import glob
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def table(d: str, top: int = 40) -> None:
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            rows += list(csv.DictReader(fh))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    iters = int(os.environ.get("FWD_ITERS", "20"))
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in rows:
        k = r["Kernel_Name"][:110]
        tot[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3
        cnt[k] += 1
    s = sum(tot.values())
    print(f"{len(rows)} dispatches, {s:.1f} us device time over the run ({s / (iters + 3):.1f} us per forward incl. warm-up share)")
    for k in sorted(tot, key=lambda k: -tot[k])[:top]:
        print(f"{tot[k]:10.1f} us {cnt[k]:6d}x {tot[k] / cnt[k]:8.2f} us  {k}")


def run() -> None:
    import torch

    import bench
    bench._load_package()
    E = bench.E
    dev = torch.device("cuda", 0)
    model = E.ESMStereo(192, True, False, "mobilenetv2_100", 16)
    bench.seeded_init(model, 1234)
    bench.load_seeded_weights(model, "S", "gwc")
    model = model.eval().to(dev)
    left, right = bench.synthetic_pair(1, 384, 1248, 192, 7, dev)
    model.capture_forward = os.environ.get("FWD_CAPTURE", "1") == "1"
    with torch.no_grad():
        for _ in range(3):
            model(left, right, False)
        torch.cuda.synchronize()
        for _ in range(int(os.environ.get("FWD_ITERS", "20"))):
            model(left, right, False)
        torch.cuda.synchronize()


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--table":
        table(sys.argv[2])
    else:
        run()
