"""Map a rocprofv3 kernel trace of `bench.py` onto the hot-path launch list.

    rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- \
        python bench.py --steps 20 --no-extra --no-cpu-baseline --kernel-table gpurun_out/ops.json
    python scripts/prof_ops.py gpurun_out/prof gpurun_out/ops.json

The timed steps replay the launch list in order, so the last (steps x ops-per-step)
dispatches of our library's kernels are assigned to ops by position.  Prints per-op
average device duration, the per-step kernel sum and the average inter-kernel gap.
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

OURS = ("esm", "conv_kernel", "smix_kernel", "gwc_kernel", "concat_kernel", "normcorr_kernel", "l2norm_kernel",
        "dispreg_kernel", "topk_kernel")


def load_trace(d: str):
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no kernel_trace.csv under {d}")
    rows = []
    for f in files:
        with open(f) as fh:
            for r in csv.DictReader(fh):
                rows.append(r)
    key = lambda r: int(r.get("Start_Timestamp") or r.get("start_timestamp") or 0)  # noqa: E731
    rows.sort(key=key)
    return rows


sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_traffic import kernel_ops, timed_steps, trailing, whole_steps  # noqa: E402


def main():
    d, ops_json = sys.argv[1], sys.argv[2]
    ops = json.load(open(ops_json))
    kop = kernel_ops(ops)
    nk = len(kop)
    rows = [r for r in load_trace(d) if any(s in (r.get("Kernel_Name") or r.get("kernel_name") or "") for s in OURS)]
    rows = rows[:len(rows) - trailing(ops_json)]
    if len(rows) < nk:
        raise SystemExit("trace shorter than one step")
    tail = whole_steps(rows, nk, timed_steps(ops_json))  # the timed region only when bench.py says so
    nsteps = len(tail) // nk
    per_step = defaultdict(lambda: defaultdict(float))  # op -> step -> summed kernel duration
    gaps = []
    prev_end = None
    for i, r in enumerate(tail):
        s = int(r.get("Start_Timestamp") or r["start_timestamp"])
        e = int(r.get("End_Timestamp") or r["end_timestamp"])
        per_step[kop[i % nk]][i // nk] += (e - s) / 1e3
        if prev_end is not None and i % nk != 0:
            gaps.append((s - prev_end) / 1e3)
        prev_end = e
    table = []
    for i, op in enumerate(ops):
        v = sorted(per_step[i].values())
        table.append((sum(v) / len(v), v[len(v) // 2], op))
    total = sum(t[0] for t in table)
    print(f"{nsteps} steps x {len(ops)} ops ({nk} kernels); kernel sum {total:.1f} us/step; "
          f"mean gap {sum(gaps) / max(1, len(gaps)):.2f} us")
    for avg, med, op in sorted(table, key=lambda t: -t[0]):
        ach = (op["flops"] / (avg * 1e-6) / 1e12, "TF") if op["kind"] == "conv" else (op["bytes"] / (avg * 1e-6) / 1e9, "GB/s")
        print(f"{avg:8.2f} us (med {med:7.2f})  {op['kind']:6s} {op['name'][:44]:44s} {op.get('shape', '')[:50]:50s} "
              f"{ach[0]:8.2f} {ach[1]}")


if __name__ == "__main__":
    main()
