"""Summarise rocprofv3 --pmc CSV output: mean counter value per dispatch, per kernel.

    python scripts/pmc_summary.py gpurun_out/pmc_conv [--top 20]

Reads every *counter_collection.csv below the directory (one file per pass).
"""
from __future__ import annotations

import argparse
import collections
import csv
import glob
import os
import re


def short(name: str) -> str:
    m = re.search(r"(\w*conv\w*_kernel)<(.*?)>\(", name)
    if m:
        return m.group(1) + "<" + m.group(2).replace("true", "1").replace("false", "0").replace(" ", "") + ">"
    name = name.replace("(anonymous namespace)::", "").replace("void ", "")
    return re.sub(r"\(.*", "", name)[:90]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--top", type=int, default=400)
    args = ap.parse_args()
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(args.dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in list(vals.items())[: args.top]:
        print(k)
        for c in sorted(cs):
            v = cs[c]
            print(f"    {c:28s} {sum(v) / len(v):14.1f}  (n={len(v)})")


if __name__ == "__main__":
    main()
