"""Per-op memory-side traffic of the bench step from two rocprofv3 PMC passes.

    rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o f -- python3 bench.py ...
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o w -- python3 bench.py ...
    python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write gpurun_out/ops.json \
        "ESMStereo-S gwc 384x1248 md192 B1" profiles/pmc_traffic.json

Dispatches of our kernels are assigned to the launch list by position (the timed steps replay
it in order; the oldest block is dropped, as in prof_ops.py).  Units and the gfx950
correction follow MI355X_MICROARCH.md §HBM: FETCH_SIZE / WRITE_SIZE are KiB, and FETCH_SIZE
reports half of the bytes a wide coalesced read moves, so
    hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.
Both raw counters are kept next to the corrected figure (the x2 is calibrated for 16-B/lane
streams; other widths are uncalibrated, so the raw numbers are the primary record).
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

OURS = ("esm::", "conv_kernel", "smix_kernel", "gwc_kernel", "concat_kernel", "normcorr_kernel", "l2norm_kernel",
        "dispreg_kernel", "topk2_kernel")


def per_dispatch(d: str, counter: str):
    vals = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter or not any(s in r["Kernel_Name"] for s in OURS):
                    continue
                k = int(r["Dispatch_Id"])
                vals[k] += float(r["Counter_Value"])
                names[k] = r["Kernel_Name"]
    order = sorted(vals)
    return [vals[k] for k in order]


def per_dispatch_named(d: str, counter: str):
    """{kernel-name fragment in OURS: [per-dispatch value, in dispatch order]}."""
    vals = defaultdict(float)
    names = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] != counter:
                    continue
                frag = next((s for s in OURS if s in r["Kernel_Name"] and s != "esm::"), None)
                if frag is None:
                    continue
                k = int(r["Dispatch_Id"])
                vals[k] += float(r["Counter_Value"])
                names[k] = frag
    out = defaultdict(list)
    for k in sorted(vals):
        out[names[k]].append(vals[k])
    return out


def kernel_ops(ops) -> list:
    """Launch-list op index of each kernel dispatch of one step (an op may launch several kernels:
    ``launches`` in its table entry, e.g. the two-launch FMBlock)."""
    return [i for i, op in enumerate(ops) for _ in range(int(op.get("launches", 1)))]


def whole_steps(seq, nk, timed=0):
    """The dispatches of the timed steps (``timed`` of them, the last whole steps before the trailing
    dispatches; 0 = every whole step but the oldest), ``nk`` kernels a step."""
    steps = len(seq) // nk
    if steps == 0:
        raise SystemExit("fewer dispatches than one step")
    if timed:
        return seq[-min(timed, steps) * nk:]
    return seq[-(steps - 1) * nk:] if steps > 1 else seq[-nk:]


def assign(seq, ops, timed=0):
    """Per-op average over the timed steps; an op's value is the sum over its kernels."""
    kop = kernel_ops(ops)
    nk = len(kop)
    tail = whole_steps(seq, nk, timed)
    acc = defaultdict(float)
    for i, v in enumerate(tail):
        acc[kop[i % nk]] += v
    steps = len(tail) // nk
    return {i: v / steps for i, v in acc.items()}


def trailing(ops_json: str) -> int:
    """Dispatches bench.py issued after its last whole step (written next to the op table)."""
    return _meta(ops_json).get("trailing_dispatches", 0)


def timed_steps(ops_json: str) -> int:
    """Whole steps of the timed region (bench.py runs marginal-cost replays with dropped ops before it)."""
    return _meta(ops_json).get("timed_steps", 0)


def _meta(ops_json: str) -> dict:
    meta = ops_json + ".meta.json"
    if not os.path.exists(meta):
        return {}
    with open(meta) as f:
        return {k: int(v) for k, v in json.load(f).items()}


def main():
    fdir, wdir, ops_json, workload, out = sys.argv[1:6]
    ops = json.load(open(ops_json))
    tr = trailing(ops_json)
    fs, ws = per_dispatch(fdir, "FETCH_SIZE"), per_dispatch(wdir, "WRITE_SIZE")
    fetch = assign(fs[:len(fs) - tr], ops, timed_steps(ops_json))
    write = assign(ws[:len(ws) - tr], ops, timed_steps(ops_json))
    tab = json.load(open(out)) if os.path.exists(out) else {}
    rows = {}
    for i, op in enumerate(ops):
        f, w = fetch.get(i, 0.0), write.get(i, 0.0)
        rows[op["name"]] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                            "hbm_bytes_per_launch": int((2 * f + w) * 1024),
                            "algorithmic_bytes": op["bytes"]}
    tab[workload] = rows
    with open(out, "w") as fh:
        json.dump(tab, fh, indent=1)
    top = sorted(rows.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:15]
    for k, v in top:
        print(f"{k[:50]:50s} {v['hbm_bytes_per_launch'] / 1e6:9.3f} MB  (alg {v['algorithmic_bytes'] / 1e6:8.3f} MB)")


if __name__ == "__main__":
    main()
