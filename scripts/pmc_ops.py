"""Per-op SQ counters of the bench step from rocprofv3 PMC passes (any counters).

    rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES ... -d gpurun_out/pmc_sq1 -o p1 -- python3 bench.py ... \
        --kernel-table gpurun_out/ops.json
    python scripts/pmc_ops.py gpurun_out/ops.json gpurun_out/pmc_sq1 [gpurun_out/pmc_sq2 ...]

Dispatches of our kernels are assigned to the launch list by position (as pmc_traffic.py).  Per op:
the mean of every counter per dispatch, and where the pass holds them
  cyc/wave  SQ_WAVE_CYCLES / SQ_WAVES x 4 (the SQ counts quad-cycles, MI355X_MICROARCH.md)
  act/wait/inst  SQ_ACTIVE_INST_ANY, SQ_WAIT_ANY, SQ_WAIT_INST_ANY as fractions of SQ_WAVE_CYCLES
  valu/lds/mfma per wave  SQ_INSTS_VALU, SQ_INSTS_LDS per wave, SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs)
"""
from __future__ import annotations

import csv
import glob
import json
import os
import sys
from collections import defaultdict

from pmc_traffic import OURS, assign, timed_steps, trailing


def per_dispatch(d: str):
    vals = defaultdict(lambda: defaultdict(float))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if not any(s in r["Kernel_Name"] for s in OURS):
                    continue
                vals[r["Counter_Name"]][int(r["Dispatch_Id"])] += float(r["Counter_Value"])
    return {c: [v[k] for k in sorted(v)] for c, v in vals.items()}


def main():
    ops_json, dirs = sys.argv[1], sys.argv[2:]
    ops = json.load(open(ops_json))
    tr = trailing(ops_json)
    per = {}
    for d in dirs:
        for c, seq in per_dispatch(d).items():
            per[c] = assign(seq[:len(seq) - tr], ops, timed_steps(ops_json))
    out = []
    for i, op in enumerate(ops):
        row = {"op": i, "name": op["name"], "median_us": round(op.get("median_ms", 0) * 1e3, 2)}
        row.update({c: round(v.get(i, 0.0), 1) for c, v in per.items()})
        w = row.get("SQ_WAVES", 0)
        wc = row.get("SQ_WAVE_CYCLES", 0)
        if w:
            row["cyc_per_wave"] = round(4 * wc / w)
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_VMEM_RD", "SQ_INSTS_MFMA"):
                if c in row:
                    row[c.replace("SQ_INSTS_", "").lower() + "_per_wave"] = round(row[c] / w, 1)
        if wc:
            for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS"):
                if c in row:
                    row[c.replace("SQ_", "").lower() + "_frac"] = round(row[c] / wc, 3)
        out.append(row)
    keys = ["median_us", "SQ_WAVES", "cyc_per_wave", "active_inst_any_frac", "wait_any_frac", "wait_inst_any_frac",
            "wait_inst_lds_frac", "valu_per_wave", "lds_per_wave", "salu_per_wave", "vmem_rd_per_wave",
            "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_LDS_BANK_CONFLICT", "GRBM_GUI_ACTIVE"]
    keys = [k for k in keys if any(k in r for r in out)]
    print("op name " + " ".join(keys))
    for r in out:
        print(f"{r['op']:2d} {r['name'][:44]:44s} " + " ".join(str(r.get(k, "-")) for k in keys))
    with open(os.path.join(os.path.dirname(ops_json), "pmc_ops.json"), "w") as fh:
        json.dump(out, fh, indent=1)


if __name__ == "__main__":
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    main()
