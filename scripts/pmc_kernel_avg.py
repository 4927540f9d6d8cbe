"""Average FETCH_SIZE / WRITE_SIZE per dispatch of each kernel from two rocprofv3 PMC passes, for
kernels launched outside the hot-path plan (scripts/gwc_ring.py).  Units and the gfx950 correction
as MI355X_MICROARCH.md §HBM: counters in KiB, FETCH_SIZE reports half of a wide streaming read:
hbm_bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024; the raw counters are kept beside it.

    python scripts/pmc_kernel_avg.py FETCH_DIR WRITE_DIR KERNEL_SUBSTR WORKLOAD NAME ALG_BYTES OUT_JSON [SKIP [COUNT]]

SKIP: dispatches of the kernel to drop from the front (warm-up / ring fill); COUNT: dispatches to
average after them (default: all the rest)."""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, sub):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                if r["Counter_Name"] == counter and sub in r["Kernel_Name"]:
                    k = int(r["Dispatch_Id"])
                    vals[k] = vals.get(k, 0.0) + float(r["Counter_Value"])
    return [vals[k] for k in sorted(vals)]


def main():
    fdir, wdir, sub, workload, name, alg, out = sys.argv[1:8]
    skip = int(sys.argv[8]) if len(sys.argv) > 8 else 0
    count = int(sys.argv[9]) if len(sys.argv) > 9 else None
    end = None if count is None else skip + count
    fs = per_dispatch(fdir, "FETCH_SIZE", sub)[skip:end]
    ws = per_dispatch(wdir, "WRITE_SIZE", sub)[skip:end]
    if not fs or not ws:
        raise SystemExit(f"no dispatches of {sub}")
    f, w = sum(fs) / len(fs), sum(ws) / len(ws)
    tab = json.load(open(out)) if os.path.exists(out) else {}
    row = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1), "hbm_bytes_per_launch": int((2 * f + w) * 1024),
           "algorithmic_bytes": int(alg), "dispatches": len(fs)}
    tab.setdefault(workload, {})[name] = row
    with open(out, "w") as fh:
        json.dump(tab, fh, indent=1)
    print(workload, name, row, f"ratio {row['hbm_bytes_per_launch'] / int(alg):.3f}")


if __name__ == "__main__":
    main()
