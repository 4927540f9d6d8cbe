#!/bin/bash
# Round 3: FETCH/WRITE counter calibration (scripts/probes/fetch_calib), then the XCD-slab tile order
# per form ($LIBS twins built by scripts/ab_define.sh -DESM_XCD_REMAP): S-K step rotation and per-op
# memory-side traffic for each build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $c --output-format csv -d "$PWD/gpurun_out/calib/$c" -o c -- \
        scripts/probes/fetch_calib > gpurun_out/calib/$c.log 2>&1 || { tail -5 gpurun_out/calib/$c.log; exit 3; }
done
python3 - <<'PY'
import csv, glob
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    rows = []
    for f in glob.glob(f"gpurun_out/calib/{c}/**/*counter_collection.csv", recursive=True):
        rows += [r for r in csv.DictReader(open(f)) if r["Counter_Name"] == c]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    for r in rows:
        print(c, r["Dispatch_Id"], r["Kernel_Name"][:40], r["Counter_Value"])
PY
LIBS="esmstereo_amd/libesmstereo_amd.so $LIBS" VARIANTS=S bash scripts/gpu_ab_multi.sh || exit 1
for L in $LIBS_PMC; do
    n=$(basename $L .so)
    ESM_LIB=$L NO_PMC= bash scripts/gpu_prof.sh $n > gpurun_out/prof_$n.out 2>&1 || { tail -5 gpurun_out/prof_$n.out; exit 1; }
    grep -E "tail4x|conv1_up|conv2.0|group_stem|conv1.1 " gpurun_out/pmc_traffic_$n.txt | sed "s|^|$n |"
done
