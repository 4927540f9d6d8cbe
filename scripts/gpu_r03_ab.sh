#!/bin/bash
# Round 3 A/B: selected GPU tests ($TESTS), step rotation of $LIBS over $VARIANTS, then per-op
# memory-side traffic at S-K for each build in $LIBS_PMC (full tables kept as pmc_traffic_<lib>.txt).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
    timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$TESTS" --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_ab.log 2>&1 || { tail -40 gpurun_out/pytest_ab.log; exit 1; }
    tail -2 gpurun_out/pytest_ab.log
fi
LIBS="esmstereo_amd/libesmstereo_amd.so $LIBS" bash scripts/gpu_ab_multi.sh || exit 1
for L in $LIBS_PMC; do
    n=$(basename $L .so)
    ESM_LIB=$L bash scripts/gpu_prof.sh $n > gpurun_out/prof_$n.out 2>&1 || { tail -5 gpurun_out/prof_$n.out; exit 1; }
    cp gpurun_out/pmc_traffic.json gpurun_out/pmc_traffic_$n.json
    python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.load(open(f"gpurun_out/pmc_traffic_{n}.json"))
d = d[[k for k in d if k.startswith("ESMStereo")][0]]
tot = sum(v["hbm_bytes_per_launch"] for v in d.values()); alg = sum(v["algorithmic_bytes"] for v in d.values())
print(n, "step total %.1f MB / alg %.1f MB" % (tot / 1e6, alg / 1e6))
for k, v in d.items():
    if any(s in k for s in ("tail4x", "conv1_up", "ref4x.conv2.0", "group_stem", "ref4x.conv1.1", "spx_4x.0", "+")):
        print(n, "%-40s %7.2f MB alg %6.2f  x%.2f" % (k, v["hbm_bytes_per_launch"] / 1e6, v["algorithmic_bytes"] / 1e6,
                                                      v["hbm_bytes_per_launch"] / max(1, v["algorithmic_bytes"])))
PY
done
