#!/bin/bash
# Round 3: wide3 tests, A/B of $LIBS against the default build (S), then the L-K step tuner over the big
# convs (writes gpurun_out/tuned_hints_L.json, a copy of the table with L's choices merged in).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "wide3 or stem_form" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_w3.log 2>&1 || { tail -30 gpurun_out/pytest_w3.log; exit 1; }
tail -1 gpurun_out/pytest_w3.log
LIBS="esmstereo_amd/libesmstereo_amd.so $LIBS" VARIANTS=S bash scripts/gpu_ab_multi.sh || exit 1
cp esmstereo_amd/tuned_hints.json gpurun_out/tuned_hints_L.json
timeout -k 10 1000 python -u scripts/step_tune.py --mode tune --variants L --rounds 3 \
    --only "group_stem,agg,aggregation_out,ref4x,spx_4x,dm4x" --out gpurun_out/tuned_hints_L.json \
    --report gpurun_out/tune_L.json > gpurun_out/tune_L.log 2>&1
rc=$?; tail -50 gpurun_out/tune_L.log; exit $rc
