#!/bin/bash
# Round 6: pointwise / tile3 GPU tests, then the L-K B4 wall-time tuner over the named ops ($ONLY), then the
# L-K B4 op table with the tuned table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "${TESTS:-pointwise or tile3}" --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
cp esmstereo_amd/tuned_hints.json gpurun_out/tuned_hints.json
timeout -k 10 900 python -u scripts/step_tune.py --mode tune --variants L --batch 4 --rounds ${ROUNDS:-3} --margin-us ${MARGIN:-3} \
    --only "$ONLY" --out gpurun_out/tuned_hints.json --report gpurun_out/step_tune_report.json > gpurun_out/step_tune.log 2>&1 \
    || { tail -30 gpurun_out/step_tune.log; exit 1; }
grep -v "0.00 us" gpurun_out/step_tune.log | tail -40
cp gpurun_out/tuned_hints.json esmstereo_amd/tuned_hints.json
NO_PMC=1 bash scripts/gpu_prof.sh iter --variant L --batch 4 > gpurun_out/prof_iter_summary.txt 2>&1 || { tail -20 gpurun_out/prof_iter_summary.txt; exit 1; }
head -3 gpurun_out/prof_ops_iter.txt
