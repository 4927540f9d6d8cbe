#!/bin/bash
# Round 6: the tiny 3-D pair's tests, then the S-K step with it on / off (three rotations) and its op table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "tiny3" --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
ENVS="ESM_TINY3=1|ESM_TINY3=0" bash scripts/ab_env.sh > gpurun_out/ab_tiny3.txt 2>&1 || { tail -5 gpurun_out/ab_tiny3.txt; exit 1; }
cat gpurun_out/ab_tiny3.txt
ESM_AB=1 ESM_TINY3=1 NO_PMC=1 bash scripts/gpu_prof.sh iter > gpurun_out/prof_iter_summary.txt 2>&1 || { tail -20 gpurun_out/prof_iter_summary.txt; exit 1; }
head -3 gpurun_out/prof_ops_iter.txt; grep -E "conv3" gpurun_out/prof_ops_iter.txt
