#!/bin/bash
# Round 6 iteration: selected GPU tests ($TESTS), then the S-K bench line and its rocprof op table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "$TESTS" --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1; rc=$?
  tail -3 gpurun_out/pytest_iter.log; [ $rc -eq 0 ] || exit $rc
fi
NO_PMC=1 bash scripts/gpu_prof.sh iter ${BENCH_ARGS:-} > gpurun_out/prof_iter_summary.txt 2>&1 || { tail -20 gpurun_out/prof_iter_summary.txt; exit 1; }
head -14 gpurun_out/prof_ops_iter.txt
if [ -n "$ENVS" ]; then bash scripts/ab_env.sh; fi
