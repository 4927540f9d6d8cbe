#!/bin/bash
# Evidence on the current tree: every GPU test, the default bench line (all side
# measurements), then rocprofv3 kernel stats + op map + PMC traffic of the S-K step.
# Usage: bash scripts/gpu_round.sh [tests|bench|prof|all]  (default all)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
what=${1:-all}
if [ "$what" = all ] || [ "$what" = tests ]; then
    timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=8 --timeout 300 --timeout-method thread -rf \
        > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
    tail -3 gpurun_out/pytest_gpu_full.log
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
    timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
    tail -1 gpurun_out/bench_full.log
fi
if [ "$what" = all ] || [ "$what" = prof ]; then
    bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
    head -14 gpurun_out/prof_SK_summary.txt
fi
