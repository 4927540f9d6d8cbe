#!/bin/bash
# New-kernel parity tests, then step-time A/B of the new forms (rotated), then per-op SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "${TESTS:-pair2 or rows3 or shuffle}" --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
ENVS="${ENVS:-X=0 ESM_PAIR2=0 ESM_SHUFFLE_CONV=0 ESM_ROWS3=0}" bash scripts/gpu_ab_env.sh || exit 1
[ -n "$NO_PMC" ] && exit 0
bash scripts/gpu_pmc_sq.sh sk > gpurun_out/pmcsq.log 2>&1 || { tail -5 gpurun_out/pmcsq.log; exit 1; }
head -70 gpurun_out/pmcsq_sk/summary.txt
