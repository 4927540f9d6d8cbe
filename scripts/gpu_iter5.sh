#!/bin/bash
# Parity tests for the touched forms, then wall-time tuning of VARIANTS and a bench line.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${TESTS:-wide}" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
[ -n "$NO_TUNE" ] && exit 0
bash scripts/gpu_step_tune.sh
