#!/bin/bash
# Round-4 iteration: the new kernels' parity tests first (tile3, shuffle_tail forms, zero-copy binding),
# then the whole GPU suite, the default bench line and the S-K rocprof summary (scripts/gpu_r04.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -rf \
    -k "tile3 or shuffle_tail or in_place or plan_modes" > gpurun_out/pytest_new.log 2>&1 || { tail -40 gpurun_out/pytest_new.log; exit 1; }
tail -2 gpurun_out/pytest_new.log
bash scripts/gpu_r04.sh "${1:-all}"
