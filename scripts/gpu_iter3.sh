#!/bin/bash
# Wide-form parity tests, then autotune of the S / M / L hot paths with every form.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${TESTS:-wide or gwc_stem or small}" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -2 gpurun_out/pytest_iter.log
[ -n "$NO_TUNE" ] && exit 0
VARIANTS=${VARIANTS:-S,M,L} bash scripts/gpu_tune.sh
