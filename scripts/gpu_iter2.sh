#!/bin/bash
# Round-2 iteration: small-form parity tests, autotune of the S hot path with the new form, bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "small" --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_small.log 2>&1 || { tail -30 gpurun_out/pytest_small.log; exit 1; }
tail -2 gpurun_out/pytest_small.log
timeout -k 10 120 python -u scripts/diag_bench_epe.py > gpurun_out/diag_epe.log 2>&1 || { tail -20 gpurun_out/diag_epe.log; exit 1; }
cat gpurun_out/diag_epe.log
timeout -k 10 600 python -u scripts/autotune.py --variants ${VARIANTS:-S} --out gpurun_out/tuned_hints.json \
    > gpurun_out/autotune.log 2>&1 || { tail -30 gpurun_out/autotune.log; exit 1; }
grep -E "step|0x200000" gpurun_out/autotune.log | tail -60
