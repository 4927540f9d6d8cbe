#!/bin/bash
# Round-end check: every GPU test, then the default bench line (all side measurements).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf \
    > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -3 gpurun_out/pytest_gpu_full.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
tail -1 gpurun_out/bench_full.log
