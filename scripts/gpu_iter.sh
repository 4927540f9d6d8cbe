#!/bin/bash
# Iteration loop on the GPU box: GPU parity tests, then a short bench with the per-op probe table.
# Stops at the first failure; every GPU step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-50} --warmup 10 --no-cpu-baseline \
    --kernel-table gpurun_out/kernel_table.json > gpurun_out/bench.log 2>&1
brc=$?
tail -2 gpurun_out/bench.log
exit $brc
