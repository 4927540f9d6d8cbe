#!/bin/bash
# Kernel iteration: selected GPU parity tests, a short S-K bench line, and the per-op device-time
# table from a rocprofv3 kernel trace of the same bench (scripts/prof_ops.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
    timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "$TESTS" \
        --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
    tail -2 gpurun_out/pytest_iter.log
fi
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench_iter.log 2>&1 \
    || { tail -20 gpurun_out/bench_iter.log; exit 1; }
tail -1 gpurun_out/bench_iter.log
rm -rf gpurun_out/prof_iter
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_iter -o run -- \
    python bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --kernel-table gpurun_out/ops_iter.json \
    > gpurun_out/prof_iter.log 2>&1 || { tail -20 gpurun_out/prof_iter.log; exit 1; }
python scripts/prof_ops.py gpurun_out/prof_iter gpurun_out/ops_iter.json > gpurun_out/ops_iter.txt
rm -rf gpurun_out/prof_iter
head -40 gpurun_out/ops_iter.txt
