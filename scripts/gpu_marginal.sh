#!/bin/bash
# Small-form parity tests, a bench line, and the per-op marginal costs of the S-K chain.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "${TESTS:-small}" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
tail -1 gpurun_out/pytest_iter.log
timeout -k 10 200 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extra > gpurun_out/bench_iter.log 2>&1 \
    || { tail -20 gpurun_out/bench_iter.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_iter.log').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
timeout -k 10 400 python -u scripts/step_tune.py --mode marginal --variants ${VARIANTS:-S} \
    --report gpurun_out/marginal.json > gpurun_out/marginal.log 2>&1 || { tail -20 gpurun_out/marginal.log; exit 1; }
sort -k4 -n -r gpurun_out/marginal.log | head -70
