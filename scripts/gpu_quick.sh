#!/bin/bash
# Quick iteration on the GPU box: selected parity tests (PYTEST_K), then a short bench (no side legs).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf -k "${PYTEST_K:-fmnet or fmblock or golden}" \
    > gpurun_out/pytest_quick.log 2>&1 || { tail -40 gpurun_out/pytest_quick.log; exit 1; }
tail -2 gpurun_out/pytest_quick.log
timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-extra > gpurun_out/bench_quick.log 2>&1 \
    || { tail -20 gpurun_out/bench_quick.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_quick.log').read().strip().splitlines()[-1]);r=d['roofline'];print('bench', d['value'], d['ms_per_step'], r['kernel'], r['avg_us'], r['frac'])"
