#!/bin/bash
# Round-3 closing run: FMBlock / hot-path parity (S, M, L), the S-K bench line, then the configs evidence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf \
    > gpurun_out/pytest_gpu_full.log 2>&1 || { tail -40 gpurun_out/pytest_gpu_full.log; exit 1; }
tail -1 gpurun_out/pytest_gpu_full.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_full.log 2>&1 || { tail -20 gpurun_out/bench_full.log; exit 1; }
python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_full.log') if l.startswith('{\"metric')][-1]);r=d['roofline'];print('S-K', d['value'], d['ms_per_step'], r['kernel'], r['avg_us'], r['frac'])"
bash scripts/gpu_r03_configs.sh
