#!/bin/bash
# group_stem row-streaming variant: parity tests, then the S-K step for ESM_W3_ROWS = 1 (off), 2, 3, 4, rotated.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -rf \
    -k "wide3 or hot_path_golden or fullsize_vs_reference or full_size_vs_oracle and S" > gpurun_out/pytest_w3.log 2>&1 \
    || { tail -40 gpurun_out/pytest_w3.log; exit 1; }
tail -1 gpurun_out/pytest_w3.log
ESM_W3_NACC=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -rf \
    -k "wide3 or hot_path_golden" > gpurun_out/pytest_w3n2.log 2>&1 || { tail -40 gpurun_out/pytest_w3n2.log; exit 1; }
tail -1 gpurun_out/pytest_w3n2.log
for rot in 1 2; do
  for r in ${ROWS:-1:1 3:1 3:2 4:2}; do
    ESM_W3_ROWS=${r%%:*} ESM_W3_NACC=${r##*:} timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-extra > gpurun_out/bench_w3r${r%%:*}_${r##*:}.log 2>&1 \
        || { tail -20 gpurun_out/bench_w3r${r%%:*}_${r##*:}.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/bench_w3r${r%%:*}_${r##*:}.log').read().strip().splitlines()[-1]);m=d.get('roofline_mfma',{});print('rows=$r', d['value'], d['ms_per_step'], 'group_stem', m.get('avg_us'), m.get('frac'))"
  done
done
