#!/bin/bash
# 3-D stems' row-streaming variant: parity tests, then the S-K step over (ESM_W3_ROWS : ESM_W3_NACC : ESM_W3_ROWS2)
# settings, rotated twice (group_stem rows / accumulators per row, agg rows; 1 = the previous form).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -rf \
    -k "wide3 or hot_path_golden or fullsize_vs_reference or full_size_vs_oracle and S" > gpurun_out/pytest_w3.log 2>&1 \
    || { tail -40 gpurun_out/pytest_w3.log; exit 1; }
tail -1 gpurun_out/pytest_w3.log
for rot in 1 2; do
  for r in ${SETS:-3:1:1 3:1:3 3:2:3 3:1:2}; do
    IFS=: read -r R N R2 <<< "$r"
    ESM_W3_ROWS=$R ESM_W3_NACC=$N ESM_W3_ROWS2=$R2 timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 \
        --no-cpu-baseline --no-extra > gpurun_out/bench_w3_$R$N$R2.log 2>&1 || { tail -20 gpurun_out/bench_w3_$R$N$R2.log; exit 1; }
    python -c "
import json;d=json.loads(open('gpurun_out/bench_w3_$R$N$R2.log').read().strip().splitlines()[-1]);m=d.get('roofline_mfma',{})
top={o['op']:o['us'] for o in d.get('top_ops_in_graph',[])}
print('set $r', d['value'], d['ms_per_step'], 'group_stem', m.get('avg_us'), m.get('frac'), 'agg', top.get('agg'))"
  done
done
