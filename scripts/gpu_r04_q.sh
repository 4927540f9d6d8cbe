#!/bin/bash
# Round-4: windowed / per-source wide forms (tests, S-K bench and op map), then PMC traffic keys for the
# L configs (configs[2] / [3] / [4]) so their bench lines carry `traffic`.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread -rf -x \
    -k "wide or in_place or hot_path or shuffle_conv" > gpurun_out/pytest_q.log 2>&1 || { tail -30 gpurun_out/pytest_q.log; exit 1; }
tail -2 gpurun_out/pytest_q.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_q.log 2>&1 || { tail -20 gpurun_out/bench_q.log; exit 1; }
tail -1 gpurun_out/bench_q.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['forward_e2e']['hot_path_call_ms'], d['roofline']['kernel'], d['roofline']['frac'])"
NO_PMC=1 bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
head -14 gpurun_out/prof_SK_summary.txt
for c in 2 3 4; do
  bash scripts/gpu_prof.sh C$c --config $c > gpurun_out/prof_C${c}_summary.txt 2>&1 || { tail -20 gpurun_out/prof_C${c}_summary.txt; exit 1; }
  head -8 gpurun_out/prof_C${c}_summary.txt
done
