#!/bin/bash
# Round-4 iteration: the whole GPU suite (new forms included), the conv form probe, the default bench
# line, then the L-K B = 4 op map (scripts/gpu_r04_L.sh, kernel trace only).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -rf --maxfail=8 \
    > gpurun_out/pytest_t.log 2>&1
rc=$?
tail -14 gpurun_out/pytest_t.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 200 python -u scripts/probes/conv_forms.py > gpurun_out/conv_forms.log 2>&1 || { tail -20 gpurun_out/conv_forms.log; exit 1; }
tail -40 gpurun_out/conv_forms.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_t.log 2>&1 || { tail -20 gpurun_out/bench_t.log; exit 1; }
tail -1 gpurun_out/bench_t.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['forward_e2e'], d['epe_vs_reference'])"
timeout -k 10 300 env ESM_SHUFFLE_CONV_MAXPIX=8192 python -u bench.py --no-extra --no-cpu-baseline > gpurun_out/bench_t_ab.log 2>&1 || { tail -20 gpurun_out/bench_t_ab.log; exit 1; }
tail -1 gpurun_out/bench_t_ab.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('A/B 4x shuffle_conv off:', d['value'], d['ms_per_step'])"
NO_PMC=1 bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
head -16 gpurun_out/prof_SK_summary.txt
NO_PMC=1 CONFIGS=1 bash scripts/gpu_r04_L.sh
