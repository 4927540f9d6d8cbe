#!/bin/bash
# Step time under alternating environment settings, rotated 3 times on one box (A/B of runtime knobs).
# Usage: ENVS="A=1 B=2|A=0" BENCH_ARGS="--config 1" bash scripts/ab_env.sh   ('|' separates the settings)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
IFS='|' read -ra SETS <<< "${ENVS:?ENVS unset}"
for i in 1 2 3; do
    for e in "${SETS[@]}"; do
        env $e ESM_AB=1 timeout -k 10 200 python -u bench.py --steps ${STEPS:-400} --warmup 30 --no-extra --no-cpu-baseline \
            --no-marginal ${BENCH_ARGS:-} > gpurun_out/ab_env.log 2>&1 || { tail -20 gpurun_out/ab_env.log; exit 1; }
        python3 -c "
import json,sys; l=[x for x in open('gpurun_out/ab_env.log') if x.startswith('{')][-1]; d=json.loads(l)
print('r$i', '[$e]', d['value'], 'pairs/s', d['ms_per_step'], 'ms')"
    done
done
