#!/bin/bash
# A/B of environment switches on the S-K step: bench.py --no-extra, alternating, two rounds.
# Usage: bash scripts/gpu_r04_ab.sh "ENV=a" "ENV=b" ...   ("-" = defaults)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i + 1))
    envs=()
    [ "$e" != "-" ] && read -r -a envs <<< "$e"
    timeout -k 10 200 env "${envs[@]}" python -u bench.py --steps 300 --warmup 30 --no-extra --no-cpu-baseline --no-marginal \
        > gpurun_out/ab_$i.log 2>&1 || { tail -20 gpurun_out/ab_$i.log; exit 1; }
    tail -1 gpurun_out/ab_$i.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('r$r', '$e', d['value'], d['ms_per_step'], d['config']['launches_per_step'])"
  done
done
