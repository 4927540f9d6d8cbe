#!/bin/bash
# ESMStereo-L evidence: the per-rank slice of configs[3] (L-K, B = 4) bench line and its rocprof op map
# (kernel trace, then FETCH / WRITE passes unless NO_PMC is set), then configs[2] / [4] bench lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_prof.sh LK4 --variant L --batch 4 > gpurun_out/prof_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4_summary.txt; exit 1; }
head -24 gpurun_out/prof_LK4_summary.txt
if [ -n "$CONFIGS" ]; then
  for c in 3 2 4; do
    timeout -k 10 600 python -u bench.py --config $c --steps 10 --warmup 3 --no-extra --no-cpu-baseline \
        > gpurun_out/bench_c$c.log 2>&1 || { tail -20 gpurun_out/bench_c$c.log; exit 1; }
    tail -1 gpurun_out/bench_c$c.log | cut -c1-200
  done
fi
