#!/bin/bash
# Round 6: rocprofv3 kernel trace + PMC FETCH / WRITE passes for every bench workload (S-K, configs[2] / [3] / [4],
# the L-K B = 4 slice), merged into gpurun_out/pmc_traffic.json (seeded from profiles/pmc_traffic.json) for bench.py's
# `traffic` fields.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
head -4 gpurun_out/prof_SK_summary.txt
bash scripts/gpu_prof.sh LK4 --variant L --batch 4 > gpurun_out/prof_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4_summary.txt; exit 1; }
head -4 gpurun_out/prof_LK4_summary.txt
for c in 2 3 4; do
  bash scripts/gpu_prof.sh c$c --config $c > gpurun_out/prof_c${c}_summary.txt 2>&1 || { tail -20 gpurun_out/prof_c${c}_summary.txt; exit 1; }
  head -4 gpurun_out/prof_c${c}_summary.txt
done
