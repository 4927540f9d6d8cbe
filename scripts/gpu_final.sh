#!/bin/bash
# Closing evidence on the final tree (part a: every GPU test, smoke(), the default bench line, the S-K
# op map + PMC traffic, the configs[2] / [3] / [4] bench lines, the L-K B = 4 op map + PMC traffic.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
part=${1:-all}
if [ "$part" = all ] || [ "$part" = a ]; then
bash scripts/gpu_round.sh all || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -20 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
fi
[ "$part" = a ] && exit 0
# configs[2] / [4] with the side measurements (EPE vs the reference fixtures) and a bounded CPU baseline;
# configs[3] (32 pairs on one GPU, the 8-rank job's global batch) without them
for c in 2 4 3; do
  extra=""; [ $c = 3 ] && extra="--no-extra --no-cpu-baseline"
  timeout -k 10 600 python -u bench.py --config $c --steps 10 --warmup 3 $extra \
      > gpurun_out/bench_c$c.log 2>&1 || { tail -20 gpurun_out/bench_c$c.log; exit 1; }
  tail -1 gpurun_out/bench_c$c.log | cut -c1-160
done
bash scripts/gpu_prof.sh LK4 --variant L --batch 4 > gpurun_out/prof_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4_summary.txt; exit 1; }
head -12 gpurun_out/prof_LK4_summary.txt
bash scripts/gpu_pmc_sq.sh LK4 --variant L --batch 4 > gpurun_out/pmcsq_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/pmcsq_LK4_summary.txt; exit 1; }
head -4 gpurun_out/pmcsq_LK4_summary.txt
