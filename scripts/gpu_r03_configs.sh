#!/bin/bash
# Round-3 evidence for the non-headline BASELINE configs on the final tree: one bench line each for configs 2, 3, 4
# (bench.py --config N), then the rocprof op map + PMC traffic of configs[3]'s per-rank slice (ESMStereo-L KITTI B=4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for c in ${CFGS:-2 3 4}; do
  timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c$c.log 2>&1 \
      || { tail -20 gpurun_out/bench_c$c.log; exit 1; }
  python -c "import json;d=json.loads([l for l in open('gpurun_out/bench_c$c.log') if l.startswith('{\"metric')][-1]);r=d['roofline'];print('config $c', d['value'], d['ms_per_step'], r['kernel'], r['avg_us'], r['frac'])"
done
bash scripts/gpu_prof.sh LK4 --variant L --batch 4 > gpurun_out/prof_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4_summary.txt; exit 1; }
head -12 gpurun_out/prof_LK4_summary.txt
