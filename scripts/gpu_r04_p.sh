#!/bin/bash
# Round-4 measurements: XCD-slab order on the 3-D launches A/B at L-K B = 4, the S-K and
# L-K B = 4 op maps with PMC traffic (refreshes gpurun_out/pmc_traffic.json), the L-K SQ counters.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
B=(bench.py --variant L --batch 4 --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-marginal)
for i in 1 2; do
  for v in 1 0; do
    timeout -k 10 300 env ESM_XCD_SLAB_3D=$v python -u "${B[@]}" > gpurun_out/xcd3d_$v.log 2>&1 || { tail -20 gpurun_out/xcd3d_$v.log; exit 1; }
    tail -1 gpurun_out/xcd3d_$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('xcd3d=$v', d['value'], d['ms_per_step'])"
  done
done
bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
tail -16 gpurun_out/prof_SK_summary.txt
bash scripts/gpu_prof.sh LK4 --variant L --batch 4 > gpurun_out/prof_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4_summary.txt; exit 1; }
tail -16 gpurun_out/prof_LK4_summary.txt
bash scripts/gpu_pmc_sq.sh lk4 --variant L --batch 4 || exit 1
