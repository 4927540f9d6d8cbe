#!/bin/bash
# Round-3 closing pass on the final tree: FMBlock phase stamps (diagnostic build in diagtmp/), every GPU test,
# the default S-K bench line, rocprof + PMC of the S-K step, then the configs evidence.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -f diagtmp/libdiag.so ]; then
  ESM_LIB=$PWD/diagtmp/libdiag.so timeout -k 10 200 python -u scripts/probes/fmnet_stamps.py > gpurun_out/fmnet_stamps.log 2>&1 \
      || { tail -20 gpurun_out/fmnet_stamps.log; exit 1; }
  grep -v "amdgpu.ids\|Cost vol" gpurun_out/fmnet_stamps.log
fi
bash scripts/gpu_r03_last.sh || exit 1
bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
head -6 gpurun_out/prof_SK_summary.txt
