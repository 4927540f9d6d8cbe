#!/bin/bash
# Round 6: per-kernel device time of the fused 4x stage under each tile (rocprofv3 kernel trace of the S-K step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
for T in 0 1 2; do
  ESM_AB=1 ESM_SC11_TILE=$T NO_PMC=1 bash scripts/gpu_prof.sh sc$T > gpurun_out/prof_sc$T.txt 2>&1 || { tail -20 gpurun_out/prof_sc$T.txt; exit 1; }
  echo "tile $T"; head -4 gpurun_out/prof_ops_sc$T.txt
done
