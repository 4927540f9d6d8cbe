#!/bin/bash
# Op map of the current default plan, then SQ counters for the 3-D stems under both stem forms.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
NO_PROF= bash scripts/gpu_iter.sh || exit 1
bash scripts/gpu_pmc_sq.sh rows3 > gpurun_out/pmcsq_rows3.log 2>&1 || { tail -5 gpurun_out/pmcsq_rows3.log; exit 1; }
ESM_ROWS3=0 bash scripts/gpu_pmc_sq.sh wide3 > gpurun_out/pmcsq_wide3.log 2>&1 || { tail -5 gpurun_out/pmcsq_wide3.log; exit 1; }
for t in rows3 wide3; do echo "== $t"; grep -E "op name|group_stem| agg " gpurun_out/pmcsq_$t/summary.txt; done
