#!/bin/bash
# A/B per-op SQ counters: the default build vs ESM_PAIR_LEGACY=1, plus the counter list of the box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
timeout -k 10 60 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1
bash scripts/gpu_pmc_sq.sh lean || exit 1
ESM_PAIR_LEGACY=1 bash scripts/gpu_pmc_sq.sh legacy || exit 1
rm -rf gpurun_out/pmcsq_*/p1 gpurun_out/pmcsq_*/p2
