#!/bin/bash
# group_stem / agg at S-K with the XCD-slab order: step A/B, then FETCH/WRITE PMC for both.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_r04_ab.sh - ESM_XCD_SLAB_OPS=group_stem ESM_XCD_SLAB_OPS=group_stem,agg || exit 1
ESM_XCD_SLAB_OPS=group_stem,agg bash scripts/gpu_prof.sh SKX > gpurun_out/prof_SKX_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SKX_summary.txt; exit 1; }
grep -E "group_stem|  agg " gpurun_out/prof_SKX_summary.txt
