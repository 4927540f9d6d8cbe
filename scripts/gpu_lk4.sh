#!/bin/bash
# L-K per-rank slice (B = 4) evidence: op map (rocprofv3 kernel trace), SQ counters, and the op map
# of the two-launch gwc + group_stem path (A/B knob ESM_GWC_STEM=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
NO_PMC=1 bash scripts/gpu_prof.sh LK4 --variant L --batch 4 > gpurun_out/prof_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4_summary.txt; exit 1; }
head -12 gpurun_out/prof_LK4_summary.txt
if [ -n "$SQ" ]; then
  bash scripts/gpu_pmc_sq.sh LK4 --variant L --batch 4 > gpurun_out/pmcsq_LK4_summary.txt 2>&1 || { tail -20 gpurun_out/pmcsq_LK4_summary.txt; exit 1; }
  head -4 gpurun_out/pmcsq_LK4_summary.txt
fi
if [ -n "$UNFUSED" ]; then
  ESM_AB=1 ESM_GWC_STEM=0 NO_PMC=1 bash scripts/gpu_prof.sh LK4u --variant L --batch 4 > gpurun_out/prof_LK4u_summary.txt 2>&1 || { tail -20 gpurun_out/prof_LK4u_summary.txt; exit 1; }
  head -8 gpurun_out/prof_LK4u_summary.txt
fi
