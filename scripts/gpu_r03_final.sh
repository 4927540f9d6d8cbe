#!/bin/bash
# Round-3 final evidence for the headline config on the final tree: every GPU test, the default bench line
# (all side measurements), then rocprofv3 kernel stats + op map + PMC traffic of the S-K step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_full.sh || exit 1
bash scripts/gpu_prof.sh SK > gpurun_out/prof_SK_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SK_summary.txt; exit 1; }
head -14 gpurun_out/prof_SK_summary.txt
