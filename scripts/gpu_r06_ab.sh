#!/bin/bash
# Round 6: (1) S-K step with the XCD-slab tile order forced on the over-fetching small ops vs the default
# order (three rotations), (2) their PMC traffic under the forced order, (3) the L-K B4 op table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
OPS="upsample_module.spx_4x.0,agg,group_stem,upsample_module.ref4x.conv3.0,upsample_module.ref2x.conv1.1,upsample_module.ref4x.conv2.1,upsample_module.ref4x.agg_0.1,upsample_module.ref2x.agg_1.1,upsample_module.ref2x.conv2.1"
ENVS="ESM_XCD_SLAB_OPS=$OPS|ESM_XCD_SLAB_OPS=" bash scripts/ab_env.sh > gpurun_out/ab_xcd_SK.txt 2>&1 || { tail -5 gpurun_out/ab_xcd_SK.txt; exit 1; }
cat gpurun_out/ab_xcd_SK.txt
ESM_AB=1 ESM_XCD_SLAB_OPS=$OPS bash scripts/gpu_prof.sh SKslab > gpurun_out/prof_SKslab_summary.txt 2>&1 || { tail -20 gpurun_out/prof_SKslab_summary.txt; exit 1; }
NO_PMC=1 bash scripts/gpu_prof.sh iter --variant L --batch 4 > gpurun_out/prof_iter_summary.txt 2>&1 || { tail -20 gpurun_out/prof_iter_summary.txt; exit 1; }
head -3 gpurun_out/prof_ops_iter.txt
