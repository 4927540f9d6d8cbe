#!/bin/bash
# Round 6: the shuffle_conv11 tiles — parity, then the S-K step with each tile (three alternations).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "shuffle_conv_pre or hot_path_golden or convt_1x1 or hot_path_fullsize_vs_reference" --timeout 120 --timeout-method thread > gpurun_out/pytest_sc11.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_sc11.log; [ $rc -eq 0 ] || exit $rc
ENVS="ESM_SC11_TILE=0|ESM_SC11_TILE=1|ESM_SC11_TILE=2" bash scripts/ab_env.sh
