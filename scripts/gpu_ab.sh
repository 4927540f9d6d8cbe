#!/bin/bash
# A/B of two library builds on one box: marginal per-op costs with ESM_LIB=$LIBA, then the in-tree
# library, then $LIBA again (drift check).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
    timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "$TESTS" \
        --timeout 120 --timeout-method thread > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
    tail -1 gpurun_out/pytest_iter.log
fi
V=${VARIANTS:-S}
ESM_LIB=${LIBA:-esmstereo_amd/_ab/libA.so} timeout -k 10 300 python -u scripts/step_tune.py --mode marginal --variants $V \
    --rounds 2 --report gpurun_out/marginal_A.json > gpurun_out/marginal_A.log 2>&1 || { tail -20 gpurun_out/marginal_A.log; exit 1; }
timeout -k 10 300 python -u scripts/step_tune.py --mode marginal --variants $V --rounds 2 \
    --report gpurun_out/marginal_B.json > gpurun_out/marginal_B.log 2>&1 || { tail -20 gpurun_out/marginal_B.log; exit 1; }
ESM_LIB=${LIBA:-esmstereo_amd/_ab/libA.so} timeout -k 10 300 python -u scripts/step_tune.py --mode marginal --variants $V \
    --rounds 2 --report gpurun_out/marginal_A2.json > gpurun_out/marginal_A2.log 2>&1 || { tail -20 gpurun_out/marginal_A2.log; exit 1; }
python scripts/ab_compare.py gpurun_out/marginal_A.json gpurun_out/marginal_B.json
python scripts/ab_compare.py gpurun_out/marginal_A.json gpurun_out/marginal_A2.json | head -3
