#!/bin/bash
# Confidence-head GPU tests, then the wall-time form tuning of the S hot path.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_confidence.py -m gpu -x -v -s --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_conf.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error|max \|" gpurun_out/pytest_conf.log | tail -30
case $rc in 0|1) ;; *) echo "pytest rc=$rc: stopping"; exit $rc ;; esac
[ -n "$NO_TUNE" ] && exit 0
bash scripts/gpu_step_tune.sh
