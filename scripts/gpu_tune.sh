#!/bin/bash
# Autotune the conv forms of the hot path for the given variants (merged into a copy of the table).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
cp esmstereo_amd/tuned_hints.json gpurun_out/tuned_hints.json
timeout -k 10 900 python -u scripts/autotune.py --variants ${VARIANTS:-M,L} --out gpurun_out/tuned_hints.json \
    > gpurun_out/autotune.log 2>&1 || { tail -30 gpurun_out/autotune.log; exit 1; }
grep -E "step" gpurun_out/autotune.log
grep -E "best" gpurun_out/autotune.log | head -150
