#!/bin/bash
# Re-tune the S-K conv forms by step time with the round-4 forms among the candidates; the merged table
# comes back as gpurun_out/tuned_hints.json (scripts/step_tune.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
cp esmstereo_amd/tuned_hints.json gpurun_out/tuned_hints.json
timeout -k 10 900 python -u scripts/step_tune.py --mode tune --variants S --rounds 3 --margin-us 0.4 \
    --out gpurun_out/tuned_hints.json > gpurun_out/step_tune.log 2>&1 || { tail -20 gpurun_out/step_tune.log; exit 1; }
grep -v "   0.00 us" gpurun_out/step_tune.log | tail -30
