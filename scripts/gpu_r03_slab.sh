#!/bin/bash
# Round 3: full GPU suite, then the XCD-slab size threshold A/B (step rotation, S and L), then the
# S-K op map + memory-side traffic of the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/pytest_full.log 2>&1 || { tail -40 gpurun_out/pytest_full.log; exit 1; }
tail -2 gpurun_out/pytest_full.log
ENVS="ESM_XCD_SLAB_MIN_PIX=65536 ESM_XCD_SLAB_MIN_PIX=1000000000" VARIANTS="S,L" bash scripts/gpu_ab_env.sh || exit 1
bash scripts/gpu_prof.sh sk > gpurun_out/prof_sk.out 2>&1 || { tail -5 gpurun_out/prof_sk.out; exit 1; }
head -3 gpurun_out/prof_ops_sk.txt; cat gpurun_out/pmc_traffic_sk.txt
