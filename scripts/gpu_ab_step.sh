#!/bin/bash
# A/B of two library builds by whole-step time only, alternated A B A B A B on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
LA=${LIBA:-esmstereo_amd/_ab/libA.so}
for i in 1 2 3; do
    ESM_LIB=$LA timeout -k 10 120 python -u scripts/step_tune.py --mode step --variants ${VARIANTS:-S} \
        --report gpurun_out/abstep_A$i.json 2>&1 | grep "step" | sed "s/^/A$i /" || exit 1
    timeout -k 10 120 python -u scripts/step_tune.py --mode step --variants ${VARIANTS:-S} \
        --report gpurun_out/abstep_B$i.json 2>&1 | grep "step" | sed "s/^/B$i /" || exit 1
done
