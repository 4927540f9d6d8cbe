#!/bin/bash
# Step time under several environment settings ($ENVS, space separated NAME=VALUE), rotated 3 times.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
    for E in $ENVS; do
        env $E timeout -k 10 120 python -u scripts/step_tune.py --mode step --variants ${VARIANTS:-S} --rounds 3 \
            --report gpurun_out/abe.json 2>&1 | grep "step" | sed "s|^|$E r$i |" || exit 1
    done
done
