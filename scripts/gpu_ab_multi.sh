#!/bin/bash
# Step time of several library builds ($LIBS, space separated), rotated 3 times on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
for i in 1 2 3; do
    for L in $LIBS; do
        ESM_LIB=$L timeout -k 10 120 python -u scripts/step_tune.py --mode step --variants ${VARIANTS:-S} --rounds 3 \
            --report gpurun_out/abm.json 2>&1 | grep "step" | sed "s|^|$(basename $L) r$i |" || exit 1
    done
done
