#!/bin/bash
# Round-3 check: every GPU test (no -x: a report of all failures), smoke, then the default bench.
# Stops at the first GPU fault / abort / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -rf ${PYTEST_ARGS:-} \
    > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -5 gpurun_out/smoke.log; exit 3; }
tail -2 gpurun_out/smoke.log
timeout -k 10 600 python -u bench.py --kernel-table gpurun_out/kernel_table.json > gpurun_out/bench.log 2>&1
brc=$?
tail -2 gpurun_out/bench.log
exit $(( rc > brc ? rc : brc ))
