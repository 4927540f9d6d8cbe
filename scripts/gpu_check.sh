#!/bin/bash
# One GPU-box session: parity tests, smoke, parity report, short bench.  Stops at the first GPU
# fault / abort / timeout (exit codes other than 0 or 1 from pytest, any failure elsewhere).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -m pytest tests -m gpu -q -rf ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -40 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc=$rc: stopping"; exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
src=$?
tail -3 gpurun_out/smoke.log
if [ $src -ne 0 ]; then echo "smoke rc=$src: stopping"; exit $src; fi
for v in S L; do
  timeout -k 10 300 python tests/parity_report.py --variant $v > gpurun_out/parity_$v.json 2> gpurun_out/parity_$v.err
  prc=$?; cat gpurun_out/parity_$v.json
  if [ $prc -ne 0 ]; then tail -5 gpurun_out/parity_$v.err; echo "parity rc=$prc: stopping"; exit $prc; fi
done
timeout -k 10 600 python bench.py --steps ${BENCH_STEPS:-50} --warmup 10 --kernel-table gpurun_out/kernel_table.json \
    > gpurun_out/bench.log 2>&1
brc=$?
tail -3 gpurun_out/bench.log
exit $(( rc > brc ? rc : brc ))
