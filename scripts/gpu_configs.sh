#!/bin/bash
# Full-size parity at every BASELINE config, then one bench line per single-GPU config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf -s -k full_size \
    > gpurun_out/pytest_full.log 2>&1
rc=$?
grep -E "PASS|FAIL|flips|Error|error" gpurun_out/pytest_full.log | tail -20
[ $rc -ne 0 ] && { echo "pytest rc=$rc: stopping"; exit $rc; }
run() {
  tag=$1; shift
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-extra --no-cpu-baseline "$@" > gpurun_out/bench_$tag.log 2>&1
  brc=$?
  tail -1 gpurun_out/bench_$tag.log
  return $brc
}
run LK --variant L && run LSF --variant L --batch 8 --height 544 --width 960 && \
run MID --variant L --height 1024 --width 1504 --maxdisp 256 && run SKnc --cv nc && run SK8 --batch 8
