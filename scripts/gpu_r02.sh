#!/bin/bash
# Round-2 GPU session: every GPU test (reports printed), the default bench, the other BASELINE
# configs, and the cache-proof cost-volume PMC passes.  Stops at the first abort / fault / timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
stop() { echo "$1 rc=$2: stopping"; exit "$2"; }
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 300 --timeout-method thread -rf ${PYTEST_ARGS:-} \
      > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -3
  [ $rc -gt 1 ] && stop pytest $rc
fi
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --kernel-table gpurun_out/kernel_table.json \
    > gpurun_out/bench.log 2>&1 || stop bench $?
tail -1 gpurun_out/bench.log
for c in 3 2 4; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-extra --no-cpu-baseline \
      > gpurun_out/bench_c$c.log 2>&1 || stop bench_c$c $?
  tail -1 gpurun_out/bench_c$c.log | cut -c1-400
done
[ -n "$NO_PMC" ] && exit 0
rm -rf gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmc_gwc_f" -o f -- \
    python3 scripts/gwc_ring.py > gpurun_out/pmc_gwc_f.log 2>&1 || stop pmc_fetch $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmc_gwc_w" -o w -- \
    python3 scripts/gwc_ring.py > gpurun_out/pmc_gwc_w.log 2>&1 || stop pmc_write $?
# gwc_ring.py: L-K ring (3 fill + 24 timed launches), then configs[2] (2 fill + 8 timed), then concat
python3 scripts/pmc_kernel_avg.py gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w gwc_kernel "gwc ring B1 96x312 D48" \
    gwc_volume 199360512 gpurun_out/pmc_traffic_gwc.json 3 24
python3 scripts/pmc_kernel_avg.py gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w gwc_kernel "gwc ring B8 136x240 D48" \
    gwc_volume 1738014720 gpurun_out/pmc_traffic_gwc.json 29 8
rm -rf gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w
exit 0
