#!/bin/bash
# SQ counter passes over a short bench run (every hot-path kernel), one rocprofv3 --pmc pass per
# counter group, no trace domains mixed in; summary per kernel symbol (scripts/pmc_summary.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_bench
rm -rf $OUT && mkdir -p $OUT
pass() {
  local n=$1; shift
  timeout -s KILL 240 rocprofv3 --pmc "$@" -d $OUT/p$n -o p$n --output-format csv -- \
    python3 bench.py --steps 5 --warmup 2 --no-extra --no-cpu-baseline > $OUT/p$n.log 2>&1
}
pass 1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
pass 2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE
rc=$?
tail -3 $OUT/p1.log $OUT/p2.log
python3 scripts/pmc_summary.py $OUT > gpurun_out/pmc_bench_summary.txt
rm -rf $OUT/p1 $OUT/p2  # raw per-dispatch CSVs: too large to bring back
exit $rc
