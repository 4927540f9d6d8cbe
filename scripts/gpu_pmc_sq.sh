#!/bin/bash
# Per-op SQ counters of the bench step: two rocprofv3 --pmc passes (8 SQ + GRBM counters each, no
# trace domains), mapped onto the launch list by scripts/pmc_ops.py.
# Usage (on the GPU box): bash scripts/gpu_pmc_sq.sh [tag] [extra bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=${1:-sk}
shift || true
OUT=gpurun_out/pmcsq_$tag
rm -rf $OUT && mkdir -p $OUT
BENCH=(bench.py --steps 10 --warmup 3 --no-extra --no-cpu-baseline --no-marginal --kernel-table $OUT/ops.json "$@")
pass() {
  local n=$1; shift
  timeout -s KILL 300 rocprofv3 --pmc "$@" -d "$PWD/$OUT/p$n" -o p$n --output-format csv -- \
    python3 "${BENCH[@]}" > $OUT/p$n.log 2>&1 || { tail -5 $OUT/p$n.log; return 3; }
}
pass 1 SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU &&
pass 2 SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_BUSY_CYCLES GRBM_GUI_ACTIVE || exit $?
python3 scripts/pmc_ops.py $OUT/ops.json $OUT/p1 $OUT/p2 > $OUT/summary.txt
head -70 $OUT/summary.txt
rm -rf $OUT/p1 $OUT/p2
