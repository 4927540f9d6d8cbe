#!/bin/bash
# SQ counter passes over a few conv layers (scripts/conv_sweep.py, automatic tile) — one
# rocprofv3 --pmc pass per counter group, no trace domains mixed in.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_conv
rm -rf $OUT && mkdir -p $OUT
ONLY="${ONLY:-ref4x.conv1.1,tail4x,group_stem 3d k3 32->8 12x}"
HINTS="${HINTS:-0}"
pass() {
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --pmc "$@" -d $OUT/p$n -o p$n --output-format csv -- \
    python3 scripts/conv_sweep.py --reps 4 --iters 2 --only "$ONLY" --hints "$HINTS" > $OUT/p$n.log 2>&1
}
PASSES="${PASSES:-1 2 3 4}"
run_pass() { case " $PASSES " in *" $1 "*) pass "$@";; *) true;; esac; }
run_pass 1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS &&
run_pass 2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE &&
run_pass 3 FETCH_SIZE &&
run_pass 4 WRITE_SIZE &&
run_pass 5 TCC_HIT_sum TCC_MISS_sum &&
run_pass 6 TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
rc=$?
python3 scripts/pmc_summary.py $OUT
exit $rc
