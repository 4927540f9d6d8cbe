cd "${GRAFT_REPO_ROOT}" || exit 2
export TMPDIR=/tmp
OUT=gpurun_out/pmc_ic; rm -rf $OUT; mkdir -p $OUT
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
grep -o "SQC_[A-Z_0-9]*\|SQ_IFETCH[A-Z_]*\|SQ_INSTS_[A-Z_0-9]*" $OUT/counters.txt | sort -u | tr '\n' ' '
echo
timeout -k 10 300 rocprofv3 --pmc SQC_ICACHE_MISSES SQC_ICACHE_HITS SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU -d $OUT/p1 -o p1 --output-format csv -- \
  python3 scripts/conv_sweep.py --reps 4 --iters 2 --only "conv3.1,ref4x.conv1.1,group_stem 3d k3 32->8 12x" --hints 0 > $OUT/p1.log 2>&1
rc=$?
python3 scripts/pmc_summary.py $OUT | grep -v "at::native" 
exit $rc
