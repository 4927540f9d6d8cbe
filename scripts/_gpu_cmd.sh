cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for v in S L; do
timeout -k 10 300 python bench.py --variant $v --steps 50 --warmup 10 --no-extra --no-cpu-baseline --kernel-table gpurun_out/kt_$v.json > gpurun_out/bench_$v.log 2>&1 || exit 1; tail -1 gpurun_out/bench_$v.log | cut -c1-140
done
