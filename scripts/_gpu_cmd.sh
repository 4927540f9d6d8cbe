cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/probes/stem_sweep.py > gpurun_out/stem_sweep.txt 2>&1; cat gpurun_out/stem_sweep.txt
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-extra --no-cpu-baseline --kernel-table gpurun_out/kt_S.json > gpurun_out/bench_S.log 2>&1 && tail -1 gpurun_out/bench_S.log | cut -c1-250 && \
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-extra --no-cpu-baseline --variant L --kernel-table gpurun_out/kt_L.json > gpurun_out/bench_L.log 2>&1 && tail -1 gpurun_out/bench_L.log | cut -c1-250
