cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -rf -k "stem or conv3d or checkpoint" > gpurun_out/pytest_a.log 2>&1; rc=$?; tail -2 gpurun_out/pytest_a.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python scripts/probes/stem_sweep.py > gpurun_out/stem_sweep.txt 2>&1; cat gpurun_out/stem_sweep.txt
