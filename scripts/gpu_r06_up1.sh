cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "convt_1x1 or hot_path_golden or conv_small or conv_tile2_transposed or conv_tile3_transposed or forward_graph or hot_path_full_size_vs_oracle" --timeout 120 --timeout-method thread > gpurun_out/pytest_up1.log 2>&1; rc=$?; tail -5 gpurun_out/pytest_up1.log; [ $rc -eq 0 ] || exit $rc
ENVS="ESM_CONVT_1X1=1|ESM_CONVT_1X1=0|ESM_CONVT_1X1=1 ESM_CONVT_1X1_PAIRED=1" bash scripts/ab_env.sh
