export PYTEST_ARGS='-k shuffle_tail'
bash scripts/gpu_iter.sh
