bash scripts/gpu_iter.sh && timeout -k 10 600 python -u scripts/autotune.py --variants S --out gpurun_out/tuned_hints.json > gpurun_out/autotune.log 2>&1; tail -2 gpurun_out/autotune.log
