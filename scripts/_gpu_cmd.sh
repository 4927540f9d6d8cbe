timeout -k 10 300 python scripts/probe_epilogue.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra > gpurun_out/probe_noact.log 2>&1; tail -3 gpurun_out/probe_noact.log | cut -c1-300
