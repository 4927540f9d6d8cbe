#!/bin/bash
# Wall-time tuning of every conv's form (scripts/step_tune.py), then a bench line with the result.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
cp esmstereo_amd/tuned_hints.json gpurun_out/tuned_hints.json
timeout -k 10 900 python -u scripts/step_tune.py --mode tune --variants ${VARIANTS:-S} --rounds ${ROUNDS:-5} --margin-us ${MARGIN:-0.5} \
    ${ONLY:+--only $ONLY} ${BATCH:+--batch $BATCH} \
    --out gpurun_out/tuned_hints.json --report gpurun_out/step_tune_report.json > gpurun_out/step_tune.log 2>&1 \
    || { tail -30 gpurun_out/step_tune.log; exit 1; }
grep -v "0.00 us" gpurun_out/step_tune.log | tail -60
cp gpurun_out/tuned_hints.json esmstereo_amd/tuned_hints.json
timeout -k 10 200 python -u bench.py --steps 300 --warmup 20 --no-cpu-baseline --no-extra ${BENCH_ARGS:-} > gpurun_out/bench_iter.log 2>&1 \
    || { tail -20 gpurun_out/bench_iter.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_iter.log').read().strip().splitlines()[-1]);print('bench', d['value'], d['ms_per_step'])"
