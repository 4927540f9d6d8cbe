#!/bin/bash
# Kernel iteration on the GPU box: selected GPU tests ($TESTS, a pytest -k expression), a short
# bench line (in-graph marginal costs per op), and the per-op device-time table from a rocprofv3
# kernel trace of the same bench (scripts/prof_ops.py).  Stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
    timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "$TESTS" --timeout 120 --timeout-method thread \
        > gpurun_out/pytest_iter.log 2>&1 || { tail -40 gpurun_out/pytest_iter.log; exit 1; }
    tail -2 gpurun_out/pytest_iter.log
fi
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-extra ${BENCH_ARGS:-} \
    --kernel-table gpurun_out/ops_bench.json > gpurun_out/bench_iter.log 2>&1 || { tail -20 gpurun_out/bench_iter.log; exit 1; }
python3 -c "
import json; l=[x for x in open('gpurun_out/bench_iter.log') if x.startswith('{')][-1]; d=json.loads(l)
print('value', d['value'], 'ms', d['ms_per_step'], 'launches', d['config']['launches_per_step'], 'sum_marg', d.get('sum_of_marginals_us'))
print('roofline', d['roofline']['kernel'], d['roofline']['avg_us'], d['roofline']['frac'])
print('top', d.get('top_ops_in_graph'))"
[ -n "$NO_PROF" ] && exit 0
rm -rf gpurun_out/prof_iter
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_iter -o run -- \
    python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-marginal ${BENCH_ARGS:-} \
    --kernel-table gpurun_out/ops_iter.json > gpurun_out/prof_iter.log 2>&1 || { tail -20 gpurun_out/prof_iter.log; exit 1; }
python3 scripts/prof_ops.py gpurun_out/prof_iter gpurun_out/ops_iter.json > gpurun_out/ops_iter.txt
rm -rf gpurun_out/prof_iter
head -70 gpurun_out/ops_iter.txt
