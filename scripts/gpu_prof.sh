#!/bin/bash
# rocprofv3 kernel trace of a short bench run, mapped onto the hot-path launch list, then two
# PMC passes (FETCH_SIZE, WRITE_SIZE — separate passes, no trace domains) for per-op traffic.
# Usage (on the GPU box): bash scripts/gpu_prof.sh [tag] [extra bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=${1:-run}
shift || true
mkdir -p gpurun_out
rm -rf "gpurun_out/prof_$tag" "gpurun_out/pmcf_$tag" "gpurun_out/pmcw_$tag"
BENCH=(bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --no-marginal "$@")
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_$tag" -o "$tag" -- \
    python3 "${BENCH[@]}" --kernel-table "gpurun_out/ops_$tag.json" > "gpurun_out/prof_bench_$tag.log" 2>&1
rc=$?
if [ $rc -ne 0 ]; then tail -20 "gpurun_out/prof_bench_$tag.log"; exit $rc; fi
python3 scripts/prof_ops.py "gpurun_out/prof_$tag" "gpurun_out/ops_$tag.json" > "gpurun_out/prof_ops_$tag.txt"
head -30 "gpurun_out/prof_ops_$tag.txt"
[ -n "$NO_PMC" ] && exit 0
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmcf_$tag" -o f -- \
    python3 "${BENCH[@]}" > "gpurun_out/pmcf_bench_$tag.log" 2>&1 || { tail -5 "gpurun_out/pmcf_bench_$tag.log"; exit 3; }
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmcw_$tag" -o w -- \
    python3 "${BENCH[@]}" > "gpurun_out/pmcw_bench_$tag.log" 2>&1 || { tail -5 "gpurun_out/pmcw_bench_$tag.log"; exit 3; }
WL=$(python3 -c "import json; l=[x for x in open('gpurun_out/prof_bench_$tag.log') if x.startswith('{\"metric')][-1]; print(json.loads(l)['config']['workload'].split(', ')[-1])")
python3 scripts/pmc_traffic.py "gpurun_out/pmcf_$tag" "gpurun_out/pmcw_$tag" "gpurun_out/ops_$tag.json" "$WL" \
    gpurun_out/pmc_traffic.json > "gpurun_out/pmc_traffic_$tag.txt"
cat "gpurun_out/pmc_traffic_$tag.txt"
