#!/bin/bash
# rocprofv3 kernel trace of a short bench run, mapped onto the hot-path launch list.
# Usage (on the GPU box): bash scripts/gpu_prof.sh [tag] [extra bench args...]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
tag=${1:-run}
shift || true
mkdir -p gpurun_out
rm -rf "gpurun_out/prof_$tag"
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_$tag" -o "$tag" -- \
    python3 bench.py --steps 20 --warmup 5 --no-extra --no-cpu-baseline --kernel-table "gpurun_out/ops_$tag.json" "$@" \
    > "gpurun_out/prof_bench_$tag.log" 2>&1
rc=$?
if [ $rc -ne 0 ]; then tail -20 "gpurun_out/prof_bench_$tag.log"; exit $rc; fi
python3 scripts/prof_ops.py "gpurun_out/prof_$tag" "gpurun_out/ops_$tag.json" > "gpurun_out/prof_ops_$tag.txt"
head -30 "gpurun_out/prof_ops_$tag.txt"
