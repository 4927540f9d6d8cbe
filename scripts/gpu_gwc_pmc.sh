#!/bin/bash
# PMC traffic of the cache-proof cost-volume launches (bench.py cost_volume_roofline / concat_volume_roofline):
# two separate counter passes (no trace domains), then the per-launch summary merged into
# profiles/pmc_traffic.json (the keys bench.py's roofline_cost_volume* lines read).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$PWD/gpurun_out/pmc_gwc_f" -o f -- \
    python3 scripts/gwc_ring.py > gpurun_out/pmc_gwc_f.log 2>&1 || { tail -5 gpurun_out/pmc_gwc_f.log; exit 3; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$PWD/gpurun_out/pmc_gwc_w" -o w -- \
    python3 scripts/gwc_ring.py > gpurun_out/pmc_gwc_w.log 2>&1 || { tail -5 gpurun_out/pmc_gwc_w.log; exit 3; }
cp profiles/pmc_traffic.json gpurun_out/pmc_traffic.json
python3 scripts/gwc_ring.py --summarize gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w gpurun_out/pmc_traffic.json
