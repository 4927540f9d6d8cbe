#!/bin/bash
# Scratch entry for ad-hoc GPU-box runs (gpurun -- 'bash scripts/_gpu_cmd.sh'): edit locally per
# experiment.  Default: the parity tests, then a short bench with the per-op probe table.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
bash scripts/gpu_iter.sh
