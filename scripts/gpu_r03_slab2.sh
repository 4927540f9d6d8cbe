#!/bin/bash
# Round 3: shuffle_tail / conv-form tests, the XCD-slab threshold A/B ($ENVS, S and L), then the S-K op
# map + memory-side traffic under each setting in $PROF_ENVS.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -k "${TESTS:-shuffle or stem_form or tile_variant or wide}" \
    --timeout 120 --timeout-method thread > gpurun_out/pytest_slab2.log 2>&1 || { tail -40 gpurun_out/pytest_slab2.log; exit 1; }
tail -1 gpurun_out/pytest_slab2.log
VARIANTS="S,L" bash scripts/gpu_ab_env.sh || exit 1
for E in $PROF_ENVS; do
    n=slab${E#*=}
    env $E bash scripts/gpu_prof.sh $n > gpurun_out/prof_$n.out 2>&1 || { tail -5 gpurun_out/prof_$n.out; exit 1; }
    cp gpurun_out/pmc_traffic.json gpurun_out/pmc_traffic_$n.json
    head -1 gpurun_out/prof_ops_$n.txt | sed "s|^|$n |"
    grep -E "tail4x|blocks" gpurun_out/prof_ops_$n.txt | sed "s|^|$n |"
    python3 - "$n" <<'PY'
import json, sys
n = sys.argv[1]
d = json.load(open(f"gpurun_out/pmc_traffic_{n}.json"))
d = d[[k for k in d if k.startswith("ESMStereo")][0]]
tot = sum(v["hbm_bytes_per_launch"] for v in d.values()); alg = sum(v["algorithmic_bytes"] for v in d.values())
print(n, "step total %.1f MB / alg %.1f MB" % (tot / 1e6, alg / 1e6))
for k, v in sorted(d.items(), key=lambda kv: -kv[1]["hbm_bytes_per_launch"])[:24]:
    print(n, "%-44s %7.2f MB alg %6.2f  x%.2f" % (k, v["hbm_bytes_per_launch"] / 1e6, v["algorithmic_bytes"] / 1e6,
                                                  v["hbm_bytes_per_launch"] / max(1, v["algorithmic_bytes"])))
PY
done
