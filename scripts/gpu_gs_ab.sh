cd "${GRAFT_REPO_ROOT}" && mkdir -p gpurun_out && export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -k "gwc_stem or tile3_form or volumes_vs" --timeout 200 --timeout-method thread > gpurun_out/pytest_gs.log 2>&1 || { tail -40 gpurun_out/pytest_gs.log; exit 1; }
tail -2 gpurun_out/pytest_gs.log
for i in 1 2; do for v in 1 0; do
  ESM_GWC_STEM=$v timeout -k 10 200 python -u scripts/step_tune.py --mode step --variants L --batch 4 --rounds 2 2>&1 | grep step | sed "s/^/gs=$v /"
done; done
