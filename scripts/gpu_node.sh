#!/bin/bash
# Node-analogue and confidence-head GPU tests, then the node CLI on two synthetic KITTI-sized pairs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_node.py tests/test_gpu_confidence.py -m gpu -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/pytest_node.log 2>&1 || { tail -40 gpurun_out/pytest_node.log; exit 1; }
tail -2 gpurun_out/pytest_node.log
python - <<'PY'
import os, numpy as np
from PIL import Image
rng = np.random.default_rng(0)
for side in ("image_2", "image_3"):
    os.makedirs(f"/tmp/kitti/{side}", exist_ok=True)
for i in range(2):
    l = rng.integers(0, 256, (375, 1242, 3), dtype=np.uint8)
    Image.fromarray(l).save(f"/tmp/kitti/image_2/{i:06d}_10.png")
    Image.fromarray(np.roll(l, -8, axis=1)).save(f"/tmp/kitti/image_3/{i:06d}_10.png")
PY
timeout -k 10 200 python -u scripts/esm_node.py --left /tmp/kitti/image_2 --right /tmp/kitti/image_3 \
    --out gpurun_out/node_out > gpurun_out/node_cli.log 2>&1 || { tail -20 gpurun_out/node_cli.log; exit 1; }
tail -3 gpurun_out/node_cli.log
python -c "from PIL import Image; im=Image.open('gpurun_out/node_out/000000_10.png'); print(im.mode, im.size)"
