"""The cache-proof cost-volume measurement of bench.py alone, for rocprofv3 PMC passes:
gwc at ESMStereo-L KITTI (B=1, 64 ch, 96x312, D=48) over a ring of buffers larger than twice the
Infinity Cache, then gwc and build_concat_volume at BASELINE configs[2] (L-SF B=8).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_gwc_f -o f -- python3 scripts/gwc_ring.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_gwc_w -o w -- python3 scripts/gwc_ring.py
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    out = {"gwc_L_K": bench.cost_volume_roofline(dev, reps=24),
           "gwc_configs2": bench.cost_volume_roofline(dev, reps=8, B=8, H=136, W=240, D=48),
           "concat_configs2": bench.concat_volume_roofline(dev)}
    print(json.dumps(out))
