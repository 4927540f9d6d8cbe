"""Graph-chain time per launch of conv layers of the hot path under the automatic form, the forced
16-block narrow-output form (conv_stem.hip) and the automatic choice without it.
    python scripts/probes/stem_sweep.py
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from chain_floor import conv_case, timed  # noqa: E402

STEM, NO_STEM = 1 << 17, 1 << 18
SHAPES = [(3, 24, 24, (24, 48, 156)), (3, 32, 8, (48, 96, 312)), (3, 8, 8, (48, 96, 312)), (2, 32, 32, (192, 624)),
          (2, 16, 16, (192, 624)), (2, 32, 16, (192, 624)), (2, 16, 8, (96, 312)), (2, 16, 16, (96, 312)),
          (2, 16, 16, (24, 78)), (3, 12, 12, (6, 12, 39)), (3, 24, 24, (2, 3, 10)), (3, 16, 16, (3, 6, 20)),
          (3, 32, 8, (12, 24, 78)), (3, 8, 8, (12, 24, 78)), (3, 24, 24, (6, 12, 39)), (2, 16, 16, (48, 156))]


def main():
    dev = torch.device("cuda")
    print(f"{'layer':36s} {'auto':>8s} {'stem':>8s} {'no-stem':>8s}  (us / launch in a graph chain)")
    for nd, cin, cout, shape in SHAPES:
        t = [timed(conv_case(dev, nd, cin, cout, 3, 1, shape, hint=h)) for h in (0, STEM, NO_STEM)]
        name = f"{nd}d {cin}->{cout} {'x'.join(map(str, shape))}"
        print(f"{name:36s} {t[0]:8.2f} {t[1]:8.2f} {t[2]:8.2f}", flush=True)


if __name__ == "__main__":
    main()
