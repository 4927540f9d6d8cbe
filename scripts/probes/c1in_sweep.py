"""Graph-chain time per launch of the single-input-channel layers: forced VALU form (hint bit 20)
vs the tuned / automatic MFMA form.    python scripts/probes/c1in_sweep.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from chain_floor import conv_case, timed  # noqa: E402

C1IN = 1 << 20
SHAPES = [(16, 3, 2, (384, 1248)), (16, 3, 2, (96, 312)), (16, 5, 1, (96, 312)), (16, 5, 1, (24, 78)),
          (32, 3, 2, (384, 1248)), (32, 5, 1, (192, 624)), (32, 5, 1, (48, 156))]


def main():
    dev = torch.device("cuda")
    for cout, k, s, hw in SHAPES:
        t_mfma = timed(conv_case(dev, 2, 1, cout, k, s, hw, hint=0x241))
        t_auto = timed(conv_case(dev, 2, 1, cout, k, s, hw, hint=0))
        t_valu = timed(conv_case(dev, 2, 1, cout, k, s, hw, hint=C1IN))
        print(f"1->{cout} k{k}s{s} {hw[0]}x{hw[1]}: direct-mfma {t_mfma:7.2f}  auto {t_auto:7.2f}  valu {t_valu:7.2f} us",
              flush=True)


if __name__ == "__main__":
    main()
