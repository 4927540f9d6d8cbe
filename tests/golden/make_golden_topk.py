"""Golden vectors for regression_topk at k != 2.

Run in the build container only (imports models/submodule.py from /root/reference through
make_golden.load_reference): ``python tests/golden/make_golden_topk.py``.  Writes
``tests/golden/topk_k.npz``: for each k in KS, a tie-free random cost [B, D, H, W], random
disparity samples, and the reference's ``regression_topk(cost, samples, k)`` output.  Tie-free
inputs make the reference's (unstable) torch.sort order unambiguous, so the fixture pins the
selection, the softmax and the weighted sum; ties are covered against the oracle in the tests.
"""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import load_reference  # noqa: E402

KS = (1, 2, 3, 4, 5, 8, 12, 48, 60)  # 48 = D (all), 60 > D (the slice clamps)


def main() -> None:
    sm, _ = load_reference()
    rng = np.random.default_rng(2024)
    B, D, H, W = 2, 48, 3, 8
    out = {"ks": np.array(KS, dtype=np.int64)}
    for k in KS:
        cost = rng.permutation(B * D * H * W).astype(np.float32).reshape(B, D, H, W) / (B * D * H * W) * 8.0 - 4.0
        samples = (rng.random((B, D, H, W)) * 48.0).astype(np.float32)
        ref = sm.regression_topk(torch.from_numpy(cost), torch.from_numpy(samples), k)
        out[f"cost_{k}"], out[f"samples_{k}"], out[f"out_{k}"] = cost, samples, ref.numpy()
    np.savez_compressed(os.path.join(HERE, "topk_k.npz"), **out)
    print("wrote topk_k.npz", {k: out[f"out_{k}"].shape for k in KS})


if __name__ == "__main__":
    main()
