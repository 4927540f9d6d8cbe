"""The profile scripts' trace-to-op mapping (scripts/pmc_traffic.py): an op that launches several kernels
(the two-launch FMBlock) takes the sum of its kernels, and the later ops keep their positions."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "scripts"))
from pmc_traffic import assign, kernel_ops, whole_steps  # noqa: E402


def test_multi_kernel_ops_map_by_position():
    ops = [{"name": "a"}, {"name": "fm", "launches": 2}, {"name": "c"}]
    assert kernel_ops(ops) == [0, 1, 1, 2]
    step = [1.0, 10.0, 20.0, 3.0]
    seq = [99.0] + step * 3  # a partial step first, then 3 whole steps
    assert whole_steps(seq, 4, timed=2) == step * 2
    assert assign(seq, ops, timed=3) == {0: 1.0, 1: 30.0, 2: 3.0}
    assert assign(step * 2, ops) == {0: 1.0, 1: 30.0, 2: 3.0}  # every whole step but the oldest
