"""Timing-only probe (never used for results): run bench.py with every conv's activation
replaced by identity, to price the activation part of the conv epilogues in the hot path.

    python scripts/probe_epilogue.py --steps 50 --warmup 10 --no-cpu-baseline --no-extra
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

torch.cuda.init()  # the HIP runtime first, as bench.py does (it imports torch before the package)
import esmstereo_amd.engine as eng  # noqa: E402

_pack = eng.pack_conv


def _pack_noact(conv, bn=None, act=eng.ACT_NONE):
    return _pack(conv, bn, eng.ACT_NONE)


for mod in ("esmstereo_amd.engine", "esmstereo_amd.blocks", "esmstereo_amd.mixer"):
    m = sys.modules.get(mod) or __import__(mod, fromlist=["x"])
    if hasattr(m, "pack_conv"):
        m.pack_conv = _pack_noact

import bench  # noqa: E402

bench.main()
