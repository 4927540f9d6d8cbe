"""Phase timeline of shuffle_conv4_kernel (S-K 4x stage: spx_4x.1 + upsampling4 + tail4x + ref4x.conv1.0)
inside the replayed S-K step (diagnostic build: ESM_LIB=<the --diag library>).  Phases: 0 start, 1 staging
(weights + pre-conv window to LDS), 2 pre-conv MFMA, 3 shuffled interior + ring, 4 tail -> x, 5 x row /
column, 6 c1 conv + stores issued, 7 stores drained."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
import esmstereo_amd as E  # noqa: E402
from esmstereo_amd import _lib  # noqa: E402
from helpers import fullsize_inputs, load_spec, seeded_state  # noqa: E402

DEV = torch.device("cuda:0")
model = E.ESMStereo(192, True, False, "mobilenetv2_100", 16, feature_cls=E.backbone.StubFeature)
model.load_state_dict(seeded_state(load_spec("spec_S_gwc.json"), 11))
model.eval().to(DEV)
a = fullsize_inputs(16, 1, 384, 1248, 192, 7, True)
ml, mr, att = (torch.from_numpy(x).to(DEV) for x in a[:3])
up = [torch.from_numpy(u).to(DEV) for u in a[3]]
for _ in range(30):
    model.hot_path(ml, mr, att, up)
torch.cuda.synchronize()
fn = _lib.lib.esm_diag_sc4_stamps
fn.restype, fn.argtypes = ctypes.c_int, [ctypes.c_void_p, ctypes.c_int]
G = int(os.environ.get("SC4_WGS", str(20 * 12)))
buf = (ctypes.c_ulonglong * (G * 8))()
assert fn(buf, G * 8) == G * 8
s = np.frombuffer(buf, dtype=np.uint64).astype(np.int64).reshape(G, 8)
names = ["stage (loads -> LDS)", "pre-conv MFMA", "shuffle interior + ring", "tail -> x", "x row / column",
         "c1 conv + stores issued", "stores drained"]
print(f"shuffle_conv4, {G} workgroups; total {(s[:, 7].max() - s[:, 0].min()) / 100:.2f} us, "
      f"start skew {(s[:, 0].max() - s[:, 0].min()) / 100:.2f} us, median WG span {np.median(s[:, 7] - s[:, 0]) / 100:.2f} us")
for k in range(7):
    d = (s[:, k + 1] - s[:, k]) / 100.0
    print(f"  {names[k]:28s} med {np.median(d):5.2f} us  max {d.max():5.2f}")
