"""Round 6 probe: the plane-pair hybrid (conv_tile3.hip tconv3hz_kernel) vs the padded MT form, bitwise, per
rows-per-wave variant, with randomised BN statistics (prints max |diff|, differing elements, their couts)."""
import copy
import sys

import torch

sys.path.insert(0, ".")
from esmstereo_amd.engine import ACT_GELU, Ctx, pack_conv, run_conv  # noqa: E402

DEV = torch.device("cuda:0")
for cin, cout, shape, B in ((24, 24, (6, 12, 39), 1), (40, 40, (5, 7, 19), 2)):
    torch.manual_seed(cin + cout)
    conv = torch.nn.Conv3d(cin, cout, 3, 1, 1, bias=False)
    bn = torch.nn.BatchNorm3d(cout).eval()
    bn.running_mean.uniform_(-0.2, 0.2)
    bn.running_var.uniform_(0.5, 1.5)
    bn.weight.data.uniform_(0.8, 1.2)
    bn.bias.data.uniform_(-0.2, 0.2)
    p = pack_conv(copy.deepcopy(conv).to(DEV), copy.deepcopy(bn).to(DEV), ACT_GELU)
    x = torch.randn(B, cin, *shape, device=DEV)
    outs = {}
    for name, h in (("hz2", 1 << 26), ("hz4", 2 << 26), ("mt1", 1 << 26 | 1 << 29), ("mt2", 2 << 26 | 1 << 29)):
        outs[name] = run_conv(Ctx(DEV), p, [x], hint=(1 << 23) | h)
    torch.cuda.synchronize()
    for a_, b_ in (("hz2", "mt1"), ("hz2", "mt2"), ("hz4", "mt2"), ("mt1", "mt2"), ("hz2", "hz4")):
        d = (outs[a_] - outs[b_]).abs()
        nz = (d > 0).nonzero()
        print(cout, a_, b_, float(d.max()), int((d > 0).sum()), sorted(set(nz[:, 1].tolist()))[:20],
              sorted(set(nz[:, 2].tolist()))[:20])
