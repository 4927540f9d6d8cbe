"""shuffle_tail forms at the S-K heads (nf 8, r 4): back-to-back launch time of each form (esm_shuffle_tail_desc
flags bits 1-2: window form, 4-row, 8-row row forms) and agreement between them.  Diagnostic only."""
import sys

import torch

sys.path.insert(0, ".")
from esmstereo_amd.engine import Ctx, pack_shuffle_tail, run_shuffle_tail  # noqa: E402

dev = torch.device("cuda")
for (H, W) in ((96, 312), (24, 78)):
    torch.manual_seed(0)
    up = torch.nn.Conv2d(8, 128, 1).to(dev)
    tail = torch.nn.Conv2d(8, 1, 3, 1, 1).to(dev)
    p = pack_shuffle_tail(up, tail, 4)
    x = torch.randn(1, 8, H, W, device=dev)
    outs = {}
    for form in (1, 2, 3):
        ctx = Ctx(dev)
        y = run_shuffle_tail(ctx, x, p, form=form)
        for _ in range(20):
            run_shuffle_tail(ctx, x, p, out=y, form=form)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(200):
            run_shuffle_tail(ctx, x, p, out=y, form=form)
        b.record()
        b.synchronize()
        outs[form] = y.clone()
        print(f"{H}x{W} form {form}: {a.elapsed_time(b) / 200 * 1e3:.2f} us/launch b2b")
    print("max |form2 - form1|", float((outs[2] - outs[1]).abs().max()), "max |form3 - form2|",
          float((outs[3] - outs[2]).abs().max()))
