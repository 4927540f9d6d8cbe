import os, sys, torch
sys.path.insert(0, '/root/repo'); sys.path.insert(0, os.environ.get('GRAFT_REPO_ROOT', '.'))
from esmstereo_amd.engine import ACT_GELU, Ctx, pack_conv, run_conv
dev = torch.device('cuda')
for (cin, cout, shape) in [(32, 8, (48, 96, 312)), (8, 8, (48, 96, 312)), (32, 8, (12, 24, 78)), (32, 8, (24, 48, 156))]:
    conv = torch.nn.Conv3d(cin, cout, 3, 1, 1, bias=False).to(dev); bn = torch.nn.BatchNorm3d(cout).eval().to(dev)
    p = pack_conv(conv, bn, ACT_GELU); x = torch.randn(1, cin, *shape, device=dev); out = torch.empty(1, cout, *shape, device=dev)
    for h in (0, 1 << 17, 1 << 24):
        run_conv(Ctx(dev), p, [x], out=out, hint=h); torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 20
        e0.record()
        for _ in range(n): run_conv(Ctx(dev), p, [x], out=out, hint=h)
        e1.record(); torch.cuda.synchronize()
        print(cin, cout, shape, hex(h), round(e0.elapsed_time(e1) / n * 1e3, 1), 'us')
