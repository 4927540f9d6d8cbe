"""The backbone side on the HIP kernels (round 5, esmstereo_amd.backbone.fast_features, model._seq_fast /
_conv_fast): timm's blocks with BatchNorm folded into esm_conv_f32 epilogues and the depthwise convs on
esm_dwconv_f32, against the same modules' own PyTorch forward (MIOpen) on the same weights.  Parity against timm
itself stays unpinned (timm is absent); this pins the fast path to the module definitions restated in
backbone.py.  Tolerance: relative 1e-4 of each output's max (fp32, different summation orders over up to 960
channels and a dozen layers)."""
import copy

import pytest
import torch
import torch.nn.functional as F

import esmstereo_amd as E
from esmstereo_amd.backbone import Feature, fast_path_ok
from esmstereo_amd.engine import ACT_NONE, ACT_RELU6, ACT_SILU, Ctx, run_dwconv

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda", 0)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def _randomize_bn(m: torch.nn.Module, seed: int) -> None:
    g = torch.Generator().manual_seed(seed)
    for mod in m.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            n = mod.num_features
            mod.running_mean.copy_(torch.randn(n, generator=g) * 0.1)
            mod.running_var.copy_(torch.rand(n, generator=g) * 0.5 + 0.5)
            mod.weight.data.copy_(torch.rand(n, generator=g) * 0.5 + 0.75)
            mod.bias.data.copy_(torch.randn(n, generator=g) * 0.1)


@pytest.mark.parametrize("k,s", [(3, 1), (3, 2), (5, 1), (5, 2)])
@pytest.mark.parametrize("act", [ACT_NONE, ACT_RELU6, ACT_SILU])
def test_dwconv_vs_torch(k, s, act):
    torch.manual_seed(k * 10 + s + act)
    B, C, H, W = 2, 24, 37, 70
    x = torch.randn(B, C, H, W)
    w = torch.randn(C, 1, k, k) * 0.3
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    p = (k - 1) // 2 if s == 1 else ((s - 1) + (k - 1)) // 2
    ref = F.conv2d(x.double(), w.double(), None, s, p, 1, C) * sc.double().view(1, C, 1, 1) + sh.double().view(1, C, 1, 1)
    ref = {ACT_NONE: ref, ACT_RELU6: ref.clamp(0, 6), ACT_SILU: F.silu(ref)}[act]
    y = run_dwconv(Ctx(DEV), x.to(DEV), w.reshape(C, k * k).contiguous().to(DEV), sc.to(DEV), sh.to(DEV), k, s, p, act)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-5


@pytest.mark.parametrize("backbone", ["mobilenetv2_100", "efficientnet_b2"])
def test_feature_fast_path_vs_modules(backbone):
    feat = Feature(backbone)
    _randomize_bn(feat, 3)
    feat = feat.eval().to(DEV)
    x = torch.randn(2, 3, 128, 256, device=DEV)
    with torch.no_grad():
        assert fast_path_ok(feat, x)
        got = feat(x)
    with torch.enable_grad():  # the modules' own PyTorch forward (MIOpen) on the same weights
        assert not fast_path_ok(feat, x)
        ref = [t.detach() for t in feat(x)]
    assert len(got) == len(ref) == 5
    for i, (g, r) in enumerate(zip(got, ref)):
        assert g.shape == r.shape, i
        assert rel(g, r) < 1e-4, (backbone, i, rel(g, r))


def test_model_prefix_fast_vs_modules():
    """The whole backbone side of ESMStereo-S (Feature + stems + desc + semantic + conv_f2 / conv_f0) on the
    HIP path vs the modules' own forward: the matching features and every upsampler feature."""
    model = E.ESMStereo(192, True, False, "mobilenetv2_100", 16)
    _randomize_bn(model, 5)
    model = model.eval().to(DEV)
    left, right = torch.randn(1, 3, 128, 256, device=DEV), torch.randn(1, 3, 128, 256, device=DEV)
    with torch.no_grad():
        got = model.prefix(left, right)
    with torch.enable_grad():
        ref = model.prefix(left, right)
    flat = lambda o: [o[0], o[1], o[2]] + list(o[3])  # noqa: E731
    for i, (g, r) in enumerate(zip(flat(got), flat(ref))):
        assert rel(g, r.detach()) < 1e-4, (i, rel(g, r.detach()))


def test_dwconv_many_planes():
    """B * C above the 65535 z-grid limit (the backbone over [left; right] at configs[3]'s 32 pairs): the planes ride
    on grid x."""
    torch.manual_seed(7)
    B, C, H, W, k = 72, 1000, 5, 6, 3
    x = torch.randn(B, C, H, W)
    w = torch.randn(C, 1, k, k) * 0.3
    sc, sh = torch.rand(C) + 0.5, torch.randn(C) * 0.1
    ref = F.conv2d(x.double(), w.double(), None, 1, 1, 1, C) * sc.double().view(1, C, 1, 1) + sh.double().view(1, C, 1, 1)
    y = run_dwconv(Ctx(DEV), x.to(DEV), w.reshape(C, k * k).contiguous().to(DEV), sc.to(DEV), sh.to(DEV), k, 1, 1, ACT_NONE)
    assert rel(y, ref) < 1e-5
