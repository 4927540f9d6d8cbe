"""CPU tests of the host side: C-ABI library loads and exports every declared symbol,
struct layouts agree, weight packing is right, the module tree mirrors the reference's
state dict, and the product path refuses CPU tensors (no fallback)."""
import ctypes
import json
import os
import re

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import GOLDEN_DIR, load_spec, module_spec

import esmstereo_amd
from esmstereo_amd import _lib
from esmstereo_amd.backbone import StubFeature
from esmstereo_amd.engine import pack_conv, pack_weight

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "esmstereo_amd.h")


def _declared_functions():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(esm_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    names = _declared_functions()
    assert len(names) >= 20
    lib = ctypes.CDLL(_lib.LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.SIGNATURES), set(names) ^ set(_lib.SIGNATURES)


def test_struct_layouts_match():
    for which, st in enumerate((_lib.EsmSrc, _lib.EsmConvDesc, _lib.EsmSmixStage, _lib.EsmSmixDesc)):
        assert _lib.lib.esm_struct_size(which) == ctypes.sizeof(st)


def test_error_path_without_gpu():
    # argument validation happens before any device work
    rc = _lib.lib.esm_gwc_volume_f32(None, None, None, None, 1, 64, 4, 4, 4, 32, None)
    assert rc == -1 and b"null" in _lib.lib.esm_last_error()
    d = _lib.EsmConvDesc()
    assert _lib.lib.esm_conv_f32(ctypes.byref(d), None) == -1


def test_plan_rebind_rejects_overlapping_ranges_without_gpu():
    """two old ranges that overlap would make the owner of a pointer ambiguous; the native
    rebind refuses them before touching any op (no device call: an empty plan)."""
    lib = _lib.lib
    plan = lib.esm_plan_create()
    try:
        n = 2
        olds = (_lib.c_void_p * n)(0x10000, 0x10100)
        sizes = (ctypes.c_uint64 * n)(0x200, 0x200)
        news = (_lib.c_void_p * n)(0x90000, 0xa0000)
        assert lib.esm_plan_rebind(plan, n, olds, sizes, news) == -1
        assert b"overlap" in lib.esm_last_error()
        olds = (_lib.c_void_p * n)(0x10000, 0x10200)  # adjacent, disjoint: accepted (nothing to move)
        assert lib.esm_plan_rebind(plan, n, olds, sizes, news) == 0
        assert lib.esm_plan_busy(plan) == 0  # never launched
    finally:
        lib.esm_plan_destroy(plan)


def _emulate_packed(x, P, transposed, k, s, p):
    """Reference-free emulation of the kernel's K-loop indexing on the CPU (3-D, float64)."""
    B, Cin, Di, Hi, Wi = x.shape
    x = x.double()
    P = P.double()
    if not transposed:
        Do, Ho, Wo = [(n + 2 * p - k) // s + 1 for n in (Di, Hi, Wi)]
        out = torch.zeros(B, P.shape[-1], Do, Ho, Wo, dtype=torch.float64)
        for od in range(Do):
            for oh in range(Ho):
                for ow in range(Wo):
                    for tap in range(k ** 3):
                        kd, kh, kw = tap // (k * k), (tap // k) % k, tap % k
                        i = (od * s - p + kd, oh * s - p + kh, ow * s - p + kw)
                        if all(0 <= a < n for a, n in zip(i, (Di, Hi, Wi))):
                            out[:, :, od, oh, ow] += x[:, :, i[0], i[1], i[2]] @ P[tap, :Cin]
        return out
    out = torch.zeros(B, P.shape[-1], 2 * Di, 2 * Hi, 2 * Wi, dtype=torch.float64)
    for od in range(2 * Di):
        for oh in range(2 * Hi):
            for ow in range(2 * Wi):
                q = (od & 1, oh & 1, ow & 1)
                m = (od >> 1, oh >> 1, ow >> 1)
                cls = (q[0] << 2) | (q[1] << 1) | q[2]
                for tap in range(8):
                    t = ((tap >> 2) & 1, (tap >> 1) & 1, tap & 1)
                    i = tuple(mi + qi - ti for mi, qi, ti in zip(m, q, t))
                    if all(0 <= a < n for a, n in zip(i, (Di, Hi, Wi))):
                        out[:, :, od, oh, ow] += x[:, :, i[0], i[1], i[2]] @ P[cls, tap, :Cin]
    return out


@pytest.mark.parametrize("k,s,p", [(3, 1, 1), (3, 2, 1), (1, 1, 0)])
def test_pack_conv3d_indexing(k, s, p):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 5, 4, 5, 6, generator=g)
    conv = torch.nn.Conv3d(5, 7, k, s, p, bias=False)
    P, cin_pad, cout_pad = pack_weight(conv.weight, False)
    assert P.shape == (k ** 3, 16, 32)
    ref = F.conv3d(x.double(), conv.weight.double(), None, s, p)
    got = _emulate_packed(x, P, False, k, s, p)[:, :7]
    assert torch.allclose(got, ref, atol=1e-9)


def test_pack_convtranspose3d_parity_classes():
    g = torch.Generator().manual_seed(1)
    x = torch.randn(1, 6, 3, 4, 5, generator=g)
    conv = torch.nn.ConvTranspose3d(6, 3, 4, 2, 1, bias=False)
    P, _, _ = pack_weight(conv.weight, True)
    assert P.shape == (8, 8, 16, 32)
    ref = F.conv_transpose3d(x.double(), conv.weight.double(), None, 2, 1)
    got = _emulate_packed(x, P, True, 4, 2, 1)[:, :3]
    assert torch.allclose(got, ref, atol=1e-9)


def test_pack_conv_folds_bn_and_bias():
    conv = torch.nn.Conv2d(4, 6, 3, 1, 1, bias=True)
    bn = torch.nn.BatchNorm2d(6).eval()
    bn.running_mean.uniform_(-1, 1)
    bn.running_var.uniform_(0.5, 2)
    bn.weight.data.uniform_(0.5, 1.5)
    bn.bias.data.uniform_(-1, 1)
    pc = pack_conv(conv, bn)
    x = torch.randn(1, 4, 5, 5)
    raw = F.conv2d(x, conv.weight, None, 1, 1)
    want = bn(F.conv2d(x, conv.weight, conv.bias, 1, 1))
    got = raw * pc.scale.view(1, -1, 1, 1) + pc.shift.view(1, -1, 1, 1)
    assert torch.allclose(got, want, atol=1e-5)


@pytest.mark.parametrize("var,cv", [(v, c) for v in "SML" for c in ("gwc", "nc")])
def test_state_dict_matches_reference(var, cv):
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        man = json.load(f)
    m = man[f"hot_{var}_{cv}.npz"]
    model = esmstereo_amd.ESMStereo(m["maxdisp"], cv == "gwc", cv == "nc", m["backbone"], m["cv_scale"],
                                    feature_cls=StubFeature)
    assert module_spec(model) == [tuple(e) for e in load_spec(m["spec"])]


def test_cpu_tensors_are_refused():
    x = torch.randn(1, 64, 4, 8)
    with pytest.raises(RuntimeError, match="ROCm"):
        esmstereo_amd.build_gwc_volume(x, x, 4, 32)
    model = esmstereo_amd.ESMStereo(64, True, False, "mobilenetv2_100", 16).eval()
    with pytest.raises(RuntimeError, match="ROCm"):
        model(torch.randn(1, 3, 64, 128), torch.randn(1, 3, 64, 128), False)


def test_training_mode_is_refused():
    model = esmstereo_amd.ESMStereo(64, True, False, "mobilenetv2_100", 16)
    with pytest.raises(NotImplementedError):
        model(torch.randn(1, 3, 64, 128), torch.randn(1, 3, 64, 128), False)


def test_models_registry():
    assert esmstereo_amd.__models__["ESMStereo"] is esmstereo_amd.ESMStereo
    assert esmstereo_amd.__models__["ESMStereo_trt"] is esmstereo_amd.ESMStereo_trt


def test_trt_signature_and_state_dict():
    """ESMStereo_trt (models/ESMStereo_trt.py:511-737): reference ctor, same state dict as ESMStereo,
    forward(left, right) without train_status (onnx_transformed.py:48-51 calls it with two inputs)."""
    import inspect
    a = esmstereo_amd.ESMStereo(192, True, False, "efficientnet_b2", 4)
    b = esmstereo_amd.__models__["ESMStereo_trt"](192, True, False, "efficientnet_b2", 4)
    assert [(k, v.shape) for k, v in a.state_dict().items()] == [(k, v.shape) for k, v in b.state_dict().items()]
    assert list(inspect.signature(b.forward).parameters) == ["left", "right"]
    with pytest.raises(RuntimeError, match="ROCm"):
        b.eval()(torch.randn(1, 3, 64, 128), torch.randn(1, 3, 64, 128))


def test_run_dwconv_rejects_bad_arguments():
    """run_dwconv refuses a W-strided view and non-positive stride / K or bad padding on the host,
    before any descriptor reaches the library."""
    import torch as _t
    from esmstereo_amd.engine import run_dwconv
    x = _t.zeros(1, 4, 8, 16)
    w = _t.zeros(4, 9)
    for kw in (dict(k=3, stride=0, pad=1), dict(k=0, stride=1, pad=0), dict(k=3, stride=1, pad=3)):
        with pytest.raises(ValueError):
            run_dwconv(None, x, w, None, None, act=0, **kw)
    with pytest.raises(ValueError):
        run_dwconv(None, x[..., ::2], w, None, None, 3, 1, 1, 0)
