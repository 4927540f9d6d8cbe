"""GPU parity tests: the HIP path (through the C ABI) against the reference goldens and the
CPU oracle.  Run on the MI355X box: ``python -m pytest tests -m gpu``.

Tolerances (fp32 everywhere; north_star: "EPE within 1e-3 of the PyTorch reference"):
* cost volumes gwc / concat and disparity_regression: bit-exact (same rounding sequence);
* norm-corr volume, top-2 regression, single convs, ShuffleMixer: relative max error <= 1e-5
  (different but equally exact fp32 summation orders);
* whole hot path, S / M: EPE (mean |d - d_ref|, px at full res) <= 1e-3 and relative max
  error <= 1e-4;
* whole hot path, L (``regression_topk`` is discontinuous at near-ties):
  the count of low-res pixels whose top-2 index set flips is reported, and EPE <= 1e-3 is
  required outside the dilated, upsampled flip mask.
"""
import copy
import json
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from helpers import GOLDEN_DIR, feature_pair, load_golden, load_spec, seeded_state, stereo_pair
from parity import check_fullsize, flip_masked, fullsize_case, fullsize_manifest, record_report, top2_sets

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a ROCm GPU")]

import esmstereo_amd as E  # noqa: E402
from esmstereo_amd.backbone import StubFeature  # noqa: E402
from esmstereo_amd.engine import Ctx, pack_conv, run_conv, ACT_GELU, ACT_SILU, ACT_NONE  # noqa: E402
from oracle import esm_oracle as O  # noqa: E402

DEV = torch.device("cuda")

with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
    MANIFEST = json.load(f)
HOT = sorted(k for k in MANIFEST if k.startswith("hot_"))


def cu(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def rel(a, b):
    a = a.detach().double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).detach().abs().max() / b.detach().abs().max().clamp_min(1e-30))


def epe(a, b):
    return float((a.detach().double().cpu() - torch.as_tensor(b).double().cpu()).abs().mean())


# ----------------------------------------------------------------------------- op level


def test_ops_golden():
    g = load_golden("ops.npz")
    V = E.build_gwc_volume(cu(g["gwc_L"]), cu(g["gwc_R"]), 8, 32)
    assert torch.equal(V.cpu(), torch.from_numpy(g["gwc_out"])), "gwc must be bit-exact"
    Va = E.build_gwc_volume(cu(g["gwc_L"]), cu(g["gwc_R"]), 8, 32, att=cu(g["gwc_att"]))
    assert torch.equal(Va.cpu(), torch.from_numpy(g["gwc_att_out"])), "gwc*att must be bit-exact"
    Vc = E.build_concat_volume(cu(g["concat_L"]), cu(g["concat_R"]), 6)
    assert torch.equal(Vc.cpu(), torch.from_numpy(g["concat_out"]))
    Vn = E.build_norm_correlation_volume(cu(g["nc_L"]), cu(g["nc_R"]), 7)
    assert rel(Vn, g["nc_out"]) < 1e-5
    r = E.disparity_regression(cu(g["reg_cost"]), 12)
    # torch's CPU sum over a strided dim is not a plain sequential sum (vectorised partial sums),
    # so the d-ordered HIP sum agrees to fp32 rounding, not bitwise
    assert rel(r, g["reg_out"]) < 1e-6
    tc = cu(g["topk_cost"])
    ds = torch.arange(0, 12, dtype=torch.float32, device=DEV).view(1, 12, 1, 1).repeat(2, 1, 5, 9)
    t = E.regression_topk(tc, ds, 2)
    assert rel(t, g["topk_out"]) < 1e-6


def test_topk_nan_ranks_first():
    """torch.sort(descending) ranks NaN above every number (the reference's regression_topk,
    submodule.py:218-225): a NaN cost plane is picked, and the softmax turns the pixel into NaN."""
    g = torch.Generator().manual_seed(4)
    cost = torch.randn(1, 12, 3, 5, generator=g)
    cost[0, 7, 1, 2] = float("nan")
    cost[0, 2, 0, 0] = cost[0, 9, 0, 0] = float("nan")
    got = E.regression_topk(cost.to(DEV), None, 2).cpu()
    ref = O.regression_topk2(cost)
    assert torch.equal(torch.isnan(got), torch.isnan(ref)) and bool(torch.isnan(ref[0, 0, 1, 2]))
    ok = ~torch.isnan(ref)
    assert rel(got[ok], ref[ok]) < 1e-6


@pytest.mark.parametrize("k", [1, 2, 3, 4, 5, 8, 9, 16, 48, 60])
def test_regression_topk_any_k(k):
    """regression_topk for any k (register top-k for k <= 8, selection passes above): vs the oracle
    (stable descending sort sliced [:, :k]) with exact ties and NaN planes, and vs the REFERENCE's
    own outputs (tests/golden/topk_k.npz, tie-free costs, random disparity samples) where the fixture
    holds k.  Relative 1e-6 (softmax and the weighted sum in rank order)."""
    gen = torch.Generator().manual_seed(100 + k)
    cost = torch.randn(2, 48, 9, 21, generator=gen)
    cost[0, 5, 0, :4] = cost[0, 9, 0, :4] = cost[0, 30, 0, :4] = 10.0  # 3-way exact ties
    cost[1, :, 3, 3] = 0.25  # a whole tied column: the lowest k indices
    cost[1, 7, 4, 4] = float("nan")
    samples = torch.rand(2, 48, 9, 21, generator=gen) * 48
    for smp in (None, samples):
        got = E.regression_topk(cost.to(DEV), None if smp is None else smp.to(DEV), k).cpu()
        ref = O.regression_topk(cost, smp, k)
        assert torch.equal(torch.isnan(got), torch.isnan(ref)), k
        ok = ~torch.isnan(ref)
        assert rel(got[ok], ref[ok]) < 1e-6, (k, smp is None)
    g = load_golden("topk_k.npz")
    if k in g["ks"].tolist():
        got = E.regression_topk(cu(g[f"cost_{k}"]), cu(g[f"samples_{k}"]), k)
        assert rel(got, g[f"out_{k}"]) < 1e-6, k
    # Python slicing of the sorted indices: k = 0 selects nothing (zeros), k = -1 all but the last
    assert torch.equal(E.regression_topk(cost.to(DEV), None, 0).cpu(), torch.zeros(2, 1, 9, 21))
    if k == 1:
        got = E.regression_topk(cost.to(DEV), None, -1).cpu()
        ref = O.regression_topk(cost, None, -1)
        ok = ~torch.isnan(ref)
        assert rel(got[ok], ref[ok]) < 1e-6


@pytest.mark.parametrize("B,C,H,W,D,G", [(1, 64, 24, 78, 12, 32), (2, 64, 7, 13, 9, 32), (1, 64, 5, 3, 8, 32),
                                          (3, 32, 6, 10, 5, 4), (1, 64, 96, 312, 48, 32), (1, 8, 4, 6, 1, 8)])
def test_volumes_vs_oracle(B, C, H, W, D, G):
    L, R = feature_pair(B, C, H, W, 5, max(D, 2))
    V = E.build_gwc_volume(L.to(DEV), R.to(DEV), D, G)
    if C // G <= 2:  # ESMStereo's 2-channel groups: bit-exact
        assert torch.equal(V.cpu(), O.gwc_volume(L, R, D, G))
    else:  # wider groups: torch's mean reduction order is not sequential
        assert rel(V, O.gwc_volume(L, R, D, G)) < 1e-6
    Vc = E.build_concat_volume(L.to(DEV), R.to(DEV), D)
    assert torch.equal(Vc.cpu(), O.concat_volume(L, R, D))
    Vn = E.build_norm_correlation_volume(L.to(DEV), R.to(DEV), D)
    assert rel(Vn, O.normcorr_volume(L, R, D)) < 1e-5


def test_regressions_vs_oracle():
    g = torch.Generator().manual_seed(3)
    cost = torch.randn(2, 48, 17, 33, generator=g)
    cost[0, 5, 0, :4] = cost[0, 9, 0, :4] = 10.0  # exact ties -> lowest index first
    out = E.disparity_regression(cost.to(DEV), 48)
    assert rel(out, O.disparity_regression(cost, 48)) < 1e-6
    full = torch.arange(48, dtype=torch.float32).view(1, 48, 1, 1).repeat(2, 1, 17, 33)  # as ESMStereo.py:719-720
    t = E.regression_topk(cost.to(DEV), full.to(DEV), 2)
    assert rel(t, O.regression_topk2(cost)) < 1e-6
    assert rel(t, O.regression_topk(cost, full, 2)) < 1e-6
    big = torch.rand(3, 50, 18, 35, generator=g) * 48  # larger than the index: gather reads its corner block
    t = E.regression_topk(cost.to(DEV), big.to(DEV), 2)
    assert rel(t, O.regression_topk(cost, big, 2)) < 1e-6
    with pytest.raises(RuntimeError):
        E.disparity_regression(cost.to(DEV), 47)
    # the reference's torch.gather(disparity_samples, 1, pool_ind) does not broadcast (submodule.py:223):
    # a [1, D, 1, 1] sample vector raises there, and here
    for bad in (full[:, :, :1, :1], full[:1], full[0], full[:, :40]):
        with pytest.raises(RuntimeError):
            O.regression_topk(cost, bad, 2)
        with pytest.raises(RuntimeError):
            E.regression_topk(cost.to(DEV), bad.contiguous().to(DEV), 2)


# ----------------------------------------------------------------------------- convs


def _ref_conv(x_list, conv, bn, act, mul=None, res=None, up=None, up_f=0, shuffle=1, post=1.0):
    x = torch.cat([t.double() for t in x_list], 1)
    w = conv.weight.detach().double()
    nd = w.dim() - 2
    if isinstance(conv, (torch.nn.ConvTranspose2d, torch.nn.ConvTranspose3d)):
        fn = F.conv_transpose3d if nd == 3 else F.conv_transpose2d
    else:
        fn = F.conv3d if nd == 3 else F.conv2d
    b = conv.bias.detach().double() if conv.bias is not None else None
    y = fn(x, w, b, conv.stride, conv.padding)
    if bn is not None:
        y = F.batch_norm(y, bn.running_mean.double(), bn.running_var.double(), bn.weight.double(), bn.bias.double(),
                         False, 0.0, bn.eps)
    if shuffle > 1:
        y = F.pixel_shuffle(y, shuffle)
    y = {ACT_GELU: F.gelu, ACT_SILU: F.silu, ACT_NONE: lambda t: t}[act](y)
    if mul is not None:
        y = y * (mul.double().unsqueeze(2) if nd == 3 else mul.double())
    if res is not None:
        y = y + res.double()
    if up is not None:
        y = F.interpolate(up.double(), scale_factor=up_f, mode="bilinear", align_corners=False) + y
    return (y * post).float()


def pk(conv, bn, act):
    """Pack a CPU-built layer after moving a copy to the GPU (kernels read device weights)."""
    conv = copy.deepcopy(conv).to(DEV)
    bn = copy.deepcopy(bn).to(DEV) if bn is not None else None
    return pack_conv(conv, bn, act)


def _mk(nd, cin, cout, k, s, p, transposed=False, bias=False, bn=True, seed=0):
    torch.manual_seed(seed)
    cls = {(2, False): torch.nn.Conv2d, (3, False): torch.nn.Conv3d, (2, True): torch.nn.ConvTranspose2d,
           (3, True): torch.nn.ConvTranspose3d}[(nd, transposed)]
    conv = cls(cin, cout, k, s, p, bias=bias)
    b = None
    if bn:
        b = (torch.nn.BatchNorm3d if nd == 3 else torch.nn.BatchNorm2d)(cout).eval()
        b.running_mean.uniform_(-0.2, 0.2)
        b.running_var.uniform_(0.5, 1.5)
        b.weight.data.uniform_(0.8, 1.2)
        b.bias.data.uniform_(-0.2, 0.2)
    return conv, b


CONV2D = [(1, 32, 5, 1, 1), (16, 16, 3, 1, 1), (16, 16, 3, 2, 1), (56, 16, 1, 1, 0), (16, 16, 1, 1, 1),
          (8, 1, 3, 1, 1), (3, 32, 3, 2, 1), (40, 72, 3, 1, 1), (16, 24, 3, 1, 1), (24, 40, 3, 2, 1)]


@pytest.mark.parametrize("cin,cout,k,s,p", CONV2D)
@pytest.mark.parametrize("act", [ACT_GELU, ACT_SILU])
def test_conv2d(cin, cout, k, s, p, act):
    conv, bn = _mk(2, cin, cout, k, s, p)
    x = torch.randn(2, cin, 23, 37)
    y = run_conv(Ctx(DEV), pk(conv, bn, act), [x.to(DEV)])
    assert rel(y, _ref_conv([x], conv, bn, act)) < 1e-5


CONV3D = [(32, 8, 3, 1, 1), (8, 8, 3, 1, 1), (8, 24, 3, 2, 1), (24, 24, 3, 1, 1), (80, 40, 1, 1, 0), (1, 8, 3, 1, 1),
          (40, 72, 3, 2, 1)]


@pytest.mark.parametrize("cin,cout,k,s,p", CONV3D)
def test_conv3d(cin, cout, k, s, p):
    conv, bn = _mk(3, cin, cout, k, s, p, seed=1)
    x = torch.randn(1, cin, 6, 9, 21)
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)])
    assert rel(y, _ref_conv([x], conv, bn, ACT_GELU)) < 1e-5


@pytest.mark.parametrize("nd,cin,cout,bn", [(2, 16, 16, True), (2, 16, 1, False), (3, 72, 40, True),
                                            (3, 24, 1, False), (3, 16, 12, True), (2, 32, 32, True)])
def test_conv_transposed(nd, cin, cout, bn):
    conv, b = _mk(nd, cin, cout, 4, 2, 1, transposed=True, bn=bn, seed=2)
    shape = (2, cin, 5, 11, 13) if nd == 3 else (2, cin, 11, 19)
    x = torch.randn(*shape)
    act = ACT_GELU if bn else ACT_NONE
    y = run_conv(Ctx(DEV), pk(conv, b, act), [x.to(DEV)])
    assert rel(y, _ref_conv([x], conv, b, act)) < 1e-5


TILE_HINTS = [0x11, 0x12, 0x14, 0x41, 0x42, 0x44, 0x211, 0x212, 0x241, 0x242]  # LDS-staged, then direct


@pytest.mark.parametrize("nd,cin,cout,k,s,tr", [(2, 16, 16, 3, 1, False), (2, 40, 72, 3, 2, False),
                                                (2, 1, 16, 3, 2, False), (3, 32, 8, 3, 1, False),
                                                (3, 16, 24, 3, 2, False), (3, 24, 12, 4, 2, True),
                                                (2, 16, 16, 4, 2, True), (2, 56, 16, 1, 1, False)])
def test_conv_every_tile_variant(nd, cin, cout, k, s, tr):
    """Every (NT, KS) tile the hint can force gives the same result as the automatic choice
    and the fp64 torch reference (tolerance 1e-5 relative)."""
    conv, bn = _mk(nd, cin, cout, k, s, 1 if k == 4 else k // 2, transposed=tr, seed=3)
    shape = (2, cin, 5, 9, 37) if nd == 3 else (2, cin, 21, 70)
    x = torch.randn(*shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    p = pk(conv, bn, ACT_GELU)
    xs = [x.to(DEV)]
    auto = run_conv(Ctx(DEV), p, xs)
    assert rel(auto, ref) < 1e-5
    for h in TILE_HINTS:
        y = run_conv(Ctx(DEV), p, xs, hint=h)
        assert rel(y, ref) < 1e-5, hex(h)
    if nd == 2 and cout <= 2:
        assert rel(run_conv(Ctx(DEV), p, xs, hint=0x114), ref) < 1e-5


HINT_TILE3 = 1 << 23
TILE3_CASES = [  # (cin, cout, k, s, shape, B): the L / M volumes' layer types, then ragged extents
    (32, 8, 3, 1, (12, 24, 78), 1),    # group_stem (plane pairs)
    (8, 8, 3, 1, (9, 13, 37), 2),      # agg, odd depth
    (1, 8, 3, 1, (7, 10, 21), 1),      # corr_stem (one channel)
    (24, 24, 3, 1, (6, 12, 39), 1),    # conv1.1 / agg_1.1
    (40, 40, 3, 1, (5, 7, 19), 2),     # conv2.1 / agg_0.1
    (72, 72, 3, 1, (3, 6, 20), 1),     # conv3.1: two cout groups
    (8, 24, 3, 2, (12, 24, 78), 1),    # conv1.0
    (24, 40, 3, 2, (7, 11, 33), 1),    # conv2.0, odd extents
    (40, 72, 3, 2, (6, 12, 39), 2),    # conv3.0
    (48, 24, 1, 1, (6, 12, 39), 1),    # agg_1.0 (one source)
    (12, 16, 3, 1, (4, 5, 17), 1),
]


@pytest.mark.parametrize("cin,cout,k,s,shape,B", TILE3_CASES)
def test_conv_tile3_form(cin, cout, k, s, shape, B):
    """LDS-tiled implicit-GEMM 3-D form (conv_tile3.hip), every rows-per-wave variant (hint bits 26-27)
    vs fp64 torch (relative 1e-5), and its general epilogue (residual, * mul broadcast over D, out2)."""
    conv, bn = _mk(3, cin, cout, k, s, k // 2, seed=cin + cout)
    x = torch.randn(B, cin, *shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    p = pk(conv, bn, ACT_GELU)
    outs = {}
    # automatic, rows 1 / 2 / 4, rows 8 (bit 28); plane pairs (<= 8 couts): bit 29 stages the weights in LDS
    # (round 5) instead of registers (round 6) -- the same products in the same order, bitwise equal
    for hint in (0, 1 << 26, 2 << 26, 3 << 26, 3 << 26 | 1 << 28, 1 << 29, 2 << 26 | 1 << 29):
        y = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | hint)
        assert rel(y, ref) < 1e-5, hex(hint)
        outs[hint] = y
    if cout <= 8 and k == 3 and s == 1:
        assert torch.equal(outs[1 << 29], outs[0]) and torch.equal(outs[2 << 26 | 1 << 29], outs[2 << 26])
        # round 6: buffer-to-LDS staging (default) bitwise the register staging (bit 28)
        for rows in (1 << 26, 2 << 26):
            assert torch.equal(run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | rows | 1 << 28), outs[rows]), hex(rows)
    if cout in (24, 40) and k == 3 and s == 1:
        # round 6: the plane-pair hybrid for 16 MF + 8 couts (default) is bitwise the padded MT form (bit 29)
        for rows in (1 << 26, 2 << 26):
            hz = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | rows)
            mt = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | rows | 1 << 29)
            assert torch.equal(hz, mt), hex(rows)
    if k == 3 and s == 2 and cout <= 32:
        # round 6: the stride-2 MT form with register weights (default) is bitwise its LDS-weight form (bit 29)
        # and its buffer-to-LDS staging (default) bitwise the register staging (bit 28)
        for rows in (0, 1 << 26, 2 << 26, 3 << 26):
            lw = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | rows | 1 << 29)
            assert torch.equal(lw, outs[rows]), hex(rows)
            if rows != 3 << 26:
                rg = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | rows | 1 << 28)
                assert torch.equal(rg, outs[rows]), hex(rows)
    res = torch.randn(ref.shape)
    mul = torch.rand(B, cout, ref.shape[3], ref.shape[4]) + 0.5
    want = _ref_conv([x], conv, bn, ACT_GELU, mul=mul, res=res)
    out2 = torch.empty(ref.shape, device=DEV)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], res=res.to(DEV), mul=mul.to(DEV), out2=out2, post_scale2=2.0,
                 hint=HINT_TILE3)
    assert rel(y, want) < 1e-5
    assert rel(out2, want * 2.0) < 1e-5


@pytest.mark.parametrize("B,G,D,H,W", [(1, 32, 12, 24, 78), (2, 32, 9, 13, 37), (1, 8, 5, 7, 20), (1, 4, 3, 5, 9),
                                       (1, 32, 48, 96, 312), (2, 32, 10, 17, 70)])
def test_gwc_stem_fused(B, G, D, H, W):
    """The gwc volume + group_stem in one launch (gwc_stem.hip; ESMStereo-L / -M): bit-identical to the
    two launches (gwc_volume, then the tiled stem: same staged window, same MFMA order and epilogue), for
    every rows-per-wave variant, 1 / 2 / many k-steps and ragged extents; and vs fp64 torch (1e-5)."""
    from esmstereo_amd.engine import run_gwc_stem
    C = 2 * G
    conv, bn = _mk(3, G, 8, 3, 1, 1, seed=G + D)
    L, R = feature_pair(B, C, H, W, 7, max(D, 2))
    Ld, Rd = L.to(DEV), R.to(DEV)
    p = pk(conv, bn, ACT_GELU)
    V = E.build_gwc_volume(Ld, Rd, D, G)
    two = run_conv(Ctx(DEV), p, [V], hint=HINT_TILE3)
    for hint in (0, 2 << 26, 3 << 26, 1 << 28, (2 << 26) | (1 << 28)):  # bit 28: LDS-staged weights (round 5)
        y = run_gwc_stem(Ctx(DEV), p, Ld, Rd, G, D, hint=hint)
        assert torch.equal(y, two), (hex(hint), float((y - two).abs().max()))
    if B * D * H * W <= 1 << 16:
        assert rel(two, _ref_conv([O.gwc_volume(L, R, D, G)], conv, bn, ACT_GELU)) < 1e-5
    with pytest.raises(E.EsmError):  # C != 2 G
        run_gwc_stem(Ctx(DEV), p, Ld[:, :C - 4].contiguous(), Rd[:, :C - 4].contiguous(), G, D)


@pytest.mark.parametrize("cin,cout,shape,B", [(40, 24, (6, 12, 39), 1), (72, 40, (3, 6, 20), 2), (24, 16, (5, 7, 17), 1),
                                              (40, 72, (3, 5, 9), 1), (16, 2, (4, 4, 20), 1)])
def test_conv_tile3_transposed(cin, cout, shape, B):
    """The tile3 ConvTranspose3d k4 s2 p1 form (the hourglass's conv3_up / conv2_up; both qw classes per
    wave, 8-byte stores) vs fp64 torch, every rows-per-wave variant, plain and general epilogues."""
    conv, bn = _mk(3, cin, cout, 4, 2, 1, transposed=True, seed=cin * 3 + cout)
    x = torch.randn(B, cin, *shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    p = pk(conv, bn, ACT_GELU)
    for rsel in (0, 1, 3):
        y = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | (rsel << 26))
        assert rel(y, ref) < 1e-5, rsel
    res = torch.randn(ref.shape)
    want = _ref_conv([x], conv, bn, ACT_GELU, res=res)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], res=res.to(DEV), hint=HINT_TILE3)
    assert rel(y, want) < 1e-5


TILE2_CASES = [  # (cins, cout, k, s, p, H, W, B): the L / M upsamplers' 2-D layers, then ragged / odd ones
    ((32, 32), 32, 3, 1, 1, 48, 156, 1),       # spx_4x.0: cat(d, feature)
    ((32, 32, 32), 32, 1, 1, 0, 24, 78, 2),    # ref agg_1.0: 1x1 over three sources
    ((32,), 32, 3, 2, 1, 48, 156, 1),          # conv2.0 (stride 2)
    ((32,), 32, 1, 1, 1, 20, 62, 1),           # dm.3 (1x1, padding 1: the map grows)
    ((16,), 8, 3, 1, 1, 33, 70, 1),            # spx_4x.1 at S
    ((16,), 16, 3, 1, 1, 37, 45, 2),
    ((1,), 32, 3, 2, 1, 29, 41, 1),            # one input channel (forced)
    ((24, 16), 40, 3, 1, 1, 9, 23, 1),
]


@pytest.mark.parametrize("cins,cout,k,s,p,H,W,B", TILE2_CASES)
def test_conv_tile2_form(cins, cout, k, s, p, H, W, B):
    """The LDS-tiled form for 2-D convs (conv_tile3.hip with one plane): every rows-per-wave variant vs fp64
    torch (relative 1e-5), with a cropped first source, and the general epilogue (residual, out2)."""
    conv, bn = _mk(2, sum(cins), cout, k, s, p, seed=sum(cins) + H)
    big = torch.randn(B, cins[0], H + 2, W + 3)
    xs = [big[:, :, :H, :W]] + [torch.randn(B, c, H, W) for c in cins[1:]]
    ref = _ref_conv(xs, conv, bn, ACT_GELU)
    bigd = big.to(DEV)
    xd = [bigd[:, :, :H, :W]] + [x.to(DEV) for x in xs[1:]]
    pc = pk(conv, bn, ACT_GELU)
    for rsel in (0, 1, 2, 3):
        y = run_conv(Ctx(DEV), pc, xd, hint=HINT_TILE3 | (rsel << 26))
        assert rel(y, ref) < 1e-5, rsel
    res = torch.randn(ref.shape)
    want = _ref_conv(xs, conv, bn, ACT_GELU, res=res)
    out2 = torch.empty(ref.shape, device=DEV)
    y = run_conv(Ctx(DEV), pc, xd, res=res.to(DEV), out2=out2, post_scale2=0.5, hint=HINT_TILE3)
    assert rel(y, want) < 1e-5
    assert rel(out2, want * 0.5) < 1e-5


@pytest.mark.parametrize("cin,cout,H,W,B", [(32, 32, 24, 78, 1), (16, 16, 13, 40, 2), (32, 16, 7, 21, 1)])
def test_conv_tile2_transposed(cin, cout, H, W, B):
    """The tile form of ConvTranspose2d k4 s2 p1 (the refinements' conv3_up / conv2_up) vs fp64 torch."""
    conv, bn = _mk(2, cin, cout, 4, 2, 1, transposed=True, seed=cin + H)
    x = torch.randn(B, cin, H, W)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    p = pk(conv, bn, ACT_GELU)
    for rsel in (0, 1, 3):
        y = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_TILE3 | (rsel << 26))
        assert rel(y, ref) < 1e-5, rsel


@pytest.mark.parametrize("cins,cout,shape", [((24, 24), 24, (6, 12, 39)), ((16, 16, 8), 16, (3, 7, 21)),
                                             ((40, 40), 40, (5, 6, 20))])
def test_conv_tile3_multisource_crop(cins, cout, shape):
    """The tile3 1x1x1 form over a channel concat with a cropped source (the hourglass's agg_1.0 /
    agg_0.0: cat(conv_up(x)[..., :D, :H, :W], skip)), vs fp64 torch."""
    conv, bn = _mk(3, sum(cins), cout, 1, 1, 0, seed=sum(cins))
    big = torch.randn(2, cins[0], shape[0] + 1, shape[1] + 2, shape[2] + 3)
    xs = [big[:, :, :shape[0], :shape[1], :shape[2]]] + [torch.randn(2, c, *shape) for c in cins[1:]]
    ref = _ref_conv(xs, conv, bn, ACT_GELU)
    bigd = big.to(DEV)
    xd = [bigd[:, :, :shape[0], :shape[1], :shape[2]]] + [x.to(DEV) for x in xs[1:]]
    for rsel in (0, 1, 2, 3):
        y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), xd, hint=HINT_TILE3 | (rsel << 26))
        assert rel(y, ref) < 1e-5, rsel


HINT_PW = HINT_TILE3 | 1 << 29  # on a 1x1: the pointwise streaming form (conv_pw.hip, round 6)
PW_CASES = [  # (nd, cins, cout, shape, B, act, bn)
    (2, (32, 32, 32), 32, (1, 48, 156), 2, ACT_GELU, True),   # up_refinement agg_1.0 (ref4x at L)
    (2, (32, 32, 48), 32, (1, 23, 36), 1, ACT_GELU, True),    # agg_0.0, ragged last pixel group
    (2, (32, 128), 32, (1, 12, 40), 2, ACT_GELU, True),       # 160 input channels
    (3, (24, 24), 24, (6, 12, 40), 2, ACT_GELU, True),        # hourglass agg_1.0 (two cout tiles, padded)
    (3, (40, 40), 40, (4, 6, 20), 1, ACT_GELU, True),         # agg_0.0 (three cout tiles)
    (3, (8,), 48, (3, 5, 12), 2, ACT_NONE, False),            # one source, bias, no BN, no activation
    (2, (16,), 8, (1, 10, 30), 1, ACT_SILU, True),            # one cout tile, 8 couts
    (3, (12, 12, 12), 16, (2, 9, 14), 1, ACT_GELU, True),     # three sources
]


@pytest.mark.parametrize("nd,cins,cout,shape,B,act,bn", PW_CASES)
def test_conv_pointwise_form(nd, cins, cout, shape, B, act, bn):
    """The pointwise streaming form for 1x1 BasicConvs over a channel concat (conv_pw.hip) vs fp64 torch
    (relative 1e-5); the LDS-tiled k1 form (TILE3 alone) for comparison."""
    conv, b = _mk(nd, sum(cins), cout, 1, 1, 0, bias=not bn, bn=bn, seed=sum(cins) + cout)
    sh = shape if nd == 3 else shape[1:]
    xs = [torch.randn(B, c, *sh) for c in cins]
    ref = _ref_conv(xs, conv, b, act)
    p = pk(conv, b, act)
    xd = [x.to(DEV) for x in xs]
    y = run_conv(Ctx(DEV), p, xd, hint=HINT_PW)
    assert rel(y, ref) < 1e-5
    assert rel(run_conv(Ctx(DEV), p, xd, hint=HINT_TILE3), ref) < 1e-5
    assert torch.equal(run_conv(Ctx(DEV), p, xd, hint=HINT_PW), y)  # deterministic


def test_conv_pointwise_form_fallback():
    """Layouts the pointwise form cannot stream (a cropped source view, P % 4 != 0) take the other forms
    when the hint asks for it, with the same results."""
    conv, bn = _mk(3, 48, 24, 1, 1, 0, seed=5)
    big = torch.randn(1, 24, 5, 8, 13)
    xs = [big[:, :, :4, :6, :10], torch.randn(1, 24, 4, 6, 10)]
    ref = _ref_conv(xs, conv, bn, ACT_GELU)
    bigd = big.to(DEV)
    xd = [bigd[:, :, :4, :6, :10], xs[1].to(DEV)]
    assert rel(run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), xd, hint=HINT_PW), ref) < 1e-5
    conv2, bn2 = _mk(2, 16, 16, 1, 1, 0, seed=6)
    x = torch.randn(1, 16, 7, 9)
    assert rel(run_conv(Ctx(DEV), pk(conv2, bn2, ACT_GELU), [x.to(DEV)], hint=HINT_PW),
               _ref_conv([x], conv2, bn2, ACT_GELU)) < 1e-5


HINT_SMALL = 1 << 21
SMALL_CASES = [(3, [16], 16, 3, 1, False, (3, 6, 20)), (3, [24], 24, 3, 1, False, (2, 3, 10)),
               (3, [16], 24, 3, 2, False, (3, 6, 20)), (3, [12], 16, 3, 2, False, (6, 12, 39)),
               (3, [8], 12, 3, 2, False, (12, 24, 78)), (3, [16, 16], 16, 1, 1, False, (3, 6, 20)),
               (3, [12, 12], 12, 1, 1, False, (5, 7, 19)), (3, [24], 16, 4, 2, True, (2, 3, 10)),
               (3, [16], 12, 4, 2, True, (3, 6, 20)), (3, [10], 40, 3, 1, False, (3, 5, 17)),
               (2, [16], 16, 3, 1, False, (22, 76)), (2, [16], 16, 3, 2, False, (48, 156)),
               (2, [1], 16, 5, 1, False, (24, 78)), (2, [16], 16, 1, 1, False, (22, 76)),
               (2, [16, 16, 32], 16, 1, 1, False, (24, 78)), (2, [16, 32], 16, 3, 1, False, (24, 78)),
               (2, [16], 16, 4, 2, True, (12, 39)), (2, [16], 8, 3, 1, False, (24, 78)),
               (2, [6], 33, 3, 1, False, (9, 21)), (2, [16], 1, 4, 2, True, (48, 156))]


@pytest.mark.parametrize("nd,cins,cout,k,s,tr,shape", SMALL_CASES)
def test_conv_small_form(nd, cins, cout, k, s, tr, shape):
    """Lean K-split form (conv_small.hip, hint 1 << 21) vs fp64 torch (1e-5 relative): 2-D / 3-D,
    k1 / k3 / k5 (k1 with padding 1 as dmNx.3), stride 2, transposed (every parity class), multi-
    source channel concat, ragged widths, cout tiles (33, 40), batch 2."""
    p_ = 1 if k == 4 else (1 if k == 1 and len(cins) == 1 and nd == 2 else k // 2)
    if k == 5:
        p_ = 1
    conv, bn = _mk(nd, sum(cins), cout, k, s, p_, transposed=tr, seed=7, bn=cout > 1)
    act = ACT_GELU if cout > 1 else ACT_NONE
    xs = [torch.randn(2, c, *shape) for c in cins]
    ref = _ref_conv(xs, conv, bn, act)
    p = pk(conv, bn, act)
    y = run_conv(Ctx(DEV), p, [x.to(DEV) for x in xs], hint=HINT_SMALL)
    assert rel(y, ref) < 1e-5
    if sum(cins) > 16:  # the 8-wave K split (hint bit 29) where it applies
        y = run_conv(Ctx(DEV), p, [x.to(DEV) for x in xs], hint=HINT_SMALL | (1 << 29))
        assert rel(y, ref) < 1e-5


HINT_WIDE = 1 << 22
WIDE_CASES = [(16, 16, 3, 1, (192, 624)), (16, 16, 3, 1, (94, 310)), (40, 16, 3, 1, (96, 312)),
              (16, 8, 3, 1, (96, 312)), (16, 16, 1, 1, (94, 310)), (56, 16, 1, 0, (96, 312)),
              (16, 32, 3, 1, (47, 83)), (6, 24, 3, 1, (33, 50)), (128, 16, 1, 0, (9, 70)), (16, 16, 3, 1, (5, 17)),
              (1, 16, 5, 1, (96, 312)), (1, 16, 5, 1, (24, 78)), (6, 16, 5, 1, (13, 40))]


@pytest.mark.parametrize("cin,cout,k,p,shape", WIDE_CASES)
def test_conv_wide_form(cin, cout, k, p, shape):
    """Register-weight row-streaming form (conv_wide.hip, hint 1 << 22) vs fp64 torch (1e-5 relative):
    k1 (with padding 1, as dmNx.3) / k3, channel counts off the 4-group grid, two cout tiles, ragged
    extents (rows not a multiple of the 2 / 4-row wave block, strips past the right edge), batch 2."""
    conv, bn = _mk(2, cin, cout, k, 1, p, seed=9)
    x = torch.randn(2, cin, *shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], hint=HINT_WIDE)
    assert rel(y, ref) < 1e-5
    res = torch.randn_like(ref)
    out2 = torch.empty_like(ref, device=DEV)
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], res=res.to(DEV), post_scale=4.0, out2=out2,
                 post_scale2=2.0, hint=HINT_WIDE)
    ref2 = _ref_conv([x], conv, bn, ACT_GELU, res=res)
    assert rel(y, ref2 * 4) < 1e-5 and rel(out2, ref2 * 2) < 1e-5
    for rsel in (1, 2, 3):  # every rows-per-wave block (hint bits 26-27)
        y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], hint=HINT_WIDE | (rsel << 26))
        assert rel(y, ref) < 1e-5
    for rsel in (2, 3):  # the K split over two waves (hint bit 28), both epilogues
        y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], hint=HINT_WIDE | (rsel << 26) | (1 << 28))
        assert rel(y, ref) < 1e-5
        y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], res=res.to(DEV), post_scale=4.0, out2=out2,
                     post_scale2=2.0, hint=HINT_WIDE | (rsel << 26) | (1 << 28))
        assert rel(y, ref2 * 4) < 1e-5 and rel(out2, ref2 * 2) < 1e-5


@pytest.mark.parametrize("cins,cout,k,p,shape", [((16, 24), 16, 3, 1, (96, 312)), ((16, 16, 24), 16, 1, 0, (96, 312)),
                                                  ((16, 16, 32), 16, 1, 0, (47, 157)), ((8, 8), 24, 3, 1, (19, 40))])
def test_conv_wide_form_multisource(cins, cout, k, p, shape):
    """Wide form over a channel concat (spx_Nx.0, agg_N.0), one descriptor per source: the sources carved
    out of one allocation (as a launch list's arena carves them), then allocated apart with 3 GiB
    between them, in both address orders; vs fp64 torch (1e-5 relative), and the two placements bitwise
    equal."""
    conv, bn = _mk(2, sum(cins), cout, k, 1, p, seed=10)
    n = [2 * c * shape[0] * shape[1] for c in cins]
    pool = torch.randn(sum(n) + 1000, device=DEV)
    xs, off = [], 500
    for c, m in zip(cins, n):
        xs.append(pool[off:off + m].view(2, c, *shape))
        off += m
    ref = _ref_conv([x.cpu() for x in xs], conv, bn, ACT_GELU)
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), xs, hint=HINT_WIDE)
    assert rel(y, ref) < 1e-5
    far, spacers = [], []
    for x in reversed(xs):
        far.append(x.clone())
        spacers.append(torch.empty(3 << 28, device=DEV))
    far.reverse()
    y2 = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), far, hint=HINT_WIDE)
    assert torch.equal(y2, y)


HINT_WIDE3 = 1 << 24


@pytest.mark.parametrize("cin,cout,shape,B", [(32, 8, (12, 24, 78), 1), (8, 8, (12, 24, 78), 1), (1, 8, (12, 24, 78), 2),
                                              (32, 8, (7, 9, 37), 2), (16, 16, (5, 6, 20), 1), (24, 12, (3, 5, 17), 1),
                                              (12, 12, (6, 12, 39), 1), (32, 8, (48, 20, 50), 1)])
def test_conv_wide3_form(cin, cout, shape, B):
    """3x3x3 plane-streaming form (conv_wide3.hip, hint 1 << 24) vs fp64 torch (1e-5 relative): every K split
    (1, 2, 4 waves over the channel groups), plane blocks not dividing D, ragged widths, batch 2; plus the
    `* att` (corr_stem of ESMStereo-S nc) and residual epilogues."""
    conv, bn = _mk(3, cin, cout, 3, 1, 1, seed=11)
    x = torch.randn(B, cin, *shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    p = pk(conv, bn, ACT_GELU)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_WIDE3)
    assert rel(y, ref) < 1e-5
    att = torch.rand(B, cout, shape[1], shape[2]) + 0.5
    res = torch.randn_like(ref)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], mul=att.to(DEV), res=res.to(DEV), hint=HINT_WIDE3)
    assert rel(y, _ref_conv([x], conv, bn, ACT_GELU, mul=att, res=res)) < 1e-5


HINT_WIDET = 1 << 25


@pytest.mark.parametrize("cin,cout,shape,B", [(16, 16, (96, 312), 1), (16, 16, (12, 39), 2), (16, 16, (48, 156), 1),
                                              (8, 16, (23, 45), 2), (4, 24, (17, 70), 1), (16, 1, (19, 33), 1)])
def test_conv_widet_form(cin, cout, shape, B):
    """ConvTranspose2d k4 s2 p1 in the all-classes-per-wave form (conv_widet.hip, hint 1 << 25) vs fp64 torch
    (1e-5 relative): ragged strips and rows, two cout tiles, batch 2, the 1-cout refinement head with the residual
    epilogue path."""
    conv, bn = _mk(2, cin, cout, 4, 2, 1, transposed=True, seed=12, bn=cout > 1)
    act = ACT_GELU if cout > 1 else ACT_NONE
    x = torch.randn(B, cin, *shape)
    ref = _ref_conv([x], conv, bn, act)
    p = pk(conv, bn, act)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_WIDET)
    assert rel(y, ref) < 1e-5
    for rsel in (1, 2):  # both sub-grid rows-per-wave blocks (hint bits 26-27)
        assert rel(run_conv(Ctx(DEV), p, [x.to(DEV)], hint=HINT_WIDET | (rsel << 26)), ref) < 1e-5
    res = torch.randn_like(ref)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], res=res.to(DEV), post_scale=4.0, hint=HINT_WIDET)
    assert rel(y, _ref_conv([x], conv, bn, act, res=res, post=4.0)) < 1e-5


def test_conv_small_form_epilogues():
    """Residual, post_scale and the second scaled copy in the small form; `* mul` / bilinear add /
    PixelShuffle are refused (the launcher falls back to the general forms for them)."""
    conv, bn = _mk(3, 16, 16, 3, 1, 1, seed=8)
    x, res = torch.randn(1, 16, 3, 6, 20), torch.randn(1, 16, 3, 6, 20)
    ref = _ref_conv([x], conv, bn, ACT_GELU, res=res, post=2.0)
    out2 = torch.empty(1, 16, 3, 6, 20, device=DEV)
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], res=res.to(DEV), post_scale=2.0, out2=out2,
                 post_scale2=0.5, hint=HINT_SMALL)
    assert rel(y, ref) < 1e-5
    assert rel(out2, ref / 4) < 1e-5
    att = torch.randn(1, 16, 6, 20)
    with pytest.raises(RuntimeError):
        run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], mul=att.to(DEV), hint=HINT_SMALL)


HINT_STEM, HINT_NO_STEM = 1 << 17, 1 << 18
STEM_CASES = [(3, 32, 8, (6, 9, 21)), (3, 1, 8, (5, 7, 30)), (3, 8, 8, (7, 5, 29)), (3, 12, 12, (4, 6, 15)),
              (3, 32, 8, (2, 3, 10)), (3, 3, 8, (9, 4, 44)), (2, 16, 8, (23, 37)), (2, 8, 12, (17, 50)),
              (2, 64, 8, (33, 15)), (3, 24, 24, (5, 9, 31)), (3, 16, 16, (3, 6, 20)), (2, 32, 32, (19, 47)),
              (2, 16, 16, (12, 39)), (3, 12, 24, (2, 3, 10)), (2, 40, 16, (9, 30)),
              (3, 24, 24, (13, 32, 100))]  # the last: 8-wave workgroups (62 KB weight slab), ragged in 8 planes


@pytest.mark.parametrize("nd,cin,cout,shape", STEM_CASES)
def test_conv_stem_form(nd, cin, cout, shape):
    """16-block MFMA narrow-output form (conv_stem.hip), forced and automatic, vs fp64 torch and
    vs the other forms (1e-5 relative)."""
    conv, bn = _mk(nd, cin, cout, 3, 1, 1, seed=4)
    x = torch.randn(2, cin, *shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    p = pk(conv, bn, ACT_GELU)
    xs = [x.to(DEV)]
    for h in (HINT_STEM, 0, HINT_NO_STEM):
        assert rel(run_conv(Ctx(DEV), p, xs, hint=h), ref) < 1e-5, hex(h)


def test_conv_stem_form_epilogues():
    """`corr_stem(volume) * att` (ESMStereo.py:703) and a residual through the stem form."""
    conv, bn = _mk(3, 1, 8, 3, 1, 1, seed=5)
    x = torch.randn(2, 1, 6, 10, 33)
    att = torch.randn(2, 8, 10, 33)
    res = torch.randn(2, 8, 6, 10, 33)
    p = pk(conv, bn, ACT_GELU)
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], mul=att.to(DEV), hint=HINT_STEM)
    assert rel(y, _ref_conv([x], conv, bn, ACT_GELU, mul=att)) < 1e-5
    y = run_conv(Ctx(DEV), p, [x.to(DEV)], res=res.to(DEV), post_scale=2.0, hint=HINT_STEM)
    assert rel(y, _ref_conv([x], conv, bn, ACT_GELU, res=res, post=2.0)) < 1e-5


ROWS_CASES = [(2, 16, 16, 3, 1, 37, 70), (2, 8, 16, 3, 1, 9, 29), (2, 1, 16, 5, 1, 24, 78), (2, 1, 16, 5, 2, 24, 78),
              (2, 16, 8, 1, 0, 11, 33), (2, 16, 32, 3, 1, 13, 45), (2, 16, 24, 3, 1, 6, 17), (2, 4, 1, 3, 1, 20, 50),
              (3, 16, 16, 3, 1, (5, 9, 37), None), (3, 8, 8, 3, 1, (6, 7, 19), None), (3, 16, 24, 1, 0, (3, 6, 20), None)]


@pytest.mark.parametrize("nd,cin,cout,k,p,H,W", ROWS_CASES)
def test_conv_rows_form(nd, cin, cout, k, p, H, W):
    """The row-streaming form (DPP-shifted B operands, LDS weights, pipelined rows) against the
    fp64 torch reference, forced (hint 0x411) and automatic; rel <= 1e-5."""
    conv, bn = _mk(nd, cin, cout, k, 1, p, seed=5)
    shape = (2, cin) + (H if nd == 3 else (H, W))
    x = torch.randn(*shape)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    pc = pk(conv, bn, ACT_GELU)
    for h in (0, 0x411):
        y = run_conv(Ctx(DEV), pc, [x.to(DEV)], hint=h)
        assert rel(y, ref) < 1e-5, hex(h)


def test_conv_rows_form_epilogues():
    conv, bn = _mk(2, 16, 16, 3, 1, 1, seed=6)
    x = torch.randn(1, 16, 30, 64)
    res = torch.randn(1, 16, 30, 64)
    mul = torch.randn(1, 16, 30, 64)
    ref = _ref_conv([x], conv, bn, ACT_GELU, mul=mul, res=res, post=4.0)
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [x.to(DEV)], mul=mul.to(DEV), res=res.to(DEV), post_scale=4.0,
                 hint=0x411)
    assert rel(y, ref) < 1e-5
    c1, _ = _mk(2, 16, 1, 3, 1, 1, bn=False, seed=9)  # the tail conv: 1 channel + bilinear residual
    up = torch.randn(1, 1, 15, 32)
    ref1 = _ref_conv([x], c1, None, ACT_NONE, up=up, up_f=2, post=4.0)
    y1 = run_conv(Ctx(DEV), pk(c1, None, ACT_NONE), [x.to(DEV)], up=up.to(DEV), up_f=2, post_scale=4.0, hint=0x411)
    assert rel(y1, ref1) < 1e-5
    c2, _ = _mk(2, 8, 64, 1, 1, 0, bias=True, bn=False, seed=7)
    x2 = torch.randn(1, 8, 12, 40)
    ref2 = _ref_conv([x2], c2, None, ACT_SILU, shuffle=4)
    y2 = run_conv(Ctx(DEV), pk(c2, None, ACT_SILU), [x2.to(DEV)], shuffle=4, hint=0x411)
    assert rel(y2, ref2) < 1e-5
    with pytest.raises(E.EsmError):  # stride 2 is not a row-streaming layer
        c3, b3 = _mk(2, 16, 16, 3, 2, 1, seed=8)
        run_conv(Ctx(DEV), pk(c3, b3, ACT_GELU), [x.to(DEV)], hint=0x411)


def test_conv_c1_hint():
    conv, _ = _mk(2, 8, 1, 3, 1, 1, bn=False, seed=4)
    x = torch.randn(1, 8, 30, 150)
    ref = _ref_conv([x], conv, None, ACT_NONE)
    p = pk(conv, None, ACT_NONE)
    for h in (0, 0x11, 0x114):
        assert rel(run_conv(Ctx(DEV), p, [x.to(DEV)], hint=h), ref) < 1e-5, hex(h)
    with pytest.raises(E.EsmError):
        run_conv(Ctx(DEV), p, [x.to(DEV)], hint=0x3)


@pytest.mark.parametrize("nd,cin", [(2, 16), (2, 32), (2, 8), (2, 24), (3, 12), (3, 24), (3, 32), (3, 8)])
def test_convt_c1_form(nd, cin):
    """Single-output-channel ConvTranspose k4 s2 p1 on the VALU form (conv_c1.h), automatic and
    forced (hint 1 << 16), ragged extents (not multiples of the 16 x 64 tile), vs fp64 torch;
    rel <= 1e-5."""
    conv, _ = _mk(nd, cin, 1, 4, 2, 1, transposed=True, bn=False, seed=11)
    shape = (2, cin, 5, 9, 37) if nd == 3 else (2, cin, 13, 45)
    x = torch.randn(*shape)
    ref = _ref_conv([x], conv, None, ACT_NONE)
    p = pk(conv, None, ACT_NONE)
    for h in (0, 1 << 16, 1 << 16 | 1 << 26):  # 3-D: register-blocked form, then the per-class form (bits 26-27 = 1)
        assert rel(run_conv(Ctx(DEV), p, [x.to(DEV)], hint=h), ref) < 1e-5, hex(h)
    if nd == 3:  # several blocked tiles per plane (64-column x 16-row input tiles), odd extents, B 3
        xb = torch.randn(3, cin, 3, 19, 70)
        assert rel(run_conv(Ctx(DEV), p, [xb.to(DEV)]), _ref_conv([xb], conv, None, ACT_NONE)) < 1e-5
    # a channel slice of a wider tensor (batch stride > C * plane): channels past Cin in a staged chunk
    # must read as zero, not as the wider tensor's next channels
    wide = torch.randn(shape[0], cin + 7, *shape[2:], device=DEV)
    wide[:, 3:3 + cin] = x.to(DEV)
    wide[:, 3 + cin:] = float("nan")
    assert rel(run_conv(Ctx(DEV), p, [wide[:, 3:3 + cin]]), ref) < 1e-5
    if nd == 2:  # the up_refinement epilogue: + bilinear(prev, x2), x4 store, unscaled copy
        prev = torch.randn(2, 1, 13, 45)
        cp = torch.empty(2, 1, 26, 90, device=DEV)
        y = run_conv(Ctx(DEV), p, [x.to(DEV)], up=prev.to(DEV), up_f=2, post_scale=4.0, out2=cp, post_scale2=1.0)
        r2 = _ref_conv([x], conv, None, ACT_NONE, up=prev, up_f=2)
        assert rel(y, r2 * 4) < 1e-5 and rel(cp, r2) < 1e-5
    with pytest.raises(E.EsmError):  # not a single-output-channel transposed layer
        c2, b2 = _mk(nd, cin, 4, 4, 2, 1, transposed=True, seed=12)
        run_conv(Ctx(DEV), pk(c2, b2, ACT_GELU), [x.to(DEV)], hint=1 << 16)


@pytest.mark.parametrize("nf,r,H,W", [(8, 4, 24, 78), (8, 4, 7, 21), (8, 2, 13, 29), (16, 2, 24, 78), (16, 2, 5, 9), (16, 2, 37, 61),
                                      (16, 4, 6, 17), (8, 4, 96, 312), (8, 2, 130, 301), (8, 4, 1, 1),
                                      (8, 4, 9, 17), (8, 4, 33, 50)])
def test_shuffle_tail(nf, r, H, W):
    """upsampling (1x1 + PixelShuffle + SiLU) fused with tail (3x3 -> 1) vs fp64 torch of the
    reference's two modules (models/ESMStereo.py:264-271,301-302); rel <= 1e-5.  Tiles: 8 x 32 (one
    output per thread), 16 x 32 at 96 x 312 (S-K's 4x head: two per thread, XCD-slab order), 16 x 64
    at 130 x 301 (four per thread, ragged)."""
    from esmstereo_amd.engine import pack_shuffle_tail, run_shuffle_tail
    torch.manual_seed(nf * 100 + r)
    up = torch.nn.Conv2d(nf, nf * r * r, 1, 1, 0)
    tail = torch.nn.Conv2d(nf, 1, 3, 1, 1)
    x = torch.randn(2, nf, H, W)
    ref = F.conv2d(F.silu(F.pixel_shuffle(F.conv2d(x.double(), up.weight.double(), up.bias.double()), r)),
                   tail.weight.double(), tail.bias.double(), 1, 1).float()
    p = pack_shuffle_tail(copy.deepcopy(up).to(DEV), copy.deepcopy(tail).to(DEV), r)
    for form in ((0, 1, 2, 3) if (nf, r) == (8, 4) else (0,)):  # (8, 4): the window and both row forms
        y = run_shuffle_tail(Ctx(DEV), x.to(DEV), p, form=form)
        assert y.shape == (2, 1, H * r, W * r)
        assert rel(y, ref) < 1e-5, form


@pytest.mark.parametrize("nf,r,C,H,W", [(8, 4, 16, 24, 78), (8, 4, 16, 96, 312), (8, 4, 16, 7, 13), (8, 2, 16, 13, 29),
                                         (16, 2, 32, 17, 40), (16, 4, 32, 9, 21), (8, 2, 16, 48, 156),
                                         (8, 4, 16, 21, 37)])
def test_shuffle_conv_fused(nf, r, C, H, W):
    """tail(upsampling(x)) + the refinement's first BasicConv(1, C, 3, 2, 1) in one launch
    (esm_shuffle_conv_f32, models/ESMStereo.py:301-303 + :190-191) vs fp64 torch of the three reference
    modules and vs the two-launch path (shuffle_tail, then the conv); relative 1e-5, batch 2, ragged."""
    from esmstereo_amd.engine import pack_shuffle_tail, run_shuffle_conv, run_shuffle_tail
    torch.manual_seed(nf * 1000 + r * 10 + H)
    up = torch.nn.Conv2d(nf, nf * r * r, 1, 1, 0)
    tail = torch.nn.Conv2d(nf, 1, 3, 1, 1)
    conv, bn = _mk(2, 1, C, 3, 2, 1, seed=H)
    x = torch.randn(2, nf, H, W)
    t = F.conv2d(F.silu(F.pixel_shuffle(F.conv2d(x.double(), up.weight.double(), up.bias.double()), r)),
                 tail.weight.double(), tail.bias.double(), 1, 1)
    ref = _ref_conv([t], conv, bn, ACT_GELU)
    p = pack_shuffle_tail(copy.deepcopy(up).to(DEV), copy.deepcopy(tail).to(DEV), r)
    pc = pk(conv, bn, ACT_GELU)
    ctx = Ctx(DEV)
    two = run_conv(ctx, pc, [run_shuffle_tail(ctx, x.to(DEV), p)])
    for form in ((0, 1, 2, 3) if (nf, r) == (8, 4) else (0,)):  # (8, 4): the window and both row forms
        y = run_shuffle_conv(ctx, x.to(DEV), p, pc, form=form)
        assert y.shape == ref.shape
        assert rel(y, ref) < 1e-5, form
        assert rel(y, two) < 1e-5, form


@pytest.mark.parametrize("cp,H,W", [(16, 96, 312), (16, 21, 37), (12, 9, 40), (16, 7, 13)])
def test_shuffle_conv_pre(cp, H, W):
    """The row-form head + ref conv launch with the stage's spx_<t>[1] (BasicConv(cp, 8, 3, 1, 1)) computed
    inside it from its input (esm_shuffle_conv_desc.pre_x) vs fp64 torch of the four reference layers and vs
    the separate launches (relative 1e-5), batch 2, ragged extents."""
    from esmstereo_amd.engine import pack_shuffle_tail, run_shuffle_conv
    torch.manual_seed(cp * 100 + H)
    up = torch.nn.Conv2d(8, 128, 1, 1, 0)
    tail = torch.nn.Conv2d(8, 1, 3, 1, 1)
    pconv, pbn = _mk(2, cp, 8, 3, 1, 1, seed=H + 1)
    conv, bn = _mk(2, 1, 16, 3, 2, 1, seed=H)
    c = torch.randn(2, cp, H, W)
    x = _ref_conv([c], pconv, pbn, ACT_GELU)
    t = F.conv2d(F.silu(F.pixel_shuffle(F.conv2d(x.double(), up.weight.double(), up.bias.double()), 4)),
                 tail.weight.double(), tail.bias.double(), 1, 1)
    ref = _ref_conv([t], conv, bn, ACT_GELU)
    p = pack_shuffle_tail(copy.deepcopy(up).to(DEV), copy.deepcopy(tail).to(DEV), 4)
    pc, pp = pk(conv, bn, ACT_GELU), pk(pconv, pbn, ACT_GELU)
    ctx = Ctx(DEV)
    two = run_shuffle_conv(ctx, run_conv(ctx, pp, [c.to(DEV)]), p, pc, form=2)
    for form in (2, 3):  # the row form with the refinement conv on the VALU / on the matrix cores
        y = run_shuffle_conv(ctx, c.to(DEV), p, pc, pre=pp, form=form)
        assert y.shape == ref.shape
        assert rel(y, ref) < 1e-5, form
        assert rel(y, two) < 1e-5, form
    # round 5: up_refinement.conv1[1] (BasicConv(16, 16, 3, 1, 1)) fused behind it: the whole conv1 in one launch
    conv2, bn2 = _mk(2, 16, 16, 3, 1, 1, seed=H + 2)
    ref2 = _ref_conv([ref.double()], conv2, bn2, ACT_GELU)
    pc2 = pk(conv2, bn2, ACT_GELU)
    from esmstereo_amd import engine as EN
    rows0 = EN.SC11_TILE
    try:
        for rows in (0, 1, 2):  # round 6: 4 low-res rows on 8 / 4 waves (two workgroups per CU); the round-5 8-row tile
            EN.SC11_TILE = rows
            y2 = run_shuffle_conv(ctx, c.to(DEV), p, pc, pre=pp, conv2=pc2)
            assert y2.shape == ref2.shape
            assert rel(y2, ref2) < 1e-5, rows
            assert rel(y2, run_conv(ctx, pc2, [y])) < 1e-5, rows
    finally:
        EN.SC11_TILE = rows0
    # the fused second conv needs the pre-conv: a descriptor with w2 and no pre_x is an argument error
    with pytest.raises((ValueError, RuntimeError)):
        run_shuffle_conv(ctx, x.to(DEV), p, pc, conv2=pc2)


PAIR2_CASES = [  # (cins, kA, sA, pA, kB, pB, coutB, H, W): the shapes the hot paths use, then ragged ones
    ((1,), 5, 1, 1, 3, 1, 16, 24, 78),           # dm<t>.0 -> dm<t>.1
    ((16,), 3, 1, 1, 1, 1, 16, 22, 76),          # dm<t>.2 -> dm<t>.3 (k1 p1: the GELU(shift) ring)
    ((16, 32), 3, 1, 1, 3, 1, 16, 24, 78),       # spx_2x.0 -> spx_2x.1 (cat of d and a feature map)
    ((16, 24), 3, 1, 1, 3, 1, 8, 96, 312),       # spx_4x.0 -> spx_4x.1 (16 -> 8)
    ((16,), 3, 2, 1, 3, 1, 16, 48, 156),         # conv2.0 (s2) -> conv2.1
    ((16,), 3, 2, 1, 3, 1, 16, 25, 79),          # odd extents
    ((16, 16, 32), 1, 1, 0, 3, 1, 16, 24, 78),   # agg_0.0 (1x1 over three sources) -> agg_0.1
    ((1,), 5, 1, 1, 3, 1, 16, 7, 9),
    ((12,), 3, 1, 1, 3, 1, 12, 5, 40),
]


@pytest.mark.parametrize("cins,ka,sa,pa,kb,pb,coutb,H,W", PAIR2_CASES)
def test_conv_pair2(cins, ka, sa, pa, kb, pb, coutb, H, W):
    """Two BasicConvs in one launch (conv_pair2.hip: the intermediate in LDS, halo recomputed) vs fp64 torch of
    the two layers and vs the two separate launches (relative 1e-5), batch 2."""
    from esmstereo_amd.engine import pair2_supported, run_pair2
    ca, ba = _mk(2, sum(cins), 16, ka, sa, pa, seed=31 + H)
    cb, bb = _mk(2, 16, coutb, kb, 1, pb, seed=32 + W)
    xs = [torch.randn(2, c, H, W) for c in cins]
    ref = _ref_conv([_ref_conv(xs, ca, ba, ACT_GELU)], cb, bb, ACT_GELU)
    pa_, pb_ = pk(ca, ba, ACT_GELU), pk(cb, bb, ACT_GELU)
    xd = [x.to(DEV) for x in xs]
    assert pair2_supported(pa_, pb_, xd)
    ctx = Ctx(DEV)
    y = run_pair2(ctx, pa_, xd, pb_, force=True)
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-5
    two = run_conv(ctx, pb_, [run_conv(ctx, pa_, xd)])
    assert rel(y, two) < 1e-5


@pytest.mark.parametrize("B,D,H,W", [(1, 12, 24, 78), (1, 24, 48, 156), (1, 12, 96, 312), (2, 5, 7, 9), (2, 12, 25, 79)])
def test_conv_pair2_regress(B, D, H, W):
    """disparity_regression folded into the dm<t>.0 -> dm<t>.1 pair (conv_pair2.hip hint bit 29): the map it
    stores is bitwise the separate regression launch's, and the pair's output bitwise the pair run on that
    map (S-K 24x78 D12, M-K 48x156 D24, the 4-row-tile form at 96x312, ragged extents, batch 2)."""
    from esmstereo_amd.engine import run_pair2
    ca, ba = _mk(2, 1, 16, 5, 1, 1, seed=41 + W)
    cb, bb = _mk(2, 16, 16, 3, 1, 1, seed=42 + H)
    pa_, pb_ = pk(ca, ba, ACT_GELU), pk(cb, bb, ACT_GELU)
    cost = torch.randn(B, D, H, W)
    costd = cost.to(DEV)
    ctx = Ctx(DEV)
    init = torch.full((B, 1, H, W), float("nan"), device=DEV)
    n0 = len(ctx.meta)
    y = run_pair2(ctx, pa_, [init], pb_, force=True, regress=costd)
    assert [m["name"] for m in ctx.meta[n0:]] == ["disparity_regression+convA+convB"]
    ref_init = torch.empty(B, 1, H, W, device=DEV)
    ctx.regression(0, costd, ref_init, B, D, H, W)
    assert torch.equal(init, ref_init)
    two = run_pair2(ctx, pa_, [ref_init], pb_, force=True)
    assert torch.equal(y, two)
    ref = (cost * torch.arange(D, dtype=torch.float32).view(1, D, 1, 1)).sum(1, keepdim=True)
    assert rel(init, ref) < 1e-6


UP1_CASES = [  # (nd, cin, cy, extra channels, coutb, input grid, crop, B, hint of the transposed conv)
    (3, 24, 16, (16,), 16, (2, 3, 10), (3, 6, 20), 1, 0),              # S aggregation conv3_up -> agg_0.0
    (3, 16, 12, (12,), 12, (3, 6, 20), (6, 12, 39), 1, 0),             # S aggregation conv2_up -> agg_1.0
    (2, 16, 16, (16, 24), 16, (48, 156), (96, 312), 1, 0x4800000),     # S ref4x conv3_up -> agg_0.0, tiled rows 1
    (2, 16, 16, (16, 24), 16, (96, 312), (192, 624), 1, 0x4800000),    # S ref4x conv2_up -> agg_1.0, tiled rows 1
    (2, 16, 16, (16, 24), 16, (96, 312), (192, 624), 1, 0x8800000),    # ... tiled rows 2
    (2, 16, 16, (16, 24), 16, (96, 312), (192, 624), 1, 0),            # ... automatic (lean)
    (2, 16, 16, (16, 32), 16, (12, 39), (24, 78), 1, 0),               # S ref2x conv3_up -> agg_0.0
    (2, 16, 16, (16, 32), 16, (24, 78), (48, 156), 1, 0),              # S ref2x conv2_up -> agg_1.0
    (3, 24, 8, (4,), 12, (3, 7, 9), (5, 13, 17), 2, 0x20200000),       # ragged crops, 8-wave lean, batch 2
    (3, 20, 16, (8, 4), 8, (3, 5, 10), (6, 9, 20), 2, 0x4800000),      # 3-D tiled rows 1, three sources
    (2, 12, 12, (16, 32), 16, (11, 19), (21, 37), 2, 0x8800000),       # 2-D tiled, odd crop, batch 2
    (2, 12, 4, (48,), 5, (11, 19), (22, 37), 2, 0),                    # 4 couts, 48 extra channels
    # round 6: two cout tiles (3-D tiled form): L aggregation conv2_up 40 -> 24 + agg_1.0 (48 -> 24)
    (3, 40, 24, (24,), 24, (3, 6, 20), (6, 12, 40), 2, 0),
    (3, 40, 24, (24,), 24, (3, 6, 20), (6, 12, 40), 1, 0x4800000),     # rows 1
    (3, 32, 20, (8, 4), 28, (3, 5, 9), (5, 9, 17), 2, 0),              # ragged crop, 20 / 28 couts, three sources
    (3, 24, 32, (32,), 32, (2, 4, 11), (4, 8, 22), 1, 0),              # 32 couts, 32 extra channels
]


@pytest.mark.parametrize("nd,cin,cy,cxs,coutb,grid,crop,B,hint", UP1_CASES)
def test_convt_1x1(nd, cin, cy, cxs, coutb, grid, crop, B, hint):
    """ConvTranspose BasicConv + crop + cat + 1x1 BasicConv in one launch (conv_up1.hip) vs fp64 torch of the
    reference layers and vs the two separate launches (relative 1e-5), in the lean and LDS-tiled forms."""
    from esmstereo_amd.engine import convt_1x1_supported, run_convt_1x1
    ca, ba = _mk(nd, cin, cy, 4, 2, 1, transposed=True, seed=51 + cin)
    cb, bb = _mk(nd, cy + sum(cxs), coutb, 1, 1, 0, seed=52 + coutb)
    x = torch.randn(B, cin, *grid)
    xs = [torch.randn(B, c, *crop) for c in cxs]
    u = _ref_conv([x], ca, ba, ACT_GELU)
    u = u[(slice(None), slice(None)) + tuple(slice(0, n) for n in crop)]
    ref = _ref_conv([u, *xs], cb, bb, ACT_GELU)
    pa_, pb_ = pk(ca, ba, ACT_GELU), pk(cb, bb, ACT_GELU)
    xd, xsd = x.to(DEV), [t.to(DEV) for t in xs]
    assert convt_1x1_supported(pa_, pb_, xsd)
    ctx = Ctx(DEV)
    from esmstereo_amd import engine as EN
    old = dict(EN.HINT_SET)
    EN.HINT_SET["convT"] = hint
    try:
        y = run_convt_1x1(ctx, pa_, [xd], pb_, xsd)
    finally:
        EN.HINT_SET.clear()
        EN.HINT_SET.update(old)
    torch.cuda.synchronize()
    assert y.shape == ref.shape
    assert rel(y, ref) < 1e-5
    ud = run_conv(ctx, pa_, [xd])
    two = run_conv(ctx, pb_, [ud[(slice(None), slice(None)) + tuple(slice(0, n) for n in crop)], *xsd])
    assert rel(y, two) < 1e-5


PRE_CASES = [  # (main channels, side channels, cout, k, H, W, B, hint): the fork-join partial sums (round 6)
    (16, 24, 16, 3, 96, 312, 1, 0x18400000),   # spx_4x.0 (S): the register-weight form, K split
    (16, 32, 16, 3, 24, 78, 1, 0),             # spx_2x.0 (S): automatic (lean)
    (16, 32, 16, 3, 24, 78, 1, 0x20200000),    # lean, 8 waves
    (32, 48, 32, 3, 96, 312, 2, 0x8800000),    # spx_2x.0 (L): LDS-tiled, 2 rows
    (32, 48, 32, 1, 48, 156, 2, 0x800000),     # agg_N.0 (L): LDS-tiled 1x1
    (16, 24, 16, 1, 37, 70, 2, 0x400000),      # 1x1 register-weight form, ragged
]


@pytest.mark.parametrize("cm,cs,cout,k,H,W,B,hint", PRE_CASES)
def test_conv_partial_sum(cm, cs, cout, k, H, W, B, hint):
    """conv(cat(main, side)) as the side channels' plain partial sum + the main channels' conv started from it
    (esm_conv_desc.pre) vs fp64 torch of the whole layer (relative 1e-5), in the forms that take `pre`."""
    from esmstereo_amd.engine import pack_conv_split
    conv, bn = _mk(2, cm + cs, cout, k, 1, k // 2, seed=cm + cs + k)
    xm, xs = torch.randn(B, cm, H, W), torch.randn(B, cs, H, W)
    ref = _ref_conv([xm, xs], conv, bn, ACT_GELU)
    c_, b_ = copy.deepcopy(conv).to(DEV), copy.deepcopy(bn).to(DEV)
    p_side, p_main = pack_conv_split(c_, None, ACT_GELU, cm, cm + cs), pack_conv_split(c_, b_, ACT_GELU, 0, cm)
    ctx = Ctx(DEV)
    part = run_conv(ctx, p_side, [xs.to(DEV)], hint=hint)
    y = run_conv(ctx, p_main, [xm.to(DEV)], pre=part, hint=hint)
    assert rel(y, ref) < 1e-5
    with pytest.raises((ValueError, E.EsmError)):  # a 3-D conv takes no partial sum
        c3, b3 = _mk(3, 8, 8, 3, 1, 1, seed=5)
        p3 = pk(c3, b3, ACT_GELU)
        x3 = torch.randn(1, 8, 4, 6, 20, device=DEV)
        run_conv(Ctx(DEV), p3, [x3], pre=torch.zeros(1, 8, 4, 6, 20, device=DEV))


def test_convt_1x1_partial_sum():
    """The fused transposed conv + 1x1 with the 1x1's image-feature channels as a side partial sum (b.pre)."""
    from esmstereo_amd.engine import pack_conv_split, run_convt_1x1
    for hint in (0x4800000, 0):
        ca, ba = _mk(2, 16, 16, 4, 2, 1, transposed=True, seed=71)
        cb, bb = _mk(2, 16 + 16 + 24, 16, 1, 1, 0, seed=72)
        x = torch.randn(1, 16, 48, 156)
        skip, feat = torch.randn(1, 16, 96, 312), torch.randn(1, 24, 96, 312)
        u = _ref_conv([x], ca, ba, ACT_GELU)
        ref = _ref_conv([u, skip, feat], cb, bb, ACT_GELU)
        cb_, bb_ = copy.deepcopy(cb).to(DEV), copy.deepcopy(bb).to(DEV)
        p_side, p_main = pack_conv_split(cb_, None, ACT_GELU, 32, 56), pack_conv_split(cb_, bb_, ACT_GELU, 0, 32)
        from esmstereo_amd import engine as EN
        old = dict(EN.HINT_SET)
        EN.HINT_SET["convT"] = hint
        try:
            ctx = Ctx(DEV)
            part = run_conv(ctx, p_side, [feat.to(DEV)])
            y = run_convt_1x1(ctx, pk(ca, ba, ACT_GELU), [x.to(DEV)], p_main, [skip.to(DEV)], pre=part)
        finally:
            EN.HINT_SET.clear()
            EN.HINT_SET.update(old)
        assert rel(y, ref) < 1e-5, hex(hint)


def test_plan_side_branch_matches_eager():
    """A plan with side-branch ops (the fork-join partial sums) gives bitwise the same outputs eagerly, as a graph,
    and after a zero-copy rebind of its inputs (the side ops read the image features), as the eager modules."""
    from esmstereo_amd import blocks as BL
    name = next(k for k in HOT if k.startswith("hot_S_gwc"))
    model, sd, m = _model_from_manifest(name)
    fork0 = BL.FORK_ENABLED
    BL.FORK_ENABLED = True  # (off by default: measured slower as a graph branch, engine.FORK_ENABLED)
    try:
        _side_branch_case(model, name)
    finally:
        BL.FORK_ENABLED = fork0


def _side_branch_case(model, name):
    g = load_golden(name)
    up = [cu(g[f"up_{i}"]) for i in range(4) if f"up_{i}" in g]
    att = cu(g["att"]) if "att" in g else None
    ml, mr = cu(g["match_left"]), cu(g["match_right"])
    B, C, h, w = (int(v) for v in ml.shape)
    hp = E.HotPath(model, B, h, w, 0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], DEV,
                   channels=C, graph=False)
    assert any(x.get("branch") for x in hp.ctx.meta), "the S plan forks"
    hp.load_inputs(ml, mr, att, up)
    hp.launch()
    torch.cuda.synchronize()
    eager = [o.clone() for o in hp.outputs]
    hp.graph = True
    hp.launch()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(eager, hp.outputs))
    up2 = [u.clone() for u in up]  # new addresses: rebind moves every op pointer, side ops included
    hp.bind(ml, mr, att, up2)
    hp.launch()
    torch.cuda.synchronize()
    assert all(torch.equal(a, b) for a, b in zip(eager, hp.outputs))
    hp.close()


def test_convt_1x1_rejects():
    """Shapes outside the fused form raise the library's argument error (no silent fallback)."""
    from esmstereo_amd.engine import run_convt_1x1
    ca, ba = _mk(2, 16, 24, 4, 2, 1, transposed=True, seed=61)  # 24 outputs: more than one cout tile
    cb, bb = _mk(2, 40, 16, 1, 1, 0, seed=62)
    with pytest.raises(E.EsmError):
        run_convt_1x1(Ctx(DEV), pk(ca, ba, ACT_GELU), [torch.randn(1, 16, 8, 8, device=DEV)], pk(cb, bb, ACT_GELU),
                      [torch.randn(1, 16, 16, 16, device=DEV)])
    ca, ba = _mk(2, 16, 16, 4, 2, 1, transposed=True, seed=63)
    cb, bb = _mk(2, 16 + 64, 16, 1, 1, 0, seed=64)  # 64 extra channels: more than the kernels hold
    with pytest.raises(E.EsmError):
        run_convt_1x1(Ctx(DEV), pk(ca, ba, ACT_GELU), [torch.randn(1, 16, 8, 8, device=DEV)], pk(cb, bb, ACT_GELU),
                      [torch.randn(1, 64, 16, 16, device=DEV)])


def test_conv_multisource_crop_and_epilogues():
    # agg_0-style: crop of a larger tensor + two more sources, 1x1 then residual/mul/up epilogues
    conv, bn = _mk(2, 16 + 16 + 24, 16, 1, 1, 0, seed=3)
    big = torch.randn(1, 16, 26, 40)
    a = torch.randn(1, 16, 24, 39)
    c = torch.randn(1, 24, 24, 39)
    crop = big.to(DEV)[:, :, :24, :39]
    y = run_conv(Ctx(DEV), pk(conv, bn, ACT_GELU), [crop, a.to(DEV), c.to(DEV)])
    assert rel(y, _ref_conv([big[:, :, :24, :39], a, c], conv, bn, ACT_GELU)) < 1e-5
    # residual + mul (att broadcast over depth) on a 3-D conv
    conv3, bn3 = _mk(3, 1, 8, 3, 1, 1, seed=4)
    x3 = torch.randn(2, 1, 4, 6, 10)
    att = torch.randn(2, 8, 6, 10)
    res3 = torch.randn(2, 8, 4, 6, 10)
    y3 = run_conv(Ctx(DEV), pk(conv3, bn3, ACT_GELU), [x3.to(DEV)], mul=att.to(DEV), res=res3.to(DEV))
    assert rel(y3, _ref_conv([x3], conv3, bn3, ACT_GELU, mul=att, res=res3)) < 1e-5
    # ConvT 16->1 + bilinear(prev, x4) + x4 scale with an unscaled copy
    ct, _ = _mk(2, 16, 1, 4, 2, 1, transposed=True, bn=False, seed=5)
    xt = torch.randn(1, 16, 24, 40)
    prev = torch.randn(1, 1, 12, 20)
    cp = torch.empty(1, 1, 48, 80, device=DEV)
    yt = run_conv(Ctx(DEV), pk(ct, None, ACT_NONE), [xt.to(DEV)], up=prev.to(DEV), up_f=4, post_scale=4.0,
                  out2=cp, post_scale2=1.0)
    ref = _ref_conv([xt], ct, None, ACT_NONE, up=prev, up_f=4)
    assert rel(yt, ref * 4) < 1e-5
    assert rel(cp, ref) < 1e-5
    # 1x1 conv + PixelShuffle(4) + SiLU
    cs, _ = _mk(2, 8, 128, 1, 1, 0, bias=True, bn=False, seed=6)
    xs = torch.randn(1, 8, 6, 20)
    ys = run_conv(Ctx(DEV), pk(cs, None, ACT_SILU), [xs.to(DEV)], shuffle=4)
    assert rel(ys, _ref_conv([xs], cs, None, ACT_SILU, shuffle=4)) < 1e-5


# ----------------------------------------------------------------------------- ShuffleMixer


@pytest.mark.parametrize("C", [8, 16])
@pytest.mark.parametrize("H,W", [(21, 45), (90, 101)])  # (90, 101) x B 2: the two-launch form (>= FM2_MIN_PIX)
def test_fmblock_vs_oracle(C, H, W):
    torch.manual_seed(7)
    blk = E.FMBlock(C, 7, 2).eval()
    with torch.no_grad():
        for n, p in blk.named_parameters():
            if n.endswith("norm1.body.weight") or n.endswith("norm2.body.weight"):
                p.uniform_(0.8, 1.2)
    sd = {k: v.clone() for k, v in blk.state_dict().items()}
    x = torch.randn(2, C, H, W)
    y = blk.to(DEV)(x.to(DEV))
    assert rel(y, O.fm_block(sd, "", x)) < 1e-5


# ----------------------------------------------------------------------------- hot path


def _model_from_manifest(name, maxdisp=None):
    m = MANIFEST[name]
    model = E.ESMStereo(maxdisp or m["maxdisp"], m["cv"] == "gwc", m["cv"] == "nc", m["backbone"], m["cv_scale"],
                        feature_cls=StubFeature)
    sd = seeded_state(load_spec(m["spec"]), m["seed"])
    model.load_state_dict(sd)
    return model.eval().to(DEV), sd, m


def _top2_sets(cost):
    return top2_sets(cost)


def _flips_and_margin(cost_hip, cost_ref):
    """[B, D, h, w] HIP and reference costs -> (flip set, reference v2 - v3 margin), [B, h, w]."""
    cost_ref = torch.as_tensor(cost_ref).double().cpu()
    flips = (top2_sets(cost_hip.detach().cpu()) != top2_sets(cost_ref)).any(1)
    sv = torch.sort(cost_ref, dim=1, descending=True)[0]
    return flips, sv[:, 1] - sv[:, 2]


def _check_disp(name, got, ref, L=None):
    """S / M (continuous): EPE <= 1e-3 and relative max error <= 1e-4.  L: ``L = (cost_hip,
    cost_ref)`` [B, D, h, w] -> the flip-masked metric of SURVEY.md §8(d)(iii) (tests/parity.py)."""
    if L is None:
        e = epe(got, ref)
        assert e <= 1e-3, (name, e)
        assert rel(got, ref) <= 1e-4, (name, rel(got, ref))
        return {"epe": e}
    flips, margin = _flips_and_margin(*L)
    return flip_masked(name, got, ref, flips, margin, 4)


def _hip_cost(model, ml, mr, att, D):
    """Cost volume -> stems -> hourglass through the eager HIP modules."""
    from esmstereo_amd.engine import Ctx as _Ctx
    with torch.no_grad():
        if model.gwc:
            V = E.build_gwc_volume(ml, mr, D, 32, att=att)
            vol = model.group_stem(V)
        else:
            V = E.build_norm_correlation_volume(ml, mr, D)
            mul = att.reshape(att.shape[0], -1, *att.shape[-2:]) if att is not None else None
            vol = model.corr_stem.emit(_Ctx(DEV), [V], mul=mul)
        return model.aggregation_out(model.agg(vol))


def _check_L_decomposed(name, model, sd, up, cost_hip, ref_cost, plan_out, ref_disp0):
    """L: the flip-masked metric end to end, plus the HIP upsampler vs the oracle upsampler on the
    SAME init (continuous, so EPE <= 1e-3 everywhere)."""
    with torch.no_grad():
        init = E.regression_topk(cost_hip.squeeze(1), None, 2)
        eager = model.upsample_module(*up, init)
        ref_up = O.upsample4({k: v.cpu() for k, v in sd.items()}, "upsample_module.", *[u.cpu() for u in up],
                             init.cpu())
    assert torch.equal(plan_out, eager[0].squeeze(1) * 4), "compiled plan must equal the eager modules bitwise"
    e_up = epe(eager[0] * 4, ref_up[0] * 4)
    assert e_up <= 1e-3, (name, "upsampler", e_up)
    rep = _check_disp(name, plan_out, ref_disp0, L=(cost_hip[:, 0], torch.as_tensor(ref_cost)[:, 0]))
    print(f"{name}: {rep}; upsampler EPE on the same init {e_up:.2e}")
    return rep


@pytest.mark.parametrize("name", HOT)
def test_hot_path_golden(name):
    model, sd, m = _model_from_manifest(name)
    g = load_golden(name)
    up = [cu(g[f"up_{i}"]) for i in range(4) if f"up_{i}" in g]
    att = cu(g["att"]) if "att" in g else None
    # module-level pieces, eager, each on the reference's own input for that stage
    cost = model.aggregation_out(cu(g["agg"]))
    assert rel(cost, g["cost"]) < 1e-5
    ups = model.upsample_module(*up, cu(g["init_pred"]))
    for i in range(len(ups)):
        assert epe(ups[i].squeeze(1) * 4, g[f"disp_{i}"]) <= 1e-3
    Lc = None
    if m["cv_scale"] == 4:
        hip_cost = _hip_cost(model, cu(g["match_left"]), cu(g["match_right"]), att, m["maxdisp"] // 4)
        Lc = (hip_cost[:, 0], g["cost"][:, 0])
    # whole hot path, compiled plan + graph, eval and train outputs
    for train in (False, True):
        outs = model.hot_path(cu(g["match_left"]), cu(g["match_right"]), att, up, train)
        n = m["n_train_outputs"] if train else 1
        assert len(outs) == n
        for i in range(n):
            assert outs[i].shape == g[f"disp_{i}"].shape
            _check_disp(name, outs[i], g[f"disp_{i}"], Lc)


@pytest.mark.parametrize("name", HOT)
def test_full_forward_golden(name):
    """The drop-in module: backbone side on PyTorch/MIOpen + HIP BasicConvs, hot path on HIP."""
    model, sd, m = _model_from_manifest(name)
    g = load_golden(name)
    with torch.no_grad():
        out = model(cu(g["left"]), cu(g["right"]), False)
        ml, mr, att, up = model.prefix(cu(g["left"]), cu(g["right"]))
    assert isinstance(out, list) and len(out) == 1
    assert rel(ml, g["match_left"]) < 1e-4 and rel(mr, g["match_right"]) < 1e-4  # MIOpen prefix vs CPU
    Lc = None
    if m["cv_scale"] == 4:  # the prefix's MIOpen-vs-CPU rounding may move near-ties: flip-masked
        Lc = (_hip_cost(model, ml, mr, att, m["maxdisp"] // 4)[:, 0], g["cost"][:, 0])
    rep = _check_disp(name, out[0], g["disp_0"], Lc)
    print(name, rep)


@pytest.mark.parametrize("name", ["hot_S_gwc.npz", "hot_L_gwc.npz"])
def test_forward_graph_matches_eager(name):
    """The captured whole forward (model.ForwardGraph: the backbone side as a torch CUDA graph, the hot
    path's plan bound to its outputs) against the same module with the backbone side launched eagerly:
    bitwise, on the first images, on new images through the same captured graph, and after an in-place
    edit of a BACKBONE weight (the capture is keyed by every parameter's version: re-captured)."""
    model, sd, m = _model_from_manifest(name)
    g = load_golden(name)
    left, right = cu(g["left"]), cu(g["right"])

    def both(a, b):
        model.capture_forward = True
        got = model(a, b, False)[0]
        model.capture_forward = False
        ref = model(a, b, False)[0]
        model.capture_forward = True
        return got, ref

    with torch.no_grad():
        got, ref = both(left, right)
        assert torch.equal(got, ref), name
        assert epe(got, g["disp_0"]) <= (1e-3 if m["cv_scale"] != 4 else 1.0)
        fg = next(iter(model._fwd_graphs.values()))
        got, ref = both(right.flip(-1).contiguous(), left.flip(-1).contiguous())  # new images, same graph
        assert torch.equal(got, ref), name
        assert next(iter(model._fwd_graphs.values())) is fg
        w = next(p for n, p in model.named_parameters() if n.startswith("feature."))
        w.mul_(1.5)  # in place: the captured backbone must not replay stale packed / cached state
        got, ref = both(left, right)
        assert torch.equal(got, ref), name
        assert fg not in model._fwd_graphs.values()


def test_trt_forward_equals_eval_output():
    """ESMStereo_trt.forward(left, right) -> disp [B, H, W] (models/ESMStereo_trt.py:638,735) is the
    eval output of ESMStereo on the same weights, and matches the reference golden."""
    model, sd, m = _model_from_manifest("hot_S_gwc.npz")
    trt = E.ESMStereo_trt(m["maxdisp"], True, False, m["backbone"], m["cv_scale"], feature_cls=StubFeature)
    trt.load_state_dict(sd)
    trt = trt.eval().to(DEV)
    g = load_golden("hot_S_gwc.npz")
    with torch.no_grad():
        d = trt(cu(g["left"]), cu(g["right"]))
        ref = model(cu(g["left"]), cu(g["right"]), False)[0]
    assert isinstance(d, torch.Tensor) and d.shape == g["disp_0"].shape
    assert torch.equal(d, ref)
    assert epe(d, g["disp_0"]) <= 1e-3


def test_dataparallel_wrapper_and_state_dict_roundtrip():
    model, sd, m = _model_from_manifest("hot_S_gwc.npz")
    dp = torch.nn.DataParallel(model, device_ids=[0])
    sd2 = {"module." + k: v for k, v in sd.items()}
    model_dict = dp.state_dict()
    model_dict.update({k: v for k, v in sd2.items() if k in model_dict})
    dp.load_state_dict(model_dict)
    g = load_golden("hot_S_gwc.npz")
    with torch.no_grad():
        out = dp(cu(g["left"]), cu(g["right"]), train_status=False)
    assert epe(out[0], g["disp_0"]) <= 1e-3


def _full_inputs(model, B, H, W, seed, maxdisp, noise=False):
    """SURVEY.md §8(d) inputs through the model's own backbone side: a sinusoid-texture pair with
    a planar disparity field (peaked cost volume), or (noise=True) white noise with a 5-px roll,
    the near-tie stress case."""
    if noise:
        torch.manual_seed(seed)
        left = torch.randn(B, 3, H, W, device=DEV)
        right = torch.roll(left, shifts=-5, dims=-1) + 0.05 * torch.randn(B, 3, H, W, device=DEV)
    else:
        left, right = (t.to(DEV) for t in stereo_pair(B, H, W, seed, max_shift=maxdisp // 2))
    with torch.no_grad():
        return model.prefix(left, right)


@pytest.mark.parametrize("var,cv,B,H,W,maxdisp,noise", [
    ("S", "gwc", 1, 384, 1248, 192, False), ("S", "nc", 2, 384, 1248, 192, False),
    ("S", "gwc", 1, 384, 1248, 192, True), ("L", "gwc", 1, 384, 1248, 192, False),
    ("M", "gwc", 1, 256, 512, 192, False), ("L", "nc", 1, 384, 1248, 192, False),
    ("L", "gwc", 1, 384, 1248, 192, True),
    # BASELINE configs[3]'s per-rank slice (ESMStereo-L KITTI, global batch 32 over 8 GPUs -> 4 per rank)
    ("L", "gwc", 4, 384, 1248, 192, False),
    # configs[2] (SceneFlow 540x960 padded to 544, B=8) and configs[4] (Middlebury ~1500x1000 padded to
    # 1504x1024, md256)
    ("L", "gwc", 8, 544, 960, 192, False), ("L", "gwc", 1, 1024, 1504, 256, False)])
def test_hot_path_full_size_vs_oracle(var, cv, B, H, W, maxdisp, noise):
    model, sd, m = _model_from_manifest(f"hot_{var}_{cv}.npz", maxdisp=maxdisp)
    ml, mr, att, up = _full_inputs(model, B, H, W, 11, maxdisp, noise)
    outs = model.hot_path(ml, mr, att, up, True)
    with torch.no_grad():
        ref = O.hot_path({k: v.cpu() for k, v in sd.items()}, m["cv_scale"], maxdisp, cv == "gwc", ml.cpu(), mr.cpu(),
                         None if att is None else att.cpu(), [u.cpu() for u in up])
    cost = _hip_cost(model, ml, mr, att, maxdisp // m["cv_scale"])
    assert rel(cost, ref["cost"]) < 1e-5
    tag = f"{var}-{cv} B{B} {H}x{W} md{maxdisp}{' noise' if noise else ''}"
    if m["cv_scale"] == 4:
        _check_L_decomposed(tag, model, sd, up, cost, ref["cost"], outs[0], ref["disp_0"])
        for i, o in enumerate(outs[1:], 1):  # the training-mode outputs, same metric
            _check_disp(f"{tag} disp_{i}", o, ref[f"disp_{i}"], L=(cost[:, 0], ref["cost"][:, 0]))
        return
    for i, o in enumerate(outs):
        _check_disp(f"{tag} disp_{i}", o, ref[f"disp_{i}"])


def test_hot_path_gwc_stem_ab():
    """The L hot path with the fused gwc volume + group_stem launch equals the two-launch path bit for bit
    (every output), at a size where the fused form is taken (>= 2^16 volume voxels)."""
    from esmstereo_amd import engine
    model, sd, m = _model_from_manifest("hot_L_gwc.npz")
    ml, mr, att, up = _full_inputs(model, 2, 192, 624, 13, 192, False)
    outs = {}
    saved = engine.GWC_STEM_ENABLED
    try:
        for on in (True, False):
            engine.GWC_STEM_ENABLED = on
            model._plans.clear()
            outs[on] = [o.clone() for o in model.hot_path(ml, mr, att, up, True)]
            names = [x["name"] for x in model._plans[next(iter(model._plans))].ctx.meta]
            assert ("gwc_volume+group_stem" in names) == on, names[:3]
    finally:
        engine.GWC_STEM_ENABLED = saved
        model._plans.clear()
    for a, b in zip(outs[True], outs[False]):
        assert torch.equal(a, b)


@pytest.mark.parametrize("name", sorted(fullsize_manifest()))
def test_hot_path_fullsize_vs_reference(name):
    """BASELINE KITTI size pinned to the REFERENCE itself (not only the oracle): the HIP plan on the
    seeded feature inputs of tests/golden/full_*.npz vs the reference's cost summaries, init_pred and
    disp_0 (tests/parity.py check_fullsize; L flip-masked), and the HIP upsampler run on the
    reference's OWN init_pred vs disp_0 at every (subsampled) pixel, no mask."""
    m, g, (ml, mr, att, up) = fullsize_case(name)
    model, sd, _ = _model_from_manifest(f"hot_{m['variant']}_{m['cv']}.npz", maxdisp=m["maxdisp"])
    model.load_state_dict(seeded_state(load_spec(m["spec"]), m["weight_seed"]))
    ml, mr = cu(ml), cu(mr)
    att = None if att is None else cu(att)
    up = [cu(u) for u in up]
    D = m["maxdisp"] // m["cv_scale"]
    cost = _hip_cost(model, ml, mr, att, D)[:, 0]
    with torch.no_grad():
        init = E.regression_topk(cost, None, 2) if m["cv_scale"] == 4 else E.disparity_regression(cost, D)
    disp0 = model.hot_path(ml, mr, att, up)[0]
    with torch.no_grad():  # upsample_module on the reference's init_pred (models/ESMStereo.py:722-735)
        d_ref_init = E.engine.eager_emit(DEV, model.upsample_module.emit, up, cu(g["init_pred"]), final_scale=4.0)[0]
    rep = check_fullsize(name, m, g, cost, init.view(m["B"], 1, *cost.shape[-2:]), disp0,
                         disp0_from_ref_init=d_ref_init[:, 0])
    record_report(name, dict(rep, workload=f"ESMStereo-{m['variant']} {m['cv']} B{m['B']} "
                                           f"{m.get('H', '')}x{m.get('W', '')} md{m['maxdisp']}"))
    print(name, rep)


def test_concat_volume_configs2_size():
    """build_concat_volume (models/submodule.py:129-140) at BASELINE configs[2]'s size: ESMStereo-L
    SceneFlow 544x960 B=8 -> [8, 128, 48, 136, 240] (6.4 GB).  Checked bit-exact against the oracle
    on sampled (b, channel, d) planes, both halves, with the zero region x < d."""
    B, C, h, w, D = 8, 64, 136, 240, 48
    L, R = feature_pair(B, C, h, w, 21, D)
    Ld, Rd = L.to(DEV), R.to(DEV)
    V = E.build_concat_volume(Ld, Rd, D)
    assert V.shape == (B, 2 * C, D, h, w)
    rng = np.random.default_rng(5)
    for _ in range(48):
        b, c, d = int(rng.integers(B)), int(rng.integers(2 * C)), int(rng.integers(D))
        ref = O.concat_volume(L[b:b + 1, c % C:c % C + 1], R[b:b + 1, c % C:c % C + 1], D)[0, (c >= C) * 1, d]
        assert torch.equal(V[b, c, d].cpu(), ref), (b, c, d)
    for d in (0, 1, D - 1):  # whole planes at the extremes of d
        ref = O.concat_volume(L[:1], R[:1], D)[0, :, d]
        assert torch.equal(V[0, :, d].cpu(), ref), d
    del V
    torch.cuda.empty_cache()


def test_plan_modes_agree_and_probe():
    model, sd, m = _model_from_manifest("hot_L_gwc.npz")
    g = load_golden("hot_L_gwc.npz")
    args = (cu(g["match_left"]), cu(g["match_right"]), None, [cu(g[f"up_{i}"]) for i in range(3)])
    B, C, h, w = args[0].shape
    hp_graph = E.HotPath(model, B, h, w, 0, [tuple(u.shape) for u in args[3]], DEV, graph=True)
    hp_eager = E.HotPath(model, B, h, w, 0, [tuple(u.shape) for u in args[3]], DEV, graph=False)
    for hp in (hp_graph, hp_eager):
        hp.load_inputs(*args)
        hp.set_probe(0, 8)
        for _ in range(3):
            hp.launch()
    torch.cuda.synchronize()
    assert torch.equal(hp_graph.outputs[0], hp_eager.outputs[0])
    for hp in (hp_graph, hp_eager):
        t = hp.probe_read()
        assert len(t) == 3 and all(v > 0 for v in t), t
    assert hp_graph.num_ops > 30


@pytest.mark.parametrize("graph", [True, False])
def test_hot_path_reads_inputs_in_place(graph):
    """Zero-copy boundary: the plan reads the caller's feature tensors where they lie
    (esm_plan_rebind), for the S plan (att, four upsampler features) and the L plan.  Against the copy
    path (load_inputs into the plan's own buffers), bitwise: fresh tensors on every call, the same
    tensors edited in place (no stale copy), ml / mr swapped between calls (each pointer moves once),
    features allocated far (> 1 GiB) from the plan's arena (still read in place: every kernel has a
    descriptor per concat source), a non-contiguous feature (copied into the plan's buffer instead) and
    back to in place, all with the graph built (its nodes updated in place) and without."""
    for name in ("hot_S_gwc.npz", "hot_L_gwc.npz"):
        model, sd, m = _model_from_manifest(name)
        model.use_graph = graph
        g = load_golden(name)
        nup = sum(1 for k in g if k.startswith("up_"))
        ml, mr = cu(g["match_left"]), cu(g["match_right"])
        att = cu(g["att"]) if "att" in g else None
        up = [cu(g[f"up_{i}"]) for i in range(nup)]
        B, C, h, w = ml.shape
        ref_hp = E.HotPath(model, B, h, w, 0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], DEV,
                           graph=False)

        def expect(a, b, at, u):
            ref_hp.load_inputs(a, b, at, u)
            ref_hp.launch()
            return ref_hp.outputs[0].clone()

        with torch.no_grad():
            first = model.hot_path(ml, mr, att, up)[0]
            assert torch.equal(first, expect(ml, mr, att, up)), name
            for it in range(3):  # fresh allocations: the bound pointers move
                ml2, mr2 = ml * (1.0 + 0.1 * it), mr.clone()
                up2 = [u + 0.01 * it for u in up]
                out = model.hot_path(ml2, mr2, att, up2)[0]
                assert torch.equal(out, expect(ml2, mr2, att, up2)), (name, it)
            spacer = torch.empty(3 << 28, device=DEV)  # 3 GiB allocated between the plan's arena and the features
            upf = [u + 0.02 for u in up]
            out = model.hot_path(ml2, mr2, att, upf)[0]
            assert torch.equal(out, expect(ml2, mr2, att, upf)), name
            hp = list(model._plans.values())[-1]
            assert hp._bound[3:] == [u.data_ptr() for u in upf], name  # every feature read where it lies
            del spacer
            ml2.mul_(0.5)  # same tensors, new values: read in place, nothing stale
            out = model.hot_path(ml2, mr2, att, up2)[0]
            assert torch.equal(out, expect(ml2, mr2, att, up2)), name
            out = model.hot_path(mr2, ml2, att, up2)[0]  # swapped
            assert torch.equal(out, expect(mr2, ml2, att, up2)), name
            out = model.hot_path(ml2, ml2, att, up2)[0]  # aliased: one tensor in two slots
            assert torch.equal(out, expect(ml2, ml2, att, up2)), name
            out = model.hot_path(ml2, mr2, att, up2)[0]  # distinct again: each slot reads its own tensor
            assert torch.equal(out, expect(ml2, mr2, att, up2)), name
            ml3 = ml2 * 0.75
            out = model.hot_path(ml3, mr2, att, up2)[0]  # only ml moves after the aliased call
            assert torch.equal(out, expect(ml3, mr2, att, up2)), name
            u0 = up2[0]
            wide = torch.zeros((u0.shape[0], 2 * u0.shape[1]) + tuple(u0.shape[2:]), device=DEV)
            wide[:, 1::2] = u0
            upn = [wide[:, 1::2]] + up2[1:]  # non-contiguous (channel stride 2): copied into the plan's buffer
            out = model.hot_path(mr2, ml2, att, upn)[0]
            assert torch.equal(out, expect(mr2, ml2, att, upn)), name
            out = model.hot_path(ml, mr, att, up)[0]  # and back in place
            assert torch.equal(out, first), name
        ref_hp.close()


def test_hot_path_rebind_while_replay_runs():
    """A slot whose caller pointer changes while the previous replay is still running switches to
    copies into the plan's own buffer (no host wait for the device), and stays correct:
    fresh tensors, then the same tensor edited in place."""
    model, sd, m = _model_from_manifest("hot_S_gwc.npz")
    g = load_golden("hot_S_gwc.npz")
    ml, mr, att = cu(g["match_left"]), cu(g["match_right"]), cu(g["att"])
    up = [cu(g[f"up_{i}"]) for i in range(4)]
    B, C, h, w = ml.shape
    ref_hp = E.HotPath(model, B, h, w, int(att.shape[1]), [tuple(u.shape) for u in up], DEV, graph=False)

    def expect(a, b, at, u):
        ref_hp.load_inputs(a, b, at, u)
        ref_hp.launch()
        return ref_hp.outputs[0].clone()

    with torch.no_grad():
        model.hot_path(ml, mr, att, up)
        hp = list(model._plans.values())[-1]
        for _ in range(300):  # a queue of replays: the next bind finds the plan busy
            hp.launch()
        ml3 = ml * 1.25
        out = model.hot_path(ml3, mr, att, up)[0]
        assert hp._copy_mode[0] and hp._bound[0] == hp._own[0].data_ptr()
        assert torch.equal(out, expect(ml3, mr, att, up))
        ml3.mul_(0.5)
        out = model.hot_path(ml3, mr, att, up)[0]
        assert torch.equal(out, expect(ml3, mr, att, up))
    ref_hp.close()


def test_expected_raises():
    # reference raises on odd D and on H, W not multiples of 32 (§0.5)
    for var, cv, H, W, maxdisp in [("S", "gwc", 128, 256, 48), ("L", "gwc", 64, 128, 52), ("S", "gwc", 80, 128, 64)]:
        model, _, _ = _model_from_manifest(f"hot_{var}_{cv}.npz", maxdisp=maxdisp)
        left = torch.randn(1, 3, H, W, device=DEV)
        with pytest.raises(RuntimeError):
            with torch.no_grad():
                model(left, left, False)


@pytest.mark.parametrize("C,H,W", [(8, 24, 78), (8, 7, 13), (16, 96, 312), (16, 5, 40), (8, 1, 1), (8, 200, 100)])
def test_fmnet_fused_bitwise(C, H, W):
    """FMBlock.net + x in one launch (esm_fmnet_f32, halo recomputation) vs the three smix launches:
    the same per-pixel operations in the same order, up to the compiler's FMA contraction choices in
    the two kernels (relative 1e-6).  96x312 and 200x100 (ragged in 3) take the 3-row tile of the whole
    block, the others the 1-row tile."""
    from esmstereo_amd.engine import run_fmnet, run_smix

    torch.manual_seed(C * 100 + H)
    blk = E.FMBlock(C, 7).to(DEV).eval()
    with torch.no_grad():
        for prm in blk.parameters():
            prm.uniform_(-0.5, 0.5)
    p = blk._packed()
    x = torch.randn(2, C, H, W, device=DEV)
    ctx = Ctx(DEV)
    fused = run_fmnet(ctx, x, [p["a1"], p["a2"], p["b1"], p["b2"]], p["dw0"], p["dw1"])
    t1 = run_smix(ctx, x, [p["a1"]])
    t2 = run_smix(ctx, t1, [p["a2"], p["b1"]], dw=p["dw0"])
    t3 = run_smix(ctx, t2, [p["b2"]], dw=p["dw1"], res=x)
    assert rel(fused, t3) < 1e-6
    # the whole block in one launch (FMBlock.conv fused behind net) vs net + the two conv launches
    whole = run_fmnet(ctx, x, [p["a1"], p["a2"], p["b1"], p["b2"]], p["dw0"], p["dw1"], conv=p["cw"], two_launch=False)
    ref = run_conv(ctx, p["c2"], [run_conv(ctx, p["c0"], [t3])], res=t3)
    assert rel(whole, ref) < 1e-5
    # the two-launch form (smix.hip fm2a / fm2b: split at dw1, FMBlock.conv on the matrix cores)
    two = run_fmnet(ctx, x, [p["a1"], p["a2"], p["b1"], p["b2"]], p["dw0"], p["dw1"], conv=p["cw"], two_launch=True)
    assert rel(two, ref) < 1e-5


@pytest.mark.parametrize("cout,k,s,p,H,W", [(16, 3, 2, 1, 384, 1248), (16, 5, 1, 0, 96, 312), (32, 5, 1, 0, 37, 50),
                                            (16, 3, 2, 1, 9, 13), (32, 3, 2, 1, 96, 312), (8, 3, 1, 1, 20, 33)])
def test_conv_c1in_form(cout, k, s, p, H, W):
    """VALU single-input-channel 2-D form (conv_stem.hip c1in_kernel), forced and automatic, vs fp64."""
    conv, bn = _mk(2, 1, cout, k, s, p, seed=7)
    x = torch.randn(2, 1, H, W)
    ref = _ref_conv([x], conv, bn, ACT_GELU)
    pc = pk(conv, bn, ACT_GELU)
    for h in (1 << 20, 0):
        assert rel(run_conv(Ctx(DEV), pc, [x.to(DEV)], hint=h), ref) < 1e-5, hex(h)


def test_gelu_epilogue_branch_free_erf():
    """The conv epilogue's GELU (common.h erf_bf: the device library's erff polynomials, evaluated
    branch-free) through a 1x1 identity conv over [-12, 12], densest around the |x / sqrt 2| = 1 switch,
    vs fp64 torch GELU: |error| <= 2.5e-7 |x| (2 fp32 ulps of the input's scale: 1 + erf cancels for
    negative x, in every fp32 evaluation of the formula, torch's own included)."""
    x = torch.cat([torch.linspace(-12, 12, 200001), torch.linspace(1.40, 1.43, 20001),
                   torch.linspace(-1.43, -1.40, 20001), torch.tensor([0.0, -0.0, 1e-30, -1e-30])])
    n = x.numel()
    conv = torch.nn.Conv2d(1, 1, 1, bias=False)
    with torch.no_grad():
        conv.weight.fill_(1.0)
    p = pk(conv, None, ACT_GELU)
    for hint in (0, HINT_SMALL, HINT_WIDE):
        y = run_conv(Ctx(DEV), p, [x.view(1, 1, 1, n).to(DEV)], hint=hint).view(-1).double().cpu()
        ref = F.gelu(x.double())
        assert bool(((y - ref).abs() <= 2.5e-7 * x.double().abs() + 1e-37).all()), hex(hint)
        yt = F.gelu(x.to(DEV)).double().cpu()  # torch's own fp32 GELU meets the same bound
        assert bool(((yt - ref).abs() <= 2.5e-7 * x.double().abs() + 1e-37).all())
