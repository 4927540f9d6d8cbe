"""The algorithmic cost the benchmark's rooflines are priced on (``Ctx.meta`` of every launch of the
compiled hot path, bench.py ``roofline`` / ``roofline_step``), checked on the CPU without a GPU: the
plan is emitted dry (``esmstereo_amd.model.plan_ops``: shape-only buffers, nothing submitted) for the
S-K, M-K, L-K and Middlebury plans and every op's flops and bytes are recomputed here, independently
of engine.py:

* the sum of the conv-like ops' flops equals what ``torch.utils.flop_counter`` counts for the CPU
  oracle (oracle/esm_oracle.py, the reference's forward restated) run on shape-only tensors: every
  convolution of models/ESMStereo.py:700-745, the ShuffleMixer heads' 1x1 / 3x3 and the FMBlocks'
  split-point MLPs / depthwise convs included;
* each conv / conv-pair / shuffle / FMBlock / volume / regression op's flops and bytes from the
  layer's own weight shape and the extents, with the conv output extent re-derived from the layer's
  kernel / stride / padding.
"""
import math
import re

import pytest
import torch
from torch.utils.flop_counter import FlopCounterMode

import esmstereo_amd as E
from esmstereo_amd.backbone import StubFeature
from esmstereo_amd.model import plan_ops
from helpers import UP_LAYOUT, load_spec, seeded_state
from oracle import esm_oracle as O

CASES = {  # name: (variant, backbone, cv_scale, B, H, W, maxdisp)
    "S-K": ("S", "mobilenetv2_100", 16, 1, 384, 1248, 192),
    "M-K": ("M", "efficientnet_b2", 8, 1, 384, 1248, 192),
    "L-K": ("L", "efficientnet_b2", 4, 1, 384, 1248, 192),
    "L-K B4": ("L", "efficientnet_b2", 4, 4, 384, 1248, 192),
    "Mid": ("L", "efficientnet_b2", 4, 1, 1024, 1504, 256),
}
CONV_KINDS = ("conv", "conv_pair", "shuffle_tail", "shuffle_conv", "fmnet", "gwc_stem", "conv_up1")


def _plan(case):
    var, bb, cvs, B, H, W, md = CASES[case]
    sd = seeded_state(load_spec(f"spec_{var}_gwc.json"), 1)
    m = E.ESMStereo(md, True, False, bb, cvs, feature_cls=StubFeature)
    m.load_state_dict(sd)
    m.eval()
    ups = [(B, c, H // s, W // s) for c, s in UP_LAYOUT[cvs]]
    return m, sd, plan_ops(m, B, H // cvs, W // cvs, 32 if cvs == 16 else 0, ups), (B, H, W, md, cvs, ups)


@pytest.mark.parametrize("case", sorted(CASES))
def test_plan_flops_equal_flop_counter_on_oracle(case):
    m, sd, meta, (B, H, W, md, cvs, ups) = _plan(case)
    h, w = H // cvs, W // cvs
    M = lambda *s: torch.empty(*s, device="meta")  # noqa: E731
    fc = FlopCounterMode(display=False)
    with fc, torch.no_grad():
        O.hot_path({k: v.to("meta") for k, v in sd.items()}, cvs, md, True, M(B, 64, h, w), M(B, 64, h, w),
                   M(B, 32, h, w) if cvs == 16 else None, [M(*u) for u in ups])
    counted = fc.get_total_flops()
    # the flop counter sees convolutions only: take out disparity_regression's 2·B·D·h·w where the first pair
    # of the upsampler computes it (the `disparity_regression+` pair)
    reg = sum(2 * B * (md // cvs) * h * w for x in meta if x["name"].startswith("disparity_regression+"))
    # and the gwc volume's 2·B·C·D·h·w where the fused gwc_stem launch forms it (round 5)
    reg += sum(2 * B * 64 * (md // cvs) * h * w for x in meta if x["kind"] == "gwc_stem")
    ours = sum(x["flops"] for x in meta if x["kind"] in CONV_KINDS) - reg
    assert ours == counted, (case, ours, counted, ours - counted)


def _ext(s):
    return tuple(int(v) for v in s.split("x"))


def _layer(model, name):
    mod = model.get_submodule(name)
    return mod.conv if isinstance(mod, E.BasicConv) else mod


def _conv_cost(conv, B, ein, eout, scale2=False, split=None):
    """(flops, bytes, output extent re-derived from the layer) of one conv launch; ``split`` = (lo, hi): the
    launch covers the layer's input channels [lo, hi) only (round 6: the fork-join partial sums)."""
    w = conv.weight if split is None else conv.weight[:, split[0]:split[1]]
    nd = w.dim() - 2
    taps = math.prod(w.shape[2:])
    tr = isinstance(conv, (torch.nn.ConvTranspose2d, torch.nn.ConvTranspose3d))
    cin, cout = (w.shape[0], w.shape[1]) if tr else (w.shape[1], w.shape[0])
    sp = ein[-nd:]
    if tr:
        want = tuple(2 * v for v in sp)
    else:
        k, s, p = conv.kernel_size[0], conv.stride[0], conv.padding[0]
        want = tuple((v + 2 * p - k) // s + 1 for v in sp)
    vin, vout = B * math.prod(sp), B * math.prod(eout[-nd:])
    flops = 2 * (vin if tr else vout) * cin * cout * taps
    byts = 4 * (vin * cin + vout * cout + cin * cout * taps)
    return flops, byts, want, vout * cout


@pytest.mark.parametrize("case", sorted(CASES))
def test_plan_per_op_cost(case):
    m, sd, meta, (B, H, W, md, cvs, ups) = _plan(case)
    h, w = H // cvs, W // cvs
    D = md // cvs
    for op in meta:
        name, kind, shape = op["name"], op["kind"], op.get("shape", "")
        if kind == "conv":
            g = re.search(r"in (\S+) out (\S+)", shape)
            ein, eout = _ext(g.group(1)), _ext(g.group(2))
            split = op.get("split")
            f, b, want, nout = _conv_cost(_layer(m, op.get("layer", name)), B, ein, eout, split=split)
            if split is not None and split[0] == 0:
                b += 4 * nout  # the chain's part reads the side branch's partial sum
            assert want == eout[-len(want):], (name, want, eout)
            assert op["flops"] == f, name
            if re.match(r"upsample_module\.ref\d+x\.conv1_up$", name):
                # the epilogue adds bilinear(previous disparity, r): its 1-channel source is read too
                r = 4 if cvs == 16 else 2
                b += 4 * B * (eout[-2] // r) * (eout[-1] // r)
            assert op["bytes"] == b, (name, op["bytes"], b)
        elif kind == "conv_pair":
            sa, sb = shape[len("pair "):].split(" + ")
            reg = name.startswith("disparity_regression+")  # convA's 1-channel input regressed from the cost
            na, nb = name.split("+")[-2:]
            nb = na.rsplit(".", 1)[0] + "." + nb
            ga, gb = re.search(r"in (\S+) out (\S+)", sa), re.search(r"in (\S+) out (\S+)", sb)
            fa, ba, wa, mid = _conv_cost(_layer(m, na), B, _ext(ga.group(1)), _ext(ga.group(2)))
            fb, bb, wb, _ = _conv_cost(_layer(m, nb), B, _ext(gb.group(1)), _ext(gb.group(2)))
            if reg:
                assert cvs != 4 and _ext(ga.group(1)) == (1, h, w), name
                fa += 2 * B * D * h * w
                ba += 4 * B * D * h * w  # the D cost planes read; the map is written instead of read
            assert op["flops"] == fa + fb, name
            assert op["bytes"] == ba + bb - 2 * 4 * mid, name  # the intermediate map never reaches HBM
        elif kind == "conv_up1":  # round 6: transposed conv + crop + cat + 1x1, the conv's output never written
            sa, sb = shape.split(" + ")
            na = name.split("+")[0]
            nb = na.rsplit(".", 1)[0] + "." + name.split("+")[1]
            ga, gb = re.search(r"in (\S+) out (\S+)", sa), re.search(r"in (\S+) out (\S+)", sb)
            la, lb = _layer(m, na), _layer(m, nb)
            fa, ba, wa, nout = _conv_cost(la, B, _ext(ga.group(1)), _ext(ga.group(2)))
            split = op.get("split")
            fb, bb, wb, nb = _conv_cost(lb, B, _ext(gb.group(1)), _ext(gb.group(2)), split=split)
            if split is not None:
                bb += 4 * nb  # the fork-join partial sum of the image-feature channels, read
            cy = la.weight.shape[1]
            crop = _ext(gb.group(1))[-la.weight.dim() + 2:]
            assert all(c <= u for c, u in zip(crop, wa)), name
            assert op["flops"] == fa + fb, name
            assert op["bytes"] == ba + bb - 4 * nout - 4 * B * cy * math.prod(crop), name
        elif kind in ("shuffle_tail", "shuffle_conv"):
            g = re.search(r"nf(\d+) r(\d+) in (\d+)x(\d+)", shape)
            nf, r, hi, wi = (int(v) for v in g.groups())
            npix = B * hi * wi * r * r
            head = 2 * B * hi * wi * nf * nf * r * r + 2 * npix * nf * 9  # 1x1 nf -> nf r^2, then 3x3 nf -> 1
            if kind == "shuffle_tail":
                assert op["flops"] == head and op["bytes"] == 4 * (B * nf * hi * wi + npix), name
            else:
                g3 = re.search(r" -> k3 C(\d+)$", shape)  # round 5: up_refinement.conv1[1] fused behind it
                if g3:
                    shape = shape[:g3.start()]
                g2 = re.search(r"C(\d+) (\d+)x(\d+)$", shape)
                c, ho, wo = (int(v) for v in g2.groups())
                gp = re.match(r"pre (\d+)->(\d+) k3 ", shape)  # the stage's spx_<t>[1] inside the launch
                cp = int(gp.group(1)) if gp else 0
                if gp:
                    spx1 = _layer(m, name.split("+")[0])
                    assert tuple(spx1.weight.shape) == (nf, cp, 3, 3), name
                pre_f = 2 * B * hi * wi * nf * cp * 9
                c2f, c2b = 0, 0
                if g3:
                    conv11 = _layer(m, name.split(".", 1)[0] + "." + name.rsplit("+", 1)[-1] + ".1")
                    assert tuple(conv11.weight.shape) == (c, c, 3, 3), name
                    c2f, c2b = 2 * B * ho * wo * c * c * 9, 4 * 9 * c * c
                assert op["flops"] == head + 2 * B * ho * wo * c * 9 + pre_f + c2f, name
                assert op["bytes"] == 4 * (B * (cp or nf) * hi * wi + B * c * ho * wo) + 4 * 9 * cp * nf + c2b, name
        elif kind == "fmnet":
            g = re.search(r"C(\d+) (\d+)x(\d+) dw(\d+)", shape)
            C, hh, ww, k = (int(v) for v in g.groups())
            hid = C + 16
            per_px = 4 * 2 * (C // 2 * C + C * C // 2) + 2 * 2 * C * k * k + 2 * (9 * C * hid + hid * C)
            assert op["flops"] == B * hh * ww * per_px, name
            conv_w = 9 * C * hid + hid + hid * C + C
            assert op["bytes"] == 4 * (2 * B * C * hh * ww + conv_w), name
        elif kind == "gwc":
            G = 32
            assert op["flops"] == 2 * B * 64 * D * h * w
            assert op["bytes"] == 4 * B * (2 * 64 * h * w + G * D * h * w + (G * h * w if cvs == 16 else 0))
        elif kind == "gwc_stem":  # the volume formed in LDS, never written: features in, stem output out
            g = re.search(r"in (\S+) out (\S+)", shape)
            stem = _layer(m, name.split("+", 1)[1])
            f, _, want, nout = _conv_cost(stem, B, _ext(g.group(1)), _ext(g.group(2)))
            assert _ext(g.group(1)) == (D, h, w) and want == (D, h, w), name
            assert op["flops"] == f + 2 * B * 64 * D * h * w, name
            assert op["bytes"] == 4 * (B * 2 * 64 * h * w + nout + stem.weight.numel()), name
        elif kind == "regression":
            assert op["bytes"] == 4 * B * (D + 1) * h * w
        else:
            raise AssertionError(f"unchecked op kind {kind} ({name})")


def test_shuffle_head_flops_s_k():
    """upsampling4 + tail4x at S-K is 2 * 384 * 1248 * 8 * (8 + 9) = 130.35 MFLOP; fused with
    ref4x.conv1[0] (the row-form shuffle_conv, round 4) plus the 1 -> 16 3x3 stride-2 conv on 192 x 624."""
    _, _, meta, _ = _plan("S-K")
    op = next(x for x in meta if "upsampling4+tail4x" in x["name"])
    head = 2 * 384 * 1248 * 8 * 17
    assert head == 130_351_104
    pre = 2 * 96 * 312 * 8 * 16 * 9 if op["name"].startswith("upsample_module.spx_4x.1+") else 0  # spx_4x[1] inside
    if op["name"].endswith("+ref4x.conv1.0"):
        assert op["kind"] == "shuffle_conv"
        assert op["flops"] == head + 2 * 192 * 624 * 16 * 9 + pre
    elif op["name"].endswith("+ref4x.conv1"):  # round 5: conv1[1] (3x3 16 -> 16 on 192 x 624) in the launch too
        assert op["kind"] == "shuffle_conv"
        assert op["flops"] == head + 2 * 192 * 624 * 16 * 9 + pre + 2 * 192 * 624 * 16 * 16 * 9
    else:
        assert op["flops"] == head
