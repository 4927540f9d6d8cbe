"""Shared parity metrics for the CPU oracle tests and the GPU parity tests.

* ``flip_masked`` — the ESMStereo-L metric (§8(d)(iii)).  ``regression_topk`` (reference
  ``models/submodule.py:218-225``) picks the top-2 disparity indices of the aggregated cost, so
  its output jumps where the 2nd and 3rd largest costs nearly tie (§0.6: the reference run against
  itself, 8 vs 1 CPU threads, flips 12 of 29,952 low-res pixels at L/KITTI).  The metric:
    1. the low-res pixels whose top-2 index SET differs from the reference's are the flips;
    2. every flip must sit where the REFERENCE's own margin (2nd minus 3rd largest cost) is at most
       ``TOPK_MARGIN_TOL``: a flip anywhere else is a real error and fails;
    3. the flips are dilated by the upsampler's receptive field (``UPSAMPLER_RF``), upsampled
       x cv_scale to full resolution, and EPE <= 1e-3 px is required over every pixel outside.
* ``check_fullsize`` — a full-size configuration against the reference's own summary fixture
  (``tests/golden/full_*.npz``, written by ``tests/golden/make_golden.py --fullsize``).
"""
from __future__ import annotations

import json
import os
from typing import Dict, Optional

import numpy as np
import torch
import torch.nn.functional as F

from helpers import GOLDEN_DIR, digest, fullsize_inputs, load_golden

EPE_TOL = 1e-3          # px, north_star: "EPE within 1e-3 of the PyTorch reference"
COST_REL_TOL = 1e-5     # aggregated cost, relative to its max |value| (fp32, different summation orders)
TOPK_MARGIN_TOL = 1e-4  # a top-2 flip is legitimate only where the reference's v2 - v3 <= this
# The flip mask may hide at most this share of the image, unless every flip sits on a reference
# margin <= MASK_TIE_TOL (a tie at fp32 resolution, where either top-2 set is the reference's answer)
MASK_MAX_FRAC = 0.25
MASK_TIE_TOL = 1e-6
# Exact support of one low-res init pixel's influence on the final disparity, in low-res pixels,
# for upsample4 (ESMStereo-L, models/ESMStereo.py:242-318): dm2x (4) + spx_2x (2) + to_feat (1) +
# 2 FMBlocks (2 x (2 x 3 depthwise 7x7 + 1)) = 21 at 1/4 res; x2 -> 42 + tail2x 1 + ref2x's
# hourglass 41 = 84 at 1/2 res; + dm4x 4 + spx_4x 2 + (tail4x 1 + ref4x 41) / 2 = 111 at 1/2 res
# -> 56 at 1/4 res.  Measured with the oracle (one init pixel perturbed, exact non-zero support):
# -49.25 .. +55 low-res px.
UPSAMPLER_RF = {4: 56}


def top2_sets(cost: torch.Tensor) -> torch.Tensor:
    """[B, D, h, w] -> [B, 2, h, w] sorted top-2 index sets (value desc, lowest index on ties)."""
    idx = torch.sort(cost.double(), dim=1, descending=True, stable=True)[1][:, :2]
    return torch.sort(idx, dim=1)[0]


def flip_masked(name: str, got: torch.Tensor, ref: torch.Tensor, flips: torch.Tensor, margin: torch.Tensor,
                cv_scale: int, ref_valid: Optional[torch.Tensor] = None) -> Dict[str, float]:
    """got/ref: [B, H', W'] disparities (H' = H or a regular subsample of it, see ``sub``); flips,
    margin: [B, h, w] low-res flip set and reference top-2/3 margin."""
    got = got.detach().double().cpu()
    ref = torch.as_tensor(ref).double().cpu()
    flips = flips.cpu()
    n = int(flips.sum())
    bad = flips & (margin.cpu().double() > TOPK_MARGIN_TOL)
    assert not bad.any(), (name, "top-2 flip where the reference margin exceeds the tolerance",
                           margin.cpu()[bad][:8].tolist())
    r = UPSAMPLER_RF[cv_scale]
    m = F.max_pool2d(flips.double().unsqueeze(1), 2 * r + 1, 1, r)[:, 0] > 0
    f = got.shape[-1] // flips.shape[-1]  # full-res (or subsampled) pixels per low-res pixel
    m = m.repeat_interleave(f, -2).repeat_interleave(f, -1)
    keep = ~m
    e_all = float((got - ref).abs().mean())
    e = float((got - ref).abs()[keep].mean()) if keep.any() else 0.0
    rep = {"flips": n, "lowres_px": int(flips.numel()), "masked_frac": float(m.double().mean()),
           "epe_outside_mask": e, "epe_all": e_all,
           "max_flip_margin": float(margin.cpu()[flips].max()) if n else 0.0}
    assert e <= EPE_TOL, (name, rep)
    assert rep["masked_frac"] <= MASK_MAX_FRAC or rep["max_flip_margin"] <= MASK_TIE_TOL, (name, rep)
    return rep


def init_nonflip(name: str, got: torch.Tensor, ref: torch.Tensor, flips: torch.Tensor, margin: torch.Tensor
                 ) -> Dict[str, float]:
    """ESMStereo-L ``init_pred`` (regression_topk at low resolution, per pixel): a top-2 flip changes that
    pixel only, so every low-res pixel whose top-2 set matches the reference's is checked, with no
    dilation: EPE <= 1e-3 px over them, and every flip must sit on a reference margin
    <= TOPK_MARGIN_TOL.  got / ref / flips / margin: [B, h, w]."""
    got = got.detach().double().cpu()
    ref = torch.as_tensor(ref).double().cpu()
    flips = flips.cpu()
    bad = flips & (margin.cpu().double() > TOPK_MARGIN_TOL)
    assert not bad.any(), (name, "top-2 flip where the reference margin exceeds the tolerance",
                           margin.cpu()[bad][:8].tolist())
    keep = ~flips
    d = (got - ref).abs()
    rep = {"flips": int(flips.sum()), "lowres_px": int(flips.numel()), "checked_frac": float(keep.double().mean()),
           "epe_nonflip": float(d[keep].mean()) if keep.any() else 0.0,
           "max_err_nonflip": float(d[keep].max()) if keep.any() else 0.0, "epe_all": float(d.mean())}
    assert rep["epe_nonflip"] <= EPE_TOL, (name, rep)
    return rep


def rel(a, b) -> float:
    a = torch.as_tensor(a).detach().double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp_min(1e-30))


def fullsize_manifest() -> Dict[str, dict]:
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        man = json.load(f)
    return {k: v for k, v in man.items() if k.startswith("full_")}


def fullsize_case(name: str):
    """(manifest entry, fixture arrays, (ml, mr, att, up) numpy inputs regenerated from the seed)."""
    m = fullsize_manifest()[name]
    g = load_golden(name)
    ins = fullsize_inputs(m["cv_scale"], m["B"], m["H"], m["W"], m["maxdisp"], m["input_seed"],
                          att=m["cv_scale"] == 16)
    ml, mr, att, up = ins
    assert digest(ml, mr, att, *up) == m["input_sha256"], "regenerated inputs differ from the fixture's"
    return m, g, ins


def check_fullsize(name: str, m: dict, g: Dict[str, np.ndarray], cost: torch.Tensor, init: torch.Tensor,
                   disp0: torch.Tensor, disp0_from_ref_init: Optional[torch.Tensor] = None) -> Dict[str, float]:
    """cost [B, D, h, w], init [B, 1, h, w], disp0 [B, H, W] from the path under test vs the
    reference fixture.  S (continuous disparity_regression): EPE <= 1e-3 on init and on the
    subsampled disp_0; L: init at every low-res pixel whose top-2 set did not flip (no dilation), the
    flip-masked metric on disp_0.  ``disp0_from_ref_init`` [B, H, W]: the
    upsampler under test run on the REFERENCE's own init_pred (g["init_pred"]), which carries every
    top-2 decision the reference made, so it must match disp_0 at EVERY pixel (EPE <= 1e-3, no mask):
    this pins the upsampler where the flip mask would hide it."""
    cost = cost.detach().double().cpu()
    flat = cost.reshape(-1)
    amax = float(g["cost_absmax"])
    rep = {"cost_sample_rel": float((flat[torch.from_numpy(g["cost_idx"])] -
                                     torch.from_numpy(g["cost_val"]).double()).abs().max() / amax),
           "cost_sum_rel": abs(float(cost.sum()) - float(g["cost_sum"])) / float(cost.abs().sum()),
           "cost_l2_rel": abs(float(cost.norm()) - float(g["cost_l2"])) / float(g["cost_l2"])}
    assert rep["cost_sample_rel"] <= COST_REL_TOL and rep["cost_l2_rel"] <= COST_REL_TOL, (name, rep)
    assert rep["cost_sum_rel"] <= COST_REL_TOL, (name, rep)
    sub = disp0.detach()[:, ::4, ::4]
    ref_sub = torch.from_numpy(g["disp0_sub"])
    d0 = disp0.detach().double().cpu()
    rep["disp0_l2_rel"] = abs(float(d0.norm()) - float(g["disp0_l2"])) / float(g["disp0_l2"])
    if disp0_from_ref_init is not None:
        dr = disp0_from_ref_init.detach()[:, ::4, ::4].double().cpu()
        rep["disp0_sub_epe_ref_init"] = float((dr - ref_sub.double()).abs().mean())
        rep["disp0_sub_max_err_ref_init"] = float((dr - ref_sub.double()).abs().max())
        assert rep["disp0_sub_epe_ref_init"] <= EPE_TOL, (name, rep)
    if m["cv_scale"] == 4:
        flips = (top2_sets(cost) != torch.sort(torch.from_numpy(g["top3_idx"][:, :2]).long(), 1)[0]).any(1)
        tv = torch.from_numpy(g["top3_val"])
        margin = tv[:, 1] - tv[:, 2]
        # init: every pixel that did not flip, no dilation; disp_0: the dilated flip mask (a flip moves the
        # upsampler's output over its receptive field)
        rep["init"] = init_nonflip(name + ":init", init[:, 0], g["init_pred"][:, 0], flips, margin)
        rep["disp0"] = flip_masked(name + ":disp0", sub, ref_sub, flips, margin, 4)
    else:
        rep["init_epe"] = float((init.detach().double().cpu() - torch.from_numpy(g["init_pred"]).double()).abs().mean())
        rep["disp0_sub_epe"] = float((sub.double().cpu() - ref_sub.double()).abs().mean())
        assert rep["init_epe"] <= EPE_TOL and rep["disp0_sub_epe"] <= EPE_TOL, (name, rep)
        assert rep["disp0_l2_rel"] <= 1e-5, (name, rep)
    return rep


REPORT_PATH = os.environ.get("ESM_PARITY_REPORT") or os.path.join(os.path.dirname(GOLDEN_DIR), os.pardir,
                                                                     "gpurun_out", "parity_fullsize.json")


def record_report(name: str, rep: Dict[str, object], path: Optional[str] = None) -> None:
    """Merge one fixture's parity report (flips, masked fraction, EPE outside the mask, the upsampler on
    the reference's own init) into a JSON file keyed by fixture name, so the numbers survive ``pytest
    -q`` (copied to profiles/ per round)."""
    path = os.path.abspath(path or REPORT_PATH)
    os.makedirs(os.path.dirname(path), exist_ok=True)
    try:
        with open(path) as f:
            allrep = json.load(f)
    except (OSError, ValueError):
        allrep = {}
    allrep[name] = rep
    with open(path, "w") as f:
        json.dump(allrep, f, indent=1, sort_keys=True)

