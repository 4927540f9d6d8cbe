"""Hot-path modules of ESMStereo, re-expressed for the HIP engine.

Class names, constructor arguments and state-dict keys follow the reference
(``models/submodule.py:12-103``, ``models/ESMStereo.py:129-509``) so checkpoints load
unchanged; every forward is a sequence of ``libesmstereo_amd`` launches described once in
an ``emit(ctx, ...)`` method (used both by the eager nn.Module forward and by the compiled
whole-hot-path plan).  Fusions relative to the reference op graph:

* ``torch.cat`` (+ the crops of ESMStereo.py:172,177,230) become extra K sources of the
  next conv; nothing is materialised;
* BatchNorm (eval) and conv biases fold into a per-channel scale/shift epilogue, GELU /
  SiLU run in the same epilogue;
* ``Conv2d(1x1) -> PixelShuffle -> SiLU -> tail Conv2d(3x3 -> 1)`` is one launch
  (``esm_shuffle_tail_f32``): the shuffled map is never written;
* ``F.interpolate(prev, bilinear) + refinement`` is the epilogue of the refinement's last
  transposed conv, and the final ``* 4`` (ESMStereo.py:737-745) folds into its store.
"""
from __future__ import annotations

from typing import List, Optional, Sequence, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .engine import (ACT_GELU, ACT_NONE, CONVT1X1_PAIRED, FORK_ENABLED, SC11_ENABLED, Ctx, PackedConv,
                     convt_1x1_supported, eager_emit, forked_packs, pack_conv, pack_shuffle_tail, pair2_auto,
                     param_token, run_conv, run_conv_forked, run_convt_1x1, run_pair2, run_shuffle_conv,
                     run_shuffle_tail, run_side_partial, shuffle_conv_pre_supported, shuffle_conv_supported)
from .mixer import FMBlock

__all__ = ["BasicConv", "Conv2x", "aggregation", "up_refinement", "upsample4", "upsample8", "upsample16"]


class BasicConv(nn.Module):
    """conv (bias=False) -> BatchNorm -> exact GELU, 2-D or 3-D, normal or transposed
    (reference models/submodule.py:12-38); one fused HIP launch."""

    def __init__(self, in_channels: int, out_channels: int, deconv: bool = False, is_3d: bool = False,
                 bn: bool = True, gelu: bool = True, **kwargs) -> None:
        super().__init__()
        self.gelu = gelu
        self.use_bn = bn
        kinds = {(False, False): nn.Conv2d, (False, True): nn.ConvTranspose2d,
                 (True, False): nn.Conv3d, (True, True): nn.ConvTranspose3d}
        self.conv = kinds[(bool(is_3d), bool(deconv))](in_channels, out_channels, bias=False, **kwargs)
        self.bn = (nn.BatchNorm3d if is_3d else nn.BatchNorm2d)(out_channels)
        self._esm = None

    def packed(self) -> PackedConv:
        tok = param_token(self.conv, self.bn) + (self.use_bn, self.gelu)
        if self._esm is None or self._esm[0] != tok:
            self._esm = (tok, pack_conv(self.conv, self.bn if self.use_bn else None,
                                        ACT_GELU if self.gelu else ACT_NONE))
        return self._esm[1]

    def emit(self, ctx: Ctx, srcs: Sequence[torch.Tensor], **epi) -> torch.Tensor:
        return run_conv(ctx, self.packed(), srcs, tag=getattr(self, "_esm_name", "BasicConv"), **epi)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return self.emit(Ctx(x.device), [x])


class Conv2x(nn.Module):
    """Decoder step of the backbone neck (reference models/submodule.py:64-103).  Out of the
    hot path (FeatUp); kept for checkpoint compatibility, convs run through BasicConv."""

    def __init__(self, in_channels: int, out_channels: int, deconv: bool = False, is_3d: bool = False,
                 concat: bool = True, keep_concat: bool = True, bn: bool = True, gelu: bool = True,
                 keep_dispc: bool = False) -> None:
        super().__init__()
        self.concat = concat
        self.is_3d = is_3d
        if deconv and is_3d and keep_dispc:
            self.conv1 = BasicConv(in_channels, out_channels, deconv, is_3d, bn=True, gelu=True,
                                   kernel_size=(1, 4, 4), stride=(1, 2, 2), padding=(0, 1, 1))
        else:
            k = (4 if not is_3d else (4, 4, 4)) if deconv else 3
            self.conv1 = BasicConv(in_channels, out_channels, deconv, is_3d, bn=True, gelu=True, kernel_size=k,
                                   stride=2, padding=1)
        mul = (2 if keep_concat else 1) if concat else 1
        cin2 = out_channels * 2 if concat else out_channels
        self.conv2 = BasicConv(cin2, out_channels * mul, False, is_3d, bn, gelu, kernel_size=3, stride=1, padding=1)

    def forward(self, x: torch.Tensor, rem: torch.Tensor) -> torch.Tensor:
        x = self.conv1(x)
        if x.shape != rem.shape:
            x = F.interpolate(x, size=(rem.shape[-2], rem.shape[-1]), mode="nearest")
        if self.concat:
            return self.conv2.emit(Ctx(x.device), [x, rem]) if x.shape[1] % 4 == 0 and rem.shape[1] % 4 == 0 \
                else self.conv2(torch.cat((x, rem), 1))
        return self.conv2(x + rem)


def _bc(cin: int, cout: int, is_3d: bool, k: int = 3, s: int = 1, p: int = 1, **kw) -> BasicConv:
    return BasicConv(cin, cout, is_3d=is_3d, kernel_size=k, stride=s, padding=p, **kw)


def _up(cin: int, cout: int, is_3d: bool, last: bool = False) -> BasicConv:
    return BasicConv(cin, cout, deconv=True, is_3d=is_3d, bn=not last, gelu=not last, kernel_size=4, padding=1,
                     stride=2)


def _pair(ctx: Ctx, first: BasicConv, srcs: Sequence[torch.Tensor], second, second_packed: Optional[PackedConv] = None,
          regress: Optional[torch.Tensor] = None, **kw) -> torch.Tensor:
    """``second(first(cat(srcs)))``: one launch with the intermediate in LDS where conv_pair2.hip has the
    shape (2-D, plain BN + GELU epilogues), else two launches.  ``regress``: see engine.run_pair2."""
    n0 = getattr(first, "_esm_name", "BasicConv")
    n1 = getattr(second, "_esm_name", "conv") if second is not None else "conv"
    pb = second_packed if second_packed is not None else second.packed()
    if not kw:
        return run_pair2(ctx, first.packed(), srcs, pb, tags=(n0, n1), regress=regress)
    if regress is not None:
        raise ValueError("_pair: regress with an epilogue")
    mid = run_conv(ctx, first.packed(), srcs, tag=n0)
    return run_conv(ctx, pb, [mid], tag=n1, **kw)


def _crop_like(t: torch.Tensor, ref: torch.Tensor) -> torch.Tensor:
    """``t[..., :ref.D, :ref.H, :ref.W]`` (ESMStereo.py:172,177,230) as a strided view."""
    idx = (slice(None), slice(None)) + tuple(slice(0, n) for n in ref.shape[2:])
    return t[idx]


class _Hourglass(nn.Module):
    """Shared 3-level encoder/decoder of ``aggregation`` (3-D) and ``up_refinement`` (2-D)."""

    is_3d = False

    def _build(self, c_in: int, c1: int, c2: int, c3: int, cat0: int, cat1: int) -> None:
        d3 = self.is_3d
        self.conv1 = nn.Sequential(_bc(c_in, c1, d3, s=2), _bc(c1, c1, d3))
        self.conv2 = nn.Sequential(_bc(c1, c2, d3, s=2), _bc(c2, c2, d3))
        self.conv3 = nn.Sequential(_bc(c2, c3, d3, s=2), _bc(c3, c3, d3))
        self.conv3_up = _up(c3, c2, d3)
        self.conv2_up = _up(c2, c1, d3)
        self.conv1_up = _up(c1, 1, d3, last=True)
        self.agg_0 = nn.Sequential(_bc(cat0, c2, d3, k=1, p=0), _bc(c2, c2, d3))
        self.agg_1 = nn.Sequential(_bc(cat1, c1, d3, k=1, p=0), _bc(c1, c1, d3))

    def _emit(self, ctx: Ctx, x: Optional[torch.Tensor], extra0: Sequence[torch.Tensor] = (),
              extra1: Sequence[torch.Tensor] = (), crop1: bool = True, c10: Optional[torch.Tensor] = None,
              c11: Optional[torch.Tensor] = None, **last) -> torch.Tensor:
        """``c10``: conv1[0]'s output, when the caller fused that layer into its producer (then ``x`` is
        not read); ``c11``: conv1's output (both of its layers fused into the producer)."""
        if c11 is not None:
            c1 = c11
        elif c10 is not None:
            c1 = self.conv1[1].emit(ctx, [c10])
        else:
            c1 = _pair(ctx, self.conv1[0], [x], self.conv1[1])
        c2 = _pair(ctx, self.conv2[0], [c1], self.conv2[1])
        c3 = _pair(ctx, self.conv3[0], [c2], self.conv3[1])
        a0 = self._up_agg(ctx, self.conv3_up, c3, self.agg_0, [c2, *extra0], True)
        a1 = self._up_agg(ctx, self.conv2_up, a0, self.agg_1, [c1, *extra1], crop1)
        return self.conv1_up.emit(ctx, [a1], **last)

    def _up_agg(self, ctx: Ctx, up: BasicConv, x: torch.Tensor, agg: nn.Sequential, skip: Sequence[torch.Tensor],
                crop: bool) -> torch.Tensor:
        """``agg(cat(crop(up(x)), *skip))`` (ESMStereo.py:163-177, 226-234): the transposed conv and agg[0] in
        one launch where conv_up1.hip has the shape (and agg[0] + agg[1] would not run as one pair), else
        the transposed conv, then agg[0] + agg[1] (one pair2 launch or two)."""
        ref = skip[0]
        if not crop and tuple(2 * v for v in x.shape[2:]) != tuple(ref.shape[2:]):
            # the reference concat at ESMStereo.py:234 does not crop and raises here
            raise RuntimeError(f"Sizes of tensors must match except in dimension 1. Expected size "
                               f"{2 * x.shape[2]} but got size {ref.shape[2]} for tensor number 1 in the list.")
        pa, pb = up.packed(), agg[0].packed()
        u_shape = tuple(2 * v for v in x.shape[2:])
        n0 = getattr(up, "_esm_name", "convT")
        n1 = getattr(agg[0], "_esm_name", "agg.0")
        paired = pair2_auto(pb, agg[1].packed(), [ref]) if not self.is_3d else False
        # the fork-join: up_refinement's image features (the last source) as a partial sum on the side branch
        fork = FORK_ENABLED and not self.is_3d and len(skip) == 2 and agg[0].use_bn and int(skip[0].shape[1]) % 4 == 0
        if fork:
            cm = pa.cout + int(skip[0].shape[1])
            p_side, p_main = forked_packs(agg[0], agg[0].conv, agg[0].bn, ACT_GELU if agg[0].gelu else ACT_NONE, cm,
                                          int(skip[1].shape[1]))
            if convt_1x1_supported(pa, p_main, skip[:1]) and all(u >= r for u, r in zip(u_shape, ref.shape[2:])):
                part = run_side_partial(ctx, p_side, skip[1], n1, cm)
                h = run_convt_1x1(ctx, pa, [x], p_main, skip[:1], tags=(n0, n1), pre=part)
                ctx.meta[-1]["split"] = (0, cm)
                return agg[1].emit(ctx, [h])
            u = _crop_like(up.emit(ctx, [x]), ref)
            part = run_side_partial(ctx, p_side, skip[1], n1, cm)
            h = run_conv(ctx, p_main, [u, skip[0]], pre=part, tag=n1)
            ctx.meta[-1].update(layer=n1, split=(0, cm))
            return agg[1].emit(ctx, [h])
        if convt_1x1_supported(pa, pb, skip) and all(u >= r for u, r in zip(u_shape, ref.shape[2:])) and \
                (CONVT1X1_PAIRED or not paired):
            h = run_convt_1x1(ctx, pa, [x], pb, skip, tags=(n0, n1))
            return agg[1].emit(ctx, [h])
        u = _crop_like(up.emit(ctx, [x]), ref)
        return _pair(ctx, agg[0], [u, *skip], agg[1])


class aggregation(_Hourglass):
    """3-D cost aggregation hourglass (reference models/ESMStereo.py:129-182).

    Channel ladder c, c+a, c+2a, c+4a (L: 8 -> 24 -> 40 -> 72).  Output depth is 2*ceil(D/2).
    """

    is_3d = True

    def __init__(self, in_channels: int, add_channel: int) -> None:
        super().__init__()
        c0, a = in_channels, add_channel
        self._build(c0, c0 + a, c0 + 2 * a, c0 + 4 * a, 2 * (c0 + 2 * a), 2 * (c0 + a))

    def emit(self, ctx: Ctx, x: torch.Tensor, **last) -> torch.Tensor:
        return self._emit(ctx, x, crop1=True, **last)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        return eager_emit(x.device, self.emit, x)


class up_refinement(_Hourglass):
    """2-D disparity refinement hourglass (reference models/ESMStereo.py:185-239)."""

    is_3d = False

    def __init__(self, C: int, cf1: int, cf2: int) -> None:
        super().__init__()
        self._build(1, C, C, C, 2 * C + cf1, 2 * C + cf2)

    def emit(self, ctx: Ctx, disp: Optional[torch.Tensor], left_f1x: torch.Tensor, left_f2x: torch.Tensor,
             c10: Optional[torch.Tensor] = None, c11: Optional[torch.Tensor] = None, **last) -> torch.Tensor:
        return self._emit(ctx, disp, extra0=[left_f1x], extra1=[left_f2x], crop1=False, c10=c10, c11=c11, **last)

    def forward(self, disp: torch.Tensor, left_f1x: torch.Tensor, left_f2x: torch.Tensor) -> torch.Tensor:
        return eager_emit(disp.device, self.emit, disp, left_f1x, left_f2x)


# ----------------------------------------------------------------------------- ESM upsampler


def _dm(c: int) -> nn.Sequential:
    """Disparity-feature stack: k5 p1, k3 p1, k3 p1, k1 p1 (reference ESMStereo.py:250-253)."""
    return nn.Sequential(_bc(1, c, False, k=5), _bc(c, c, False), _bc(c, c, False), _bc(c, c, False, k=1, p=1))


def _spx(cin: int, c: int, cout: int) -> nn.Sequential:
    return nn.Sequential(_bc(cin, c, False), nn.Conv2d(c, cout, 3, 1, 1, bias=False), nn.BatchNorm2d(cout), nn.GELU())


def _shuffle_up(nf: int, r: int) -> nn.Sequential:
    return nn.Sequential(nn.Conv2d(nf, nf * r * r, 1, 1, 0), nn.PixelShuffle(r), nn.SiLU(inplace=True))


class _ESMUpsampler(nn.Module):
    """Generic ESM cascade: each stage refines the previous disparity by a factor r.

    ``STAGES`` rows: (tag, C, cat_channels, spx_out, r, cf1, cf2, cat_src, ref_src_a, ref_src_b) where
    the *_src entries index the forward()'s feature arguments.
    """

    STAGES: Tuple = ()
    N_FEATS = 8

    def __init__(self) -> None:
        super().__init__()
        nf = self.N_FEATS
        for i, (tag, C, catc, spx_out, r, cf1, cf2, *_src) in enumerate(self.STAGES):
            setattr(self, f"dm{tag}", _dm(C))
            setattr(self, f"spx_{tag}", _spx(C + catc, C, spx_out))
            if i == 0:
                self.to_feat = nn.Conv2d(C, nf, 3, 1, 1, bias=False)
                self.blocks = nn.Sequential(*[FMBlock(nf, 7, 2) for _ in range(2)])
            setattr(self, f"upsampling{tag[:-1]}", _shuffle_up(nf, r))
            setattr(self, f"tail{tag}", nn.Conv2d(nf, 1, 3, 1, 1))
            setattr(self, f"ref{tag}", up_refinement(C, cf1, cf2))
        self._esm = None

    def _packed(self):
        tok = param_token(*self.modules())
        if self._esm is None or self._esm[0] != tok:
            p = {"to_feat": pack_conv(self.to_feat)}
            for (tag, _C, _cat, _spx, r, *_r) in self.STAGES:
                spx = getattr(self, f"spx_{tag}")
                p[f"spx1_{tag}"] = pack_conv(spx[1], spx[2], ACT_GELU)
                p[f"up_{tag}"] = pack_shuffle_tail(getattr(self, f"upsampling{tag[:-1]}")[0], getattr(self, f"tail{tag}"),
                                                   r)
            self._esm = (tok, p)
        return self._esm[1]

    def emit(self, ctx: Ctx, feats: Sequence[torch.Tensor], init_disp: torch.Tensor, final_scale: float = 1.0,
             scaled_copies: Optional[float] = None, init_cost: Optional[torch.Tensor] = None) -> List[torch.Tensor]:
        """Returns [finest, ..., coarsest] like the reference forward.  ``final_scale`` scales the
        finest output in its store; with ``scaled_copies`` every coarser output also gets a
        scaled second copy (returned second): ([outputs], [scaled copies]).  ``init_cost``: ``init_disp`` is
        still to be computed as disparity_regression of this [B, D, H, W] cost (by the first pair)."""
        p = self._packed()
        me = getattr(self, "_esm_name", "upsample")
        prev = init_disp
        outs, copies = [], []
        n = len(self.STAGES)
        for i, (tag, C, catc, spx_out, r, cf1, cf2, cat_i, ra, rb) in enumerate(self.STAGES):
            dm = getattr(self, f"dm{tag}")
            d = _pair(ctx, dm[0], [prev], dm[1], regress=init_cost if i == 0 else None)
            d = _pair(ctx, dm[2], [d], dm[3])
            spx = getattr(self, f"spx_{tag}")
            ref = getattr(self, f"ref{tag}")
            # spx_<t>[1] inside the row-form head + ref conv launch where it fits (stages after the first;
            # the first one's c feeds to_feat and the FMBlocks), else the pair / two launches
            pre = None
            paired = pair2_auto(spx[0].packed(), p[f"spx1_{tag}"], [d, feats[cat_i]])
            if i > 0 and not paired and \
                    shuffle_conv_pre_supported(p[f"up_{tag}"], ref.conv1[0].packed(), p[f"spx1_{tag}"]) and \
                    shuffle_conv_supported(p[f"up_{tag}"], ref.conv1[0].packed(), d):
                c = self._spx0(ctx, spx[0], d, feats[cat_i])
                pre = p[f"spx1_{tag}"]
            elif not paired:
                c = run_conv(ctx, p[f"spx1_{tag}"], [self._spx0(ctx, spx[0], d, feats[cat_i])],
                             tag=f"{getattr(spx[0], '_esm_name', 'spx.0')[:-2]}.1")
            else:
                c = _pair(ctx, spx[0], [d, feats[cat_i]], spx[1], p[f"spx1_{tag}"])
            x = c
            if i == 0:
                x = run_conv(ctx, p["to_feat"], [x], tag=f"{me}.to_feat")
                for blk in self.blocks:
                    x = blk.emit(ctx, x)
            # upsampling (1x1 -> PixelShuffle -> SiLU) + tail (3x3 -> 1): one launch, with the refinement
            # hourglass's first conv fused behind it where the kernel has the shape
            c10 = c11 = None
            if pre is not None and SC11_ENABLED:  # ... and the refinement's conv1[1] too (the whole conv1)
                c11 = run_shuffle_conv(ctx, x, p[f"up_{tag}"], ref.conv1[0].packed(), pre=pre, conv2=ref.conv1[1].packed(),
                                       tag=f"{me}.spx_{tag}.1+upsampling{tag[:-1]}+tail{tag}+ref{tag}.conv1")
                x = None
            elif pre is not None:
                c10 = run_shuffle_conv(ctx, x, p[f"up_{tag}"], ref.conv1[0].packed(), pre=pre,
                                       tag=f"{me}.spx_{tag}.1+upsampling{tag[:-1]}+tail{tag}+ref{tag}.conv1.0")
                x = None
            elif shuffle_conv_supported(p[f"up_{tag}"], ref.conv1[0].packed(), x):
                c10 = run_shuffle_conv(ctx, x, p[f"up_{tag}"], ref.conv1[0].packed(),
                                       tag=f"{me}.upsampling{tag[:-1]}+tail{tag}+ref{tag}.conv1.0")
                x = None
            else:
                x = run_shuffle_tail(ctx, x, p[f"up_{tag}"], tag=f"{me}.upsampling{tag[:-1]}+tail{tag}")
            last = i == n - 1
            epi = dict(up=prev, up_f=r, post_scale=final_scale if last else 1.0)
            if scaled_copies is not None and not last:
                B, _, H, W = prev.shape
                r_ = p[f"up_{tag}"].r
                cp = ctx.empty(B, 1, H * r_, W * r_)
                epi.update(out2=cp, post_scale2=scaled_copies)
                copies.append(cp)
            prev = ref.emit(ctx, x, feats[ra], feats[rb], c10=c10, c11=c11, **epi)
            outs.append(prev)
        outs.reverse()
        copies.reverse()
        return (outs, copies) if scaled_copies is not None else outs

    def _spx0(self, ctx: Ctx, spx0: BasicConv, d: torch.Tensor, feat: torch.Tensor) -> torch.Tensor:
        """spx_<t>[0](cat(d, feat)) (ESMStereo.py:488, 501): with the fork-join, feat's part of the 3x3 sum runs on
        the plan's side branch (it depends on the backbone features only) and the chain's conv covers d's
        channels from it; else one conv over the concat."""
        name = getattr(spx0, "_esm_name", "spx.0")
        if FORK_ENABLED and spx0.use_bn and int(d.shape[1]) % 4 == 0:
            return run_conv_forked(ctx, spx0, spx0.conv, spx0.bn, ACT_GELU if spx0.gelu else ACT_NONE, [d], feat,
                                   tag=name)
        return run_conv(ctx, spx0.packed(), [d, feat], tag=name)

    def forward(self, *args: torch.Tensor) -> Tuple[torch.Tensor, ...]:
        *feats, init = args
        return tuple(eager_emit(init.device, self.emit, feats, init))


class upsample4(_ESMUpsampler):
    """ESMStereo-L upsampler, two x2 stages (reference models/ESMStereo.py:242-318).
    forward(left_f1x, left_f2x, left_f4x, init_disp) -> (x4 disparity, x2 disparity)."""

    N_FEATS = 16
    STAGES = (("2x", 32, 48, 32, 2, 96, 48, 1, 0, 1),
              ("4x", 32, 32, 16, 2, 48, 32, 2, 1, 2))


class upsample8(_ESMUpsampler):
    """ESMStereo-M upsampler, three x2 stages (reference models/ESMStereo.py:320-428).
    forward(left_f2x, left_f4x, left_f8x, stem_f2, init_disp) -> (x8, x4, x2)."""

    N_FEATS = 8
    STAGES = (("2x", 16, 96, 16, 2, 240, 96, 1, 0, 1),
              ("4x", 16, 24, 8, 2, 96, 24, 2, 1, 2),
              ("8x", 16, 32, 8, 2, 24, 32, 3, 2, 3))


class upsample16(_ESMUpsampler):
    """ESMStereo-S upsampler, two x4 stages (reference models/ESMStereo.py:430-509).
    forward(left_f1x, left_f2x, left_f4x, left_f8x, init_disp) -> (x16, x4)."""

    N_FEATS = 8
    STAGES = (("2x", 16, 32, 16, 4, 32, 32, 1, 1, 0),
              ("4x", 16, 24, 8, 4, 24, 24, 2, 2, 3))
