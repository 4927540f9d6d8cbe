"""Host side of the HIP hot path: weight packing, launch descriptors, eager/plan contexts.

Every op here goes to ``libesmstereo_amd.so`` through ``_lib`` (ctypes over the C ABI of
``include/esmstereo_amd.h``).  Nothing computes on the CPU and there is no PyTorch
fallback: CPU tensors, non-fp32 tensors or a missing library raise.

A :class:`Ctx` either launches each op immediately on the current torch stream (``eager``)
or appends it to a native ``esm_plan`` (``plan``) whose launch list is later replayed —
eagerly or as one hipGraph.  The module classes (blocks.py, mixer.py, model.py) describe the
reference's forward passes once, against a Ctx, so the eager nn.Module forward and the
compiled whole-hot-path plan run the very same kernels with the very same fusions.
"""
from __future__ import annotations

import contextlib
import ctypes
import json
import math
import os
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence, Tuple

import torch

from . import _lib
from ._lib import (ACT_GELU, ACT_NONE, ACT_RELU, ACT_RELU6, ACT_SIGMOID, ACT_SILU, EsmConfDesc, EsmConvDesc, EsmShuffleConvDesc,
                   EsmShuffleTailDesc, EsmSmixDesc, check, lib)

__all__ = ["Ctx", "PackedConv", "pack_conv", "run_conv", "run_smix", "run_fmnet", "run_shuffle_tail", "pack_shuffle_tail",
           "ACT_NONE", "ACT_GELU", "ACT_SILU", "ACT_RELU", "ACT_SIGMOID", "ACT_RELU6", "run_dwconv", "cached_pack", "run_convt_1x1",
           "convt_1x1_supported", "pack_conv_split", "run_conv_forked",
           "forked_packs", "run_side_partial"]


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


# Dry emission (Ctx(dry=True)): the launch list is walked with shape-only ``meta`` tensors, nothing is
# submitted and no device memory is touched.  It sizes a plan's arena before the real emission and
# lets CPU tests read every op's algorithmic cost (ctx.meta).  While one is active IN THIS THREAD, meta
# tensors pass the device checks below; they can never reach a kernel, because a dry Ctx submits nothing.
# The depth is thread-local: a dry emission in one thread never relaxes another thread's eager checks
# (ADVICE r4).
_DRY = threading.local()


def _dry_depth() -> int:
    return getattr(_DRY, "depth", 0)


def require_device(t: torch.Tensor, what: str) -> None:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{what}: expected a torch.Tensor")
    if t.device.type == "meta" and _dry_depth():
        return
    if t.device.type != "cuda":
        raise RuntimeError(f"{what}: esmstereo_amd runs on ROCm devices only (got a {t.device.type} tensor); "
                           "there is no CPU path")
    if t.dtype != torch.float32:
        raise TypeError(f"{what}: expected float32, got {t.dtype}")
    if t.dim() > 0 and t.stride(-1) != 1:
        raise ValueError(f"{what}: innermost dimension must be contiguous")


def require_on(dev: torch.device, what: str, *ts: Optional[torch.Tensor]) -> None:
    """Every pointer a kernel dereferences must live on the launch device (a host or
    other-device pointer would fault the GPU, so this is checked on the host first)."""
    dry = _dry_depth()
    for t in ts:
        if t is None:
            continue
        if dry and (t.device.type == "meta" or torch.device(dev).type == "meta"):
            continue  # a dry emission submits nothing (its buffers are shape-only)
        if t.device != dev or t.dtype != torch.float32:
            raise RuntimeError(f"{what}: tensor on {t.device} ({t.dtype}); expected float32 on {dev} "
                               "(move the module to the input's device)")


# ----------------------------------------------------------------------------- packing


@dataclass
class PackedConv:
    """A conv layer ready for ``esm_conv_f32``: packed weights + folded BN/bias epilogue."""

    w: torch.Tensor
    scale: Optional[torch.Tensor]
    shift: Optional[torch.Tensor]
    act: int
    nd: int
    k: int
    stride: int
    pad: int
    transposed: bool
    cin: int
    cout: int
    cin_pad: int
    cout_pad: int


def _bits(v: int, n: int) -> Tuple[int, ...]:
    return tuple((v >> (n - 1 - i)) & 1 for i in range(n))


def pack_weight(W: torch.Tensor, transposed: bool) -> Tuple[torch.Tensor, int, int]:
    """Pack a Conv/ConvTranspose weight for the implicit-GEMM kernel.

    normal      W[cout][cin][k..]  -> P[tap][cin_pad][cout_pad]
    transposed  W[cin][cout][4..]  -> P[cls][tap][cin_pad][cout_pad]; for output parity q and
                tap t of a dim the kernel index is 1 - q + 2t (input index m + q - t).
    """
    W = W.detach().to(torch.float32)
    nd = W.dim() - 2
    if not transposed:
        cout, cin = W.shape[:2]
        taps = int(W[0, 0].numel())
        cin_pad, cout_pad = _rup(cin, 16), _rup(cout, 32)
        P = W.new_zeros(taps, cin_pad, cout_pad)
        P[:, :cin, :cout] = W.reshape(cout, cin, taps).permute(2, 1, 0)
        return P.contiguous(), cin_pad, cout_pad
    cin, cout = W.shape[:2]
    if any(s != 4 for s in W.shape[2:]):
        raise ValueError("transposed conv: only kernel 4 is supported")
    cin_pad, cout_pad = _rup(cin, 16), _rup(cout, 32)
    n = 2 ** nd
    P = W.new_zeros(n, n, cin_pad, cout_pad)
    for cls in range(n):
        q = _bits(cls, nd)
        for tap in range(n):
            t = _bits(tap, nd)
            k = tuple(1 - qi + 2 * ti for qi, ti in zip(q, t))
            P[cls, tap, :cin, :cout] = W[(slice(None), slice(None)) + k]
    return P.contiguous(), cin_pad, cout_pad


def bn_affine(bn: torch.nn.Module) -> Tuple[torch.Tensor, torch.Tensor]:
    """Eval BatchNorm as y = x*alpha + beta with alpha = w/sqrt(var+eps), beta = b - mean*alpha."""
    invstd = 1.0 / torch.sqrt(bn.running_var.detach().float() + bn.eps)
    alpha = invstd * bn.weight.detach().float()
    beta = bn.bias.detach().float() - bn.running_mean.detach().float() * alpha
    return alpha.contiguous(), beta.contiguous()


def pack_conv(conv: torch.nn.Module, bn: Optional[torch.nn.Module] = None, act: int = ACT_NONE) -> PackedConv:
    transposed = isinstance(conv, (torch.nn.ConvTranspose2d, torch.nn.ConvTranspose3d))
    W = conv.weight
    nd = W.dim() - 2
    ks = set(conv.kernel_size)
    ss = set(conv.stride)
    ps = set(conv.padding) if not isinstance(conv.padding, str) else {-1}
    if len(ks) != 1 or len(ss) != 1 or len(ps) != 1 or set(conv.dilation) != {1} or conv.groups != 1:
        raise ValueError(f"unsupported conv geometry {conv}")
    P, cin_pad, cout_pad = pack_weight(W, transposed)
    scale = shift = None
    if bn is not None:
        scale, shift = bn_affine(bn)
        if conv.bias is not None:  # conv bias feeds BN: (x + cb)*a + b = x*a + (cb*a + b)
            shift = (conv.bias.detach().float() * scale + shift).contiguous()
    elif conv.bias is not None:
        shift = conv.bias.detach().float().contiguous()
    cin, cout = (W.shape[0], W.shape[1]) if transposed else (W.shape[1], W.shape[0])
    return PackedConv(P, scale, shift, act, nd, ks.pop(), ss.pop(), ps.pop(), transposed, int(cin), int(cout),
                      cin_pad, cout_pad)


def pack_conv_split(conv: torch.nn.Module, bn: Optional[torch.nn.Module], act: int, lo: int, hi: int) -> PackedConv:
    """The input channels [lo, hi) of a 2-D Conv2d as their own conv (a partial sum of the layer): with ``bn``
    the folded BN + ``act`` epilogue (the part that finishes the layer), else a plain sum (no bias, no act)."""
    W = conv.weight
    if isinstance(conv, (torch.nn.ConvTranspose2d, torch.nn.ConvTranspose3d)) or W.dim() != 4 or conv.bias is not None:
        raise ValueError("pack_conv_split: a bias-free Conv2d")
    P, cin_pad, cout_pad = pack_weight(W[:, lo:hi], False)
    scale = shift = None
    if bn is not None:
        scale, shift = bn_affine(bn)
    k, s_, p_ = conv.kernel_size[0], conv.stride[0], conv.padding[0]
    return PackedConv(P, scale, shift, act if bn is not None else ACT_NONE, 2, k, s_, p_, False, hi - lo,
                      int(W.shape[0]), cin_pad, cout_pad)


def cached_pack(owner: torch.nn.Module, name: str, mods: Sequence[Optional[torch.nn.Module]], build, *extra):
    """``build()`` (packed weights of ``mods``) cached on ``owner`` under ``name`` until a tensor of ``mods`` is
    replaced, moved or edited in place (param_token)."""
    tok = param_token(*mods) + tuple(extra)
    packs = owner.__dict__.setdefault("_esm_packs", {})
    c = packs.get(name)
    if c is None or c[0] != tok:
        c = packs[name] = (tok, build())
    return c[1]


def param_token(*mods: torch.nn.Module) -> Tuple:
    """Cheap identity of a module's own tensors (storage + in-place version)."""
    tok = []
    for m in mods:
        if m is None:
            continue
        for t in list(m.parameters(recurse=False)) + list(m.buffers(recurse=False)):
            tok.append((t.data_ptr(), t._version, t.device.index))
    return tuple(tok)


# ----------------------------------------------------------------------------- context


def _spans(*ts) -> List[Tuple[int, int]]:
    """(base address, bytes) of the allocations behind tensors: the unit the plan's
    dependency analysis works in (a view depends on its whole allocation)."""
    out = []
    for t in ts:
        if t is not None:
            st = t.untyped_storage()
            out.append((st.data_ptr(), st.nbytes()))
    return out


class Ctx:
    """Where ops go: launched now (``plan=False``), appended to a native plan (``plan=True``), or
    only recorded (``dry=True``: shape-only ``meta`` buffers, nothing submitted; use as a context
    manager, ``with Ctx(dev, dry=True) as ctx: ...``)."""

    def __init__(self, device: torch.device, plan: bool = False, dry: bool = False):
        self.device = torch.device(device)
        self.dry = bool(dry)
        self.plan = lib.esm_plan_create() if plan and not dry else None
        if plan and not dry and not self.plan:
            raise RuntimeError("esm_plan_create failed")
        self.keep: List[object] = []  # tensors (and ctypes descs) that must outlive the plan
        # one entry per launch-list op: name, kernel family, algorithmic flops / HBM bytes
        self.meta: List[dict] = []
        self.stream = None if (plan or dry) else ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
        self._arena: Optional[torch.Tensor] = None
        self._arena_off = 0
        self.arena_bytes = 0   # bytes carved out of the arena (256-B granules)
        self.arena_chunks = 0
        self.num_ops = 0       # ops submitted (or, dry, recorded)
        self._branch = 0       # 1 inside side(): ops go to the plan's side branch
        self._join_next = False

    def __enter__(self) -> "Ctx":
        if self.dry:
            _DRY.depth = _dry_depth() + 1
        return self

    def __exit__(self, *exc) -> None:
        if self.dry:
            _DRY.depth = _dry_depth() - 1

    def _submit(self) -> bool:
        """Count one op; True when it is to be handed to the library (not a dry emission).  The op's meta entry
        (the last one appended) records its branch."""
        self.num_ops += 1
        if self.dry and not _dry_depth():
            raise RuntimeError("a dry Ctx must be used as a context manager")
        if self.meta:
            self.meta[-1]["branch"] = self._branch
        return not self.dry

    @contextlib.contextmanager
    def side(self):
        """Ops emitted inside run on the plan's side branch (esm_plan_set_branch): they overlap the main chain
        and may read only the plan's inputs (eagerly they run in place, on the current stream)."""
        prev, self._branch = self._branch, 1
        try:
            yield self
        finally:
            self._branch = prev

    def join_next(self) -> None:
        """The next main-chain op waits for every side op emitted before it (esm_plan_set_join)."""
        self._join_next = True

    def _placed(self, idx: int) -> int:
        """Branch / join attributes of the op just added to the native plan at ``idx``."""
        if self._branch:
            check(lib.esm_plan_set_branch(self.plan, idx, 1), "plan_set_branch")
        elif self._join_next:
            check(lib.esm_plan_set_join(self.plan, idx, 1), "plan_set_join")
            self._join_next = False
        return idx

    def launch(self, graph: bool = True, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Run a plan context's launch list (as a hipGraph by default) on the current stream."""
        if not self.plan:
            raise RuntimeError("launch() needs a plan context")
        s = ctypes.c_void_p((stream or torch.cuda.current_stream(self.device)).cuda_stream)
        if graph:
            if not getattr(self, "_graph_ready", False):
                check(lib.esm_plan_graph_build(self.plan, s), "graph_build")
                self._graph_ready = True
            check(lib.esm_plan_graph_launch(self.plan, s), "graph_launch")
        else:
            check(lib.esm_plan_run(self.plan, s), "plan_run")

    def close(self) -> None:
        if self.plan:
            lib.esm_plan_destroy(self.plan)
            self.plan = None
        self.keep.clear()

    def __del__(self):  # pragma: no cover - interpreter teardown order
        try:
            self.close()
        except Exception:
            pass

    ARENA_CHUNK = 256 << 20  # bytes: the largest arena chunk (every buffer of an S / M plan at KITTI size)
    ARENA_FIRST = 16 << 20   # the first chunk; each further chunk doubles, up to ARENA_CHUNK

    def empty(self, *shape: int) -> torch.Tensor:
        """A float32 buffer.  A plan's buffers are carved (256-B aligned) out of arena chunks (one
        chunk sized by a dry emission for a compiled plan; 16 MiB doubling chunks otherwise), so a
        launch list's buffers sit together and come from one allocation."""
        if self.dry:  # the plan's arena accounting, with shape-only buffers
            n = math.prod(shape)
            self.arena_bytes += (4 * n + 255) // 256 * 256
            return torch.empty(shape, device="meta", dtype=torch.float32)
        if not self.plan:
            return torch.empty(shape, device=self.device, dtype=torch.float32)
        n = math.prod(shape)
        nb = (4 * n + 255) // 256 * 256
        if self._arena is None or self._arena_off + nb > self._tail_lo():
            size = self.ARENA_FIRST if self._arena is None else min(self.ARENA_CHUNK, 2 * self._arena.numel())
            self._arena = torch.empty(max(size, nb), device=self.device, dtype=torch.uint8)
            self._arena_off = 0
            self._tail = None
            self.arena_chunks += 1
            self.keep.append(self._arena)
        t = self._arena[self._arena_off:self._arena_off + 4 * n].view(torch.float32).view(shape)
        self._arena_off += nb
        self.arena_bytes += nb
        return t

    def empty_tail(self, *shape: int) -> torch.Tensor:
        """A float32 buffer carved from the END of the current arena chunk (which must have room):
        the hot path's backbone-feature inputs go there, next to the upsampler's buffers (the last
        ones the plan allocates from the front) that they are concatenated with."""
        n = math.prod(shape)
        nb = (4 * n + 255) // 256 * 256
        if self.dry or not self.plan or self._arena is None or self._arena_off + nb > self._tail_lo():
            return self.empty(*shape)
        self._tail = self._tail_lo() - nb
        self.arena_bytes += nb
        return self._arena[self._tail:self._tail + 4 * n].view(torch.float32).view(shape)

    def _tail_lo(self) -> int:
        t = getattr(self, "_tail", None)
        return self._arena.numel() if t is None or t > self._arena.numel() else t

    def hold(self, *objs) -> None:
        if self.plan:
            self.keep.extend(o for o in objs if o is not None)

    # --- op submission
    def conv(self, d: EsmConvDesc) -> None:
        if not self._submit():
            return
        if self.plan:
            self._placed(check(lib.esm_plan_add_conv(self.plan, ctypes.byref(d)), "plan_add_conv"))
        else:
            check(lib.esm_conv_f32(ctypes.byref(d), self.stream), "conv")

    def smix(self, d: EsmSmixDesc) -> None:
        if not self._submit():
            return
        if self.plan:
            self._placed(check(lib.esm_plan_add_smix(self.plan, ctypes.byref(d)), "plan_add_smix"))
        else:
            check(lib.esm_smix_f32(ctypes.byref(d), self.stream), "smix")

    def fmnet(self, d) -> None:
        if not self._submit():
            return
        if self.plan:
            self._placed(check(lib.esm_plan_add_fmnet(self.plan, ctypes.byref(d)), "plan_add_fmnet"))
        else:
            check(lib.esm_fmnet_f32(ctypes.byref(d), self.stream), "fmnet")

    def shuffle_tail(self, d: EsmShuffleTailDesc) -> None:
        if not self._submit():
            return
        if self.plan:
            self._placed(check(lib.esm_plan_add_shuffle_tail(self.plan, ctypes.byref(d)), "plan_add_shuffle_tail"))
        else:
            check(lib.esm_shuffle_tail_f32(ctypes.byref(d), self.stream), "shuffle_tail")

    def pair2(self, a: EsmConvDesc, b: EsmConvDesc) -> None:
        if not self._submit():
            return
        if self.plan:
            self._placed(check(lib.esm_plan_add_conv_pair2(self.plan, ctypes.byref(a), ctypes.byref(b)), "plan_add_conv_pair2"))
        else:
            check(lib.esm_conv_pair2_f32(ctypes.byref(a), ctypes.byref(b), self.stream), "conv_pair2")

    def shuffle_conv(self, d: EsmShuffleConvDesc) -> None:
        if not self._submit():
            return
        if self.plan:
            self._placed(check(lib.esm_plan_add_shuffle_conv(self.plan, ctypes.byref(d)), "plan_add_shuffle_conv"))
        else:
            check(lib.esm_shuffle_conv_f32(ctypes.byref(d), self.stream), "shuffle_conv")

    def dwconv(self, d) -> None:
        if not self._submit():
            return
        if self.plan:
            raise RuntimeError("dwconv: the backbone's depthwise convs run eagerly (no plan op)")
        check(lib.esm_dwconv_f32(ctypes.byref(d), self.stream), "dwconv")

    def gwc(self, L, R, att, V, B, C, H, W, D, G) -> None:
        self.meta.append(dict(name="gwc_volume", kind="gwc", flops=2 * B * C * D * H * W,
                              bytes=4 * B * (2 * C * H * W + G * D * H * W + (G * H * W if att is not None else 0)),
                              reads=_spans(L, R, att), writes=_spans(V)))
        a = att.data_ptr() if att is not None else None
        if not self._submit():
            return
        if self.plan:
            self.hold(L, R, att, V)
            self._placed(check(lib.esm_plan_add_gwc(self.plan, L.data_ptr(), R.data_ptr(), a, V.data_ptr(), B, C, H, W, D, G), "gwc"))
        else:
            check(lib.esm_gwc_volume_f32(L.data_ptr(), R.data_ptr(), a, V.data_ptr(), B, C, H, W, D, G, self.stream),
                  "gwc")

    def gwc_stem(self, d: EsmConvDesc, L, R, C: int, G: int) -> None:
        if not self._submit():
            return
        if self.plan:
            self.hold(L, R)
            self._placed(check(lib.esm_plan_add_gwc_stem(self.plan, ctypes.byref(d), L.data_ptr(), R.data_ptr(), C, G), "gwc_stem"))
        else:
            check(lib.esm_gwc_stem_f32(ctypes.byref(d), L.data_ptr(), R.data_ptr(), C, G, self.stream), "gwc_stem")

    def concat(self, L, R, V, B, C, H, W, D) -> None:
        self.meta.append(dict(name="concat_volume", kind="concat", flops=0,
                              bytes=4 * B * (2 * C * H * W + 2 * C * D * H * W), reads=_spans(L, R), writes=_spans(V)))
        if not self._submit():
            return
        if self.plan:
            self.hold(L, R, V)
            self._placed(check(lib.esm_plan_add_concat(self.plan, L.data_ptr(), R.data_ptr(), V.data_ptr(), B, C, H, W, D), "concat"))
        else:
            check(lib.esm_concat_volume_f32(L.data_ptr(), R.data_ptr(), V.data_ptr(), B, C, H, W, D, self.stream),
                  "concat")

    def normcorr(self, L, R, V, work, B, C, H, W, D) -> None:
        self.meta.append(dict(name="normcorr_volume", kind="normcorr", flops=2 * B * C * D * H * W,
                              bytes=4 * B * (2 * C * H * W + D * H * W), reads=_spans(L, R), writes=_spans(V, work)))
        if not self._submit():
            return
        if self.plan:
            self.hold(L, R, V, work)
            self._placed(check(lib.esm_plan_add_normcorr(self.plan, L.data_ptr(), R.data_ptr(), V.data_ptr(), work.data_ptr(), B, C,
                                            H, W, D), "normcorr"))
        else:
            check(lib.esm_normcorr_volume_f32(L.data_ptr(), R.data_ptr(), V.data_ptr(), work.data_ptr(), B, C, H, W, D,
                                              self.stream), "normcorr")

    def conf(self, op: int, xs: Sequence[Optional[torch.Tensor]], out: torch.Tensor, B: int, C: int, D: int, H: int,
             W: int, name: str = "conf") -> None:
        """One per-pixel stage of the confidence head (esm_conf_f32; contiguous NCHW operands)."""
        for t in list(xs) + [out]:
            if t is not None and not t.is_contiguous():
                raise ValueError(f"{name}: confidence-head operands must be contiguous")
        d = EsmConfDesc()
        d.op, d.B, d.C, d.D, d.H, d.W = op, B, C, D, H, W
        for i, t in enumerate(xs):
            d.x[i] = t.data_ptr() if t is not None else None
        d.out = out.data_ptr()
        nbytes = 4 * (sum(t.numel() for t in xs if t is not None) + out.numel())
        self.meta.append(dict(name=name, kind="conf", flops=0, bytes=nbytes, reads=_spans(*xs), writes=_spans(out)))
        if not self._submit():
            return
        if self.plan:
            self.hold(*xs, out)
            self._placed(check(lib.esm_plan_add_conf(self.plan, ctypes.byref(d)), name))
        else:
            check(lib.esm_conf_f32(ctypes.byref(d), self.stream), name)

    def regression(self, kind, cost, out, B, D, H, W, samples=None, k: int = 2) -> None:
        """kind 0: disparity_regression; kind 1: regression_topk with ``k`` (2 in the hot path)."""
        name = "disparity_regression" if kind == 0 else f"regression_topk{k}"
        self.meta.append(dict(name=name, kind="regression", flops=2 * B * D * H * W, bytes=4 * B * (D + 1) * H * W,
                              reads=_spans(cost, samples), writes=_spans(out)))
        if not self._submit():
            return
        if self.plan:
            if samples is not None or (kind and k != 2):
                raise ValueError("plan regression: disparity_regression or regression_topk(k=2) over arange(D)")
            self.hold(cost, out)
            self._placed(check(lib.esm_plan_add_regression(self.plan, kind, cost.data_ptr(), out.data_ptr(), B, D, H, W),
                  "regression"))
        elif kind == 0:
            check(lib.esm_disp_regression_f32(cost.data_ptr(), out.data_ptr(), B, D, H, W, self.stream), "regression")
        else:
            s = samples.data_ptr() if samples is not None else None
            check(lib.esm_topk_regression_f32(cost.data_ptr(), s, out.data_ptr(), B, D, H, W, int(k), self.stream),
                  "regression_topk")


def eager_emit(device: torch.device, fn, *args, **kw):
    """Run ``fn(ctx, *args, **kw)`` (a module's ``emit``) eagerly: every launch is submitted on the
    current stream as it is emitted, its buffers from PyTorch's allocator."""
    return fn(Ctx(device), *args, **kw)


# ----------------------------------------------------------------------------- ops


# A/B switches.  The kernel-selection knobs below are read from the environment only when ESM_AB=1 (the
# measurement scripts set it); otherwise every knob takes its measured default, so a caller's environment
# can never select a combination of forms the GPU suite did not run.
AB = os.environ.get("ESM_AB") == "1"


def _ab(name: str, default: str) -> str:
    return os.environ.get(name, default) if AB else default


# Measured tile choices (scripts/autotune.py on MI355X, in the hot path's own launch sequence):
# XCD-slab tile order (esm_conv_desc.hint bit 30, esm_shuffle_tail_desc.flags bit 0; common.h xcd_block)
# for launches whose input or output map (B x D x H x W) has at least this many pixels: there it takes
# the memory-side bytes of the full-resolution convs from 2.1-2.9x the algorithmic to 1.05-1.13x at no
# cost in step time, while on the hourglasses' small maps it measured 0.1-1 us slower per launch
# (round 3, S-K, rocprofv3 op maps; every launch remapped: +10 us on the S-K step).
HINT_XCD_SLAB = 1 << 30
XCD_SLAB_MIN_PIX = int(_ab("ESM_XCD_SLAB_MIN_PIX", "65536"))
# the same order on 3-D volumes (B x D x H x W output or input voxels over the threshold); ESM_XCD_SLAB_3D=0
# leaves every 3-D launch in the default order (A/B measurements)
XCD_SLAB_3D = _ab("ESM_XCD_SLAB_3D", "1") != "0"
# 3-D launches with >= 32 input channels from this many output voxels: the S / M `group_stem` (12x24x78),
# whose 32-channel input each workgroup re-reads with its halo: 15.8 -> 7.8 MB per launch, step time
# unchanged (round 4, two alternations, profiles/r04_xcd_group_stem_SK.txt)
XCD_SLAB_MIN_VOX_WIDE = int(_ab("ESM_XCD_SLAB_MIN_VOX_WIDE", "16384"))
# per-launch hints by op name, "name=0x...,name=0x..." (A/B measurements; replaces the tuned / automatic choice)
HINT_SET: Dict[str, int] = {k: int(v, 0) for k, v in (t.split("=") for t in _ab("ESM_HINT_SET", "").split(",") if t)}
# launches (by name, comma-separated) given the slab order whatever their size (A/B measurements)
XCD_SLAB_OPS = tuple(t for t in _ab("ESM_XCD_SLAB_OPS", "").split(",") if t)

# shape key -> esm_conv_desc.hint.  Layers not in the table take the library's automatic rules.
_TUNED_PATH = _ab("ESM_TUNED", "") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "tuned_hints.json")
TUNED_HINTS: Dict[str, int] = {}
if os.path.exists(_TUNED_PATH) and not _ab("ESM_NO_TUNED", ""):
    with open(_TUNED_PATH) as _f:
        TUNED_HINTS = {k: int(v) for k, v in json.load(_f).get("hints", {}).items()}


def conv_key(d: EsmConvDesc, nd: int) -> str:
    """Shape key of a conv launch: geometry, source channel split, batch, input extent and the
    epilogue features that change the store path."""
    cins = "+".join(str(d.src[i].C) for i in range(d.nsrc))
    return (f"{nd}d{'T' if d.transposed else ''} k{d.kh}s{d.stride}p{d.ph} {cins}->{d.Cout} B{d.B} "
            f"{d.Di}x{d.Hi}x{d.Wi} sh{d.shuffle}{'u' if d.up else ''}{'m' if d.mul else ''}"
            f"{'r' if d.res else ''}{'2' if d.out2 else ''}")


def _spatial(t: torch.Tensor, nd: int) -> Tuple[int, int, int]:
    if nd == 3:
        return int(t.shape[2]), int(t.shape[3]), int(t.shape[4])
    return 1, int(t.shape[2]), int(t.shape[3])


def run_conv(ctx: Ctx, pc: PackedConv, srcs: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None, *,
             mul: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None,
             up: Optional[torch.Tensor] = None, up_f: int = 0, post_scale: float = 1.0, shuffle: int = 1,
             out2: Optional[torch.Tensor] = None, post_scale2: float = 1.0, tag: str = "conv",
             hint: int = 0, pre: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One implicit-GEMM conv launch; ``srcs`` are concatenated along channels (each may be a
    cropped view), the epilogue applies BN/bias, activation, ``*mul``, ``+res``,
    ``+bilinear(up)``, ``*post_scale`` and an optional PixelShuffle(``shuffle``).  ``pre`` (2-D,
    [B, Cout, Ho, Wo]): a partial conv sum over other input channels, added before BN."""
    d, out, meta = _conv_desc(ctx, pc, srcs, out, mul=mul, res=res, up=up, up_f=up_f, post_scale=post_scale,
                              shuffle=shuffle, out2=out2, post_scale2=post_scale2, tag=tag, hint=hint, pre=pre)
    ctx.meta.append(meta)
    ctx.conv(d)
    return out


def _conv_desc(ctx: Ctx, pc: PackedConv, srcs: Sequence[torch.Tensor], out: Optional[torch.Tensor] = None, *,
               mul: Optional[torch.Tensor] = None, res: Optional[torch.Tensor] = None,
               up: Optional[torch.Tensor] = None, up_f: int = 0, post_scale: float = 1.0, shuffle: int = 1,
               out2: Optional[torch.Tensor] = None, post_scale2: float = 1.0, tag: str = "conv",
               hint: int = 0, alloc_out: bool = True, pre: Optional[torch.Tensor] = None):
    """Validate one conv and build its ``esm_conv_desc``; returns (desc, output tensor, meta).
    ``alloc_out=False`` (the first conv of a fused pair) leaves the output pointer NULL."""
    nd = pc.nd
    d = EsmConvDesc()
    if not srcs or len(srcs) > _lib.MAX_SRC:
        raise ValueError("conv: 1..3 sources")
    x0 = srcs[0]
    if x0.dim() != nd + 2:
        raise ValueError(f"conv: expected a {nd + 2}-D input, got shape {tuple(x0.shape)}")
    dev = x0.device
    B = int(x0.shape[0])
    Di, Hi, Wi = _spatial(x0, nd)
    cin = 0
    for i, s in enumerate(srcs):
        require_device(s, "conv input")
        if s.dim() != nd + 2 or int(s.shape[0]) != B or _spatial(s, nd) != (Di, Hi, Wi):
            # torch.cat of mismatching tensors raises RuntimeError in the reference
            raise RuntimeError(f"Sizes of tensors must match except in dimension 1 (conv sources "
                               f"{[tuple(t.shape) for t in srcs]})")
        st = s.stride()
        d.src[i].ptr = s.data_ptr()
        d.src[i].C = int(s.shape[1])
        d.src[i].sb, d.src[i].sc = st[0], st[1]
        d.src[i].sd = st[2] if nd == 3 else 0
        d.src[i].sh = st[-2]
        cin += int(s.shape[1])
    if cin != pc.cin:
        raise RuntimeError(f"conv: input has {cin} channels, layer expects {pc.cin}")
    require_on(dev, "conv", *srcs, pc.w, pc.scale, pc.shift, out, mul, res, up, out2, pre)
    d.nsrc = max(1, len(srcs))
    d.B, d.Cin = B, cin
    d.Di, d.Hi, d.Wi = Di, Hi, Wi
    k, s, p = pc.k, pc.stride, pc.pad
    if pc.transposed:
        if (k, s, p) != (4, 2, 1):
            raise ValueError("transposed conv: only k=4 s=2 p=1")
        Do, Ho, Wo = (2 * Di if nd == 3 else 1), 2 * Hi, 2 * Wi
    else:
        Ho, Wo = (Hi + 2 * p - k) // s + 1, (Wi + 2 * p - k) // s + 1
        Do = (Di + 2 * p - k) // s + 1 if nd == 3 else 1
    if min(Do, Ho, Wo) <= 0:
        raise RuntimeError(f"conv: empty output for input extent {(B, cin, Di, Hi, Wi)}")
    d.Do, d.Ho, d.Wo = Do, Ho, Wo
    d.kd = k if nd == 3 else 1
    d.kh = d.kw = k
    d.stride, d.transposed = s, int(pc.transposed)
    d.pd = p if nd == 3 else 0
    d.ph = d.pw = p
    d.Cout, d.cin_pad, d.cout_pad = pc.cout, pc.cin_pad, pc.cout_pad
    d.w = pc.w.data_ptr()
    d.scale = pc.scale.data_ptr() if pc.scale is not None else None
    d.shift = pc.shift.data_ptr() if pc.shift is not None else None
    d.act = pc.act
    r = int(shuffle)
    d.shuffle = r
    if out is None and alloc_out:
        if r > 1:
            if pc.cout % (r * r):
                raise ValueError("pixel shuffle: Cout not divisible by r^2")
            out = ctx.empty(B, pc.cout // (r * r), Ho * r, Wo * r)
        else:
            out = ctx.empty(B, pc.cout, Do, Ho, Wo) if nd == 3 else ctx.empty(B, pc.cout, Ho, Wo)
    if out is not None:
        require_device(out, "conv output")
        require_on(dev, "conv output", out)
        ost = out.stride()
        d.out = out.data_ptr()
        d.ob, d.oc = ost[0], ost[1]
        d.od = ost[2] if nd == 3 else 0
        d.oh = ost[-2]
    if mul is not None:
        require_device(mul, "conv mul")
        d.mul = mul.data_ptr()
        d.mb, d.mc, d.mh = mul.stride(0), mul.stride(1), mul.stride(-2)
    if res is not None:
        require_device(res, "conv residual")
        if out is None or tuple(res.shape) != tuple(out.shape):
            raise ValueError("conv: residual shape must match the output")
        rs = res.stride()
        d.res = res.data_ptr()
        d.rb, d.rc = rs[0], rs[1]
        d.rd = rs[2] if nd == 3 else 0
        d.rh = rs[-2]
    if up is not None:
        require_device(up, "conv bilinear source")
        d.up = up.data_ptr()
        d.up_h, d.up_w, d.up_f = int(up.shape[-2]), int(up.shape[-1]), int(up_f)
        d.ub, d.uh = up.stride(0), up.stride(-2)
        if d.up_h * up_f != Ho or d.up_w * up_f != Wo:
            raise ValueError("conv: bilinear source extent x factor must equal the output extent")
    d.post_scale = float(post_scale)
    if out2 is not None:
        require_device(out2, "conv out2")
        if out2.stride() != out.stride() or out2.shape != out.shape:
            raise ValueError("conv: out2 must have the output's shape and strides")
        d.out2 = out2.data_ptr()
        d.post_scale2 = float(post_scale2)
    if pre is not None:
        require_device(pre, "conv pre")
        if nd != 2 or pc.transposed or shuffle > 1 or up is not None or tuple(pre.shape) != (B, pc.cout, Ho, Wo):
            raise ValueError("conv: a partial sum (pre) is [B, Cout, Ho, Wo] of a 2-D, non-transposed conv")
        d.pre = pre.data_ptr()
        d.prb, d.prc, d.prh = pre.stride(0), pre.stride(1), pre.stride(2)
    key = conv_key(d, nd)  # (a conv with `pre` shares the tuned form of its shape)
    d.hint = int(hint) if hint else HINT_SET.get(tag, TUNED_HINTS.get(key, 0))
    if (B * max(Di * Hi * Wi, Do * Ho * Wo) >= XCD_SLAB_MIN_PIX and (nd == 2 or XCD_SLAB_3D)) or \
            (nd == 3 and XCD_SLAB_3D and pc.cin >= 32 and B * Do * Ho * Wo >= XCD_SLAB_MIN_VOX_WIDE) or \
            tag in XCD_SLAB_OPS:
        d.hint |= HINT_XCD_SLAB
    ctx.hold(pc.w, pc.scale, pc.shift, *srcs, out, out2, mul, res, up, pre)
    taps = pc.k ** nd
    if pc.transposed:  # algorithmic ConvT count: every input voxel meets every kernel tap
        macs = B * Di * Hi * Wi * pc.cin * pc.cout * taps
    else:
        macs = B * Do * Ho * Wo * pc.cin * pc.cout * taps
    in_bytes = 4 * B * cin * Di * Hi * Wi
    out_bytes = 4 * B * pc.cout * Do * Ho * Wo * (2 if out2 is not None else 1)
    extra = 4 * sum(t.numel() for t in (res, mul, up, pre) if t is not None)
    w_bytes = 4 * pc.cin * pc.cout * taps  # the layer's weights (the packed slab's padding is not algorithmic)
    meta = dict(name=tag, kind="conv", flops=2 * macs, bytes=in_bytes + out_bytes + extra + w_bytes,
                shape=f"{'T' if pc.transposed else ''}{nd}d k{pc.k}s{pc.stride} {cin}->{pc.cout} "
                      f"in {Di}x{Hi}x{Wi} out {Do}x{Ho}x{Wo}",
                reads=_spans(*srcs, mul, res, up, pre), writes=_spans(out, out2), key=key, hint=d.hint)
    return d, out, meta


# The gwc volume and group_stem as one launch (esm_gwc_stem_f32, gwc_stem.hip) on the volumes the LDS-tiled
# stem takes (ESMStereo-L / -M); ESM_GWC_STEM=0 keeps the two launches (A/B measurements)
GWC_STEM_ENABLED = _ab("ESM_GWC_STEM", "1") != "0"
# its composite weights staged in LDS per k-step (round 5; gwc_stem.hip hint bit 28) instead of loaded into
# registers (round 6): A/B knob
GWC_STEM_WLDS = _ab("ESM_GWC_STEM_WLDS", "0") == "1"


def gwc_stem_supported(pc: PackedConv, L: torch.Tensor, G: int, D: int, att) -> bool:
    """Python mirror of gwc_stem.hip gwc_stem_check, restricted to where the fused form replaces the tiled
    stem (tile3_auto: >= 2^16 output voxels; the S volumes keep their row-streaming stem)."""
    if att is not None or pc.nd != 3 or pc.transposed or (pc.k, pc.stride, pc.pad) != (3, 1, 1):
        return False
    B, C, H, W = (int(v) for v in L.shape)
    if pc.cin != G or G % 4 or C != 2 * G or pc.cout > 8 or not L.is_contiguous():
        return False
    return B * D * H * W >= (1 << 16) and 4 * C * H * W < (1 << 30) and 4 * pc.cout * D * H * W < (1 << 30)


def run_gwc_stem(ctx: Ctx, pc: PackedConv, L: torch.Tensor, R: torch.Tensor, G: int, D: int,
                 tag: str = "gwc_volume+group_stem", hint: int = 0) -> torch.Tensor:
    """``group_stem(build_gwc_volume(L, R, D, G))`` (models/submodule.py:151-161, models/ESMStereo.py:703-704)
    as one launch: the volume is formed in LDS per k-step and never written (bit-identical to the two
    launches with the tiled stem)."""
    B, C, H, W = (int(v) for v in L.shape)
    if tuple(R.shape) != (B, C, H, W) or not R.is_contiguous() or not L.is_contiguous():
        raise ValueError("gwc_stem: L and R must be contiguous tensors of one shape")
    virt = L.as_strided((B, G, D, H, W), (0, 0, 0, 0, 1))  # the volume's geometry only, never read
    d, out, meta = _conv_desc(ctx, pc, [virt], tag=tag, hint=hint)
    # tile order and rows per wave (+ the weight form when the caller passes a hint); a standalone stem's
    # tuned form bits do not apply
    d.hint &= HINT_XCD_SLAB | (3 << 26) | ((1 << 28) if hint else 0)
    if GWC_STEM_WLDS:
        d.hint |= 1 << 28
    vol_flops = 2 * B * C * D * H * W
    meta.update(kind="gwc_stem", flops=meta["flops"] + vol_flops,
                bytes=4 * B * 2 * C * H * W + 4 * B * pc.cout * D * H * W + 4 * pc.cin * pc.cout * 27,
                reads=_spans(L, R), shape=f"gwc G{G} D{D} + " + meta["shape"])
    ctx.meta.append(meta)
    ctx.gwc_stem(d, L, R, C, G)
    return out


# Two consecutive 2-D BasicConvs as one launch (esm_conv_pair2_f32, conv_pair2.hip); ESM_PAIR2=0
# runs every pair as two launches (A/B measurements)
PAIR2_ENABLED = _ab("ESM_PAIR2", "1") != "0"


def pair2_supported(pa: PackedConv, pb: PackedConv, srcs: Sequence[torch.Tensor]) -> bool:
    """Python mirror of conv_pair2.hip pair2_ok (plus the on/off switch)."""
    if not PAIR2_ENABLED or pa.nd != 2 or pb.nd != 2 or pa.transposed or pb.transposed:
        return False
    if pa.cout != 16 or pb.cin != 16 or pb.cout > 16 or pa.cin > (64 if pa.k == 1 else 48):
        return False
    if not ((pa.k == 3 and pa.stride in (1, 2)) or (pa.k in (1, 5) and pa.stride == 1)):
        return False
    if pb.stride != 1 or pb.k not in (1, 3) or pa.act != ACT_GELU or pb.act != ACT_GELU:
        return False
    return len(srcs) == 1 or all(int(t.shape[1]) % 4 == 0 for t in srcs)


def pair2_auto(pa: PackedConv, pb: PackedConv, srcs: Sequence[torch.Tensor]) -> bool:
    """Where the hot path takes the fused pair.  Measured in the S-K chain (rocprofv3, round 3): the pair
    wins where convA is light -- the dm stacks' 5x5 single-channel head (dm.0 + dm.1: 6.1 vs 9.1 us at
    24x78, 10.6 vs 11.5 at 96x312), a 1x1 convB (dm.2 + dm.3: 6.5 vs 9.2, 7.6 vs 10.4), the 1x1 agg.0 of
    the small refinement levels (7.6 vs 9.0, 8.7 vs 9.3) -- and loses where convA's recomputed halo is
    heavy work for one workgroup (spx 48 / 40 -> 16 3x3: 13.7 vs 9.1, 32.9 vs 14.8; the 192x624 agg_1:
    48.4 vs 20.5; the stride-2 conv pairs at 96x312 and up: 24.2 vs 13.7; the refinement's 1 -> 16
    stride-2 head + conv1.1 at 192x624: 23.6 vs 19.0)."""
    if not pair2_supported(pa, pb, srcs):
        return False
    B = int(srcs[0].shape[0])
    Ho = (int(srcs[0].shape[2]) + 2 * pa.pad - pa.k) // pa.stride + 1
    Wo = (int(srcs[0].shape[3]) + 2 * pa.pad - pa.k) // pa.stride + 1
    light = pa.cin * pa.k * pa.k
    return pb.k == 1 or (light <= 25 and pa.stride == 1) or (pa.k == 1 and B * Ho * Wo <= 8192)


# A ConvTranspose BasicConv + crop + cat + the 1x1 BasicConv after it as one launch (esm_convt_1x1_f32,
# conv_up1.hip): the hourglasses' conv3_up -> agg_0[0] and conv2_up -> agg_1[0].  ESM_CONVT_1X1=0 keeps two
# launches; ESM_CONVT_1X1_PAIRED=0 keeps agg_N[0] + agg_N[1] as one pair2 launch where pair2_auto takes it
# (A/B measurements).  S-K, three alternations on one box (round 6): 0.3202-0.3214 ms with two launches,
# 0.3127-0.3140 fused where agg_N[0] is not paired, 0.3077-0.3080 fused everywhere (the default)
CONVT1X1_ENABLED = _ab("ESM_CONVT_1X1", "1") != "0"
CONVT1X1_PAIRED = _ab("ESM_CONVT_1X1_PAIRED", "1") == "1"
CONVT1X1_MAX_EXTRA = 48  # extra channels the fused kernels instantiate (conv_up1.hip kUp1MaxXB * 4)

# Fork-join (round 6): the image-feature part of the upsampler stages' concat convs (spx_<t>[0] over
# cat(disparity features, left features), models/ESMStereo.py:488, 501) as a partial sum on the plan's side
# branch, overlapping the cost-volume -> hourglass chain; the chain's conv then reads only the disparity
# features and starts from that sum (esm_conv_desc.pre).  Measured (round 6, three alternations on one box) and
# NOT taken: a captured hipGraph with a second branch costs far more per replay than the overlap saves (S-K
# 0.4166-0.4204 ms forked vs 0.3069-0.3072 ms as one chain; L-K B = 4 4.885-4.896 vs 4.685-4.696 ms), so the
# default keeps one conv over the concat; ESM_FORK=1 forks (A/B; the kernels and the plan's branch API stay
# tested: test_conv_partial_sum, test_convt_1x1_partial_sum, test_plan_side_branch_matches_eager).
FORK_ENABLED = _ab("ESM_FORK", "0") == "1"


def convt_1x1_supported(pa: PackedConv, pb: PackedConv, extra: Sequence[torch.Tensor]) -> bool:
    """Python mirror of conv_up1.h up1_check (plus the on/off switch)."""
    if not CONVT1X1_ENABLED or not pa.transposed or pb.transposed or (pa.k, pa.stride, pa.pad) != (4, 2, 1):
        return False
    # 17-32 couts on either side: the two-tile 3-D tiled form, <= 32 extra channels (round 6: L's conv2_up + agg_1.0)
    wide = pa.cout > 16 or pb.cout > 16
    if pa.act != ACT_GELU or pa.scale is None or pa.shift is None or pa.cout > 32 or pa.cout % 4:
        return False
    if (pb.k, pb.stride, pb.pad) != (1, 1, 0) or pb.act != ACT_GELU or pb.cout > 32 or pb.nd != pa.nd:
        return False
    if wide and (pa.nd != 3 or pa.cout < 2):
        return False
    cx = sum(int(t.shape[1]) for t in extra)
    return 1 <= len(extra) <= 2 and all(int(t.shape[1]) % 4 == 0 for t in extra) and \
        4 <= cx <= (32 if wide else CONVT1X1_MAX_EXTRA)


def run_convt_1x1(ctx: Ctx, pa: PackedConv, srcs: Sequence[torch.Tensor], pb: PackedConv, extra: Sequence[torch.Tensor],
                  tags: Tuple[str, str] = ("convT", "conv1x1"), pre: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``pb(cat(crop(pa(srcs)), *extra))`` (models/ESMStereo.py:163-175, 221-234) as one launch: the transposed
    conv's output is cropped to the extra sources' extent and never written."""
    da, _, ma = _conv_desc(ctx, pa, srcs, tag=tags[0], alloc_out=False)
    nd = pa.nd
    e0 = extra[0]
    geo = (int(e0.shape[0]), pa.cout) + tuple(int(v) for v in e0.shape[2:])
    virt = srcs[0].as_strided(geo, (0,) * (len(geo) - 1) + (1,))  # the crop's geometry only, never read
    db, out, mb = _conv_desc(ctx, pb, [virt, *extra], tag=tags[1], pre=pre)
    db.hint = 0
    B = int(e0.shape[0])
    vox = math.prod(int(v) for v in e0.shape[2:])
    full = 4 * B * pa.cout * int(da.Ho) * int(da.Wo) * (int(da.Do) if nd == 3 else 1)
    name = f"{tags[0]}+{'.'.join(tags[1].split('.')[-2:])}"
    ctx.meta.append(dict(name=name, kind="conv_up1", flops=ma["flops"] + mb["flops"],
                         bytes=ma["bytes"] - full + mb["bytes"] - 4 * B * pa.cout * vox,
                         shape=f"{ma['shape']} + {mb['shape']}", reads=ma["reads"] + _spans(*extra), writes=mb["writes"],
                         key=ma["key"] + " | " + mb["key"], hint=da.hint))
    if ctx._submit():
        if ctx.plan:
            ctx._placed(check(lib.esm_plan_add_convt_1x1(ctx.plan, ctypes.byref(da), ctypes.byref(db)), "plan_add_convt_1x1"))
        else:
            check(lib.esm_convt_1x1_f32(ctypes.byref(da), ctypes.byref(db), ctx.stream), "convt_1x1")
    return out


def forked_packs(owner: torch.nn.Module, conv: torch.nn.Module, bn: Optional[torch.nn.Module], act: int, cm: int,
                 cs: int) -> Tuple[PackedConv, PackedConv]:
    """(side part: input channels [cm, cm + cs), plain sum; main part: [0, cm) + BN + act) of a 2-D conv."""
    def build():
        return (pack_conv_split(conv, None, act, cm, cm + cs), pack_conv_split(conv, bn, act, 0, cm))
    return cached_pack(owner, f"fork{cm}", [conv, bn], build)


def run_side_partial(ctx: Ctx, p_side: PackedConv, side: torch.Tensor, tag: str, cm: int) -> torch.Tensor:
    """The side channels' partial sum on the plan's side branch (it reads only plan inputs); the next main op
    joins it."""
    with ctx.side():
        part = run_conv(ctx, p_side, [side], tag=tag + "[side]")
    ctx.meta[-1].update(layer=tag, split=(cm, cm + p_side.cin))
    ctx.join_next()
    return part


def run_conv_forked(ctx: Ctx, owner: torch.nn.Module, conv: torch.nn.Module, bn: Optional[torch.nn.Module], act: int,
                    main: Sequence[torch.Tensor], side: torch.Tensor, tag: str = "conv") -> torch.Tensor:
    """``conv(cat(*main, side))`` + BN + ``act`` as two launches: the ``side`` channels' partial sum on the plan's
    side branch, then the ``main`` channels' conv starting from it (esm_conv_desc.pre), on the main chain behind
    a join.  fp32 reassociation of the channel sum only (tests hold it to 1e-5)."""
    cm = sum(int(t.shape[1]) for t in main)
    p_side, p_main = forked_packs(owner, conv, bn, act, cm, int(side.shape[1]))
    part = run_side_partial(ctx, p_side, side, tag, cm)
    out = run_conv(ctx, p_main, list(main), pre=part, tag=tag)
    ctx.meta[-1].update(layer=tag, split=(0, cm))
    return out


# the hot path's disparity_regression folded into the upsampler's first pair (conv_pair2.hip hint bit 29):
# one launch less on the S / M chains; ESM_PAIR_REGRESS=0 keeps the separate launch (A/B)
PAIR_REGRESS_ENABLED = _ab("ESM_PAIR_REGRESS", "1") != "0"
# tile rows of the pairs whose first conv's name contains one of the comma-separated substrings (A/B knobs;
# conv_pair2.hip: 2 / 4 / 8 rows, 8 only up to 16 input channels; default: the launcher's choice)
PAIR2_TH = {sel: tuple(x for x in _ab(f"ESM_PAIR2_TH{n}", "").split(",") if x)
            for sel, n in ((1, 2), (2, 4), (3, 8))}
HINT_PAIR_REGRESS = 1 << 29


def run_pair2(ctx: Ctx, pa: PackedConv, srcs: Sequence[torch.Tensor], pb: PackedConv,
              tags: Tuple[str, str] = ("convA", "convB"), force: bool = False,
              regress: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``pb(pa(cat(srcs)))`` (two BasicConvs, BN + GELU each) as one launch where ``pair2_auto`` takes it
    (``force``: wherever supported), else two launches.

    ``regress``: a [B, D, H, W] cost volume whose disparity_regression (models/submodule.py:211-216) is
    ``srcs[0]``, still to be computed: the pair computes it per staged pixel and stores it to ``srcs[0]``
    where the kernel has the shape (5x5 1 -> 16 head, 3x3 convB), else the regression runs first as its
    own launch."""
    take = pair2_supported(pa, pb, srcs) if force else pair2_auto(pa, pb, srcs)
    if regress is not None:
        B_, D_, H_, W_ = (int(v) for v in regress.shape)
        init = srcs[0]
        fuse = (take and PAIR_REGRESS_ENABLED and len(srcs) == 1 and pa.k == 5 and pb.k == 3 and pa.cin == 1
                and regress.stride(3) == 1 and tuple(init.shape) == (B_, 1, H_, W_) and init.stride(3) == 1)
        if not fuse:
            ctx.regression(0, regress, init, B_, D_, H_, W_)
            regress = None
    if not take:
        return run_conv(ctx, pb, [run_conv(ctx, pa, srcs, tag=tags[0])], tag=tags[1])
    da, _, ma = _conv_desc(ctx, pa, srcs, tag=tags[0], alloc_out=False)
    da.hint &= ~HINT_PAIR_REGRESS
    B = int(srcs[0].shape[0])
    geo = (B, pa.cout) + ((int(da.Do),) if pa.nd == 3 else ()) + (int(da.Ho), int(da.Wo))
    virt = srcs[0].as_strided(geo, (0,) * (len(geo) - 1) + (1,))  # geometry only, never read
    db, out, mb = _conv_desc(ctx, pb, [virt], tag=tags[1])
    db.hint &= ~(3 << 26)  # convB's bits 26-27 pick the pair's tile rows (a standalone conv's tuned hint does not)
    for sel, subs in PAIR2_TH.items():
        if any(x in tags[0] for x in subs):
            db.hint |= sel << 26
    mid = 4 * B * pa.cout * int(da.Ho) * int(da.Wo) * (int(da.Do) if pa.nd == 3 else 1)
    name = f"{tags[0]}+{tags[1].rsplit('.', 1)[-1]}"
    flops, byts, reads, writes = ma["flops"] + mb["flops"], ma["bytes"] - mid + mb["bytes"] - mid, ma["reads"], mb["writes"]
    if regress is not None:
        # convA reads the D cost planes instead of the map, and the map is stored once
        require_on(init.device, "pair regression", regress)
        st = regress.stride()
        da.src[0].ptr, da.src[0].C = regress.data_ptr(), D_
        da.src[0].sb, da.src[0].sc, da.src[0].sh = st[0], st[1], st[2]
        da.out = init.data_ptr()
        da.ob, da.oc, da.oh = init.stride(0), init.stride(1), init.stride(2)
        da.hint |= HINT_PAIR_REGRESS
        ctx.hold(regress, init)
        name = "disparity_regression+" + name
        flops += 2 * B_ * D_ * H_ * W_
        byts += 4 * B_ * D_ * H_ * W_
        reads, writes = _spans(regress), writes + _spans(init)
    ctx.meta.append(dict(name=name, kind="conv_pair", flops=flops, bytes=byts, shape=f"pair {ma['shape']} + {mb['shape']}",
                         reads=reads, writes=writes, key=ma["key"] + " | " + mb["key"], hint=0))
    ctx.pair2(da, db)
    return out


def run_dwconv(ctx: Ctx, x: torch.Tensor, w: torch.Tensor, scale: Optional[torch.Tensor], shift: Optional[torch.Tensor],
               k: int, stride: int, pad: int, act: int, tag: str = "dwconv") -> torch.Tensor:
    """Depthwise KxK conv (groups = C) + folded BN + activation (``esm_dwconv_f32``): timm's ``conv_dw -> bn``
    (+ act) of the backbone blocks.  ``w``: [C, K*K] contiguous."""
    if stride <= 0 or k <= 0 or not 0 <= pad < k:
        raise ValueError("dwconv: stride and K must be positive, 0 <= pad < K")
    if x.dim() != 4 or x.stride(3) != 1:
        raise ValueError("dwconv: a [B, C, H, W] input with unit W stride")
    require_device(x, "dwconv input")
    B, C, H, W = (int(v) for v in x.shape)
    Ho, Wo = (H + 2 * pad - k) // stride + 1, (W + 2 * pad - k) // stride + 1
    out = ctx.empty(B, C, Ho, Wo)
    require_on(x.device, "dwconv", x, w, scale, shift, out)
    d = _lib.EsmDwconvDesc()
    d.x, d.xb, d.xc, d.xh = x.data_ptr(), x.stride(0), x.stride(1), x.stride(2)
    d.w = w.data_ptr()
    d.scale = scale.data_ptr() if scale is not None else None
    d.shift = shift.data_ptr() if shift is not None else None
    d.out, d.ob, d.oc, d.oh = out.data_ptr(), out.stride(0), out.stride(1), out.stride(2)
    d.B, d.C, d.H, d.W, d.K, d.stride, d.pad, d.act, d.Ho, d.Wo = B, C, H, W, k, stride, pad, act, Ho, Wo
    ctx.meta.append(dict(name=tag, kind="dwconv", flops=2 * B * C * Ho * Wo * k * k,
                         bytes=4 * (x.numel() + out.numel() + C * k * k), reads=_spans(x), writes=_spans(out)))
    ctx.dwconv(d)
    return out


@dataclass
class SmixStage:
    ln_w: torch.Tensor
    fc0_w: torch.Tensor
    fc0_b: torch.Tensor
    fc2_w: torch.Tensor
    fc2_b: torch.Tensor


def run_smix(ctx: Ctx, x: torch.Tensor, stages: Sequence[SmixStage], *, dw: Optional[Tuple[torch.Tensor, torch.Tensor]] = None,
             res: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None, tag: str = "smix") -> torch.Tensor:
    require_device(x, "smix input")
    if not x.is_contiguous():
        raise ValueError("smix: input must be contiguous")
    B, C, H, W = (int(v) for v in x.shape)
    if out is None:
        out = ctx.empty(B, C, H, W)
    d = EsmSmixDesc()
    d.x, d.out = x.data_ptr(), out.data_ptr()
    if res is not None:
        require_device(res, "smix residual")
        if not res.is_contiguous() or res.shape != x.shape:
            raise ValueError("smix: residual must be contiguous and shaped like the input")
        d.res = res.data_ptr()
    if dw is not None:
        d.dw_w, d.dw_b = dw[0].data_ptr(), dw[1].data_ptr()
        d.dw_k = int(dw[0].shape[-1])
    if len(stages) > _lib.SMIX_MAX_STAGES:
        raise ValueError("smix: at most 2 stages per launch")
    require_on(x.device, "smix", x, out, res, *(dw or ()),
               *[t for st in stages for t in (st.ln_w, st.fc0_w, st.fc0_b, st.fc2_w, st.fc2_b)])
    d.nstages = len(stages)
    for i, st in enumerate(stages):
        d.stage[i].ln_w = st.ln_w.data_ptr()
        d.stage[i].fc0_w, d.stage[i].fc0_b = st.fc0_w.data_ptr(), st.fc0_b.data_ptr()
        d.stage[i].fc2_w, d.stage[i].fc2_b = st.fc2_w.data_ptr(), st.fc2_b.data_ptr()
        ctx.hold(st.ln_w, st.fc0_w, st.fc0_b, st.fc2_w, st.fc2_b)
    d.B, d.C, d.H, d.W = B, C, H, W
    ctx.hold(x, out, res, *(dw or ()))
    npix = B * H * W
    ctx.meta.append(dict(name=tag, kind="smix", flops=npix * (2 * C * C * len(stages) + (2 * C * d.dw_k ** 2 if dw else 0)),
                         bytes=4 * npix * C * (3 if res is not None else 2), shape=f"C{C} {H}x{W} dw{d.dw_k}",
                         reads=_spans(x, res), writes=_spans(out)))
    ctx.smix(d)
    return out


# The whole FMBlock as two launches (esm_fmnet_desc.work, smix.hip fm2a / fm2b) on maps of at least this
# many pixels (B x H x W); smaller maps keep the one-launch form, whose halo recompute is cheap there and
# whose single launch boundary matters (S-K: 24 x 78)
FM2_MIN_PIX = int(_ab("ESM_FM2_MIN_PIX", "16384"))


def run_fmnet(ctx: Ctx, x: torch.Tensor, stages: Sequence[SmixStage], dw0: Tuple[torch.Tensor, torch.Tensor],
              dw1: Tuple[torch.Tensor, torch.Tensor], out: Optional[torch.Tensor] = None,
              tag: str = "fmnet", conv: Optional[Tuple[torch.Tensor, ...]] = None,
              two_launch: Optional[bool] = None) -> torch.Tensor:
    """``FMBlock.net(x) + x`` (shufflemixer.py:129-130) in one launch: stages = SMLayer0.mlp1, .mlp2,
    SMLayer1.mlp1, .mlp2; dw0 / dw1 = the two SMLayers' depthwise convs (weight, bias).  With ``conv`` =
    (conv0 weight [C+16, C, 3, 3], bias, conv2 weight [C, C+16, 1, 1], bias) the whole FMBlock
    (shufflemixer.py:129-131: ``t = net(x) + x; conv(t) + t``) is the one launch, or on large maps
    (``two_launch``; default: B x H x W >= FM2_MIN_PIX) two launches through a scratch buffer."""
    require_device(x, "fmnet input")
    if not x.is_contiguous():
        raise ValueError("fmnet: input must be contiguous")
    if len(stages) != 4:
        raise ValueError("fmnet: four mlp stages")
    B, C, H, W = (int(v) for v in x.shape)
    if out is None:
        out = ctx.empty(B, C, H, W)
    d = _lib.EsmFmnetDesc()
    d.x, d.out = x.data_ptr(), out.data_ptr()
    d.dw_w[0], d.dw_b[0] = dw0[0].data_ptr(), dw0[1].data_ptr()
    d.dw_w[1], d.dw_b[1] = dw1[0].data_ptr(), dw1[1].data_ptr()
    d.dw_k = int(dw0[0].shape[-1])
    if int(dw1[0].shape[-1]) != d.dw_k:
        raise ValueError("fmnet: both SMLayers need the same depthwise kernel")
    require_on(x.device, "fmnet", x, out, *dw0, *dw1,
               *[t for st in stages for t in (st.ln_w, st.fc0_w, st.fc0_b, st.fc2_w, st.fc2_b)])
    for i, st in enumerate(stages):
        d.stage[i].ln_w = st.ln_w.data_ptr()
        d.stage[i].fc0_w, d.stage[i].fc0_b = st.fc0_w.data_ptr(), st.fc0_b.data_ptr()
        d.stage[i].fc2_w, d.stage[i].fc2_b = st.fc2_w.data_ptr(), st.fc2_b.data_ptr()
        ctx.hold(st.ln_w, st.fc0_w, st.fc0_b, st.fc2_w, st.fc2_b)
    d.B, d.C, d.H, d.W = B, C, H, W
    if conv is not None:
        w0, b0, w2, b2 = conv
        hid = int(w0.shape[0])
        if tuple(w0.shape) != (hid, C, 3, 3) or tuple(w2.shape[:2]) != (C, hid) or hid != C + 16:
            raise ValueError("fmnet: FMBlock.conv must be Conv2d(C, C+16, 3) and Conv2d(C+16, C, 1)")
        for t in conv:
            if not t.is_contiguous():
                raise ValueError("fmnet: conv weights must be contiguous")
        require_on(x.device, "fmnet conv", *conv)
        d.conv0_w, d.conv0_b, d.conv2_w, d.conv2_b = (t.data_ptr() for t in conv)
        d.hid = hid
        ctx.hold(*conv)
        if two_launch is None:
            two_launch = B * H * W >= FM2_MIN_PIX
        if two_launch:
            work = ctx.empty(B, C, H, W)
            d.work = work.data_ptr()
            ctx.hold(work)
    ctx.hold(x, out, *dw0, *dw1)
    npix = B * H * W
    # algorithmic flops per pixel: four split-point MLPs (C/2 -> C -> C/2: 2 * C * C), two depthwise
    # KxK convs, and with the fused FMBlock.conv the 3x3 C -> hid and the 1x1 hid -> C
    flops = 2 * C * C * 4 + 2 * 2 * C * d.dw_k ** 2 + (2 * d.hid * C * 9 + 2 * C * d.hid if conv is not None else 0)
    ctx.meta.append(dict(name=tag, kind="fmnet", flops=npix * flops,
                         bytes=4 * npix * C * 2 + 4 * (sum(int(t.numel()) for t in conv) if conv is not None else 0),
                         shape=f"C{C} {H}x{W} dw{d.dw_k} x2" + (f" +conv{d.hid}" if conv is not None else ""),
                         reads=_spans(x), writes=_spans(out), launches=2 if d.work else 1))
    ctx.fmnet(d)
    return out


@dataclass
class PackedShuffleTail:
    """``upsampling`` (Conv2d 1x1 + PixelShuffle + SiLU) and ``tail`` (Conv2d 3x3 -> 1) weights."""

    up_w: torch.Tensor
    up_b: torch.Tensor
    tail_w: torch.Tensor
    tail_b: Optional[torch.Tensor]
    nf: int
    r: int


def pack_shuffle_tail(up: torch.nn.Conv2d, tail: torch.nn.Conv2d, r: int) -> PackedShuffleTail:
    nf = int(tail.weight.shape[1])
    if tuple(up.weight.shape) != (nf * r * r, nf, 1, 1) or up.bias is None:
        raise ValueError("shuffle_tail: upsampling must be Conv2d(nf, nf*r*r, 1) with bias")
    if tuple(tail.weight.shape) != (1, nf, 3, 3) or tuple(tail.padding) != (1, 1) or tuple(tail.stride) != (1, 1):
        raise ValueError("shuffle_tail: tail must be Conv2d(nf, 1, 3, 1, 1)")
    return PackedShuffleTail(up.weight.detach().float().reshape(nf * r * r, nf).contiguous(),
                             up.bias.detach().float().contiguous(),
                             tail.weight.detach().float().reshape(nf, 3, 3).contiguous(),
                             tail.bias.detach().float().contiguous() if tail.bias is not None else None, nf, int(r))


def run_shuffle_tail(ctx: Ctx, x: torch.Tensor, p: PackedShuffleTail, out: Optional[torch.Tensor] = None,
                     tag: str = "shuffle_tail", form: int = 0) -> torch.Tensor:
    """``tail(SiLU(PixelShuffle(r)(up(x))))`` as one launch (``esm_shuffle_tail_f32``): the
    ``upsampling`` + ``tail`` pair of the ESM upsamplers (models/ESMStereo.py:264-271,301-302).
    ``form`` (nf 8, r 4): 0 automatic, 1 window form, 2 / 3 the row form with 4 / 8 rows per workgroup."""
    require_device(x, "shuffle_tail input")
    B, nf, H, W = (int(v) for v in x.shape)
    r = p.r
    if nf != p.nf:
        raise RuntimeError(f"shuffle_tail: input has {nf} channels, layer expects {p.nf}")
    if out is None:
        out = ctx.empty(B, 1, H * r, W * r)
    require_device(out, "shuffle_tail output")
    if tuple(out.shape) != (B, 1, H * r, W * r):
        raise ValueError("shuffle_tail: output must be [B, 1, r*H, r*W]")
    require_on(x.device, "shuffle_tail", x, out, p.up_w, p.up_b, p.tail_w, p.tail_b)
    d = EsmShuffleTailDesc()
    d.x = x.data_ptr()
    d.xb, d.xc, d.xh = x.stride(0), x.stride(1), x.stride(2)
    d.up_w, d.up_b, d.tail_w = p.up_w.data_ptr(), p.up_b.data_ptr(), p.tail_w.data_ptr()
    d.tail_b = p.tail_b.data_ptr() if p.tail_b is not None else None
    d.out = out.data_ptr()
    d.ob, d.oh = out.stride(0), out.stride(2)
    d.B, d.nf, d.H, d.W, d.r = B, nf, H, W, r
    npix = B * H * W * r * r
    d.flags = (1 if npix >= XCD_SLAB_MIN_PIX else 0) | (int(form) & 3) << 1
    ctx.hold(x, out, p.up_w, p.up_b, p.tail_w, p.tail_b)
    # upsampling: the 1x1 nf -> nf*r^2 on H x W = nf^2 MACs per full-resolution pixel; tail: 3x3 nf -> 1
    ctx.meta.append(dict(name=tag, kind="shuffle_tail", flops=2 * npix * nf * (nf + 9),
                         bytes=4 * (B * nf * H * W + npix), shape=f"nf{nf} r{r} in {H}x{W} out {H * r}x{W * r}",
                         reads=_spans(x), writes=_spans(out)))
    ctx.shuffle_tail(d)
    return out


# tail(upsampling(x)) and the refinement's first conv in one launch (esm_shuffle_conv_f32);
# ESM_SHUFFLE_CONV=0 runs them as two launches (A/B measurements)
SHUFFLE_CONV_ENABLED = _ab("ESM_SHUFFLE_CONV", "1") != "0"
# largest low-resolution input (B * H * W) the window form is used on.  Round 3: faster than the two launches
# at S-K's 2x stage (24x78 in: 8.4 vs 10.5 us), slower at the 4x stage (96x312 in: 23.2 vs 20.8 us).  The
# row form (shuffle_conv4_kernel, nf 8, r 4, C 16 only; round 4) has no cap: it won at the 4x stage.  Heads
# without a row form (L's nf 16) keep the cap (at L-K B=4 the fused window form took 145.8 us
# against 116.3 + 26.8 us as two launches).
SHUFFLE_CONV_MAX_PIX = int(_ab("ESM_SHUFFLE_CONV_MAXPIX", "8192"))


def shuffle_conv_supported(p: PackedShuffleTail, conv: PackedConv, x: Optional[torch.Tensor] = None) -> bool:
    row_form = (p.nf, p.r, conv.cout) == (8, 4, 16)
    if x is not None and not row_form and int(x.shape[0]) * int(x.shape[2]) * int(x.shape[3]) > SHUFFLE_CONV_MAX_PIX:
        return False
    return SHUFFLE_CONV_ENABLED and (p.nf, p.r, conv.cout) in ((8, 4, 16), (8, 2, 16), (16, 2, 32), (16, 4, 32)) and \
        conv.nd == 2 and not conv.transposed and (conv.k, conv.stride, conv.pad, conv.cin) == (3, 2, 1, 1) and \
        conv.act == ACT_GELU


# the (nf 8, r 4, C 16) head + conv form with the pre-conv (the 4x stage) where the caller leaves the choice to the
# library (A/B knob: 2 shuffle_conv4_kernel, 3 shuffle_conv5_kernel; 0 = the library's rule)
SC_FORM = int(_ab("ESM_SC_FORM", "0"))
# the upsampler stage's spx_<t>[1] computed inside the row-form shuffle_conv launch (ESM_SHUFFLE_PRE=0: its own
# launch, A/B measurements)
SHUFFLE_PRE_ENABLED = _ab("ESM_SHUFFLE_PRE", "1") != "0"


# the refinement's conv1[1] inside the same launch as well (esm_shuffle_conv_desc.w2, the whole conv1 of the 4x
# stage in one launch; ESM_SC11=0: conv1[1] as its own launch, A/B measurements)
SC11_ENABLED = _ab("ESM_SC11", "1") != "0"
# tile of that launch (esm_shuffle_tail_desc.flags bits 3-4; A/B knob): 0 = 4 low-res rows on 8 waves, two
# workgroups per CU (round 6, the default); 1 = 8 rows on 8 waves (round 5); 2 = 4 rows on 4 waves
SC11_TILE = int(_ab("ESM_SC11_TILE", "1"))


def shuffle_conv_pre_supported(p: PackedShuffleTail, conv: PackedConv, pre: PackedConv) -> bool:
    """Whether ``pre`` (BasicConv(Cp <= 16, nf, 3, 1, 1), BN + GELU) can run inside the row-form launch."""
    return SHUFFLE_PRE_ENABLED and shuffle_conv_supported(p, conv) and (p.nf, p.r, conv.cout) == (8, 4, 16) and \
        pre.nd == 2 and not pre.transposed and (pre.k, pre.stride, pre.pad) == (3, 1, 1) and pre.cin <= 16 and \
        pre.cout == p.nf and pre.act == ACT_GELU


def run_shuffle_conv(ctx: Ctx, x: torch.Tensor, p: PackedShuffleTail, conv: PackedConv,
                     tag: str = "shuffle_conv", form: int = 0, pre: Optional[PackedConv] = None,
                     conv2: Optional[PackedConv] = None) -> torch.Tensor:
    """``conv(tail(SiLU(PixelShuffle(r)(up(x)))))`` with ``conv`` = up_refinement.conv1[0] (BasicConv(1, C,
    3, 2, 1): BN + GELU), one launch (``esm_shuffle_conv_f32``); the 1-channel map between them is never
    stored.  Returns the conv output [B, C, ceil(r*H/2), ceil(r*W/2)].  ``form`` (nf 8, r 4, C 16): 0
    automatic, 1 the window form, 2 the row form (8 low-res rows), 3 the row form with the refinement conv on
    the matrix cores.  ``pre`` (nf 8, r 4, C 16): ``x`` is then the input of
    ``pre`` (the stage's spx_<t>[1], BasicConv(Cp, nf, 3, 1, 1)), computed inside the launch as well.
    ``conv2`` (with ``pre``): up_refinement.conv1[1] (BasicConv(C, C, 3, 1, 1)) too; the result is then its
    output (the whole conv1), the first conv's map never stored."""
    require_device(x, "shuffle_conv input")
    B, nf, H, W = (int(v) for v in x.shape)
    r = p.r
    if (p.nf, p.r, conv.cout) == (8, 4, 16) and form == 0 and SC_FORM and pre is not None:
        form = SC_FORM
    if pre is not None:
        if not shuffle_conv_pre_supported(p, conv, pre):
            raise ValueError("shuffle_conv: unsupported pre-conv")
        if nf != pre.cin:
            raise RuntimeError(f"shuffle_conv: pre-conv input has {nf} channels, layer expects {pre.cin}")
        if x.stride(3) != 1:
            raise ValueError("shuffle_conv: pre-conv input rows must be contiguous")
        nf = p.nf
    if nf != p.nf:
        raise RuntimeError(f"shuffle_conv: input has {nf} channels, layer expects {p.nf}")
    if not shuffle_conv_supported(p, conv):  # (size policy is the caller's: blocks.py)
        raise ValueError("shuffle_conv: unsupported head / conv geometry")
    Ho2, Wo2 = (H * r + 1) // 2, (W * r + 1) // 2
    out = ctx.empty(B, conv.cout, Ho2, Wo2)
    require_on(x.device, "shuffle_conv", x, out, p.up_w, p.up_b, p.tail_w, p.tail_b, conv.w, conv.scale, conv.shift)
    d = EsmShuffleConvDesc()
    t = d.st
    if pre is None:
        t.x = x.data_ptr()
        t.xb, t.xc, t.xh = x.stride(0), x.stride(1), x.stride(2)
    else:
        t.x = None
        t.xb, t.xc, t.xh = nf * H * W, H * W, W  # the virtual head input (never read)
        d.pre_x = x.data_ptr()
        d.pb, d.pc, d.ph = x.stride(0), x.stride(1), x.stride(2)
        d.pre_w = pre.w.data_ptr()
        d.pre_scale = pre.scale.data_ptr() if pre.scale is not None else None
        d.pre_shift = pre.shift.data_ptr() if pre.shift is not None else None
        d.pre_cin, d.pre_cin_pad, d.pre_cout_pad = pre.cin, pre.cin_pad, pre.cout_pad
        require_on(x.device, "shuffle_conv pre-conv", pre.w, pre.scale, pre.shift)
        ctx.hold(pre.w, pre.scale, pre.shift)
        form = form if form == 3 else 2  # the row forms (3: the refinement conv on the matrix cores)
    t.up_w, t.up_b, t.tail_w = p.up_w.data_ptr(), p.up_b.data_ptr(), p.tail_w.data_ptr()
    t.tail_b = p.tail_b.data_ptr() if p.tail_b is not None else None
    t.out = None
    t.B, t.nf, t.H, t.W, t.r = B, nf, H, W, r
    t.flags = (1 if B * H * W * r * r >= XCD_SLAB_MIN_PIX else 0) | (int(form) & 3) << 1
    d.w = conv.w.data_ptr()
    d.scale = conv.scale.data_ptr() if conv.scale is not None else None
    d.shift = conv.shift.data_ptr() if conv.shift is not None else None
    d.out = out.data_ptr()
    d.ob, d.oc, d.oh = out.stride(0), out.stride(1), out.stride(2)
    d.C, d.cin_pad, d.cout_pad = conv.cout, conv.cin_pad, conv.cout_pad
    ctx.hold(x, out, p.up_w, p.up_b, p.tail_w, p.tail_b, conv.w, conv.scale, conv.shift)
    if conv2 is not None:
        if pre is None or (p.nf, p.r, conv.cout) != (8, 4, 16) or conv2.nd != 2 or conv2.transposed or \
                (conv2.k, conv2.stride, conv2.pad, conv2.cin, conv2.cout) != (3, 1, 1, conv.cout, conv.cout) or \
                conv2.act != ACT_GELU:
            raise ValueError("shuffle_conv: the fused second conv must be BasicConv(C, C, 3, 1, 1) behind the "
                             "(8, 4, 16) row form with its pre-conv")
        require_on(x.device, "shuffle_conv second conv", conv2.w, conv2.scale, conv2.shift)
        d.w2 = conv2.w.data_ptr()
        d.scale2 = conv2.scale.data_ptr() if conv2.scale is not None else None
        d.shift2 = conv2.shift.data_ptr() if conv2.shift is not None else None
        d.cin_pad2, d.cout_pad2 = conv2.cin_pad, conv2.cout_pad
        t.flags |= (SC11_TILE & 3) << 3
        ctx.hold(conv2.w, conv2.scale, conv2.shift)
    npix = B * H * W * r * r
    flops = 2 * npix * nf * (nf + 9) + 2 * B * Ho2 * Wo2 * conv.cout * 9  # head as shuffle_tail + the 1 -> C 3x3
    cin_read = nf
    if pre is not None:  # + the 3x3 Cp -> nf pre-conv on the low-resolution map, whose weights are read too
        flops += 2 * B * H * W * nf * pre.cin * 9
        cin_read = pre.cin
    if conv2 is not None:  # + the 3x3 C -> C second conv on the output map
        flops += 2 * B * Ho2 * Wo2 * conv.cout * conv.cout * 9
    ctx.meta.append(dict(name=tag, kind="shuffle_conv", flops=flops,
                         bytes=4 * (B * cin_read * H * W + B * conv.cout * Ho2 * Wo2) +
                         (4 * 9 * pre.cin * nf if pre is not None else 0) +
                         (4 * 9 * conv.cout * conv.cout if conv2 is not None else 0),
                         shape=(f"pre {pre.cin}->{nf} k3 " if pre is not None else "") +
                         f"nf{nf} r{r} in {H}x{W} -> x {H * r}x{W * r} -> C{conv.cout} {Ho2}x{Wo2}" +
                         (f" -> k3 C{conv.cout}" if conv2 is not None else ""),
                         reads=_spans(x), writes=_spans(out)))
    ctx.shuffle_conv(d)
    return out
