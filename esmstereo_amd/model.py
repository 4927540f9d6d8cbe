"""Drop-in ``ESMStereo`` module (reference ``models/ESMStereo.py:511-745``).

Same constructor ``ESMStereo(maxdisp, gwc=False, norm_correlation=True,
backbone="efficientnet_b2", cv_scale=4)``, same ``forward(left, right, train_status)``
returning ``[disp]`` in eval (``[disp_1, disp_2(, disp_4)]`` with ``train_status``), same
state-dict keys for every module (the backbone with timm's key layout, ``backbone.Feature``),
so ``test_kitti.py`` / ``save_disp.py`` run unchanged with ``from esmstereo_amd import
__models__`` and load a reference checkpoint.  The backbone starts from random weights (the
reference's ``pretrained=True`` ImageNet weights are not fetchable offline): loading a state
dict that leaves every ``feature.*`` tensor untouched (e.g. through the callers' key filter,
``test_kitti.py:57-61``, with a checkpoint of another layout) warns that the backbone stays
random.

Split of the forward:

* backbone side (``:640-697``: feature pyramid, FeatUp, stems, matching descriptor,
  ``semantic``, ``conv_f2/f0``) - OUT of the hot path; PyTorch modules on the device, with
  every ``BasicConv`` among them running through the HIP conv kernel;
* hot path (``:700-745``: cost volume -> 3-D stems -> hourglass -> regression -> ESM
  upsampler -> ``*4``) - compiled once per input shape into a native ``esm_plan`` of ~70
  HIP launches and replayed as one hipGraph (:class:`HotPath`).
"""
from __future__ import annotations

import collections
import ctypes
import itertools
import math
import operator
import os
import warnings
from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.nn as nn

from . import _lib
from ._lib import check, lib
from .backbone import Feature, fast_path_ok
from .blocks import BasicConv, Conv2x, aggregation, upsample4, upsample8, upsample16
from . import engine as _engine
from .engine import (ACT_NONE, ACT_RELU, Ctx, cached_pack, gwc_stem_supported, pack_conv, require_device, run_conv,
                     run_gwc_stem)

__all__ = ["ESMStereo", "ESMStereo_trt", "ESMStereo_confidence", "FeatUp", "HotPath", "plan_ops"]

_VERSION = operator.attrgetter("_version")

# Bumped whenever any module anywhere registers a parameter, buffer or submodule (torch's global
# registration hooks): the only way a hot-path tensor can be REPLACED by another object.  The plan key
# re-collects the hot-path tensors after a bump, and otherwise only sums their in-place version counters.
_REG_EPOCH = [0]


def _bump_epoch(*_args) -> None:
    _REG_EPOCH[0] += 1


torch.nn.modules.module.register_module_parameter_registration_hook(_bump_epoch)
torch.nn.modules.module.register_module_buffer_registration_hook(_bump_epoch)
torch.nn.modules.module.register_module_module_registration_hook(_bump_epoch)


class FeatUp(nn.Module):
    """Backbone neck (reference models/ESMStereo.py:79-125); out of the hot path."""

    def __init__(self, chans: List[int], vol_size: int) -> None:
        super().__init__()
        self.v = vol_size
        self.deconv32_16 = Conv2x(chans[4], chans[3], deconv=True, concat=True)
        if self.v == 16:
            self.conv16 = BasicConv(chans[3] * 2, chans[2] * 2, kernel_size=3, stride=1, padding=1)
        if self.v in (8, 4):
            self.deconv16_8 = Conv2x(chans[3] * 2, chans[2], deconv=True, concat=True)
        if self.v == 8:
            self.conv8 = BasicConv(chans[2] * 2, chans[2] * 2, kernel_size=3, stride=1, padding=1)
        if self.v == 4:
            self.deconv8_4 = Conv2x(chans[2] * 2, chans[1], deconv=True, concat=True)
            self.conv4 = BasicConv(chans[1] * 2, chans[1] * 2, kernel_size=3, stride=1, padding=1)
        for m in self.modules():  # He-normal init as the reference SubModule.weight_init (:25-38)
            if isinstance(m, (nn.Conv2d, nn.Conv3d)):
                n = math.prod(m.kernel_size) * m.out_channels
                m.weight.data.normal_(0, math.sqrt(2.0 / n))
            elif isinstance(m, (nn.BatchNorm2d, nn.BatchNorm3d)):
                m.weight.data.fill_(1)
                m.bias.data.zero_()

    def one(self, feats):
        """The neck on one feature list (both images at once when the pyramid is batched [left; right]:
        every op is per sample, so this equals the reference's two passes)."""
        x2, x4, x8, x16, x32 = feats
        x16 = self.deconv32_16(x32, x16)
        if self.v == 16:
            x16 = self.conv16(x16)
        if self.v in (8, 4):
            x8 = self.deconv16_8(x16, x8)
        if self.v == 8:
            x8 = self.conv8(x8)
        if self.v == 4:
            x4 = self.conv4(self.deconv8_4(x8, x4))
        return [x4, x8, x16, x32]

    def forward(self, featL, featR):
        return self.one(featL), self.one(featR)


def _stem(cin: int, c: int) -> nn.Sequential:
    return nn.Sequential(BasicConv(cin, c, kernel_size=3, stride=2, padding=1), nn.Conv2d(c, c, 3, 1, 1, bias=False),
                         nn.BatchNorm2d(c), nn.ReLU())


def _seq_fast(seq: nn.Sequential, x: torch.Tensor) -> torch.Tensor:
    """A backbone-side Sequential of [BasicConv, Conv2d(, BatchNorm2d, ReLU)] (the stems, ESMStereo.py:528-583;
    ``semantic``, :600-607) with the trailing plain conv (+ BN + ReLU) as one HIP conv launch (BN folded, ReLU in
    the epilogue) in eval mode without autograd; the module's own forward otherwise."""
    if not fast_path_ok(seq, x):
        return seq(x)
    y = seq[0](x)
    conv = seq[1]
    bn = seq[2] if len(seq) > 2 else None
    act = ACT_RELU if len(seq) > 3 else ACT_NONE
    pc = cached_pack(seq, "conv", (conv, bn), lambda: pack_conv(conv, bn, act), act)
    return run_conv(Ctx(y.device), pc, [y], tag=getattr(seq, "_esm_name", "stem") + ".1")


def _conv_fast(conv: nn.Conv2d, x: torch.Tensor) -> torch.Tensor:
    """A plain nn.Conv2d of the backbone side (``desc``, ESMStereo.py:597) as one HIP conv launch in eval mode."""
    if not fast_path_ok(conv, x):
        return conv(x)
    pc = cached_pack(conv, "conv", (conv,), lambda: pack_conv(conv, None, ACT_NONE))
    return run_conv(Ctx(x.device), pc, [x], tag=getattr(conv, "_esm_name", "conv"))


# stems per cost-volume scale (reference ESMStereo.py:528-583): name -> (cin, cout)
_STEMS = {
    4: (("stem_2", 3, 32), ("stem_4", 32, 48)),
    8: (("stem_2", 3, 32), ("stem_4", 32, 48), ("stem_8", 48, 64)),
    16: (("stem_2", 3, 16), ("stem_4", 16, 24), ("stem_8", 24, 32), ("stem_16", 32, 40)),
}
# matching-descriptor input channels (ESMStereo.py:585-597) and hourglass add_channel (:624-634)
_DESC_IN = {4: 96, 8: 160, 16: 136}
_ADD_CHANNEL = {4: 16, 8: 8, 16: 4}
_UPSAMPLERS = {4: upsample4, 8: upsample8, 16: upsample16}


class HotPath:
    """The hot path (ESMStereo.py:700-745) compiled for one set of input shapes.

    The plan owns static device buffers for its inputs (``ml``, ``mr``, ``att``, ``up``) and its
    outputs; ``launch()`` replays the native plan (a hipGraph by default) on the current stream.
    :meth:`bind` makes the plan read the caller's own tensors where they lie (zero-copy, as the
    reference's forward does), :meth:`load_inputs` copies into the plan's buffers; ``outputs`` are
    static buffers holding the ``*4``-scaled disparities.
    """

    def __init__(self, model: "ESMStereo", B: int, h: int, w: int, att_ch: int, up_shapes: Sequence[Tuple[int, ...]],
                 device: torch.device, train_status: bool = False, graph: bool = True, channels: int = 64):
        self.device = torch.device(device)
        args = (model, B, h, w, att_ch, up_shapes, train_status, channels)
        # size the arena with a dry emission (shape-only buffers, nothing submitted), then emit once
        # into ONE arena chunk (one allocation; the plan's buffers together)
        with Ctx(self.device, dry=True) as dry:
            self._emit(dry, *args)
        self.ctx = Ctx(self.device, plan=True)
        self.ctx.ARENA_FIRST = dry.arena_bytes + (1 << 20)
        self._emit(self.ctx, *args)
        self.num_ops = lib.esm_plan_num_ops(self.ctx.plan)
        if self.ctx.arena_chunks != 1 or self.num_ops != dry.num_ops:
            raise RuntimeError(f"HotPath: dry emission disagrees with the plan ({dry.num_ops} vs {self.num_ops} ops, "
                               f"{self.ctx.arena_chunks} arena chunks)")
        self.graph = bool(graph)
        self._graph_ready = False
        arena = self.ctx._arena
        self._arena_span = (arena.data_ptr(), arena.data_ptr() + arena.numel())
        self._own = [self.ml, self.mr, self.att] + list(self.up)    # the plan's own input buffers
        self._bound = [None if t is None else t.data_ptr() for t in self._own]  # what the plan reads now
        # slots whose caller pointer changed while the previous replay was still running: they are copied
        # into the plan's own buffer from then on (stream-ordered, no host wait)
        self._copy_mode = [False] * len(self._own)

    def _emit(self, ctx: Ctx, model, B, h, w, att_ch, up_shapes, train_status, channels) -> None:
        e = ctx.empty
        self.ml = e(B, channels, h, w)
        self.mr = e(B, channels, h, w)
        self.att = e(B, att_ch, h, w) if att_ch else None
        # the upsampler's feature inputs at the arena's far end, next to the buffers allocated last
        # (the upsampler's own, which they are concatenated with)
        self.up = [ctx.empty_tail(*s) for s in up_shapes]
        self.outputs = model._emit_hot(ctx, self.ml, self.mr, self.att, self.up, train_status)

    def op_kinds(self) -> List[int]:
        return [lib.esm_plan_op_kind(self.ctx.plan, i) for i in range(self.num_ops)]

    def set_probe(self, index: int, ring: int = 1024) -> None:
        check(lib.esm_plan_set_probe(self.ctx.plan, index, ring), "set_probe")
        self._graph_ready = False

    def probe_read(self, max_n: int = 4096) -> List[float]:
        buf = (_lib.c_float * max_n)()
        n = check(lib.esm_plan_probe_read(self.ctx.plan, buf, max_n), "probe_read")
        return [buf[i] for i in range(n)]

    def run_op(self, index: int, reps: int = 1, stream: Optional[torch.cuda.Stream] = None) -> None:
        """Launch op ``index`` of the plan alone, ``reps`` times back to back (kernel timing)."""
        s = _lib.c_void_p((stream or torch.cuda.current_stream(self.device)).cuda_stream)
        check(lib.esm_plan_run_op(self.ctx.plan, index, reps, s), "plan_run_op")

    def launch(self, stream: Optional[torch.cuda.Stream] = None) -> None:
        s = _lib.c_void_p((stream or torch.cuda.current_stream(self.device)).cuda_stream)
        if self.graph:
            if not self._graph_ready:
                check(lib.esm_plan_graph_build(self.ctx.plan, s), "graph_build")
                self._graph_ready = True
            check(lib.esm_plan_graph_launch(self.ctx.plan, s), "graph_launch")
        else:
            check(lib.esm_plan_run(self.ctx.plan, s), "plan_run")

    # ------------------------------------------------------------------ inputs
    def _slots(self, ml, mr, att, up) -> list:
        if len(up) != len(self.up):
            raise ValueError(f"hot path: expected {len(self.up)} upsampler features, got {len(up)}")
        if (att is None) != (self.att is None):
            raise ValueError("hot path: att given to a plan built without it, or missing")
        a = None if att is None else att.reshape(self.att.shape)
        return [ml, mr, a] + list(up)

    def _in_place_ok(self, i: int, t: torch.Tensor) -> bool:
        """Whether the plan may read ``t`` where it lies: contiguous fp32 on the plan's device, not
        overlapping the plan's arena (whose buffers the launches overwrite) unless it IS the slot's own
        buffer.  Every kernel addresses each concat source through a descriptor of its own, so a
        feature may lie anywhere."""
        if t.data_ptr() == self._own[i].data_ptr():
            return True
        if t.device != self.device or t.dtype != torch.float32 or not t.is_contiguous():
            return False
        lo, hi = t.data_ptr(), t.data_ptr() + 4 * t.numel()
        a_lo, a_hi = self._arena_span
        return not (lo < a_hi and a_lo < hi)

    def _rebind(self, ptrs: Sequence[Optional[int]]) -> None:
        olds, sizes, news, idx = [], [], [], []
        for i, p in enumerate(ptrs):
            if p is not None and p != self._bound[i]:
                olds.append(self._bound[i])
                sizes.append(4 * self._own[i].numel())
                news.append(p)
                idx.append(i)
        if olds:
            n = len(olds)
            check(lib.esm_plan_rebind(self.ctx.plan, n, (_lib.c_void_p * n)(*olds), (ctypes.c_uint64 * n)(*sizes),
                                      (_lib.c_void_p * n)(*news)), "plan_rebind")
            for i, p in zip(idx, news):  # only once the native side has moved them
                self._bound[i] = p

    def bind(self, ml, mr, att, up) -> None:
        """Point the plan at the caller's tensors (zero-copy; models/ESMStereo.py:700-745 reads its
        features where they lie).  A tensor the plan cannot read in place (non-contiguous, another
        device, or aliasing the plan's buffers) is copied into the
        plan's own buffer instead.  The plan keeps no reference: the caller keeps the tensors alive
        until the launch that reads them has run (stream order, as for any PyTorch op).  When the
        pointers are the ones already bound (a serving loop whose allocator hands back the same
        blocks), nothing happens; otherwise the graph's affected nodes are updated in place.

        Two slots never read overlapping memory through a binding: a tensor that overlaps another
        slot's tensor of the same call (``hot_path(x, x, ...)``) is copied into its slot's own buffer,
        so every bound range belongs to exactly one slot and a later rebind moves each pointer to the
        right tensor.  A slot whose pointer changes while the previous replay is still
        running (a caller handing over fresh tensors every step) switches to copies for good: a rebind
        would make the host wait for the device."""
        busy = None
        ptrs, spans = [], []
        for i, (t, own) in enumerate(zip(self._slots(ml, mr, att, up), self._own)):
            if own is None:
                ptrs.append(None)
                continue
            require_device(t, "hot-path input")
            if tuple(t.shape) != tuple(own.shape):
                raise ValueError(f"hot path input {i}: shape {tuple(t.shape)}, plan built for {tuple(own.shape)}")
            copy = self._copy_mode[i] or not self._in_place_ok(i, t)
            if not copy:
                lo, hi = t.data_ptr(), t.data_ptr() + 4 * t.numel()
                copy = any(lo < b and a < hi for a, b in spans)  # aliases an earlier slot of this call
            if not copy and t.data_ptr() != self._bound[i]:
                if busy is None:
                    busy = check(lib.esm_plan_busy(self.ctx.plan), "plan_busy") > 0
                if busy:
                    self._copy_mode[i] = copy = True
            if copy and t.data_ptr() != own.data_ptr():
                own.copy_(t)
                t = own
            ptrs.append(t.data_ptr())
            spans.append((t.data_ptr(), t.data_ptr() + 4 * t.numel()))
        self._rebind(ptrs)

    def load_inputs(self, ml, mr, att, up) -> None:
        """Copy the inputs into the plan's own buffers (and read those)."""
        for t, own in zip(self._slots(ml, mr, att, up), self._own):
            if own is not None:
                own.copy_(t)
        self._rebind([None if t is None else t.data_ptr() for t in self._own])

    def close(self) -> None:
        # the plan's buffers came from torch's caching allocator on the stream current at build
        # time, but replays may run on other streams (launch(stream)): drain the device before
        # the memory can be handed out again
        if self.device.type == "cuda":
            torch.cuda.synchronize(self.device)
        self.ctx.close()


class ForwardGraph:
    """The whole eval forward (reference ``models/ESMStereo.py:638-745``) for one input shape, replayed
    without host work per launch:

    * the backbone side (:meth:`ESMStereo.prefix`: the timm-layout feature pyramid on MIOpen, the neck, the
      stems and the matching descriptor, whose ``BasicConv``s run the HIP conv kernels) is captured once
      into a torch CUDA graph (hipGraph) over static image buffers; its outputs then live at fixed
      addresses in the graph's memory pool;
    * the hot path's own plan (:class:`HotPath`) is bound zero-copy to those outputs and replayed as its
      hipGraph right behind it, on the same stream.

    ``run(left, right)`` copies the images into the static buffers, replays both graphs and returns fresh
    output tensors (the reference returns new tensors).  Captured after two eager warm-up passes on a side
    stream (MIOpen's algorithm choice and every lazily packed weight settle there, as torch's capture rules
    require)."""

    def __init__(self, model: "ESMStereo", left: torch.Tensor, right: torch.Tensor, train_status: bool):
        self.device = left.device
        # capture, streams and the torch ops of prefix() on the input's device, whatever device is current
        # (torch.cuda.graph() makes its capture stream on the current device)
        with torch.cuda.device(self.device):
            self._build(model, left, right, train_status)

    def _build(self, model: "ESMStereo", left: torch.Tensor, right: torch.Tensor, train_status: bool) -> None:
        B = int(left.shape[0])
        self.both = torch.cat((left, right), 0)  # the static image buffer: [left; right], the backbone's batch
        self.left, self.right = self.both[:B], self.both[B:]
        cur = torch.cuda.current_stream(self.device)
        side = torch.cuda.Stream(self.device)
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(2):
                ml, mr, att, up = model.prefix(self.left, self.right, self.both)
        cur.wait_stream(side)
        torch.cuda.synchronize(self.device)
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self.ml, self.mr, self.att, self.up = model.prefix(self.left, self.right, self.both)
        self.hp = HotPath(model, int(self.ml.shape[0]), int(self.ml.shape[2]), int(self.ml.shape[3]),
                          0 if self.att is None else int(self.att.shape[1]), [tuple(u.shape) for u in self.up],
                          self.device, train_status, graph=True, channels=int(self.ml.shape[1]))
        self.hp.bind(self.ml, self.mr, self.att, self.up)

    def run(self, left: torch.Tensor, right: torch.Tensor) -> List[torch.Tensor]:
        with torch.cuda.device(self.device):
            self.left.copy_(left)
            self.right.copy_(right)
            self.graph.replay()
            self.hp.launch()
            return [o.clone() for o in self.hp.outputs]

    def close(self) -> None:
        self.hp.close()
        self.graph.reset()


def plan_ops(model: "ESMStereo", B: int, h: int, w: int, att_ch: int, up_shapes: Sequence[Tuple[int, ...]],
             train_status: bool = False, channels: int = 64) -> List[dict]:
    """The launch list the hot path compiles to for these input shapes, one dict per launch (name,
    kernel family, shape, algorithmic flops and bytes: ``Ctx.meta``), from a dry emission: nothing runs
    and no device is needed (the weights may sit on the CPU)."""
    with Ctx(torch.device("meta"), dry=True) as ctx:
        e = ctx.empty
        up = [e(*s) for s in up_shapes]
        model._emit_hot(ctx, e(B, channels, h, w), e(B, channels, h, w), e(B, att_ch, h, w) if att_ch else None, up,
                        train_status)
    return ctx.meta


class ESMStereo(nn.Module):
    """ESMStereo stereo network with the HIP hot path (reference models/ESMStereo.py:511-745)."""

    _HOT_MODULES = ("group_stem", "corr_stem", "agg", "aggregation_out", "upsample_module")
    FORWARD_GRAPHS = 4  # captured whole-forward graphs kept (input shapes), as the hot-path plan cache

    def __init__(self, maxdisp: int, gwc: bool = False, norm_correlation: bool = True,
                 backbone: str = "efficientnet_b2", cv_scale: int = 4, *, feature_cls=None) -> None:
        """Reference positional signature (ESMStereo.py:512).  ``feature_cls`` (keyword only)
        replaces the backbone class; the golden-vector tests pass ``backbone.StubFeature``."""
        super().__init__()
        self.maxdisp = maxdisp
        self.vol_size = cv_scale
        self.gwc = gwc
        self.norm_correlation = norm_correlation
        self.backbone = backbone
        if cv_scale not in _STEMS:
            raise ValueError("Choose the cost volume resolution: 4, 8, 16")
        self.feature = (feature_cls or Feature)(self.backbone)
        if cv_scale in (4, 8):
            self.feature_up = FeatUp(self.feature.chans, cv_scale)
        for name, cin, c in _STEMS[cv_scale]:
            setattr(self, name, _stem(cin, c))
        self.conv = BasicConv(_DESC_IN[cv_scale], 64, kernel_size=3, padding=1, stride=1)
        self.desc = nn.Conv2d(64, 64, kernel_size=1, padding=0, stride=1)
        if cv_scale == 16:
            self.conv_f2 = BasicConv(96, 32, kernel_size=3, padding=1, stride=1)
            self.conv_f0 = BasicConv(16, 24, kernel_size=3, padding=1, stride=1)
        red = 8
        if norm_correlation:
            print("Cost volumes: norm correlation")
            if cv_scale == 16:
                self.semantic = nn.Sequential(BasicConv(96, 32, kernel_size=3, stride=1, padding=1),
                                              nn.Conv2d(32, 8, 3, 1, 1, bias=False))
            self.corr_stem = BasicConv(1, red, is_3d=True, kernel_size=3, padding=1, stride=1)
        if gwc:
            print("Cost volumes: gwc ")
            if cv_scale == 16:
                self.semantic = nn.Sequential(BasicConv(96, 64, kernel_size=3, stride=1, padding=1),
                                              nn.Conv2d(64, 32, 3, 1, 1, bias=False))
            self.num_groups = 32
            self.group_stem = BasicConv(self.num_groups, red, is_3d=True, kernel_size=3, padding=1, stride=1)
        self.agg = BasicConv(red, red, is_3d=True, kernel_size=3, padding=1, stride=1)
        self.upsample_module = _UPSAMPLERS[cv_scale]()
        self.aggregation_out = aggregation(red, _ADD_CHANNEL[cv_scale])
        for name, mod in self.named_modules():  # launch names for profiles / the bench probe
            object.__setattr__(mod, "_esm_name", name)
        self._plans: "collections.OrderedDict" = collections.OrderedDict()
        # ESM_GRAPH=0 replays the plan eagerly (A/B measurements; read only with ESM_AB=1)
        self.use_graph = not (os.environ.get("ESM_AB") == "1" and os.environ.get("ESM_GRAPH", "1") == "0")
        # the whole eval forward (backbone side + hot path) replayed from captured graphs (ForwardGraph);
        # False runs the backbone side eagerly and only the hot path from its plan's graph
        self.capture_forward = True

    # ------------------------------------------------------------------ plan cache
    def invalidate_plans(self) -> None:
        """Drop compiled hot-path plans.  In-place edits, replaced Parameter / buffer objects,
        ``load_state_dict`` and ``.to()`` are detected on their own; call this after adding or
        removing a hot-path submodule."""
        for hp in self._plans.values():
            hp.close()
        self._plans.clear()
        for fg in self.__dict__.get("_fwd_graphs", {}).values():
            fg.close()
        self.__dict__["_fwd_graphs"] = collections.OrderedDict()
        self.__dict__["_all_state"] = None
        self.__dict__["_hot_dicts"] = None
        self.__dict__["_hot_state"] = None

    def _apply(self, fn, *args, **kwargs):
        self.invalidate_plans()
        return super()._apply(fn, *args, **kwargs)

    def _hot_tensors(self) -> list:
        """Every hot-path Parameter and buffer, read afresh from the modules' own ``_parameters`` /
        ``_buffers`` dicts: the list of dicts is collected once (``_apply`` / ``load_state_dict``
        rebuild it), the tensors in them on every call, so a replaced Parameter object
        (``mod.weight = nn.Parameter(...)``) is seen as well as an in-place edit."""
        dicts = self.__dict__.get("_hot_dicts")
        if dicts is None:
            mods = [m for name in self._HOT_MODULES if getattr(self, name, None) is not None
                    for m in getattr(self, name).modules()]
            dicts = [d for m in mods for d in (m._parameters, m._buffers)]
            self.__dict__["_hot_dicts"] = dicts
        return [t for t in itertools.chain.from_iterable(map(dict.values, dicts)) if t is not None]

    def _hot_param_token(self) -> tuple:
        """(identity, in-place state) of the hot-path tensors: a weight edited in place (``param.copy_``,
        BN statistics updated elsewhere) bumps its version counter, so the sum of the counters changes
        (they only grow); a tensor replaced by another object (``mod.weight = nn.Parameter(...)``) goes
        through module registration, which bumps ``_REG_EPOCH``, and the identities are then
        re-collected (their hash is the first field).  So the plan cache never replays stale packed
        weights, and the per-call cost is one C-level sum over the 383 tensors of ESMStereo-S (~35 us;
        the per-tensor tuples it replaced cost ~240 us a call, most of a KITTI-size step's host budget).
        Reassigning ``param.data`` changes neither: call :meth:`invalidate_plans` after doing that."""
        ep = _REG_EPOCH[0]
        st = self.__dict__.get("_hot_state")
        if st is None or st[0] != ep:
            ts = self._hot_tensors()
            st = (ep, ts, hash(tuple(map(id, ts))))
            self.__dict__["_hot_state"] = st
        return st[2], sum(map(_VERSION, st[1]))

    def _all_param_token(self) -> tuple:
        """As :meth:`_hot_param_token` over EVERY parameter and buffer (the backbone side included): the
        key of the captured whole-forward graphs."""
        ep = _REG_EPOCH[0]
        st = self.__dict__.get("_all_state")
        if st is None or st[0] != ep:
            ts = [t for t in itertools.chain(self.parameters(), self.buffers())]
            st = (ep, ts, hash(tuple(map(id, ts))))
            self.__dict__["_all_state"] = st
        return st[2], sum(map(_VERSION, st[1]))

    def _load_from_state_dict(self, state_dict, prefix, *args, **kwargs):
        self.invalidate_plans()
        # Warn when a checkpoint supplied hot-path weights but no usable backbone weight: every
        # feature.* entry is absent, mis-shaped, or the model's own tensor handed back (the callers'
        # key filter, test_kitti.py:56-60, refills dropped keys from model.state_dict()).  A
        # same-weights reload or a state-dict round trip supplies its own tensors and stays quiet.
        own = {t.data_ptr() for t in list(self.parameters()) + list(self.buffers())}
        feat = dict(self.feature.state_dict())
        fp = prefix + "feature."
        supplied_feat = any(isinstance(v, torch.Tensor) and k[len(fp):] in feat and v.shape == feat[k[len(fp):]].shape
                            and v.data_ptr() not in own for k, v in state_dict.items() if k.startswith(fp))
        supplied_hot = any(isinstance(v, torch.Tensor) and v.data_ptr() not in own
                           for k, v in state_dict.items() if k.startswith(prefix) and not k.startswith(fp))
        if feat and supplied_hot and not supplied_feat:
            warnings.warn("ESMStereo.load_state_dict: the checkpoint supplies no feature.* (backbone) weight; the "
                          "backbone keeps its random initialisation (checkpoint of another backbone layout?)",
                          RuntimeWarning, stacklevel=3)
        return super()._load_from_state_dict(state_dict, prefix, *args, **kwargs)

    # ------------------------------------------------------------------ forward pieces
    def prefix(self, left: torch.Tensor, right: torch.Tensor, both: Optional[torch.Tensor] = None):
        """Backbone side, reference lines 640-697 -> (match_left, match_right, att, upsampler feats).
        ``both``: [left; right] already as one [2B, ...] tensor (left / right its halves): no concat."""
        return self._prefix(left, right, both)[:4]

    def _prefix(self, left: torch.Tensor, right: torch.Tensor, both: Optional[torch.Tensor] = None):
        """The backbone side with left and right as ONE batch [left; right] (eval BatchNorm and every other
        op are per sample, so each half equals the reference's separate left / right passes, :640-697):
        every backbone launch covers both images, half the launches of the reference's order."""
        vs = self.vol_size
        B = int(left.shape[0])
        if tuple(left.shape) != tuple(right.shape):
            raise RuntimeError(f"left {tuple(left.shape)} and right {tuple(right.shape)} image sizes differ")
        if both is None:
            both = torch.cat((left, right), 0)
        f = self.feature(both)
        if vs in (4, 8):
            f = self.feature_up.one(f)
        stems = [_seq_fast(self.stem_2, both)]
        for name, _, _ in _STEMS[vs][1:]:
            stems.append(_seq_fast(getattr(self, name), stems[-1]))
        idx = {4: 0, 8: 1, 16: 3}[vs]
        src = [f[idx], stems[-1]]
        if fast_path_ok(self.conv, both) and all(int(t.shape[1]) % 4 == 0 for t in src):
            mc = self.conv.emit(Ctx(both.device), src)  # the concat as two conv sources, never materialised
        else:
            mc = self.conv(torch.cat(src, 1))
        m = _conv_fast(self.desc, mc)
        ml, mr = m[:B], m[B:]
        fl = [t[:B] for t in f]
        sx = stems[0][:B]
        att = _seq_fast(self.semantic, fl[3]) if vs == 16 else None
        if vs == 4:
            up = [fl[1], fl[0], sx]
        elif vs == 8:
            up = [fl[2], fl[1], fl[0], sx]
        else:
            up = [fl[2], self.conv_f2(fl[3]), fl[1], self.conv_f0(fl[0])]
        return ml, mr, att, up, fl

    def _emit_hot(self, ctx: Ctx, ml: torch.Tensor, mr: torch.Tensor, att: Optional[torch.Tensor],
                  up: Sequence[torch.Tensor], train_status: bool) -> List[torch.Tensor]:
        B, C, h, w = (int(v) for v in ml.shape)
        D = self.maxdisp // self.vol_size
        vs = self.vol_size
        if self.gwc:
            a = att.reshape(B, self.num_groups, h, w) if (vs == 16 and att is not None) else None
            pc = self.group_stem.packed()
            if _engine.GWC_STEM_ENABLED and gwc_stem_supported(pc, ml, self.num_groups, D, a):
                vol = run_gwc_stem(ctx, pc, ml, mr, self.num_groups, D,
                                   tag=f"gwc_volume+{self.group_stem._esm_name}")
            else:
                V = ctx.empty(B, self.num_groups, D, h, w)
                ctx.gwc(ml, mr, a, V, B, C, h, w, D, self.num_groups)
                vol = self.group_stem.emit(ctx, [V])
        elif self.norm_correlation:
            V = ctx.empty(B, 1, D, h, w)
            work = ctx.empty(2, B, C, h, w)
            ctx.normcorr(ml, mr, V, work, B, C, h, w, D)
            mul = att.reshape(B, -1, h, w) if (vs == 16 and att is not None) else None
            vol = self.corr_stem.emit(ctx, [V], mul=mul)
        else:
            raise UnboundLocalError("local variable 'volume' referenced before assignment")
        vol = self.agg.emit(ctx, [vol])
        cost = self.aggregation_out.emit(ctx, vol)
        Dc = int(cost.shape[2])
        if Dc != D:
            raise RuntimeError(f"The size of tensor a ({Dc}) must match the size of tensor b ({D}) at non-singleton "
                               f"dimension 1 (maxdisp // cv_scale must be even, SURVEY.md §0.4)")
        init = ctx.empty(B, 1, h, w)
        reg_cost = None
        if vs == 4:
            ctx.regression(1, cost.view(B, D, h, w), init, B, D, h, w)
        else:  # disparity_regression: inside the upsampler's first pair where it fits, else its own launch there
            reg_cost = cost.view(B, D, h, w)
        outs = self.upsample_module.emit(ctx, up, init, final_scale=4.0,
                                         scaled_copies=4.0 if train_status else None, init_cost=reg_cost)
        extra = self._emit_extra(ctx, cost.view(B, D, h, w), init, ml, up)
        if extra:
            return [outs[0].view(B, outs[0].shape[-2], outs[0].shape[-1])] + extra
        if train_status:
            finals, copies = outs
            return [finals[0].view(B, finals[0].shape[-2], finals[0].shape[-1])] + \
                   [c.view(B, c.shape[-2], c.shape[-1]) for c in copies]
        return [outs[0].view(B, outs[0].shape[-2], outs[0].shape[-1])]

    def _emit_extra(self, ctx: Ctx, cost: torch.Tensor, init: torch.Tensor, ml: torch.Tensor,
                    up: Sequence[torch.Tensor]) -> List[torch.Tensor]:
        """Heads that read the hot path's intermediates (ESMStereo_confidence); none here."""
        return []

    def hot_path(self, ml: torch.Tensor, mr: torch.Tensor, att: Optional[torch.Tensor], up: Sequence[torch.Tensor],
                 train_status: bool = False) -> List[torch.Tensor]:
        """Run reference lines 700-745 on given matching features (compiled + cached plan)."""
        for t in [ml, mr, *up] + ([att] if att is not None else []):
            require_device(t, "hot-path input")
        key = (tuple(ml.shape), None if att is None else tuple(att.shape), tuple(tuple(u.shape) for u in up),
               bool(train_status), ml.device, self._hot_param_token())
        hp = self._plans.get(key)
        if hp is None:
            hp = HotPath(self, int(ml.shape[0]), int(ml.shape[2]), int(ml.shape[3]),
                         0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], ml.device,
                         train_status, graph=self.use_graph, channels=int(ml.shape[1]))
            self._plans[key] = hp
            while len(self._plans) > 4:
                self._plans.popitem(last=False)[1].close()
        else:
            self._plans.move_to_end(key)
        hp.bind(ml, mr, att, up)
        hp.launch()
        return [o.clone() for o in hp.outputs]

    def forward(self, left: torch.Tensor, right: torch.Tensor, train_status: bool) -> List[torch.Tensor]:
        if self.training:
            raise NotImplementedError("esmstereo_amd is an inference engine (eval-mode BatchNorm folded into the "
                                      "kernels); call model.eval()")
        require_device(left, "left")
        require_device(right, "right")
        with torch.no_grad():
            if self.use_graph and self.capture_forward:
                return self._forward_graph(left, right, train_status)
            ml, mr, att, up = self.prefix(left, right)
            return self.hot_path(ml, mr, att, up, train_status)

    def _forward_graph(self, left: torch.Tensor, right: torch.Tensor, train_status: bool) -> List[torch.Tensor]:
        """The forward through a captured :class:`ForwardGraph` per (input shapes, weights)."""
        key = (tuple(left.shape), tuple(right.shape), left.device, bool(train_status), self._all_param_token())
        graphs = self.__dict__.setdefault("_fwd_graphs", collections.OrderedDict())
        fg = graphs.get(key)
        if fg is None:
            for k in [k for k in graphs if k[-1] != key[-1]]:  # captured under older weights: never hit again
                graphs.pop(k).close()
            # a caller cycling through more input shapes than the cache holds would re-capture (two warm-up
            # forwards, a capture and a new plan) on every call: after that many evictions, shapes not in the
            # cache take the eager backbone + cached plan instead
            if self.__dict__.get("_fwd_evictions", 0) >= self.FORWARD_GRAPHS:
                ml, mr, att, up = self.prefix(left, right)
                return self.hot_path(ml, mr, att, up, train_status)
            fg = ForwardGraph(self, left, right, train_status)
            graphs[key] = fg
            while len(graphs) > self.FORWARD_GRAPHS:
                graphs.popitem(last=False)[1].close()
                self.__dict__["_fwd_evictions"] = self.__dict__.get("_fwd_evictions", 0) + 1
        else:
            graphs.move_to_end(key)
        return fg.run(left, right)


class ESMStereo_trt(ESMStereo):
    """The export / deployment signature (reference ``models/ESMStereo_trt.py:511-737``, exported by
    ``onnx_transformed.py:48-51`` with inputs ``left``, ``right`` and output ``disp``): the same
    module tree and state dict as :class:`ESMStereo`, and ``forward(left, right) -> disp [B, H, W]``,
    the eval output of ``ESMStereo.forward`` (``ESMStereo_trt.py:638,735``), over the same compiled
    HIP plan."""

    def forward(self, left: torch.Tensor, right: torch.Tensor) -> torch.Tensor:  # type: ignore[override]
        return super().forward(left, right, False)[0]


class ESMStereo_confidence(ESMStereo):
    """ESMStereo with the LAFNet confidence head (reference ``models/ESMStereo_confidence.py:746-974``).

    Same constructor as the reference (``device`` is accepted; tensors follow the module), the
    :class:`ESMStereo` module tree plus ``confidence_net = LAFNet_ESM(16)`` for ``cv_scale=16`` (the
    only scale the reference builds it for, ``:915-916``), and ``forward(left, right) -> (disp * 4,
    confidence)`` (``:974``).  The head is emitted into the same compiled plan as the hot path: it
    reads the aggregated cost, ``init_pred`` and ``match_left`` in place (``:972``)."""

    # the head is emitted into the same plan, so its weights key the plan cache too
    _HOT_MODULES = ESMStereo._HOT_MODULES + ("confidence_net",)

    def __init__(self, maxdisp: int, gwc: bool = False, norm_correlation: bool = True,
                 backbone: str = "efficientnet_b2", cv_scale: int = 4, device=None, *, feature_cls=None) -> None:
        super().__init__(maxdisp, gwc, norm_correlation, backbone, cv_scale, feature_cls=feature_cls)
        self.device = device
        if cv_scale == 16:
            from .confidence import LAFNet_ESM
            self.confidence_net = LAFNet_ESM(16)
            for name, mod in self.confidence_net.named_modules():
                object.__setattr__(mod, "_esm_name", "confidence_net" + ("." + name if name else ""))

    def prefix(self, left: torch.Tensor, right: torch.Tensor, both: Optional[torch.Tensor] = None):
        """As :meth:`ESMStereo.prefix`, with features_left[3] appended to the upsampler features
        (the confidence head's ``left_f1x``, ``:972``)."""
        ml, mr, att, up, fl = self._prefix(left, right, both)
        if self.vol_size == 16:
            up = list(up) + [fl[3]]
        return ml, mr, att, up

    def _emit_extra(self, ctx: Ctx, cost: torch.Tensor, init: torch.Tensor, ml: torch.Tensor,
                    up: Sequence[torch.Tensor]) -> List[torch.Tensor]:
        net = getattr(self, "confidence_net", None)
        if net is None:
            return []
        B = int(cost.shape[0])
        # confidence_net(cost.squeeze(1), init_pred, match_left, features_left[3], features_left[1]) (:972)
        conf = net.emit(ctx, cost, init, ml, up[4], up[2])
        return [conf.view(B, conf.shape[-2], conf.shape[-1])]

    def forward(self, left: torch.Tensor, right: torch.Tensor):  # type: ignore[override]
        if self.vol_size != 16:
            # the reference returns conf_out, which only the cv_scale=16 branch assigns (:966-974)
            raise UnboundLocalError("local variable 'conf_out' referenced before assignment")
        outs = super().forward(left, right, False)
        return outs[0], outs[1]
