"""ctypes binding of ``include/esmstereo_amd.h`` (the C ABI of libesmstereo_amd.so).

Loading is strict: if the in-tree library is missing or its struct layout does not match
these declarations, importing raises — the package has no CPU / PyTorch fallback.
"""
from __future__ import annotations

import ctypes
import os
from ctypes import POINTER, Structure, c_float, c_int, c_int32, c_int64, c_void_p

PKG = os.path.dirname(os.path.abspath(__file__))
# ESM_LIB: load another build of the same ABI (the diagnostic build of esmstereo_amd/build.py)
LIB_PATH = os.environ.get("ESM_LIB") or os.path.join(PKG, "libesmstereo_amd.so")
ROOT = os.path.dirname(PKG)
HEADER_PATH = os.path.join(ROOT, "include", "esmstereo_amd.h")

MAX_SRC = 3
SMIX_MAX_STAGES = 2

ACT_NONE, ACT_GELU, ACT_SILU, ACT_RELU, ACT_SIGMOID, ACT_RELU6 = 0, 1, 2, 3, 4, 5
CONF_COST_FEATURES, CONF_ATTEND, CONF_ENLARGE, CONF_COMBINE, CONF_SIGMOID = 1, 2, 3, 4, 5


class EsmSrc(Structure):
    _fields_ = [("ptr", c_void_p), ("C", c_int32), ("reserved", c_int32),
                ("sb", c_int64), ("sc", c_int64), ("sd", c_int64), ("sh", c_int64)]


class EsmConvDesc(Structure):
    _fields_ = [
        ("src", EsmSrc * MAX_SRC), ("nsrc", c_int32), ("B", c_int32), ("Cin", c_int32),
        ("Di", c_int32), ("Hi", c_int32), ("Wi", c_int32),
        ("Do", c_int32), ("Ho", c_int32), ("Wo", c_int32),
        ("kd", c_int32), ("kh", c_int32), ("kw", c_int32),
        ("stride", c_int32), ("transposed", c_int32),
        ("pd", c_int32), ("ph", c_int32), ("pw", c_int32),
        ("Cout", c_int32), ("cin_pad", c_int32), ("cout_pad", c_int32),
        ("w", c_void_p), ("scale", c_void_p), ("shift", c_void_p),
        ("act", c_int32), ("shuffle", c_int32),
        ("mul", c_void_p), ("mb", c_int64), ("mc", c_int64), ("mh", c_int64),
        ("res", c_void_p), ("rb", c_int64), ("rc", c_int64), ("rd", c_int64), ("rh", c_int64),
        ("out", c_void_p), ("ob", c_int64), ("oc", c_int64), ("od", c_int64), ("oh", c_int64),
        ("up", c_void_p), ("up_h", c_int32), ("up_w", c_int32), ("up_f", c_int32), ("hint", c_int32),
        ("ub", c_int64), ("uh", c_int64),
        ("post_scale", c_float), ("post_scale2", c_float), ("out2", c_void_p),
        ("pre", c_void_p), ("prb", c_int64), ("prc", c_int64), ("prh", c_int64),
    ]


class EsmSmixStage(Structure):
    _fields_ = [("ln_w", c_void_p), ("fc0_w", c_void_p), ("fc0_b", c_void_p), ("fc2_w", c_void_p),
                ("fc2_b", c_void_p)]


class EsmSmixDesc(Structure):
    _fields_ = [("x", c_void_p), ("out", c_void_p), ("res", c_void_p), ("dw_w", c_void_p), ("dw_b", c_void_p),
                ("dw_k", c_int32), ("nstages", c_int32), ("stage", EsmSmixStage * SMIX_MAX_STAGES),
                ("B", c_int32), ("C", c_int32), ("H", c_int32), ("W", c_int32)]


class EsmFmnetDesc(Structure):
    _fields_ = [("x", c_void_p), ("out", c_void_p), ("dw_w", c_void_p * 2), ("dw_b", c_void_p * 2),
                ("dw_k", c_int32), ("reserved", c_int32), ("stage", EsmSmixStage * 4),
                ("B", c_int32), ("C", c_int32), ("H", c_int32), ("W", c_int32),
                ("conv0_w", c_void_p), ("conv0_b", c_void_p), ("conv2_w", c_void_p), ("conv2_b", c_void_p),
                ("hid", c_int32), ("reserved2", c_int32), ("work", c_void_p)]


class EsmShuffleTailDesc(Structure):
    _fields_ = [("x", c_void_p), ("xb", c_int64), ("xc", c_int64), ("xh", c_int64),
                ("up_w", c_void_p), ("up_b", c_void_p), ("tail_w", c_void_p), ("tail_b", c_void_p),
                ("out", c_void_p), ("ob", c_int64), ("oh", c_int64),
                ("B", c_int32), ("nf", c_int32), ("H", c_int32), ("W", c_int32), ("r", c_int32),
                ("flags", c_int32)]


class EsmShuffleConvDesc(Structure):
    _fields_ = [("st", EsmShuffleTailDesc), ("w", c_void_p), ("scale", c_void_p), ("shift", c_void_p),
                ("out", c_void_p), ("ob", c_int64), ("oc", c_int64), ("oh", c_int64),
                ("C", c_int32), ("cin_pad", c_int32), ("cout_pad", c_int32), ("reserved", c_int32),
                ("pre_x", c_void_p), ("pb", c_int64), ("pc", c_int64), ("ph", c_int64), ("pre_w", c_void_p),
                ("pre_scale", c_void_p), ("pre_shift", c_void_p), ("pre_cin", c_int32), ("pre_cin_pad", c_int32),
                ("pre_cout_pad", c_int32), ("pre_reserved", c_int32), ("w2", c_void_p), ("scale2", c_void_p),
                ("shift2", c_void_p), ("cin_pad2", c_int32), ("cout_pad2", c_int32)]


class EsmConfDesc(Structure):
    _fields_ = [("op", c_int32), ("B", c_int32), ("C", c_int32), ("D", c_int32), ("H", c_int32), ("W", c_int32),
                ("x", c_void_p * 4), ("out", c_void_p)]


class EsmDwconvDesc(Structure):
    _fields_ = [("x", c_void_p), ("xb", c_int64), ("xc", c_int64), ("xh", c_int64), ("w", c_void_p),
                ("scale", c_void_p), ("shift", c_void_p), ("out", c_void_p), ("ob", c_int64), ("oc", c_int64),
                ("oh", c_int64), ("B", c_int32), ("C", c_int32), ("H", c_int32), ("W", c_int32), ("K", c_int32),
                ("stride", c_int32), ("pad", c_int32), ("act", c_int32), ("Ho", c_int32), ("Wo", c_int32)]


# name -> (restype, argtypes); every symbol declared in include/esmstereo_amd.h
SIGNATURES = {
    "esm_last_error": (ctypes.c_char_p, []),
    "esm_version": (c_int, []),
    "esm_struct_size": (c_int, [c_int]),
    "esm_gwc_volume_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 6 + [c_void_p]),
    "esm_gwc_stem_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_int, c_int, c_void_p]),
    "esm_concat_volume_f32": (c_int, [c_void_p, c_void_p, c_void_p] + [c_int] * 5 + [c_void_p]),
    "esm_normcorr_volume_f32": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 5 + [c_void_p]),
    "esm_disp_regression_f32": (c_int, [c_void_p, c_void_p] + [c_int] * 4 + [c_void_p]),
    "esm_topk2_regression_f32": (c_int, [c_void_p, c_void_p, c_void_p] + [c_int] * 4 + [c_void_p]),
    "esm_topk_regression_f32": (c_int, [c_void_p, c_void_p, c_void_p] + [c_int] * 5 + [c_void_p]),
    "esm_conv_f32": (c_int, [POINTER(EsmConvDesc), c_void_p]),
    "esm_smix_f32": (c_int, [POINTER(EsmSmixDesc), c_void_p]),
    "esm_fmnet_f32": (c_int, [POINTER(EsmFmnetDesc), c_void_p]),
    "esm_shuffle_tail_f32": (c_int, [POINTER(EsmShuffleTailDesc), c_void_p]),
    "esm_shuffle_conv_f32": (c_int, [POINTER(EsmShuffleConvDesc), c_void_p]),
    "esm_conv_pair2_f32": (c_int, [POINTER(EsmConvDesc), POINTER(EsmConvDesc), c_void_p]),
    "esm_convt_1x1_f32": (c_int, [POINTER(EsmConvDesc), POINTER(EsmConvDesc), c_void_p]),
    "esm_conf_f32": (c_int, [POINTER(EsmConfDesc), c_void_p]),
    "esm_dwconv_f32": (c_int, [POINTER(EsmDwconvDesc), c_void_p]),
    "esm_preprocess_u8": (c_int, [c_void_p, c_void_p] + [c_int] * 8 + [c_void_p]),
    "esm_disp_to_u16": (c_int, [c_void_p, c_void_p] + [c_int] * 7 + [c_void_p]),
    "esm_node_filter_u16": (c_int, [c_void_p, c_void_p, c_void_p] + [c_int] * 7 + [c_float, c_void_p]),
    "esm_plan_create": (c_void_p, []),
    "esm_plan_destroy": (None, [c_void_p]),
    "esm_plan_add_conv": (c_int, [c_void_p, POINTER(EsmConvDesc)]),
    "esm_plan_add_smix": (c_int, [c_void_p, POINTER(EsmSmixDesc)]),
    "esm_plan_add_fmnet": (c_int, [c_void_p, POINTER(EsmFmnetDesc)]),
    "esm_plan_add_shuffle_tail": (c_int, [c_void_p, POINTER(EsmShuffleTailDesc)]),
    "esm_plan_add_shuffle_conv": (c_int, [c_void_p, POINTER(EsmShuffleConvDesc)]),
    "esm_plan_add_conv_pair2": (c_int, [c_void_p, POINTER(EsmConvDesc), POINTER(EsmConvDesc)]),
    "esm_plan_add_convt_1x1": (c_int, [c_void_p, POINTER(EsmConvDesc), POINTER(EsmConvDesc)]),
    "esm_plan_set_branch": (c_int, [c_void_p, c_int, c_int]),
    "esm_plan_set_join": (c_int, [c_void_p, c_int, c_int]),
    "esm_plan_add_gwc": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 6),
    "esm_plan_add_gwc_stem": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int]),
    "esm_plan_add_concat": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 5),
    "esm_plan_add_normcorr": (c_int, [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p] + [c_int] * 5),
    "esm_plan_add_regression": (c_int, [c_void_p, c_int, c_void_p, c_void_p] + [c_int] * 4),
    "esm_plan_add_conf": (c_int, [c_void_p, POINTER(EsmConfDesc)]),
    "esm_plan_num_ops": (c_int, [c_void_p]),
    "esm_plan_op_kind": (c_int, [c_void_p, c_int]),
    "esm_plan_set_conv_hint": (c_int, [c_void_p, c_int, c_int]),
    "esm_plan_set_repeat": (c_int, [c_void_p, c_int, c_int]),
    "esm_plan_run": (c_int, [c_void_p, c_void_p]),
    "esm_plan_run_op": (c_int, [c_void_p, c_int, c_int, c_void_p]),
    "esm_plan_graph_build": (c_int, [c_void_p, c_void_p]),
    "esm_plan_graph_launch": (c_int, [c_void_p, c_void_p]),
    "esm_plan_rebind": (c_int, [c_void_p, c_int, POINTER(c_void_p), POINTER(ctypes.c_uint64), POINTER(c_void_p)]),
    "esm_plan_busy": (c_int, [c_void_p]),
    "esm_plan_set_probe": (c_int, [c_void_p, c_int, c_int]),
    "esm_plan_probe_read": (c_int, [c_void_p, POINTER(c_float), c_int]),
}


class EsmError(RuntimeError):
    """A non-zero status from the HIP library."""


def _load() -> ctypes.CDLL:
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"esmstereo_amd: native library {LIB_PATH} not found. Build it with "
            "`python esmstereo_amd/build.py` (hipcc --offload-arch=gfx950); there is no fallback.")
    lib = ctypes.CDLL(LIB_PATH)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    for which, st in ((0, EsmSrc), (1, EsmConvDesc), (2, EsmSmixStage), (3, EsmSmixDesc), (4, EsmShuffleTailDesc),
                      (5, EsmFmnetDesc), (6, EsmConfDesc), (8, EsmShuffleConvDesc), (9, EsmDwconvDesc)):
        if lib.esm_struct_size(which) != ctypes.sizeof(st):
            raise ImportError(f"esmstereo_amd: ABI mismatch for {st.__name__}: "
                              f"C {lib.esm_struct_size(which)} vs ctypes {ctypes.sizeof(st)}")
    return lib


lib = _load()


def check(rc: int, what: str = "esmstereo_amd") -> int:
    if rc < 0:
        msg = lib.esm_last_error()
        raise EsmError(f"{what}: status {rc}: {msg.decode() if msg else ''}")
    return rc
