"""Build the gfx950 shared library ``esmstereo_amd/libesmstereo_amd.so`` in-tree.

``python esmstereo_amd/build.py`` (or ``__graft_entry__.build()``) compiles every
``csrc/*.hip`` with ``hipcc --offload-arch=gfx950`` into objects (in parallel, skipping
up-to-date ones) and links one C-ABI shared library.  No torch headers are involved: the
library's interface is ``include/esmstereo_amd.h``.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIB = os.path.join(PKG, "libesmstereo_amd.so")
HEADER = os.path.join(ROOT, "include", "esmstereo_amd.h")
ARCH = os.environ.get("ESM_OFFLOAD_ARCH", "gfx950")
CXXFLAGS = ["-O3", "-fPIC", "-std=c++17", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result"]


def _hipcc() -> str:
    h = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(h):
        raise RuntimeError("hipcc not found: the esmstereo_amd HIP library cannot be built")
    return h


def _deps():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith(".h")] + [HEADER]


# diagnostic build (per-wave timeline stamps in the direct conv kernels): separate objects and
# library, loaded only when ESM_LIB points at it; never used for results
DIAG_BUILD = os.path.join(PKG, "_build_diag")
DIAG_LIB = os.path.join(DIAG_BUILD, "libesmstereo_amd.so")


def _stale(obj: str, src: str) -> bool:
    if not os.path.exists(obj):
        return True
    t = os.path.getmtime(obj)
    return any(os.path.getmtime(p) > t for p in [src] + _deps())


# kernels whose results must be bit-exact with the reference's separately rounded ops
NO_CONTRACT = {"volumes.hip", "regression.hip"}


def _compile(src: str, obj: str, defines=()) -> str:
    extra = ["-ffp-contract=off"] if os.path.basename(src) in NO_CONTRACT else []
    extra += [f"-D{d}" for d in defines]
    cmd = [_hipcc()] + CXXFLAGS + extra + ["-c", src, "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc failed for {os.path.basename(src)}:\n{r.stderr}")
    return obj


def build(verbose: bool = False, jobs: int = 8, diag: bool = False) -> str:
    bdir, lib_path = (DIAG_BUILD, DIAG_LIB) if diag else (BUILD, LIB)
    defines = ("ESM_CONV_STAMPS",) if diag else ()
    os.makedirs(bdir, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    objs = []
    todo = []
    for f in srcs:
        src = os.path.join(CSRC, f)
        obj = os.path.join(bdir, f[:-4] + ".o")
        objs.append(obj)
        if _stale(obj, src):
            todo.append((src, obj))
    if todo:
        with cf.ThreadPoolExecutor(max_workers=max(1, min(jobs, len(todo)))) as ex:
            for fut in [ex.submit(_compile, s, o, defines) for s, o in todo]:
                o = fut.result()
                if verbose:
                    print("compiled", os.path.relpath(o, ROOT))
    if todo or not os.path.exists(lib_path) or any(os.path.getmtime(o) > os.path.getmtime(lib_path) for o in objs):
        tmp = lib_path + ".tmp"
        cmd = [_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmp] + objs
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed:\n{r.stderr}")
        os.replace(tmp, lib_path)
        if verbose:
            print("linked", os.path.relpath(lib_path, ROOT))
    return lib_path


if __name__ == "__main__":
    build(verbose=True, diag="--diag" in sys.argv)
    sys.exit(0)
