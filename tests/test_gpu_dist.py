"""The multi-GPU code path executed on ROCm with RCCL.  The pool's boxes have one GPU,
so the process group has one rank, but every call is the N > 1 one: ``init_process_group("nccl",
device_id=...)`` (bench.py), ``all_gather_into_tensor`` (esmstereo_amd.dist gather_disparities,
DisparityGather forced onto the collective) and ``sharded_forward``.  Each runs in a child process
(a process group is per process; the test runner keeps none)."""
import os
import socket
import subprocess
import sys
import json

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _env() -> dict:
    env = dict(os.environ, RANK="0", LOCAL_RANK="0", WORLD_SIZE="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(_port()), HSA_ENABLE_IPC_MODE_LEGACY="0")
    return env


@pytest.mark.gpu
def test_rccl_one_rank_collectives():
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "tests", "rccl_child.py")], env=_env(), cwd=ROOT,
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0 and "RCCL-OK" in r.stdout, (r.stdout[-2000:], r.stderr[-4000:])


@pytest.mark.gpu
def test_bench_dist_path_one_rank():
    """bench.py's rank code under RCCL: init with device_id, the timed steps with the per-step
    all_gather_into_tensor of the disparities, barrier + max over ranks."""
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--dist", "--steps", "5", "--warmup", "2",
                        "--no-extra", "--no-cpu-baseline", "--no-marginal"], env=_env(), cwd=ROOT,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    line = json.loads([x for x in r.stdout.splitlines() if x.startswith('{"metric"')][-1])
    assert line["n_gpus"] == 1 and line["value"] > 0
    assert line["collective"] and line["collective"].startswith("nccl all_gather_into_tensor"), line.get("collective")
