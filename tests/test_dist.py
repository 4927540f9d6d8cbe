"""Multi-process (gloo, world size 2, CPU) tests of the batch-sharding / gather / timing logic used by
bench.py and esmstereo_amd.dist.sharded_forward.  bench.py's multi-rank step is
esmstereo_amd.dist.{local_batch, DisparityGather, timed_steps}: the same functions run here under
gloo with a per-pair stand-in for the HIP hot path."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from esmstereo_amd.dist import (DisparityGather, gather_disparities, local_batch, max_over_ranks, shard, shard_range,
                                sharded_forward, timed_steps)


def test_shard_range_covers_batch_contiguously():
    for batch in (0, 1, 5, 8, 32, 33):
        for world in (1, 2, 3, 8):
            rows = [shard_range(batch, world, r) for r in range(world)]
            assert rows[0][0] == 0 and rows[-1][1] == batch
            assert all(a[1] == b[0] for a, b in zip(rows, rows[1:]))
            sizes = [hi - lo for lo, hi in rows]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        shard_range(4, 2, 2)


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


class _PairModel(torch.nn.Module):
    """Stands in for ESMStereo on CPU: a per-pair function, so sharding must not change it."""

    def forward(self, left, right, train_status):
        if left.shape[0] == 0:  # the HIP path refuses B = 0 ('conv: bad B/Cout'): so does this stand-in
            raise RuntimeError("empty batch")
        return [(left - right).abs().sum(1) * 4]


def _worker(rank, world, port, batch, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = torch.Generator().manual_seed(7)
        left = torch.randn(batch, 3, 8, 16, generator=g)
        right = torch.randn(batch, 3, 8, 16, generator=g)
        local = shard(left, world, rank)
        lo, hi = shard_range(batch, world, rank)
        assert torch.equal(local, left[lo:hi])
        full = gather_disparities((left[lo:hi] * 2).sum(1), batch)
        ok1 = torch.equal(full, (left * 2).sum(1))
        out = sharded_forward(_PairModel(), left, right)
        ok2 = torch.equal(out, _PairModel()(left, right, False)[0])
        q.put((rank, ok1, ok2, tuple(out.shape)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("batch", [4, 5, 1])
def test_gloo_world2_gather_and_sharded_forward(batch):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    codes = [p.exitcode for p in procs]
    assert codes == [0, 0], codes
    res = sorted(q.get(timeout=5) for _ in range(world))
    for rank, ok1, ok2, shape in res:
        assert ok1 and ok2, (rank, ok1, ok2)
        assert shape == (batch, 8, 16)


def test_local_batch_weak_and_strong():
    assert local_batch(8, 3, batch=1) == (1, "weak", 8)
    assert local_batch(8, 7, global_batch=32) == (4, "strong", 32)
    assert local_batch(1, 0, global_batch=32) == (32, "strong", 32)
    with pytest.raises(ValueError):
        local_batch(3, 0, global_batch=32)  # uneven shards: ranks would time different work
    with pytest.raises(ValueError):
        local_batch(2, 0)


def _bench_worker(rank, world, port, mode, q):
    """bench.py's measured loop with a CPU stand-in step: each rank runs its shard of synthetic pairs
    through a per-pair function, the disparities are gathered every step, rank 1 is made slower."""
    import time

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        b, scaling, total = local_batch(world, rank, **({"batch": 2} if mode == "weak" else {"global_batch": 6}))
        g = torch.Generator().manual_seed(100 + rank)  # per-rank synthetic input, as bench.py
        left, right = torch.randn(b, 3, 8, 16, generator=g), torch.randn(b, 3, 8, 16, generator=g)
        model = _PairModel()
        out = torch.empty(b, 8, 16)
        gather = DisparityGather(out)
        calls = []

        def step():
            out.copy_(model(left, right, False)[0])
            gather(out)
            calls.append(1)
            if rank == 1:
                time.sleep(0.02)

        el = timed_steps(step, steps=5, warmup=2, device=torch.device("cpu"))
        # every rank's gathered buffer holds every rank's result, in rank order
        allL = [torch.empty(b, 3, 8, 16) for _ in range(world)]
        allR = [torch.empty(b, 3, 8, 16) for _ in range(world)]
        dist.all_gather(allL, left)
        dist.all_gather(allR, right)
        ok = all(torch.equal(gather.buf[r], model(allL[r], allR[r], False)[0]) for r in range(world))
        q.put((rank, ok, el, len(calls), b, scaling, total, max_over_ranks(float(rank), torch.device("cpu"))))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["weak", "strong"])
def test_gloo_world2_bench_step(mode):
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=120)
    assert [p.exitcode for p in procs] == [0, 0]
    res = sorted(q.get(timeout=5) for _ in range(world))
    els = [r[2] for r in res]
    assert els[0] == els[1] and els[0] >= 5 * 0.02  # max over ranks: both report the slow rank's time
    for rank, ok, el, ncalls, b, scaling, total, mx in res:
        assert ok and ncalls == 7 and mx == 1.0
        assert scaling == mode and (b, total) == ((2, 4) if mode == "weak" else (3, 6))


def _bench(*argv, env=None, timeout=180):
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    e.update(env or {})
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), *argv], capture_output=True, text=True,
                       env=e, timeout=timeout)
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    return r.returncode, [json.loads(ln) for ln in lines], r.stderr


@pytest.mark.parametrize("extra,want", [((), (2, [2, 1, 8, 16], "weak")),
                                        (("--global-batch", "6"), (6, [2, 3, 8, 16], "strong"))])
def test_bench_launches_its_own_ranks(extra, want):
    """`python bench.py --gpus 2` with no launcher starts the 2 ranks itself: one JSON
    line from rank 0 with n_gpus 2, the per-step gather's [world, b, H, W] buffer, the pairs of both
    ranks counted.  The ranks run the real launcher / dist path with a gloo CPU stand-in step."""
    rc, lines, err = _bench("--gpus", "2", "--cpu-standin", "--steps", "3", "--warmup", "1", *extra)
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    line = lines[0]
    assert line["n_gpus"] == 2 and line["global_batch"] == want[0]
    assert line["gathered_shape"] == want[1] and line["scaling"] == want[2]
    assert line["gather_rank_order_ok"] is True
    assert line["value"] > 0


def test_bench_world8_configs3_strong_scaling():
    """configs[3]'s shape at world size 8: `bench.py --gpus 8 --global-batch 32` starts 8 gloo
    ranks with 4 pairs each, gathers [8, 4, H, W] every step in rank order, and counts all 32 pairs."""
    rc, lines, err = _bench("--gpus", "8", "--cpu-standin", "--global-batch", "32", "--steps", "3", "--warmup", "1",
                            timeout=300)
    assert rc == 0, err[-2000:]
    assert len(lines) == 1, lines
    line = lines[0]
    assert line["n_gpus"] == 8 and line["global_batch"] == 32 and line["scaling"] == "strong"
    assert line["gathered_shape"] == [8, 4, 8, 16]
    assert line["gather_rank_order_ok"] is True
    assert line["value"] > 0


def test_bench_gpus_must_match_launcher_world():
    rc, lines, err = _bench("--gpus", "1", "--cpu-standin", env={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert rc != 0 and not lines and "disagrees with WORLD_SIZE" in err


def test_bench_parent_reports_a_failing_rank():
    """A rank that fails makes the parent exit non-zero (and stops the other rank): a strong-scaling
    batch that does not split evenly raises in every rank."""
    rc, lines, err = _bench("--gpus", "2", "--cpu-standin", "--global-batch", "3", "--steps", "1", "--warmup", "0")
    assert rc != 0 and not lines
