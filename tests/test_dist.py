"""Multi-process (gloo, world size 2, CPU) tests of the batch-sharding / gather logic used by
bench.py and esmstereo_amd.dist.sharded_forward."""
from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from esmstereo_amd.dist import gather_disparities, shard, shard_range, sharded_forward


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
