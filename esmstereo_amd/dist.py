"""Batch sharding of the hot path over the GPUs of one node.

Stereo pairs are independent in eval mode, so a global batch splits into contiguous slices,
one per rank (one process per GPU); the only exchange is gathering the disparity maps.  Over
RCCL (backend "nccl" on ROCm) that is one ``all_gather_into_tensor`` over xGMI; over gloo
(CPU tests) the list form of ``all_gather``.  Uneven batches are padded to the largest slice
for the collective and trimmed after it.
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.distributed as dist


def shard_range(batch: int, world: int, rank: int) -> Tuple[int, int]:
    """[lo, hi) of ``rank``'s contiguous slice of a ``batch``-pair global batch; the first
    ``batch % world`` ranks take one extra pair."""
    if world < 1 or not 0 <= rank < world:
        raise ValueError(f"shard_range: rank {rank} outside world {world}")
    if batch < 0:
        raise ValueError("shard_range: negative batch")
    base, extra = divmod(batch, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def shard(t: torch.Tensor, world: Optional[int] = None, rank: Optional[int] = None) -> torch.Tensor:
    """This rank's slice (a view) of a global-batch tensor."""
    world = dist.get_world_size() if world is None else world
    rank = dist.get_rank() if rank is None else rank
    lo, hi = shard_range(int(t.shape[0]), world, rank)
    return t[lo:hi]


def gather_disparities(local: torch.Tensor, batch: int, group=None) -> torch.Tensor:
    """Concatenate every rank's ``[b_r, ...]`` result into the ``[batch, ...]`` global result
    on every rank (rank order = batch order)."""
    world = dist.get_world_size(group)
    rows = [shard_range(batch, world, r) for r in range(world)]
    mx = max(hi - lo for lo, hi in rows)
    me = dist.get_rank(group)
    if local.shape[0] != rows[me][1] - rows[me][0]:
        raise ValueError(f"gather_disparities: rank {me} holds {local.shape[0]} pairs, expected "
                         f"{rows[me][1] - rows[me][0]}")
    buf = local.contiguous()
    if buf.shape[0] < mx:  # pad to a uniform slice for the collective
        buf = torch.cat([buf, buf.new_zeros((mx - buf.shape[0],) + tuple(buf.shape[1:]))])
    if dist.get_backend(group) == "nccl":
        full = buf.new_empty((world * mx,) + tuple(buf.shape[1:]))
        dist.all_gather_into_tensor(full, buf, group=group)
        parts = full.split(mx)
    else:
        parts = [torch.empty_like(buf) for _ in range(world)]
        dist.all_gather(parts, buf, group=group)
    return torch.cat([p[: hi - lo] for p, (lo, hi) in zip(parts, rows)])


def sharded_forward(model, left: torch.Tensor, right: torch.Tensor, group=None) -> torch.Tensor:
    """Eval forward of a global batch split across the ranks of ``group``: every rank runs its
    slice through ``model`` and receives the full ``[B, H, W]`` disparity batch."""
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    lo, hi = shard_range(int(left.shape[0]), world, rank)
    if hi == lo:  # fewer pairs than ranks: nothing to run here, but every rank joins the gather
        disp = left.new_empty((0,) + tuple(left.shape[-2:]))
    else:
        with torch.no_grad():
            disp = model(left[lo:hi], right[lo:hi], False)[0]
    return gather_disparities(disp, int(left.shape[0]), group)


# ----------------------------------------------------------------------------- timed multi-rank steps
# The measurement loop of bench.py, kept here so that the same code runs under RCCL on the GPU node
# and under gloo in the CPU tests (tests/test_dist.py): W untimed warm-up steps, a barrier +
# device synchronisation, K timed steps, a barrier + synchronisation, and the elapsed time reduced
# to its maximum over the ranks.


def world_info(group=None) -> Tuple[int, int]:
    """(world size, rank); (1, 0) when torch.distributed is not initialised."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_world_size(group), dist.get_rank(group)
    return 1, 0


def local_batch(world: int, rank: int, batch: Optional[int] = None,
                global_batch: Optional[int] = None) -> Tuple[int, str, int]:
    """(pairs this rank runs per step, "weak" | "strong", pairs all ranks run per step).

    weak scaling: every rank runs ``batch`` pairs; strong scaling: ``global_batch`` pairs split
    into contiguous shards (``shard_range``), which must split evenly so every rank's step is the
    same work."""
    if (batch is None) == (global_batch is None):
        raise ValueError("local_batch: give exactly one of batch (weak) and global_batch (strong)")
    if global_batch is not None:
        if global_batch % world:
            raise ValueError(f"global batch {global_batch} must split evenly over {world} ranks")
        lo, hi = shard_range(global_batch, world, rank)
        return hi - lo, "strong", global_batch
    return batch, "weak", batch * world


def _sync(device: torch.device) -> None:
    if device.type == "cuda":
        torch.cuda.synchronize(device)


class DisparityGather:
    """Per-step exchange of the ranks' disparity maps into one preallocated ``[world, *shape]``
    buffer: ``all_gather_into_tensor`` over RCCL, the list form over gloo.  Every rank holds the
    same number of pairs (``local_batch`` enforces it), so no padding is needed on the hot loop."""

    def __init__(self, local: torch.Tensor, group=None, collective: Optional[bool] = None):
        """``collective``: exchange through the process group even at world size 1 (default: only
        when there is more than one rank; the single-GPU RCCL test forces it)."""
        self.group = group
        self.world, _ = world_info(group)
        self.buf = local.new_empty((self.world,) + tuple(local.shape))
        self.collective = self.world > 1 if collective is None else bool(collective)
        if self.collective and not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("DisparityGather: collective exchange needs an initialised process group")
        self.nccl = self.collective and dist.get_backend(group) == "nccl"

    def __call__(self, local: torch.Tensor) -> torch.Tensor:
        if not self.collective:
            self.buf[0].copy_(local)
        elif self.nccl:
            dist.all_gather_into_tensor(self.buf, local, group=self.group)
        else:
            dist.all_gather(list(self.buf.unbind(0)), local, group=self.group)
        return self.buf


def max_over_ranks(value: float, device: torch.device, group=None) -> float:
    """The largest ``value`` over the ranks (the slowest rank bounds a synchronous step)."""
    world, _ = world_info(group)
    if world == 1:
        return float(value)
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def timed_steps(step, steps: int, warmup: int, device: torch.device, group=None) -> float:
    """Run ``step()`` ``warmup`` times untimed, then ``steps`` times between two
    barrier + synchronise brackets; returns the max-over-ranks wall time of the timed steps (s)."""
    import time

    world, _ = world_info(group)
    for _ in range(warmup):
        step()
    _sync(device)
    if world > 1:
        dist.barrier(group=group)
    _sync(device)
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    _sync(device)
    if world > 1:
        dist.barrier(group=group)
    elapsed = time.perf_counter() - t0
    return max_over_ranks(elapsed, device, group)
