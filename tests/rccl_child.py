"""Child process of tests/test_gpu_dist.py (not a test module): a ONE-rank RCCL process group on cuda:0
(backend "nccl" is RCCL on ROCm), initialised with ``device_id`` as bench.py does, and the collective
branches of esmstereo_amd.dist driven through it: ``gather_disparities`` (all_gather_into_tensor),
``DisparityGather`` forced onto the collective, and ``sharded_forward`` of the hot path (reference
``test_kitti.py:18,53`` runs one GPU; SURVEY.md §8(e) shards the batch).  Prints RCCL-OK on success."""
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import esmstereo_amd as E  # noqa: E402
from esmstereo_amd import dist as D  # noqa: E402
from esmstereo_amd.backbone import StubFeature  # noqa: E402
from helpers import load_spec, seeded_state  # noqa: E402


def main() -> None:
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev)
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    g = torch.Generator(device="cpu").manual_seed(7)
    x = torch.randn(3, 40, 72, generator=g).to(dev)
    full = D.gather_disparities(x, 3)  # the nccl branch: all_gather_into_tensor
    assert torch.equal(full, x)
    gath = D.DisparityGather(x, collective=True)
    assert gath.nccl
    assert torch.equal(gath(x)[0], x)
    model = E.ESMStereo(64, True, False, "mobilenetv2_100", 16, feature_cls=StubFeature)
    model.load_state_dict(seeded_state(load_spec("spec_S_gwc.json"), 11))
    model = model.eval().to(dev)
    left = torch.randn(2, 3, 64, 128, generator=g).to(dev)
    right = torch.randn(2, 3, 64, 128, generator=g).to(dev)
    with torch.no_grad():
        ref = model(left, right, False)[0]
    got = D.sharded_forward(model, left, right)
    torch.cuda.synchronize()
    assert got.shape == ref.shape and torch.equal(got, ref), float((got - ref).abs().max())
    t = torch.tensor([2.5], dtype=torch.float64, device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    assert D.max_over_ranks(1.25, dev) == 1.25
    dist.barrier()
    dist.destroy_process_group()
    print("RCCL-OK", flush=True)


if __name__ == "__main__":
    main()
