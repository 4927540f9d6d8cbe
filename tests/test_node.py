"""The ROS-node analogue (esmstereo_amd/node.py, kitti_publisher_cuda_node.cpp:136-175,323-430).

CPU: the oracle restatement of the node's steps (pads, medianBlur, mask, 16-bit conversion) checked
against independent implementations (scipy's median filter).  GPU (-m gpu): the device filter is
bit-exact with the oracle, and StereoNode.process reproduces model output -> oracle filter."""
import numpy as np
import pytest
import scipy.ndimage
import torch

from oracle import io_oracle as IO


def test_node_pads_always_next_multiple():
    assert IO.node_pads(375, 1242) == (9, 6)
    assert IO.node_pads(384, 1248) == (32, 32)  # divisible sizes still gain a block (:141-146)


def test_median_oracle_matches_scipy():
    rng = np.random.default_rng(0)
    d = rng.standard_normal((23, 41)).astype(np.float32)
    assert np.array_equal(IO.median5_replicate(d), scipy.ndimage.median_filter(d, size=5, mode="nearest"))


def test_node_filter_oracle_mask_and_rounding():
    d = np.zeros((8, 8), np.float32)
    d[:] = 3.5 / 256  # d*256 = 3.5 -> rint to even = 4
    d[0, 0] = -1
    u, m = IO.node_filter_u16(d, 0, 0, 8, 8, 192.0)
    assert u.dtype == np.uint16 and (u == 4).all()
    big = np.full((8, 8), 300.0, np.float32)
    u, m = IO.node_filter_u16(big, 0, 0, 8, 8, 192.0)
    assert (u == 0).all() and (m == 0).all()  # outside (0, max_disp) -> 0


@pytest.mark.gpu
def test_node_filter_kernel_bit_exact():
    from esmstereo_amd._lib import check, lib
    dev = torch.device("cuda")
    rng = np.random.default_rng(1)
    Hp, Wp, top, left, h, w = 40, 70, 3, 5, 31, 59
    d = rng.uniform(-20, 220, (2, Hp, Wp)).astype(np.float32)
    d[0, 10, 10:20] = np.float32(2.5 / 256)  # half-way rounding cases
    dd = torch.from_numpy(d).to(dev)
    out = torch.empty(2, h, w, dtype=torch.int16, device=dev)
    filt = torch.empty(2, h, w, device=dev)
    check(lib.esm_node_filter_u16(dd.data_ptr(), out.data_ptr(), filt.data_ptr(), 2, Hp, Wp, top, left, h, w, 192.0,
                                  None), "node_filter")
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    for b in range(2):
        ref_u, ref_m = IO.node_filter_u16(d[b], top, left, h, w, 192.0)
        assert np.array_equal(got[b], ref_u)
        assert np.array_equal(filt[b].cpu().numpy(), ref_m)


@pytest.mark.gpu
def test_stereo_node_process_end_to_end():
    import json
    import os
    import esmstereo_amd as E
    from esmstereo_amd.backbone import StubFeature
    from esmstereo_amd.node import StereoNode
    from helpers import GOLDEN_DIR, load_spec, seeded_state
    with open(os.path.join(GOLDEN_DIR, "manifest.json")) as f:
        m = json.load(f)["hot_S_gwc.npz"]
    dev = torch.device("cuda")
    model = E.ESMStereo_trt(192, True, False, m["backbone"], 16, feature_cls=StubFeature)
    model.load_state_dict(seeded_state(load_spec(m["spec"]), m["seed"]))
    model = model.eval().to(dev)
    H, W = 100, 220
    rng = np.random.default_rng(2)
    left = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
    right = np.roll(left, -6, axis=1)
    node = StereoNode(model, H, W, max_disp=192.0)
    u16, ms = node.process(left, right)
    assert u16.shape == (H, W) and u16.dtype == np.uint16 and ms > 0
    # the same frames through the oracle's preprocessing, the model, and the oracle's filter
    x = [torch.from_numpy(np.ascontiguousarray(IO.node_preprocess(a))).unsqueeze(0).to(dev) for a in (left, right)]
    assert torch.equal(node.net_in[0], x[0]) and torch.equal(node.net_in[1], x[1])
    with torch.no_grad():
        disp = model(x[0], x[1])[0].cpu().numpy()
    ref, _ = IO.node_filter_u16(disp, 0, 0, H, W, 192.0)
    assert np.array_equal(u16, ref)
    # the loop form yields one result per pair
    outs = list(node.run([(left, right), (right, left)]))
    assert len(outs) == 2 and np.array_equal(outs[0][0], u16)
