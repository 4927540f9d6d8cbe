"""GPU parity of the input / output kernels (csrc/io.hip) against the CPU oracle (oracle/io_oracle.py):
bit-exact (same fp32 operation sequence; integer rounding)."""
import numpy as np
import pytest
import torch

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not torch.cuda.is_available(), reason="needs a ROCm GPU")]

from esmstereo_amd import io as EIO  # noqa: E402
from oracle import io_oracle as IO  # noqa: E402

DEV = torch.device("cuda")


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("h,w", [(375, 1242), (370, 1224), (376, 1241), (64, 96), (1, 1)])
def test_kitti_test_transform_bit_exact(h, w):
    u8 = _img(h, w, h * 7 + w)
    x, pads = EIO.kitti_test_transform(torch.from_numpy(u8).to(DEV))
    ref, rpads = IO.kitti_test_transform(u8)
    assert pads == rpads
    assert np.array_equal(x[0].cpu().numpy(), ref)


def test_kitti_test_transform_batch():
    u8 = np.stack([_img(100, 150, s) for s in range(3)])
    x, _ = EIO.kitti_test_transform(torch.from_numpy(u8).to(DEV))
    for b in range(3):
        assert np.array_equal(x[b].cpu().numpy(), IO.kitti_test_transform(u8[b])[0])


@pytest.mark.parametrize("h,w", [(375, 1242), (370, 1224), (352, 1216)])
def test_kitti_dataset_transform_bit_exact(h, w):
    u8 = _img(h, w, 11 + h)
    x, top_pad, right_pad = EIO.kitti_dataset_transform(torch.from_numpy(u8).to(DEV))
    ref, rt, rr = IO.kitti_dataset_transform(u8)
    assert (top_pad, right_pad) == (rt, rr)
    assert np.array_equal(x[0].cpu().numpy(), ref)
    with pytest.raises(AssertionError):  # the reference asserts positive pads
        EIO.kitti_dataset_transform(torch.from_numpy(_img(384, 1000, 0)).to(DEV))


def test_disparity_to_u16_bit_exact():
    g = torch.Generator().manual_seed(5)
    d = torch.rand(2, 384, 1248, generator=g) * 200
    d[0, 10, :8] = torch.tensor([0.0, 1 / 512, 3 / 512, 5 / 512, 100.25, 7 / 512, 255.998, 2.5 / 256])  # ties
    got = EIO.disparity_to_u16(d.to(DEV), 9, 6, 375, 1242).cpu().numpy()
    assert got.dtype == np.uint16
    assert np.array_equal(got, IO.disp_to_u16(d.numpy(), 9, 6, 375, 1242))
    whole = EIO.disparity_to_u16(d.to(DEV), 0, 0, 384, 1248).cpu().numpy()
    assert np.array_equal(whole, IO.disp_to_u16(d.numpy(), 0, 0, 384, 1248))


def test_round_trip_through_png(tmp_path):
    from PIL import Image

    d = torch.rand(1, 96, 128, device=DEV) * 150
    u16 = EIO.disparity_to_u16(d, 0, 0, 96, 128)[0]
    p = tmp_path / "disp.png"
    EIO.write_png_u16(str(p), u16)
    back = np.asarray(Image.open(p)).astype(np.uint16)
    assert np.array_equal(back, u16.cpu().numpy())
    # KITTI devkit reading convention (test_kitti.py:108): png / 256
    assert np.abs(back / 256.0 - d[0].cpu().numpy()).max() <= 0.5 / 256 + 1e-6
