"""CPU tests of the input / output steps around the hot path: the oracle's restatement of the
reference's PIL pad + normalise and its uint16 rounding, and the host PNG writer (read back with
PIL).  The HIP kernels themselves are checked against this oracle in test_gpu_io.py."""
import io

import numpy as np
from PIL import Image

from oracle import io_oracle as IO


def _img(h, w, seed):
    return np.random.default_rng(seed).integers(0, 256, size=(h, w, 3), dtype=np.uint8)


def test_oracle_test_kitti_pad_is_normalised_zero():
    u8 = _img(375, 1242, 0)
    x, (top, left) = IO.kitti_test_transform(u8)
    assert x.shape == (3, 384, 1248) and (top, left) == (9, 6)
    pad = ((np.float32(0) / np.float32(255)) - IO.MEAN) / IO.STD
    for c in range(3):
        assert np.all(x[c, :top, :] == pad[c]) and np.all(x[c, :, :left] == pad[c])
    ref = (u8.astype(np.float32).transpose(2, 0, 1) / np.float32(255) - IO.MEAN[:, None, None]) / IO.STD[:, None, None]
    assert np.array_equal(x[:, top:, left:], ref)
    # (w // 32 + 1) * 32 pads a multiple of 32 by a full 32 (test_kitti.py:94-95)
    assert IO.kitti_test_transform(_img(64, 96, 1))[0].shape == (3, 96, 128)


def test_oracle_kitti_dataset_pad_is_zero():
    x, top_pad, right_pad = IO.kitti_dataset_transform(_img(370, 1224, 2))
    assert x.shape == (3, 384, 1248) and (top_pad, right_pad) == (14, 24)
    assert np.all(x[:, :top_pad] == 0) and np.all(x[:, :, 1224:] == 0)


def test_oracle_u16_round_half_even():
    d = np.array([[0.0, 1 / 512, 3 / 512, 5 / 512, 100.25, 255.998]], dtype=np.float32)
    assert IO.disp_to_u16(d, 0, 0, 1, 6).tolist() == [[0, 0, 2, 2, 25664, 65535]]


def test_png_u16_writer_round_trip():
    from esmstereo_amd.io import png_u16_bytes

    a = np.random.default_rng(3).integers(0, 65536, size=(37, 53), dtype=np.uint16)
    a[0, 0], a[-1, -1] = 0, 65535
    img = Image.open(io.BytesIO(png_u16_bytes(a)))
    assert img.size == (53, 37)
    assert np.array_equal(np.asarray(img).astype(np.uint16), a)
