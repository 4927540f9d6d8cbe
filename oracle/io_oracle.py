"""CPU oracle for the input / output steps around the hot path — TEST INFRASTRUCTURE, NOT PRODUCT.

Only ``tests/`` may import this module (as the checker).  A from-scratch numpy restatement of:

* ``kitti_test_transform``   test_kitti.py:93-106 — PIL ``crop((w - wi, h - hi, w, h))`` (zero
  padding of the uint8 image at the top-left; PIL is the reference's own image library and is
  used here for exactly that call), then torchvision ``ToTensor`` (``float32(u8) / 255``) and
  ``Normalize`` (``(x - mean) / std`` with fp32 mean/std, datasets/data_io.py:7-16);
* ``kitti_dataset_transform`` datasets/kitti_dataset.py:151-170 — ToTensor + Normalize, then
  ``np.lib.pad`` (numpy 2: ``np.pad``) with 0.0 at the top and right;
* ``disp_to_u16``             save_disp.py:81,85 — crop, ``np.round(disp * 256).astype(np.uint16)``.

torchvision itself is not installed, so its two transforms are restated from
their published definitions (``to_tensor``: ``img.to(float32).div(255)``; ``normalize``:
``tensor.sub_(mean).div_(std)``); parity against torchvision's own output is unpinned.
"""
from __future__ import annotations

import numpy as np
from PIL import Image

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def _to_tensor_normalize(u8_hwc: np.ndarray) -> np.ndarray:
    x = u8_hwc.astype(np.float32).transpose(2, 0, 1) / np.float32(255)
    return (x - MEAN[:, None, None]) / STD[:, None, None]


def kitti_test_transform(u8_hwc: np.ndarray):
    """-> ([3, hi, wi] float32, (hi - h, wi - w)); test_kitti.py:93-106."""
    h, w = u8_hwc.shape[:2]
    m = 32
    wi, hi = (w // m + 1) * m, (h // m + 1) * m
    img = Image.fromarray(np.ascontiguousarray(u8_hwc)).crop((w - wi, h - hi, w, h))
    return _to_tensor_normalize(np.asarray(img)), (hi - h, wi - w)


def kitti_dataset_transform(u8_hwc: np.ndarray, size=(384, 1248)):
    """-> ([3, 384, 1248] float32, top_pad, right_pad); kitti_dataset.py:151-170."""
    h, w = u8_hwc.shape[:2]
    x = _to_tensor_normalize(u8_hwc)
    top_pad, right_pad = size[0] - h, size[1] - w
    assert top_pad > 0 and right_pad > 0
    x = np.pad(x, ((0, 0), (top_pad, 0), (0, right_pad)), mode="constant", constant_values=0)
    return x, top_pad, right_pad


def disp_to_u16(disp: np.ndarray, top: int, left: int, h: int, w: int) -> np.ndarray:
    """save_disp.py:81,85 (window form, as test_kitti.py:115 crops)."""
    d = np.array(disp[..., top:top + h, left:left + w], dtype=np.float32)
    return np.round(d * 256).astype(np.uint16)
