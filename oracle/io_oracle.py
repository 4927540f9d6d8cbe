"""CPU oracle for the input / output steps around the hot path — TEST INFRASTRUCTURE, NOT PRODUCT.

Only ``tests/`` may import this module (as the checker).  A from-scratch numpy restatement of:

* ``kitti_test_transform``   test_kitti.py:93-106 — PIL ``crop((w - wi, h - hi, w, h))`` (zero
  padding of the uint8 image at the top-left; PIL is the reference's own image library and is
  used here for exactly that call), then torchvision ``ToTensor`` (``float32(u8) / 255``) and
  ``Normalize`` (``(x - mean) / std`` with fp32 mean/std, datasets/data_io.py:7-16);
* ``kitti_dataset_transform`` datasets/kitti_dataset.py:151-170 — ToTensor + Normalize, then
  ``np.lib.pad`` (numpy 2: ``np.pad``) with 0.0 at the top and right;
* ``disp_to_u16``             save_disp.py:81,85 — crop, ``np.round(disp * 256).astype(np.uint16)``;
* ``node_preprocess``          kitti_publisher_cuda_node.cpp:136-175 — pad right / bottom to the next
  multiple of 32 with zeros (``copyMakeBorder``), ``/ 255``, ``(x - mean) / std``, CHW;
* ``node_filter_u16``          kitti_publisher_cuda_node.cpp:385-403 — crop, ``cv::medianBlur(., 5)``
  (replicated border), valid mask ``(0, max_disp)``, ``convertTo(CV_16UC1, 256.0)``.

OpenCV is not installed either: the node's two OpenCV steps are restated from OpenCV's documented
semantics (medianBlur: exact 5x5 median with BORDER_REPLICATE; ``convertTo`` to 16U:
``saturate_cast<ushort>`` = round half to even, clamp to [0, 65535]); parity against OpenCV's own
output is unpinned.

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


def node_pads(h: int, w: int, m: int = 32):
    """(pad_bottom, pad_right) of kitti_publisher_cuda_node.cpp:141-146: wi = (w / m + 1) * m."""
    return (h // m + 1) * m - h, (w // m + 1) * m - w


def node_preprocess(u8_hwc: np.ndarray) -> np.ndarray:
    """kitti_publisher_cuda_node.cpp:136-175 -> [3, Hp, Wp] float32 (channel order as given)."""
    h, w, _ = u8_hwc.shape
    pb, pr = node_pads(h, w)
    padded = np.zeros((h + pb, w + pr, 3), dtype=np.uint8)
    padded[:h, :w] = u8_hwc
    return _to_tensor_normalize(padded)


def median5_replicate(d: np.ndarray) -> np.ndarray:
    """Exact 5x5 median of a 2-D float32 map with replicated borders (cv::medianBlur, ksize 5)."""
    p = np.pad(d, 2, mode="edge")
    h, w = d.shape
    stack = np.stack([p[dy:dy + h, dx:dx + w] for dy in range(5) for dx in range(5)], 0)
    return np.sort(stack, axis=0)[12]


def node_filter_u16(disp: np.ndarray, top: int, left: int, h: int, w: int, max_disp: float):
    """kitti_publisher_cuda_node.cpp:385-403 on one [Hp, Wp] disparity -> (uint16 [h, w], masked median)."""
    m = median5_replicate(np.ascontiguousarray(disp[top:top + h, left:left + w], dtype=np.float32))
    m = np.where((m > 0) & (m < np.float32(max_disp)), m, np.float32(0)).astype(np.float32)
    r = np.rint(m * np.float32(256))
    return np.clip(r, 0, 65535).astype(np.uint16), m
