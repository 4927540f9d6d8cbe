"""The steps on either side of the hot path, on device-resident data.

Input side — the reference turns an 8-bit RGB image into the network input two ways:

* ``kitti_test_transform`` — test_kitti.py:93-106 (and test_mid / save_vid / latest): PIL
  ``crop((w - wi, h - hi, w, h))`` pads the uint8 image with zeros at the TOP-LEFT to
  ``wi, hi = (w // 32 + 1) * 32, (h // 32 + 1) * 32``, then ``ToTensor`` + ``Normalize`` — so the
  padding holds ``(0 - mean) / std``; the prediction is cropped back with
  ``pred[:, hi - h:, wi - w:]`` (test_kitti.py:115).
* ``kitti_dataset_transform`` — datasets/kitti_dataset.py:151-170 (the loader of save_disp.py):
  ``ToTensor`` + ``Normalize`` first, then ``np.pad`` with 0.0 at the TOP and RIGHT to 384 x 1248;
  the prediction is cropped back with ``disp[top_pad:, :-right_pad]`` (save_disp.py:81).

Output side — ``disparity_to_u16``: ``np.round(disp * 256).astype(np.uint16)`` of the cropped map
(save_disp.py:85), and ``write_png_u16`` writes it as the 16-bit grayscale PNG that
``skimage.io.imsave`` produces there (save_disp.py:86; skimage is not a dependency here).

Both transforms and the rounding are one HIP launch each (``csrc/io.hip``), bit-exact with the
torchvision / numpy arithmetic; there is no CPU fallback.
"""
from __future__ import annotations

import struct
import zlib
from typing import Tuple

import numpy as np
import torch

from ._lib import check, lib

IMAGENET_MEAN = (0.485, 0.456, 0.406)  # datasets/data_io.py:8
IMAGENET_STD = (0.229, 0.224, 0.225)   # datasets/data_io.py:9


def _as_batch_u8(img: torch.Tensor) -> torch.Tensor:
    if img.dtype != torch.uint8:
        raise TypeError(f"expected a uint8 RGB image, got {img.dtype}")
    if img.dim() == 3:
        img = img.unsqueeze(0)
    if img.dim() != 4 or img.shape[-1] != 3:
        raise ValueError(f"expected [H, W, 3] or [B, H, W, 3] uint8, got {tuple(img.shape)}")
    if not img.is_cuda:
        raise RuntimeError("esmstereo_amd.io: the image must be on the GPU (no CPU fallback)")
    return img.contiguous()


def _stream(t: torch.Tensor):
    import ctypes

    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _pad_normalize(img: torch.Tensor, Hp: int, Wp: int, top: int, left: int, pad_normalized: bool) -> torch.Tensor:
    B, H, W, _ = img.shape
    out = torch.empty(B, 3, Hp, Wp, device=img.device, dtype=torch.float32)
    check(lib.esm_preprocess_u8(img.data_ptr(), out.data_ptr(), B, H, W, Hp, Wp, top, left, int(pad_normalized),
                                _stream(img)), "preprocess")
    return out


def kitti_test_size(h: int, w: int, m: int = 32) -> Tuple[int, int]:
    """Padded extent of test_kitti.py:94-95: ``(x // m + 1) * m`` (always at least one pixel of pad)."""
    return (h // m + 1) * m, (w // m + 1) * m


def kitti_test_transform(img: torch.Tensor) -> Tuple[torch.Tensor, Tuple[int, int]]:
    """uint8 RGB ``[H, W, 3]`` / ``[B, H, W, 3]`` on the GPU -> (input ``[B, 3, hi, wi]``, (top, left)).

    test_kitti.py:93-106; crop the prediction back with ``pred[:, top:, left:]``."""
    img = _as_batch_u8(img)
    h, w = int(img.shape[1]), int(img.shape[2])
    hi, wi = kitti_test_size(h, w)
    return _pad_normalize(img, hi, wi, hi - h, wi - w, True), (hi - h, wi - w)


def kitti_dataset_transform(img: torch.Tensor, size: Tuple[int, int] = (384, 1248)) -> Tuple[torch.Tensor, int, int]:
    """uint8 RGB on the GPU -> (input ``[B, 3, 384, 1248]``, top_pad, right_pad), as
    datasets/kitti_dataset.py:151-170 (which asserts both pads are positive)."""
    img = _as_batch_u8(img)
    h, w = int(img.shape[1]), int(img.shape[2])
    top_pad, right_pad = size[0] - h, size[1] - w
    if not (top_pad > 0 and right_pad > 0):
        raise AssertionError(f"kitti_dataset: image {h}x{w} does not fit {size[0]}x{size[1]} with a pad")
    return _pad_normalize(img, size[0], size[1], top_pad, 0, False), top_pad, right_pad


def disparity_to_u16(disp: torch.Tensor, top: int, left: int, h: int, w: int) -> torch.Tensor:
    """``np.round(disp[:, top:top+h, left:left+w] * 256).astype(np.uint16)`` on the GPU
    (save_disp.py:81,85; test_kitti.py:115 crop) -> uint16 ``[B, h, w]``."""
    if disp.dim() == 4 and disp.shape[1] == 1:
        disp = disp[:, 0]
    if disp.dim() == 2:
        disp = disp.unsqueeze(0)
    if disp.dim() != 3 or disp.dtype != torch.float32 or not disp.is_cuda:
        raise ValueError("disparity_to_u16: expected a float32 [B, H, W] GPU tensor")
    disp = disp.contiguous()
    B, Hp, Wp = (int(v) for v in disp.shape)
    out = torch.empty(B, h, w, device=disp.device, dtype=torch.int16)
    check(lib.esm_disp_to_u16(disp.data_ptr(), out.data_ptr(), B, Hp, Wp, top, left, h, w, _stream(disp)),
          "disp_to_u16")
    return out.view(torch.uint16)


def png_u16_bytes(a: np.ndarray) -> bytes:
    """A 16-bit grayscale PNG (big-endian samples, zlib-deflated, filter 0 per row) of ``a``."""
    a = np.ascontiguousarray(a, dtype=np.uint16)
    if a.ndim != 2:
        raise ValueError("png_u16_bytes: expected a 2-D array")
    h, w = a.shape
    raw = np.empty((h, 1 + 2 * w), dtype=np.uint8)
    raw[:, 0] = 0
    raw[:, 1:] = a.astype(">u2").view(np.uint8).reshape(h, 2 * w)

    def chunk(tag: bytes, data: bytes) -> bytes:
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    ihdr = struct.pack(">IIBBBBB", w, h, 16, 0, 0, 0, 0)
    return (b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", ihdr) + chunk(b"IDAT", zlib.compress(raw.tobytes(), 6)) +
            chunk(b"IEND", b""))


def write_png_u16(path: str, a) -> None:
    """``skimage.io.imsave(fn, disp_est_uint)`` of save_disp.py:86 for a uint16 map."""
    if isinstance(a, torch.Tensor):
        a = a.cpu().numpy()
    with open(path, "wb") as f:
        f.write(png_u16_bytes(a))
