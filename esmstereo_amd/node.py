"""HIP-runtime analogue of the reference's ROS2 stereo node loop
(``kitti_publisher/src/kitti_publisher_cuda_node.cpp:323-430``, ``preprocess_image`` ``:136-175``).

The reference node, per timer tick: reads a stereo pair (OpenCV, BGR), pads it right / bottom to
``(w // 32 + 1) * 32`` x ``(h // 32 + 1) * 32`` and normalises it on the CPU, copies it to the
device, runs the TensorRT engine of ``ESMStereo_trt`` (``enqueueV3``), copies the disparity back,
crops it, median-blurs it (5x5), masks it to ``(0, max_disp)``, converts it to 16-bit (x256) and
publishes it.  :class:`StereoNode` does the same work with the device doing all of it:

* the uint8 frames go host -> device as bytes (a quarter of the reference's fp32 copy) from pinned
  staging buffers on the node's own stream;
* pad + normalise: ``esm_preprocess_u8`` (pad right / bottom with normalised zeros, as
  ``copyMakeBorder`` before ``convertTo`` / normalise);
* inference: ``ESMStereo_trt.forward`` (backbone on PyTorch/MIOpen, hot path as one hipGraph);
* crop + medianBlur(5) + valid mask + ``convertTo(CV_16UC1, 256)``: ``esm_node_filter_u16``;
* only the uint16 disparity comes back to the host.

``elapsed_ms`` is measured as the node measures it (``:357-376``): from the input copy to the end
of inference.  The first frame also builds the hot path's launch plan and hipGraph, so
:meth:`StereoNode.warmup` runs one frame untimed (:meth:`run` calls it first).  Publishing (ROS
topics) and the OpenCV visualisation window are outside this package; :meth:`StereoNode.run` yields
the per-frame results to whatever publishes them.

Parity: the post-filter is bit-exact against ``oracle/io_oracle.py``, whose median restatement
matches ``scipy.ndimage.median_filter(mode="nearest")``.  Parity with OpenCV itself is UNPINNED: cv2
is not importable here and the reference holds no node outputs.  That ``cv::medianBlur`` on the
cropped ROI replicates the ROI's own border (rather than reading the padded image around it) is an
assumption of this restatement.
"""
from __future__ import annotations

import ctypes
import time
from typing import Iterable, Iterator, Tuple

import numpy as np
import torch

from ._lib import check, lib

__all__ = ["StereoNode", "node_pads"]


def node_pads(h: int, w: int, m: int = 32) -> Tuple[int, int]:
    """(pad_bottom, pad_right) of ``preprocess_image`` (:141-146): always up to the NEXT multiple
    of 32, so an already divisible size still gains 32 rows / columns."""
    return (h // m + 1) * m - h, (w // m + 1) * m - w


class StereoNode:
    """The node's per-frame work on one device stream (see the module docstring).

    ``model``: an ``ESMStereo_trt`` (or any module whose ``forward(left, right)`` returns
    ``[B, H, W]`` disparities); ``height`` x ``width``: the camera frame size.
    """

    def __init__(self, model: torch.nn.Module, height: int, width: int, max_disp: float = 192.0,
                 device: torch.device = torch.device("cuda")) -> None:
        self.model = model
        self.device = torch.device(device)
        self.h, self.w = int(height), int(width)
        pb, pr = node_pads(self.h, self.w)
        self.hp, self.wp = self.h + pb, self.w + pr
        self.max_disp = float(max_disp)
        self.stream = torch.cuda.Stream(self.device)
        self.host_u8 = torch.empty(2, self.h, self.w, 3, dtype=torch.uint8).pin_memory()
        self.host_u16 = torch.empty(self.h, self.w, dtype=torch.int16).pin_memory()
        self.dev_u8 = torch.empty(2, self.h, self.w, 3, dtype=torch.uint8, device=self.device)
        self.net_in = torch.empty(2, 1, 3, self.hp, self.wp, device=self.device)
        self.dev_u16 = torch.empty(self.h, self.w, dtype=torch.int16, device=self.device)
        self.filtered = torch.empty(self.h, self.w, device=self.device)

    def process(self, left: np.ndarray, right: np.ndarray) -> Tuple[np.ndarray, float]:
        """One frame pair ``[H, W, 3] uint8`` (channel order as read: the reference feeds OpenCV's
        BGR) -> (disparity ``[H, W] uint16``, elapsed ms of copy-in + inference)."""
        if left.shape != (self.h, self.w, 3) or right.shape != (self.h, self.w, 3):
            raise ValueError(f"StereoNode: frames must be {(self.h, self.w, 3)} uint8")
        self.host_u8[0].numpy()[...] = left
        self.host_u8[1].numpy()[...] = right
        s = self.stream
        sp = ctypes.c_void_p(s.cuda_stream)
        with torch.cuda.stream(s):
            t0 = time.perf_counter()
            self.dev_u8.copy_(self.host_u8, non_blocking=True)
            for k in range(2):
                check(lib.esm_preprocess_u8(self.dev_u8[k].data_ptr(), self.net_in[k].data_ptr(), 1, self.h, self.w,
                                            self.hp, self.wp, 0, 0, 1, sp), "node preprocess")
            with torch.no_grad():
                disp = self.model(self.net_in[0], self.net_in[1])
            s.synchronize()
            elapsed_ms = (time.perf_counter() - t0) * 1e3
            disp = disp.contiguous()
            check(lib.esm_node_filter_u16(disp.data_ptr(), self.dev_u16.data_ptr(), self.filtered.data_ptr(), 1,
                                          self.hp, self.wp, 0, 0, self.h, self.w, self.max_disp, sp), "node filter")
            self.host_u16.copy_(self.dev_u16, non_blocking=True)
            s.synchronize()
        return self.host_u16.numpy().view(np.uint16).copy(), elapsed_ms

    def warmup(self, left: np.ndarray, right: np.ndarray) -> None:
        """One untimed frame: builds the plan / hipGraph so later frames' elapsed_ms is steady state."""
        self.process(left, right)
        self._warm = True

    def run(self, pairs: Iterable[Tuple[np.ndarray, np.ndarray]]) -> Iterator[Tuple[np.ndarray, float]]:
        """The timer loop's body over a frame source (the node cycles its image list, :325-327); the
        first pair is also run once untimed (warmup) before its timed frame."""
        for left, right in pairs:
            if not getattr(self, "_warm", False):
                self.warmup(left, right)
            yield self.process(left, right)
