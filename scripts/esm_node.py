"""Command-line form of the node loop (the reference's kitti_publisher node without ROS):

    python scripts/esm_node.py --left DIR --right DIR --out DIR [--variant S] [--max-disp 192]
        [--checkpoint ckpt.tar] [--frames N]

Reads the sorted PNG pairs of two directories (KITTI image_2 / image_3 layout), feeds them in
OpenCV's BGR channel order as the reference node does (cv::imread), runs esmstereo_amd.node.
StereoNode and writes each 16-bit disparity PNG (x256, KITTI convention) to --out, printing the
per-frame elapsed time the node prints (kitti_publisher_cuda_node.cpp:376).  Without a checkpoint
the model keeps its random initialisation (the pretrained backbone is not fetchable offline).
"""
from __future__ import annotations

import argparse
import os
import sys

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import esmstereo_amd as E  # noqa: E402
from esmstereo_amd.node import StereoNode  # noqa: E402

VARIANTS = {"S": ("mobilenetv2_100", 16), "M": ("efficientnet_b2", 8), "L": ("efficientnet_b2", 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--left", required=True)
    ap.add_argument("--right", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--variant", default="S", choices=sorted(VARIANTS))
    ap.add_argument("--cv", default="gwc", choices=["gwc", "nc"])
    ap.add_argument("--max-disp", type=float, default=192.0)
    ap.add_argument("--checkpoint", default="")
    ap.add_argument("--frames", type=int, default=0)
    args = ap.parse_args()
    backbone, cvs = VARIANTS[args.variant]
    model = E.ESMStereo_trt(192, args.cv == "gwc", args.cv == "nc", backbone, cvs)
    if args.checkpoint:
        sd = torch.load(args.checkpoint, map_location="cpu", weights_only=True)
        sd = sd.get("model", sd)
        model.load_state_dict({k.replace("module.", "", 1): v for k, v in sd.items()}, strict=False)
    model = model.eval().cuda()
    names = sorted(f for f in os.listdir(args.left) if f.endswith(".png"))
    if args.frames:
        names = names[:args.frames]
    os.makedirs(args.out, exist_ok=True)
    node = None
    for n in names:
        left = np.asarray(Image.open(os.path.join(args.left, n)).convert("RGB"))[..., ::-1]  # BGR, as cv::imread
        right = np.asarray(Image.open(os.path.join(args.right, n)).convert("RGB"))[..., ::-1]
        if node is None or left.shape[:2] != (node.h, node.w):
            node = StereoNode(model, left.shape[0], left.shape[1], args.max_disp)
            node.warmup(np.ascontiguousarray(left), np.ascontiguousarray(right))  # plan + graph build, untimed
        disp, ms = node.process(np.ascontiguousarray(left), np.ascontiguousarray(right))
        Image.fromarray(disp).save(os.path.join(args.out, n))
        print(f"{n}: Elapsed time =: {ms:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
