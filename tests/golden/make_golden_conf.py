"""Golden vectors for the confidence head (reference ``models/ESMStereo_confidence.py``).

Run in the build container only (it imports the reference from /root/reference):

    python tests/golden/make_golden_conf.py

Imports ``models/ESMStereo_confidence.py`` the way ``make_golden.py`` imports ``ESMStereo.py``
(inert ``cv2`` / ``timm``), builds ``LAFNet_ESM(16)`` (``:551-744``, the head ESMStereo-S builds at
``:916``), draws its state dict from the seeded PCG64 generator (tests/helpers.py seeded_state),
runs ``forward(cost, disp, imag, left_f1x, left_f2x, device)`` on seeded inputs shaped as
``ESMStereo_confidence.forward`` passes them (``:974``: the aggregated cost, init_pred,
match_left, features_left[3], features_left[1]) and saves inputs, the output and the outputs of
the two ``conf_upsample`` stages and the three fusion iterations.  Only data is written.
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, HERE)

from helpers import module_spec, seeded_state  # noqa: E402
from make_golden import load_reference  # noqa: E402

# (name, B, D, h, w, seed): h, w at 1/16 of the image (the head's output is 16x larger)
CASES = [("conf_S_a", 2, 12, 6, 10, 31), ("conf_S_b", 1, 12, 8, 24, 32)]


def load_conf_module():
    load_reference()  # registers the synthetic package, cv2 / timm stand-ins, submodule, shufflemixer
    import importlib.util
    spec = importlib.util.spec_from_file_location("refmodels.ESMStereo_confidence",
                                                  "/root/reference/models/ESMStereo_confidence.py")
    m = importlib.util.module_from_spec(spec)
    sys.modules[spec.name] = m
    spec.loader.exec_module(m)
    return m


def inputs(B, D, h, w, seed):
    rng = np.random.default_rng(seed)
    f = lambda *s: torch.from_numpy(rng.standard_normal(s).astype(np.float32))  # noqa: E731
    cost = f(B, D, h, w)
    disp = torch.from_numpy(rng.uniform(0, D - 1, (B, 1, h, w)).astype(np.float32))
    return {"cost": cost, "disp": disp, "imag": f(B, 64, h, w), "left_f1x": f(B, 96, h, w),
            "left_f2x": f(B, 24, 4 * h, 4 * w)}


def main():
    torch.set_num_threads(8)
    cm = load_conf_module()
    manifest_path = os.path.join(HERE, "manifest.json")
    with open(manifest_path) as fh:
        manifest = json.load(fh)
    for name, B, D, h, w, seed in CASES:
        net = cm.LAFNet_ESM(16).eval()
        spec = module_spec(net)
        net.load_state_dict(seeded_state(spec, seed))
        with open(os.path.join(HERE, "spec_conf.json"), "w") as fh:
            json.dump(spec, fh)
        x = inputs(B, D, h, w, seed)
        caught = {}
        hooks = [net.conf_up4.register_forward_hook(lambda m, i, o: caught.__setitem__("out4", o)),
                 net.conf_up1.register_forward_hook(lambda m, i, o: caught.__setitem__("out1", o)),
                 net.scale_bn3.register_forward_hook(lambda m, i, o: caught.__setitem__("scale_bn", o))]
        fus = []
        hooks.append(net.fusion_conv3.register_forward_hook(lambda m, i, o: fus.append(o)))
        with torch.no_grad():
            out = net(x["cost"], x["disp"], x["imag"], x["left_f1x"], x["left_f2x"], torch.device("cpu"))
        for hk in hooks:
            hk.remove()
        arrays = dict(x)
        arrays["conf"] = out
        arrays.update(caught)
        for i, t in enumerate(fus):
            arrays[f"fusion_conv3_{i}"] = t
        np.savez_compressed(os.path.join(HERE, name + ".npz"), **{k: v.detach().numpy() for k, v in arrays.items()})
        manifest[name + ".npz"] = dict(B=B, D=D, h=h, w=w, seed=seed, spec="spec_conf.json")
        print(name, {k: tuple(v.shape) for k, v in arrays.items()})
    with open(manifest_path, "w") as fh:
        json.dump(manifest, fh, indent=1)


if __name__ == "__main__":
    main()
