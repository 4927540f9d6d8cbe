"""The cache-proof cost-volume measurement of bench.py alone, for rocprofv3 PMC passes:
gwc at ESMStereo-L KITTI (B=1, 64 ch, 96x312, D=48) over a ring of buffers larger than twice the
Infinity Cache, then gwc and build_concat_volume at BASELINE configs[2] (L-SF B=8).

    rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_gwc_f -o f -- python3 scripts/gwc_ring.py
    rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_gwc_w -o w -- python3 scripts/gwc_ring.py
    python3 scripts/gwc_ring.py --summarize gpurun_out/pmc_gwc_f gpurun_out/pmc_gwc_w profiles/pmc_traffic.json
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402

RING_CASES = (  # (workload key, kernel, B, H, W, D, timed launches) in bench.py's launch order
    ("gwc ring B1 96x312 D48", "gwc_volume", 1, 96, 312, 48, 24),
    ("gwc ring B8 136x240 D48", "gwc_volume", 8, 136, 240, 48, 8),
    ("concat B8 136x240 D48", "concat_volume", 8, 136, 240, 48, 6),
)


def _ring_buffers(kernel: str, B: int, H: int, W: int, D: int) -> int:
    if kernel == "concat_volume":
        return 2
    vol, feat = 4 * B * 32 * D * H * W, 4 * B * 2 * 64 * H * W
    return max(2, -(-(2 * bench.INFINITY_CACHE_BYTES) // (vol + feat)))


def summarize(fdir: str, wdir: str, table: str) -> dict:
    """Per-launch memory-side bytes of the timed (steady-state) launches of each case, from the two PMC
    passes, with the gfx950 FETCH_SIZE correction of scripts/pmc_traffic.py; merged into ``table``
    (profiles/pmc_traffic.json) under the keys bench.py looks up."""
    sys.path.insert(0, os.path.join(ROOT, "scripts"))
    from pmc_traffic import per_dispatch_named  # noqa: E402
    fetch, write = per_dispatch_named(fdir, "FETCH_SIZE"), per_dispatch_named(wdir, "WRITE_SIZE")
    out = {}
    for kname, seq_f, seq_w in (("gwc_kernel", fetch["gwc_kernel"], write["gwc_kernel"]),
                                ("concat_kernel", fetch["concat_kernel"], write["concat_kernel"])):
        pos = 0
        for key, kern, B, H, W, D, timed in RING_CASES:
            if (kern == "gwc_volume") != (kname == "gwc_kernel"):
                continue
            n = _ring_buffers(kern, B, H, W, D) + timed  # warm-up launches over the ring, then the timed ones
            f, w = seq_f[pos + n - timed:pos + n], seq_w[pos + n - timed:pos + n]
            pos += n
            if len(f) != timed or len(w) != timed:
                raise SystemExit(f"{key}: expected {timed} timed dispatches, found {len(f)} / {len(w)}")
            fk, wk = sum(f) / timed, sum(w) / timed
            alg = 4 * B * (2 * 64 * H * W + (32 if kern == "gwc_volume" else 128) * D * H * W)
            out[key] = {kern: {"fetch_size_kib": round(fk, 1), "write_size_kib": round(wk, 1),
                               "hbm_bytes_per_launch": int((2 * fk + wk) * 1024), "algorithmic_bytes": alg}}
    with open(table) as fh:
        tab = json.load(fh)
    tab.update(out)
    with open(table, "w") as fh:
        json.dump(tab, fh, indent=1)
    return out


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "--summarize":
    print(json.dumps(summarize(*sys.argv[2:5]), indent=1))
elif __name__ == "__main__":
    bench._load_package()
    dev = torch.device("cuda", 0)
    out = {"gwc_L_K": bench.cost_volume_roofline(dev, reps=24),
           "gwc_configs2": bench.cost_volume_roofline(dev, reps=8, B=8, H=136, W=240, D=48),
           "concat_configs2": bench.concat_volume_roofline(dev)}
    print(json.dumps(out))
