"""Benchmark: stereo pairs/sec of the ESMStereo hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config 1..4]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

Without a launcher (WORLD_SIZE unset) and --gpus N > 1, this process starts the N ranks itself: N
fresh child processes, one per GPU, with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* set (before any HIP
call here, and never by re-exec), waits for them and exits non-zero if any rank fails.  Under a
launcher, --gpus must equal WORLD_SIZE.

A "step" is one pass of the hot path (models/ESMStereo.py:700-745: cost volume -> 3-D stems ->
3-D hourglass -> regression -> ESM/ShuffleMixer upsampler -> x4) over one batch of synthetic
matching features already resident in HBM: by default BASELINE.json configs[1], ESMStereo-S
(mobilenetv2_100 channel ladder, cv_scale 16, gwc volume) at KITTI 384x1248, maxdisp 192, batch 1
per GPU.  The backbone side that produces the features is out of scope; the inputs
are tests/helpers.py fullsize_inputs (at configs[1] exactly the reference fixture's).  Each rank
runs its own batch (weak scaling; --config 3 splits a global batch: strong); with N > 1 the
disparity maps are all-gathered over RCCL every step.  The multi-rank loop (shards, gather, barrier,
max-over-ranks time) is esmstereo_amd.dist, which tests/test_dist.py runs under gloo.

Printed (rank 0, one JSON line): the contract fields, plus
  roofline        the dominant op: the largest in-graph duration, measured as its marginal cost in
                  the replayed graph (step minus the step with the op dropped), against the fp32
                  MFMA or HBM peak by its algorithmic intensity; traffic = PMC bytes from profiles/;
  roofline_mfma   the same for group_stem (the MFMA-bound 3-D stem);
  roofline_step   the whole step: sum over ops of max(flops / MFMA peak, bytes / HBM peak) vs the
                  measured step, and the algorithmic-bytes-only HBM fraction (north_star);
  roofline_cost_volume  the gwc cost-volume kernel at KITTI full res for ESMStereo-L (cache-proof);
  cpu_baseline    the CPU oracle (oracle/esm_oracle.py, PyTorch fp32 on the host cores) on a bounded
                  sample of the same workload, rank 0 at N = 1 only;
  epe_vs_oracle   mean |disparity_HIP - disparity_oracle| (px) on the benchmark input;
  epe_vs_reference  the reference's own full-size fixture (tests/golden/full_*.npz);
  concurrent      (N = 1) --streams independent hot-path instances replayed on as many HIP streams;
  forward_e2e     (N = 1) model(left, right, False) end to end, backbone included.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import socket
import statistics
import subprocess
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# the package (and its HIP library) is loaded by the rank processes only (_load_package): a parent that
# launches the ranks itself never touches the GPU
E = D = lib = None


def _load_package() -> None:
    global E, D, lib
    import esmstereo_amd
    from esmstereo_amd import dist
    from esmstereo_amd._lib import lib as _native

    E, D, lib = esmstereo_amd, dist, _native

VARIANTS = {"S": ("mobilenetv2_100", 16), "M": ("efficientnet_b2", 8), "L": ("efficientnet_b2", 4)}
METRIC = "stereo pairs/sec at 384×1248 maxdisp=192; EPE vs reference"
PEAK_HBM_GBS = 8000.0      # MI355X HBM3E spec (MI355X_MICROARCH.md)
PEAK_F32_MFMA_TFS = 157.3  # dense fp32 MFMA (v_mfma_f32_16x16x4_f32), spec


def seeded_init(model: torch.nn.Module, seed: int) -> None:
    """Random-init weights of the architecture (no checkpoints offline): He-normal convs,
    randomised eval BatchNorm statistics."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for name, m in model.named_modules():
            if isinstance(m, (torch.nn.Conv2d, torch.nn.Conv3d, torch.nn.ConvTranspose2d, torch.nn.ConvTranspose3d)):
                w = m.weight
                fan = w[0].numel() if not isinstance(m, (torch.nn.ConvTranspose2d, torch.nn.ConvTranspose3d)) \
                    else max(1, w.shape[0] * w[0, 0].numel() // (2 ** (w.dim() - 2)))
                # refinement residual heads at 0.1x (as tests/helpers.py REFINE_HEAD): realistic disparities
                gain = 0.1 if (name.startswith("upsample_module.ref") and name.endswith("conv1_up.conv")) else 1.0
                gain = 0.25 if name == "aggregation_out.conv1_up.conv" else gain  # cost head, as tests/helpers.py
                w.copy_(torch.randn(w.shape, generator=g) * math.sqrt(2.0 / fan) * gain)
                if m.bias is not None:
                    m.bias.copy_(torch.rand(m.bias.shape, generator=g) * 0.2 - 0.1)
            elif isinstance(m, (torch.nn.BatchNorm2d, torch.nn.BatchNorm3d)):
                m.weight.copy_(torch.rand(m.weight.shape, generator=g) * 0.4 + 0.8)
                m.bias.copy_(torch.rand(m.bias.shape, generator=g) * 0.2 - 0.1)
                m.running_mean.copy_(torch.rand(m.running_mean.shape, generator=g) * 0.2 - 0.1)
                m.running_var.copy_(torch.rand(m.running_var.shape, generator=g) + 0.5)


def synthetic_pair(B: int, H: int, W: int, maxdisp: int, seed: int, device) -> tuple:
    """Smooth sinusoid texture (ImageNet-normalised range) + right view shifted by a planar
    disparity field."""
    g = torch.Generator().manual_seed(seed)
    yy, xx = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W + maxdisp, dtype=torch.float32),
                            indexing="ij")
    full = torch.zeros(B, 3, H, W + maxdisp)
    for b in range(B):
        for c in range(3):
            for _ in range(8):
                fx, fy, ph = (torch.rand(3, generator=g) * torch.tensor([0.33, 0.33, 6.28]) + 0.02).tolist()
                full[b, c] += torch.sin(fx * xx + fy * yy + ph) / 2
    left = full[..., maxdisp:]
    right = torch.empty_like(left)
    for y in range(H):
        d = int((0.1 + 0.8 * y / max(1, H - 1)) * (maxdisp - 1))
        right[:, :, y] = full[:, :, y, maxdisp - d: maxdisp - d + W]
    return left.to(device), right.to(device)


RIDGE_FLOP_PER_BYTE = PEAK_F32_MFMA_TFS * 1e12 / (PEAK_HBM_GBS * 1e9)  # ~19.7


def kernel_roofline(meta: dict, avg_ms: float) -> dict:
    """Price the kernel against the roof its arithmetic intensity puts it under: MFMA when
    algorithmic flops / algorithmic bytes exceeds the fp32 ridge point, HBM otherwise."""
    sec = avg_ms * 1e-3
    if meta["flops"] > RIDGE_FLOP_PER_BYTE * meta["bytes"]:
        ach = meta["flops"] / sec / 1e12
        return {"bound": "mfma", "achieved": round(ach, 3), "peak": PEAK_F32_MFMA_TFS, "unit": "TFLOP/s",
                "frac": round(ach / PEAK_F32_MFMA_TFS, 4)}
    ach = meta["bytes"] / sec / 1e9
    return {"bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4)}


def pmc_traffic(name: str, workload: str):
    """HBM bytes per launch of `name` from the committed rocprofv3 PMC summary, or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        tab = json.load(f)
    e = tab.get(workload, {}).get(name)
    return None if e is None else e.get("hbm_bytes_per_launch")


def _replay_us(hp: E.HotPath, reps: int) -> float:
    """us per graph replay over ``reps`` back-to-back replays between one hipEvent pair."""
    for _ in range(2):
        hp.launch()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        hp.launch()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def marginal_costs(hp: E.HotPath, rounds: int = 3, window_ms: float = 6.0) -> tuple:
    """Each op's duration INSIDE the replayed graph, as its marginal cost: the step time of the graph
    minus the step time of the same graph with that op dropped (``esm_plan_set_repeat(i, 0)``; the
    median of ``rounds`` interleaved windows each).  This counts what the op costs the chain: its own
    device time with the caches the chain leaves it, and its launch boundary.  No event nodes sit in
    the measured graphs (they perturb the chain).  Returns (per-op us, full step us)."""
    plan = hp.ctx.plan
    hp._graph_ready = False
    base0 = _replay_us(hp, 10)
    reps = max(8, int(window_ms * 1e3 / base0))
    base_all, out = [], []
    for i in range(hp.num_ops):
        base, drop = [], []
        for _ in range(rounds):
            hp._graph_ready = False
            base.append(_replay_us(hp, reps))
            lib.esm_plan_set_repeat(plan, i, 0)
            hp._graph_ready = False
            drop.append(_replay_us(hp, reps))
            lib.esm_plan_set_repeat(plan, i, 1)
        out.append(statistics.median(base) - statistics.median(drop))
        base_all += base
        if (i + 1) % 8 == 0:  # progress for long steps (configs 3 / 4): a silent minute reads as a hang
            print(f"marginal costs: {i + 1}/{hp.num_ops} ops", file=sys.stderr, flush=True)
    hp._graph_ready = False
    return out, statistics.median(base_all)


def step_roofline(meta: list, step_ms: float, pairs: int) -> dict:
    """The whole step against the roofs (north_star: pairs/s "as fraction of the HBM roofline"): each
    op's roof time is max(algorithmic flops / fp32 MFMA peak, algorithmic bytes / HBM peak) and the ops
    run one after the other (the path's DAG has width 1), so the step's roof time is their sum."""
    flops = sum(m["flops"] for m in meta)
    byts = sum(m["bytes"] for m in meta)
    roof_s = sum(max(m["flops"] / (PEAK_F32_MFMA_TFS * 1e12), m["bytes"] / (PEAK_HBM_GBS * 1e9)) for m in meta)
    hbm_s = byts / (PEAK_HBM_GBS * 1e9)
    step_s = step_ms * 1e-3
    return {"flops_per_pair": round(flops / pairs), "bytes_per_pair": round(byts / pairs),
            "roof_us_per_step": round(roof_s * 1e6, 2), "roof_pairs_per_s": round(pairs / roof_s, 1),
            "frac": round(roof_s / step_s, 4),
            "hbm_roof_pairs_per_s": round(pairs / hbm_s, 1), "hbm_frac": round(hbm_s / step_s, 4),
            "launches": len(meta),
            "rule": "sum over ops of max(flops / 157.3 TF/s, bytes / 8 TB/s) vs the measured step; "
                    "hbm_* = algorithmic bytes only"}


INFINITY_CACHE_BYTES = 256 << 20  # MI355X die-level L3 (MI355X_MICROARCH.md)


def cost_volume_roofline(device, reps: int = 24, B: int = 1, H: int = 96, W: int = 312, D: int = 48) -> dict:
    """gwc kernel alone at ESMStereo-L KITTI full res (B=1, C=64, 96x312, D=48, G=32), cache-proof:
    every launch writes the next buffer of a ring of output volumes (and reads the next of a ring of
    feature pairs) whose total exceeds the 256 MiB Infinity Cache, so no launch finds its output
    lines or its inputs resident from the previous one.  Timed as ``reps`` back-to-back launches
    between one hipEvent pair (per-launch event pairs add their own overhead)."""
    C, G = 64, 32
    vol = 4 * B * G * D * H * W
    feat = 4 * B * 2 * C * H * W
    nbuf = max(2, -(-(2 * INFINITY_CACHE_BYTES) // (vol + feat)))  # footprint >= 2x the Infinity Cache
    Ls = [torch.randn(B, C, H, W, device=device) for _ in range(nbuf)]
    Rs = [torch.randn(B, C, H, W, device=device) for _ in range(nbuf)]
    Vs = [torch.empty(B, G, D, H, W, device=device) for _ in range(nbuf)]
    ctx = E.engine.Ctx(device)
    for i in range(nbuf):
        ctx.gwc(Ls[i], Rs[i], None, Vs[i], B, C, H, W, D, G)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for r in range(reps):
        i = r % nbuf
        ctx.gwc(Ls[i], Rs[i], None, Vs[i], B, C, H, W, D, G)
    ev1.record()
    torch.cuda.synchronize()
    avg = ev0.elapsed_time(ev1) / reps
    byts = 4 * B * (2 * C * H * W + G * D * H * W)
    ach = byts / (avg * 1e-3) / 1e9
    out = {"kernel": "gwc_volume", "config": f"ESMStereo-L B={B} C=64 {H}x{W} D={D} G=32",
           "bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
           "frac": round(ach / PEAK_HBM_GBS, 4), "bytes_per_launch": byts, "avg_us": round(avg * 1e3, 2),
           "ring_buffers": nbuf, "footprint_bytes": nbuf * (vol + feat), "timing": f"{reps} launches, one event pair",
           "traffic": pmc_traffic("gwc_volume", f"gwc ring B{B} {H}x{W} D{D}")}
    del Ls, Rs, Vs
    torch.cuda.empty_cache()
    return out


def concat_volume_roofline(device, reps: int = 6, B: int = 8, H: int = 136, W: int = 240, D: int = 48) -> dict:
    """build_concat_volume (submodule.py:129-140) at BASELINE configs[2]'s size: [8, 128, 48, 136, 240]
    = 6.4 GB written per launch, two output buffers alternating (12.8 GB, far past the Infinity Cache)."""
    C = 64
    L = torch.randn(B, C, H, W, device=device)
    R = torch.randn(B, C, H, W, device=device)
    Vs = [torch.empty(B, 2 * C, D, H, W, device=device) for _ in range(2)]
    ctx = E.engine.Ctx(device)
    for V in Vs:
        ctx.concat(L, R, V, B, C, H, W, D)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for r in range(reps):
        ctx.concat(L, R, Vs[r % 2], B, C, H, W, D)
    ev1.record()
    torch.cuda.synchronize()
    avg = ev0.elapsed_time(ev1) / reps
    byts = 4 * B * (2 * C * H * W + 2 * C * D * H * W)
    ach = byts / (avg * 1e-3) / 1e9
    del Vs
    torch.cuda.empty_cache()
    return {"kernel": "concat_volume", "config": f"ESMStereo-L B={B} C=64 {H}x{W} D={D} (BASELINE configs[2])",
            "bound": "hbm", "achieved": round(ach, 1), "peak": PEAK_HBM_GBS, "unit": "GB/s",
            "frac": round(ach / PEAK_HBM_GBS, 4), "bytes_per_launch": byts, "avg_us": round(avg * 1e3, 2),
            "traffic": pmc_traffic("concat_volume", f"concat B{B} {H}x{W} D{D}")}


def concurrent_streams(model, ml, mr, att, up, n: int, steps: int, warmup: int, device) -> dict:
    """Serving-style throughput at batch 1: ``n`` independent hot-path instances (own buffers, own
    hipGraph) replayed concurrently on ``n`` HIP streams, so one pair's latency-bound small launches
    overlap another's.  Reported beside the contract value, which stays the single-stream B=1 rate."""
    B, C, h, w = (int(v) for v in ml.shape)
    paths = []
    for _ in range(n):
        hp = E.HotPath(model, B, h, w, 0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], device,
                       graph=True, channels=C)
        hp.load_inputs(ml, mr, att, up)
        paths.append(hp)
    streams = [torch.cuda.Stream(device) for _ in range(n)]
    main = torch.cuda.current_stream(device)

    def round_():
        for hp, st in zip(paths, streams):
            st.wait_stream(main)
            hp.launch(st)
        for st in streams:
            main.wait_stream(st)

    for _ in range(warmup):
        round_()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        round_()
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    same = all(torch.equal(hp.outputs[0], paths[0].outputs[0]) for hp in paths[1:])
    return {"streams": n, "value": round(n * B * steps / el, 2), "unit": "pairs/s", "batch_per_stream": B,
            "ms_per_round": round(el / steps * 1e3, 4), "outputs_identical": bool(same)}


def host_cores() -> tuple:
    """(cores this process may use, CPUs the host reports).  On the GPU box os.cpu_count() is the
    whole machine while the job gets a share of it (its affinity mask and cgroup CPU quota): the
    baseline runs one thread per core of that share."""
    total = os.cpu_count() or 1
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else total
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(int(quota) // int(period))))
    except (OSError, ValueError):
        pass
    return max(1, n), total


def cpu_baseline(model, ml, mr, att, up, args, budget_s: float) -> tuple:
    """The oracle (PyTorch fp32 CPU restatement) on every core of the job's host share, one pair
    (the first of the batch) per forward; value = 1 / (min over >= 3 forwards) pairs/s."""
    from oracle import esm_oracle as O

    threads, host_total = host_cores()
    torch.set_num_threads(threads)
    sd = {k: v.detach().cpu() for k, v in model.state_dict().items()}
    one = lambda t: None if t is None else t[:1].cpu()  # noqa: E731
    ins = (one(ml), one(mr), one(att), [one(u) for u in up])
    _, cvs = VARIANTS[args.variant]
    times, t0, out = [], time.perf_counter(), None
    with torch.no_grad():
        while len(times) < 3 or (time.perf_counter() - t0 < budget_s and len(times) < 400):
            t1 = time.perf_counter()
            out = O.hot_path(sd, cvs, args.maxdisp, args.cv == "gwc", *ins)
            times.append(time.perf_counter() - t1)
    el = time.perf_counter() - t0
    best = min(times)
    return ({"value": round(1.0 / best, 3), "unit": "pairs/s", "cores": threads, "host_cpus": host_total,
             "kind": "port", "timing": f"min of {len(times)} forwards (mean {sum(times) / len(times) * 1e3:.1f} ms)",
             "sample": f"{len(times)} hot-path forwards of one {args.height}x{args.width} md{args.maxdisp} "
                       f"ESMStereo-{args.variant} {args.cv} pair, oracle/esm_oracle.py (PyTorch fp32 CPU, "
                       f"{threads} threads = the job's CPU share of {host_total} host CPUs), {el:.1f} s"},
            out["disp_0"])


# BASELINE.json configs (configs[0] is the reference's CPU plumbing case: tests/test_gpu_parity.py
# test_expected_raises pins its error).  Default: configs[1], the headline metric.
CONFIGS = {
    1: dict(variant="S", cv="gwc", height=384, width=1248, maxdisp=192, batch=1, scaling="weak",
            name="ESMStereo-S KITTI 384x1248 maxdisp=192 batch=1 per GPU"),
    2: dict(variant="L", cv="gwc", height=544, width=960, maxdisp=192, batch=8, scaling="weak",
            name="ESMStereo-L SceneFlow 540x960 (padded to 544x960) maxdisp=192 batch=8 per GPU"),
    3: dict(variant="L", cv="gwc", height=384, width=1248, maxdisp=192, global_batch=32, scaling="strong",
            name="ESMStereo-L KITTI 384x1248 maxdisp=192, global batch 32 split over the GPUs"),
    4: dict(variant="L", cv="gwc", height=1024, width=1504, maxdisp=256, batch=1, scaling="weak",
            name="Middlebury ~1500x1000 (padded to 1504x1024) maxdisp=256 batch=1 per GPU"),
}
WEIGHT_SEED = {("S", "gwc"): 11, ("S", "nc"): 12, ("M", "gwc"): 13, ("M", "nc"): 14, ("L", "gwc"): 15, ("L", "nc"): 16}


def load_seeded_weights(model: torch.nn.Module, variant: str, cv: str) -> None:
    """The hot path's weights from the seeded generator the reference fixtures were made with
    (tests/helpers.py seeded_state over the reference's state-dict spec): random-init weights of the
    architecture, and the same network the full-size reference fixture ran, so the benchmark can
    report its EPE against the reference.  The backbone keeps its own random init."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import load_spec, seeded_state

    import warnings

    sd = seeded_state(load_spec(f"spec_{variant}_{cv}.json"), WEIGHT_SEED[(variant, cv)])
    with warnings.catch_warnings():  # the backbone deliberately keeps its random init here
        warnings.filterwarnings("ignore", message=".*backbone.*", category=RuntimeWarning)
        missing, unexpected = model.load_state_dict({k: v for k, v in sd.items() if not k.startswith("feature.")},
                                                    strict=False)
    assert not unexpected and all(k.startswith("feature.") for k in missing), (missing, unexpected)


def epe_vs_reference(model, args, dev):
    """The plan on the seeded inputs of the reference's full-size fixture for this configuration
    (tests/golden/full_*.npz, made by running the reference itself), EPE of disp_0 at every 4th row and
    column; ESMStereo-L flip-masked (tests/parity.py).  None when no fixture matches."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from parity import check_fullsize, fullsize_case, fullsize_manifest

    for name, m in sorted(fullsize_manifest().items()):
        if (m["variant"], m["cv"], m["H"], m["W"], m["maxdisp"]) == (args.variant, args.cv, args.height, args.width,
                                                                      args.maxdisp):
            break
    else:
        return None
    m, g, (ml, mr, att, up) = fullsize_case(name)
    T = lambda a: None if a is None else torch.from_numpy(a).to(dev)  # noqa: E731
    ml, mr, att, up = T(ml), T(mr), T(att), [T(u) for u in up]
    D = m["maxdisp"] // m["cv_scale"]
    with torch.no_grad():
        V = E.build_gwc_volume(ml, mr, D, 32, att=att) if args.cv == "gwc" else E.build_norm_correlation_volume(ml, mr, D)
        if args.cv == "gwc":
            vol = model.group_stem(V)
        else:
            vol = model.corr_stem.emit(E.engine.Ctx(dev), [V], mul=None if att is None else att)
        cost = model.aggregation_out(model.agg(vol))[:, 0]
        init = E.regression_topk(cost, None, 2) if m["cv_scale"] == 4 else \
            E.disparity_regression(cost, D).unsqueeze(1)
        disp0 = model.hot_path(ml, mr, att, up)[0]
        d_ref_init = E.engine.eager_emit(dev, model.upsample_module.emit, up, T(g["init_pred"]), final_scale=4.0)[0]
    rep = check_fullsize(name, m, g, cost, init, disp0, disp0_from_ref_init=d_ref_init[:, 0])
    d = rep.get("disp0")
    epe = d["epe_outside_mask"] if d else rep["disp0_sub_epe"]
    return {"epe_px": epe, "fixture": "tests/golden/" + name, "pixels": "every 4th row and column of disp_0",
            "epe_px_upsampler_on_reference_init": rep["disp0_sub_epe_ref_init"],
            "top2_flips": None if d is None else d["flips"], "cost_rel": max(rep["cost_sample_rel"], rep["cost_l2_rel"])}


def bench_inputs(variant: str, cv: str, B: int, H: int, W: int, maxdisp: int, seed: int, dev) -> tuple:
    """Synthetic hot-path inputs: matching features of a smooth texture with the right
    view shifted by a planar disparity field inside [0.1, 0.8] x maxdisp, attention weights (S) and
    smooth upsampler feature maps, as tests/helpers.py fullsize_inputs (the generator of the reference's
    full-size fixtures: at configs[1] with seed 101 the input IS tests/golden/full_S_gwc_K.npz's)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from helpers import fullsize_inputs

    cvs = VARIANTS[variant][1]
    ml, mr, att, up = fullsize_inputs(cvs, B, H, W, maxdisp, seed, att=cvs == 16)
    T = lambda a: None if a is None else torch.from_numpy(a).to(dev)  # noqa: E731
    return T(ml), T(mr), T(att), [T(u) for u in up]


INPUT_SEED = {1: 101, 2: 201, 3: 102, 4: 401}  # configs[1] / [3]: the reference fixtures' input seeds


def forward_e2e(model, args, dev, iters: int = 10) -> dict:
    """The public forward end to end: ``model(left, right, False)`` on a synthetic
    image pair, backbone side (PyTorch/MIOpen, out of the hot path) included, plus the host cost of one
    ``hot_path()`` call on resident features (plan-cache key, input copies, graph launch, output clone)."""
    left, right = synthetic_pair(args.batch, args.height, args.width, args.maxdisp, 7, dev)
    with torch.no_grad():
        for _ in range(2):
            model(left, right, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            model(left, right, False)
        torch.cuda.synchronize()
        el = (time.perf_counter() - t0) / iters
        model.capture_forward = False  # the backbone side eagerly (each launch from the host), for comparison
        for _ in range(2):
            model(left, right, False)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            model(left, right, False)
        torch.cuda.synchronize()
        el_eager = (time.perf_counter() - t0) / iters
        model.capture_forward = True
        ml, mr, att, up = model.prefix(left, right)
        model.hot_path(ml, mr, att, up)
        torch.cuda.synchronize()
        hp_iters = 10 * iters  # the first call's host work runs with the device idle: amortise it
        t0 = time.perf_counter()
        for _ in range(hp_iters):
            model.hot_path(ml, mr, att, up)
        t_host = time.perf_counter() - t0
        torch.cuda.synchronize()
        hp_ms = (time.perf_counter() - t0) / hp_iters * 1e3
    return {"value": round(args.batch / el, 2), "unit": "pairs/s", "ms_per_forward": round(el * 1e3, 3),
            "ms_per_forward_eager_backbone": round(el_eager * 1e3, 3),
            "hot_path_call_ms": round(hp_ms, 4), "hot_path_host_us": round(t_host / hp_iters * 1e6, 1),
            "what": f"model(left, right, False) with the random-init backbone, replayed from the captured "
                    f"whole-forward graphs (model.ForwardGraph; ms_per_forward_eager_backbone: the backbone side "
                    f"launched eagerly instead); hot_path_call_ms = one "
                    f"model.hot_path() call on resident features ({hp_iters} back to back), host work included "
                    f"(plan key, binding, graph launch, output clone); hot_path_host_us = its host time alone"}


def _free_port() -> int:
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


def launch_ranks(argv: list, n: int) -> int:
    """Start ``n`` rank processes of this script (one per GPU, as torch.distributed.run would) and wait
    for them.  If one fails the others are stopped (a rank blocked in a collective would never return);
    returns 0 or the first failing rank's exit status."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + list(argv), env=env))
    failed = 0
    while any(p.poll() is None for p in procs):
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad and not failed:
            failed = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.terminate()
        time.sleep(0.05)
    for p in procs:
        if p.returncode != 0 and not failed:
            failed = p.returncode
    return 0 if not failed else (failed if failed > 0 else 1)


def standin_cpu(args, world: int, rank: int) -> None:
    """The multi-rank bench loop (shards, per-step gather, barrier + max-over-ranks time) over gloo on
    the CPU with a per-pair stand-in for the HIP hot path: the launcher path is exercised without a GPU
    (tests/test_dist.py).  Rank 0 prints the contract line with the gathered buffer's shape."""
    if world > 1:
        torch.distributed.init_process_group("gloo")
    world, rank = D.world_info()
    if args.global_batch is not None:
        b, scaling, total = D.local_batch(world, rank, global_batch=args.global_batch)
    else:
        b, scaling, total = D.local_batch(world, rank, batch=args.batch)
    g = torch.Generator().manual_seed(100 + rank)
    left, right = torch.randn(b, 3, 8, 16, generator=g), torch.randn(b, 3, 8, 16, generator=g)
    out = torch.empty(b, 8, 16)
    gather = D.DisparityGather(out)

    def step():
        out.copy_((left - right).abs().sum(1) * 4)
        gather(out)

    elapsed = D.timed_steps(step, args.steps, args.warmup, torch.device("cpu"))
    if rank == 0:
        # the gathered buffer holds rank r's shard at [r] (rank order): every rank's input is regenerated here
        order_ok = True
        for r in range(world):
            gr = torch.Generator().manual_seed(100 + r)
            lr_, rr_ = torch.randn(b, 3, 8, 16, generator=gr), torch.randn(b, 3, 8, 16, generator=gr)
            order_ok = order_ok and torch.equal(gather.buf[r], (lr_ - rr_).abs().sum(1) * 4)
        print(json.dumps({"metric": METRIC, "value": round(total * args.steps / elapsed, 2), "unit": "pairs/s",
                          "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "scaling": scaling,
                          "standin": "cpu gloo (no GPU work)", "global_batch": total,
                          "gathered_shape": list(gather.buf.shape), "gather_rank_order_ok": bool(order_ok)}),
              flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=1, choices=sorted(CONFIGS),
                    help="BASELINE.json configs[i] preset (default 1, the headline); the flags below override it")
    ap.add_argument("--variant", default=None, choices=sorted(VARIANTS))
    ap.add_argument("--cv", default=None, choices=["gwc", "nc"])
    ap.add_argument("--batch", type=int, default=None, help="pairs per GPU per step (weak scaling)")
    ap.add_argument("--global-batch", type=int, default=None, help="pairs per step over all GPUs (strong scaling)")
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--maxdisp", type=int, default=None)
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-gather", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the side measurements (cost-volume rooflines, "
                    "concurrent streams, EPE vs the reference fixture, end-to-end forward)")
    ap.add_argument("--no-marginal", action="store_true", help="skip the per-op in-graph marginal costs (the "
                    "dominant op is then the longest back-to-back launch)")
    ap.add_argument("--kernel-table", default="", help="write the per-op table (json) here")
    ap.add_argument("--streams", type=int, default=2,
                    help="side measurement: independent B-pair instances on this many concurrent streams")
    ap.add_argument("--cpu-standin", action="store_true", help=argparse.SUPPRESS)  # launcher test (no GPU)
    ap.add_argument("--dist", action="store_true", help="initialise the RCCL process group and gather through the "
                    "collective even at one rank (tests/test_gpu_dist.py: the N > 1 code path on a one-GPU box)")
    args = ap.parse_args()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        if not args.cpu_standin and args.gpus > torch.cuda.device_count():  # device_count: no HIP init here
            raise SystemExit(f"bench.py: --gpus {args.gpus} but {torch.cuda.device_count()} GPU(s) visible")
        sys.exit(launch_ranks(sys.argv[1:], args.gpus))
    if int(env_world or 1) != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE {env_world} from the launcher")
    _load_package()
    cfg = CONFIGS[args.config]
    for k in ("variant", "cv", "height", "width", "maxdisp"):
        if getattr(args, k) is None:
            setattr(args, k, cfg[k])
    if args.global_batch is None and args.batch is None:
        args.global_batch = cfg.get("global_batch")
        args.batch = cfg.get("batch")

    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.cpu_standin:
        standin_cpu(args, world, local)
        return
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    use_dist = world > 1 or args.dist
    if use_dist:
        if world == 1:  # a one-rank group without a launcher: a local rendezvous
            os.environ.setdefault("RANK", "0")
            os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
            os.environ.setdefault("MASTER_PORT", str(_free_port()))
            os.environ["WORLD_SIZE"] = "1"
        torch.distributed.init_process_group("nccl", device_id=dev)
    world, rank = D.world_info()
    if args.global_batch is not None:
        args.batch, scaling, total_batch = D.local_batch(world, rank, global_batch=args.global_batch)
    else:
        args.batch, scaling, total_batch = D.local_batch(world, rank, batch=args.batch)

    backbone, cvs = VARIANTS[args.variant]
    model = E.ESMStereo(args.maxdisp, args.cv == "gwc", args.cv == "nc", backbone, cvs)
    seeded_init(model, 1234)  # the backbone side (only the end-to-end side measurement runs it)
    load_seeded_weights(model, args.variant, args.cv)
    model = model.eval().to(dev)
    ml, mr, att, up = bench_inputs(args.variant, args.cv, args.batch, args.height, args.width, args.maxdisp,
                                   INPUT_SEED.get(args.config, 500) + 1000 * rank, dev)
    B, C, h, w = (int(v) for v in ml.shape)
    hp = E.HotPath(model, B, h, w, 0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], dev,
                   graph=not args.no_graph, channels=C)
    hp.load_inputs(ml, mr, att, up)
    meta = hp.ctx.meta
    assert len(meta) == hp.num_ops, (len(meta), hp.num_ops)

    # the dominant op: the longest inside the replayed graph (marginal cost), before the timed region
    marg = None
    if hp.graph and not args.no_marginal:
        marg, _ = marginal_costs(hp)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def b2b_ms(i: int, reps: int) -> float:
        hp.run_op(i, 3)
        ev0.record()
        hp.run_op(i, reps)
        ev1.record()
        torch.cuda.synchronize()
        return ev0.elapsed_time(ev1) / reps

    if marg is not None:
        dom = max(range(hp.num_ops), key=lambda i: marg[i])
    else:
        dom = max(range(hp.num_ops), key=lambda i: b2b_ms(i, 10))
    if args.kernel_table and rank == 0:
        with open(args.kernel_table, "w") as f:
            json.dump([dict(m, marginal_us=None if marg is None else round(marg[i], 3))
                       for i, m in enumerate(meta)], f, indent=1)
        # the timed region's whole steps, and the launches after them (the dominant op's
        # back-to-back batch), for the position-based trace mapping of scripts/prof_ops.py / pmc_traffic.py
        has_stem = marg is not None and any(m["name"] == "group_stem" for m in meta)
        with open(args.kernel_table + ".meta.json", "w") as f:  # dominant-op batch (+ group_stem's batch)
            json.dump({"timed_steps": args.steps,
                       "trailing_dispatches": meta[dom].get("launches", 1) * (3 + args.steps) + (23 if has_stem else 0)}, f)

    # the timed region: the plain plan (one hipGraph per step) + the per-step disparity all-gather
    gather = D.DisparityGather(hp.outputs[0], collective=use_dist) if use_dist and not args.no_gather else None

    def step():
        hp.launch()
        if gather is not None:
            gather(hp.outputs[0])

    elapsed = D.timed_steps(step, args.steps, args.warmup, dev)
    batch_ms = b2b_ms(dom, args.steps)  # the dominant op alone, K launches back to back, warm caches

    if rank == 0:
        ms_step = elapsed / args.steps * 1e3
        dom_ms = marg[dom] * 1e-3 if marg is not None else batch_ms
        roof = kernel_roofline(meta[dom], dom_ms)
        workload = f"ESMStereo-{args.variant} {args.cv} {args.height}x{args.width} md{args.maxdisp} B{args.batch}"
        roof.update({"traffic": pmc_traffic(meta[dom]["name"], workload), "kernel": meta[dom]["name"],
                     "kernel_shape": meta[dom].get("shape", ""), "avg_us": round(dom_ms * 1e3, 2),
                     "timing": "marginal cost inside the replayed graph (step time minus the step with this op "
                               "dropped; median of 3 interleaved windows): the op's in-chain duration incl. its "
                               "launch boundary" if marg is not None else "back-to-back launches, warm caches",
                     "avg_us_back_to_back_warm": round(batch_ms * 1e3, 2),
                     "algorithmic_flops_per_launch": meta[dom]["flops"],
                     "algorithmic_bytes_per_launch": meta[dom]["bytes"]})
        line = {
            "metric": METRIC,
            "value": round(total_batch * args.steps / elapsed, 2),
            "unit": "pairs/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_step, 4),
            "higher_is_better": True,
            "scaling": scaling,
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (matching features of a smooth texture shifted by a planar disparity field, "
                    "tests/helpers.py fullsize_inputs; seeded random-init weights, tests/helpers.py seeded_state)",
            "config": {"workload": "hot path: cost volume -> 3D stems -> 3D hourglass -> regression -> "
                                   "ESM upsampler (models/ESMStereo.py:700-745), " + workload,
                       "baseline_config": (f"configs[{args.config}]: {cfg['name']}" if all(
                           getattr(args, k) == cfg[k] for k in ("variant", "cv", "height", "width", "maxdisp"))
                           else f"none (configs[{args.config}] overridden on the command line)"),
                       "variant": args.variant, "cv": args.cv, "global_batch": total_batch,
                       "height": args.height, "width": args.width, "maxdisp": args.maxdisp,
                       "parallelism": f"dp{world}", "graph": hp.graph,
                       "launches_per_step": sum(m.get("launches", 1) for m in meta), "ops_per_step": hp.num_ops},
            "roofline": roof,
            "roofline_step": step_roofline(meta, ms_step, args.batch),
        }
        if use_dist:
            line["collective"] = (f"{torch.distributed.get_backend()} all_gather_into_tensor of the [{args.batch}, "
                                  f"{args.height}, {args.width}] disparities per step" if gather is not None else None)
        mf = [i for i, m in enumerate(meta) if m["name"] == "group_stem"]
        if mf and marg is not None:
            r = kernel_roofline(meta[mf[0]], marg[mf[0]] * 1e-3)
            r.update({"kernel": "group_stem", "kernel_shape": meta[mf[0]].get("shape", ""),
                      "avg_us": round(marg[mf[0]], 2), "timing": "marginal cost inside the replayed graph",
                      "avg_us_back_to_back_warm": round(b2b_ms(mf[0], 20) * 1e3, 2),
                      "traffic": pmc_traffic("group_stem", workload)})
            line["roofline_mfma"] = r
        if marg is not None:
            top = sorted(range(len(marg)), key=lambda i: -marg[i])[:8]
            line["top_ops_in_graph"] = [{"op": meta[i]["name"], "us": round(marg[i], 2)} for i in top]
            line["sum_of_marginals_us"] = round(sum(marg), 1)
        if not args.no_extra:
            line["epe_vs_reference"] = epe_vs_reference(model, args, dev)
            line["roofline_cost_volume"] = cost_volume_roofline(dev)
            # BASELINE configs[2]'s volumes: gwc and build_concat_volume at L-SF B=8 (1.74 / 6.4 GB per launch)
            line["roofline_cost_volume_configs2"] = cost_volume_roofline(dev, reps=8, B=8, H=136, W=240, D=48)
            line["roofline_concat_volume_configs2"] = concat_volume_roofline(dev)
            if world == 1 and args.streams > 1:
                line["concurrent"] = concurrent_streams(model, ml, mr, att, up, args.streams, args.steps, args.warmup,
                                                        dev)
            if world == 1:
                line["forward_e2e"] = forward_e2e(model, args, dev)
        if world == 1 and not args.no_cpu_baseline:
            cb, ref = cpu_baseline(model, ml, mr, att, up, args, args.cpu_seconds)
            line["cpu_baseline"] = cb
            got = hp.outputs[0][:1].detach().cpu()  # the oracle ran the batch's first pair
            line["epe_vs_oracle"] = float((got - ref).abs().mean())
            line["disparity_range_oracle"] = [round(float(ref.min()), 3), round(float(ref.max()), 3)]
        else:
            line["cpu_baseline"] = None
        print(json.dumps(line), flush=True)
    if use_dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
