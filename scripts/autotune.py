"""Pick each conv's tile form by measuring it inside the hot path's own launch sequence.

    ESM_NO_TUNED=1 python scripts/autotune.py [--variants S] [--out esmstereo_amd/tuned_hints.json]

For every conv op of the compiled hot path (bench.py's model and synthetic input), each tile
hint the library accepts is forced on that op alone (esm_plan_set_conv_hint), the plan is
replayed as a hipGraph with a hipEvent probe around the op, and the median duration is
recorded.  Ops are tuned in launch order and keep their best hint, so each op is measured
behind the already-chosen producers (the cache state it will run in).  A hint replaces the
automatic choice only when it is faster by more than `--margin`.  The table is keyed by
engine.conv_key (geometry, channel split, batch, extent, epilogue), merged into --out.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

os.environ.setdefault("ESM_AB", "1")  # the package reads A/B knobs only with ESM_AB=1
os.environ.setdefault("ESM_NO_TUNED", "1")
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402
import esmstereo_amd as E  # noqa: E402
from esmstereo_amd._lib import check, lib  # noqa: E402

# 0 = automatic; LDS-staged NT|KS<<4; direct 0x200 (+ rows/wave << 12); rows 0x400; C1 0x114;
# VALU transposed C1 0x10000
# narrow-output 16-block form 1 << 17, automatic without it 1 << 18, VALU 1-input-channel form 1 << 20,
# lean K-split small form 1 << 21, register-weight row-streaming wide form 1 << 22,
# its 3-D plane-streaming twin 1 << 24, the transposed 2-D twin 1 << 25; bits 26-27 = rows per wave of
# the two register-weight 2-D forms; bit 28 = the wide form's K split over two waves, bit 29 = the small form on 8 waves
CANDIDATES = [0, 0x11, 0x12, 0x14, 0x41, 0x42, 0x211, 0x212, 0x241, 0x242, 0x1211, 0x2211, 0x4211, 0x1212,
              0x2212, 0x400, 0x114, 0x10000, 1 << 17, 1 << 18, 1 << 20, 1 << 21, 1 << 22, 1 << 24, 1 << 25,
              (1 << 22) | (1 << 26), (1 << 22) | (2 << 26), (1 << 22) | (3 << 26), (1 << 25) | (1 << 26),
              (1 << 25) | (2 << 26), (1 << 22) | (1 << 28), (1 << 22) | (2 << 26) | (1 << 28),
              (1 << 22) | (3 << 26) | (1 << 28), (1 << 21) | (1 << 29),
              # round 4: the LDS-tiled form (rows per wave automatic / 1 / 2 / 4) and the rules without it
              1 << 23, (1 << 23) | (1 << 26), (1 << 23) | (2 << 26), (1 << 23) | (3 << 26), 1 << 19,
              # round 6: bit 29 with the LDS-tiled form = its LDS-staged weights / padded MT (A/B of the register forms)
              (1 << 23) | (1 << 29), (1 << 23) | (1 << 26) | (1 << 29), (1 << 23) | (2 << 26) | (1 << 29),
              (1 << 23) | (3 << 26) | (1 << 29)]


def op_time(hp, i: int, reps: int) -> float:
    hp.set_probe(i, reps + 2)
    for _ in range(reps + 2):
        hp.launch()
    torch.cuda.synchronize()
    t = sorted(hp.probe_read()[2:])
    return t[len(t) // 2] * 1e3


def step_time(hp, reps: int = 50) -> float:
    hp.set_probe(-1, 1)
    for _ in range(5):
        hp.launch()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        hp.launch()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def tune_variant(variant: str, dev, reps: int, margin: float) -> dict:
    backbone, cvs = bench.VARIANTS[variant]
    model = E.ESMStereo(192, True, False, backbone, cvs)
    bench.seeded_init(model, 1234)
    model = model.eval().to(dev)
    left, right = bench.synthetic_pair(1, 384, 1248, 192, 100, dev)
    with torch.no_grad():
        ml, mr, att, up = model.prefix(left, right)
    B, C, h, w = (int(v) for v in ml.shape)
    hp = E.HotPath(model, B, h, w, 0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], dev,
                   channels=C)
    hp.load_inputs(ml, mr, att, up)
    plan = hp.ctx.plan
    meta = hp.ctx.meta
    base_step = step_time(hp)
    rows = []
    chosen = {}
    for i, m in enumerate(meta):
        if m["kind"] != "conv":
            continue
        res = {}
        for h in CANDIDATES:
            if check(lib.esm_plan_set_conv_hint(plan, i, h), "set_conv_hint") < 0:
                continue
            hp._graph_ready = False
            try:
                res[h] = op_time(hp, i, reps)
            except E.EsmError:
                res[h] = None
        ok = {h: t for h, t in res.items() if t is not None}
        best = min(ok, key=ok.get)
        if best != 0 and ok[best] > ok[0] * (1 - margin):
            best = 0
        lib.esm_plan_set_conv_hint(plan, i, best)
        hp._graph_ready = False
        chosen[m["key"]] = best
        rows.append({"op": m["name"], "key": m["key"], "auto_us": round(ok[0], 2), "best": hex(best),
                     "best_us": round(ok[best], 2), "all": {hex(h): (None if t is None else round(t, 2))
                                                           for h, t in res.items()}})
        print(f"{variant} {m['name'][:44]:44s} auto {ok[0]:7.2f}  best {hex(best):>8s} {ok[best]:7.2f}", flush=True)
    tuned_step = step_time(hp)
    print(f"{variant}: step {base_step:.1f} us (automatic) -> {tuned_step:.1f} us (tuned)", flush=True)
    hp.close()
    return {"variant": variant, "step_auto_us": round(base_step, 1), "step_tuned_us": round(tuned_step, 1),
            "ops": rows, "hints": {k: v for k, v in chosen.items() if v}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="S")
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--margin", type=float, default=0.03)
    ap.add_argument("--out", default=os.path.join(ROOT, "esmstereo_amd", "tuned_hints.json"))
    ap.add_argument("--report", default=os.path.join(ROOT, "gpurun_out", "autotune_report.json"))
    args = ap.parse_args()
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    reports = [tune_variant(v, dev, args.reps, args.margin) for v in args.variants.split(",")]
    table = {"hints": {}}
    if os.path.exists(args.out):
        with open(args.out) as f:
            table = json.load(f)
    for r in reports:
        for op in r["ops"]:  # a key whose best is now the automatic choice drops its old hint
            if op["best"] == "0x0":
                table["hints"].pop(op["key"], None)
        table["hints"].update(r["hints"])
    table["source"] = ("scripts/autotune.py on " + torch.cuda.get_device_name(0) + ": " +
                       ", ".join(f"{r['variant']} {r['step_auto_us']}->{r['step_tuned_us']} us/step" for r in reports))
    os.makedirs(os.path.dirname(args.report), exist_ok=True)
    with open(args.report, "w") as f:
        json.dump(reports, f, indent=1)
    with open(args.out, "w") as f:
        json.dump(table, f, indent=1, sort_keys=True)
    print("wrote", args.out)


if __name__ == "__main__":
    main()
