"""Measure and tune the hot path by its own step time (no profiler, no probe events in the graph).

    python scripts/step_tune.py --mode marginal --variants S      # per-op marginal cost in the chain
    ESM_NO_TUNED=1 python scripts/step_tune.py --mode tune --variants S,M,L --out esmstereo_amd/tuned_hints.json

`marginal`: each op is dropped from the replayed graph in turn (esm_plan_set_repeat(i, 0)); the
step time with the op minus the step time without it is what the op costs the chain, its launch
gap and its cache effects on the next op included.  Baseline and dropped replays are interleaved.

`tune`: for each conv op in launch order, every tile hint the library accepts is forced on that
op, the graph is rebuilt and the whole step is timed with an event pair around a batch of
replays; rounds over the candidates are interleaved (clock drift hits all of them alike) and the
median per candidate decides.  A hint replaces the current choice only when the step is faster
by more than --margin-us.  The event probe of scripts/autotune.py adds its own graph nodes around
the op, whose cost (~15 us) hides the 1-2 us differences that matter at S-K; this does not.
"""
from __future__ import annotations

import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))

os.environ.setdefault("ESM_AB", "1")  # the package reads A/B knobs only with ESM_AB=1
import torch  # noqa: E402

import bench  # noqa: E402
import esmstereo_amd as E  # noqa: E402
from esmstereo_amd._lib import lib  # noqa: E402
from autotune import CANDIDATES  # noqa: E402


BATCH = 1  # --batch: pairs per plan (the L-K per-rank slice of configs[3] is B = 4)
HW = (384, 1248, 192)  # --height / --width / --maxdisp (configs[2]: 544 x 960; configs[4]: 1024 x 1504 md256)


def build(variant: str, dev):
    backbone, cvs = bench.VARIANTS[variant]
    model = E.ESMStereo(HW[2], True, False, backbone, cvs)
    bench.seeded_init(model, 1234)
    model = model.eval().to(dev)
    left, right = bench.synthetic_pair(BATCH, HW[0], HW[1], HW[2], 100, dev)
    with torch.no_grad():
        ml, mr, att, up = model.prefix(left, right)
    B, C, h, w = (int(v) for v in ml.shape)
    hp = E.HotPath(model, B, h, w, 0 if att is None else int(att.shape[1]), [tuple(u.shape) for u in up], dev,
                   channels=C)
    hp.load_inputs(ml, mr, att, up)
    return hp


def graph_ok(hp) -> bool:
    hp._graph_ready = False
    try:
        hp.launch()
    except E.EsmError:
        hp._graph_ready = False
        return False
    torch.cuda.synchronize()
    return True


def window(hp, reps: int, warm: int = 3) -> float:
    """us per replay of the built graph over `reps` back-to-back replays (one event pair)."""
    for _ in range(warm):
        hp.launch()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        hp.launch()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / reps * 1e3


def reps_for(hp) -> int:
    graph_ok(hp)
    t = window(hp, 10)
    return max(8, int(16000 / t))  # ~16 ms per window


def marginal(variant: str, dev, rounds: int) -> dict:
    hp = build(variant, dev)
    plan, meta = hp.ctx.plan, hp.ctx.meta
    reps = reps_for(hp)
    rows = []
    for i, m in enumerate(meta):
        base, drop = [], []
        for _ in range(rounds):
            graph_ok(hp)
            base.append(window(hp, reps))
            lib.esm_plan_set_repeat(plan, i, 0)
            graph_ok(hp)
            drop.append(window(hp, reps))
            lib.esm_plan_set_repeat(plan, i, 1)
        b, d = statistics.median(base), statistics.median(drop)
        rows.append({"op": m["name"], "kind": m["kind"], "shape": m.get("shape", ""), "hint": m.get("hint", 0),
                     "step_us": round(b, 2), "marginal_us": round(b - d, 2)})
        print(f"{variant} {i:3d} {m['name'][:48]:48s} {b - d:7.2f} us   (step {b:7.1f})", flush=True)
    graph_ok(hp)
    step = statistics.median(window(hp, reps) for _ in range(5))
    tot = sum(r["marginal_us"] for r in rows)
    print(f"{variant}: step {step:.1f} us, sum of marginals {tot:.1f} us", flush=True)
    hp.close()
    return {"variant": variant, "step_us": round(step, 1), "ops": rows}


def step_only(variant: str, dev, rounds: int) -> dict:
    hp = build(variant, dev)
    reps = reps_for(hp)
    graph_ok(hp)
    ts = [window(hp, reps) for _ in range(max(rounds, 5) * 4)]
    hp.close()
    med = statistics.median(ts)
    print(f"{variant}: step {med:.2f} us (min {min(ts):.2f}, max {max(ts):.2f}, {len(ts)} windows of {reps})", flush=True)
    return {"variant": variant, "step_us": round(med, 2), "windows": [round(t, 2) for t in ts]}


def tune(variant: str, dev, rounds: int, margin_us: float, only=()) -> dict:
    hp = build(variant, dev)
    plan, meta = hp.ctx.plan, hp.ctx.meta
    reps = reps_for(hp)
    graph_ok(hp)
    step0 = statistics.median(window(hp, reps) for _ in range(5))
    chosen, rows = {}, []
    for i, m in enumerate(meta):
        if m["kind"] != "conv" or (only and not any(o in m["name"] for o in only)):
            continue
        cur = lib.esm_plan_set_conv_hint(plan, i, 0)
        lib.esm_plan_set_conv_hint(plan, i, cur)
        cands = []
        for h in dict.fromkeys([cur, 0] + CANDIDATES):
            if lib.esm_plan_set_conv_hint(plan, i, h) >= 0 and graph_ok(hp):
                cands.append(h)
        times = {h: [] for h in cands}
        for _ in range(rounds):
            for h in cands:
                lib.esm_plan_set_conv_hint(plan, i, h)
                graph_ok(hp)
                times[h].append(window(hp, reps))
        med = {h: statistics.median(v) for h, v in times.items()}
        best = min(med, key=med.get)
        if med[best] > med[cur] - margin_us:
            best = cur
        lib.esm_plan_set_conv_hint(plan, i, best)
        chosen.setdefault(m["key"], []).append(best)
        rows.append({"op": m["name"], "key": m["key"], "was": hex(cur), "best": hex(best),
                     "gain_us": round(med[cur] - med[best], 2),
                     "all": {hex(h): round(t - med[cur], 2) for h, t in sorted(med.items(), key=lambda kv: kv[1])}})
        print(f"{variant} {m['name'][:44]:44s} {hex(cur):>9s} -> {hex(best):>9s}  {med[cur] - med[best]:6.2f} us", flush=True)
    graph_ok(hp)
    step1 = statistics.median(window(hp, reps) for _ in range(5))
    print(f"{variant}: step {step0:.1f} -> {step1:.1f} us", flush=True)
    hp.close()
    # ops sharing a key took their choices in order; the last (seen behind every earlier choice) wins
    return {"variant": variant, "step_before_us": round(step0, 1), "step_after_us": round(step1, 1), "ops": rows,
            "hints": {k: v[-1] for k, v in chosen.items()}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", choices=["marginal", "tune", "step"], default="marginal")
    ap.add_argument("--variants", default="S")
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--margin-us", type=float, default=0.3)
    ap.add_argument("--out", default="")
    ap.add_argument("--only", default="", help="tune: comma-separated substrings of the op names to tune")
    ap.add_argument("--batch", type=int, default=1, help="pairs per plan (hint keys carry B)")
    ap.add_argument("--height", type=int, default=384)
    ap.add_argument("--width", type=int, default=1248)
    ap.add_argument("--maxdisp", type=int, default=192)
    ap.add_argument("--report", default=os.path.join(ROOT, "gpurun_out", "step_tune_report.json"))
    args = ap.parse_args()
    global BATCH, HW
    BATCH = args.batch
    HW = (args.height, args.width, args.maxdisp)
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    variants = args.variants.split(",")
    if args.mode == "marginal":
        reports = [marginal(v, dev, args.rounds) for v in variants]
    elif args.mode == "step":
        reports = [step_only(v, dev, args.rounds) for v in variants]
    else:
        only = tuple(o for o in args.only.split(",") if o)
        reports = [tune(v, dev, args.rounds, args.margin_us, only) for v in variants]
    os.makedirs(os.path.dirname(args.report), exist_ok=True)
    with open(args.report, "w") as f:
        json.dump(reports, f, indent=1)
    if args.mode == "tune" and args.out:
        table = {"hints": {}}
        if os.path.exists(args.out):
            with open(args.out) as f:
                table = json.load(f)
        for r in reports:
            for k, h in r["hints"].items():
                if h:
                    table["hints"][k] = h
                else:
                    table["hints"].pop(k, None)
        table["source"] = ("scripts/step_tune.py on " + torch.cuda.get_device_name(0) + ": " +
                           ", ".join(f"{r['variant']} {r['step_before_us']}->{r['step_after_us']} us/step"
                                     for r in reports))
        with open(args.out, "w") as f:
            json.dump(table, f, indent=1, sort_keys=True)
        print("wrote", args.out)


if __name__ == "__main__":
    main()
