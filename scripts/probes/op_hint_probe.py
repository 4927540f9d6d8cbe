"""Per-op form probe inside the replayed graph: for each hint, the op is launched R times per replay
(esm_plan_set_repeat) and its time is (step(R) - step(1)) / (R - 1), the median over interleaved rounds.
Usage: python scripts/probes/op_hint_probe.py --variant L --batch 4 --op aggregation_out.conv1.0 --hints 0x800000,0x4800000
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
import step_tune as ST  # noqa: E402
from esmstereo_amd._lib import lib  # noqa: E402
import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="L")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--op", action="append", required=True)
    ap.add_argument("--hints", action="append", required=True,
                    help="per --op (same order): comma-separated hints (hex ok); 'cur' = the table's")
    ap.add_argument("--repeat", type=int, default=5)
    ap.add_argument("--rounds", type=int, default=3)
    args = ap.parse_args()
    ST.BATCH = args.batch
    dev = torch.device("cuda:0")
    hp = ST.build(args.variant, dev)
    plan, meta = hp.ctx.plan, hp.ctx.meta
    for name, hint_list in zip(args.op, args.hints):
        idx = [i for i, m in enumerate(meta) if m["name"] == name]
        if not idx:
            print(f"{name}: not in the plan"); continue
        i = idx[0]
        cur = lib.esm_plan_set_conv_hint(plan, i, 0)
        lib.esm_plan_set_conv_hint(plan, i, cur)
        hints = [cur if h == "cur" else int(h, 0) for h in hint_list.split(",")]
        res = {h: [] for h in hints}
        for _ in range(args.rounds):
            for h in hints:
                if lib.esm_plan_set_conv_hint(plan, i, h) < 0:
                    continue
                lib.esm_plan_set_repeat(plan, i, 1)
                if not ST.graph_ok(hp):
                    continue
                t1 = statistics.median(ST.window(hp, 20) for _ in range(3))
                lib.esm_plan_set_repeat(plan, i, args.repeat)
                ST.graph_ok(hp)
                tr = statistics.median(ST.window(hp, 20) for _ in range(3))
                res[h].append((tr - t1) / (args.repeat - 1))
        lib.esm_plan_set_repeat(plan, i, 1)
        lib.esm_plan_set_conv_hint(plan, i, cur)
        for h, v in res.items():
            if v:
                print(f"{name:40s} hint {h:#010x}{' (cur)' if h == cur else ''}: {statistics.median(v):8.2f} us "
                      f"({', '.join(f'{x:.1f}' for x in v)})", flush=True)
    hp.close()


if __name__ == "__main__":
    main()
