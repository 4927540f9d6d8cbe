"""Per-op comparison of two step_tune.py --mode marginal reports (A/B libraries on one box).

    python scripts/ab_compare.py gpurun_out/marginal_A.json gpurun_out/marginal_B.json
"""
import json
import sys

a, b = (json.load(open(p)) for p in sys.argv[1:3])
for ra, rb in zip(a, b):
    print(f"{ra['variant']}: step A {ra['step_us']} us  B {rb['step_us']} us  (B - A {rb['step_us'] - ra['step_us']:+.1f})")
    rows = [(ob["marginal_us"] - oa["marginal_us"], oa, ob) for oa, ob in zip(ra["ops"], rb["ops"])]
    for d, oa, ob in sorted(rows, key=lambda r: r[0]):
        if abs(d) >= 0.25:
            print(f"  {d:+6.2f}  {oa['op'][:50]:50s} A {oa['marginal_us']:6.2f}  B {ob['marginal_us']:6.2f}")
