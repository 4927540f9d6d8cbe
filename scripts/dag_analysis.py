"""Dependency DAG of the hot-path launch list and its critical path.

    python bench.py --kernel-table ops.json ...        (on the GPU box)
    python scripts/dag_analysis.py ops.json

An op depends on every earlier op it has a RAW / WAW / WAR hazard with, judged on the
allocations (base, bytes) each op reads and writes.  With per-op probe times this gives the
serial sum, the critical path (the floor for a graph whose independent ops run concurrently)
and the DAG width per level.
"""
from __future__ import annotations

import json
import sys


def overlaps(a, b):
    return any(p < q + m and q < p + n for p, n in a for q, m in b)


def build_deps(ops):
    deps = []
    for j, oj in enumerate(ops):
        d = []
        for i in range(j):
            oi = ops[i]
            if (overlaps(oi["writes"], oj["reads"]) or overlaps(oi["writes"], oj["writes"])
                    or overlaps(oi["reads"], oj["writes"])):
                d.append(i)
        deps.append(d)
    return deps


def main():
    ops = json.load(open(sys.argv[1]))
    t = [o["median_ms"] * 1e3 for o in ops]
    deps = build_deps(ops)
    finish, prev, level = [], [], []
    for j in range(len(ops)):
        best = max(deps[j], key=lambda i: finish[i], default=None)
        finish.append((finish[best] if best is not None else 0.0) + t[j])
        prev.append(best)
        level.append(1 + max((level[i] for i in deps[j]), default=-1))
    end = max(range(len(ops)), key=lambda j: finish[j])
    path = []
    while end is not None:
        path.append(end)
        end = prev[end]
    path.reverse()
    print(f"ops {len(ops)}  serial sum {sum(t):.1f} us  critical path {finish[path[-1]]:.1f} us  "
          f"levels {max(level) + 1}")
    width = {}
    for lv in level:
        width[lv] = width.get(lv, 0) + 1
    print("width per level:", [width[k] for k in sorted(width)])
    print("critical path:")
    for j in path:
        print(f"  {t[j]:7.2f} us  {ops[j]['name'][:50]:50s} {ops[j].get('shape', '')}")
    off = [j for j in range(len(ops)) if j not in set(path)]
    print(f"off the critical path: {len(off)} ops, {sum(t[j] for j in off):.1f} us")
    for j in sorted(off, key=lambda j: -t[j])[:20]:
        print(f"  {t[j]:7.2f} us  {ops[j]['name'][:50]:50s} deps {deps[j][-3:]}")


if __name__ == "__main__":
    main()
