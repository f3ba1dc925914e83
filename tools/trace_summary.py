"""Summarise a rocprofv3 kernel_trace.csv per (kernel, grid): time per step, calls per step, and the
device idle time between dispatches.

  python tools/trace_summary.py <kernel_trace.csv> <steps> [top]
"""
import csv
import sys
from collections import defaultdict


def short(name):
    n = name.replace("unsigned short", "bf16").replace("(anonymous namespace)::", "").replace("void ", "")
    if n.startswith("mg::gemm"):
        n = n.split(">(")[0] + ">"
        return n.replace("mg::", "")
    return n.split("(")[0].split("<")[0] if "<" not in n.split("(")[0] else n.split("(")[0]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    key = lambda r, k: next((r[c] for c in r if c.lower() == k.lower()), None)  # noqa: E731
    evs = []
    for r in rows:
        s, e = int(key(r, "Start_Timestamp")), int(key(r, "End_Timestamp"))
        grid = tuple(int(key(r, f"Grid_Size_{a}") or 0) for a in "XYZ")
        wg = tuple(int(key(r, f"Workgroup_Size_{a}") or 0) for a in "XYZ")
        blocks = tuple(g // max(w, 1) for g, w in zip(grid, wg))
        evs.append((s, e, short(key(r, "Kernel_Name")), blocks))
    evs.sort()
    busy = sum(e - s for s, e, _, _ in evs)
    span = evs[-1][1] - evs[0][0]
    print(f"{len(evs)} dispatches, {len(evs) / steps:.0f}/step; busy {busy / 1e6 / steps:.3f} ms/step, "
          f"span {span / 1e6 / steps:.3f} ms/step, idle {(span - busy) / 1e6 / steps:.3f} ms/step")
    agg = defaultdict(lambda: [0, 0])
    byname = defaultdict(lambda: [0, 0])
    for s, e, n, b in evs:
        agg[(n, b)][0] += e - s
        agg[(n, b)][1] += 1
        byname[n][0] += e - s
        byname[n][1] += 1
    print("\n-- by kernel --")
    for n, (t, c) in sorted(byname.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / 1e3 / steps:9.1f} us/step {100 * t / busy:5.1f}% {c / steps:6.1f}/step  {n}")
    print("\n-- by kernel and grid (blocks) --")
    for (n, b), (t, c) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:top]:
        print(f"{t / 1e3 / steps:9.1f} us/step {c / steps:5.1f}/step avg {t / c / 1e3:8.1f} us  {b}  {n}")


if __name__ == "__main__":
    main()
