"""Summarise a rocprofv3 kernel_stats.csv: top kernels by total time."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else None
tot = sum(float(r["TotalDurationNs"]) for r in rows)
if steps:
    print(f"total kernel time {tot / 1e6:.2f} ms ({tot / 1e6 / steps:.2f} ms per step over {steps:g} steps)")
else:  # the stats cover everything the command ran (setup, warm-up, timed steps): no per-step figure
    print(f"total kernel time {tot / 1e6:.2f} ms over the whole traced command")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    n = r["Name"].replace("unsigned short", "bf16").replace("(anonymous namespace)::", "")
    n = n.split("(")[0] if not n.startswith("void mg::gemm") else n[:150]
    print(f"{float(r['TotalDurationNs']) / 1e6:8.2f} ms {100 * float(r['TotalDurationNs']) / tot:5.1f}% "
          f"calls {r['Calls']:>5} avg {float(r['AverageNs']) / 1e3:8.1f} us  {n}")
