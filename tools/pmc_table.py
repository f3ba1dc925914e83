"""Aggregate rocprofv3 --pmc CSVs: mean counter value per (kernel, grid) across dispatches."""
import collections
import csv
import glob
import sys

agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].replace("unsigned short", "bf16")
            short = name[:90]
            grid = r.get("Grid_Size", "")
            key = (short, grid)
            agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
for key, cs in sorted(agg.items()):
    if "gemm_kernel" not in key[0] and "k_" not in key[0]:
        continue
    print(key[0], "grid", key[1])
    line = []
    for c, v in sorted(cs.items()):
        line.append(f"{c}={sum(v) / len(v):.4g}")
    print("   ", "  ".join(line))
