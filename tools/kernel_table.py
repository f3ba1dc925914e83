"""Per-step time of kernels whose name matches any of the given substrings, from a bench kernel trace (window
between the first and last k_d_loss, as tools/family_time.py), grouped by (kernel, grid blocks).

  python tools/kernel_table.py run_kernel_trace.csv SUBSTR [SUBSTR ...]   ("" = all kernels)
"""
import csv
import sys
from collections import defaultdict

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
pats = sys.argv[2:]
an = [i for i, r in enumerate(rows) if "k_d_loss" in r["Kernel_Name"]]
t, n = defaultdict(float), defaultdict(int)
for r in rows[an[0]:an[-1]]:
    k = r["Kernel_Name"]
    if "spin_kernel" in k or not any(p in k for p in pats):
        continue
    g = (int(r["Grid_Size_X"]) // int(r["Workgroup_Size_X"]), int(r["Grid_Size_Y"]) // max(1, int(r["Workgroup_Size_Y"])),
         int(r["Grid_Size_Z"]))
    name = k.replace("(anonymous namespace)::", "").replace("void ", "").replace("unsigned short", "bf16")
    name = name.replace("mg::", "").split(">(")[0][:110] if "gemm" in name else name.split("(")[0][:70]
    t[(name, g)] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    n[(name, g)] += 1
s = len(an) - 1
tot = sum(t.values()) / s
print(f"{tot:.1f} us/step in {sum(n.values()) / s:.1f} dispatches/step over {s} steps")
for k in sorted(t, key=lambda k: -t[k]):
    print(f"{t[k] / s:8.1f} us {n[k] / s:5.1f}/step avg {t[k] / n[k]:7.1f}  {k[1]}  {k[0]}")
