"""One traced step in launch order: every dispatch of the last whole step (between two k_d_loss dispatches) with its
duration, the idle gap before it, family and grid -- to see the step's structure and its launch-latency tail.

    python tools/step_sequence.py run_kernel_trace.csv [--min-us 0]
"""
import argparse
import csv
import os
import re
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "moe-gan_cpsc541_amd"))
from moegan_mi.roofline import kernel_family  # noqa: E402


def short(name):
    n = name.replace("unsigned short", "bf16").replace("(anonymous namespace)::", "").replace("mg::", "")
    n = n.replace("void ", "")
    return re.sub(r"\(.*", "", n)[:110]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--min-us", type=float, default=0.0)
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    anchors = [i for i, r in enumerate(rows) if "k_d_loss" in r["Kernel_Name"]]
    win = rows[anchors[-2]:anchors[-1]]
    t0 = int(win[0]["Start_Timestamp"])
    prev_end = t0
    busy = 0.0
    for r in win:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        d = (e - s) / 1e3
        busy += d
        gap = (s - prev_end) / 1e3
        prev_end = max(prev_end, e)
        if d >= a.min_us:
            grid = f'{r["Grid_Size_X"]}x{r["Grid_Size_Y"]}x{r["Grid_Size_Z"]}/{r["Workgroup_Size_X"]}'
            print(f"{(s - t0) / 1e3:9.1f} {d:8.1f} gap {gap:6.1f}  {kernel_family(r['Kernel_Name']) or '-':16s} "
                  f"{grid:20s} {short(r['Kernel_Name'])}")
    span = (int(win[-1]["End_Timestamp"]) - t0) / 1e3
    print(f"# {len(win)} dispatches, busy {busy:.1f} us, span {span:.1f} us")


if __name__ == "__main__":
    main()
