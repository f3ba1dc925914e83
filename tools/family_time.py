"""Kernel time per family per step from a rocprofv3 --kernel-trace CSV of bench.py.

  python tools/family_time.py run_kernel_trace.csv OUT.json [batch E dtype [fp8]]

The window runs over whole steps between dispatches of ``k_d_loss`` (launched once per training step).  With
FAMILY_LAST=N (the scripts pass the timed step count minus one) only the last N whole steps count: with bench.py
--no-families those are hipGraph replays of the timed region, not the eager warm-up steps (a window
that included the eager and attribution steps made the per-family busy time exceed the timed step).  Kernels map
to families by name (moegan_mi/roofline.py KERNELS).
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "moe-gan_cpsc541_amd"))
from moegan_mi.roofline import kernel_family  # noqa: E402


def main():
    path, out = sys.argv[1], sys.argv[2]
    batch = int(sys.argv[3]) if len(sys.argv) > 3 else 256
    experts = int(sys.argv[4]) if len(sys.argv) > 4 else 8
    dtype = sys.argv[5] if len(sys.argv) > 5 else "bf16"
    fp8 = len(sys.argv) > 6 and sys.argv[6] in ("1", "fp8", "mx8")
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    anchors = [i for i, r in enumerate(rows) if "k_d_loss" in r["Kernel_Name"]]
    if len(anchors) < 2:
        raise SystemExit("need at least two traced steps")
    last = int(os.environ.get("FAMILY_LAST", "0"))
    if last > 0:
        anchors = anchors[-(last + 1):]
    steps = len(anchors) - 1
    win = rows[anchors[0]:anchors[-1]]
    t = defaultdict(float)
    n = defaultdict(int)
    for r in win:
        if "spin_kernel" in r["Kernel_Name"]:  # the attribution step's lead spin (moegan_mi/roofline.py)
            continue
        f = kernel_family(r["Kernel_Name"])
        t[f] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        n[f] += 1
    span = (int(win[-1]["End_Timestamp"]) - int(win[0]["Start_Timestamp"])) / 1e6 / steps
    busy = sum(t.values()) / steps
    fams = {f: {"ms_per_step": round(t[f] / steps, 4), "dispatches_per_step": round(n[f] / steps, 1)} for f in t}
    rec = {"batch": batch, "experts": experts, "dtype": dtype, "fp8": fp8, "steps_in_window": steps,
           "busy_ms_per_step": round(busy, 4), "span_ms_per_step": round(span, 4),
           "source": (f"rocprofv3 --kernel-trace of bench.py, the last {steps} replayed timed steps" if last > 0 else
                      f"rocprofv3 --kernel-trace of bench.py, {steps} steps between the first and last k_d_loss"),
           "families": fams}
    json.dump(rec, open(out, "w"), indent=1)
    print(f"{steps} steps; busy {busy:.3f} ms/step, span {span:.3f} ms/step")
    for f, v in sorted(fams.items(), key=lambda kv: -kv[1]["ms_per_step"]):
        print(f"{f:18s} {v['ms_per_step']:8.3f} ms/step  {v['dispatches_per_step']:6.1f} dispatches/step")


if __name__ == "__main__":
    main()
