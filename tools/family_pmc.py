"""HBM traffic per kernel family per step from two rocprofv3 --pmc passes over the eager bench step.

  rocprofv3 --pmc FETCH_SIZE -d D1 -o run --output-format csv -- python3 bench.py --eager --steps S --warmup W ...
  rocprofv3 --pmc WRITE_SIZE -d D2 ...  (same command)
  python tools/family_pmc.py D1/..counter_collection.csv D2/..counter_collection.csv STEPS OUT.json [batch E dtype [fp8]]

Kernels map to families by name (moegan_mi/roofline.py KERNELS).  gfx950 correction (MI355X_MICROARCH.md §HBM):
FETCH_SIZE counts half the bytes of a wide coalesced read -> doubled; WRITE_SIZE exact.  Both counters in KiB.
The totals include Infinity-Cache hits (the counters sit on the L2's memory side).
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "moe-gan_cpsc541_amd"))
from moegan_mi.roofline import kernel_family  # noqa: E402


def per_family(path, counter):
    acc = defaultdict(float)
    n = defaultdict(int)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        f = kernel_family(r["Kernel_Name"])
        acc[f] += float(r["Counter_Value"]) * 1024.0
        n[f] += 1
    return acc, n


def main():
    fetch_csv, write_csv, steps, out = sys.argv[1], sys.argv[2], float(sys.argv[3]), sys.argv[4]
    batch = int(sys.argv[5]) if len(sys.argv) > 5 else 256
    experts = int(sys.argv[6]) if len(sys.argv) > 6 else 8
    dtype = sys.argv[7] if len(sys.argv) > 7 else "bf16"
    fp8 = len(sys.argv) > 8 and sys.argv[8] in ("1", "fp8", "mx8")
    rd, nr = per_family(fetch_csv, "FETCH_SIZE")
    wr, _ = per_family(write_csv, "WRITE_SIZE")
    fams = {}
    for f in sorted(set(rd) | set(wr)):
        r, w = 2.0 * rd.get(f, 0.0) / steps, wr.get(f, 0.0) / steps
        fams[f] = {"mb_per_step": round((r + w) / 1e6, 2), "read_mb_per_step": round(r / 1e6, 2),
                   "write_mb_per_step": round(w / 1e6, 2), "dispatches_per_step": round(nr.get(f, 0) / steps, 1)}
    rec = {"batch": batch, "experts": experts, "dtype": dtype, "fp8": fp8, "steps_profiled": steps,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --eager (FETCH x2, KiB x1024)",
           "families": fams}
    json.dump(rec, open(out, "w"), indent=1)
    for f, v in sorted(fams.items(), key=lambda kv: -kv[1]["mb_per_step"]):
        print(f"{f:18s} {v['mb_per_step']:10.1f} MB/step (read {v['read_mb_per_step']:.1f}, write "
              f"{v['write_mb_per_step']:.1f}), {v['dispatches_per_step']} dispatches/step")


if __name__ == "__main__":
    main()
