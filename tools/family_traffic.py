"""HBM traffic per family per step from the two rocprofv3 --pmc passes of tools/gpu.sh pmc (FETCH_SIZE and
WRITE_SIZE, one counter set per run, over ``bench.py --eager --steps 2 --warmup 1``).

  python tools/family_traffic.py FETCH.csv WRITE.csv OUT.json [batch E dtype]

The window runs between the first and the last ``k_d_loss`` dispatch (once per training step), so it holds whole
steps; kernels map to families by name (moegan_mi/roofline.py).  gfx950 corrections (MI355X_MICROARCH.md,
HBM / rocprofv3): FETCH_SIZE reports half the bytes of a wide coalesced read, so it is doubled; WRITE_SIZE is
exact; both counters are in KiB.  The counters sit on the L2's memory side (Infinity-Cache hits included).
"""
import csv
import json
import os
import sys
from collections import defaultdict

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "moe-gan_cpsc541_amd"))
from moegan_mi.roofline import kernel_family  # noqa: E402


def per_family(path, counter):
    rows = [r for r in csv.DictReader(open(path)) if r["Counter_Name"] == counter]
    rows.sort(key=lambda r: int(r["Dispatch_Id"]))
    anchors = [i for i, r in enumerate(rows) if "k_d_loss" in r["Kernel_Name"]]
    if len(anchors) < 2:
        raise SystemExit(f"{path}: need at least two k_d_loss dispatches")
    win = rows[anchors[0]:anchors[-1]]
    kib = defaultdict(float)
    n = defaultdict(int)
    for r in win:
        f = kernel_family(r["Kernel_Name"])
        kib[f] += float(r["Counter_Value"])
        n[f] += 1
    return kib, n, len(anchors) - 1


def main():
    fetch, write, out = sys.argv[1:4]
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 256
    experts = int(sys.argv[5]) if len(sys.argv) > 5 else 8
    dtype = sys.argv[6] if len(sys.argv) > 6 else "bf16"
    fk, fn, steps = per_family(fetch, "FETCH_SIZE")
    wk, _, wsteps = per_family(write, "WRITE_SIZE")
    assert steps == wsteps, (steps, wsteps)
    fams = {}
    for f in sorted(set(fk) | set(wk)):
        rd = fk.get(f, 0.0) * 2 * 1024 / steps / 1e6
        wr = wk.get(f, 0.0) * 1024 / steps / 1e6
        fams[f] = {"mb_per_step": round(rd + wr, 2), "read_mb_per_step": round(rd, 2), "write_mb_per_step": round(wr, 2),
                   "dispatches_per_step": round(fn.get(f, 0) / steps, 1)}
    rec = {"batch": batch, "experts": experts, "dtype": dtype, "fp8": False, "steps_profiled": float(steps),
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes over bench.py --eager (FETCH x2, KiB x1024)",
           "families": fams}
    json.dump(rec, open(out, "w"), indent=1)
    tot = sum(v["mb_per_step"] for v in fams.values())
    print(f"{steps} steps; {tot:.0f} MB of HBM traffic per step")
    for f, v in sorted(fams.items(), key=lambda kv: -kv[1]["mb_per_step"]):
        print(f"{f:18s} {v['mb_per_step']:9.1f} MB/step  (read {v['read_mb_per_step']:.1f}, write "
              f"{v['write_mb_per_step']:.1f})  {v['dispatches_per_step']:5.1f} dispatches/step")


if __name__ == "__main__":
    main()
