"""Per-kernel issue profile of the step from one rocprofv3 --pmc pass (SQ counters): summed over dispatches,
ranked by wave-cycles; VALU / MFMA instruction ratio and the parked (WAIT_ANY) share.
    python tools/pmc_step_issue.py <counter_collection.csv> [steps] [second pass: LDS counters csv]"""
import collections
import csv
import sys

tot = collections.defaultdict(lambda: collections.defaultdict(float))
tot2 = collections.defaultdict(lambda: collections.defaultdict(float))
calls = collections.Counter()
seen = set()
for r in csv.DictReader(open(sys.argv[1])):
    name = r["Kernel_Name"].replace("unsigned short", "bf16").replace("(anonymous namespace)::", "").replace("mg::", "").replace("void ", "")[:110]
    tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
    did = r.get("Dispatch_Id") or r.get("Correlation_Id")
    if (name, did) not in seen:
        seen.add((name, did))
        calls[name] += 1
if len(sys.argv) > 3:
    for r in csv.DictReader(open(sys.argv[3])):
        name = r["Kernel_Name"].replace("unsigned short", "bf16").replace("(anonymous namespace)::", "").replace("mg::", "").replace("void ", "")[:110]
        tot2[name][r["Counter_Name"]] += float(r["Counter_Value"])
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
allwc = sum(c.get("SQ_WAVE_CYCLES", 0) for c in tot.values())
print(f"{'share':>6} {'calls':>6} {'VALU/MFMA':>9} {'wait%':>6} {'active%':>7} {'LDSwait%':>8} {'bankconf%':>9} "
      f"{'MFMAbusy%':>9}  kernel")
for name, c in sorted(tot.items(), key=lambda kv: -kv[1].get("SQ_WAVE_CYCLES", 0))[:40]:
    wc = c.get("SQ_WAVE_CYCLES", 0)
    mf = c.get("SQ_INSTS_MFMA", 0)
    ratio = c.get("SQ_INSTS_VALU", 0) / mf if mf else float("inf")
    c2 = tot2.get(name, {})
    wc2 = max(c2.get("SQ_WAVE_CYCLES", 0), 1)
    lds_idx = max(c2.get("SQ_LDS_IDX_ACTIVE", 0), 1)
    print(f"{100 * wc / allwc:5.1f}% {calls[name] / steps:6.1f} {ratio:9.1f} {100 * c.get('SQ_WAIT_ANY', 0) / max(wc, 1):5.0f}% "
          f"{100 * c.get('SQ_ACTIVE_INST_ANY', 0) / max(wc, 1):6.0f}% "
          f"{100 * c2.get('SQ_WAIT_INST_LDS', 0) / wc2:7.0f}% {100 * c2.get('SQ_LDS_BANK_CONFLICT', 0) / lds_idx:8.0f}% "
          f"{100 * c2.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / wc2:8.0f}%  {name}")
