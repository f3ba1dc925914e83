"""Rocprof duration and PMC traffic of bench.py's roofline kernel, found between its mg_mark kernels.

bench.py times the largest call of the step's dominant family live (moegan_mi/_lib.LiveTimer) and brackets every
launch of it with an empty k_roofline_mark_begin / k_roofline_mark_end dispatch.  In a rocprofv3 kernel trace (or
a --pmc counter CSV) of the same bench command, the dispatches between a begin and the next end mark are exactly
that call's kernels, so their summed duration (trace) and summed FETCH_SIZE / WRITE_SIZE (PMC) are per-launch
figures of the same call -- no kernel-name matching.

    python tools/roofline_kernel.py CONFIG BENCH_JSON_LINE_FILE TRACE.csv [FETCH.csv WRITE.csv] [--last N]

Updates profiles/roofline_kernel.json[CONFIG] with the call's signature (from the bench line of the same run), the
workload (batch, experts), the rocprof average per launch over the last N bracketed launches (the timed region's;
default: every launch after the first two), and -- from the PMC passes -- the HBM bytes per launch (FETCH_SIZE x2,
the gfx950 correction of MI355X_MICROARCH.md §HBM, + WRITE_SIZE; counters in KiB).
"""
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OUT = os.path.join(REPO, "profiles", "roofline_kernel.json")


def bracketed_trace(path):
    """[(duration_ms, [kernel names])] per begin/end pair of a kernel-trace CSV, in time order."""
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    out, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "k_roofline_mark_begin" in n:
            cur = (r["Queue_Id"], [])
        elif "k_roofline_mark_end" in n:
            if cur is not None and cur[1]:
                out.append((sum(d for d, _ in cur[1]), [k for _, k in cur[1]]))
            cur = None
        elif cur is not None and r["Queue_Id"] == cur[0]:
            cur[1].append(((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6, n))
    return out


def bracketed_counter(path, counter):
    """[summed counter value] per begin/end pair of a --pmc counter CSV (dispatch order)."""
    disp = defaultdict(float)
    names = {}
    for r in csv.DictReader(open(path)):
        d = int(r["Dispatch_Id"])
        names[d] = r["Kernel_Name"]
        if r["Counter_Name"] == counter:
            disp[d] += float(r["Counter_Value"])
    out, cur = [], None
    for d in sorted(names):
        n = names[d]
        if "k_roofline_mark_begin" in n:
            cur = []
        elif "k_roofline_mark_end" in n:
            if cur:
                out.append(sum(cur))
            cur = None
        elif cur is not None:
            cur.append(disp.get(d, 0.0))
    return out


def main():
    argv = sys.argv[1:]
    last = None
    if "--last" in argv:
        i = argv.index("--last")
        last = int(argv[i + 1])
        del argv[i:i + 2]
    cfg, line_file, trace = argv[:3]
    pmc = argv[3:5] if len(argv) >= 5 else None
    line = json.loads([x for x in open(line_file) if x.startswith("{")][-1])
    roof = line["roofline"]
    launches = bracketed_trace(trace)
    if not launches:
        raise SystemExit("no bracketed launches in the trace (run bench.py without --no-families)")
    sel = launches[-last:] if last else launches[2:] or launches
    avg = sum(d for d, _ in sel) / len(sel)
    kernels = sorted({k for _, ks in sel for k in ks})
    rec = {"batch": line["config"]["global_batch"] // max(1, line["n_gpus"]), "experts": line["config"]["experts"],
           "signature": None, "kernel": roof.get("kernel"), "rocprof_avg_ms": round(avg, 5),
           "rocprof_launches": len(sel), "live_avg_ms_same_run": roof.get("avg_launch_ms"),
           "kernels": [k[:160] for k in kernels],
           "source": f"rocprofv3 --kernel-trace of the bench run ({os.path.basename(os.path.dirname(trace))}): the "
                     f"dispatches between mg_mark begin / end, last {len(sel)} launches"}
    rec["signature"] = roof.get("signature")
    if pmc:
        f = bracketed_counter(pmc[0], "FETCH_SIZE")
        w = bracketed_counter(pmc[1], "WRITE_SIZE")
        if f and w:
            rd = 2.0 * sum(f) / len(f) * 1024
            wr = sum(w) / len(w) * 1024
            alg = roof.get("algorithmic_bytes_per_launch")
            rec.update({"read_bytes_per_launch": round(rd), "write_bytes_per_launch": round(wr),
                        "traffic_bytes_per_launch": round(rd + wr), "pmc_launches": min(len(f), len(w)),
                        "pmc_source": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE (separate runs) of bench.py "
                                      "--eager over the same bracketed call; FETCH_SIZE x2 (gfx950), KiB x1024"})
            if alg:
                rec["algorithmic_bytes_per_launch"] = alg
                rec["traffic_over_algorithmic"] = round((rd + wr) / alg, 3)
    allrec = json.load(open(OUT)) if os.path.exists(OUT) else {}
    allrec[cfg] = rec
    json.dump(allrec, open(OUT, "w"), indent=1)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
