"""K-loop census of one kernel in a hipcc -S listing: for every loop (backward branch) that contains MFMAs, the
counts of MFMA / VALU / buffer loads / barriers and the s_waitcnt lines in it.

  python tools/kloop.py <file.s> <mangled-name-prefix>
"""
import re
import sys


def main(path, prefix):
    lines = open(path).read().split("\n")
    i = next(k for k, l in enumerate(lines) if l.startswith(prefix) and l.split(":")[0].startswith(prefix) and ": ;" in l)
    j = i
    while not lines[j].strip().startswith("s_endpgm"):
        j += 1
    body = lines[i:j]
    labels = {}
    for k, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = k
    print("mfma in kernel:", sum("v_mfma" in x for x in body), "lines:", len(body))
    for k, l in enumerate(body):
        m = re.search(r"s_cbranch_\w+\s+(\.LBB\w+)|s_branch\s+(\.LBB\w+)", l)
        if not m:
            continue
        t = m.group(1) or m.group(2)
        if t in labels and labels[t] < k:
            seg = body[labels[t]:k + 1]
            n_mf = sum("v_mfma" in x for x in seg)
            if n_mf:
                valu = sum(x.strip().startswith("v_") and "mfma" not in x for x in seg)
                print(f"loop {t} [{labels[t]}..{k}] mfma {n_mf} valu {valu} salu "
                      f"{sum(x.strip().startswith('s_') for x in seg)} buffer_load {sum('buffer_load' in x for x in seg)} "
                      f"ds_read {sum('ds_read' in x for x in seg)} ds_write {sum('ds_write' in x for x in seg)} "
                      f"barrier {sum('s_barrier' in x for x in seg)}")
                print("   waits:", [x.strip().split(";")[0] for x in seg if "s_waitcnt" in x])


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
