"""Instruction-class census of the loops of one kernel in a hipcc -S listing (gfx950).

  python tools/isa_loops.py <file.s> <symbol-substring> [...more substrings]

Prints the kernel's register/occupancy metadata and, for every backward branch (a loop), the counts of
MFMA / VALU / SALU / VMEM / DS / waitcnt instructions between the target label and the branch.
"""
import re
import sys
from collections import Counter


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith("s_barrier"):
        return "barrier"
    if op.startswith("s_"):
        return "salu"
    if op.startswith(("global_load", "buffer_load", "flat_load")):
        return "vmem_ld"
    if op.startswith(("global_store", "buffer_store", "flat_store", "global_atomic", "buffer_atomic")):
        return "vmem_st"
    if op.startswith("ds_read") or op.startswith("ds_load"):
        return "ds_rd"
    if op.startswith("ds_"):
        return "ds_wr"
    return "other"


def main():
    src = open(sys.argv[1]).read().split("\n")
    subs = sys.argv[2:]
    start = None
    for i, l in enumerate(src):
        if re.match(r"^_Z\S*:", l) and all(s in l for s in subs):
            start = i
            break
    if start is None:
        print("kernel not found")
        return
    name = src[start].split(":")[0]
    end = next(i for i in range(start, len(src)) if src[i].startswith(".Lfunc_end"))
    body = src[start:end]
    labels = {}
    instrs = []
    for l in body:
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            if re.match(r"^\.LBB\S+:", s):
                labels[s[:-1]] = len(instrs)
            continue
        if re.match(r"^\S+:", s):
            continue
        instrs.append(s.split(";")[0].strip())
    print(name, "instructions:", len(instrs))
    for l in src[end:end + 400]:
        if any(k in l for k in (".vgpr_count", ".sgpr_count", ".agpr_count", "lds_size", "Occupancy",
                                 "spill", "ScratchSize", "private_segment")):
            print("  ", l.strip())
        if l.startswith(".end_amdgpu_metadata"):
            break
    for i, ins in enumerate(instrs):
        op = ins.split()[0]
        if op.startswith("s_cbranch") or op == "s_branch":
            tgt = ins.split()[-1]
            if tgt in labels and labels[tgt] <= i:
                c = Counter(classify(x.split()[0]) for x in instrs[labels[tgt]:i + 1])
                print(f"loop {tgt} [{labels[tgt]}..{i}] len {i + 1 - labels[tgt]}: " +
                      " ".join(f"{k}={v}" for k, v in sorted(c.items())))


if __name__ == "__main__":
    main()
