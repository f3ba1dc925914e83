"""Source hash of libmoegan_hip: sha256 over the HIP sources, their headers and the C-ABI header.

The Makefile bakes it into the library (mg_source_hash()); the Python binding recomputes it from the
tree it ships with and smoke() asserts the two agree, so the binary that runs is the one these sources
build (a stale prebuilt .so fails loudly).  Standard library only: the build runs it before torch exists.
"""
import glob
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))


def source_files(csrc=HERE):
    files = sorted(glob.glob(os.path.join(csrc, "*.hip")) + glob.glob(os.path.join(csrc, "*.h")))
    files.append(os.path.join(csrc, "..", "..", "include", "moegan_hip.h"))
    return files


def source_hash(csrc=HERE):
    h = hashlib.sha256()
    for f in source_files(csrc):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_hash())
