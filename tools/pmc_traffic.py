"""HBM traffic per launch of one kernel from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE).

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports exactly half the bytes of a
wide coalesced streaming read -> doubled; WRITE_SIZE is exact for 16-B/lane streaming stores.
Both counters are in KiB.  Usage:
  python tools/pmc_traffic.py FETCH.csv WRITE.csv "<kernel-name substring>" GRID_SIZE
"""
import csv
import sys


def per_launch(path, counter, name, grid):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and name in r["Kernel_Name"] and int(r["Grid_Size"]) == grid]
    return (sum(vals) / len(vals) if vals else None), len(vals)


def main():
    fetch_csv, write_csv, name, grid = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4])
    f, nf = per_launch(fetch_csv, "FETCH_SIZE", name, grid)
    w, nw = per_launch(write_csv, "WRITE_SIZE", name, grid)
    read_b = 2.0 * f * 1024 if f is not None else None
    write_b = w * 1024 if w is not None else None
    tot = (read_b or 0) + (write_b or 0)
    print(f"launches: fetch {nf}, write {nw}")
    print(f"FETCH_SIZE {f} KiB -> corrected read {read_b / 1e6 if read_b else None} MB")
    print(f"WRITE_SIZE {w} KiB -> write {write_b / 1e6 if write_b else None} MB")
    print(f"traffic per launch: {tot:.0f} bytes ({tot / 1e6:.2f} MB)")


if __name__ == "__main__":
    main()
