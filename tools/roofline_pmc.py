"""HBM traffic per launch of the bench line's roofline kernels from two rocprofv3 --pmc passes over the eager C2 step
(tools/gpu.sh pmc: FETCH_SIZE and WRITE_SIZE in separate runs), written to profiles/pmc_roofline_kernel.json.

gfx950 correction (MI355X_MICROARCH.md §HBM): FETCH_SIZE reports half the bytes of a wide coalesced read -> doubled;
WRITE_SIZE is exact for 16-B/lane stores and fp32 atomics.  Counters in KiB.  The counters sit on the L2's memory
side, so Infinity-Cache hits are included.

    python tools/roofline_pmc.py FETCH.csv WRITE.csv OUT.json
"""
import csv
import json
import sys

# (key, kernel-name substring, Grid_Size in threads, algorithmic bytes per launch, description)
B = 256
KERNELS = [
    ("moe_ffn_bwd_16", "k_moe_ffn_bwd_w2<128, 128>", 1032 * 512,
     # gG in (n x C bf16), Pre in (n x 4C), gP out (n x 4C), gX out (n x C); n = 2 * B * 256 routed rows
     (2 * B * 256) * (128 * 2 + 512 * 2 + 512 * 2 + 128 * 2),
     "fused expert FFN backward, 16x16 block (mg_moe_ffn_bwd, C=128, Hd=512, 131072 routed rows)"),
    ("d_conv1", "128, 256, true, true, mg::LdKCConv", 512 * 256,
     # h0 in (B x 32 x 32 x 128 bf16) + weights (256 x 2048 bf16) + h1 out (B x 16 x 16 x 256 bf16)
     B * 32 * 32 * 128 * 2 + 256 * 2048 * 2 + B * 16 * 16 * 256 * 2,
     "D conv_layers.2 forward (mg_conv2d_fwd, implicit GEMM M=65536 N=256 K=2048, 128x256 tiles)"),
]


def per_launch(path, counter, name, grid):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and name in r["Kernel_Name"] and int(r["Grid_Size"]) == grid]
    return (sum(vals) / len(vals) if vals else None), len(vals)


def main():
    fetch_csv, write_csv, out = sys.argv[1:4]
    rec = {"batch": B, "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate runs) over "
                                 "bench.py --eager --steps 2 --warmup 1 --no-families (tools/gpu.sh pmc); "
                                 "FETCH_SIZE x2 (gfx950 correction), KiB x1024", "kernels": {}}
    for key, name, grid, alg, desc in KERNELS:
        f, nf = per_launch(fetch_csv, "FETCH_SIZE", name, grid)
        w, nw = per_launch(write_csv, "WRITE_SIZE", name, grid)
        if f is None or w is None:
            print(f"{key}: not found (fetch {nf}, write {nw} launches)")
            continue
        rd, wr = 2.0 * f * 1024, w * 1024
        rec["kernels"][key] = {"kernel": desc, "launches": min(nf, nw), "read_bytes_per_launch": round(rd),
                               "write_bytes_per_launch": round(wr), "traffic_bytes_per_launch": round(rd + wr),
                               "algorithmic_bytes_per_launch": alg, "traffic_over_algorithmic": round((rd + wr) / alg, 3)}
        print(f"{key}: {nf} launches, read {rd / 1e6:.1f} MB + write {wr / 1e6:.1f} MB = {(rd + wr) / 1e6:.1f} MB per "
              f"launch (algorithmic {alg / 1e6:.1f} MB, x{(rd + wr) / alg:.2f})")
    json.dump(rec, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
