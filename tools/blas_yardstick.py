"""Library yardstick for the GEMM core: the C2 step's GEMM shapes as PLAIN bf16 GEMMs, timed with torch.matmul
(hipBLASLt) and with mg_gemm on the same explicit operands, in one process.  The implicit convolutions appear as
their im2col-equivalent [pixels x taps*Cin] GEMMs, so the hipBLASLt figure is what a library reaches on the same
arithmetic without the conv loaders; weight gradients as C = A^T B over K = pixels / routed rows.

    python tools/blas_yardstick.py [--iters 20]
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))

import torch  # noqa: E402

# (name, M, N, K, kind): kind "nt" C = A B^T (A [M,K], B [N,K]); "tn" C = A^T B (A [K,M], B [K,N]) (weight gradients)
SHAPES = [
    ("d_conv1_fwd", 65536, 256, 2048, "nt"),
    ("conv16_fwd 3x3 128->128", 65536, 128, 1152, "nt"),
    ("conv16_fwd 3x3 256->128", 65536, 128, 2304, "nt"),
    ("conv8_fwd 3x3 256->256", 16384, 256, 2304, "nt"),
    ("conv8_fwd 3x3 512->256", 16384, 256, 4608, "nt"),
    ("conv4_fwd 3x3 512->512", 4096, 512, 4608, "nt"),
    ("expert fc1 8^2 (one expert x8)", 4096 * 8, 1024, 256, "nt"),
    ("expert fc2 8^2", 4096 * 8, 256, 1024, "nt"),
    ("expert fc1 4^2", 1024 * 8, 2048, 512, "nt"),
    ("token proj 16^2 (K=128)", 65536, 384, 128, "nt"),
    ("styles fp32-size M=256", 256, 4864, 512, "nt"),
    ("wgrad conv16 3x3", 128, 1152, 65536, "tn"),
    ("wgrad conv8 3x3", 256, 4608, 16384, "tn"),
    ("wgrad conv4 3x3", 512, 4608, 4096, "tn"),
    ("wgrad d_conv1", 256, 2048, 65536, "tn"),
    ("wgrad expert 16^2 (per expert x1)", 128, 512, 16384, "tn"),
    ("wgrad expert 4^2", 512, 2048, 1024, "tn"),
]


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from moegan_mi import ops
    dev = "cuda"
    bf = torch.bfloat16
    torch.manual_seed(0)
    print(f"{'shape':36s} {'M':>6} {'N':>6} {'K':>6}   hipBLASLt us  TF/s |   mg_gemm us  TF/s")
    for name, M, N, K, kind in SHAPES:
        fl = 2.0 * M * N * K
        if kind == "nt":
            A = torch.randn(M, K, device=dev).to(bf)
            Bm = torch.randn(N, K, device=dev).to(bf)
            t_lib = timeit(lambda: torch.matmul(A, Bm.t()), a.iters)
            out = torch.empty(M, N, device=dev, dtype=bf)
            t_mg = timeit(lambda: ops.gemm(A, Bm, M, N, K, out=out), a.iters)
        else:
            A = torch.randn(K, M, device=dev).to(bf)
            Bm = torch.randn(K, N, device=dev).to(bf)
            t_lib = timeit(lambda: torch.matmul(A.t(), Bm), a.iters)
            out = torch.zeros(M, N, device=dev)
            t_mg = timeit(lambda: ops.gemm(A, Bm, M, N, K, a_kc=False, b_kc=False, out=out, ep=ops.E(atomic=1),
                                           splits=0), a.iters)
        print(f"{name:36s} {M:6d} {N:6d} {K:6d}   {t_lib:10.1f} {fl / t_lib / 1e6:6.0f} | {t_mg:10.1f} "
              f"{fl / t_mg / 1e6:6.0f}")


if __name__ == "__main__":
    main()
