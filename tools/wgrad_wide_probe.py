"""Isolated timing of the step's long-reduction weight gradients (C += A^T B, bf16 [K][M] x [K][N], fp32 C through
an atomic epilogue) at their C2 shapes -- the linear layers' (attention in / out projections, router features) and
the 1x1 convolutions' (Cout x Cin over B*H*W pixels) -- through the long-reduction kernel (mg_wgrad_wide.hip) at
several grid targets vs the generic split-K GEMM, and a parity check of the kernel against the generic result."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"
SHAPES = [(384, 128, 65536), (128, 128, 65536), (128, 256, 65536), (768, 256, 16384), (256, 256, 16384),
          (256, 512, 16384), (1536, 512, 4096), (512, 512, 4096), (256, 16, 65536)]
MODES = (2, 4)


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


for M, N, K in SHAPES:
    g = torch.Generator(device=DEV).manual_seed(0)
    A = torch.randn(K, M, device=DEV, generator=g).bfloat16()
    B = torch.randn(K, N, device=DEV, generator=g).bfloat16()
    C = torch.zeros(M, N, device=DEV)
    fn = lambda: ops.gemm(A, B, M, N, K, a_kc=False, b_kc=False, out=C, ep=ops.E(atomic=1), splits=0)  # noqa
    res = {}
    L.call("mg_set_tuning", 15, 1)
    res["generic"] = timeit(fn)
    C.zero_()
    fn()
    ref = C.clone()
    errs = []
    for mode in MODES:
        L.call("mg_set_tuning", 15, mode)
        for tb in (128, 256, 512):
            L.call("mg_set_tuning", 27, tb)
            res[f"{'w' if mode == 2 else 'w256'}/{tb}"] = timeit(fn)
        L.call("mg_set_tuning", 27, 0)
        C.zero_()
        fn()
        torch.cuda.synchronize()
        errs.append(((C - ref).norm() / ref.norm()).item())
    err = max(errs)
    L.call("mg_set_tuning", 15, 0)
    res["auto"] = timeit(fn)
    mb = K * (M + N) * 2 / 1e6
    best = min(v for k_, v in res.items() if k_.startswith("w"))
    print(f"({M:5d},{N:4d},{K:6d}) " + "  ".join(f"{k_} {v:6.1f}" for k_, v in res.items()) +
          f"  us | {mb:.0f} MB operands, best wide {mb / best:.2f} TB/s, rel diff vs generic {err:.1e}", flush=True)
