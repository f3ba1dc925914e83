"""Isolated timing of the step's linear-layer weight gradients (C += A^T B, bf16 [K][M] x [K][N], fp32 C through an
atomic epilogue) at their C2 shapes: the wide split-K kernel (mg_wgrad_wide.hip) vs the generic split-K GEMM."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"
SHAPES = [(384, 128, 65536), (128, 128, 65536), (768, 256, 16384), (256, 256, 16384), (1536, 512, 4096),
          (512, 512, 4096), (256, 16, 65536)]
for M, N, K in SHAPES:
    g = torch.Generator(device=DEV).manual_seed(0)
    A = torch.randn(K, M, device=DEV, generator=g).bfloat16()
    B = torch.randn(K, N, device=DEV, generator=g).bfloat16()
    C = torch.zeros(M, N, device=DEV)
    res = []
    for mode in (1, 2, 0):  # generic, wide (forced), automatic routing
        L.call("mg_set_tuning", 15, mode)
        fn = lambda: ops.gemm(A, B, M, N, K, a_kc=False, b_kc=False, out=C, ep=ops.E(atomic=1), splits=0)  # noqa
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / 20 * 1e3)
    L.call("mg_set_tuning", 15, 0)
    mb = K * (M + N) * 2 / 1e6
    print(f"({M:5d},{N:4d},{K:6d}) generic {res[0]:7.1f} us  wide {res[1]:7.1f} us  auto {res[2]:7.1f} us  "
          f"({mb:.0f} MB operands: {mb / res[1]:.2f} TB/s wide)", flush=True)
