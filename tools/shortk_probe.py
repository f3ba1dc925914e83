"""Isolated timing of the step's short-K GEMMs (K = 128 .. 384 over 16K-64K token rows: the attention / MoE
projections and the 1x1 skip convs) under each tile override (tuning slot 3: 0 automatic, 64, 128, 256 = 256x128,
257 = 128x256), HIP events over 20 launches, with the algorithmic HBM bytes (A + B read once, C written once)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV, bf = "cuda", torch.bfloat16
# (M, N, K, a_kc, b_kc, bias)
SHAPES = [(65536, 384, 128, 1, 1, True), (65536, 256, 128, 1, 0, False), (65536, 128, 128, 1, 1, True),
          (65536, 128, 128, 1, 0, False), (16384, 768, 256, 1, 1, True), (16384, 512, 256, 1, 0, False),
          (65536, 128, 384, 1, 0, False), (4096, 512, 512, 1, 0, False)]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for M, N, K, akc, bkc, has_bias in SHAPES:
    g = torch.Generator(device=DEV).manual_seed(0)
    A = torch.randn(M, K, device=DEV, generator=g).to(bf)
    B = (torch.randn(N, K, device=DEV, generator=g) if bkc else torch.randn(K, N, device=DEV, generator=g)).to(bf)
    C = torch.empty(M, N, device=DEV, dtype=bf)
    ep = ops.E(bias=torch.randn(N, device=DEV, generator=g)) if has_bias else None
    mb = (M * K + N * K + M * N) * 2 / 1e6
    res = []
    for tile in (0, 64, 128, 256, 257):
        L.call("mg_set_tuning", 3, tile)
        res.append(timed(lambda: ops.gemm(A, B, M, N, K, a_kc=bool(akc), b_kc=bool(bkc), out=C, ep=ep)))
    L.call("mg_set_tuning", 3, 0)
    print(f"({M:5d},{N:4d},{K:4d}) kc={akc}{bkc} " + "  ".join(f"{t}:{r:6.1f}" for t, r in
                                                             zip(("auto", 64, 128, 256, 257), res)) +
          f" us  ({mb:.0f} MB: {mb / min(res):.2f} TB/s best)", flush=True)
