"""Isolated timing of the step's grouped expert weight gradients (out[g] += A_g^T B_g over each expert's routed
rows; E=8 top-2 at B=256: 16x16 block 131072 rows, C=128, Hd=512; 8x8 block 32768 rows, C=256; 4x4 block 8192 rows,
C=512) against the split-K count (fp32 atomics across splits), HIP events over 20 launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import ops  # noqa: E402

DEV, bf, E = "cuda", torch.bfloat16, 8


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


for T, C in ((65536, 128), (16384, 256), (4096, 512)):
    g = torch.Generator(device=DEV).manual_seed(0)
    n, Hd = 2 * T, 4 * C
    topi = torch.randint(0, E, (T, 2), device=DEV, generator=g, dtype=torch.int32)
    gate = torch.rand(T, 2, device=DEV, generator=g)
    row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
    gP = torch.randn(n, Hd, device=DEV, generator=g).to(bf)
    X = torch.randn(n, C, device=DEV, generator=g).to(bf)
    for M, N, A, Bm in ((Hd, C, gP, X), (C, Hd, X, gP)):
        out = torch.zeros(E, M, N, device=DEV)
        res = []
        for sp in (0, 2, 4, 8, 16, 32):
            res.append(timed(lambda: ops.gemm_grouped_wgrad(A, Bm, row_off, n, M, N, out, splits=sp)))
        gf = 2.0 * n * M * N / 1e9
        print(f"grouped wgrad ({M:4d},{N:4d}) rows {n:6d}: " + "  ".join(
            f"{'auto' if s == 0 else s}:{t:6.1f}" for s, t in zip((0, 2, 4, 8, 16, 32), res)) +
              f" us  (best {gf / min(res) * 1e3:.0f} TF/s)", flush=True)
