"""Isolated timing of the step's grouped expert GEMMs (8x8 block: 32768 routed rows, C=256, Hd=1024; 4x4 block:
8192 rows, C=512, Hd=2048; E=8) and the dense short-K projections under the XCD tile-order setting (tuning slot 6:
0 none, 1 every launch), HIP events over 20 launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV, bf = "cuda", torch.bfloat16


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


E = 8
for T, C in ((16384, 256), (4096, 512)):
    g = torch.Generator(device=DEV).manual_seed(0)
    n, Hd = 2 * T, 4 * C
    topi = torch.randint(0, E, (T, 2), device=DEV, generator=g, dtype=torch.int32)
    gate = torch.rand(T, 2, device=DEV, generator=g)
    row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
    mt = (n + 127) // 128 + E
    X = torch.randn(n, C, device=DEV, generator=g).to(bf)
    W1 = (torch.randn(E * Hd, C, device=DEV, generator=g) * C ** -0.5).to(bf)
    W2 = (torch.randn(E * C, Hd, device=DEV, generator=g) * Hd ** -0.5).to(bf)
    b1 = torch.zeros(E * Hd, device=DEV)
    Hid = torch.empty(n, Hd, device=DEV, dtype=bf)
    Y = torch.empty(n, C, device=DEV, dtype=bf)
    cases = {
        f"grouped ({n},{Hd},{C}) GELU": lambda: ops.gemm_grouped(X, W1, row_off, tile_off, mt, Hd, C, b_gstride=Hd * C,
                                                                 out=Hid, ldb=C, ep=ops.E(bias=b1, act=L.ACT_GELU)),
        f"grouped ({n},{C},{Hd})": lambda: ops.gemm_grouped(Hid, W2, row_off, tile_off, mt, C, Hd, b_gstride=C * Hd,
                                                            out=Y, ldb=Hd),
    }
    for name, fn in cases.items():
        res = []
        for v in (0, 1):
            L.call("mg_set_tuning", 6, v)
            res.append(timed(fn))
        L.call("mg_set_tuning", 6, 0)
        L.call("mg_set_tuning", 3, 257)  # 128 x 256 tiles
        res.append(timed(fn))
        L.call("mg_set_tuning", 3, 0)
        print(f"{name:34s} no-xcd {res[0]:6.1f} us  xcd {res[1]:6.1f} us  128x256 {res[2]:6.1f} us", flush=True)
for M, N, K in ((65536, 384, 128), (65536, 256, 128), (16384, 768, 256), (16384, 512, 256)):
    g = torch.Generator(device=DEV).manual_seed(0)
    A = torch.randn(M, K, device=DEV, generator=g).to(bf)
    Bw = torch.randn(N, K, device=DEV, generator=g).to(bf)
    Cc = torch.empty(M, N, device=DEV, dtype=bf)
    res = []
    for v in (0, 1):
        L.call("mg_set_tuning", 6, v)
        res.append(timed(lambda: ops.gemm(A, Bw, M, N, K, out=Cc)))
    L.call("mg_set_tuning", 6, 0)
    print(f"dense ({M},{N},{K}){'':14s} no-xcd {res[0]:6.1f} us  xcd {res[1]:6.1f} us", flush=True)
