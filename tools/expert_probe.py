"""Where the expert FFN time goes (C2 shapes, B=256, E=8 top-2, uniform routing): the grouped layer-1 GEMM with no
epilogue, + bias, + bias & GELU, + the saved pre-activation, against a dense GEMM of the same size; the fused C=128
forward with and without saved tensors; the layer-2 GEMM.  HIP events over 20 launches.

    python tools/expert_probe.py
"""
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
for T, C in ((65536, 128), (16384, 256), (4096, 512)):
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
    b2 = torch.zeros(E * C, device=DEV)
    Hid = torch.empty(n, Hd, device=DEV, dtype=bf)
    Pre = torch.empty(n, Hd, device=DEV, dtype=bf)
    Y = torch.empty(n, C, device=DEV, dtype=bf)
    fl1 = 2.0 * n * Hd * C
    g1 = lambda ep: (lambda: ops.gemm_grouped(X, W1, row_off, tile_off, mt, Hd, C, b_gstride=Hd * C, out=Hid, ldb=C,  # noqa
                                              ep=ep))
    cases = [
        ("dense fc1 (same size)", fl1, lambda: ops.gemm(X, W1[:Hd], n, Hd, C, out=Hid)),
        ("grouped fc1 plain", fl1, g1(None)),
        ("grouped fc1 +bias", fl1, g1(ops.E(bias=b1))),
        ("grouped fc1 +bias+GELU", fl1, g1(ops.E(bias=b1, act=L.ACT_GELU))),
        ("grouped fc1 +bias+GELU+Pre", fl1, g1(ops.E(bias=b1, act=L.ACT_GELU, out_pre=Pre, ld_pre=Hd))),
        ("grouped fc2 +bias", fl1, lambda: ops.gemm_grouped(Hid, W2, row_off, tile_off, mt, C, Hd, b_gstride=C * Hd,
                                                            out=Y, ldb=Hd, ep=ops.E(bias=b2))),
    ]
    if ops.ffn_fusable(bf, C) or C == 256:
        W1v, W2v = W1.view(E, Hd, C), W2.view(E, C, Hd)
        cases += [("fused fwd (no save)", 2 * fl1, lambda: ops.moe_ffn_fwd(X, W1v, b1, W2v, b2, row_off, tile_off, mt, Y)),
                  ("fused fwd (Pre+Hid)", 2 * fl1, lambda: ops.moe_ffn_fwd(X, W1v, b1, W2v, b2, row_off, tile_off, mt, Y,
                                                                          pre=Pre, hid=Hid)),
                  ("fused fwd (Pre)", 2 * fl1, lambda: ops.moe_ffn_fwd(X, W1v, b1, W2v, b2, row_off, tile_off, mt, Y,
                                                                      pre=Pre))]
    # weight gradients: gW2 from the stored GELU output vs GELU(Pre) on load; gW1
    gG = torch.randn(n, C, device=DEV, generator=g).to(bf)
    gW2 = torch.zeros(E, C, Hd, device=DEV)
    gW1 = torch.zeros(E, Hd, C, device=DEV)
    cases += [
        ("gW2 from Hid", fl1, lambda: ops.gemm_grouped_wgrad(gG, Hid, row_off, n, C, Hd, gW2)),
        ("gW2 from GELU(Pre) on load", fl1, lambda: ops.gemm_grouped_wgrad(gG, Pre, row_off, n, C, Hd, gW2, b_gelu=1)),
        ("gW1", fl1, lambda: ops.gemm_grouped_wgrad(Hid, X, row_off, n, Hd, C, gW1)),
    ]
    print(f"== T={T} C={C} (rows {n}, Hd {Hd})", flush=True)
    for name, fl, fn in cases:
        t = timed(fn)
        line = f"  {name:30s} {t:7.1f} us  {fl / t / 1e6:6.0f} TF/s"
        if name.startswith("grouped"):  # the same launch on 64^2 tiles (two sub-tiles per dispatch tile)
            L.call("mg_set_tuning", 3, 64)
            t64 = timed(fn)
            L.call("mg_set_tuning", 3, 0)
            line += f" | 64x64 {t64:7.1f} us  {fl / t64 / 1e6:6.0f} TF/s"
        print(line, flush=True)
