"""Isolated timing of the fused expert FFN (mg_moe_ffn_fwd) at the C2 16x16 block shape (T = 65536 tokens, C = 128,
E = 8 top-2) with and without the saved pre-activation / GELU output, next to the two grouped GEMMs it replaces.
GPU diagnostic:  python tools/ffn_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "moe-gan_cpsc541_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    from moegan_mi import _lib as L, ops
    from test_ffn_gpu import _case
    bf = torch.bfloat16
    for T, C, E, k in ((65536, 128, 8, 2), (16384, 256, 8, 2)):
        tok, W1, b1, W2, b2, topi, gate = _case(T, C, E, k, 1)
        Hd = 4 * C
        row_off, tile_off, perm, _, _ = ops.moe_dispatch(topi, gate, E)
        n = T * k
        mt = (n + 127) // 128 + E
        Xg = ops.gather_rows(tok, perm, k)
        Pre = torch.empty(n, Hd, device="cuda", dtype=bf)
        Hid = torch.empty(n, Hd, device="cuda", dtype=bf)
        Y = torch.empty(n, C, device="cuda", dtype=bf)
        flop = 4.0 * n * C * Hd
        t_ng = timed(lambda: ops.moe_ffn_fwd(tok, W1, b1, W2, b2, row_off, tile_off, mt, Y, x_idx=perm, x_idx_div=k))
        t_sv = timed(lambda: ops.moe_ffn_fwd(Xg, W1, b1, W2, b2, row_off, tile_off, mt, Y, pre=Pre, hid=Hid))

        def unfused():
            ops.gemm_grouped(Xg, W1.view(-1), row_off, tile_off, mt, Hd, C, b_gstride=Hd * C, out=Hid, ldb=C,
                             ep=ops.E(bias=b1, act=L.ACT_GELU, out_pre=Pre, ld_pre=Hd))
            ops.gemm_grouped(Hid, W2.view(-1), row_off, tile_off, mt, C, Hd, b_gstride=C * Hd, out=Y, ldb=Hd,
                             ep=ops.E(bias=b2))
        t_un = timed(unfused)
        print(f"T={T} C={C} E={E} k={k}: fused no-grad {t_ng:.1f} us ({flop / t_ng / 1e6:.0f} TF/s), fused saving "
              f"{t_sv:.1f} us, two grouped GEMMs {t_un:.1f} us")


if __name__ == "__main__":
    main()
