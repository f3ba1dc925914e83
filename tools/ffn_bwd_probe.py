"""Isolated timing of the expert FFN backward at the C2 16x16 block (B=256 -> T = 65536 tokens, E=8 top-2,
C=128, Hd=512): the fused kernel (mg_moe_ffn_bwd) against the unfused gP GEMM + gX GEMM + bias column sums."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

bf, DEV = torch.bfloat16, "cuda"
C = int(os.environ.get("C", "128"))
T, E, k = int(os.environ.get("T", str(65536 * 128 // C))), int(os.environ.get("E", "8")), int(os.environ.get("K", "2"))
Hd, n = 4 * C, T * k
g = torch.Generator(device=DEV).manual_seed(0)
W1 = (torch.randn(E, Hd, C, device=DEV, generator=g) * C ** -0.5).to(bf)
W2 = (torch.randn(E, C, Hd, device=DEV, generator=g) * Hd ** -0.5).to(bf)
topi = torch.stack([torch.randperm(E, device=DEV, generator=g)[:k] for _ in range(1)]).repeat(T, 1).int()
topi = torch.randint(0, E, (T, k), device=DEV, generator=g, dtype=torch.int32)
gate = torch.rand(T, k, device=DEV, generator=g)
row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
max_tiles = (n + 127) // 128 + E
gG = torch.randn(n, C, device=DEV, generator=g).to(bf)
Pre = torch.randn(n, Hd, device=DEV, generator=g).to(bf)
gP = torch.empty(n, Hd, device=DEV, dtype=bf)
gX = torch.empty(n, C, device=DEV, dtype=bf)
gb1 = torch.zeros(E, Hd, device=DEV)
gb2 = torch.zeros(E, C, device=DEV)


def unfused():
    ops.gemm_grouped(gG, W2.view(-1), row_off, tile_off, max_tiles, Hd, C, b_kc=False, b_gstride=C * Hd, out=gP,
                     ldb=Hd, ep=ops.E(act=L.ACT_MUL_GELU_GRAD, aux=Pre, ld_aux=Hd))
    ops.gemm_grouped(gP, W1.view(-1), row_off, tile_off, max_tiles, C, Hd, b_kc=False, b_gstride=Hd * C, out=gX, ldb=C)
    ops.grouped_colsum(gP, row_off, Hd, n, gb1.view(-1))


def fused():
    ops.moe_ffn_bwd(gG, Pre, W1, W2, row_off, tile_off, max_tiles, gP, gX, gb1, gb2)


gf = 2 * 2.0 * n * C * Hd / 1e9
def fused_2blk():
    L.call("mg_set_tuning", 14, 2)
    fused()
    L.call("mg_set_tuning", 14, 0)


for name, fn in (("unfused gP+gX+colsum", unfused), ("fused (1 block/CU)", fused), ("fused, 2 blocks/CU", fused_2blk)):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(20):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / 20 * 1e3
    print(f"C={C} {name:24s} {us:8.1f} us  {gf / us * 1e3:7.1f} TF/s ({gf:.1f} GF)", flush=True)
