"""Fused expert FFN forward (mg_moe_ffn_fwd) against the two grouped GEMMs it replaces (mg_gemm_grouped with the
bias + GELU (pre-activation saved) and bias epilogues): bit-identical Y, pre-activation and GELU output, with the
dispatch gather inside the kernel or from pre-gathered rows; skewed and empty experts, ragged last tiles."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"
bf = torch.bfloat16


def _case(T, C, E, k, seed, empty_expert=False):
    g = torch.Generator(device=DEV).manual_seed(seed)
    tok = (torch.randn(T, C, device=DEV, generator=g)).to(bf)
    Hd = 4 * C
    W1 = (torch.randn(E, Hd, C, device=DEV, generator=g) * C ** -0.5).to(bf)
    b1 = torch.randn(E * Hd, device=DEV, generator=g) * 0.1
    W2 = (torch.randn(E, C, Hd, device=DEV, generator=g) * Hd ** -0.5).to(bf)
    b2 = torch.randn(E * C, device=DEV, generator=g) * 0.1
    topi = torch.randint(0, E, (T, k), device=DEV, generator=g, dtype=torch.int32)
    topi[: T // 3, 0] = 2  # skew
    if empty_expert:
        topi[topi == E - 1] = 0
    gate = torch.rand(T, k, device=DEV, generator=g)
    return tok, W1, b1, W2, b2, topi, gate


@pytest.mark.parametrize("T,C,E,k", [(65536, 128, 8, 2), (16384, 256, 8, 2), (1000, 128, 8, 2), (300, 256, 4, 1),
                                     (2048, 128, 32, 4)])
def test_fused_ffn_matches_grouped_gemms(T, C, E, k):
    tok, W1, b1, W2, b2, topi, gate = _case(T, C, E, k, T + C, empty_expert=(T == 1000))
    Hd = 4 * C
    row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
    n = T * k
    max_tiles = (n + 127) // 128 + E
    Xg = ops.gather_rows(tok, perm, k)
    # reference: the unfused path of engine_g.moe_fwd
    Pre_r = torch.empty(n, Hd, device=DEV, dtype=bf)
    Hid_r = torch.empty(n, Hd, device=DEV, dtype=bf)
    ops.gemm_grouped(Xg, W1.view(-1), row_off, tile_off, max_tiles, Hd, C, b_gstride=Hd * C, out=Hid_r, ldb=C,
                     ep=ops.E(bias=b1, act=L.ACT_GELU, out_pre=Pre_r, ld_pre=Hd))
    Y_r = torch.empty(n, C, device=DEV, dtype=bf)
    ops.gemm_grouped(Hid_r, W2.view(-1), row_off, tile_off, max_tiles, C, Hd, b_gstride=C * Hd, out=Y_r, ldb=Hd,
                     ep=ops.E(bias=b2))
    # fused, saved tensors
    Pre = torch.empty(n, Hd, device=DEV, dtype=bf)
    Hid = torch.empty(n, Hd, device=DEV, dtype=bf)
    Y = torch.empty(n, C, device=DEV, dtype=bf)
    ops.moe_ffn_fwd(Xg, W1, b1, W2, b2, row_off, tile_off, max_tiles, Y, pre=Pre, hid=Hid)
    # fused, gather inside, nothing saved
    Y2 = torch.empty(n, C, device=DEV, dtype=bf)
    ops.moe_ffn_fwd(tok, W1, b1, W2, b2, row_off, tile_off, max_tiles, Y2, x_idx=perm, x_idx_div=k)
    torch.cuda.synchronize()
    assert torch.equal(Pre, Pre_r)
    assert torch.equal(Hid, Hid_r)
    assert torch.equal(Y, Y_r)
    assert torch.equal(Y2, Y_r)
    # and against float64 math on the same bf16 operands (sampled rows)
    rows = torch.randperm(n, device=DEV)[:64]
    e_of = torch.bucketize(rows.int(), row_off[1:].contiguous(), right=True)
    x = Xg[rows].double()
    h = torch.einsum("rc,rhc->rh", x, W1[e_of].double()) + b1.view(E, Hd)[e_of].double()
    hg = torch.nn.functional.gelu(h).to(bf).double()
    y = torch.einsum("rh,rch->rc", hg, W2[e_of].double()) + b2.view(E, C)[e_of].double()
    assert (Y[rows].double() - y).abs().max() <= 2e-2 * y.abs().max() + 1e-3


@pytest.mark.parametrize("occ", [0, 2])
@pytest.mark.parametrize("T,E,k,skew,C", [(65536, 8, 2, False, 128), (1000, 8, 2, True, 128), (2048, 32, 4, False, 128),
                                          (77, 4, 1, True, 128), (16384, 8, 2, False, 256), (300, 4, 1, True, 256)])
def test_fused_ffn_backward_matches_grouped_gemms(T, E, k, skew, C, occ):
    """Fused expert backward (mg_moe_ffn_bwd, t2i_moe_gan.py:257-263 backward) against the unfused path of
    engine_g.moe_bwd: gP = gG W2_e with the GELU' epilogue and gX = gP W1_e (mg_gemm_grouped) bit-identical; the
    bias gradient against mg_grouped_colsum of the same gP (fp32 summation order) and against float64 sums; C = 128
    and 256 (the 16x16 / 8x8 blocks), both occupancy forms (tuning slot 14), empty experts, ragged last tiles, the C5
    routing (E=32 top-4)."""
    Hd = 4 * C
    L.call("mg_set_tuning", 14, occ)
    tok, W1, b1, W2, b2, topi, gate = _case(T, C, E, k, T * 3 + E, empty_expert=skew)
    row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
    n = T * k
    max_tiles = (n + 127) // 128 + E
    g = torch.Generator(device=DEV).manual_seed(T + 1)
    gG = torch.randn(n, C, device=DEV, generator=g).to(bf)
    Pre = torch.randn(n, Hd, device=DEV, generator=g).to(bf)
    gP_r = torch.empty(n, Hd, device=DEV, dtype=bf)
    ops.gemm_grouped(gG, W2.view(-1), row_off, tile_off, max_tiles, Hd, C, b_kc=False, b_gstride=C * Hd, out=gP_r,
                     ldb=Hd, ep=ops.E(act=L.ACT_MUL_GELU_GRAD, aux=Pre, ld_aux=Hd))
    gX_r = torch.empty(n, C, device=DEV, dtype=bf)
    ops.gemm_grouped(gP_r, W1.view(-1), row_off, tile_off, max_tiles, C, Hd, b_kc=False, b_gstride=Hd * C, out=gX_r,
                     ldb=C)
    gb1_r = torch.full((E * Hd,), 0.25, device=DEV)
    ops.grouped_colsum(gP_r, row_off, Hd, n, gb1_r)
    gP = torch.empty(n, Hd, device=DEV, dtype=bf)
    gX = torch.empty(n, C, device=DEV, dtype=bf)
    gb1 = torch.full((E, Hd), 0.25, device=DEV)
    gb2 = torch.full((E, C), -0.5, device=DEV)
    Hid = torch.empty(n, Hd, device=DEV, dtype=bf)
    ops.moe_ffn_bwd(gG, Pre, W1, W2, row_off, tile_off, max_tiles, gP, gX, gb1, gb2, hid=Hid)
    # GELU(Pre) out of the backward = the GELU the W2 weight gradient forms on load: the two weight gradients are
    # bit-identical (deterministic mode: one writer per element, same MFMA inputs and order)
    L.call("mg_set_tuning", 11, 1)
    try:
        gw_load = ops.gemm_grouped_wgrad(gG, Pre, row_off, n, C, Hd, torch.zeros(E, C, Hd, device=DEV), b_gelu=1)
        gw_hid = ops.gemm_grouped_wgrad(gG, Hid, row_off, n, C, Hd, torch.zeros(E, C, Hd, device=DEV))
    finally:
        L.call("mg_set_tuning", 11, 0)
    gb2_r = torch.full((E * C,), -0.5, device=DEV)
    ops.grouped_colsum(gG, row_off, C, n, gb2_r)
    torch.cuda.synchronize()
    L.call("mg_set_tuning", 14, 0)
    assert torch.equal(gP, gP_r)
    assert torch.equal(gX, gX_r)
    assert torch.equal(gw_hid, gw_load)
    hid_ref = F.gelu(Pre.float()).to(bf)  # (exact erf vs the fast form: at most one bf16 ulp apart)
    assert float((Hid.float() - hid_ref.float()).abs().max()) <= float(hid_ref.float().abs().max()) * 2 ** -7
    scale = float((gb1_r - 0.25).abs().max())
    assert float((gb1.view(-1) - gb1_r).abs().max()) <= 1e-5 * scale + 1e-7
    # float64 column sums of the bf16 gP (layer-1 bias) and of gG (layer-2 bias), per expert
    ro = row_off.cpu().tolist()
    ref = torch.stack([gP[ro[e]:ro[e + 1]].double().sum(0) for e in range(E)]) + 0.25
    assert float((gb1.double() - ref.to(DEV)).abs().max()) <= 1e-5 * float(ref.abs().max())
    ref2 = torch.stack([gG[ro[e]:ro[e + 1]].double().sum(0) for e in range(E)]) - 0.5
    assert float((gb2.double() - ref2.to(DEV)).abs().max()) <= 1e-5 * float(ref2.abs().max())
    assert float((gb2.view(-1) - gb2_r).abs().max()) <= 1e-5 * float((gb2_r + 0.5).abs().max()) + 1e-7
    # and the gradients against float64 math on the same bf16 operands (sampled rows)
    rows = torch.randperm(n, device=DEV)[:64]
    e_of = torch.bucketize(rows.int(), row_off[1:].contiguous(), right=True)
    gh = torch.einsum("rc,rch->rh", gG[rows].double(), W2[e_of].double())
    p = Pre[rows].double()
    gelu_grad = 0.5 * (1 + torch.erf(p / 2 ** 0.5)) + p * torch.exp(-p * p / 2) / (2 * torch.pi) ** 0.5
    assert (gP[rows].double() - gh * gelu_grad).abs().max() <= 1e-2 * (gh * gelu_grad).abs().max()
    gx = torch.einsum("rh,rhc->rc", gP[rows].double(), W1[e_of].double())
    assert (gX[rows].double() - gx).abs().max() <= 1e-2 * gx.abs().max()


@pytest.mark.parametrize("T,C,E,k", [(16384, 256, 8, 2), (4096, 512, 8, 2), (1000, 128, 8, 2), (77, 256, 4, 1)])
def test_grouped_64x64_subtiles_bit_identical(T, C, E, k):
    """Grouped expert GEMMs on 64x64 tiles over the dispatch's 128-row tile table (two sub-tiles per table tile,
    Grouping.sub_shift; tuning slot 3 = 64, and the automatic choice) equal the 128^2-tile launch bit for bit: the same MFMA k order per
    output element.  Layer 1 with the bias + GELU + saved pre-activation epilogue, layer 2, and the data gradient
    (MC weight operand); skewed / empty experts and ragged last tiles (rows past a group's end in the second
    sub-tile)."""
    tok, W1, b1, W2, b2, topi, gate = _case(T, C, E, k, 7 * T + C, empty_expert=(T == 1000))
    Hd = 4 * C
    row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
    n = T * k
    max_tiles = (n + 127) // 128 + E
    Xg = ops.gather_rows(tok, perm, k)

    def run():
        Pre = torch.empty(n, Hd, device=DEV, dtype=bf)
        Hid = torch.empty(n, Hd, device=DEV, dtype=bf)
        ops.gemm_grouped(Xg, W1.view(-1), row_off, tile_off, max_tiles, Hd, C, b_gstride=Hd * C, out=Hid, ldb=C,
                         ep=ops.E(bias=b1, act=L.ACT_GELU, out_pre=Pre, ld_pre=Hd))
        Y = torch.empty(n, C, device=DEV, dtype=bf)
        ops.gemm_grouped(Hid, W2.view(-1), row_off, tile_off, max_tiles, C, Hd, b_gstride=C * Hd, out=Y, ldb=Hd,
                         ep=ops.E(bias=b2))
        gX = torch.empty(n, C, device=DEV, dtype=bf)
        ops.gemm_grouped(Hid, W1.view(-1), row_off, tile_off, max_tiles, C, Hd, b_kc=False, b_gstride=Hd * C, out=gX,
                         ldb=C)
        torch.cuda.synchronize()
        return Pre, Hid, Y, gX
    L.call("mg_set_tuning", 3, 128)  # 128^2 tiles everywhere
    try:
        ref = run()
        L.call("mg_set_tuning", 3, 64)  # 64^2 sub-tiles everywhere
        got = run()
        L.call("mg_set_tuning", 3, 0)  # the automatic choice (64^2 for K <= 512)
        auto = run()
    finally:
        L.call("mg_set_tuning", 3, 0)
    for a, b in zip(auto, ref):
        assert torch.equal(a, b)
    for a, b in zip(got, ref):
        assert torch.equal(a, b)
