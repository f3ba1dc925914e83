"""Router / MoE token kernels across expert counts (E = 4, 8, 16, 32; the C5 config uses 32 top-4) and the
fused MTM warp + modulation prescale, against plain PyTorch fp32 on the GPU.

The router math follows the oracle (oracle/aurora_cpu.py `router` / `topk_route`, t2i_moe_gan.py:364-402);
top-k indices must match exactly (inputs are drawn so that no two probabilities of a token tie).
"""
import pytest
import torch

pytestmark = pytest.mark.gpu

from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


def ref_router(tok, Wfc, Lt, HW, temp, anneal, k):
    T = tok.shape[0]
    b = torch.arange(T, device=tok.device) // HW
    z = (tok.double() @ Wfc.double() + Lt.double()[b]) / min(max(temp * anneal, 0.5), 5.0)
    p = torch.softmax(z.clamp(-20.0, 20.0), dim=1).clamp(1e-6, 1.0)
    p = p / p.sum(dim=1, keepdim=True)
    top = torch.topk(p, k, dim=1, sorted=True)
    gate = top.values if k == p.shape[1] else top.values / top.values.sum(dim=1, keepdim=True)
    return p, z, top.indices, gate


@pytest.mark.parametrize("E,k", [(4, 2), (8, 2), (16, 2), (32, 4), (8, 8)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
def test_router_fwd_across_experts(E, k, dtype):
    g = torch.Generator(device=DEV).manual_seed(E * 7 + k)
    B, HW, C = 8, 64, 128
    T = B * HW
    tok = torch.randn(T, C, device=DEV, generator=g).to(dtype)
    Wfc = torch.randn(C, E, device=DEV, generator=g) * 0.2
    Lt = torch.randn(B, E, device=DEV, generator=g)
    temp = torch.tensor([1.3], device=DEV)
    probs, zlog, topi, gate = ops.router_fwd(tok, Wfc, Lt, E, k, HW, temp, 1.0)
    p, z, ti, gt = ref_router(tok.float(), Wfc, Lt, HW, 1.3, 1.0, k)
    assert rel(zlog, z) < 1e-5
    assert rel(probs, p) < 1e-5
    # exact indices wherever the k-th and (k+1)-th probabilities are not within rounding of each other
    srt = torch.sort(p, dim=1, descending=True).values
    clear = (srt[:, k - 1] - srt[:, k]).abs() > 1e-6 if k < E else torch.ones(T, dtype=torch.bool, device=DEV)
    order = torch.sort(topi.long(), dim=1).values
    assert torch.equal(order[clear], torch.sort(ti, dim=1).values[clear])
    assert clear.float().mean() > 0.95
    assert rel(torch.sort(gate, dim=1).values[clear], torch.sort(gt, dim=1).values.float()[clear]) < 1e-5


@pytest.mark.parametrize("T,C,E,k,HW", [(4096 - 5, 512, 32, 4, 16), (65536 + 3, 128, 32, 4, 256),
                                        (1000, 256, 8, 2, 8), (70000, 128, 16, 2, 1024), (48, 192, 8, 8, 16)])
def test_router_fwd_mfma_shapes(T, C, E, k, HW):
    """bf16 router logits on the matrix cores (Wfc as bf16 hi + lo): several channel chunks (C = 512), ragged
    token counts, several tiles per wave (T > 65536), C not a multiple of the chunk; against fp64 and against the
    lane-FMA team kernel (tuning slot 24 = 1)."""
    from moegan_mi import _lib as L
    g = torch.Generator(device=DEV).manual_seed(T + C + E)
    B = (T + HW - 1) // HW
    tok = torch.randn(T, C, device=DEV, generator=g).to(torch.bfloat16)
    Wfc = torch.randn(C, E, device=DEV, generator=g) * (2.0 / C ** 0.5)
    Lt = torch.randn(B, E, device=DEV, generator=g)
    temp = torch.tensor([1.1], device=DEV)
    probs, zlog, topi, gate = ops.router_fwd(tok, Wfc, Lt, E, k, HW, temp, 1.0)
    L.call("mg_set_tuning", 24, 1)
    try:
        probs_t, zlog_t, topi_t, gate_t = ops.router_fwd(tok, Wfc, Lt, E, k, HW, temp, 1.0)
    finally:
        L.call("mg_set_tuning", 24, 0)
    p, z, ti, gt = ref_router(tok.float(), Wfc, Lt, HW, 1.1, 1.0, k)
    assert rel(zlog, z) < 1e-5 and rel(zlog, zlog_t) < 1e-5
    assert rel(probs, p) < 1e-5
    srt = torch.sort(p, dim=1, descending=True).values
    clear = (srt[:, k - 1] - srt[:, k]).abs() > 1e-6 if k < E else torch.ones(T, dtype=torch.bool, device=DEV)
    order = torch.sort(topi.long(), dim=1).values
    assert torch.equal(order[clear], torch.sort(ti, dim=1).values[clear])
    assert torch.equal(order[clear], torch.sort(topi_t.long(), dim=1).values[clear])
    assert clear.float().mean() > 0.95
    assert rel(torch.sort(gate, dim=1).values[clear], torch.sort(gt, dim=1).values.float()[clear]) < 1e-5


@pytest.mark.parametrize("E,k,HW,B", [(32, 4, 16, 64), (32, 4, 256, 9), (8, 2, 64, 17), (16, 16, 1, 300),
                                      (8, 2, 4, 33), (4, 2, 16, 8)])
def test_router_bwd_against_autograd(E, k, HW, B):
    """mg_router_bwd (8-lane teams for E >= 8, thread per token for E = 4) against fp64 autograd of the router's
    softmax / clamp / renormalise / top-k gate (t2i_moe_gan.py:375-402): the raw-logit gradient, the per-image
    sums and the temperature gradient; and against the thread-per-token kernel (tuning slot 24 = 2)."""
    from moegan_mi import _lib as L
    g = torch.Generator(device=DEV).manual_seed(E * 1000 + HW + B)
    T, C = B * HW, 128
    tok = torch.randn(T, C, device=DEV, generator=g).to(torch.bfloat16)
    Wfc = torch.randn(C, E, device=DEV, generator=g) * 0.3
    Lt = torch.randn(B, E, device=DEV, generator=g)
    temp = torch.tensor([1.3], device=DEV)
    probs, zlog, topi, gate = ops.router_fwd(tok, Wfc, Lt, E, k, HW, temp, 0.9)
    g_gate = torch.randn(T, k, device=DEV, generator=g)
    g_probs = torch.randn(T, E, device=DEV, generator=g)
    g_logits = torch.randn(T, E, device=DEV, generator=g) * 0.1
    coef = torch.randn(E, device=DEV, generator=g)

    def run():
        gt = torch.zeros(1, device=DEV)
        g_raw, gsum = ops.router_bwd(probs, zlog, topi, gate, g_gate, g_probs, coef, HW, temp, 0.9, gt, B,
                                     g_logits=g_logits)
        ops.fold_flush()
        torch.cuda.synchronize()
        return g_raw, gsum, gt

    g_raw, gsum, gt = run()
    L.call("mg_set_tuning", 24, 2)
    try:
        g_raw2, gsum2, gt2 = run()
    finally:
        L.call("mg_set_tuning", 24, 0)
    te = min(max(1.3 * 0.9, 0.5), 5.0)
    raw = (zlog.double() * te).requires_grad_(True)
    tp = torch.tensor([1.3], dtype=torch.float64, device=DEV, requires_grad=True)
    z = raw / (tp * 0.9).clamp(0.5, 5.0)
    lz = z.clamp(-20.0, 20.0)
    q = torch.softmax(lz, dim=1).clamp(1e-6, 1.0)
    p = q / q.sum(dim=1, keepdim=True)
    pk = p.gather(1, topi.long())
    gk = pk if k == E else pk / pk.sum(dim=1, keepdim=True)
    loss = (p * (coef.double() + g_probs.double())).sum() + (gk * g_gate.double()).sum() + \
        (lz * g_logits.double()).sum()
    ref_raw, ref_t = torch.autograd.grad(loss, (raw, tp))
    assert rel(g_raw, ref_raw) < 1e-5
    assert rel(gsum, ref_raw.view(B, HW, E).sum(1)) < 1e-5
    assert abs(gt.item() - ref_t.item()) <= 1e-5 * max(1.0, abs(ref_t.item()))
    assert rel(g_raw, g_raw2) < 1e-6 and rel(gsum, gsum2) < 1e-5
    again = run()
    assert all(torch.equal(a, b) for a, b in zip((g_raw, gsum, gt), again))  # fixed reduction order


@pytest.mark.parametrize("E", [4, 8, 16, 32])
def test_token_and_feature_grad_across_experts(E):
    g = torch.Generator(device=DEV).manual_seed(100 + E)
    T, C, k = 2048, 128, 2
    gX = torch.randn(T * k, C, device=DEV, generator=g).to(torch.bfloat16)
    pos_of = torch.randperm(T * k, device=DEV, generator=g).to(torch.int32)
    g_raw = torch.randn(T, E, device=DEV, generator=g)
    Wfc = torch.randn(C, E, device=DEV, generator=g)
    out = torch.empty(T, C, device=DEV)
    ops.moe_token_grad(gX, pos_of, g_raw, Wfc, out, k)
    ref = gX.float()[pos_of.long().view(T, k)].sum(1) + g_raw @ Wfc.T
    assert rel(out, ref) < 1e-5
    tok = torch.randn(T, C, device=DEV, generator=g).to(torch.bfloat16)
    G1 = torch.zeros(C, E, device=DEV)
    ops.router_feat_grad(tok, g_raw, G1)
    assert rel(G1, tok.float().T @ g_raw) < 1e-5


@pytest.mark.parametrize("T,C,E,k,out_dtype", [(4096 - 3, 512, 32, 4, torch.float32), (16384, 256, 32, 4, torch.bfloat16),
                                               (65536 + 5, 128, 32, 4, torch.float32), (1000, 128, 8, 2, torch.float32),
                                               (3000, 256, 16, 2, torch.bfloat16)])
def test_token_grad_mfma_shapes(T, C, E, k, out_dtype):
    """Token gradient with the router term on the matrix cores (both fp32 operands as bf16 hi + lo): one and
    several tiles per block, ragged token counts, E = 8 / 16 (zero k-rows); against fp64 and against the lane-FMA
    kernel (tuning slot 24 = 4)."""
    from moegan_mi import _lib as L
    g = torch.Generator(device=DEV).manual_seed(T + C * 3 + E)
    gX = torch.randn(T * k, C, device=DEV, generator=g).to(torch.bfloat16)
    pos_of = torch.randperm(T * k, device=DEV, generator=g).to(torch.int32)
    g_raw = torch.randn(T, E, device=DEV, generator=g)
    Wfc = torch.randn(C, E, device=DEV, generator=g) * 0.5
    out = ops.moe_token_grad(gX, pos_of, g_raw, Wfc, torch.empty(T, C, device=DEV, dtype=out_dtype), k)
    L.call("mg_set_tuning", 24, 4)
    try:
        out_l = ops.moe_token_grad(gX, pos_of, g_raw, Wfc, torch.empty(T, C, device=DEV, dtype=out_dtype), k)
    finally:
        L.call("mg_set_tuning", 24, 0)
    ref = gX.double()[pos_of.long().view(T, k)].sum(1) + g_raw.double() @ Wfc.double().T
    tol = 1e-5 if out_dtype == torch.float32 else 8e-3
    assert rel(out, ref) < tol and rel(out_l, ref) < tol
    if out_dtype == torch.float32:
        assert rel(out, out_l) < 1e-5


@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("H,C", [(16, 128), (8, 256), (4, 512)])
def test_warp_fwd_scaled_matches_warp_then_scale(dtype, H, C):
    """mg_warp_fwd_scaled == mg_warp_fwd followed by mg_scale_bc, bit for bit (same rounding order)."""
    g = torch.Generator(device=DEV).manual_seed(H + C)
    B = 4
    x = torch.randn(B, H, H, C, device=DEV, generator=g).to(dtype)
    o1 = torch.randn(B, H, H, 32, device=DEV, generator=g).to(dtype)
    w2 = torch.randn(2, 32, 3, 3, device=DEV, generator=g) * 0.5
    b2 = torch.randn(2, device=DEV, generator=g)
    S = torch.randn(B, 3 * C, device=DEV, generator=g)
    s = S[:, C:2 * C]  # a column slice of a batched style matrix (row stride 3C)
    out, samp = ops.warp_fwd(x, o1, w2, b2)
    xs_ref = ops.scale_bc(out, s)
    out2, samp2, xs = ops.warp_fwd(x, o1, w2, b2, s=s)
    assert torch.equal(out, out2) and torch.equal(samp, samp2)
    assert torch.equal(xs, xs_ref)


def test_router_kl_batch_bit_identical():
    """mg_router_kl_batch (every router's KL terms in two launches) == mg_router_kl per router, bit for bit, for
    routers of different sizes (each record keeps the single-router partial split), and > 8 routers (chunked)."""
    g = torch.Generator(device=DEV).manual_seed(11)
    routers = []
    for C, E in ((512, 8), (256, 8), (128, 32), (64, 4), (512, 16), (128, 8), (256, 32), (128, 16), (64, 8)):
        shapes = ((C, 128), (C, 128), (512, 128), (512, 128), (256, E), (256, E))
        # mu ~ 0, rho ~ softplus^-1(1): sigma ~ 1, so the sums stay below the 120 clamp (KL ~ 1e-4 per element)
        routers.append(tuple(torch.randn(*sh, device=DEV, generator=g) * 0.01 + (0.5413 if i % 2 else 0.0)
                             for i, sh in enumerate(shapes)))
    out = torch.empty(len(routers), 2, device=DEV)
    ops.router_kl_batch(routers, out)
    for j, r in enumerate(routers):
        one = torch.empty(2, device=DEV)
        ops.router_kl(*r, one)
        assert torch.equal(out[j], one), (j, out[j], one)
        assert one[1].item() == 1.0 and 0.0 < one[0].item() < 120.0  # a real (unclamped) sum
