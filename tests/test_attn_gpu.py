"""bf16 MFMA self-attention (mg_attn_mfma.hip) vs a plain PyTorch fp32 reference on the same bf16 inputs."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("L,C", [(16, 512), (64, 256), (256, 128), (64, 512), (16, 256), (64, 128)])
def test_attention_bf16_mfma_vs_fp32(L, C):
    B, heads = 5, 8
    D = C // heads
    g = torch.Generator(device=DEV).manual_seed(L + C)
    qkv = (torch.randn(B * L, 3 * C, device=DEV, generator=g) * 1.5).bfloat16()
    gout = torch.randn(B * L, C, device=DEV, generator=g).bfloat16()
    out, lse = ops.attn_fwd(qkv, B, L, C)
    g_qkv = ops.attn_bwd(qkv, out, gout, lse, B, L, C)
    torch.cuda.synchronize()
    x = qkv.float().view(B, L, 3, heads, D).permute(2, 0, 3, 1, 4).detach().requires_grad_(True)  # [3,B,h,L,D]
    q, k, v = x[0], x[1], x[2]
    s = q @ k.transpose(-1, -2) / D ** 0.5
    o = torch.softmax(s, -1) @ v
    ref = o.permute(0, 2, 1, 3).reshape(B * L, C)
    assert rel(out, ref) < 2e-2
    ref_lse = torch.logsumexp(s, -1)  # [B, h, L]
    assert (lse.view(B, heads, L) - ref_lse).abs().max().item() < 2e-2
    ref.backward(gout.float())
    gref = x.grad.permute(1, 3, 0, 2, 4).reshape(B * L, 3 * C)
    for part in range(3):
        sl = slice(part * C, (part + 1) * C)
        assert rel(g_qkv[:, sl], gref[:, sl]) < 3e-2, part


@pytest.mark.parametrize("L", [50, 33, 63])
def test_attention_ragged_tokens_forward(L):
    """Forward-only ragged sequence (the CLIP ViT-B/32 image tower: 50 tokens, 12 heads of 64) on the 64-token MFMA
    tiles: rows past L masked on load and store; the image after the last one is never touched."""
    B, heads, C = 7, 12, 768
    D = C // heads
    g = torch.Generator(device=DEV).manual_seed(L)
    qkv = (torch.randn(B * L, 3 * C, device=DEV, generator=g) * 1.5).bfloat16()
    out = torch.full((B * L + 16, C), 7.0, device=DEV).bfloat16()  # guard rows after the last image
    lse = torch.full((B * heads * L + 16,), 7.0, device=DEV)
    ops.call("mg_attn_fwd", ops.dt(qkv), ops.ptr(qkv), B, L, C, heads, ops.ptr(out), ops.ptr(lse), ops.S())
    torch.cuda.synchronize()
    x = qkv.float().view(B, L, 3, heads, D).permute(2, 0, 3, 1, 4)
    q, k, v = x[0], x[1], x[2]
    s = q @ k.transpose(-1, -2) / D ** 0.5
    ref = (torch.softmax(s, -1) @ v).permute(0, 2, 1, 3).reshape(B * L, C)
    assert rel(out[:B * L], ref) < 2e-2
    assert (lse[:B * heads * L].view(B, heads, L) - torch.logsumexp(s, -1)).abs().max().item() < 2e-2
    assert bool((out[B * L:].float() == 7.0).all()) and bool((lse[B * heads * L:] == 7.0).all())


@pytest.mark.parametrize("R,C", [(65536, 128), (16384, 256), (4096, 512), (1000, 128), (7, 512)])
@pytest.mark.parametrize("accumulate", [0, 1])
def test_layernorm_bwd_vs_autograd(R, C, accumulate):
    """LayerNorm backward (AttentionBlock.norm1 / norm2, t2i_moe_gan.py:545-560) at the step's row counts and ragged
    ones: input gradient (optionally accumulated) and the gamma / beta gradients (per-block partial rows + the
    fixed-order rows fold) against fp32 autograd on the same bf16 operands; two calls give the same bits."""
    g = torch.Generator(device=DEV).manual_seed(R + C)
    x = (torch.randn(R, C, device=DEV, generator=g) * 2 + 0.5).bfloat16()
    gy = torch.randn(R, C, device=DEV, generator=g).bfloat16()
    gamma = torch.rand(C, device=DEV, generator=g) + 0.5
    beta = torch.randn(C, device=DEV, generator=g)
    base = torch.randn(R, C, device=DEV, generator=g).bfloat16()
    _, mean, rstd = ops.layernorm_fwd(x, gamma, beta)
    xr = x.float().requires_grad_(True)
    gr, br = gamma.clone().requires_grad_(True), beta.clone().requires_grad_(True)
    torch.nn.functional.layer_norm(xr, (C,), gr, br, 1e-5).backward(gy.float())

    def run():
        gx = base.clone()
        gg = torch.full((C,), 0.25, device=DEV)
        gb = torch.full((C,), -0.5, device=DEV)
        ops.layernorm_bwd(gy, x, mean, rstd, gamma, gx, gg, gb, accumulate=accumulate)
        return gx, gg, gb
    gx, gg, gb = run()
    gx2, gg2, gb2 = run()
    torch.cuda.synchronize()
    want_gx = xr.grad + (base.float() if accumulate else 0)
    assert float((gx.float() - want_gx).abs().max()) <= 2e-2 * float(want_gx.abs().max()) + 1e-2
    assert torch.allclose(gg, gr.grad + 0.25, rtol=1e-4, atol=1e-3 * (R / 1000) ** 0.5)
    assert torch.allclose(gb, br.grad - 0.5, rtol=1e-4, atol=1e-3 * (R / 1000) ** 0.5)
    assert torch.equal(gx, gx2) and torch.equal(gg, gg2) and torch.equal(gb, gb2)
