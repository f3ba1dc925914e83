"""Fused per-image MTM backward (mg_mtm_bwd_fused: gather-form grid_sample data gradient + offset head backward)
against the scatter kernels it replaces (mg_warp_bwd with fp32 atomics + mg_offset_head_bwd), which the module
tests pin to the oracle (t2i_moe_gan.py:222-239).  Large offsets make many output pixels clamp onto the same
border source pixels (long per-pixel gather lists)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("B,H,C", [(4, 16, 128), (8, 8, 256), (8, 4, 512), (3, 16, 64), (2, 20, 32)])
@pytest.mark.parametrize("dtype", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("acc", [0, 1])
@pytest.mark.parametrize("off_scale", [0.3, 40.0])
def test_mtm_bwd_fused_vs_scatter(B, H, C, dtype, acc, off_scale):
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + H * 10 + C + acc)
    W = H
    x = torch.randn(B, H, W, C, device=DEV, generator=g).to(dtype)
    o1 = torch.randn(B, H, W, 32, device=DEV, generator=g).to(dtype)
    w2 = torch.randn(2, 32, 3, 3, device=DEV, generator=g) * (off_scale / 32)
    b2 = torch.randn(2, device=DEV, generator=g) * off_scale
    _, samp = ops.warp_fwd(x, o1, w2, b2)
    gout = torch.randn(B, H, W, C, device=DEV, generator=g).to(dtype)
    P = B * H * W
    # reference: scatter kernels
    gx32 = torch.zeros(B, H, W, C, device=DEV)
    goff = torch.empty(P, 2, device=DEV)
    ops.warp_bwd(gout, x, samp, gx32, goff)
    ga1_r = torch.empty(B, H, W, 32, device=DEV, dtype=dtype)
    gw2_r = torch.zeros(2, 32, 3, 3, device=DEV)
    gb2_r = torch.zeros(2, device=DEV)
    ops.offset_head_bwd(goff, o1, w2, ga1_r, gw2_r, gb2_r)
    prior = torch.randn(B, H, W, C, device=DEV, generator=g).to(dtype)
    gx_r = gx32 + (prior.float() if acc else 0.0)
    # fused
    gx = prior.clone() if acc else torch.full_like(prior, float("nan"))
    ga1 = torch.empty_like(ga1_r)
    gw2 = torch.ones(2, 32, 3, 3, device=DEV)  # accumulates
    gb2 = torch.ones(2, device=DEV)
    ops.mtm_bwd_fused(gout, x, samp, o1, w2, gx, ga1, gw2, gb2, accumulate=acc)
    torch.cuda.synchronize()
    tol = 1e-5 if dtype == torch.float32 else 1e-2
    assert torch.isfinite(gx.float()).all()
    assert rel(gx, gx_r) < tol
    assert rel(ga1, ga1_r) < (1e-4 if dtype == torch.float32 else 2e-2)
    assert rel(gw2 - 1.0, gw2_r) < 1e-4
    assert rel(gb2 - 1.0, gb2_r) < 1e-4
