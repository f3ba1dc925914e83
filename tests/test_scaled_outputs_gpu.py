"""Fused modulated-conv inputs: the MoE combine and the bilinear upsample also write the next modulated conv's input
x * s (t2i_moe_gan.py:158-161; AttentionBlock.proj_out :574 reads the combine, ConvolutionBlock.skip_proj :615-616
reads the upsampled block input).  Both outputs must equal, bit for bit, the unfused pair (the plain kernel, then
mg_scale_bc on its stored output), in bf16 and fp32, with the style rows a strided column slice of the step's
batched style matrix as the engine passes them."""
import pytest
import torch

from moegan_mi import ops

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _styles(B, C, g):
    S = torch.randn(B, 3 * C + 8, device=DEV, generator=g)  # a wider batched-style matrix; the conv's slice
    return S[:, C + 8:2 * C + 8]


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,HW,C,E,k", [(4, 16, 512, 8, 2), (3, 64, 256, 32, 4), (2, 256, 128, 8, 2)])
def test_combine_scaled_equals_combine_then_scale(dtype, B, HW, C, E, k):
    g = torch.Generator(device=DEV).manual_seed(B * HW + C)
    T = B * HW
    n = T * k
    Y = torch.randn(n, C, device=DEV, generator=g).to(dtype)
    pos_of = torch.randperm(n, device=DEV, generator=g).int()
    gate = torch.rand(T, k, device=DEV, generator=g)
    resid = torch.randn(T, C, device=DEV, generator=g).to(dtype)
    s = _styles(B, C, g)
    ref = torch.empty(T, C, device=DEV, dtype=dtype)
    ops.moe_combine(Y, pos_of, gate, resid, ref)
    xs_ref = torch.empty_like(ref)
    ops.call("mg_scale_bc", ops.dt(ref), ops.ptr(ref), C, ops.ptr(s), s.stride(0), B, HW, C, ops.ptr(xs_ref), C,
             ops.S())
    out = torch.empty_like(ref)
    out2, xs = ops.moe_combine(Y, pos_of, gate, resid, out, style=s, HW=HW)
    torch.cuda.synchronize()
    assert out2 is out
    assert torch.equal(out, ref)
    assert torch.equal(xs, xs_ref)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,C", [(4, 4, 512), (3, 8, 256)])
def test_upsample_scaled_equals_upsample_then_scale(dtype, B, H, C):
    g = torch.Generator(device=DEV).manual_seed(B * H * C)
    x = torch.randn(B, H, H, C, device=DEV, generator=g).to(dtype)
    s = _styles(B, C, g)
    ref = ops.upsample2x(x)
    HW = 4 * H * H
    xs_ref = torch.empty_like(ref)
    ops.call("mg_scale_bc", ops.dt(ref), ops.ptr(ref), C, ops.ptr(s), s.stride(0), B, HW, C, ops.ptr(xs_ref), C,
             ops.S())
    out, xs = ops.upsample2x(x, style=s)
    torch.cuda.synchronize()
    assert torch.equal(out, ref)
    assert torch.equal(xs, xs_ref)
