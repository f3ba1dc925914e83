"""The 32-channel 3x3 convolutions of the MTM offset heads (offset_net.0: Cin -> 32 + LeakyReLU,
t2i_moe_gan.py:199-216, and its backward) on the direct halo-tile kernels of csrc/mg_narrow.hip, routed from
mg_conv2d_fwd / mg_conv2d_wgrad for 4x4 .. 16x16 maps, against

  * the implicit-GEMM path they replace (tuning slot 16 = 1): the same products summed in another order (channel
    chunks outermost, split slabs on the small maps), so fp32 results agree to summation noise and bf16 results to
    one rounding;
  * plain fp32 / fp64 PyTorch convolutions on the same bf16 operands.

Cases: the three map sizes the offset heads run at, Cin 128 / 256 / 512, a batch that leaves the last 128-pixel
tile ragged (odd B on the multi-image tiles), the bias + LeakyReLU forward epilogue, the data gradient accumulated
into fp32 and bf16 buffers, and the weight gradient accumulated into the reference [32][Cin][3][3] layout
(deterministic: two calls give the same bits)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"
bf = torch.bfloat16


def _set(v):
    from moegan_mi import _lib as L
    L.call("mg_set_tuning", 16, v)


@pytest.mark.parametrize("wpx", [0, 4])
@pytest.mark.parametrize("B,S,Cin,out_dtype", [(8, 16, 256, bf), (3, 16, 128, torch.float32), (6, 8, 512, bf),
                                               (5, 8, 256, bf), (9, 4, 512, bf), (2, 4, 128, torch.float32)])
def test_offset_head_forward(B, S, Cin, out_dtype, wpx):
    """``wpx``: tuning slot 19 (0: 128-pixel tiles, 4: 256-pixel tiles with four pixel fragments per wave)."""
    from moegan_mi import _lib as L
    from moegan_mi import ops
    L.call("mg_set_tuning", 19, wpx)
    g = torch.Generator(device=DEV).manual_seed(B * 100 + S + Cin)
    x = (torch.randn(B, S, S, Cin, device=DEV, generator=g)).to(bf)
    W = (torch.randn(32, Cin, 3, 3, device=DEV, generator=g) * (9 * Cin) ** -0.5)
    bias = torch.randn(32, device=DEV, generator=g) * 0.1
    wp = ops.pack_conv(W, bf)
    ep = ops.E(bias=bias, act=L.ACT_LRELU)
    y = ops.conv2d(x, wp, 32, 3, 3, 1, 1, out_dtype=out_dtype, ep=ep)
    _set(1)
    try:
        y_ref = ops.conv2d(x, wp, 32, 3, 3, 1, 1, out_dtype=out_dtype, ep=ep)
    finally:
        _set(0)
    torch.cuda.synchronize()
    t = F.leaky_relu(F.conv2d(x.float().permute(0, 3, 1, 2), W.to(bf).float(), bias, padding=1), 0.2)
    t = t.permute(0, 2, 3, 1)
    scale = float(t.abs().max())
    tol = 2e-5 if out_dtype == torch.float32 else 1e-2
    assert float((y.float() - y_ref.float()).abs().max()) <= tol * scale
    assert float((y.float() - t).abs().max()) <= tol * scale
    y2 = ops.conv2d(x, wp, 32, 3, 3, 1, 1, out_dtype=out_dtype, ep=ep)
    torch.cuda.synchronize()
    L.call("mg_set_tuning", 19, 0)
    assert torch.equal(y, y2)


@pytest.mark.parametrize("B,S,Cout,out_dtype", [(8, 16, 256, bf), (4, 16, 128, torch.float32), (2, 16, 128, bf),
                                                (6, 8, 512, bf), (5, 8, 256, torch.float32), (9, 4, 512, bf)])
def test_offset_head_data_gradient(B, S, Cout, out_dtype):
    """gx += conv(g, flipped W): the 32 -> Cin direction (mtm_bwd, engine_g.py), accumulated into gx.  (16x16 into
    >= 256 channels stays on the implicit GEMM: both sides of the first comparison are then that path.)"""
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(B * 7 + S + Cout)
    ga = torch.randn(B, S, S, 32, device=DEV, generator=g).to(bf)
    W = torch.randn(32, Cout, 3, 3, device=DEV, generator=g) * (9 * 32) ** -0.5  # the head's weight [32][Cin][3][3]
    wflip = ops.pack_conv(W, bf, flip=True)
    gx0 = (torch.randn(B, S, S, Cout, device=DEV, generator=g) * 0.5).to(out_dtype)
    gx = gx0.clone()
    ops.conv2d(ga, wflip, Cout, 3, 3, 1, 1, out=gx, ep=ops.E(accumulate=1))
    gx_ref = gx0.clone()
    _set(1)
    try:
        ops.conv2d(ga, wflip, Cout, 3, 3, 1, 1, out=gx_ref, ep=ops.E(accumulate=1))
    finally:
        _set(0)
    torch.cuda.synchronize()
    # fp64 autograd of the forward conv on the same bf16 operands
    xx = torch.zeros(B, Cout, S, S, dtype=torch.float64, device=DEV, requires_grad=True)
    (F.conv2d(xx, W.to(bf).double(), padding=1) * ga.permute(0, 3, 1, 2).double()).sum().backward()
    t = gx0.double() + xx.grad.permute(0, 2, 3, 1)
    scale = float(t.abs().max())
    tol = 1e-5 if out_dtype == torch.float32 else 1e-2
    assert float((gx.double() - gx_ref.double()).abs().max()) <= tol * scale
    assert float((gx.double() - t).abs().max()) <= tol * scale


@pytest.mark.parametrize("B,S,Cin", [(8, 16, 256), (4, 16, 128), (6, 8, 512), (5, 8, 256), (9, 4, 512), (3, 4, 64)])
def test_offset_head_weight_gradient(B, S, Cin):
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(B * 13 + S + Cin)
    x = torch.randn(B, S, S, Cin, device=DEV, generator=g).to(bf)
    ga = torch.randn(B, S, S, 32, device=DEV, generator=g).to(bf)

    def run():
        gw = torch.full((32, Cin, 3, 3), 0.25, device=DEV)
        ops.conv2d_wgrad(ga, x, 32, 3, 3, 1, 1, gw)
        return gw
    gw1, gw2 = run(), run()
    _set(1)
    try:
        gw_ref = run()
    finally:
        _set(0)
    torch.cuda.synchronize()
    w = torch.zeros(32, Cin, 3, 3, dtype=torch.float64, device=DEV, requires_grad=True)
    (F.conv2d(x.permute(0, 3, 1, 2).double(), w, padding=1) * ga.permute(0, 3, 1, 2).double()).sum().backward()
    t = w.grad + 0.25
    scale = float(w.grad.abs().max())
    assert float((gw1.double() - t).abs().max()) <= 1e-5 * scale
    assert float((gw1 - gw_ref).abs().max()) <= 2e-5 * scale
    assert torch.equal(gw1, gw2)
