"""The discriminator's first conv (conv_layers.0: 3 -> 128, 4x4 / s2 / p1, t2i_moe_gan.py:874-880) on the direct
MFMA kernels of the bf16 step (csrc/mg_dfirst.hip: mg_d0_fwd / mg_d0_wgrad / mg_d0_dgrad), against

  * the im2col + GEMM path they replace in the bf16 step (mg_im2col_4x4s2 + mg_gemm, the dgrad GEMM +
    mg_col2im_4x4s2): the same MFMA products in the same k order and the same fp32 epilogue, so the forward, the R1
    forward-mode pass and the image gradient are held bit-identical; the weight gradient sums the pixels in another
    order (per-block partials), so it is held to fp32 summation noise;
  * a plain PyTorch fp32 restatement of the same op on the same bf16 operands (F.conv2d / its autograd gradients).

Shapes: the C2 real batch (64x64 -> 32x32 maps), the 16x16 fakes (8x8 maps, several images per 128-pixel tile),
the C4 stage's 128x128 images (64-wide maps: the 4-row dgrad band), a ragged last tile (pixels not a multiple of
128), fp32 NCHW images (real batches) and the channel-padded bf16 NHWC layouts (R1's u, ld 4; the generator's
images, ld 8)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _img(B, H, layout, g):
    x = torch.rand(B, 3, H, H, device=DEV, generator=g) * 2 - 1
    if layout == "nchw":
        return x, (3 * H * H, H, 1, H * H), x
    ld = layout
    t = torch.zeros(B, H, H, ld, device=DEV, dtype=torch.bfloat16)
    t[..., :3] = x.permute(0, 2, 3, 1).bfloat16()
    return t, (H * H * ld, H * ld, ld, 1), t[..., :3].permute(0, 3, 1, 2).float()


def _w0(g):
    """Packed bf16 weight [128, 48] (k = tap*3 + c) and the same weight as an OIHW fp32 tensor."""
    w = (torch.randn(128, 3, 4, 4, device=DEV, generator=g) * 0.2).bfloat16().float()
    return w.permute(0, 2, 3, 1).reshape(128, 48).contiguous().bfloat16(), w


CASES = [(4, 64, "nchw"), (2, 64, 4), (3, 16, 8), (1, 16, "nchw"), (2, 128, "nchw"), (5, 8, 4)]


@pytest.mark.parametrize("store", [0, 2])
@pytest.mark.parametrize("B,H,layout", CASES)
def test_d0_forward_and_r1_pass(B, H, layout, store):
    """``store``: the output path (tuning slot MG_TUNE_D0_STORE: 0 automatic, 2 LDS-staged rows)."""
    from moegan_mi import _lib as L
    from moegan_mi import ops
    L.call("mg_set_tuning", 13, store)
    g = torch.Generator(device=DEV).manual_seed(B * 1000 + H)
    x, strides, xr = _img(B, H, layout, g)
    w0p, w = _w0(g)
    bias = torch.randn(128, device=DEV, generator=g) * 0.1
    h0 = ops.d0_fwd(x, strides, B, H, H, w0p, bias=bias)
    cols = ops.im2col_4x4s2(x, strides, B, H, H, 3, 48, torch.bfloat16)
    h0_ref = ops.linear(cols, w0p, bias=bias, act=L.ACT_LRELU).view(B, H // 2, H // 2, 128)
    torch.cuda.synchronize()
    assert torch.equal(h0, h0_ref), float((h0.float() - h0_ref.float()).abs().max())
    # plain fp32 torch on the same bf16 operands
    t = F.leaky_relu(F.conv2d(xr.bfloat16().float(), w, bias, stride=2, padding=1), 0.2).permute(0, 2, 3, 1)
    assert float((h0.float() - t).abs().max()) <= 1e-2 * float(t.abs().max())
    # R1 forward-mode pass: conv(u) * LeakyReLU'(h0), no bias
    m = ops.d0_fwd(x, strides, B, H, H, w0p, aux=h0)
    m_ref = torch.empty_like(m)
    ops.gemm(cols, w0p, cols.shape[0], 128, 48, out=m_ref.view(-1, 128),
             ep=ops.E(act=L.ACT_MUL_LRELU_GRAD, aux=h0, ld_aux=128))
    torch.cuda.synchronize()
    L.call("mg_set_tuning", 13, 0)
    assert torch.equal(m, m_ref), float((m.float() - m_ref.float()).abs().max())


@pytest.mark.parametrize("B,H,layout", CASES)
def test_d0_weight_gradient(B, H, layout):
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(B * 7 + H)
    x, strides, xr = _img(B, H, layout, g)
    gy = torch.randn(B, H // 2, H // 2, 128, device=DEV, generator=g).bfloat16()
    dw = torch.full((128, 48), 0.5, device=DEV)  # accumulates
    ops.d0_wgrad(x, strides, B, H, H, gy, dw)
    cols = ops.im2col_4x4s2(x, strides, B, H, H, 3, 48, torch.bfloat16)
    dw_ref = torch.full((128, 48), 0.5, device=DEV)
    ops.gemm(gy.view(-1, 128), cols, 128, 48, gy.numel() // 128, a_kc=False, b_kc=False, out=dw_ref,
             ep=ops.E(atomic=1), splits=0)
    torch.cuda.synchronize()
    scale = float((dw_ref - 0.5).abs().max())
    assert float((dw - dw_ref).abs().max()) <= 2e-5 * scale
    # fp64 restatement on the bf16 operands: dW[o][tap*3+c] = sum_p gy[p, o] * patch[p, tap*3+c]
    xb = xr.bfloat16().double()
    w = torch.zeros(128, 3, 4, 4, dtype=torch.float64, device=DEV, requires_grad=True)
    y = F.conv2d(xb, w, stride=2, padding=1)
    (y * gy.permute(0, 3, 1, 2).double()).sum().backward()
    ref = w.grad.permute(0, 2, 3, 1).reshape(128, 48)
    assert float((dw.double() - 0.5 - ref).abs().max()) <= 1e-5 * float(ref.abs().max())
    # deterministic: the same call twice gives the same bits
    dw2 = torch.full((128, 48), 0.5, device=DEV)
    ops.d0_wgrad(x, strides, B, H, H, gy, dw2)
    torch.cuda.synchronize()
    assert torch.equal(dw, dw2)


@pytest.mark.parametrize("B,H,out_dtype,ldo", [(4, 64, torch.float32, 4), (3, 16, torch.bfloat16, 8),
                                               (2, 128, torch.float32, 4), (1, 32, torch.float32, 4),
                                               (2, 16, torch.float32, 6)])
def test_d0_image_gradient(B, H, out_dtype, ldo):
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(B * 31 + H)
    w0p, w = _w0(g)
    gy = torch.randn(B, H // 2, H // 2, 128, device=DEV, generator=g).bfloat16()
    out = torch.full((B, H, H, ldo), 7.0, device=DEV, dtype=out_dtype)
    ops.d0_dgrad(gy, w0p, out)
    ref = torch.full((B, H, H, ldo), 7.0, device=DEV, dtype=out_dtype)
    ops.dgrad_s2_small(gy, w0p, 3, ref)
    torch.cuda.synchronize()
    assert torch.equal(out[..., :3], ref[..., :3]), float((out[..., :3].float() - ref[..., :3].float()).abs().max())
    # a one-vector pixel pitch (4 fp32 / 8 bf16) is written whole, padding channels 0; other pitches keep them
    pad = 0.0 if ldo * out.element_size() == 16 else 7.0
    assert bool((out[..., 3:] == pad).all())
    # fp64 autograd of the conv on the same bf16 operands
    xx = torch.zeros(B, 3, H, H, dtype=torch.float64, device=DEV, requires_grad=True)
    (F.conv2d(xx, w.double(), stride=2, padding=1) * gy.permute(0, 3, 1, 2).double()).sum().backward()
    t = xx.grad.permute(0, 2, 3, 1)
    tol = 1e-5 if out_dtype == torch.float32 else 8e-3
    assert float((out[..., :3].double() - t).abs().max()) <= tol * float(t.abs().max())


@pytest.mark.parametrize("B,Hf,bcast", [(4, 16, False), (3, 4, False), (2, 32, False), (5, 8, False), (3, 16, True)])
def test_d_head_kernels(B, Hf, bcast):
    """The discriminator head's image part (output_layer.0, t2i_moe_gan.py:901-907) on the one-block-per-image
    kernels (mg_d_head_fwd / mg_d_head_bwd) against the GEMM path they replace in the bf16 step: P = h1 W2 +
    mg_disc_head_sum (forward; fp32 summation order) and mg_disc_head_gmat + GEMM with the LeakyReLU' epilogue
    (backward; bit-identical);
    ``bcast``: one gradient map for every image (the R1 pass)."""
    from moegan_mi import _lib as L
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(B * 100 + Hf)
    h1 = torch.randn(B, Hf, Hf, 256, device=DEV, generator=g).bfloat16()
    W2img = torch.randn(256, 16, device=DEV, generator=g) * 0.05
    w2c, w2t = W2img.bfloat16().contiguous(), W2img.t().contiguous().bfloat16()
    Ho = Hf - 3
    out = ops.d_head_fwd(h1, w2t, B, Hf)
    P = ops.gemm(h1.view(-1, 256), w2t, B * Hf * Hf, 16, 256, out_dtype=torch.float32)
    ref = ops.disc_head_sum(P, B, Hf)
    gl = torch.randn(1 if bcast else B, Ho * Ho, device=DEV, generator=g)
    gs = 0 if bcast else Ho * Ho
    ga1 = torch.empty_like(h1)
    ops.d_head_bwd(gl, gs, h1, w2c, B, Hf, ga1)
    G = ops.disc_head_gmat(gl, gs, B, Hf, torch.bfloat16)
    ga1_ref = torch.empty_like(h1)
    ops.gemm(G, w2c, B * Hf * Hf, 256, 16, out=ga1_ref.view(-1, 256),
             ep=ops.E(act=L.ACT_MUL_LRELU_GRAD, aux=h1.view(-1, 256), ld_aux=256))
    torch.cuda.synchronize()
    # the GEMM path may split the 256-channel reduction differently: fp32 summation-order agreement
    assert float((out - ref).abs().max()) <= 2e-6 * float(ref.abs().max()), float((out - ref).abs().max())
    assert torch.equal(ga1, ga1_ref), float((ga1.float() - ga1_ref.float()).abs().max())
    # plain fp32 torch on the same bf16 operands
    t = F.conv2d(h1.float().permute(0, 3, 1, 2), w2c.float().reshape(1, 256, 4, 4))
    assert float((out - t.reshape(B, -1)).abs().max()) <= 1e-4 * float(t.abs().max())
