"""MX-fp8 path (BASELINE config C5): mg_quant_mx8 and mg_conv2d_fwd_mx8 on the GPU.

Two bars:
* exact -- the quantizer against a torch restatement of the OCP MX rule (e = ceil(log2(amax / 448)), e4m3
  round-to-nearest-even via torch.float8_e4m3fn), byte for byte; the conv against an fp64 convolution of the
  dequantized operands (activations quantized by mg_quant_mx8 of the NHWC rows), at the fp32-accumulation tolerance 5e-5 of max |y| (K up to 4608);
* precision -- the conv against the unquantized bf16 operands: relative RMS error <= 6e-2 and cosine
  >= 0.998 (the stated fp8 tolerance of the C5 path; measured values are printed).
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def mx_ref(x2):
    """torch restatement of mg_quant_mx8 for [rows, K] bf16: (e4m3 bytes, E8M0 bytes)."""
    rows, K = x2.shape
    xb = x2.float().view(rows, K // 32, 32)
    amax = xb.abs().amax(-1)
    m, ex = torch.frexp(amax / 448.0)
    e = torch.where(m == 0.5, ex - 1, ex) + 127
    e = torch.where(amax == 0, torch.ones_like(e), e.clamp(1, 254))
    q = (xb * torch.exp2(127.0 - e.float())[..., None]).to(torch.float8_e4m3fn)
    return q.view(torch.uint8).view(rows, K), e.to(torch.uint8)


def deq(q, sc):
    rows, K = q.shape
    v = q.view(torch.float8_e4m3fn).double().view(rows, K // 32, 32)
    return (v * torch.exp2(sc.double() - 127.0)[..., None]).view(rows, K)


def pack(Wt):  # [Cout, Cin, 3, 3] -> [Cout, 9 * Cin] ((kh, kw, ci) order, mg_pack_conv layout)
    return Wt.permute(0, 2, 3, 1).reshape(Wt.shape[0], -1).contiguous()


def test_quant_mx8_matches_ocp_rule():
    g = torch.Generator(device=DEV).manual_seed(0)
    rows, K = 300, 256
    # per-block magnitudes over 2^-20 .. 2^20, plus an all-zero block and exact powers of two
    x = torch.randn(rows, K, device=DEV, generator=g) * torch.exp2(torch.randint(-20, 20, (rows, K // 32, 1), device=DEV,
                                                                                  generator=g).float()).repeat_interleave(32, -1).view(rows, K)
    x[3, 64:96] = 0
    x[5, :32] = 448.0
    x[6, :32] = torch.tensor([2.0 ** i for i in range(-16, 16)], device=DEV)
    xb = x.bfloat16()
    q, sc = ops.quant_mx8(xb)
    qr, scr = mx_ref(xb)
    assert torch.equal(sc, scr)
    assert torch.equal(q, qr)
    # nothing saturates: each element is within half an e4m3 step (2^-4 relative, or half the subnormal step
    # 2^-10 of the block scale for elements far below the block maximum)
    step = torch.exp2(sc.double() - 127.0).repeat_interleave(32, -1) * 2.0 ** -10
    err = (deq(q, sc) - xb.double()).abs()
    assert bool((err <= 2.0 ** -4 * xb.double().abs() + step + 1e-300).all())


@pytest.mark.parametrize("B,H,Cin,Cout,tile", [(4, 4, 512, 512, 0), (8, 8, 512, 256, 0), (4, 8, 256, 256, 128),
                                               (128, 16, 128, 128, 0), (2, 16, 256, 128, 0), (3, 8, 128, 40, 0)])
def test_conv_mx8_exact_vs_dequantized(B, H, Cin, Cout, tile):
    g = torch.Generator(device=DEV).manual_seed(B * 7 + Cin)
    x = (torch.randn(B, H, H, Cin, device=DEV, generator=g) *
         torch.rand(B, H, H, 1, device=DEV, generator=g).mul(4).exp()).bfloat16()
    Wt = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (3 * Cin ** 0.5)
    wp = pack(Wt).bfloat16()
    wq, wsc = ops.quant_mx8(wp)
    xq, xsc = ops.quant_mx8(x.view(-1, Cin))
    L.call("mg_set_tuning", 2, tile)
    try:
        y = ops.conv2d_mx8(xq.view(B, H, H, Cin), xsc, wq, wsc, Cout, 3, 3, 1, 1, out_dtype=torch.float32)
    finally:
        L.call("mg_set_tuning", 2, 0)
    torch.cuda.synchronize()
    xd = deq(xq, xsc).view(B, H, H, Cin).permute(0, 3, 1, 2)
    wd = deq(wq, wsc).view(Cout, 3, 3, Cin).permute(0, 3, 1, 2)
    ref = F.conv2d(xd, wd, padding=1).permute(0, 2, 3, 1)
    assert ((y.double() - ref).abs().max() / ref.abs().max()).item() < 5e-5
    # precision vs the unquantized bf16 operands
    full = F.conv2d(x.double().permute(0, 3, 1, 2), wp.double().view(Cout, 3, 3, Cin).permute(0, 3, 1, 2),
                    padding=1).permute(0, 2, 3, 1)
    rrms = ((y.double() - full).norm() / full.norm()).item()
    cos = F.cosine_similarity(y.double().flatten(), full.flatten(), dim=0).item()
    print(f"mx8 conv B={B} H={H} {Cin}->{Cout}: rel RMS {rrms:.4f}, cosine {cos:.6f}")
    assert rrms <= 6e-2 and cos >= 0.998


def test_conv_mx8_epilogue_bf16():
    """Demodulation scale + LeakyReLU + residual epilogue with bf16 output, as the modulated-conv forward uses it."""
    g = torch.Generator(device=DEV).manual_seed(5)
    B, H, Cin, Cout = 8, 8, 256, 256
    x = torch.randn(B, H, H, Cin, device=DEV, generator=g).bfloat16()
    Wt = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (3 * Cin ** 0.5)
    d = torch.rand(B, Cout, device=DEV, generator=g) + 0.5
    R = torch.randn(B, H, H, Cout, device=DEV, generator=g).bfloat16()
    wq, wsc = ops.quant_mx8(pack(Wt).bfloat16())
    xq, xsc = ops.quant_mx8(x.view(-1, Cin))
    xq = xq.view(B, H, H, Cin)
    ep = L.epilogue(scale=d, scale_shift=6, scale_ld=Cout, act=L.ACT_LRELU, resid=R, ld_res=Cout)
    y = ops.conv2d_mx8(xq, xsc, wq, wsc, Cout, 3, 3, 1, 1, ep=ep)
    y32 = ops.conv2d_mx8(xq, xsc, wq, wsc, Cout, 3, 3, 1, 1, out_dtype=torch.float32)
    torch.cuda.synchronize()
    ref = F.leaky_relu(y32 * d[:, None, None, :], 0.2) + R.float()
    assert y.dtype == torch.bfloat16
    assert ((y.float() - ref).abs().max() / ref.abs().max()).item() < 1e-2


def test_conv_mx8_rejects_bad_shapes():
    x = torch.zeros(2, 4, 4, 64, device=DEV, dtype=torch.uint8)
    xs = torch.zeros(32, 2, device=DEV, dtype=torch.uint8)
    wq = torch.zeros(64, 9 * 64, device=DEV, dtype=torch.uint8)
    sc = torch.zeros(64, 18, device=DEV, dtype=torch.uint8)
    with pytest.raises(RuntimeError, match="Cin"):
        ops.conv2d_mx8(x, xs, wq, sc, 64, 3, 3, 1, 1)


def test_quant_mx8_batch_equals_single():
    """mg_quant_mx8_batch (the per-step MX-fp8 weight copies in one launch) gives, descriptor by descriptor, the bytes
    of separate mg_quant_mx8 calls: ragged row counts and K, a strided source, more descriptors than one launch holds."""
    g = torch.Generator(device="cuda").manual_seed(5)
    xs = []
    for i in range(37):
        rows, K = 1 + (i * 53) % 700, 32 * (1 + (i * 7) % 40)
        base = (torch.randn(rows, K + 32 * (i % 3), device="cuda", generator=g) * (10.0 ** (i % 5 - 2))).bfloat16()
        xs.append(base[:, :K])
    got = ops.quant_mx8_batch(xs)
    torch.cuda.synchronize()
    for x, (q, sc) in zip(xs, got):
        q1, sc1 = ops.quant_mx8(x)
        assert torch.equal(q, q1) and torch.equal(sc, sc1)
