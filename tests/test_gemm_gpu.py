"""HIP MFMA GEMM / implicit-conv kernels vs plain PyTorch fp32 on the GPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def rel(a, b):
    return ((a.float() - b.float()).abs().max() / b.float().abs().max().clamp_min(1e-12)).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("a_kc,b_kc", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(200, 72, 96), (512, 512, 520), (64, 8, 8), (1000, 136, 64)])
def test_gemm_orientations(dtype, tol, a_kc, b_kc, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(0)
    A = torch.randn(M, K, device=DEV, generator=g)
    B = torch.randn(N, K, device=DEV, generator=g)
    ref = A.double() @ B.double().T
    As = A.to(dtype) if a_kc else A.T.contiguous().to(dtype)
    Bs = B.to(dtype) if b_kc else B.T.contiguous().to(dtype)
    if dtype == torch.bfloat16:
        ref = As.double() @ Bs.double().T if (a_kc and b_kc) else A.to(dtype).double() @ B.to(dtype).double().T
    C = ops.gemm(As, Bs, M, N, K, a_kc=a_kc, b_kc=b_kc, out_dtype=torch.float32)
    torch.cuda.synchronize()
    assert rel(C, ref) < tol


def test_gemm_epilogue_bias_act_resid_splitk():
    g = torch.Generator(device=DEV).manual_seed(1)
    M, N, K = 300, 256, 1024
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / 32
    b = torch.randn(N, device=DEV, generator=g)
    R = torch.randn(M, N, device=DEV, generator=g)
    y = ops.linear(A, W, bias=b, act=L.ACT_GELU, resid=R, ld_res=N)
    ref = F.gelu(A @ W.T + b) + R
    assert rel(y, ref) < 1e-5
    y2 = torch.zeros(M, N, device=DEV)
    ops.gemm(A, W, M, N, K, out=y2, ep=L.epilogue(atomic=1), splits=4)
    assert rel(y2, A @ W.T) < 1e-5


def test_gemm_slab_splitk_accumulate_and_bf16_out():
    """Few-tile GEMMs take the split-K slab path: the epilogue runs once on the reduced sum."""
    g = torch.Generator(device=DEV).manual_seed(2)
    M, N, K = 256, 512, 512
    A = torch.randn(M, K, device=DEV, generator=g)
    W = torch.randn(N, K, device=DEV, generator=g) / 16
    R = torch.randn(M, N, device=DEV, generator=g)
    C = R.clone()
    ops.gemm(A, W, M, N, K, out=C, ep=L.epilogue(alpha=0.5, accumulate=1))
    assert rel(C, R + 0.5 * (A @ W.T)) < 1e-5
    y = ops.linear(A.bfloat16(), W.bfloat16(), act=L.ACT_LRELU)
    ref = F.leaky_relu(A.bfloat16().float() @ W.bfloat16().float().T, 0.2)
    assert y.dtype == torch.bfloat16 and rel(y, ref) < 1e-2


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("B,H,Cin,Cout,k,stride,pad", [(3, 8, 64, 96, 3, 1, 1), (2, 16, 128, 32, 3, 1, 1),
                                                       (2, 4, 512, 256, 1, 1, 0), (2, 16, 128, 256, 4, 2, 1)])
def test_conv_fwd_wgrad(dtype, tol, B, H, Cin, Cout, k, stride, pad):
    g = torch.Generator(device=DEV).manual_seed(2)
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / (Cin * k * k) ** 0.5
    s = torch.rand(B, Cin, device=DEV, generator=g) + 0.5
    xs = x * s[:, :, None, None]
    ref = F.conv2d(xs, w, stride=stride, padding=pad)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dtype)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous().to(dtype)
    y = ops.conv2d(xn, wp, Cout, k, k, stride, pad, in_scale=s, out_dtype=torch.float32)
    assert rel(y.permute(0, 3, 1, 2), ref) < tol
    # weight gradient
    gy = torch.randn_like(ref)
    xr = xs.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    (F.conv2d(xr, wr, stride=stride, padding=pad) * gy).sum().backward()
    gw = torch.zeros_like(w)
    ops.conv2d_wgrad(gy.permute(0, 2, 3, 1).contiguous().to(dtype), xn, Cout, k, k, stride, pad, gw, in_scale=s)
    assert rel(gw, wr.grad) < tol * 2


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("C", [64, 96, 128, 192])  # one / two K steps take the short-reduction path
def test_grouped_gemm_and_wgrad(dtype, tol, C):
    g = torch.Generator(device=DEV).manual_seed(3)
    E, H4 = 4, 256
    counts = [37, 0, 300, 129]
    rows = sum(counts)
    row_off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=DEV)
    tiles = [(c + 127) // 128 for c in counts]
    tile_off = torch.tensor([0] + list(torch.tensor(tiles).cumsum(0)), dtype=torch.int32, device=DEV)
    tok = torch.randn(500, C, device=DEV, generator=g)
    perm = torch.randint(0, 500 * 2, (rows,), device=DEV, generator=g, dtype=torch.int32)  # assignment ids (t*k+j)
    W1 = torch.randn(E, H4, C, device=DEV, generator=g) / 8
    b1 = torch.randn(E, H4, device=DEV, generator=g)
    out = torch.empty(rows, H4, device=DEV, dtype=dtype)
    ops.gemm_grouped(tok.to(dtype), W1.to(dtype), row_off, tile_off, sum(tiles) + 2, H4, C, b_gstride=H4 * C,
                     out=out, ep=L.epilogue(bias=b1, act=L.ACT_GELU, a_idx=perm, a_idx_div=2))
    ref = torch.empty(rows, H4, device=DEV)
    src = tok[(perm // 2).long()]
    for e in range(E):
        r0, r1 = int(row_off[e]), int(row_off[e + 1])
        ref[r0:r1] = F.gelu(src[r0:r1] @ W1[e].T + b1[e])
    assert rel(out, ref) < tol
    # grouped wgrad: gW[e] = sum_r gP[r]^T tok[perm[r]/2]
    gP = torch.randn(rows, H4, device=DEV, generator=g)
    gW = torch.zeros(E, H4, C, device=DEV)
    ops.gemm_grouped_wgrad(gP.to(dtype), tok.to(dtype), row_off, rows, H4, C, gW, b_idx=perm, b_idx_div=2)
    refw = torch.stack([gP[int(row_off[e]):int(row_off[e + 1])].T @ src[int(row_off[e]):int(row_off[e + 1])]
                        for e in range(E)])
    assert rel(gW, refw) < tol * 2


@pytest.mark.parametrize("C,H4", [(128, 512), (256, 1024)])
def test_grouped_gelu_grad_epilogue(C, H4):
    """The expert backward's gP GEMM (engine_g.moe_bwd): gP = (gG @ W2_e) * GELU'(pre), B = W2 [E, C, H4]
    N-contiguous, bf16.  Its epilogue loads the pre-activation for the whole tile ahead of the band loop
    (MG_EPI_PREFETCH); ragged groups, an empty group and a partial last tile cover the row guards."""
    g = torch.Generator(device=DEV).manual_seed(11)
    E = 4
    counts = [200, 0, 333, 129]
    rows = sum(counts)
    row_off = torch.tensor([0] + list(torch.tensor(counts).cumsum(0)), dtype=torch.int32, device=DEV)
    tiles = [(c + 127) // 128 for c in counts]
    tile_off = torch.tensor([0] + list(torch.tensor(tiles).cumsum(0)), dtype=torch.int32, device=DEV)
    gG = (torch.randn(rows, C, device=DEV, generator=g) * 0.5).bfloat16()
    W2 = (torch.randn(E, C, H4, device=DEV, generator=g) / 16).bfloat16()
    pre = (torch.randn(rows, H4, device=DEV, generator=g) * 1.5).bfloat16()
    out = torch.full((rows, H4), float("nan"), device=DEV, dtype=torch.bfloat16)
    ops.gemm_grouped(gG, W2, row_off, tile_off, sum(tiles) + E, H4, C, b_kc=False, b_gstride=C * H4, out=out,
                     ldb=H4, ep=L.epilogue(act=L.ACT_MUL_GELU_GRAD, aux=pre, ld_aux=H4))
    torch.cuda.synchronize()
    x = pre.float()
    dgelu = 0.5 * (1 + torch.erf(x / 2 ** 0.5)) + x * torch.exp(-0.5 * x * x) / (2 * torch.pi) ** 0.5
    ref = torch.empty(rows, H4, device=DEV)
    for e in range(E):
        r0, r1 = int(row_off[e]), int(row_off[e + 1])
        ref[r0:r1] = gG[r0:r1].float() @ W2[e].float()
    ref = ref * dgelu
    assert torch.isfinite(out.float()).all()
    assert ((out.float() - ref).abs() <= 1e-2 * ref.abs() + 2e-3).all()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2), ("x3", 1e-4)])
@pytest.mark.parametrize("a_kc,b_kc", [(1, 1), (1, 0), (0, 0)])
@pytest.mark.parametrize("split", [0, 512, 64])
def test_gemm_batch_matches_individual(dtype, tol, a_kc, b_kc, split):
    """mg_gemm_batch: 11 problems of different shapes / epilogues (two launches) == plain GEMMs; split 0 = one K
    pass per tile (default), 512 = split-K slabs at a 512-block target (tuning slot 21), 64 = a 64-block target
    (no split: the batch has more tiles); "x3" = fp32 operands through split-bf16 products."""
    x3 = dtype == "x3"
    if x3:
        dtype = torch.float32
    L.call("mg_set_tuning", 21, split)
    prev = ops.set_f32x3(x3)
    try:
        _gemm_batch_case(dtype, tol, a_kc, b_kc)
    finally:
        ops.set_f32x3(prev)
        L.call("mg_set_tuning", 21, 0)


def test_gemm_batch_split_atomic():
    """Split-K slabs under atomic epilogues: three problems accumulate into one fp32 output (the value chain's
    shared text-sequence gradient) and one into its own, each slab sum added once."""
    L.call("mg_set_tuning", 21, 512)
    try:
        _split_atomic_case()
    finally:
        L.call("mg_set_tuning", 21, 0)


def _split_atomic_case():
    g = torch.Generator(device=DEV).manual_seed(7)
    out = torch.randn(256, 512, device=DEV, generator=g)
    own = torch.randn(128, 256, device=DEV, generator=g)
    ref = out.double().clone()
    ref_own = own.double().clone()
    probs = []
    for K in (512, 1024, 384):
        A = torch.randn(256, K, device=DEV, generator=g)
        Bm = torch.randn(512, K, device=DEV, generator=g) / K ** 0.5
        probs.append(dict(A=A, B=Bm, M=256, N=512, K=K, out=out, ep=L.epilogue(atomic=1)))
        ref += A.double() @ Bm.double().T
    A = torch.randn(128, 640, device=DEV, generator=g)
    Bm = torch.randn(256, 640, device=DEV, generator=g) / 640 ** 0.5
    probs.append(dict(A=A, B=Bm, M=128, N=256, K=640, out=own, ep=L.epilogue(atomic=1, alpha=0.5)))
    ref_own += 0.5 * (A.double() @ Bm.double().T)
    ops.gemm_batch(probs)
    torch.cuda.synchronize()
    assert rel(out, ref) < 1e-5 and rel(own, ref_own) < 1e-5


def _gemm_batch_case(dtype, tol, a_kc, b_kc):
    g = torch.Generator(device=DEV).manual_seed(3)
    shapes = [(256, 512, 512), (256, 256, 128), (8, 64, 512), (200, 72, 96), (512, 16, 256), (64, 8, 8),
              (256, 8, 128), (128, 512, 256), (256, 128, 512), (72, 40, 64), (256, 1024, 256)]
    probs, refs = [], []
    for i, (M, N, K) in enumerate(shapes):
        A = torch.randn(M, K, device=DEV, generator=g)
        Bm = torch.randn(N, K, device=DEV, generator=g) / K ** 0.5
        bias = torch.randn(N, device=DEV, generator=g)
        As = A.to(dtype) if a_kc else A.T.contiguous().to(dtype)
        Bs = Bm.to(dtype) if b_kc else Bm.T.contiguous().to(dtype)
        act = [0, L.ACT_LRELU, L.ACT_RSQRT_EPS][i % 3]
        Ad, Bd = A.to(dtype).double(), Bm.to(dtype).double()
        r = Ad @ Bd.T + bias.double()
        if act == L.ACT_LRELU:
            r = torch.where(r > 0, r, 0.2 * r)
        elif act == L.ACT_RSQRT_EPS:
            r = torch.rsqrt(r.abs() + 1.0)
            bias = bias + 0  # keep
        out = torch.empty(M, N, device=DEV)
        if act == L.ACT_RSQRT_EPS:  # keep the argument positive: add |min| through the bias
            shift = (Ad @ Bd.T).min().item()
            bias = bias * 0 + (1.0 - shift)
            r = torch.rsqrt(Ad @ Bd.T + bias.double() + 1e-8)
        ep = L.epilogue(bias=bias, act=act)
        probs.append(dict(A=As, B=Bs, M=M, N=N, K=K, out=out, ep=ep))
        refs.append(r)
    ops.gemm_batch(probs, a_kc=a_kc, b_kc=b_kc)
    torch.cuda.synchronize()
    for q, r in zip(probs, refs):
        assert rel(q["out"], r) < tol, (q["M"], q["N"], q["K"])


# tuning slots (mg_common.h): 0 = conv weight-gradient tile, 2 = conv forward tile, 3 = plain GEMM tile
@pytest.mark.parametrize("tile", [128, 256, 257])
@pytest.mark.parametrize("B,H,Cin,Cout,k,stride,pad", [(3, 8, 64, 96, 3, 1, 1), (4, 32, 128, 256, 4, 2, 1),
                                                       (2, 8, 256, 512, 3, 1, 1)])
@pytest.mark.parametrize("scaled", [False, True])
def test_conv_wide_tiles_bf16(tile, B, H, Cin, Cout, k, stride, pad, scaled):
    """Forced 128x128 / 256x128 / 128x256 tiles (ragged M / N tails included) vs fp32 PyTorch."""
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, k, k, device=DEV, generator=g) / (Cin * k * k) ** 0.5
    s = torch.rand(B, Cin, device=DEV, generator=g) + 0.5 if scaled else None
    xs = x * s[:, :, None, None] if scaled else x
    xn = x.permute(0, 2, 3, 1).contiguous().bfloat16()
    wp = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous().bfloat16()
    ref = F.conv2d(xs, w, stride=stride, padding=pad)
    gy = torch.randn_like(ref)
    xr = xs.clone().requires_grad_(True)
    wr = w.clone().requires_grad_(True)
    (F.conv2d(xr, wr, stride=stride, padding=pad) * gy).sum().backward()
    try:
        L.call("mg_set_tuning", 0, tile)
        L.call("mg_set_tuning", 2, tile)
        y = ops.conv2d(xn, wp, Cout, k, k, stride, pad, in_scale=s, out_dtype=torch.float32)
        gw = torch.zeros_like(w)
        ops.conv2d_wgrad(gy.permute(0, 2, 3, 1).contiguous().bfloat16(), xn, Cout, k, k, stride, pad, gw, in_scale=s)
        torch.cuda.synchronize()
    finally:
        L.call("mg_set_tuning", 0, 0)
        L.call("mg_set_tuning", 2, 0)
    assert rel(y.permute(0, 3, 1, 2), ref) < 2e-2
    assert rel(gw, wr.grad) < 4e-2


@pytest.mark.parametrize("a_kc,b_kc", [(1, 1), (1, 0), (0, 1), (0, 0)])
@pytest.mark.parametrize("M,N,K", [(1000, 520, 264), (512, 256, 64)])
def test_gemm_wide_tile_bf16(a_kc, b_kc, M, N, K):
    g = torch.Generator(device=DEV).manual_seed(6)
    A = torch.randn(M, K, device=DEV, generator=g).bfloat16()
    Bm = torch.randn(N, K, device=DEV, generator=g).bfloat16()
    ref = A.float() @ Bm.float().T
    Aa = A if a_kc else A.T.contiguous()
    Bb = Bm if b_kc else Bm.T.contiguous()
    try:
        L.call("mg_set_tuning", 3, 257)
        C = ops.gemm(Aa, Bb, M, N, K, a_kc=a_kc, b_kc=b_kc, out_dtype=torch.float32)
        torch.cuda.synchronize()
    finally:
        L.call("mg_set_tuning", 3, 0)
    assert rel(C, ref) < 1e-2


@pytest.mark.parametrize("M,N,K", [(300, 256, 128), (4096, 512, 128)])
def test_bf16_gelu_epilogues(M, N, K):
    """bf16 GELU / GELU' epilogues (polynomial erf, |err| <= 1.5e-7) vs exact fp32 on the same bf16 operands:
    the only difference left is the bf16 rounding of the result."""
    g = torch.Generator(device=DEV).manual_seed(7)
    A = (torch.randn(M, K, device=DEV, generator=g) * 0.5).bfloat16()
    W = (torch.randn(N, K, device=DEV, generator=g) / 8).bfloat16()
    b = torch.randn(N, device=DEV, generator=g)
    pre_ref = A.float() @ W.float().T + b
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    y = ops.gemm(A, W, M, N, K, out_dtype=torch.bfloat16, ep=L.epilogue(bias=b, act=L.ACT_GELU, out_pre=pre, ld_pre=N))
    torch.cuda.synchronize()
    ref = F.gelu(pre_ref)
    assert ((y.float() - ref).abs() <= 1e-2 * ref.abs() + 2e-3).all()
    # GELU' times an upstream gradient, with the bf16 pre-activation as aux
    x = pre
    xg = x.float()
    cdf = 0.5 * (1 + torch.erf(xg / 2 ** 0.5))
    dref = cdf + xg * torch.exp(-0.5 * xg * xg) / (2 * torch.pi) ** 0.5
    gy = ops.gemm(A, W, M, N, K, out_dtype=torch.bfloat16, ep=L.epilogue(act=L.ACT_MUL_GELU_GRAD, aux=x, ld_aux=N))
    torch.cuda.synchronize()
    gref = (A.float() @ W.float().T) * dref
    assert ((gy.float() - gref).abs() <= 1e-2 * gref.abs() + 2e-3).all()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("Cin,Cg,OH", [(3, 128, 32), (128, 256, 16), (16, 64, 8)])
def test_dgrad_s2(dtype, tol, Cin, Cg, OH):
    """4x4 / stride-2 / pad-1 conv data gradient (parity-class split) vs torch's conv autograd, incl. the
    128 x 32 tiles of the image gradient (Cin = 3, output channel-padded to 4)."""
    g = torch.Generator(device=DEV).manual_seed(8)
    B = 4
    W = torch.randn(Cg, Cin, 4, 4, device=DEV, generator=g) / (Cin * 16) ** 0.5
    gy = torch.randn(B, Cg, OH, OH, device=DEV, generator=g)
    x = torch.zeros(B, Cin, 2 * OH, 2 * OH, device=DEV, requires_grad=True)
    (F.conv2d(x, W, stride=2, padding=1) * gy).sum().backward()
    ld = (Cin + 3) // 4 * 4 if Cin < 8 else Cin
    out = torch.zeros(B, 2 * OH, 2 * OH, ld, device=DEV)
    wcls = ops.pack_dgrad_s2(W, dtype, rows=Cin)
    ops.dgrad_s2(gy.permute(0, 2, 3, 1).contiguous().to(dtype), wcls, Cin, out)
    torch.cuda.synchronize()
    assert rel(out[..., :Cin].permute(0, 3, 1, 2), x.grad) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-5), (torch.bfloat16, 2e-2)])
@pytest.mark.parametrize("Cout", [32, 24])
def test_conv_narrow_output(dtype, tol, Cout):
    """Narrow implicit convs over many pixels (the MTM offset heads: 128 -> 32, 3x3 at 16x16, B = 128) take
    128 x 32 tiles; ragged Cout included."""
    g = torch.Generator(device=DEV).manual_seed(9)
    B, H, Cin = 128, 16, 128
    x = torch.randn(B, Cin, H, H, device=DEV, generator=g)
    w = torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) / (Cin * 9) ** 0.5
    bias = torch.randn(Cout, device=DEV, generator=g)
    ref = F.leaky_relu(F.conv2d(x.to(dtype).float(), w.to(dtype).float(), bias, padding=1), 0.2)
    xn = x.permute(0, 2, 3, 1).contiguous().to(dtype)
    wp = w.permute(0, 2, 3, 1).reshape(Cout, -1).contiguous().to(dtype)
    y = ops.conv2d(xn, wp, Cout, 3, 3, 1, 1, out_dtype=torch.float32, ep=ops.E(bias=bias, act=L.ACT_LRELU))
    torch.cuda.synchronize()
    assert rel(y.permute(0, 3, 1, 2), ref) < tol


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
@pytest.mark.parametrize("B,H,Cin,Cout,k", [(256, 4, 512, 512, 3), (37, 8, 256, 256, 3), (16, 16, 128, 128, 3),
                                            (6, 32, 64, 32, 3), (9, 16, 256, 128, 1), (256, 16, 128, 32, 3)])
def test_conv_wgrad_stride1_loader(dtype, B, H, Cin, Cout, k):
    """Weight gradients of stride-1 "same" convolutions (the generator's modulated 3x3 / 1x1 convs and MTM offset
    heads, t2i_moe_gan.py:169-180) through the cheap-address column loader (LdMCConvS1): bit-identical to the
    generic implicit-conv loader (MG_TUNE_S1_OFF = 12 switches it back: same values, same summation order), and
    equal to the torch reference within the dtype's tolerance."""
    from moegan_mi import _lib as L
    g = torch.Generator(device=DEV).manual_seed(B * H + Cin)
    x = torch.randn(B, H, H, Cin, device=DEV, generator=g).to(dtype)
    gy = torch.randn(B, H, H, Cout, device=DEV, generator=g).to(dtype)
    pad = k // 2
    gw1 = torch.zeros(Cout, Cin, k, k, device=DEV)
    ops.conv2d_wgrad(gy, x, Cout, k, k, 1, pad, gw1)
    L.call("mg_set_tuning", 12, 1)
    try:
        gw0 = torch.zeros(Cout, Cin, k, k, device=DEV)
        ops.conv2d_wgrad(gy, x, Cout, k, k, 1, pad, gw0)
    finally:
        L.call("mg_set_tuning", 12, 0)
    torch.cuda.synchronize()
    xr = x.float().permute(0, 3, 1, 2).contiguous()
    wr = torch.zeros(Cout, Cin, k, k, device=DEV, requires_grad=True)
    (F.conv2d(xr, wr, padding=pad) * gy.float().permute(0, 3, 1, 2)).sum().backward()
    assert rel(gw1, wr.grad) < (1e-5 if dtype == torch.float32 else 1e-2)
    if dtype == torch.bfloat16:  # slabs + fixed-order fold: deterministic, so the two loaders agree bit for bit
        assert torch.equal(gw1, gw0)
    else:
        assert rel(gw1, gw0) < 1e-6


@pytest.mark.parametrize("M,N,K,alpha", [(384, 128, 65536, 1.0), (128, 128, 65536, 1.0), (256, 256, 16384, 0.5),
                                         (1536, 512, 4096, 1.0), (256, 16, 65536, 1.0), (136, 200, 5000, 1.0),
                                         (128, 256, 65536, 1.0), (512, 512, 2048, 1.0), (8, 128, 3000, 2.0)])
def test_wide_weight_gradient(M, N, K, alpha):
    """Linear-layer weight gradients C += alpha * A^T B (bf16 [K][M] x [K][N], fp32 C through an atomic epilogue):
    the long-reduction kernel (csrc/mg_wgrad_wide.hip, forced onto every eligible shape: tuning slot 15 = 2, and on
    256^2 tiles: 4) against
    fp64 on the same bf16 operands and against the generic split-K GEMM (slot 15 = 1); fixed-order fold: two calls
    give the same bits.  The automatic routing (slot 15 = 0) is held to the same fp64 bound."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn(K, M, device=DEV, generator=g).bfloat16()
    B = torch.randn(K, N, device=DEV, generator=g).bfloat16()
    ref = alpha * (A.double().T @ B.double()) + 0.5

    def run():
        C = torch.full((M, N), 0.5, device=DEV)
        ops.gemm(A, B, M, N, K, a_kc=False, b_kc=False, out=C, ep=ops.E(alpha=alpha, atomic=1), splits=0)
        return C
    C4 = run()
    L.call("mg_set_tuning", 15, 2)
    try:
        C1, C2 = run(), run()
        L.call("mg_set_tuning", 15, 4)  # 256^2 tiles where M, N >= 256
        C5 = run()
        L.call("mg_set_tuning", 15, 1)
        C3 = run()
    finally:
        L.call("mg_set_tuning", 15, 0)
    torch.cuda.synchronize()
    scale = float(ref.abs().max())
    assert float((C1.double() - ref).abs().max()) <= 2e-6 * scale * (K / 4096) ** 0.5 + 1e-6
    assert float((C1 - C3).abs().max()) <= 4e-6 * scale * (K / 4096) ** 0.5 + 1e-6
    assert torch.equal(C1, C2)
    assert float((C5.double() - ref).abs().max()) <= 2e-6 * scale * (K / 4096) ** 0.5 + 1e-6
    assert float((C4.double() - ref).abs().max()) <= 2e-6 * scale * (K / 4096) ** 0.5 + 1e-6


@pytest.mark.parametrize("B,H,Cin,Cout", [(64, 16, 256, 128), (256, 8, 256, 256), (16, 8, 512, 512), (8, 16, 128, 8)])
def test_conv1x1_weight_gradient_long_reduction(B, H, Cin, Cout):
    """1x1 / stride-1 conv weight gradients (ConvolutionBlock.skip_proj, AttentionBlock.proj_in / proj_out,
    t2i_moe_gan.py:574, :615-616) go through the long-reduction kernel (mg_wgrad_wide.hip) when it takes the shape:
    gw += gy^T x over the B*H*W pixels, against fp64 on the same bf16 operands and against the generic conv weight
    gradient (tuning slot 15 = 1), accumulating into a non-zero gradient."""
    g = torch.Generator(device=DEV).manual_seed(B * H + Cin)
    x = torch.randn(B, H, H, Cin, device=DEV, generator=g).bfloat16()
    gy = torch.randn(B, H, H, Cout, device=DEV, generator=g).bfloat16()
    base = torch.randn(Cout, Cin, 1, 1, device=DEV, generator=g)
    ref = base.double() + (gy.reshape(-1, Cout).double().T @ x.reshape(-1, Cin).double()).view(Cout, Cin, 1, 1)

    def run():
        gw = base.clone()
        ops.conv2d_wgrad(gy, x, Cout, 1, 1, 1, 0, gw)
        return gw
    gw_auto = run()
    L.call("mg_set_tuning", 15, 1)
    try:
        gw_gen = run()
    finally:
        L.call("mg_set_tuning", 15, 0)
    torch.cuda.synchronize()
    scale = float((ref - base.double()).abs().max())
    P = B * H * H
    bound = 2e-6 * scale * (P / 4096) ** 0.5 + 1e-5
    assert float((gw_auto.double() - ref).abs().max()) <= bound
    assert float((gw_gen.double() - ref).abs().max()) <= bound
