"""Split-bf16 fp32 GEMMs (MG_F32X3: fp32 operands, products hi*hi + hi*lo + lo*hi on the bf16 MFMA, fp32
accumulation) -- the bf16 step's mapping / text-projection / style / demodulation / router-vector GEMMs
(t2i_moe_gan.py:158, :664-690, :364-371).  Held against an fp64 torch product at 3e-5 relative L2 (exact-fp32
MFMA: ~1e-6; plain bf16 operands: ~4e-3), in every operand orientation, through the few-tile split-K slab path,
the atomic split-K weight-gradient path, the fused epilogue (bias + LeakyReLU / rsqrt) and the batched launch."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
TOL = 3e-5


def _rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


@pytest.fixture(autouse=True)
def _x3():
    from moegan_mi import ops
    prev = ops.set_f32x3(True)
    yield
    ops.set_f32x3(prev)


@pytest.mark.parametrize("M,N,K", [(256, 512, 512), (256, 4864, 512), (4864, 512, 256), (256, 128, 1024),
                                   (8, 16, 48), (1000, 72, 200)])
@pytest.mark.parametrize("a_kc,b_kc", [(1, 1), (1, 0), (0, 1), (0, 0)])
def test_gemm_x3_orientations(M, N, K, a_kc, b_kc):
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(M + N + K + 7 * a_kc + 3 * b_kc)
    A = torch.randn(M, K, device=DEV, generator=g)
    B = torch.randn(N, K, device=DEV, generator=g)
    Aop = A.contiguous() if a_kc else A.t().contiguous()
    Bop = B.contiguous() if b_kc else B.t().contiguous()
    out = ops.gemm(Aop, Bop, M, N, K, a_kc=bool(a_kc), b_kc=bool(b_kc), out_dtype=torch.float32)
    ref = A.double() @ B.double().t()
    assert _rel(out, ref) <= TOL
    ops.set_f32x3(False)  # the exact-fp32 path on the same operands, for the printed comparison
    exact = ops.gemm(Aop, Bop, M, N, K, a_kc=bool(a_kc), b_kc=bool(b_kc), out_dtype=torch.float32)
    print(f"M={M} N={N} K={K} a_kc={a_kc} b_kc={b_kc}: x3 {_rel(out, ref):.2e}, f32 {_rel(exact, ref):.2e}")


def test_linear_x3_epilogue_and_wgrad():
    from moegan_mi import _lib as L
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(256, 512, device=DEV, generator=g)
    W = torch.randn(512, 512, device=DEV, generator=g) * 0.05
    b = torch.randn(512, device=DEV, generator=g)
    y = ops.linear(x, W, bias=b, act=L.ACT_LRELU)
    pre = x.double() @ W.double().t() + b.double()
    ref = torch.where(pre > 0, pre, 0.2 * pre)
    assert _rel(y, ref) <= TOL
    gy = torch.randn(256, 512, device=DEV, generator=g)
    gW = torch.zeros(512, 512, device=DEV)
    ops.linear_wgrad(gy, x, gW)  # atomic split-K over the 256 rows
    assert _rel(gW, gy.double().t() @ x.double()) <= TOL
    gx = ops.linear_dgrad(gy, W)
    assert _rel(gx, gy.double() @ W.double()) <= TOL


def test_gemm_batch_x3():
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(2)
    probs, refs = [], []
    for M, N, K in ((256, 128, 512), (512, 8, 128), (256, 8, 128), (64, 512, 256)):
        A = torch.randn(M, K, device=DEV, generator=g)
        B = torch.randn(N, K, device=DEV, generator=g)
        out = torch.empty(M, N, device=DEV)
        probs.append(dict(A=A, B=B, M=M, N=N, K=K, out=out))
        refs.append(A.double() @ B.double().t())
    ops.gemm_batch(probs)
    for q, r in zip(probs, refs):
        assert _rel(q["out"], r) <= TOL
