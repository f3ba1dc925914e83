"""Gradient folds (mg_fold.hip): deferred vs immediate, chained and overlapping records, thin / wide row folds.

Every two-pass gradient reduction of the step ends in a fold; inside a training step the folds are deferred and run
batched (ops.fold_defer / ops.fold_flush).  The folded gradients must be bit-identical to the immediate folds (the
same kernels and summation order), and records that write the same output in one batch (the real, fake and R1
weight gradients of one discriminator conv) must neither race nor reorder."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def _conv_wgrads(shapes, gw, seed):
    """conv2d_wgrad of each (B, H, Cin, Cout, k, stride, pad, dtype) into gw[i] (gw entries may repeat)."""
    g = torch.Generator(device=DEV).manual_seed(seed)
    for (B, H, Cin, Cout, k, stride, pad, dtype), out in zip(shapes, gw):
        OH = (H + 2 * pad - k) // stride + 1
        x = torch.randn(B, H, H, Cin, device=DEV, generator=g).to(dtype)
        gy = torch.randn(B, OH, OH, Cout, device=DEV, generator=g).to(dtype)
        ops.conv2d_wgrad(gy, x, Cout, k, k, stride, pad, out)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_deferred_conv_wgrad_folds_bit_identical(dtype):
    """Three weight gradients into one tensor (a chain), two into another, one into a third: deferred + one flush
    equals immediate folds bit for bit, and matches an fp64 reference of the summed gradients."""
    shapes = [(16, 16, 128, 128, 3, 1, 1, dtype), (16, 16, 128, 128, 3, 1, 1, dtype),
              (32, 32, 128, 256, 4, 2, 1, dtype), (16, 16, 128, 128, 3, 1, 1, dtype),
              (32, 32, 128, 256, 4, 2, 1, dtype), (8, 8, 256, 256, 3, 1, 1, dtype)]
    which = [0, 0, 1, 0, 1, 2]

    def run(defer):
        gws = [torch.zeros(128, 128, 3, 3, device=DEV), torch.zeros(256, 128, 4, 4, device=DEV),
               torch.zeros(256, 256, 3, 3, device=DEV)]
        ops.fold_defer(defer)
        try:
            _conv_wgrads(shapes, [gws[w] for w in which], seed=3)
        finally:
            ops.fold_defer(False)
        torch.cuda.synchronize()
        return gws

    imm, dfr = run(False), run(True)
    for a, b in zip(imm, dfr):
        assert torch.equal(a, b)
    # fp64 reference of the first tensor's chain
    g = torch.Generator(device=DEV).manual_seed(3)
    ref = torch.zeros(128, 128, 3, 3, dtype=torch.float64, device=DEV)
    for (B, H, Cin, Cout, k, stride, pad, dt), w in zip(shapes, which):
        OH = (H + 2 * pad - k) // stride + 1
        x = torch.randn(B, H, H, Cin, device=DEV, generator=g).to(dt)
        gy = torch.randn(B, OH, OH, Cout, device=DEV, generator=g).to(dt)
        if w != 0:
            continue
        ref += torch.nn.grad.conv2d_weight(x.double().permute(0, 3, 1, 2), (Cout, Cin, k, k),
                                           gy.double().permute(0, 3, 1, 2), stride=stride, padding=pad)
    err = ((imm[0].double() - ref).norm() / ref.norm()).item()
    assert err < (1e-5 if dtype == torch.float32 else 1e-5), err


@pytest.mark.parametrize("nrows,ncols,vec", [(1, 4096, True), (7, 1000, False), (16, 65536, True), (17, 2048, True),
                                             (300, 578, False), (512, 6144, True)])
def test_rows_fold_queue(nrows, ncols, vec):
    """Rows folds through mg_fold_rows_queue (ops.fold_add is its one-row case): thin (<= 16 rows) and wide
    records, vector and scalar, chained records on one output, deferred == immediate bit for bit, == the
    sequential fp32 row sum."""
    import ctypes
    g = torch.Generator(device=DEV).manual_seed(nrows * 7 + ncols)
    stride = ncols + (0 if vec else 1)
    srcs = [torch.randn(nrows, stride, device=DEV, generator=g) for _ in range(3)]
    na = ncols // 2 // 4 * 4

    def run(defer):
        out_a = torch.randn(na, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1))
        out_b = torch.randn(ncols - na, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))
        recs = (ops._FoldRows * 3)()
        for i, s in enumerate(srcs):
            recs[i] = ops._FoldRows(s.data_ptr(), stride, nrows, ncols, na, out_a.data_ptr(), out_b.data_ptr())
        ops.fold_defer(defer)
        try:
            ops.call("mg_fold_rows_queue", 3, ctypes.addressof(recs), ops.S())
        finally:
            ops.fold_defer(False)
        torch.cuda.synchronize()
        return torch.cat([out_a, out_b])

    imm, dfr = run(False), run(True)
    assert torch.equal(imm, dfr)
    exp = torch.cat([torch.randn(na, device=DEV, generator=torch.Generator(device=DEV).manual_seed(1)),
                     torch.randn(ncols - na, device=DEV, generator=torch.Generator(device=DEV).manual_seed(2))])
    ref = exp.double() + sum(s[:, :ncols].double().sum(0) for s in srcs)
    assert torch.allclose(imm.double(), ref, rtol=1e-5, atol=1e-4 * (nrows ** 0.5))


def test_fold_add_keeps_tensors_until_flush():
    """ops.fold_add under deferral: the queued record's tensors stay allocated until the flush, so a temporary
    source dropped by the caller is still read correctly."""
    dst = torch.zeros(4096, device=DEV)
    ops.fold_defer(True)
    try:
        ops.fold_add([(torch.full((4096,), 2.0, device=DEV), dst)])
        junk = [torch.full((4096,), -1.0, device=DEV) for _ in range(8)]  # would reuse a freed block
        del junk
    finally:
        ops.fold_defer(False)
    torch.cuda.synchronize()
    assert torch.equal(dst, torch.full((4096,), 2.0, device=DEV))


def _splitk_modes(fn):
    """fn() under the two-launch split-K reduction (the default) and the in-launch one (tuning slot 23 = 1, A/B),
    the latter twice (the tile counters reset themselves)."""
    from moegan_mi import _lib as L
    two = fn()
    L.call("mg_set_tuning", 23, 1)
    try:
        one, again = fn(), fn()
    finally:
        L.call("mg_set_tuning", 23, 0)
    torch.cuda.synchronize()
    return two, one, again


@pytest.mark.parametrize("dtype,M,N,K", [(torch.bfloat16, 256, 512, 1024), (torch.float32, 257, 512, 512),
                                         (torch.bfloat16, 100, 72, 4096), (torch.float32, 64, 1024, 2048)])
def test_splitk_in_launch_reduction_bit_identical(dtype, M, N, K):
    """Few-tile GEMMs split K into fp32 slabs; the last-arriving split of each tile reduces them through the real
    epilogue (bias + leaky ReLU here) inside the launch: bit-identical to the separate reduction launch, and the
    per-stream tile counters come back to zero (a repeat gives the same bits)."""
    g = torch.Generator(device=DEV).manual_seed(M + N + K)
    A = torch.randn(M, K, device=DEV, generator=g).to(dtype)
    B = (torch.randn(N, K, device=DEV, generator=g) * K ** -0.5).to(dtype)
    bias = torch.randn(N, device=DEV, generator=g)
    ep = ops.E(bias=bias, act=1)  # ACT_LRELU
    out_dtype = torch.float32 if dtype == torch.float32 else torch.bfloat16
    two, one, again = _splitk_modes(lambda: ops.gemm(A, B, M, N, K, ep=ep, out_dtype=out_dtype))
    assert torch.equal(two, one) and torch.equal(one, again)
    ref = torch.nn.functional.leaky_relu(A.double() @ B.double().T + bias.double(), 0.2)
    err = ((one.double() - ref).norm() / ref.norm()).item()
    assert err < (2e-2 if dtype == torch.bfloat16 else 2e-3), err


def test_splitk_in_launch_reduction_conv():
    """A few-tile implicit conv (16 output tiles, K = 2304) with K split into slabs: in-launch reduction
    bit-identical to the two-launch form."""
    g = torch.Generator(device=DEV).manual_seed(5)
    x = torch.randn(4, 16, 16, 256, device=DEV, generator=g).bfloat16()
    W = torch.randn(64, 256, 3, 3, device=DEV, generator=g) * (9 * 256) ** -0.5
    wp = ops.pack_conv(W, torch.bfloat16)
    bias = torch.randn(64, device=DEV, generator=g)
    two, one, again = _splitk_modes(lambda: ops.conv2d(x, wp, 64, 3, 3, 1, 1, ep=ops.E(bias=bias, act=1)))
    assert torch.equal(two, one) and torch.equal(one, again)
    ref = torch.nn.functional.leaky_relu(torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), W.double(),
                                                                     bias.double(), padding=1), 0.2)
    err = ((one.double().permute(0, 3, 1, 2) - ref).norm() / ref.norm()).item()
    assert err < 2e-2, err


def test_fold_arena_release_and_size():
    """The deferred-fold arena is reported (mg_fold_arena_bytes) and freed by mg_fold_release once the stream no
    longer defers; releasing a deferring stream is refused."""
    import torch
    from moegan_mi import _lib as L
    from moegan_mi import ops
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        ops.fold_defer(True)
        x = torch.randn(64, 4, 4, 128, device="cuda", dtype=torch.bfloat16)
        gy = torch.randn(64, 4, 4, 256, device="cuda", dtype=torch.bfloat16)
        gw = torch.zeros(256, 128, 3, 3, device="cuda")
        ops.conv2d_wgrad(gy.view(-1, 256), x, 256, 3, 3, 1, 1, gw)
        held = ops.fold_arena_bytes()
        with pytest.raises(L.MGError):
            ops.fold_release()
        ops.fold_defer(False)
        ops.fold_release()
        assert ops.fold_arena_bytes() == 0
    torch.cuda.synchronize()
    assert held >= 0
