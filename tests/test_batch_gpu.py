"""Multi-tensor launches (mg_prep_batch, mg_colsum_batch) against the single-tensor kernels they replace in the
training step: packs / demodulation sums / reparameterisation bit-exact, column sums against a float64 sum.
Shapes are the generator's (3x3 modulated convs 128..512, 1x1 skips, 32-channel offset heads, 4x4 D convs) plus
ragged ones, more than 32 descriptors (two launches) and empty entries."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from moegan_mi import ops  # noqa: E402

DEV = "cuda"


def _w(shape, seed):
    g = torch.Generator(device=DEV).manual_seed(seed)
    return torch.randn(*shape, device=DEV, generator=g) * 0.05


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_prep_batch_matches_single_kernels(dtype):
    shapes = [(512, 512, 3, 3), (256, 512, 3, 3), (128, 256, 3, 3), (32, 128, 3, 3), (3, 128, 1, 1),
              (256, 128, 1, 1), (128, 3, 4, 4), (256, 128, 4, 4), (5, 7, 3, 3)]
    pb = ops.PrepBatch(dtype)
    got, want = [], []
    for i, shp in enumerate(shapes):
        W = _w(shp, i)
        Cout, Cin, KH, KW = shp
        rows = max(Cout, 8)
        got.append(pb.pack(W, rows=rows))
        want.append(ops.pack_conv(W, dtype, rows=rows))
        got.append(pb.pack(W, flip=True))
        want.append(ops.pack_conv(W, dtype, flip=True))
        got.append(pb.wsq(W, rows=rows))
        want.append(ops.wsq(W, rows=rows))
        if KH == 4:
            got.append(pb.pack_dgrad_s2(W, rows=max(Cin, 3)))
            want.append(ops.pack_dgrad_s2(W, dtype, rows=max(Cin, 3)))
        gwsq = _w((Cout, Cin), 100 + i)
        gA, gB = _w(shp, 200 + i), None
        gB = gA.clone()
        pb.wsq_bwd(W, gwsq, gA)
        ops.wsq_bwd(W, gwsq, gB)
        got.append(gA)
        want.append(gB)
    for i, n in enumerate((512 * 128, 512 * 128, 256 * 8, 3)):
        mu, rho, eps = _w((n,), 300 + i), _w((n,), 400 + i) * 40, _w((n,), 500 + i) * 60
        got.append(pb.reparam(mu, rho, eps))
        want.append(ops.reparam(mu, rho, eps))
    assert len(pb.descs) > 32  # exercises the 32-descriptor split
    pb.run()
    torch.cuda.synchronize()
    for i, (a, b) in enumerate(zip(got, want)):
        assert a.shape == b.shape and torch.equal(a, b), i


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_colsum_batch(dtype):
    shapes = [(65536, 32), (65536, 128), (16384, 256), (4096, 512), (256, 512), (256, 1), (8, 3), (0, 16),
              (1000, 40), (3, 2048)]
    q = ops.ColsumQueue()
    q.active = True
    srcs, outs = [], []
    for i, (R, C) in enumerate(shapes * 4):  # 40 descriptors: two launches
        X = _w((R, C), i).mul(20).to(dtype)
        o = _w((C,), 1000 + i)
        srcs.append((X, o.clone()))
        outs.append(o)
        q.add(X, o, R, C, C)
    q.flush()
    torch.cuda.synchronize()
    for (X, o0), o in zip(srcs, outs):
        ref = (o0.double() + X.double().sum(0)).float()
        tol = 1e-5 * (X.double().abs().sum(0).float() + 1)
        assert ((o - ref).abs() <= tol).all()


def test_colsum_defer_only_inside_a_step():
    X = _w((64, 16), 0)
    o = torch.zeros(16, device=DEV)
    assert not ops.COLSUMS.active
    ops.colsum(X, o, defer=True)  # no step running: immediate
    torch.cuda.synchronize()
    assert torch.allclose(o, X.sum(0), atol=1e-5) and not ops.COLSUMS.items


@pytest.mark.parametrize("T,k,E", [(65536, 2, 8), (4096, 2, 8), (1000, 4, 32), (256, 1, 8), (5, 2, 4)])
def test_moe_dispatch_is_a_stable_sort_by_expert(T, k, E):
    """mg_moe_dispatch: perm = stable argsort of the assignments by expert (assignment order kept inside an
    expert, which the oracle's per-expert index lists follow), its inverse, the gates in dispatch order and the
    row / 128-row tile prefixes."""
    g = torch.Generator(device=DEV).manual_seed(T + E)
    topi = torch.randint(0, E, (T, k), device=DEV, generator=g, dtype=torch.int32)
    if T > 100:
        topi[: T // 3] = 1  # a skewed expert
    gate = torch.rand(T, k, device=DEV, generator=g)
    row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
    flat = topi.reshape(-1).long()
    want = torch.sort(flat, stable=True).indices
    assert torch.equal(perm.long(), want)
    assert torch.equal(pos_of.long()[want], torch.arange(T * k, device=DEV))
    assert torch.equal(gate_pos, gate.reshape(-1)[want])
    cnt = torch.bincount(flat, minlength=E)
    assert torch.equal(row_off.long(), torch.cat([cnt.new_zeros(1), cnt.cumsum(0)]))
    tiles = (cnt + 127) // 128
    assert torch.equal(tile_off.long(), torch.cat([tiles.new_zeros(1), tiles.cumsum(0)]))


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_im2col_4x4s2_matches_unfold(dtype):
    B, C, H = 4, 3, 64
    x = _w((B, C, H, H), 7)
    Kp = 48
    out = ops.im2col_4x4s2(x, (C * H * H, H, 1, H * H), B, H, H, C, Kp, dtype)  # NCHW strides
    cols = torch.nn.functional.unfold(x, 4, padding=1, stride=2)  # [B, C*16, L], index c*16 + kh*4 + kw
    want = cols.view(B, C, 16, -1).permute(0, 3, 2, 1).reshape(B * (H // 2) ** 2, 16 * C)  # (tap, c)
    torch.cuda.synchronize()
    assert torch.equal(out.float(), want.to(dtype).float())


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_const_bwd(dtype):
    B, Hc, C = 256, 4, 512
    gsrc = _w((B, Hc, Hc, C), 9).to(dtype)
    gc = _w((C, Hc * Hc), 10)
    want = gc.double() + gsrc.double().sum(0).permute(2, 0, 1).reshape(C, -1)
    ops.const_bwd(gsrc, gc)
    torch.cuda.synchronize()
    assert torch.allclose(gc.double(), want, atol=1e-5, rtol=1e-5)


@pytest.mark.parametrize("dtype", [torch.bfloat16, torch.float32])
def test_dgrad_s2_small_matches_parity_class_gemms(dtype):
    """The few-channel data gradient (GEMM + mg_col2im_4x4s2) against mg_conv2d_dgrad_s2 on the same operands
    and against torch's conv_transpose2d in float64."""
    B, OH, Cg, Cin = 8, 32, 128, 3
    g = _w((B, OH, OH, Cg), 11).mul(10).to(dtype)
    W = _w((Cg, Cin, 4, 4), 12)
    a = torch.zeros(B, 2 * OH, 2 * OH, 4, device=DEV)
    ops.dgrad_s2_small(g, ops.pack_conv(W, dtype), Cin, a)
    b = torch.zeros(B, 2 * OH, 2 * OH, 4, device=DEV)
    ops.dgrad_s2(g, ops.pack_dgrad_s2(W, dtype, rows=Cin), Cin, b)
    ref = torch.nn.functional.conv_transpose2d(g.double().permute(0, 3, 1, 2), W.to(dtype).double(), stride=2,
                                               padding=1).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    assert (a[..., 3] == 0).all()
    err = (a[..., :3].double() - ref).abs().max().item()
    assert err <= 1e-4 * ref.abs().max().item(), err
    assert (a - b).abs().max().item() <= 1e-4 * ref.abs().max().item()
