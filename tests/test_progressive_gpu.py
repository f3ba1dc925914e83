"""Progressive generator extension (BASELINE config C4) on the GPU, fp32 parity mode.

The reference defines no block above 16x16 (gen_block_32 / _64 appear only in the dead
create_optimizer_for_active_blocks, t2i_moe_gan.py:1005-1026), so the block list is the build's
(moegan_mi/layout.py gen_blocks) and this parity is "unpinned" against the reference: both sides compose the
same pinned reference functions (upsample :657, ConvolutionBlock :604-621 with MTMs that have no offset head
above 16x16, :199, ModulatedConv to_rgb :154-186), the oracle in plain PyTorch autograd
(oracle/aurora_cpu.generator), the device through the HIP engines.  The MTM LeakyReLU slopes the device took are
replayed in the oracle (steputil.lrelu_slope_replay, like the top-k routes): a pre-activation within rounding of
0 on the other slope moves a whole data gradient by ~4e-3 (measured, tools/gen_grad_probe.py).  The oracle runs in fp64: in fp32 its own CPU
grid_sample / conv backward reorderings were measured at up to 5e-3 of a gradient's scale (tools/diag_cb.py), so
an fp32 oracle cannot hold an fp32 device to F8's bars.  Bars are the fp32 ones of F7 / F8: 1e-4 relative on
values, 1e-3 on the generator's gradients for a given upstream gradient; for the full step 2e-3 relative L2 and
2e-3 of the tensor's scale max-abs per gradient tensor (discriminator and generator alike), 2e-2 on |g|-weighted
AdamW deltas.  Covered stages: 32^2, 64^2 and 128^2 (the C4 stage: generator, discriminator and R1 on 128^2
images).
"""
import pytest
import torch

from goldens import close
from oracle import aurora_cpu as O
from oracle.recipe import fill_state
from steputil import gpu_step, lrelu_slope_replay, make_inputs, nchw, oracle_models

pytestmark = pytest.mark.gpu
DEV = "cuda"
torch.set_num_threads(8)


def _tensor_errors(actual, expected):
    """(relative L2 error, max-abs error / max |expected|) of one tensor."""
    a = actual.detach().double().cpu().reshape(-1)
    e = expected.detach().double().cpu().reshape(-1)
    return (float((a - e).norm() / max(float(e.norm()), 1e-30)),
            float((a - e).abs().max()) / max(float(e.abs().max()), 1e-30))


def _tensor_close(actual, expected, rtol, atol, what, maxabs=True, rtol_max=None):
    """The full-step bar of F8 (test_engine_gpu._train_replay): relative L2 error <= rtol over the whole tensor,
    plus max-abs error within rtol_max (default rtol) of the tensor's scale.  (Per-element bars do not hold for the modulation-weight
    gradients after a full step: they are sums over the batch of cancelling terms, so an element at 1/3 of the
    tensor's RMS can carry a few % fp32 reordering error while the tensor as a whole agrees to 1e-4.)"""
    a = actual.detach().double().cpu().reshape(-1)
    e = expected.detach().double().cpu().reshape(-1)
    err = float((a - e).abs().max())
    scale = float(e.abs().max())
    rm = rtol if rtol_max is None else rtol_max
    assert not maxabs or err <= atol + rm * scale, f"{what}: max abs err {err:.3e} (scale {scale:.3e})"
    rel = float((a - e).norm() / max(float(e.norm()), 1e-30))
    assert rel <= rtol or err <= atol, f"{what}: relative L2 error {rel:.3e}"


def _nhwc_pad(x):
    B, C, H, W = x.shape
    out = torch.zeros(B, H, W, 8, device=DEV)
    out[..., :C] = x.permute(0, 2, 3, 1).to(DEV)
    return out


@pytest.mark.parametrize("R", [32, 64, 128])
def test_progressive_generator_fwd_bwd(R):
    from moegan_mi.engine_g import GeneratorEngine
    from moegan_mi.layout import frozen_rgb_prefixes, generator_shapes
    from moegan_mi.params import ParamStore
    E, B = 4, 2
    shapes = generator_shapes(E, R)
    vals = fill_state(shapes, 0)
    st = ParamStore(shapes, DEV, frozen_prefixes=frozen_rgb_prefixes(R))
    st.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    ge = GeneratorEngine(st, E)
    assert ge.max_res == R and ge.attn_blocks == ["gen_block_4", "gen_block_8", "gen_block_16"]
    ge.prep()
    g = torch.Generator().manual_seed(R)
    z, text = torch.randn(B, 512, generator=g), torch.randn(B, 512, generator=g)
    eps = [tuple(torch.randn(s, generator=g) for s in ((c, 128), (512, 128), (256, E))) for c in (512, 256, 128)]
    P = {n: torch.from_numpy(v).double().requires_grad_(not n.split(".")[-1].startswith("epsilon_"))
         for n, v in vals.items()}
    epsd = [tuple(t.to(DEV) for t in trip) for trip in eps]
    with lrelu_slope_replay() as slopes:  # the device's LeakyReLU slopes, replayed in the oracle (steputil)
        im, ih, kl2s, pr, _, ctx = ge.forward(z.to(DEV), text.to(DEV), epsd, 3.0, 0.7, train=True, save=True,
                                              want_img8=True)
    with slopes.oracle():
        img, img_half, kl, probs = O.generator(z.double(), text.double(), P, [tuple(t.double() for t in e) for e in eps],
                                               True, 3.0, 0.7)
    assert img.shape == (B, 3, R, R) and img_half.shape == (B, 3, R // 2, R // 2)
    R_img = torch.randn(img.shape, generator=g)
    R_half = torch.randn(img_half.shape, generator=g)
    Rp = [torch.randn(p.shape, generator=g) * 1e-2 for p in probs]
    loss = ((img * R_img.double()).sum() + (img_half * R_half.double()).sum() + 0.37 * kl +
            sum((p * r.double()).sum() for p, r in zip(probs, Rp)))
    loss.backward()

    close(nchw(im), img.detach(), rtol=1e-4, what="img")
    close(nchw(ih), img_half.detach(), rtol=1e-4, what="img_half")
    kl2 = torch.stack(kl2s)
    close(kl2[:, 0].sum(), kl.detach(), rtol=1e-5, what="kl")
    for i in range(3):
        close(pr[i], probs[i].detach(), rtol=1e-4, what=f"probs{i}")
    ge.backward(ctx, _nhwc_pad(R_img), kl_coef=(0.37 * kl2[:, 1]).contiguous(), g_probs=[r.to(DEV) for r in Rp],
                g_img8=_nhwc_pad(R_half))
    torch.cuda.synchronize()
    n_checked = 0
    for n, t in P.items():
        if not t.requires_grad:
            continue
        if t.grad is None:  # the unused lower to_rgb layers: frozen tail, gradient stays zero
            assert n.startswith(frozen_rgb_prefixes(R)), n
            assert float(st.gview(n).abs().max()) == 0.0, n
            continue
        close(st.gview(n), t.grad, rtol=1e-3, atol=1e-7, what=n)
        n_checked += 1
    assert n_checked > 200


@pytest.mark.parametrize("R,B", [(16, 2), (32, 2), (128, 1)])
def test_progressive_train_step(R, B):
    """One full fp32 G+D step at R x R (real and fake images R x R: multi-logit fakes in the D and G losses; at
    128 the C4 stage's discriminator and R1 double backward on 128^2 images) vs the fp64 oracle's train_step:
    losses, the R1 input gradient, clipped gradients and AdamW deltas of every tensor."""
    E = 4
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=7, res=R)
    PG, PD, optG, optD, grads = oracle_models(E, max_res=R, dtype=torch.float64)
    gb = {n: v.detach().clone() for n, v in PG.items()}
    db = {n: v.detach().clone() for n, v in PD.items()}
    ts = gpu_step(E, None, "fp32", max_res=R)
    g0, d0 = ts.gs.data.clone(), ts.ds.data.clone()
    dv = lambda trips: [tuple(t.to(DEV) for t in trip) for trip in trips]  # noqa: E731
    with lrelu_slope_replay() as slopes:  # the device's LeakyReLU slopes, replayed in the oracle (steputil)
        out = ts.step(real.to(DEV), text.to(DEV), z.to(DEV), dv(eps_d), dv(eps_g), perm.int().to(DEV), anneal=3.0,
                      eff_kl_weight=1e-8)
        torch.cuda.synchronize()
    d64 = lambda trips: [tuple(t.double() for t in trip) for trip in trips]  # noqa: E731
    with slopes.oracle():
        ref = O.train_step(PG, PD, optG, optD, real.double(), text.double(), z.double(), d64(eps_d), d64(eps_g),
                           perm, kl_weight_eff=1e-8)
    assert not ref["skipped"]
    assert abs(float(out["d_losses"][0]) - ref["d_loss_gan"]) < 1e-4 * abs(ref["d_loss_gan"])
    assert abs(float(out["r1"][0]) - ref["r1"]) < 1e-4 * abs(ref["r1"]) + 1e-7
    assert abs(float(out["g_gan"][0]) - ref["g_loss_gan"]) < 1e-4 * abs(ref["g_loss_gan"])
    assert abs(float(out["balance"][0]) - ref["balance"]) < 1e-3 * ref["balance"] + 1e-7
    assert out["fake_pred"].numel() == B * (R // 4 - 3) ** 2
    # the R1 input gradient d sum D(real) / d real (:1282-1284), every pixel
    _tensor_close(out["r1_grad"][..., :3].permute(0, 3, 1, 2), ref["r1_grad"], 1e-4, 1e-9, "r1_grad")
    fails, rows = [], []
    for which, store, before, P, P0, max_norm in (("D", ts.ds, d0, PD, db, 0.7), ("G", ts.gs, g0, PG, gb, 0.8)):
        gn = float(store.grad[:store.n_opt].double().norm())
        coef = min(1.0, max_norm / (gn + 1e-6))
        for n, (off, numel) in store.offsets.items():
            if n.split(".")[-1].startswith("epsilon_"):
                continue
            shape = store.shapes[n]
            gref = grads[which].get(n)
            if gref is None:
                assert off >= store.n_opt, n  # frozen tail: never stepped
                assert torch.equal(store.data[off:off + numel], before[off:off + numel]), n
                continue
            g = (store.grad[off:off + numel] * coef).view(shape)
            rows.append(_tensor_errors(g, gref) + (f"{which} grad {n}",))
            try:
                _tensor_close(g, gref, 2e-3, 1e-8, f"{which} grad {n}")
            except AssertionError as e:
                fails.append(str(e))
            delta = (store.data[off:off + numel] - before[off:off + numel]).view(shape)
            # first AdamW step: ~lr * sign(g) per element, so elements whose gradient is ~0 flip freely (|err| 2 lr,
            # e.g. the batch-summed modulation-weight gradients): the delta error is weighted by the oracle's |g|,
            # as the bf16 step test does (test_step_bf16_gpu.py)
            wgt = gref.detach().double().abs().reshape(shape)
            try:
                _tensor_close(delta.double() * wgt.to(delta.device), (P[n].detach() - P0[n]).double() * wgt, 2e-2,
                              0.0, f"{which} |g|-weighted delta {n}", maxabs=False)
            except AssertionError as e:
                fails.append(str(e))
    rows.sort(reverse=True)
    print("worst gradient errors (rel L2, max-abs / scale):\n" +
          "\n".join(f"  {r:.2e} {m:.2e} {n}" for r, m, n in rows[:8]))
    assert not fails, fails
    assert out["img16"].shape[1] == R
