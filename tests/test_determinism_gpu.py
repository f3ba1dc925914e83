"""Deterministic mode (atomics-free backward variants behind one flag, ops.set_deterministic /
StepConfig(deterministic=True) / MOEGAN_DETERMINISTIC=1): two identically initialised bf16 training steps on the same
inputs give bit-identical gradients, parameters and logged losses.  Run at B=8 (the parity tests' size) and at the
benchmarked B=256, where the split-K and multi-block reductions that use fp32 atomics in the default mode are
active.  The default (atomic) mode is checked to agree with the deterministic one to fp32 summation-order noise."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _one_step(B, det, seed=7, res=64):
    import bench
    from moegan_mi.init import init_discriminator, init_generator
    from moegan_mi.step import StepConfig, TrainStep
    E, k = 8, 2
    ts = TrainStep(StepConfig(E=E, topk=k, dtype="bf16", deterministic=det, max_res=16 if res == 64 else res), DEV)
    init_generator(ts.gs, seed=0)
    init_discriminator(ts.ds, seed=1)
    g = torch.Generator(device=DEV).manual_seed(seed)
    real = torch.rand(B, 3, res, res, device=DEV, generator=g) * 2 - 1
    text = torch.randn(B, 512, device=DEV, generator=g)
    z = torch.randn(B, 512, device=DEV, generator=g)
    fd, eps_d = bench.eps_buffers(E, DEV)
    fg, eps_g = bench.eps_buffers(E, DEV)
    fd.normal_(generator=g)
    fg.normal_(generator=g)
    perm = torch.randperm(B, device=DEV, generator=g).int()
    out = ts.step(real, text, z, eps_d, eps_g, perm, anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)
    torch.cuda.synchronize()
    scal = {n: out[n].detach().float().cpu().clone() for n in ("d_losses", "r1", "g_gan", "balance", "kl",
                                                                  "g_grad_sumsq", "d_grad_sumsq")}
    state = {f"{w}:{n}": st.gview(n).detach().cpu().clone() for w, st in (("G", ts.gs), ("D", ts.ds))
             for n in st.offsets}
    params = torch.cat([ts.gs.data.cpu(), ts.ds.data.cpu()])
    return scal, state, params


@pytest.mark.parametrize("B", [8, 256])
def test_deterministic_mode_bit_identical(B):
    from moegan_mi import ops
    try:
        a = _one_step(B, True)
        b = _one_step(B, True)
    finally:
        ops.set_deterministic(False)
    bad_s = [n for n in a[0] if not torch.equal(a[0][n], b[0][n])]
    bad_g = [n for n in a[1] if not torch.equal(a[1][n], b[1][n])]
    print(f"B={B}: scalars differing {bad_s}; gradient tensors differing {len(bad_g)}/{len(a[1])} {bad_g[:8]}")
    assert not bad_s and not bad_g
    assert torch.equal(a[2], b[2])


def test_deterministic_mode_matches_default_mode():
    from moegan_mi import ops
    try:
        d = _one_step(8, True)
    finally:
        ops.set_deterministic(False)
    n = _one_step(8, False)
    for k in d[0]:
        assert torch.allclose(d[0][k], n[0][k], rtol=1e-4, atol=1e-7), (k, d[0][k], n[0][k])
    g_d = torch.cat([v.reshape(-1) for v in d[1].values()]).double()
    g_n = torch.cat([v.reshape(-1) for v in n[1].values()]).double()
    assert float((g_d - g_n).norm() / g_n.norm()) < 1e-3


def test_deterministic_mode_multi_logit_fakes():
    """Deterministic mode with the progressive generator at 32^2 (real and fake images 32x32, so the D loss sees
    Nf = 25 logits per fake image and k_d_loss runs 2B+1 blocks): the logged D losses agree with the default
    (atomic) mode -- block B, idle when Nf > 1, still writes its (zero) partial row for the fixed-order fold
     -- and two deterministic steps are bit-identical."""
    from moegan_mi import ops
    try:
        a = _one_step(4, True, res=32)
        b = _one_step(4, True, res=32)
    finally:
        ops.set_deterministic(False)
    n = _one_step(4, False, res=32)
    for k in a[0]:
        assert torch.equal(a[0][k], b[0][k]), k
        assert torch.allclose(a[0][k], n[0][k], rtol=1e-4, atol=1e-7), (k, a[0][k], n[0][k])
    assert torch.isfinite(a[0]["d_losses"]).all()
