"""Edge cases of the whole step in fp32 parity mode against the CPU oracle (oracle.train_step): a single image
(B = 1: the mismatched pair is the image with its own caption, R1 and balance over one image, most experts of
the 4x4 block receive no token) and an odd batch (B = 3: ragged last tiles in every GEMM / implicit conv, token
counts 48 / 192 / 768 that are not multiples of the 64-row expert tiles), E = 8 top-2 (the benchmarked routing)
and E = 4 dense.

The device's top-k selections are replayed into the oracle (as test_step_bf16_gpu.py does) after checking that
they agree with the oracle's own fp32 selection away from near-ties.  Bars are the full-step fp32 bars of F8 /
the progressive step (test_progressive_gpu.py): losses 1e-4 relative (balance 1e-3), 2e-3 relative L2 per
discriminator gradient tensor, 5e-3 per generator tensor (1e-2 for the batch-summed style / offset-head
parameters), max-abs within 4x that of the tensor's scale, and 2e-2 on |g|-weighted AdamW deltas.
"""
import pytest
import torch

from oracle import aurora_cpu as O
from steputil import gpu_step, make_inputs, oracle_models, routing_agreement
from test_progressive_gpu import _tensor_close

pytestmark = pytest.mark.gpu
DEV = "cuda"
torch.set_num_threads(8)


@pytest.mark.parametrize("B,E,k", [(1, 8, 2), (3, 8, 2), (3, 4, None)])
def test_step_edge_batches_vs_oracle(B, E, k):
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=900 + B * 10 + E)
    ts = gpu_step(E, k, "fp32")
    g0, d0 = ts.gs.data.clone(), ts.ds.data.clone()
    dv = lambda trips: [tuple(t.to(DEV) for t in trip) for trip in trips]  # noqa: E731
    out = ts.step(real.to(DEV), text.to(DEV), z.to(DEV), dv(eps_d), dv(eps_g), perm.int().to(DEV), anneal=3.0,
                  eff_kl_weight=1e-8)
    torch.cuda.synchronize()
    assert int(out["flags"][0]) == 0
    PG, PD, optG, optD, grads = oracle_models(E)
    gb = {n: v.detach().clone() for n, v in PG.items()}
    db = {n: v.detach().clone() for n, v in PD.items()}
    routes = {}
    if k is not None:
        routes = dict(routes_d=[t.cpu().long() for t in out["topi_d"]], routes_g=[t.cpu().long() for t in out["topi"]])
    ref = O.train_step(PG, PD, optG, optD, real, text, z, eps_d, eps_g, perm, topk=k, kl_weight_eff=1e-8,
                       full=True, **routes)
    assert not ref["skipped"]
    if k is not None:  # the replayed selections are the oracle's own away from near-ties (fp32: drift ~1e-5)
        for i, (ti, pd) in enumerate(zip(out["topi"], out["probs"])):
            ra = routing_agreement(ti, pd, ref["probs"][i], k, 1e-3)
            assert ra["self_mismatch"] == 0 and ra["bad"] == 0, (i, ra)
    assert abs(float(out["d_losses"][0]) - ref["d_loss_gan"]) <= 1e-4 * abs(ref["d_loss_gan"])
    assert abs(float(out["r1"][0]) - ref["r1"]) <= 1e-4 * abs(ref["r1"]) + 1e-7
    assert abs(float(out["g_gan"][0]) - ref["g_loss_gan"]) <= 1e-4 * abs(ref["g_loss_gan"])
    assert abs(float(out["balance"][0]) - ref["balance"]) <= 1e-3 * ref["balance"] + 1e-7
    n_checked = 0
    for which, store, before, P, P0, max_norm in (("D", ts.ds, d0, PD, db, 0.7), ("G", ts.gs, g0, PG, gb, 0.8)):
        gn = float(store.grad[:store.n_opt].double().norm())
        coef = min(1.0, max_norm / (gn + 1e-6))
        for n, (off, numel) in store.offsets.items():
            if n.split(".")[-1].startswith("epsilon_"):
                continue
            shape = store.shapes[n]
            gref = grads[which].get(n)
            if gref is None:  # to_rgb_8: feeds only the gradient-free CLIP loss; AdamW skips it (F8)
                assert off >= store.n_opt, n
                assert torch.equal(store.data[off:off + numel], before[off:off + numel]), n
                continue
            tol = 2e-3 if which == "D" else (1e-2 if (".modulation." in n or ".offset_net." in n) else 5e-3)
            _tensor_close((store.grad[off:off + numel] * coef).view(shape), gref, tol, 1e-8, f"{which} grad {n}",
                          rtol_max=4 * tol)
            delta = (store.data[off:off + numel] - before[off:off + numel]).view(shape)
            wgt = gref.detach().double().abs().reshape(shape)
            _tensor_close(delta.double() * wgt.to(delta.device), (P[n].detach() - P0[n]).double() * wgt, 2e-2, 0.0,
                          f"{which} |g|-weighted delta {n}", maxabs=False)
            n_checked += 1
    assert n_checked > 200


@pytest.mark.parametrize("n", [1, 256, 4095, 215296, 1048577])
def test_g_loss_sizes(n):
    """mg_g_loss (softplus(-f).mean(), t2i_moe_gan.py:917-924, and its gradient) from one logit up to the multi-block
    fold of the progressive stages' per-patch fakes (B x 841 at 128^2); two calls give the same bits."""
    from moegan_mi import ops
    f = torch.randn(n, generator=torch.Generator().manual_seed(n)) * 4
    fd = f.to(DEV)
    out, g = torch.zeros(1, device=DEV), torch.empty(n, device=DEV)
    ops.g_loss(fd, out, g, 0.5)
    out2, g2 = torch.zeros(1, device=DEV), torch.empty(n, device=DEV)
    ops.g_loss(fd, out2, g2, 0.5)
    torch.cuda.synchronize()
    ref = torch.nn.functional.softplus(-f.double()).mean()
    gref = -torch.sigmoid(-f.double()) / n * 0.5
    assert abs(float(out) - float(ref)) <= 1e-5 * float(ref)
    assert float((g.cpu().double() - gref).abs().max()) <= 1e-6 * float(gref.abs().max())
    assert torch.equal(out, out2) and torch.equal(g, g2)
