"""The training loop's loss guards on the device (t2i_moe_gan.py:1315-1320, :1367-1376, :1396-1404), fp32 mode,
against the CPU oracle that keeps the reference's host-side checks:
  * a NaN in the real batch makes the discriminator loss non-finite: the batch is skipped (no parameter, moment
    or step counter changes anywhere);
  * a NaN in the G-phase router noise makes only the generator loss non-finite: the D step is normal, the
    generator loss is replaced by 0 so only the routers' KL parameters receive a gradient (and a step), every
    other generator parameter is untouched (torch's AdamW skips a None gradient);
  * with gradient_accumulation_steps=2 the same NaN in the second batch keeps the first batch's generator
    gradient (the window still steps every generator parameter) -- the reference's accumulation semantics.
Tolerances: fp32 AdamW deltas (each ~lr * sign(g)), cosine >= 0.9999 and relative norm error <= 1e-2 (F8 / F10
compare deltas at 2e-2)."""
import pytest
import torch

from oracle import aurora_cpu as O
from steputil import cosine, gpu_step, make_inputs, oracle_models, rel_norm_diff

pytestmark = pytest.mark.gpu
DEV = "cuda"
EFF_KL = 0.001 * 1e-5
torch.set_num_threads(8)


def _state(ts):
    return {k: t.clone() for k, t in (("gd", ts.gs.data), ("gm", ts.gs.m), ("gv", ts.gs.v), ("dd", ts.ds.data),
                                      ("dm", ts.ds.m), ("dv", ts.ds.v), ("gs", ts.gs.step_dev),
                                      ("gk", ts.gs.step_dev_kl), ("ds", ts.ds.step_dev))}


def _step(ts, inp, **kw):
    real, text, z, eps_d, eps_g, perm = inp
    cu = lambda t: t.to(DEV)  # noqa: E731
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, eff_kl_weight=EFF_KL, **kw)
    torch.cuda.synchronize()
    return out


def _compare_deltas(store, before, P, pbefore, which):
    for n, (off, numel) in store.offsets.items():
        dd = (store.data[off:off + numel] - before[off:off + numel]).cpu()
        rd = (P[n].detach() - pbefore[n]).reshape(-1)
        if float(rd.abs().max()) == 0.0:
            assert float(dd.abs().max()) == 0.0, (which, n, "moved on the device only")
            continue
        assert cosine(dd, rd) >= 0.9999 and rel_norm_diff(dd, rd) <= 1e-2, (which, n, cosine(dd, rd))


def test_nan_discriminator_loss_skips_batch():
    E, B = 4, 2
    ts = gpu_step(E, None, "fp32", DEV)
    _step(ts, make_inputs(B, E, seed=1))  # one normal step first: moments and counters are non-trivial
    inp = list(make_inputs(B, E, seed=2))
    inp[0] = inp[0].clone()
    inp[0][1, 2, 5, 7] = float("nan")
    before = _state(ts)
    out = _step(ts, inp)
    assert int(out["flags"][0]) & 1
    after = _state(ts)
    for k in before:
        assert torch.equal(before[k], after[k]), k
    PG, PD, optG, optD, _ = oracle_models(E)
    r = O.train_step(PG, PD, optG, optD, *inp[:5], inp[5].long(), kl_weight_eff=EFF_KL)
    assert r["skipped"]


@pytest.mark.parametrize("acc", [1, 2])
def test_nan_generator_loss_keeps_only_kl(acc):
    E, B = 4, 2
    ts = gpu_step(E, None, "fp32", DEV)
    PG, PD, optG, optD, _ = oracle_models(E)
    batches = [list(make_inputs(B, E, seed=10 + i)) for i in range(acc)]
    bad = batches[-1]
    bad[4] = [tuple(t.clone() for t in e) for e in bad[4]]
    bad[4][0][0][3, 5] = float("nan")  # G-phase router noise of gen_block_4 only
    g0, d0 = ts.gs.data.clone(), ts.ds.data.clone()
    pg0 = {n: v.detach().clone() for n, v in PG.items()}
    pd0 = {n: v.detach().clone() for n, v in PD.items()}
    for bi, inp in enumerate(batches):
        last = bi == acc - 1
        out = _step(ts, inp, acc=acc, zero_grads=bi == 0, step_optim=last)
        r = O.train_step(PG, PD, optG, optD, *inp[:5], inp[5].long(), kl_weight_eff=EFF_KL, acc=acc,
                         zero_grads=bi == 0, step_optim=last)
        assert not r["skipped"]
        assert r["g_zeroed"] == last
        assert (int(out["flags"][0]) == 2) == last
    _compare_deltas(ts.ds, d0, PD, pd0, "D")
    _compare_deltas(ts.gs, g0, PG, pg0, "G")
    if acc == 1:  # only the KL range moved, with its own step counter
        n_main = ts.gs.n_main
        assert torch.equal(ts.gs.data[:n_main], g0[:n_main])
        assert int(ts.gs.step_dev[0]) == 0 and int(ts.gs.step_dev_kl[0]) == 1
    else:
        assert int(ts.gs.step_dev[0]) == 1 and int(ts.gs.step_dev_kl[0]) == 1
