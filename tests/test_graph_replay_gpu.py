"""The launch mode bench.py times, at the benchmarked size: the C2 training step (B=256, E=8 top-2, bf16, R1 on)
captured as hipGraphs and replayed on fixed input buffers (steputil.ReplayedStep, the same SegmentedGraph calls as
bench.py), against the same step run eagerly (t2i_moe_gan.py:1262-1421 per step).

* Replay vs eager, deterministic mode (ops.set_deterministic: every cross-workgroup reduction in a fixed order):
  three consecutive steps from one state; every loss value, both gradient vectors and the final parameters and
  AdamW moments of the replay are BIT-IDENTICAL to the eager run's.
* Replay vs eager, default (atomic) mode: the eager step is itself not bit-reproducible, so its run-to-run spread
  is measured by a second eager run from the same state; the first step's losses and gradient vectors of the replay
  sit within REPLAY_X x that spread (plus 1e-6 relative) of the first eager run.  (Later steps are covered by the
  deterministic comparison: after an AdamW step the spread itself is chaotic -- elements whose gradient sign is
  noise move by +-lr.)
* Full-size property check against the fp32 device step (the fp32 mode is pinned to the oracle and the reference
  fixtures at small batches, test_engine_gpu.py): one step from the same state with the learning rates at 0 (so
  the G phase of both runs sees the same discriminator), whole-model clipped gradient cosine >= 0.999 (D) /
  0.98 (G, the bf16 floor analysis of test_step_bf16_gpu.py), every MoE layer's top-2 sets equal wherever the
  fp32 margin log(p_(2)/p_(3)) exceeds DELTA, flips below 10 % of tokens.
The B=8 replay against the oracle itself is test_step_bf16_gpu.py::test_bf16_c2_graph_replay_vs_oracle.
"""
import pytest
import torch

from steputil import ReplayedStep, cosine, rel_norm_diff, restore, routing_agreement, snapshot, step_state

pytestmark = pytest.mark.gpu
DEV = "cuda"
REPLAY_X = 4.0
DELTA = 0.25
E, K, B = 8, 2, 256
KW = dict(anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)


def _model(dtype):
    from moegan_mi.init import init_discriminator, init_generator
    from moegan_mi.step import StepConfig, TrainStep
    ts = TrainStep(StepConfig(E=E, topk=K, dtype=dtype), DEV)
    init_generator(ts.gs, seed=0)
    init_discriminator(ts.ds, seed=1)
    return ts


def _inputs(n):
    from bench import eps_buffers
    g = torch.Generator(device=DEV).manual_seed(11)
    out = []
    for _ in range(n):
        real = torch.rand(B, 3, 64, 64, device=DEV, generator=g) * 2 - 1
        text = torch.randn(B, 512, device=DEV, generator=g)
        z = torch.randn(B, 512, device=DEV, generator=g)
        fd, eps_d = eps_buffers(E, DEV)
        fg, eps_g = eps_buffers(E, DEV)
        fd.normal_(generator=g)
        fg.normal_(generator=g)
        out.append((real, text, z, eps_d, eps_g, torch.randperm(B, device=DEV, generator=g).int()))
    return out


def _record(ts, out):
    torch.cuda.synchronize()
    return dict(scal={k: float(out[k].reshape(-1)[0]) for k in ("d_losses", "r1", "g_gan", "balance", "kl")},
                gg=ts.gs.grad[:ts.gs.n_opt].clone(), dg=ts.ds.grad[:ts.ds.n_opt].clone())


def _replay_vs_eager(nsteps, modes):
    ts = _model("bf16")
    inputs = _inputs(nsteps)
    rs = ReplayedStep(ts, *inputs[0], **KW)
    s0 = snapshot(ts)

    def run(mode):
        restore(ts, s0)
        recs = []
        for inp in inputs:
            out = rs(*inp) if mode == "replay" else ts.step(*inp, **KW)
            assert int(out["flags"][0]) == 0
            recs.append(_record(ts, out))
        return recs, [t.clone() for t in step_state(ts)]
    return [run(m) for m in modes]


def test_c2_graph_replay_bit_identical_deterministic_full_size():
    from moegan_mi import ops
    ops.set_deterministic(True)
    try:
        (eager, eager_p), (rep, rep_p) = _replay_vs_eager(3, ("eager", "replay"))
    finally:
        ops.set_deterministic(False)
    for si, (a, r) in enumerate(zip(eager, rep)):
        for key in a["scal"]:
            assert a["scal"][key] == r["scal"][key], (si, key, a["scal"][key], r["scal"][key])
        for key in ("gg", "dg"):
            assert torch.equal(a[key], r[key]), (si, key, float((a[key] - r[key]).abs().max()))
    for x, y in zip(eager_p, rep_p):
        assert torch.equal(x, y)
    print("3 replayed steps bit-identical to 3 eager steps (losses, gradients, parameters, moments)")


def test_c2_graph_replay_matches_eager_full_size():
    (eager, eager_p), (eager2, eager2_p), (rep, rep_p) = _replay_vs_eager(1, ("eager", "eager", "replay"))
    report, fails = [], []
    for si in range(len(eager)):
        a, a2, r = eager[si], eager2[si], rep[si]
        for key in a["scal"]:
            noise = abs(a2["scal"][key] - a["scal"][key])
            err = abs(r["scal"][key] - a["scal"][key])
            report.append(f"step{si} {key}: replay {r['scal'][key]:.7e} eager {a['scal'][key]:.7e} (|diff| {err:.2e}, "
                          f"eager spread {noise:.2e})")
            if err > REPLAY_X * noise + 1e-6 * abs(a["scal"][key]):
                fails.append(report[-1])
        for key in ("gg", "dg"):
            noise, err = rel_norm_diff(a2[key], a[key]), rel_norm_diff(r[key], a[key])
            report.append(f"step{si} {key}: replay rel err {err:.2e} (eager spread {noise:.2e})")
            if err > REPLAY_X * noise + 1e-6:
                fails.append(report[-1])
    print("\n".join(report))
    assert not fails, fails


def test_c2_full_size_bf16_vs_fp32_device():
    ts, tf = _model("bf16"), _model("fp32")
    inp = _inputs(1)[0]
    kw = dict(KW, lr_g=0.0, lr_d=0.0)  # both G phases see the same (unchanged) discriminator
    ob = ts.step(*inp, **kw)
    of = tf.step(*inp, **kw)
    torch.cuda.synchronize()
    report, fails = [], []
    for which, sb, sf, bar in (("D", ts.ds, tf.ds, 0.999), ("G", ts.gs, tf.gs, 0.98)):
        c = cosine(sb.grad[:sb.n_opt], sf.grad[:sf.n_opt])
        report.append(f"{which}: whole-model gradient cosine bf16 vs fp32 {c:.6f} (rel {rel_norm_diff(sb.grad[:sb.n_opt], sf.grad[:sf.n_opt]):.2e})")
        if c < bar:
            fails.append(report[-1])
    for tag, tb, pb, pf in (("D", ob["topi_d"], ob["probs_d"], of["probs_d"]), ("G", ob["topi"], ob["probs"], of["probs"])):
        for li in range(3):
            a = routing_agreement(tb[li], pb[li], pf[li], K, DELTA)
            report.append(f"{tag}-phase layer{li}: {a['n']} tokens, {a['mismatch']} top-{K} set mismatches, {a['near']} "
                          f"near-ties, outside them {a['bad']}, max margin drift {a['drift']:.4f}")
            if a["self_mismatch"] or a["bad"] or a["mismatch"] > a["n"] // 10:
                fails.append(report[-1])
    for key in ("d_losses", "r1", "g_gan", "balance"):
        x, y = float(ob[key].reshape(-1)[0]), float(of[key].reshape(-1)[0])
        report.append(f"{key}: bf16 {x:.6f} fp32 {y:.6f}")
        if abs(x - y) > 2e-2 * max(abs(y), 1e-6):
            fails.append(report[-1])
    print("\n".join(report))
    assert not fails, fails
