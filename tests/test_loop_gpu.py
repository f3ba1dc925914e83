"""The drop-in training loop (train_aurora_gan, t2i_moe_gan.py:1214-1421 per batch) runs the benchmarked launch
mode: every batch body a replayed hipGraph (t2i_moe_gan._StepRunner), the guard word and logged losses read one
batch late.  Checked against the same loop run eagerly from the same seed, C2 configuration (E=8 top-2, bf16) at
B=8, with gradient accumulation (acc=2: the four window positions capture two graph variants and replay them):
the final generator / discriminator parameters after four batches sit within REPLAY_X x the eager loop's own
run-to-run spread (fp32 atomics in some backward reductions) plus 1e-6 relative."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
REPLAY_X = 4.0


def _loader(B=8, n=4, seed=3):
    g = torch.Generator().manual_seed(seed)
    imgs = (torch.rand(B * n, 3, 64, 64, generator=g) * 2 - 1).pin_memory()
    text = torch.randn(B * n, 512, generator=g).pin_memory()
    return [(imgs[i:i + B], text[i:i + B]) for i in range(0, B * n, B)]


def _train(use_graphs, tmp_path, acc=2, B=8, n=4):
    import t2i_moe_gan as M
    seen = []
    G, D = M.train_aurora_gan(_loader(B, n), num_epochs=1, lr=2e-4, gradient_accumulation_steps=acc,
                              checkpoint_activation=False, num_experts=8, topk=2, dtype="bf16", seed=0,
                              save_dir=str(tmp_path), log_interval=1, device=DEV, use_graphs=use_graphs,
                              on_batch_done=lambda e, b, f: seen.append(b))
    torch.cuda.synchronize()
    assert seen == list(range(n))
    return G._store.data.clone(), D._store.data.clone()


def test_graph_loop_bit_identical_deterministic(tmp_path, caplog):
    """Deterministic mode: the graph-replayed loop's parameters equal the eager loop's bit for bit, and so do the
    per-batch losses it reads back (logged every batch), across the window's variant switches -- a variant's outputs
    are read before another variant replays (the _StepRunner invariant: the variants share one graph pool)."""
    import logging
    from moegan_mi import ops
    caplog.set_level(logging.INFO, logger="t2i_moe_gan")
    logs = {}
    ops.set_deterministic(True)
    try:
        for mode in (False, True):
            caplog.clear()
            res = _train(mode, tmp_path)
            logs[mode] = [r.getMessage().strip() for r in caplog.records if "D_loss" in r.getMessage()]
            if mode:
                g = res
            else:
                e = res
    finally:
        ops.set_deterministic(False)
    assert torch.equal(e[0], g[0]) and torch.equal(e[1], g[1])
    assert len(logs[False]) == 4, logs[False]
    assert logs[True] == logs[False], (logs[True], logs[False])


def test_graph_loop_matches_eager_loop(tmp_path):
    e1 = _train(False, tmp_path)
    e2 = _train(False, tmp_path)
    g = _train(True, tmp_path)
    rel = lambda a, b: float((a.double() - b.double()).norm() / b.double().norm())  # noqa: E731
    for i, name in enumerate(("generator", "discriminator")):
        noise, err = rel(e2[i], e1[i]), rel(g[i], e1[i])
        print(f"{name}: graph-loop rel err {err:.3e}, eager loop spread {noise:.3e}")
        assert err <= REPLAY_X * noise + 1e-6, (name, err, noise)


def test_graph_loop_peak_memory_acc8(tmp_path):
    """The reference's default window (gradient_accumulation_steps=8, :1043) makes the loop capture three variants
    (window start / middle / end).  They share one capture stream and one graph pool (t2i_moe_gan._StepRunner), so
    the replayed loop's peak allocated memory stays near the eager loop's instead of growing with the variant
    count."""
    import gc
    B, n = 64, 8
    peaks = {}
    for mode in (False, True):
        gc.collect()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        _train(mode, tmp_path, acc=8, B=B, n=n)
        peaks[mode] = (torch.cuda.max_memory_allocated() - base) / 2 ** 20
    print(f"acc=8, B={B}: peak allocated above baseline: eager loop {peaks[False]:.0f} MiB, "
          f"graph-replayed loop (3 variants) {peaks[True]:.0f} MiB")
    assert peaks[True] <= 1.5 * peaks[False] + 64, peaks
