"""Drop-in surfaces around the step, on the CPU: the hyperparameter coercion / HPO-config schema
(sagemaker_train.py:85-102, :271-294; configs/hyperparameter_config.json consumed by
scripts/hyperparameter_tuning.py:97-100, :191-209) and the resume-checkpoint layout with torch-format AdamW state
(t2i_moe_gan.py:1484-1491, :1642-1652)."""
import json
import os

import pytest
import torch

from conftest import REPO


def test_coercion_matches_sagemaker_rules():
    from moegan_mi.hparams import coerce_hyperparameters
    raw = {"batch_size": "9", "epochs": "50", "kl_annealing_epochs": "20", "lr_warmup_epochs": "3",
           "learning_rate": "0.00067", "beta1": "0.882", "beta2": "0.939", "r1_gamma": "9.67",
           "clip_weight_16": "0.192", "clip_weight_8": "0.040", "kl_weight": "0.000675", "balance_weight": "0.0065",
           "clip_weight_64": "0.1", "sagemaker_program": "train.py"}
    p = coerce_hyperparameters(raw)
    for k in ("batch_size", "epochs", "kl_annealing_epochs", "lr_warmup_epochs"):
        assert type(p[k]) is int
    for k in ("learning_rate", "beta1", "beta2", "r1_gamma", "clip_weight_16", "clip_weight_8", "kl_weight",
              "balance_weight", "clip_weight_64"):
        assert type(p[k]) is float
    assert p["sagemaker_program"] == "train.py"  # everything else passes through unchanged
    assert p["learning_rate"] == pytest.approx(0.00067)


def test_train_kwargs_mapping_and_defaults():
    from moegan_mi.hparams import given_train_kwargs, train_kwargs, unapplied_keys
    kw = train_kwargs({"learning_rate": 1e-4, "epochs": 6, "clip_weight_64": 0.3})
    assert kw["lr"] == 1e-4 and kw["num_epochs"] == 6 and kw["clip_weight_16"] == 0.3
    assert kw["clip_weight_8"] == 0.05 and kw["r1_gamma"] == 10.0  # sagemaker_train.py:271-294 defaults
    assert kw["gradient_accumulation_steps"] == 8 and kw["max_resolution"] == 16
    assert given_train_kwargs({"kl_weight": 0.002, "clip_weight_32": 0.07}) == {"kl_weight": 0.002,
                                                                                  "clip_weight_8": 0.07}
    # keys that reach neither the loaders nor train_aurora_gan are reported, not dropped silently
    assert unapplied_keys({"batch_size": 4, "kl_weight": 1e-3, "clip_weight_64": 0.1, "sagemaker_program": "x"}) \
        == {"sagemaker_program"}


def test_validation_shard_has_no_padding():
    """Each rank validates indices rank::world, every sample exactly once over the ranks (train_model.py), so the
    all-reduced sums equal the single-process reference's (t2i_moe_gan.py:1519-1639)."""
    from train_model import ShardSampler
    for n, world in ((10, 4), (3, 8), (16, 2)):
        shards = [list(ShardSampler(n, r, world)) for r in range(world)]
        assert sorted(i for sh in shards for i in sh) == list(range(n))
        assert all(len(ShardSampler(n, r, world)) == len(sh) for r, sh in enumerate(shards))


def test_hpo_config_schema():
    from moegan_mi.hparams import load_hpo_config, static_train_kwargs, validate_hpo_config
    cfg = load_hpo_config(os.path.join(REPO, "configs", "hyperparameter_config.json"))
    assert cfg["objective_metric"]["name"] == "val_clip_loss"
    kw = static_train_kwargs(cfg)
    assert kw["num_epochs"] == 6 and kw["clip_weight_16"] == 0.1 and kw["clip_weight_8"] == 0.05
    bad = json.loads(json.dumps(cfg))
    bad["hyperparameter_ranges"]["learning_rate"]["min_value"] = 1.0  # min > max
    with pytest.raises(ValueError, match="min_value > max_value"):
        validate_hpo_config(bad)
    bad = json.loads(json.dumps(cfg))
    bad["static_hyperparameters"]["epochs"] = 6  # SageMaker passes strings
    with pytest.raises(ValueError, match="strings"):
        validate_hpo_config(bad)
    bad = json.loads(json.dumps(cfg))
    bad["integer_parameter_ranges"]["kl_annealing_epochs"]["max_value"] = 4.5
    with pytest.raises(ValueError, match="integer"):
        validate_hpo_config(bad)


def _store(E=4, seed=0):
    from moegan_mi.layout import generator_shapes
    from moegan_mi.params import ParamStore
    st = ParamStore(generator_shapes(E), "cpu", frozen_prefixes=("to_rgb_8.",))
    g = torch.Generator().manual_seed(seed)
    st.data.copy_(torch.randn(st.total, generator=g) * 0.05)
    st.m.copy_(torch.randn(st.total, generator=g) * 1e-3)
    st.v.copy_(torch.rand(st.total, generator=g) * 1e-6)
    st.m[st.n_opt:] = 0
    st.v[st.n_opt:] = 0
    st.step_dev.fill_(7)
    st.step_dev_kl.fill_(5)
    return st


def test_optimizer_state_roundtrip_and_torch_compatibility():
    from moegan_mi.checkpoint import load_optimizer_state_dict, optimizer_state_dict
    from moegan_mi.layout import is_buffer
    st = _store()
    sd = optimizer_state_dict(st, lr=2e-4)
    names = [n for n in st.shapes if not is_buffer(n)]
    # frozen parameters (never stepped) carry no state; the KL parameters their own step count
    for i, n in enumerate(names):
        if n.startswith("to_rgb_8."):
            assert i not in sd["state"]
        elif ".router." in n and n.endswith(("_mu", "_rho")):
            assert float(sd["state"][i]["step"]) == 5.0
        else:
            assert float(sd["state"][i]["step"]) == 7.0
    # a torch AdamW over reference-ordered parameters accepts it
    params = [torch.nn.Parameter(st.view(n).clone()) for n in names]
    opt = torch.optim.AdamW(params, lr=2e-4, betas=(0.5, 0.999), weight_decay=0.01)
    opt.load_state_dict(sd)
    off, numel = st.offsets[names[3]]
    assert torch.equal(opt.state[params[3]]["exp_avg"].reshape(-1), st.m[off:off + numel])
    # and back into a fresh store
    st2 = _store(seed=1)
    load_optimizer_state_dict(st2, opt.state_dict())
    for n in names:
        off, numel = st.offsets[n]
        if off < st.n_opt:
            assert torch.equal(st2.m[off:off + numel], st.m[off:off + numel]), n
            assert torch.equal(st2.v[off:off + numel], st.v[off:off + numel]), n
    assert int(st2.step_dev[0]) == 7 and int(st2.step_dev_kl[0]) == 5


def test_torch_adamw_state_loads_into_store():
    """A reference run's optimizer_g (AdamW over generator.parameters(), one real step) loads exactly."""
    from moegan_mi.checkpoint import load_optimizer_state_dict
    from moegan_mi.layout import generator_shapes, is_buffer
    from moegan_mi.params import ParamStore
    shapes = generator_shapes(4)
    names = [n for n in shapes if not is_buffer(n)]
    params = [torch.nn.Parameter(torch.randn(shapes[n]) * 0.02) for n in names]
    opt = torch.optim.AdamW(params, lr=2e-4, betas=(0.5, 0.999), weight_decay=0.01)
    for n, p in zip(names, params):
        p.grad = None if n.startswith("to_rgb_8.") else torch.randn_like(p)
    opt.step()
    st = ParamStore(shapes, "cpu", frozen_prefixes=("to_rgb_8.",))
    load_optimizer_state_dict(st, opt.state_dict())
    for n, p in zip(names, params):
        off, numel = st.offsets[n]
        s = opt.state.get(p)
        if not s:
            assert float(st.m[off:off + numel].abs().max()) == 0.0
            continue
        assert torch.equal(st.m[off:off + numel], s["exp_avg"].reshape(-1)), n
        assert torch.equal(st.v[off:off + numel], s["exp_avg_sq"].reshape(-1)), n
    assert int(st.step_dev[0]) == 1 and int(st.step_dev_kl[0]) == 1


def test_resume_checkpoint_layout(tmp_path):
    import t2i_moe_gan as M
    G, D = M.AuroraGenerator(seed=3), M.AuroraDiscriminator(seed=4)
    G._store.step_dev.fill_(2)
    G._store.m.normal_()
    path = os.path.join(tmp_path, "ck.pt")
    M.save_resume(path, G, D, epoch=3, step=40, lr_g=1e-4, lr_d=1e-4)
    ck = torch.load(path, weights_only=True)
    # exactly the reference's keys (:1484-1491)
    assert set(ck) == {"generator", "discriminator", "optimizer_g", "optimizer_d", "epoch", "step"}
    G2, D2 = M.AuroraGenerator(seed=5), M.AuroraDiscriminator(seed=6)
    assert M.load_resume(path, G2, D2) == (3, 40)  # a mid-epoch checkpoint resumes that (0-based) epoch
    # an end-of-epoch checkpoint stores epoch + 1 as the reference's does (:1648), resumes at the next epoch and
    # continues the stored random streams
    g = torch.Generator().manual_seed(11)
    torch.randn(5, generator=g)
    M.save_resume(path, G, D, epoch=3, step=40, lr_g=1e-4, lr_d=1e-4, epoch_complete=True,
                  generators={"shared": g})
    assert torch.load(path, weights_only=True)["epoch"] == 4
    expect = torch.randn(4, generator=g)
    g2 = torch.Generator().manual_seed(0)
    assert M.load_resume(path, G2, D2, generators={"shared": g2, "absent": torch.Generator()}) == (4, 40)
    assert torch.equal(torch.randn(4, generator=g2), expect)
    for k, v in G.state_dict().items():
        assert torch.equal(G2.state_dict()[k], v), k
    off, numel = G._store.offsets["mapping.0.weight"]
    assert torch.equal(G2._store.m[off:off + numel], G._store.m[off:off + numel]) and int(G2._store.step_dev[0]) == 2
    # a round-3 file (0-based epoch + epoch_complete flag) still resumes at the next epoch
    ck = torch.load(path, weights_only=True)
    ck.update(epoch=3, epoch_complete=True)
    torch.save(ck, path)
    assert M.load_resume(path, G2, D2)[0] == 4
    # model-only checkpoints (sagemaker_train.py:297-301) and bare generator state dicts load too
    torch.save({"generator": G.state_dict(), "discriminator": D.state_dict()}, path)
    assert M.load_resume(path, G2, D2) == (0, 0)
    torch.save(G.state_dict(), path)
    assert M.load_resume(path, G2, D2) == (0, 0)


def test_prefetcher_passthrough_on_cpu():
    """Without a HIP device the prefetcher hands the loader's batches through unchanged (same objects, order)."""
    from moegan_mi.prefetch import DevicePrefetcher
    batches = [(torch.full((2, 3), float(i)), torch.full((2, 4), -float(i))) for i in range(3)]
    out = list(DevicePrefetcher(batches, "cpu"))
    assert len(out) == 3 and all(a is b for x, y in zip(out, batches) for a, b in zip(x, y))
