"""Checkpoint I/O in the reference's layouts.

* Model-only (sagemaker_train.py:297-301, read by inference.py:34-49 / generate_images.py:37-40):
  ``{'generator': G.state_dict(), 'discriminator': D.state_dict()}``.
* Resume (t2i_moe_gan.py:1484-1491 and :1642-1652, commented out in the reference):
  ``{'generator', 'discriminator', 'optimizer_g', 'optimizer_d', 'epoch', 'step'}`` where the optimizer entries
  are ``torch.optim.AdamW.state_dict()`` of an AdamW built over ``module.parameters()`` -- parameter indices in
  the reference's registration order, per-parameter ``step`` / ``exp_avg`` / ``exp_avg_sq``, parameters never
  stepped (no gradient yet, e.g. to_rgb_8) without state.  A reference run's resume file loads here, and ours
  loads into the reference's optimizer.

The flat stores keep the AdamW moments in ``store.m`` / ``store.v`` and the step counts on the device
(``step_dev`` for the main range, ``step_dev_kl`` for the routers' KL parameters, see params.py); this module
converts between that and torch's per-parameter format.  Loading uses ``torch.load(weights_only=True)``.
"""
import torch

from .layout import is_buffer


def _param_names(store):
    return [n for n in store.shapes if not is_buffer(n)]


def _step_of(store, name):
    off, _ = store.offsets[name]
    if off >= store.n_opt:
        return 0  # frozen tail: the reference never steps it (no gradient)
    cnt = store.step_dev_kl if off >= store.n_main else store.step_dev
    return int(cnt[0])


def optimizer_state_dict(store, lr, betas=(0.5, 0.999), eps=1e-8, weight_decay=0.01):
    """torch.optim.AdamW.state_dict() equivalent of a flat store's optimizer state."""
    state = {}
    names = _param_names(store)
    for i, n in enumerate(names):
        step = _step_of(store, n)
        if step == 0:
            continue
        off, numel = store.offsets[n]
        shape = store.shapes[n]
        state[i] = {"step": torch.tensor(float(step)),
                    "exp_avg": store.m[off:off + numel].view(shape).detach().cpu().clone(),
                    "exp_avg_sq": store.v[off:off + numel].view(shape).detach().cpu().clone()}
    group = {"lr": lr, "betas": tuple(betas), "eps": eps, "weight_decay": weight_decay, "amsgrad": False,
             "maximize": False, "foreach": None, "capturable": False, "differentiable": False, "fused": None,
             "decoupled_weight_decay": True, "params": list(range(len(names)))}
    return {"state": state, "param_groups": [group]}


def load_optimizer_state_dict(store, sd):
    """Fill ``store.m`` / ``store.v`` / the device step counters from a torch AdamW state_dict (reference
    parameter order).  Returns the param-group hyperparameters (lr, betas, eps, weight_decay)."""
    names = _param_names(store)
    groups = sd["param_groups"]
    idx = [i for g in groups for i in g["params"]]
    if len(idx) != len(names):
        raise ValueError(f"optimizer state covers {len(idx)} parameters, the model has {len(names)}")
    steps_main, steps_kl = set(), set()
    with torch.no_grad():
        store.m.zero_()
        store.v.zero_()
        for pos, i in enumerate(idx):
            st = sd["state"].get(i) or sd["state"].get(str(i))
            if not st:
                continue
            n = names[pos]
            off, numel = store.offsets[n]
            if off >= store.n_opt:
                raise ValueError(f"optimizer state for {n}, which the training step never updates")
            store.m[off:off + numel].copy_(torch.as_tensor(st["exp_avg"]).reshape(-1).to(store.m.device))
            store.v[off:off + numel].copy_(torch.as_tensor(st["exp_avg_sq"]).reshape(-1).to(store.v.device))
            (steps_kl if off >= store.n_main else steps_main).add(int(float(st["step"])))
        for steps, cnt in ((steps_main, store.step_dev), (steps_kl, store.step_dev_kl)):
            if len(steps) > 1:
                raise ValueError(f"parameters of one optimizer range carry different step counts {sorted(steps)}")
            cnt.fill_(steps.pop() if steps else 0)
    g = groups[0]
    return {k: g[k] for k in ("lr", "betas", "eps", "weight_decay") if k in g}


def save_resume(path, generator, discriminator, epoch, step, lr_g, lr_d, betas=(0.5, 0.999), epoch_complete=False,
                generators=None):
    """Write the reference's resume layout (t2i_moe_gan.py:1484-1491) with only the reference's keys.  ``epoch``
    is the 0-based epoch the state belongs to.  A mid-epoch checkpoint stores it as is (:1489); an end-of-epoch
    one (``epoch_complete``) stores ``epoch + 1``, as the reference's end-of-epoch file does (:1648), so a tool
    that reads 'epoch' the reference's way resumes at the next epoch.  ``generators``: name -> torch.Generator
    state (or the generator itself) stored as ``rng/<name>``, so a resumed run continues the same z, permutation
    and router-noise streams (every rank's local stream under data parallelism: ``rng/local<r>``)."""
    ck = {"generator": generator.state_dict(), "discriminator": discriminator.state_dict(),
          "optimizer_g": optimizer_state_dict(generator._store, lr_g, betas),
          "optimizer_d": optimizer_state_dict(discriminator._store, lr_d, betas),
          "epoch": int(epoch) + (1 if epoch_complete else 0), "step": int(step)}
    for name, g in (generators or {}).items():
        ck["rng/" + name] = g.get_state() if hasattr(g, "get_state") else g
    torch.save(ck, path)


def resume_start_epoch(ck_epoch, ck):
    """The epoch a resumed run starts at: the stored one (the reference's convention: a mid-epoch checkpoint
    repeats its epoch, an end-of-epoch one already stores the next).  Round-3 files stored the 0-based epoch plus
    an ``epoch_complete`` flag; they still resume at the next epoch."""
    return int(ck_epoch) + (1 if ck.get("epoch_complete", False) else 0)


def load_resume(path, generator, discriminator, generators=None):
    """Load a resume checkpoint (ours or the reference's); returns (start epoch, step).  A model-only checkpoint
    ({'generator', 'discriminator'}) or a bare generator state dict loads the weights and returns (0, 0).
    ``generators``: name -> torch.Generator restored from the checkpoint's ``rng/<name>`` states when present."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    if "generator" not in ck:  # bare generator state dict (inference.py:44-49)
        generator.load_state_dict(ck)
        return 0, 0
    generator.load_state_dict(ck["generator"])
    if "discriminator" in ck:
        discriminator.load_state_dict(ck["discriminator"])
    if "optimizer_g" in ck:
        load_optimizer_state_dict(generator._store, ck["optimizer_g"])
    if "optimizer_d" in ck:
        load_optimizer_state_dict(discriminator._store, ck["optimizer_d"])
    for name, g in (generators or {}).items():
        st = ck.get("rng/" + name)
        if st is not None:
            g.set_state(st)
    return resume_start_epoch(ck.get("epoch", 0), ck), int(ck.get("step", 0))
