"""Generate the golden fixtures F1-F10 by running the REFERENCE (this container only).

Run from the repo root:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Recipe: a local ``clip`` test double goes first on sys.path,
then /root/reference/moegan, bytecode writing is disabled (the mount must not
be modified), and ``import t2i_moe_gan``.  Weights come from the name-seeded
recipe in oracle/recipe.py; router epsilon, z and the mismatch permutation are
captured from the reference as it runs and stored, so the build's oracle and
HIP path can be replayed on exactly the same randomness.  Nothing from
/root/reference is copied: only inputs and outputs are written, to
tests/golden/*.npz.  The reference never travels to the GPU box; these fixtures
do.  Generated with torch 2.10.0 CPU (the reference pins 1.12.1; the ops used
have stable semantics across those versions).
"""
import json
import os
import sys
import zlib

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, "clip_double"))
sys.path.insert(0, "/root/reference/moegan")
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import t2i_moe_gan as R  # noqa: E402  (the reference, imported read-only)
from oracle.recipe import fill_state, input_batch  # noqa: E402

torch.set_num_threads(8)
OUT = HERE
FULL_MAX = 65536  # tensors up to this many elements are stored whole
N_SAMPLES = 64


def load_recipe(module, seed=0):
    sd = module.state_dict()
    vals = fill_state({k: tuple(v.shape) for k, v in sd.items()}, seed)
    module.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})


def sample_idx(name, numel):
    rng = np.random.default_rng(zlib.crc32(name.encode()) ^ 77)
    k = min(N_SAMPLES, numel)
    return np.sort(rng.choice(numel, size=k, replace=False))


def pack_tensor(out, prefix, name, t, full_max=FULL_MAX):
    """Store tensor ``t`` under ``prefix/name``: whole if small, else stats + samples."""
    a = t.detach().double().reshape(-1).numpy()
    key = f"{prefix}/{name}"
    if a.size <= full_max:
        out[key] = t.detach().float().numpy()
    else:
        idx = sample_idx(name, a.size)
        out[key + "#idx"] = idx.astype(np.int64)
        out[key + "#val"] = a[idx].astype(np.float32)
        out[key + "#shape"] = np.array(t.shape, dtype=np.int64)
    out[key + "#sum"] = np.array(a.sum())
    out[key + "#sumsq"] = np.array((a * a).sum())


def rnd(seed, *shape):
    return torch.from_numpy(np.random.default_rng(seed).standard_normal(shape).astype(np.float32))


def save(name, d, meta=None):
    d = dict(d)
    d["__meta__"] = np.array(json.dumps(meta or {}))
    path = os.path.join(OUT, name + ".npz")
    np.savez_compressed(path, **d)
    print(f"wrote {path} ({os.path.getsize(path)/1024:.1f} KiB)")


# ---------------------------------------------------------------------------
# F1: ModulatedConv (t2i_moe_gan.py:122-186)
# ---------------------------------------------------------------------------
def f1_modconv():
    out = {}
    cfgs = [(16, 8, 3, 4), (16, 16, 1, 8), (8, 3, 1, 16), (32, 16, 3, 8)]
    for ci_, (cin, cout, k, h) in enumerate(cfgs):
        m = R.ModulatedConv(cin, cout, k, padding=k // 2)
        load_recipe(m, seed=ci_)
        x = rnd(100 + ci_, 2, cin, h, h).requires_grad_(True)
        w = rnd(200 + ci_, 2, 512).requires_grad_(True)
        y = m(x, w)
        gy = rnd(300 + ci_, *y.shape)
        (y * gy).sum().backward()
        p = f"c{ci_}"
        out[p + "/cfg"] = np.array([cin, cout, k, h])
        out[p + "/x"] = x.detach().numpy()
        out[p + "/w"] = w.detach().numpy()
        out[p + "/y"] = y.detach().numpy()
        out[p + "/gy"] = gy.numpy()
        out[p + "/gx"] = x.grad.numpy()
        out[p + "/gw"] = w.grad.numpy()
        for n, prm in m.named_parameters():
            out[p + "/param/" + n] = prm.detach().numpy()
            out[p + "/grad/" + n] = prm.grad.numpy()
    save("F1_modconv", out, {"ref": "t2i_moe_gan.py:122-186", "seed_rule": "recipe seed=cfg index"})


# ---------------------------------------------------------------------------
# F2: ModulatedTransformationModule with offsets (t2i_moe_gan.py:188-247)
# ---------------------------------------------------------------------------
def f2_mtm():
    out = {}
    cfgs = [(16, 8, 4), (8, 8, 8), (8, 16, 16)]
    for ci_, (cin, cout, h) in enumerate(cfgs):
        m = R.ModulatedTransformationModule(cin, cout, 3, use_offset=True, resolution=h)
        load_recipe(m, seed=10 + ci_)
        # larger offsets so that the deformation is visible through the 0.05 scale
        with torch.no_grad():
            m.offset_net[2].weight.mul_(20.0)
        x = rnd(400 + ci_, 2, cin, h, h).requires_grad_(True)
        w = rnd(500 + ci_, 2, 512).requires_grad_(True)
        y = m(x, w)
        gy = rnd(600 + ci_, *y.shape)
        (y * gy).sum().backward()
        p = f"c{ci_}"
        out[p + "/cfg"] = np.array([cin, cout, h])
        out[p + "/x"] = x.detach().numpy()
        out[p + "/w"] = w.detach().numpy()
        out[p + "/y"] = y.detach().numpy()
        out[p + "/gy"] = gy.numpy()
        out[p + "/gx"] = x.grad.numpy()
        out[p + "/gw"] = w.grad.numpy()
        for n, prm in m.named_parameters():
            out[p + "/param/" + n] = prm.detach().numpy()
            out[p + "/grad/" + n] = prm.grad.numpy()
    save("F2_mtm", out, {"ref": "t2i_moe_gan.py:188-247", "note": "offset_net.2.weight scaled x20 after recipe"})


# ---------------------------------------------------------------------------
# F3: BayesianRouter (t2i_moe_gan.py:265-423)
# ---------------------------------------------------------------------------
def f3_router():
    out = {}
    cases = [("e4", 4, False), ("e8", 8, False), ("e8kl", 8, True)]
    for tag, E, klfree in cases:
        C, B, HW, TD = 32, 4, 16, 64
        T = B * HW
        r = R.BayesianRouter(C, TD, E)
        load_recipe(r, seed=20 + E)
        if klfree:  # sigma = 1, tiny mu: the KL stays under its 120 clamp -> live gradient
            with torch.no_grad():
                for n in ("feature", "text", "combined"):
                    getattr(r, n + "_rho").fill_(float(np.log(np.e - 1.0)))
                    getattr(r, n + "_mu").mul_(0.02)
        feat = rnd(700 + E, T, C).requires_grad_(True)
        wimg = rnd(800 + E, B, TD)
        text = wimg.repeat_interleave(HW, 0).requires_grad_(True)
        r.train()
        torch.manual_seed(3)
        probs, logits = r(feat, text, sampling=True, annealing_factor=3.0)
        kl = r.kl_divergence()
        gp = rnd(900 + E, T, E)
        gl = rnd(901 + E, T, E)
        ((probs * gp).sum() + (logits * gl).sum() + 0.37 * kl).backward()
        p = tag
        out[p + "/E"] = np.array(E)
        out[p + "/feature"] = feat.detach().numpy()
        out[p + "/text"] = text.detach().numpy()
        for n in ("epsilon_f", "epsilon_t", "epsilon_c"):
            out[p + "/" + n] = getattr(r, n).detach().numpy().copy()
        out[p + "/probs"] = probs.detach().numpy()
        out[p + "/logits"] = logits.detach().numpy()
        out[p + "/kl"] = kl.detach().numpy()
        out[p + "/gp"] = gp.numpy()
        out[p + "/gl"] = gl.numpy()
        out[p + "/gfeature"] = feat.grad.numpy()
        out[p + "/gtext"] = text.grad.numpy()
        for n, prm in r.named_parameters():
            out[p + "/param/" + n] = prm.detach().numpy()
            out[p + "/grad/" + n] = prm.grad.numpy()
        # eval: mean weights, hard top-1 one-hot (t2i_moe_gan.py:357-361, 391-400)
        r.eval()
        with torch.no_grad():
            pe, le = r(feat, text, sampling=False, annealing_factor=3.0)
        out[p + "/eval_probs"] = pe.numpy()
        out[p + "/eval_logits"] = le.numpy()
    save("F3_router", out, {"ref": "t2i_moe_gan.py:265-423", "anneal": 3.0})


# ---------------------------------------------------------------------------
# F4: SparseMoE (t2i_moe_gan.py:426-491)
# ---------------------------------------------------------------------------
def f4_moe():
    out = {}
    C, B, H = 32, 2, 4
    m = R.SparseMoE(C, 64, 4)
    load_recipe(m, seed=40)
    x = rnd(1000, B, C, H, H).requires_grad_(True)
    w = rnd(1001, B, 64).requires_grad_(True)
    m.train()
    torch.manual_seed(5)
    y, kl, probs = m(x, w, annealing_factor=3.0)
    gy = rnd(1002, *y.shape)
    gp = rnd(1003, *probs.shape)
    ((y * gy).sum() + (probs * gp).sum()).backward()
    out["x"] = x.detach().numpy()
    out["w"] = w.detach().numpy()
    for n in ("epsilon_f", "epsilon_t", "epsilon_c"):
        out[n] = getattr(m.router, n).detach().numpy().copy()
    out["y"] = y.detach().numpy()
    out["kl"] = kl.detach().numpy()
    out["probs"] = probs.detach().numpy()
    out["gy"] = gy.numpy()
    out["gp"] = gp.numpy()
    out["gx"] = x.grad.numpy()
    out["gw"] = w.grad.numpy()
    for n, prm in m.named_parameters():
        out["param/" + n] = prm.detach().numpy()
        out["grad/" + n] = prm.grad.numpy()
    m.eval()
    with torch.no_grad():
        ye, _, pe = m(x, w, annealing_factor=3.0)
    out["eval_y"] = ye.numpy()
    out["eval_probs"] = pe.numpy()
    out["eval_idx"] = pe.argmax(1).numpy()
    save("F4_moe", out, {"ref": "t2i_moe_gan.py:426-491", "anneal": 3.0})


# ---------------------------------------------------------------------------
# F5: AuroraDiscriminator + R1 double backward (t2i_moe_gan.py:858-907, 1276-1312)
# ---------------------------------------------------------------------------
def f5_disc():
    out = {}
    D = R.AuroraDiscriminator()
    load_recipe(D, seed=50)
    B = 2
    img, txt, _ = input_batch(B)
    real = torch.from_numpy(img).requires_grad_(True)
    text = torch.from_numpy(txt)
    fake = torch.from_numpy(np.random.default_rng(9).uniform(-1, 1, (B, 3, 16, 16)).astype(np.float32))
    perm = torch.tensor([1, 0])
    real_pred = D(real, text)
    g, = torch.autograd.grad(real_pred.sum(), real, create_graph=True)
    r1 = (10.0 / 2) * (g.view(B, -1).norm(2, dim=1) ** 2).mean()
    fake_pred = D(fake, text)
    mism_pred = D(real.detach(), text[perm])
    d_gan = F.softplus(-real_pred).mean() + F.softplus(fake_pred).mean() + F.softplus(mism_pred).mean()
    (d_gan + r1).backward()
    out["real"] = img
    out["text"] = txt
    out["fake"] = fake.numpy()
    out["perm"] = perm.numpy()
    out["real_pred"] = real_pred.detach().numpy()
    out["fake_pred"] = fake_pred.detach().numpy()
    out["mism_pred"] = mism_pred.detach().numpy()
    out["r1_grad"] = g.detach().numpy()
    out["r1"] = r1.detach().numpy()
    out["d_gan"] = d_gan.detach().numpy()
    for n, prm in D.named_parameters():
        pack_tensor(out, "grad", n, prm.grad)
    # separate pins: R1-only gradient (the double-backward path alone)
    D.zero_grad()
    real2 = torch.from_numpy(img).requires_grad_(True)
    g2, = torch.autograd.grad(D(real2, text).sum(), real2, create_graph=True)
    ((10.0 / 2) * (g2.view(B, -1).norm(2, dim=1) ** 2).mean()).backward()
    for n, prm in D.named_parameters():
        if prm.grad is not None:
            pack_tensor(out, "r1grad", n, prm.grad)
    # first-order gradient into a 16x16 input (the G-phase path, t2i_moe_gan.py:1379)
    D.zero_grad()
    f2 = fake.clone().requires_grad_(True)
    fp = D(f2, text)
    F.softplus(-fp).mean().backward()
    out["gfake"] = f2.grad.numpy()
    save("F5_disc", out, {"ref": "t2i_moe_gan.py:858-907,1276-1312", "r1_gamma": 10.0})


# ---------------------------------------------------------------------------
# F6: losses (t2i_moe_gan.py:909-1000)
# ---------------------------------------------------------------------------
def f6_losses():
    out = {}
    L = R.AuroraGANLoss("cpu")
    real = rnd(1100, 2 * 169)
    fake = rnd(1101, 2)
    mism = rnd(1102, 2 * 169)
    out["real"], out["fake"], out["mism"] = real.numpy(), fake.numpy(), mism.numpy()
    out["d_loss"] = L.discriminator_loss(real, fake, mism).numpy()
    out["g_loss"] = L.generator_loss(fake).numpy()
    for E in (4, 8):
        logits = rnd(1110 + E, 512, E) * 2
        probs = torch.softmax(logits, 1).requires_grad_(True)
        bl = L.moe_balance_loss([None, probs], balance_weight=0.01)
        bl.backward()
        out[f"bal{E}/probs"] = probs.detach().numpy()
        out[f"bal{E}/loss"] = bl.detach().numpy()
        out[f"bal{E}/grad"] = probs.grad.numpy()
    img = torch.tanh(rnd(1120, 2, 3, 16, 16))
    txt = rnd(1121, 2, 512)
    out["clip_img"], out["clip_txt"] = img.numpy(), txt.numpy()
    out["clip_loss"] = L.compute_clip_loss(img, txt).numpy()
    save("F6_losses", out, {"ref": "t2i_moe_gan.py:909-1000", "clip": "local test double (unpinned vs real CLIP)"})


# ---------------------------------------------------------------------------
# F7: full AuroraGenerator forward (+ backward of a probe loss) (t2i_moe_gan.py:668-855)
# ---------------------------------------------------------------------------
def _router_recorder(G):
    calls = []

    def hook(mod, inp, outp):
        calls.append({n: getattr(mod, n).detach().clone() for n in ("epsilon_f", "epsilon_t", "epsilon_c")})

    hs = [m.register_forward_hook(hook) for m in G.modules() if isinstance(m, R.BayesianRouter)]
    return calls, hs


def f7_generator():
    out = {}
    G = R.AuroraGenerator()
    load_recipe(G, seed=0)
    G.train()
    B = 2
    _, txt, z = input_batch(B)
    zt = torch.from_numpy(z).requires_grad_(True)
    tt = torch.from_numpy(txt).requires_grad_(True)
    calls, hs = _router_recorder(G)
    torch.manual_seed(3)
    img16, img8, kl, probs = G(zt, tt, return_intermediate=True, return_routing=True, annealing_factor=3.0)
    for h in hs:
        h.remove()
    R16, R8 = rnd(1200, *img16.shape), rnd(1201, *img8.shape)
    Rp = [rnd(1202 + i, *p.shape) for i, p in enumerate(probs)]
    loss = (img16 * R16).sum() + (img8 * R8).sum() + sum((p * r).sum() for p, r in zip(probs, Rp)) + 0.37 * kl
    loss.backward()
    out["z"], out["text"] = z, txt
    out["img16"] = img16.detach().numpy()
    out["img8"] = img8.detach().numpy()
    out["kl"] = kl.detach().numpy()
    for i, p in enumerate(probs):
        out[f"probs{i}"] = p.detach().numpy()
        out[f"Rp{i}"] = Rp[i].numpy()
    out["R16"], out["R8"] = R16.numpy(), R8.numpy()
    for i, c in enumerate(calls):
        for n, v in c.items():
            out[f"eps{i}/{n}"] = v.numpy()
    out["gz"] = zt.grad.numpy()
    out["gtext"] = tt.grad.numpy()
    for n, prm in G.named_parameters():
        if prm.grad is None:
            out["nograd/" + n] = np.array(1)
        else:
            pack_tensor(out, "grad", n, prm.grad, full_max=4096)
    # eval-mode forward: mean router weights, hard top-1 dispatch (t2i_moe_gan.py:391-400, 471-483)
    G.eval()
    with torch.no_grad():
        e16, e8, ekl, eprobs = G(torch.from_numpy(z), torch.from_numpy(txt), return_intermediate=True,
                                 return_routing=True, annealing_factor=3.0)
    out["eval_img16"] = e16.numpy()
    out["eval_img8"] = e8.numpy()
    for i, p in enumerate(eprobs):
        out[f"eval_idx{i}"] = p.argmax(1).numpy()
    save("F7_generator", out, {"ref": "t2i_moe_gan.py:668-855", "B": B, "psi": 0.7, "anneal": 3.0, "E": 4})


# ---------------------------------------------------------------------------
# F8: one full step of train_aurora_gan (t2i_moe_gan.py:1029-1495), B=2, acc=1
# ---------------------------------------------------------------------------
def f8_train_step():
    _train_capture("F8_train_step", n_batches=1, acc=1)


def f10_train_acc2():
    """Two batches with gradient_accumulation_steps=2: one D and one G optimizer step at batch 1, gradients
    summed over both batches (including the G-phase loss's D gradients of batch 0, :1353-1413)."""
    _train_capture("F10_train_acc2", n_batches=2, acc=2)


def _train_capture(name, n_batches, acc):
    out = {}
    B = 2
    batches = []
    for bi in range(n_batches):
        img, txt, _ = input_batch(B, seed_img=10 * bi, seed_txt=10 * bi + 1)
        batches.append((torch.from_numpy(img), torch.from_numpy(txt)))

    inst = {}
    origG, origD = R.AuroraGenerator.__init__, R.AuroraDiscriminator.__init__

    def g_init(self, *a, **k):
        origG(self, *a, **k)
        load_recipe(self, seed=0)
        inst["G"] = self

    def d_init(self, *a, **k):
        origD(self, *a, **k)
        load_recipe(self, seed=50)
        inst["D"] = self

    R.AuroraGenerator.__init__, R.AuroraDiscriminator.__init__ = g_init, d_init

    rec = {"randn": [], "randperm": [], "router": [], "opt": []}
    orig_randn, orig_randperm = torch.randn, torch.randperm

    def randn(*a, **k):
        t = orig_randn(*a, **k)
        rec["randn"].append(t.detach().clone())
        return t

    def randperm(*a, **k):
        t = orig_randperm(*a, **k)
        rec["randperm"].append(t.clone())
        return t

    orig_router_fwd = R.BayesianRouter.forward

    def router_fwd(self, *a, **k):
        res = orig_router_fwd(self, *a, **k)
        if self.training:
            rec["router"].append({n: getattr(self, n).detach().clone() for n in ("epsilon_f", "epsilon_t", "epsilon_c")})
        return res

    losses = {}

    def wrap(name, fn):
        def w(*a, **k):
            v = fn(*a, **k)
            losses.setdefault(name, []).append(float(v.detach()))
            return v
        return w

    for nm in ("discriminator_loss", "generator_loss", "moe_balance_loss", "compute_clip_loss"):
        setattr(R.AuroraGANLoss, nm, wrap(nm, getattr(R.AuroraGANLoss, nm)))
    orig_grad = torch.autograd.grad

    def agrad(*a, **k):
        res = orig_grad(*a, **k)
        rec.setdefault("r1g", []).append(res[0].detach().clone())
        return res

    def pre_hook(opt, args, kwargs):
        snap = []
        for grp in opt.param_groups:
            for p_ in grp["params"]:
                snap.append((p_, None if p_.grad is None else p_.grad.detach().clone(), p_.detach().clone(), grp["lr"]))
        rec["opt"].append([opt, snap])

    def post_hook(opt, args, kwargs):
        rec["opt"][-1].append([p_.detach().clone() for p_, _, _, _ in rec["opt"][-1][1]])

    from torch.optim.optimizer import register_optimizer_step_post_hook, register_optimizer_step_pre_hook
    h1 = register_optimizer_step_pre_hook(pre_hook)
    h2 = register_optimizer_step_post_hook(post_hook)
    torch.randn, torch.randperm = randn, randperm
    R.BayesianRouter.forward = router_fwd
    torch.autograd.grad = agrad
    torch.manual_seed(1234)
    try:
        R.train_aurora_gan(batches, num_epochs=1, gradient_accumulation_steps=acc, checkpoint_activation=False,
                           device="cpu", save_dir="/tmp/scratch/ckpt", log_interval=1)
    finally:
        torch.randn, torch.randperm = orig_randn, orig_randperm
        R.BayesianRouter.forward = orig_router_fwd
        torch.autograd.grad = orig_grad
        R.AuroraGenerator.__init__, R.AuroraDiscriminator.__init__ = origG, origD
        h1.remove()
        h2.remove()

    G, D = inst["G"], inst["D"]
    names = {id(p_): ("G", n) for n, p_ in G.named_parameters()}
    names.update({id(p_): ("D", n) for n, p_ in D.named_parameters()})
    # module construction also calls torch.randn (weights); z is the one [B, 512] draw per batch (:1266)
    zs = [t for t in rec["randn"] if tuple(t.shape) == (B, 512)][-n_batches:]
    assert len(zs) == n_batches and len(rec["randperm"]) == n_batches
    assert len(rec["router"]) == 6 * n_batches, len(rec["router"])
    for bi in range(n_batches):
        sfx = "" if n_batches == 1 else f"@{bi}"
        out["real" + sfx], out["text" + sfx] = batches[bi][0].detach().numpy(), batches[bi][1].detach().numpy()
        out["z" + sfx] = zs[bi].numpy()
        out["perm" + sfx] = rec["randperm"][bi].numpy()
        for i, c in enumerate(rec["router"][6 * bi:6 * bi + 6]):
            for n, v in c.items():
                out[f"eps{i}/{n}" + sfx] = v.numpy()
        out["r1_grad" + sfx] = rec["r1g"][bi].numpy()
    order = []
    for opt, snap, after in rec["opt"]:
        which = names[id(snap[0][0])][0]
        order.append(which)
        out[f"lr/{which}"] = np.array(snap[0][3])
        for (p_, g, before, _), aft in zip(snap, after):
            _, n = names[id(p_)]
            if g is None:
                out[f"{which}/nograd/{n}"] = np.array(1)
            else:
                pack_tensor(out, f"{which}/grad", n, g, full_max=4096)
            pack_tensor(out, f"{which}/delta", n, aft - before, full_max=4096)
    meta = {"ref": "t2i_moe_gan.py:1029-1495", "B": B, "acc": acc, "n_batches": n_batches, "order": order,
            "losses": losses, "torch": torch.__version__,
            "note": "checkpoint_activation=False (identical math; keeps router-call capture clean)"}
    save(name, out, meta)


# ---------------------------------------------------------------------------
# F9: the reference state_dict layout (keys, shapes) of AuroraGenerator / AuroraDiscriminator (drop-in
# checkpoints: sagemaker_train.py:297-301, inference.py:34-49)
# ---------------------------------------------------------------------------
def f9_layout():
    torch.manual_seed(0)
    lay = {}
    for tag, mod in (("G", R.AuroraGenerator()), ("D", R.AuroraDiscriminator()),
                     ("G8", R.AuroraGenerator(num_experts=8) if "num_experts" in
                      R.AuroraGenerator.__init__.__code__.co_varnames else None)):
        if mod is None:
            continue
        sd = mod.state_dict()
        lay[tag] = {"keys": list(sd.keys()), "shapes": [list(v.shape) for v in sd.values()],
                    "params": [n for n, _ in mod.named_parameters()]}
    path = os.path.join(OUT, "F9_layout.json")
    with open(path, "w") as f:
        json.dump({"ref": "t2i_moe_gan.py:668-907", **lay}, f)
    print(f"wrote {path}")


if __name__ == "__main__":
    which = sys.argv[1:] or ["f1", "f2", "f3", "f4", "f5", "f6", "f7", "f8", "f9", "f10"]
    for w in which:
        globals()[{"f1": "f1_modconv", "f2": "f2_mtm", "f3": "f3_router", "f4": "f4_moe", "f5": "f5_disc",
                   "f6": "f6_losses", "f7": "f7_generator", "f8": "f8_train_step", "f9": "f9_layout",
                   "f10": "f10_train_acc2"}[w]]()
