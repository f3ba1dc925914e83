"""Pin the CPU oracle (oracle/aurora_cpu.py) to the reference's golden fixtures F1-F10."""
import numpy as np
import pytest
import torch

from goldens import T, check_packed, close, load
from oracle import aurora_cpu as O
from oracle.recipe import fill_state

torch.set_num_threads(8)


def _params(d, prefix):
    return {k[len(prefix):]: T(d[k]).requires_grad_(True) for k in d.files if k.startswith(prefix)}


def test_f1_modconv():
    d, _ = load("F1_modconv")
    for c in range(4):
        p = f"c{c}/"
        cin, cout, k, h = d[p + "cfg"]
        P = _params(d, p + "param/")
        x, w = T(d[p + "x"]).requires_grad_(True), T(d[p + "w"]).requires_grad_(True)
        y = O.modconv(x, w, P, "", padding=int(k) // 2)
        close(y, d[p + "y"], what="y")
        (y * T(d[p + "gy"])).sum().backward()
        close(x.grad, d[p + "gx"], what="gx")
        close(w.grad, d[p + "gw"], what="gw")
        for n, t in P.items():
            close(t.grad, d[p + "grad/" + n], what=n)


def test_f2_mtm():
    d, _ = load("F2_mtm")
    for c in range(3):
        p = f"c{c}/"
        P = _params(d, p + "param/")
        x, w = T(d[p + "x"]).requires_grad_(True), T(d[p + "w"]).requires_grad_(True)
        y = O.mtm(x, w, P, "")
        close(y, d[p + "y"], what="y")
        (y * T(d[p + "gy"])).sum().backward()
        close(x.grad, d[p + "gx"], what="gx")
        close(w.grad, d[p + "gw"], what="gw")
        for n, t in P.items():
            close(t.grad, d[p + "grad/" + n], rtol=2e-4, what=n)


@pytest.mark.parametrize("tag", ["e4", "e8", "e8kl"])
def test_f3_router(tag):
    d, _ = load("F3_router")
    p = tag + "/"
    P = _params(d, p + "param/")
    feat, text = T(d[p + "feature"]).requires_grad_(True), T(d[p + "text"]).requires_grad_(True)
    eps = tuple(T(d[p + n]) for n in ("epsilon_f", "epsilon_t", "epsilon_c"))
    probs, logits = O.router(feat, text, P, "", eps, True, 3.0)
    kl = O.router_kl(P, "")
    close(probs, d[p + "probs"], what="probs")
    close(logits, d[p + "logits"], what="logits")
    close(kl, d[p + "kl"], what="kl")
    ((probs * T(d[p + "gp"])).sum() + (logits * T(d[p + "gl"])).sum() + 0.37 * kl).backward()
    close(feat.grad, d[p + "gfeature"], what="gfeature")
    close(text.grad, d[p + "gtext"], what="gtext")
    for n, t in P.items():
        close(t.grad, d[p + "grad/" + n], what=n)
    with torch.no_grad():
        pe, le = O.router(feat, text, P, "", None, False, 3.0)
    close(pe, d[p + "eval_probs"], what="eval probs")
    assert np.array_equal(pe.argmax(1).numpy(), d[p + "eval_probs"].argmax(1))


def test_f4_moe():
    d, _ = load("F4_moe")
    P = _params(d, "param/")
    x, w = T(d["x"]).requires_grad_(True), T(d["w"]).requires_grad_(True)
    eps = tuple(T(d[n]) for n in ("epsilon_f", "epsilon_t", "epsilon_c"))
    y, kl, probs = O.sparse_moe(x, w, P, "", 4, eps, True, 3.0)
    close(y, d["y"], what="y")
    close(kl, d["kl"], what="kl")
    close(probs, d["probs"], what="probs")
    ((y * T(d["gy"])).sum() + (probs * T(d["gp"])).sum()).backward()
    close(x.grad, d["gx"], what="gx")
    close(w.grad, d["gw"], what="gw")
    for n, t in P.items():
        close(t.grad, d["grad/" + n], what=n)
    with torch.no_grad():
        ye, _, pe = O.sparse_moe(x, w, P, "", 4, None, False, 3.0)
    close(ye, d["eval_y"], what="eval y")
    assert np.array_equal(pe.argmax(1).numpy(), d["eval_idx"])


def _disc_params(seed=50):
    shapes = {
        "text_projection.0.bias": (128,), "text_projection.0.weight_g": (128, 1),
        "text_projection.0.weight_v": (128, 512), "conv_layers.0.bias": (128,),
        "conv_layers.0.weight_g": (128, 1, 1, 1), "conv_layers.0.weight_v": (128, 3, 4, 4),
        "conv_layers.2.bias": (256,), "conv_layers.2.weight_g": (256, 1, 1, 1),
        "conv_layers.2.weight_v": (256, 128, 4, 4), "output_layer.0.bias": (1,),
        "output_layer.0.weight_g": (1, 1, 1, 1), "output_layer.0.weight_v": (1, 384, 4, 4)}
    return {k: torch.from_numpy(v).requires_grad_(True) for k, v in fill_state(shapes, seed).items()}


def test_f5_disc_r1():
    d, meta = load("F5_disc")
    PD = _disc_params()
    real = T(d["real"]).requires_grad_(True)
    text = T(d["text"])
    fake = T(d["fake"])
    perm = torch.from_numpy(d["perm"])
    rp = O.discriminator(real, text, PD)
    close(rp, d["real_pred"], what="real_pred")
    g, = torch.autograd.grad(rp.sum(), real, create_graph=True)
    close(g, d["r1_grad"], what="r1_grad")
    r1 = 5.0 * (g.reshape(2, -1).norm(dim=1) ** 2).mean()
    close(r1, d["r1"], what="r1")
    fp = O.discriminator(fake, text, PD)
    mp = O.discriminator(real.detach(), text[perm], PD)
    close(fp, d["fake_pred"], what="fake_pred")
    close(mp, d["mism_pred"], what="mism_pred")
    (O.d_loss(rp, fp, mp) + r1).backward()
    for n, t in PD.items():
        check_packed(d, "grad/" + n, t.grad)


def test_f6_losses():
    d, _ = load("F6_losses")
    close(O.d_loss(T(d["real"]), T(d["fake"]), T(d["mism"])), d["d_loss"], what="d_loss")
    close(O.g_loss(T(d["fake"])), d["g_loss"], what="g_loss")
    for E in (4, 8):
        p = T(d[f"bal{E}/probs"]).requires_grad_(True)
        bl = O.balance_loss([p])
        close(bl, d[f"bal{E}/loss"], what="balance")
        bl.backward()
        close(p.grad, d[f"bal{E}/grad"], what="balance grad")
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "clip_double"))
    import clip
    model, _ = clip.load("ViT-B/32")
    close(O.clip_loss(T(d["clip_img"]), T(d["clip_txt"]), model.encode_image), d["clip_loss"], what="clip")


def generator_params(E=4, seed=0):
    """Reference-layout generator state (names/shapes of t2i_moe_gan.AuroraGenerator)."""
    from moegan_mi.layout import generator_shapes
    return {k: torch.from_numpy(v) for k, v in fill_state(generator_shapes(E), seed).items()}


def test_f7_generator():
    d, _ = load("F7_generator")
    P = generator_params()
    for k, v in P.items():
        if not k.split(".")[-1].startswith("epsilon_"):
            v.requires_grad_(True)
    z, text = T(d["z"]).requires_grad_(True), T(d["text"]).requires_grad_(True)
    eps = [tuple(T(d[f"eps{i}/{n}"]) for n in ("epsilon_f", "epsilon_t", "epsilon_c")) for i in range(3)]
    img16, img8, kl, probs = O.generator(z, text, P, eps, True, 3.0)
    close(img16, d["img16"], what="img16")
    close(img8, d["img8"], what="img8")
    close(kl, d["kl"], what="kl")
    for i in range(3):
        close(probs[i], d[f"probs{i}"], what=f"probs{i}")
    loss = (img16 * T(d["R16"])).sum() + (img8 * T(d["R8"])).sum() + 0.37 * kl
    loss = loss + sum((probs[i] * T(d[f"Rp{i}"])).sum() for i in range(3))
    loss.backward()
    close(z.grad, d["gz"], rtol=2e-4, what="gz")
    close(text.grad, d["gtext"], rtol=2e-4, what="gtext")
    for n, t in P.items():
        if not t.requires_grad:
            continue
        if "nograd/" + n in d.files:
            assert t.grad is None, n
        else:
            check_packed(d, "grad/" + n, t.grad, rtol=5e-4, atol=1e-7)
    with torch.no_grad():
        e16, e8, _, ep = O.generator(z, text, P, None, False, 3.0)
    close(e16, d["eval_img16"], what="eval img16")
    for i in range(3):
        assert np.array_equal(ep[i].argmax(1).numpy(), d[f"eval_idx{i}"])


def _replay_train(name):
    d, meta = load(name)
    nb, acc = meta.get("n_batches", 1), meta["acc"]
    PG = generator_params()
    PD = _disc_params()
    for k, v in PG.items():
        if not k.split(".")[-1].startswith("epsilon_"):
            v.requires_grad_(True)
    gparams = [v for v in PG.values() if v.requires_grad]
    optG = torch.optim.AdamW(gparams, lr=float(d["lr/G"]), betas=(0.5, 0.999), weight_decay=0.01)
    optD = torch.optim.AdamW(list(PD.values()), lr=float(d["lr/D"]), betas=(0.5, 0.999), weight_decay=0.01)
    before_g = {k: v.detach().clone() for k, v in PG.items()}
    before_d = {k: v.detach().clone() for k, v in PD.items()}
    import sys, os
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "golden", "clip_double"))
    import clip
    model, _ = clip.load("ViT-B/32")
    grads = {}
    for opt, which, P in ((optD, "D", PD), (optG, "G", PG)):
        def pre(o, a, k, which=which, P=P):
            grads[which] = {n: (None if t.grad is None else t.grad.clone()) for n, t in P.items() if t.requires_grad}
        opt.register_step_pre_hook(pre)
    L = meta["losses"]
    for bi in range(nb):
        sfx = "" if nb == 1 else f"@{bi}"
        eps = [tuple(T(d[f"eps{i}/{n}{sfx}"]) for n in ("epsilon_f", "epsilon_t", "epsilon_c")) for i in range(6)]
        logs = O.train_step(PG, PD, optG, optD, T(d["real" + sfx]), T(d["text" + sfx]), T(d["z" + sfx]), eps[:3],
                            eps[3:], torch.from_numpy(d["perm" + sfx]), kl_weight_eff=0.001 * 1e-5,
                            encode_image=model.encode_image, acc=acc, zero_grads=bi % acc == 0,
                            step_optim=(bi + 1) % acc == 0 or bi + 1 == nb)
        assert abs(logs["d_loss_gan"] - L["discriminator_loss"][bi]) < 1e-4 * abs(L["discriminator_loss"][bi])
        assert abs(logs["g_loss_gan"] - L["generator_loss"][bi]) < 1e-4 * abs(L["generator_loss"][bi]) + 1e-6
        assert abs(logs["balance"] - L["moe_balance_loss"][bi]) < 1e-4 * abs(L["moe_balance_loss"][bi]) + 1e-7
        assert abs(logs["clip16"] - L["compute_clip_loss"][2 * bi]) < 1e-5
        close(logs["r1_grad"], d["r1_grad" + sfx], what="r1_grad")
    assert meta["order"] == ["D", "G"]
    for which, P, before in (("D", PD, before_d), ("G", PG, before_g)):
        for n, t in P.items():
            if not t.requires_grad:
                continue
            if f"{which}/nograd/{n}" in d.files:
                assert grads[which][n] is None, n
                assert torch.equal(t.detach(), before[n]), n
                continue
            check_packed(d, f"{which}/grad/{n}", grads[which][n], rtol=5e-4, atol=1e-8)
            # AdamW step 1 moves each element by ~lr*sign(g): compare deltas loosely (sign flips at g~0)
            check_packed(d, f"{which}/delta/{n}", t.detach() - before[n], rtol=2e-2, atol=2e-6)


def test_f8_train_step():
    _replay_train("F8_train_step")


def test_f10_train_acc2():
    """gradient_accumulation_steps=2 over two batches: summed /acc gradients, one optimizer step each."""
    _replay_train("F10_train_acc2")
