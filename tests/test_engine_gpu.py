"""HIP engine vs the CPU oracle and the reference's golden fixtures (fp32 parity mode).

Module-level tests compare one engine module (forward + backward) against the
oracle's autograd at the model's real channel counts; fixture tests pin the
whole generator (F7), the discriminator with R1 (F5) and one full training
step (F8) to values produced by the reference itself.
Tolerances: fp32 relative 1e-4 for values, 5e-4 for gradients.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

from goldens import T, check_packed, close, load  # noqa: E402
from oracle import aurora_cpu as O  # noqa: E402
from oracle.recipe import fill_state  # noqa: E402

from moegan_mi.engine_d import DiscriminatorEngine  # noqa: E402
from moegan_mi.engine_g import GeneratorEngine  # noqa: E402
from moegan_mi.layout import discriminator_shapes, generator_shapes, is_buffer  # noqa: E402
from moegan_mi.params import ParamStore  # noqa: E402
from moegan_mi.step import StepConfig, TrainStep  # noqa: E402

DEV = "cuda"


def gen_store(E=4, seed=0, cdt=torch.float32):
    st = ParamStore(generator_shapes(E), DEV, frozen_prefixes=("to_rgb_8.",), shadow_dtype=cdt)
    vals = fill_state(generator_shapes(E), seed)
    st.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return st, {k: torch.from_numpy(v) for k, v in vals.items()}


def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


def cpu_params(vals):
    return {k: v.clone().requires_grad_(not is_buffer(k)) for k, v in vals.items()}


# ---------------------------------------------------------------------------
# module-level parity vs the oracle
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("pre,B,H,k,act", [("gen_block_16.conv_block.mtm2.modulated_conv.", 3, 16, 3, 1),
                                          ("gen_block_8.conv_block.skip_proj.", 2, 8, 1, 0),
                                          ("gen_block_4.attn_block.proj_in.", 4, 4, 1, 0),
                                          ("to_rgb_16.", 2, 16, 1, 0)])
def test_modconv_vs_oracle(pre, B, H, k, act):
    st, vals = gen_store()
    ge = GeneratorEngine(st, 4)
    ge.prep()
    Wt = vals[pre + "weight"]
    Cout, Cin = Wt.shape[:2]
    g = torch.Generator().manual_seed(5)
    x = torch.randn(B, Cin, H, H, generator=g)
    w = torch.randn(B, 512, generator=g)
    P = cpu_params(vals)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = O.modconv(xr, wr, P, pre, padding=k // 2)
    if act:
        y = torch.nn.functional.leaky_relu(y, 0.2)
    gy = torch.randn(y.shape, generator=g)
    (y * gy).sum().backward()
    yd, sv = ge.mc_fwd(pre, nhwc(x).to(DEV), w.to(DEV), act=act)
    rows = yd.shape[-1]
    close(yd[..., :Cout].permute(0, 3, 1, 2), y.detach(), rtol=1e-4, what="y")
    gz = torch.zeros(B, H, H, rows, device=DEV)
    gz[..., :Cout] = nhwc(gy).to(DEV)
    gx = torch.empty(B, H, H, Cin, device=DEV)
    gw = torch.zeros(B, 512, device=DEV)
    ge.mc_bwd(pre, sv, gz, gx, gw)
    torch.cuda.synchronize()
    close(gx.permute(0, 3, 1, 2), xr.grad, rtol=2e-4, what="gx")
    close(gw, wr.grad, rtol=2e-4, what="gw")
    for n in ("weight", "modulation.weight", "modulation.bias"):
        close(st.gview(pre + n), P[pre + n].grad, rtol=5e-4, what=n)


@pytest.mark.parametrize("pre,B,H,resid", [("gen_block_16.conv_block.mtm2.", 2, 16, False),
                                           ("gen_block_8.conv_block.mtm1.", 2, 8, True)])
def test_mtm_vs_oracle(pre, B, H, resid):
    st, vals = gen_store()
    ge = GeneratorEngine(st, 4)
    ge.prep()
    Wt = vals[pre + "modulated_conv.weight"]
    Cout, Cin = Wt.shape[:2]
    g = torch.Generator().manual_seed(6)
    x = torch.randn(B, Cin, H, H, generator=g)
    w = torch.randn(B, 512, generator=g)
    R = torch.randn(B, Cout, H, H, generator=g) if resid else None
    P = cpu_params(vals)
    with torch.no_grad():  # visible offsets through the 0.05 scale
        P[pre + "offset_net.2.weight"].mul_(20.0)
        st.view(pre + "offset_net.2.weight").mul_(20.0)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = O.mtm(xr, wr, P, pre)
    if resid:
        y = y + R
    gy = torch.randn(y.shape, generator=g)
    (y * gy).sum().backward()
    yd, sv = ge.mtm_fwd(pre, nhwc(x).to(DEV), w.to(DEV), resid=nhwc(R).to(DEV) if resid else None)
    close(yd.permute(0, 3, 1, 2), y.detach(), rtol=1e-4, what="y")
    gx = torch.empty(B, H, H, Cin, device=DEV)
    gw = torch.zeros(B, 512, device=DEV)
    ge.mtm_bwd(pre, sv, nhwc(gy).to(DEV), gx, gw)
    torch.cuda.synchronize()
    close(gx.permute(0, 3, 1, 2), xr.grad, rtol=3e-4, what="gx")
    close(gw, wr.grad, rtol=3e-4, what="gw")
    for n in ("offset_net.0.weight", "offset_net.0.bias", "offset_net.2.weight", "offset_net.2.bias",
              "modulated_conv.weight", "modulated_conv.modulation.weight"):
        close(st.gview(pre + n), P[pre + n].grad, rtol=5e-4, what=n)


@pytest.mark.parametrize("E,topk", [(4, None), (8, 2), (8, None)])
def test_attention_block_vs_oracle(E, topk):
    st, vals = gen_store(E=E)
    ge = GeneratorEngine(st, E, topk)
    ge.prep()
    pre = "gen_block_16.attn_block."
    B, H, C = 2, 16, 128
    g = torch.Generator().manual_seed(7)
    x = torch.randn(B, C, H, H, generator=g)
    w = torch.randn(B, 512, generator=g)
    ts = torch.randn(B, 1, 512, generator=g)
    eps = tuple(torch.randn(s, generator=g) for s in ((C, 128), (512, 128), (256, E)))
    P = cpu_params(vals)
    xr, wr, tr = (t.clone().requires_grad_(True) for t in (x, w, ts))
    y, kl, probs = O.attention_block(xr, wr, tr, P, pre, E, eps, True, 3.0, topk)
    gy = torch.randn(y.shape, generator=g)
    gp = torch.randn(probs.shape, generator=g)
    ((y * gy).sum() + (probs * gp).sum() + 0.25 * kl).backward()
    epsd = tuple(e.to(DEV) for e in eps)
    yd, pd, kl2, topi, sv = ge.attn_fwd(pre, nhwc(x).to(DEV), w.to(DEV), ts[:, 0].contiguous().to(DEV), epsd, 3.0)
    close(yd.permute(0, 3, 1, 2), y.detach(), rtol=1e-4, what="y")
    close(pd, probs.detach(), rtol=1e-4, what="probs")
    close(kl2[0], kl.detach(), rtol=1e-4, what="kl")
    gx = torch.empty(B, H, H, C, device=DEV)
    gw = torch.zeros(B, 512, device=DEV)
    gts = torch.zeros(B, 512, device=DEV)
    klc = (kl2[1:2] * 0.25).contiguous()
    ge.attn_bwd(pre, sv, nhwc(gy).to(DEV), gx, gw, gts, kl_coef=klc, g_probs=gp.to(DEV))
    torch.cuda.synchronize()
    close(gx.permute(0, 3, 1, 2), xr.grad, rtol=5e-4, what="gx")
    close(gw, wr.grad, rtol=5e-4, what="gw")
    close(gts, tr.grad[:, 0], rtol=5e-4, what="gtext_seq")
    for n, t in P.items():
        if n.startswith(pre) and t.requires_grad and t.grad is not None:
            close(st.gview(n), t.grad, rtol=1e-3, atol=1e-6, what=n)


# ---------------------------------------------------------------------------
# fixture parity (reference-produced values)
# ---------------------------------------------------------------------------
def test_generator_vs_F7():
    d, _ = load("F7_generator")
    st, _ = gen_store()
    ge = GeneratorEngine(st, 4)
    ge.prep()
    eps = [tuple(T(d[f"eps{i}/{n}"]).to(DEV) for n in ("epsilon_f", "epsilon_t", "epsilon_c")) for i in range(3)]
    z, text = T(d["z"]).to(DEV), T(d["text"]).to(DEV)
    img16, img8, kl2s, probs, topis, ctx = ge.forward(z, text, eps, 3.0, 0.7, train=True, save=True, want_img8=True)
    close(img16[..., :3].permute(0, 3, 1, 2), d["img16"], rtol=1e-4, what="img16")
    close(img8[..., :3].permute(0, 3, 1, 2), d["img8"], rtol=1e-4, what="img8")
    kl2 = torch.stack(kl2s)
    close(kl2[:, 0].sum(), d["kl"], rtol=1e-5, what="kl")
    for i in range(3):
        close(probs[i], d[f"probs{i}"], rtol=1e-4, what=f"probs{i}")
    g16 = torch.zeros_like(img16)
    g16[..., :3] = nhwc(T(d["R16"])).to(DEV)
    g8 = torch.zeros_like(img8)
    g8[..., :3] = nhwc(T(d["R8"])).to(DEV)
    gps = [T(d[f"Rp{i}"]).to(DEV) for i in range(3)]
    kl_coef = (0.37 * kl2[:, 1]).contiguous()
    gz, gtext = ge.backward(ctx, g16, kl_coef=kl_coef, want_input_grads=True, g_probs=gps, g_img8=g8)
    torch.cuda.synchronize()
    close(gz, d["gz"], rtol=5e-4, what="gz")
    close(gtext, d["gtext"], rtol=5e-4, what="gtext")
    for n in st.offsets:
        if "nograd/" + n in d.files:
            continue
        check_packed(d, "grad/" + n, st.gview(n).cpu(), rtol=1e-3, atol=1e-7)


def disc_store(seed=50):
    st = ParamStore(discriminator_shapes(), DEV)
    vals = fill_state(discriminator_shapes(), seed)
    st.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    return st


def test_disc_r1_vs_F5():
    d, _ = load("F5_disc")
    st = disc_store()
    de = DiscriminatorEngine(st)
    de.prep()
    real = T(d["real"]).to(DEV)
    text = T(d["text"]).to(DEV)
    fake = torch.zeros(2, 16, 16, 8, device=DEV)
    fake[..., :3] = nhwc(T(d["fake"])).to(DEV)
    perm = torch.from_numpy(d["perm"].astype(np.int32)).to(DEV)
    res = de.d_phase(real, text, fake, ("nhwc", 8), perm, 10.0)
    torch.cuda.synchronize()
    close(res["real_pred"].reshape(-1), d["real_pred"], rtol=1e-4, what="real_pred")
    close(res["fake_pred"], d["fake_pred"], rtol=1e-4, what="fake_pred")
    close(res["mism_pred"].reshape(-1), d["mism_pred"], rtol=1e-4, what="mism_pred")
    close(res["r1_grad"][..., :3].permute(0, 3, 1, 2), d["r1_grad"], rtol=1e-4, what="r1_grad")
    close(res["r1"][0], d["r1"], rtol=1e-4, what="r1")
    close(res["losses"][0], d["d_gan"], rtol=1e-5, what="d_gan")
    for n in st.offsets:
        check_packed(d, "grad/" + n, st.gview(n).cpu(), rtol=5e-4)
    # G-phase path: gradient into a 16x16 image
    _, _, g_img = de.g_phase(fake, ("nhwc", 8), text)
    torch.cuda.synchronize()
    close(g_img[..., :3].permute(0, 3, 1, 2), d["gfake"], rtol=1e-4, what="gfake")


def _train_replay(name, cdt="fp32"):
    d, meta = load(name)
    nb, acc = meta.get("n_batches", 1), meta["acc"]
    ts = TrainStep(StepConfig(E=4), DEV)
    gvals = fill_state(generator_shapes(4), 0)
    ts.gs.load_state_dict({k: torch.from_numpy(v) for k, v in gvals.items()})
    dvals = fill_state(discriminator_shapes(), 50)
    ts.ds.load_state_dict({k: torch.from_numpy(v) for k, v in dvals.items()})
    g_before = ts.gs.data.clone()
    d_before = ts.ds.data.clone()
    L = meta["losses"]
    for bi in range(nb):
        sfx = "" if nb == 1 else f"@{bi}"
        eps = [tuple(T(d[f"eps{i}/{n}{sfx}"]).to(DEV) for n in ("epsilon_f", "epsilon_t", "epsilon_c"))
               for i in range(6)]
        out = ts.step(T(d["real" + sfx]).to(DEV), T(d["text" + sfx]).to(DEV), T(d["z" + sfx]).to(DEV), eps[:3],
                      eps[3:], torch.from_numpy(d["perm" + sfx].astype(np.int32)).to(DEV), anneal=3.0,
                      lr_g=float(d["lr/G"]), lr_d=float(d["lr/D"]), eff_kl_weight=0.001 * 1e-5, acc=acc,
                      zero_grads=bi % acc == 0, step_optim=(bi + 1) % acc == 0 or bi + 1 == nb)
        torch.cuda.synchronize()
        dl, gl, bl = L["discriminator_loss"][bi], L["generator_loss"][bi], L["moe_balance_loss"][bi]
        assert abs(float(out["d_losses"][0]) - dl) < 1e-4 * abs(dl), (bi, float(out["d_losses"][0]), dl)
        assert abs(float(out["g_gan"][0]) - gl) < 1e-4 * abs(gl) + 1e-6, (bi, float(out["g_gan"][0]), gl)
        assert abs(float(out["balance"][0]) - bl) < 1e-3 * bl + 1e-7
        close(out["r1_grad"][..., :3].permute(0, 3, 1, 2), d["r1_grad" + sfx], rtol=1e-4, what="r1_grad")
    for which, store, before, ref_max in (("D", ts.ds, d_before, 0.7), ("G", ts.gs, g_before, 0.8)):
        n_opt = store.n_opt
        gbuf = store.acc if acc > 1 else store.grad  # the buffer AdamW stepped with (window accumulator)
        gn = float(gbuf[:n_opt].double().norm())
        coef = min(1.0, ref_max / (gn + 1e-6))
        for n, (off, numel) in store.offsets.items():
            shape = store.shapes[n]
            if f"{which}/nograd/{n}" in d.files:
                assert off >= n_opt, n
                assert torch.equal(store.data[off:off + numel], before[off:off + numel]), n
                continue
            g = (gbuf[off:off + numel] * coef).view(shape).cpu()
            check_packed(d, f"{which}/grad/{n}", g, rtol=2e-3, atol=1e-8)
            delta = (store.data[off:off + numel] - before[off:off + numel]).view(shape).cpu()
            check_packed(d, f"{which}/delta/{n}", delta, rtol=2e-2, atol=2e-6)


def test_train_step_vs_F8():
    _train_replay("F8_train_step")


def test_train_step_acc2_vs_F10():
    """gradient_accumulation_steps=2: D gradients of batch 0 include the G-phase loss (reference quirk)."""
    _train_replay("F10_train_acc2")
