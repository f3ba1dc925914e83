"""The reference's sub-module classes on the GPU (moegan_mi/modules.py), fp32, against the reference's own
fixtures F1 (ModulatedConv), F2 (ModulatedTransformationModule), F3 (BayesianRouter, train + KL + eval) and F4
(SparseMoE, train + eval top-1), and against the CPU oracle for the composite blocks (AttentionBlock,
ConvolutionBlock, GenerativeBlock) at the generator's real channel counts.  Forward outputs, input gradients and
every parameter gradient; fp32 tolerances as the engine tests (1e-4 values, 5e-4 .. 1e-3 gradients)."""
import numpy as np
import pytest
import torch

from goldens import T, close, load
from oracle import aurora_cpu as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _M():
    import t2i_moe_gan as M
    return M


def _load(mod, d, prefix):
    sd = mod.state_dict()
    sd.update({k[len(prefix):]: T(d[k]) for k in d.files if k.startswith(prefix)})
    mod.load_state_dict(sd)
    return mod.to(DEV)


def _pgrad(mod, name):
    st = mod._store
    off, numel = st.offsets[mod._IPRE + name]
    return mod.flat.grad[off:off + numel].view(st.shapes[mod._IPRE + name])


def _cuda_leaf(a):
    return T(a).to(DEV).requires_grad_(True)


def test_modulated_conv_vs_F1():
    M = _M()
    d, _ = load("F1_modconv")
    for c in range(4):
        p = f"c{c}/"
        cin, cout, k, h = (int(v) for v in d[p + "cfg"])
        m = _load(M.ModulatedConv(cin, cout, k, padding=k // 2), d, p + "param/")
        x, w = _cuda_leaf(d[p + "x"]), _cuda_leaf(d[p + "w"])
        y = m(x, w)
        close(y, d[p + "y"], rtol=1e-4, what=f"c{c} y")
        (y * T(d[p + "gy"]).to(DEV)).sum().backward()
        close(x.grad, d[p + "gx"], rtol=2e-4, what=f"c{c} gx")
        close(w.grad, d[p + "gw"], rtol=2e-4, what=f"c{c} gw")
        for n in ("weight", "modulation.weight", "modulation.bias"):
            close(_pgrad(m, n), d[p + "grad/" + n], rtol=5e-4, what=f"c{c} {n}")


def test_mtm_vs_F2():
    M = _M()
    d, _ = load("F2_mtm")
    for c in range(3):
        p = f"c{c}/"
        cin, cout, h = (int(v) for v in d[p + "cfg"])
        m = _load(M.ModulatedTransformationModule(cin, cout, 3, use_offset=True, resolution=h), d, p + "param/")
        x, w = _cuda_leaf(d[p + "x"]), _cuda_leaf(d[p + "w"])
        y = m(x, w)
        close(y, d[p + "y"], rtol=1e-4, what=f"c{c} y")
        (y * T(d[p + "gy"]).to(DEV)).sum().backward()
        close(x.grad, d[p + "gx"], rtol=3e-4, what=f"c{c} gx")
        close(w.grad, d[p + "gw"], rtol=3e-4, what=f"c{c} gw")
        for n in ("modulated_conv.weight", "modulated_conv.modulation.weight", "modulated_conv.modulation.bias",
                  "offset_net.0.weight", "offset_net.0.bias", "offset_net.2.weight", "offset_net.2.bias"):
            close(_pgrad(m, n), d[p + "grad/" + n], rtol=1e-3, what=f"c{c} {n}")


@pytest.mark.parametrize("tag", ["e4", "e8", "e8kl"])
def test_bayesian_router_vs_F3(tag):
    M = _M()
    d, meta = load("F3_router")
    p = tag + "/"
    E = int(d[p + "E"])
    feat_dim, text_dim = d[p + "feature"].shape[1], d[p + "text"].shape[1]
    m = _load(M.BayesianRouter(feat_dim, text_dim, E), d, p + "param/")
    eps = tuple(T(d[p + n]).to(DEV) for n in ("epsilon_f", "epsilon_t", "epsilon_c"))
    m._eps = lambda pre: eps  # the fixture's captured noise instead of a fresh draw
    feat, text = _cuda_leaf(d[p + "feature"]), _cuda_leaf(d[p + "text"])
    probs, logits = m(feat, text, sampling=True, annealing_factor=meta["anneal"])
    kl = m.kl_divergence()
    close(probs, d[p + "probs"], rtol=1e-4, what="probs")
    close(logits, d[p + "logits"], rtol=1e-4, what="logits")
    close(kl, d[p + "kl"], rtol=1e-5, what="kl")
    ((probs * T(d[p + "gp"]).to(DEV)).sum() + (logits * T(d[p + "gl"]).to(DEV)).sum() + 0.37 * kl).backward()
    close(feat.grad, d[p + "gfeature"], rtol=5e-4, what="gfeature")
    close(text.grad, d[p + "gtext"], rtol=5e-4, what="gtext")
    for n in ("feature_mu", "feature_rho", "text_mu", "text_rho", "combined_mu", "combined_rho", "temperature"):
        close(_pgrad(m, n), d[p + "grad/" + n], rtol=1e-3, atol=1e-7, what=n)
    with torch.no_grad():
        pe, le = m(feat, text, sampling=False, annealing_factor=meta["anneal"])
    close(pe, d[p + "eval_probs"], rtol=1e-6, what="eval probs")
    close(le, d[p + "eval_logits"], rtol=1e-4, what="eval logits")
    assert np.array_equal(pe.argmax(1).cpu().numpy(), d[p + "eval_probs"].argmax(1))


def test_sparse_moe_vs_F4():
    M = _M()
    d, meta = load("F4_moe")
    m = _load(M.SparseMoE(32, 64, 4), d, "param/")
    eps = tuple(T(d[n]).to(DEV) for n in ("epsilon_f", "epsilon_t", "epsilon_c"))
    m._eps = lambda pre: eps
    x, w = _cuda_leaf(d["x"]), _cuda_leaf(d["w"])
    y, kl, probs = m(x, w, annealing_factor=meta["anneal"])
    close(y, d["y"], rtol=1e-4, what="y")
    close(kl, d["kl"], rtol=1e-5, what="kl")
    close(probs, d["probs"], rtol=1e-4, what="probs")
    ((y * T(d["gy"]).to(DEV)).sum() + (probs * T(d["gp"]).to(DEV)).sum()).backward()
    close(x.grad, d["gx"], rtol=5e-4, what="gx")
    close(w.grad, d["gw"], rtol=5e-4, what="gw")
    for k in d.files:
        if k.startswith("grad/"):
            close(_pgrad(m, k[5:]), d[k], rtol=1e-3, atol=1e-7, what=k)
    m.eval()
    with torch.no_grad():
        ye, _, pe = m(x, w, annealing_factor=meta["anneal"])
    close(ye, d["eval_y"], rtol=1e-4, what="eval y")
    assert np.array_equal(pe.argmax(1).cpu().numpy(), d["eval_idx"])


def _oracle_params(mod, dtype=torch.float32):
    """The module's weights as reference-named CPU leaves (buffers without grad)."""
    from moegan_mi.layout import is_buffer
    return {k: v.detach().cpu().to(dtype).clone().requires_grad_(not is_buffer(k)) for k, v in mod.state_dict().items()}


def _check_param_grads(mod, P, rtol=1e-3):
    for n, t in P.items():
        if t.requires_grad and t.grad is not None:
            close(_pgrad(mod, n), t.grad, rtol=rtol, atol=1e-7, what=n)


@pytest.mark.parametrize("E,topk", [(4, None), (8, 2)])
def test_attention_block_module_vs_oracle(E, topk):
    M = _M()
    C, B, H = 128, 2, 16
    m = M.AttentionBlock(C, num_experts=E, topk=topk, seed=3).to(DEV)
    P = _oracle_params(m)
    g = torch.Generator().manual_seed(11)
    x, w, ts = torch.randn(B, C, H, H, generator=g), torch.randn(B, 512, generator=g), torch.randn(B, 1, 512, generator=g)
    eps = tuple(torch.randn(s, generator=g) for s in ((C, 128), (512, 128), (256, E)))
    m._eps = lambda pre: tuple(e.to(DEV) for e in eps)
    xr, wr, tr = (t.clone().requires_grad_(True) for t in (x, w, ts))
    # routing is replayed from the module's own selection only if it is top-k (indices are checked in the engine tests)
    kls = []
    xd, wd, td = (t.to(DEV).requires_grad_(True) for t in (x, w, ts))
    yd, pd = m(xd, wd, td, kls, annealing_factor=3.0)
    route = None if topk is None else torch.topk(pd.detach().cpu(), topk, dim=1).indices
    y, kl, probs = O.attention_block(xr, wr, tr, P, "", E, eps, True, 3.0, topk, route)
    close(yd, y.detach(), rtol=1e-4, what="y")
    close(pd, probs.detach(), rtol=1e-4, what="probs")
    close(kls[0], kl.detach(), rtol=1e-5, what="kl")
    gy = torch.randn(y.shape, generator=g)
    gp = torch.randn(probs.shape, generator=g)
    ((y * gy).sum() + (probs * gp).sum() + 0.25 * kl).backward()
    ((yd * gy.to(DEV)).sum() + (pd * gp.to(DEV)).sum() + 0.25 * kls[0]).backward()
    close(xd.grad, xr.grad, rtol=5e-4, what="gx")
    close(wd.grad, wr.grad, rtol=5e-4, what="gw")
    close(td.grad, tr.grad, rtol=5e-4, what="gtext_seq")
    _check_param_grads(m, P)


@pytest.mark.parametrize("cin,cout,H", [(256, 128, 16), (512, 512, 4), (512, 256, 8)])
def test_convolution_block_module_vs_oracle(cin, cout, H):
    M = _M()
    B = 2
    m = M.ConvolutionBlock(cin, cout, resolution=H, seed=5).to(DEV)
    # the oracle runs in fp64 here: with offsets this large its fp32 CPU grid_sample backward is itself off by
    # 5e-3 of the input gradient's scale (measured against fp64, tools/diag_cb.py), the device by 2e-6
    P = _oracle_params(m, torch.float64)
    with torch.no_grad():  # visible offsets through the 0.05 scale
        for pre in ("mtm1.", "mtm2."):
            P[pre + "offset_net.2.weight"].mul_(20.0)
        sd = m.state_dict()
        sd.update({k: v.detach().float() for k, v in P.items() if "offset_net.2.weight" in k})
        m.load_state_dict(sd)
    g = torch.Generator().manual_seed(13)
    x, w = torch.randn(B, cin, H, H, generator=g), torch.randn(B, 512, generator=g)
    xr, wr = x.double().requires_grad_(True), w.double().requires_grad_(True)
    y = O.conv_block(xr, wr, P, "")
    xd, wd = x.to(DEV).requires_grad_(True), w.to(DEV).requires_grad_(True)
    yd = m(xd, wd)
    close(yd, y.detach(), rtol=1e-4, what="y")
    gy = torch.randn(y.shape, generator=g)
    (y * gy.double()).sum().backward()
    (yd * gy.to(DEV)).sum().backward()
    close(xd.grad, xr.grad, rtol=5e-4, what="gx")
    close(wd.grad, wr.grad, rtol=5e-4, what="gw")
    _check_param_grads(m, P)


def test_generative_block_module_vs_oracle():
    M = _M()
    B, cin, cout, E = 2, 256, 128, 4
    m = M.GenerativeBlock(cin, cout, text_dim=512, upsample=True, resolution=16, seed=7).to(DEV)
    P = _oracle_params(m)
    g = torch.Generator().manual_seed(17)
    x, w, ts = torch.randn(B, cin, 8, 8, generator=g), torch.randn(B, 512, generator=g), torch.randn(B, 1, 512,
                                                                                                     generator=g)
    eps = tuple(torch.randn(s, generator=g) for s in ((cout, 128), (512, 128), (256, E)))
    m._eps = lambda pre: tuple(e.to(DEV) for e in eps)
    xr, wr, tr = (t.clone().requires_grad_(True) for t in (x, w, ts))
    y, kl, probs = O.gen_block(xr, wr, tr, P, "", True, E, eps, True, 3.0)
    kls = []
    xd, wd, td = (t.to(DEV).requires_grad_(True) for t in (x, w, ts))
    yd, pd = m(xd, wd, td, kls, annealing_factor=3.0)
    close(yd, y.detach(), rtol=1e-4, what="y")
    close(pd, probs.detach(), rtol=1e-4, what="probs")
    gy = torch.randn(y.shape, generator=g)
    ((y * gy).sum() + 0.5 * kl).backward()
    ((yd * gy.to(DEV)).sum() + 0.5 * kls[0]).backward()
    close(xd.grad, xr.grad, rtol=5e-4, what="gx")
    close(wd.grad, wr.grad, rtol=5e-4, what="gw")
    close(td.grad, tr.grad, rtol=5e-4, what="gtext_seq")
    _check_param_grads(m, P)


def test_expert_ffn_module_vs_torch():
    M = _M()
    m = M.SparseExpertFFN(128, seed=2).to(DEV)
    P = _oracle_params(m)
    g = torch.Generator().manual_seed(19)
    x = torch.randn(300, 128, generator=g)
    xr = x.clone().requires_grad_(True)
    y = O.expert_ffn(xr, P, "")
    xd = x.to(DEV).requires_grad_(True)
    yd = m(xd)
    close(yd, y.detach(), rtol=1e-4, what="y")
    gy = torch.randn(y.shape, generator=g)
    (y * gy).sum().backward()
    (yd * gy.to(DEV)).sum().backward()
    close(xd.grad, xr.grad, rtol=5e-4, what="gx")
    _check_param_grads(m, P)


def test_create_optimizer_for_active_blocks():
    """Reference :1005-1026: AdamW over text projection + mapping + constant + the active blocks only."""
    M = _M()
    G = M.AuroraGenerator(seed=1).to(DEV)
    with pytest.raises(AttributeError):
        M.create_optimizer_for_active_blocks(G, [4, 32], 1e-3, (0.5, 0.999), 0.01)
    opt = M.create_optimizer_for_active_blocks(G, [4, 8], 1e-3, (0.5, 0.999), 0.01)
    before = G.flat.detach().clone()
    gen = torch.Generator(device=DEV).manual_seed(0)
    G.flat.grad = torch.randn(G.flat.shape, device=DEV, generator=gen)
    opt.step()
    st = G._store
    # torch's AdamW on the same named subset, on the CPU
    names = opt.names
    ps = [torch.nn.Parameter(st.view(n).detach().cpu().clone()) for n in names]
    with torch.no_grad():
        for p, n in zip(ps, names):
            off, numel = st.offsets[n]
            p.copy_(before[off:off + numel].view(p.shape).cpu())
            p.grad = G.flat.grad[off:off + numel].view(p.shape).cpu()
    ref = torch.optim.AdamW(ps, lr=1e-3, betas=(0.5, 0.999), weight_decay=0.01)
    ref.step()
    active = set(names)
    for n, (off, numel) in st.offsets.items():
        got = G.flat.detach()[off:off + numel].cpu()
        if n in active:
            close(got, ps[names.index(n)].detach().reshape(-1), rtol=1e-5, what=n)
        else:
            assert torch.equal(got, before[off:off + numel].cpu()), n
    assert set(opt.state_dict()["state"]) == set(range(len(names)))
