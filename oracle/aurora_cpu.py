"""CPU restatement of the reference MoE-GAN training step (TEST INFRASTRUCTURE).

This module is the *checker*.  Only ``tests/``, ``__graft_entry__.smoke()`` and
``bench.py``'s ``cpu_baseline`` leg may import it; the product path
(``moe-gan_cpsc541_amd/``) never does, and fails loudly without its HIP library.

It restates, as plain functional fp32 PyTorch on the CPU, every function on the
hot path of ``moegan/t2i_moe_gan.py`` (citations are to that file).  Parameters
are passed as a flat ``{state_dict_key: tensor}`` dict in the reference's own
naming, and every random draw (router epsilon, z, the mismatch permutation) is
an explicit argument so that runs can be replayed exactly.

Parity is pinned: tests/test_oracle_golden.py checks this module against the
fixtures F1-F8 that tests/golden/make_golden.py produced by running the
reference itself.  The top-k (k < E) routing mode is a build extension that the
reference does not have (it trains dense, t2i_moe_gan.py:465-470): for k < E
this module *defines* the semantics (renormalised top-k combine) and that case
is "parity unpinned" against the reference.
"""
import math

import torch
import torch.nn.functional as F

LATENT_DIM = 512
TEXT_DIM = 512


# ---------------------------------------------------------------------------
# ModulatedConv  (t2i_moe_gan.py:122-186)
# ---------------------------------------------------------------------------
def modconv(x, w, P, pre, padding=0, demod=True):
    """Per-sample modulated/demodulated conv, materialised as in :158-180."""
    B, Cin, H, W = x.shape
    weight = P[pre + "weight"]
    Cout, _, k, _ = weight.shape
    style = F.linear(w, P[pre + "modulation.weight"], P[pre + "modulation.bias"])  # :158
    wmod = weight.unsqueeze(0) * style.view(B, 1, Cin, 1, 1)  # :161
    if demod:
        d = torch.rsqrt(wmod.pow(2).sum(dim=(2, 3, 4), keepdim=True) + 1e-8)  # :165
        wmod = wmod * d
    y = F.conv2d(x.reshape(1, B * Cin, H, W), wmod.reshape(B * Cout, Cin, k, k), padding=padding, groups=B)
    return y.view(B, Cout, y.shape[-2], y.shape[-1])


# ---------------------------------------------------------------------------
# Modulated Transformation Module  (t2i_moe_gan.py:188-247)
# ---------------------------------------------------------------------------
def base_grid(H, W, device=None, dtype=torch.float32):
    """linspace grid of :226-230 ([H, W, 2], last dim = (x, y))."""
    gy = torch.linspace(-1, 1, H, device=device, dtype=dtype).view(H, 1).expand(H, W)
    gx = torch.linspace(-1, 1, W, device=device, dtype=dtype).view(1, W).expand(H, W)
    return torch.stack((gx, gy), dim=2)


# LeakyReLU slope replay (test hook, like the top-k ``routes``): {MTM prefix: bool mask [B, C, H, W]} of a device
# run's pre-activation signs.  A pre-activation within rounding of 0 can land on the other slope in the device's
# arithmetic; the gradient at that element then differs by 0.8 g, which no reordering tolerance covers (measured:
# one flipped element of 32768 at 8x8 puts 4e-3 on a whole fp32 data gradient).  Used by the backward-carrying
# (grad-enabled) calls only.
LRELU_SLOPES = None


def _mtm_lrelu(y, pre):
    m = LRELU_SLOPES.get(pre) if LRELU_SLOPES is not None and y.requires_grad else None
    if m is None:
        return F.leaky_relu(y, 0.2)
    assert m.shape == y.shape, (pre, m.shape, y.shape)
    return torch.where(m, y, 0.2 * y)


def offset_act(o):
    """The offset head's LeakyReLU(0.2) (offset_net.1, t2i_moe_gan.py:199-203), a named step of mtm() so that a
    bf16 emulation (tests/steputil.bf16_module_rounding) can round the activation the device stores in bf16."""
    return F.leaky_relu(o, 0.2)


def warp(x, grid):
    """Bilinear sampling of the MTM input at the offset grid (:239); named like offset_act (the device's warped
    map is bf16, its gradient fp32)."""
    return F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=False)


def mtm(x, w, P, pre, use_offset=True):
    B, C, H, W = x.shape
    if use_offset:
        o = F.conv2d(x, P[pre + "offset_net.0.weight"], P[pre + "offset_net.0.bias"], padding=1)  # :223
        o = offset_act(o)
        o = F.conv2d(o, P[pre + "offset_net.2.weight"], P[pre + "offset_net.2.bias"], padding=1)
        grid = base_grid(H, W, dtype=x.dtype).unsqueeze(0) + o.permute(0, 2, 3, 1) * 0.05  # :226-235
        grid = grid.clamp(-1, 1)  # :236
        x = warp(x, grid)
    x = modconv(x, w, P, pre + "modulated_conv.", padding=1)
    return _mtm_lrelu(x, pre)  # :245


# ---------------------------------------------------------------------------
# Bayesian router  (t2i_moe_gan.py:265-423)
# ---------------------------------------------------------------------------
def reparam(mu, rho, eps):
    """:302-333 -- clamp(mu) + clamp(softplus(clamp(rho))) * clamp(eps)."""
    mu = mu.clamp(-10.0, 10.0)
    rho = rho.clamp(-8.0, 4.0)
    sigma = torch.log1p(torch.exp(rho)).clamp(1e-6, 10.0)
    return mu + sigma * eps.clamp(-2.0, 2.0)


def router(feature, text, P, pre, eps=None, training=True, anneal=1.0):
    """:335-402.  ``eps`` = (eps_f, eps_t, eps_c) when sampling; returns (probs, logits)."""
    if training:
        wf = reparam(P[pre + "feature_mu"], P[pre + "feature_rho"], eps[0])
        wt = reparam(P[pre + "text_mu"], P[pre + "text_rho"], eps[1])
        wc = reparam(P[pre + "combined_mu"], P[pre + "combined_rho"], eps[2])
    else:
        wf, wt, wc = P[pre + "feature_mu"], P[pre + "text_mu"], P[pre + "combined_mu"]
    logits = torch.cat([feature @ wf, text @ wt], dim=1) @ wc  # :364-371
    t_eff = (P[pre + "temperature"] * anneal).clamp(0.5, 5.0)  # :375
    logits = (logits / t_eff).clamp(-20.0, 20.0)  # :378-381
    probs = F.softmax(logits, dim=1).clamp(1e-6, 1.0)  # :384-387
    probs = probs / probs.sum(dim=1, keepdim=True)  # :389
    if not training:  # :392-400
        idx = probs.topk(1, dim=1).indices
        probs = torch.zeros_like(probs).scatter_(1, idx, 1.0)
    return probs, logits


def router_kl(P, pre):
    """:405-423."""
    total = 0.0
    for n in ("feature", "text", "combined"):
        lv = 2 * torch.log(torch.log1p(torch.exp(P[pre + n + "_rho"])))
        total = total + 0.5 * torch.sum(torch.exp(lv) + P[pre + n + "_mu"].pow(2) - 1 - lv)
    total = torch.nan_to_num(total, nan=0.0, posinf=200.0, neginf=0.0)
    return total.clamp(0.0, 120.0)


# ---------------------------------------------------------------------------
# Experts + SparseMoE  (t2i_moe_gan.py:249-263, 426-491)
# ---------------------------------------------------------------------------
def expert_ffn(x, P, pre):
    h = F.gelu(F.linear(x, P[pre + "net.0.weight"], P[pre + "net.0.bias"]))  # exact erf GELU
    return F.linear(h, P[pre + "net.2.weight"], P[pre + "net.2.bias"])


def topk_route(probs, k, idx=None):
    """Build extension: top-k (lowest index wins ties) with renormalised weights.

    For k == E this is exactly the reference's dense soft combine (weights = probs).
    ``idx`` [T, k] replays a given selection instead of recomputing it (tests resolve near-ties -- tokens
    whose top-k margin is within the device's rounding -- the way the device did, then compare the rest).
    """
    E = probs.shape[1]
    if k >= E:
        return probs
    if idx is None:
        idx = torch.topk(probs, k, dim=1, sorted=True).indices
    vals = probs.gather(1, idx.long())
    wsel = vals / vals.sum(dim=1, keepdim=True)
    return torch.zeros_like(probs).scatter(1, idx.long(), wsel)


def sparse_moe(x, w, P, pre, E, eps=None, training=True, anneal=1.0, topk=None, route=None):
    B, C, H, W = x.shape
    tok = x.permute(0, 2, 3, 1).reshape(-1, C)  # :455
    wtok = w[:, None, None, :].expand(B, H, W, w.shape[1]).reshape(-1, w.shape[1])  # :456
    probs, _ = router(tok, wtok, P, pre + "router.", eps, training, anneal)
    out = torch.zeros_like(tok)
    if training:
        gate = probs if topk is None else topk_route(probs, topk, route)
        for e in range(E):  # :467-470 (dense soft combine)
            if topk is not None and topk < E:
                # an expert that no token selected still runs on its (empty) token set, so its parameters get
                # a zero gradient rather than None -- the extension's defined semantics (the device's grouped
                # GEMMs produce zero gradients for an empty group, and AdamW then applies its decay step)
                idx = (gate[:, e] > 0).nonzero().squeeze(1)
                y = expert_ffn(tok[idx], P, f"{pre}experts.{e}.")
                out = out.index_add(0, idx, gate[idx, e:e + 1] * y)
            else:
                out = out + gate[:, e:e + 1] * expert_ffn(tok, P, f"{pre}experts.{e}.")
    else:
        idx = probs.argmax(dim=1)  # :473-483
        for e in range(E):
            m = idx == e
            if m.any():
                out = out.index_put((m.nonzero().squeeze(1),), expert_ffn(tok[m], P, f"{pre}experts.{e}."))
    y = out.reshape(B, H, W, C).permute(0, 3, 1, 2)
    kl = router_kl(P, pre + "router.") if training else torch.tensor(0.0)
    return y, kl, probs


# ---------------------------------------------------------------------------
# Attention block  (t2i_moe_gan.py:493-576)
# ---------------------------------------------------------------------------
def mha(q_in, kv_in, P, pre, heads=8):
    """nn.MultiheadAttention(batch_first=True) forward, restated."""
    B, Tq, C = q_in.shape
    Tk = kv_in.shape[1]
    Wi, bi = P[pre + "in_proj_weight"], P[pre + "in_proj_bias"]
    q = F.linear(q_in, Wi[:C], bi[:C])
    k = F.linear(kv_in, Wi[C:2 * C], bi[C:2 * C])
    v = F.linear(kv_in, Wi[2 * C:], bi[2 * C:])
    d = C // heads
    q = q.view(B, Tq, heads, d).transpose(1, 2)
    k = k.view(B, Tk, heads, d).transpose(1, 2)
    v = v.view(B, Tk, heads, d).transpose(1, 2)
    att = torch.softmax((q / math.sqrt(d)) @ k.transpose(-1, -2), dim=-1)
    o = (att @ v).transpose(1, 2).reshape(B, Tq, C)
    return F.linear(o, P[pre + "out_proj.weight"], P[pre + "out_proj.bias"])


def attention_block(x, w, text_seq, P, pre, E, eps=None, training=True, anneal=1.0, topk=None, route=None):
    B, C, H, W = x.shape
    xin = modconv(x, w, P, pre + "proj_in.")  # :539
    xf = xin.permute(0, 2, 3, 1).reshape(B, H * W, C)
    ln = lambda t, n: F.layer_norm(t, (C,), P[pre + n + ".weight"], P[pre + n + ".bias"])  # noqa: E731
    xn = ln(xf, "norm1")
    xf = xf + mha(xn, xn, P, pre + "self_attn.")  # :545-547
    tp = F.linear(text_seq, P[pre + "text_proj.weight"], P[pre + "text_proj.bias"])  # :550
    xf = xf + mha(ln(xf, "norm2"), tp, P, pre + "cross_attn.")  # :553-555
    xs = xf.reshape(B, H, W, C).permute(0, 3, 1, 2)
    xn3 = ln(xf, "norm3").reshape(B, H, W, C).permute(0, 3, 1, 2)  # :561
    mo, kl, probs = sparse_moe(xn3, w, P, pre + "moe.", E, eps, training, anneal, topk, route)  # :564
    return modconv(xs + mo, w, P, pre + "proj_out."), kl, probs  # :571-574


# ---------------------------------------------------------------------------
# Conv / generative blocks + generator  (t2i_moe_gan.py:579-855)
# ---------------------------------------------------------------------------
def conv_block(x, w, P, pre):
    off = (pre + "mtm1.offset_net.0.weight") in P  # offset heads only at resolution <= 16 (:199)
    out = mtm(x, w, P, pre + "mtm1.", off)
    out = mtm(out, w, P, pre + "mtm2.", off)
    skip = modconv(x, w, P, pre + "skip_proj.") if (pre + "skip_proj.weight") in P else x  # :615-616
    return out + skip


def gen_block(x, w, text_seq, P, pre, upsample, E, eps=None, training=True, anneal=1.0, topk=None, route=None):
    if upsample:  # :657-658
        x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
    x = conv_block(x, w, P, pre + "conv_block.")
    return attention_block(x, w, text_seq, P, pre + "attn_block.", E, eps, training, anneal, topk, route)


BLOCKS = (("gen_block_4", False), ("gen_block_8", True), ("gen_block_16", True))
# progressive extension (BASELINE C4; no reference definition, t2i_moe_gan.py:1005-1026 names gen_block_32 / _64
# only): upsample + ConvolutionBlock without offset heads, no attention block.  The composition of reference
# functions is restated here; the block list itself is the build's (moegan_mi/layout.py) -- parity unpinned.
EXT_BLOCKS = (("gen_block_32", 32), ("gen_block_64", 64), ("gen_block_128", 128))


def max_resolution(P):
    return max([16] + [r for n, r in EXT_BLOCKS if f"to_rgb_{r}.weight" in P])


def num_experts(P):
    e = 0
    while f"gen_block_4.attn_block.moe.experts.{e}.net.0.weight" in P:
        e += 1
    return e


def mapping(zt, P):
    h = zt
    for i in (0, 2, 4):
        h = F.leaky_relu(F.linear(h, P[f"mapping.{i}.weight"], P[f"mapping.{i}.bias"]), 0.2)
    return F.linear(h, P["mapping.6.weight"], P["mapping.6.bias"])


def generator(z, text, P, eps=None, training=True, anneal=1.0, psi=0.7, topk=None, routes=None):
    """:762-855.  ``eps`` = list of 3 (eps_f, eps_t, eps_c) tuples, one per MoE block; ``routes`` = optional
    list of 3 top-k index tensors to replay (topk_route)."""
    B = z.shape[0]
    E = num_experts(P)
    if text.shape[0] != B and text.shape[0] == 1:  # :781-787
        text = text.repeat(B, 1)
    t = F.linear(text, P["text_projection.0.weight"], P["text_projection.0.bias"])  # :682-687, :790
    t = F.layer_norm(t, (t.shape[1],), P["text_projection.1.weight"], P["text_projection.1.bias"])
    t = F.linear(F.leaky_relu(t, 0.2), P["text_projection.3.weight"], P["text_projection.3.bias"])
    text_seq = t.unsqueeze(1)
    w = mapping(torch.cat([z, text], dim=1), P)  # :793-796
    if psi < 1.0:  # :799-808
        with torch.no_grad():
            mean = mapping(torch.zeros(1, z.shape[1] + text.shape[1], dtype=z.dtype), P)
        w = mean + psi * (w - mean)
    x = P["constant"].repeat(B, 1, 1, 1)
    kls, probs = [], []
    feats = {}
    for i, (name, up) in enumerate(BLOCKS):
        x, kl, p = gen_block(x, w, text_seq, P, name + ".", up, E, None if eps is None else eps[i],
                             training, anneal, topk, None if routes is None else routes[i])
        kls.append(kl)
        probs.append(p)
        feats[4 << i] = x
    R = max_resolution(P)
    for name, r in EXT_BLOCKS:  # progressive extension only (R > 16)
        if r > R:
            break
        x = F.interpolate(x, scale_factor=2, mode="bilinear", align_corners=False)
        x = conv_block(x, w, P, name + ".conv_block.")
        feats[r] = x
    img8 = modconv(feats[R // 2], w, P, f"to_rgb_{R // 2}.")  # reference (R = 16): to_rgb_8, :831
    img16 = modconv(feats[R], w, P, f"to_rgb_{R}.")  # to_rgb_16, :839
    return img16, img8, sum(kls), probs


# ---------------------------------------------------------------------------
# Discriminator  (t2i_moe_gan.py:858-907)
# ---------------------------------------------------------------------------
def wn(PD, pre):
    """weight_norm(dim=0): W = g * v / ||v|| (norm over all dims but 0)."""
    v, g = PD[pre + "weight_v"], PD[pre + "weight_g"]
    norm = v.reshape(v.shape[0], -1).norm(dim=1).view(-1, *([1] * (v.dim() - 1)))
    return v * (g / norm)


def round_bf16_st(t):
    """Straight-through bf16 rounding: the value is rounded, the gradient passes unchanged.  Used only to MEASURE
    the bf16 sensitivity floor of a quantity (tests/steputil.py), never in a parity reference."""
    return t + (t.detach().bfloat16().float() - t.detach())


def discriminator(img, text, PD, rnd=None):
    """``rnd`` (floor measurements only): applied to the image and to every effective weight; its optional ``act``
    attribute to the two conv activations (the tensors a bf16 device stores between the layers)."""
    r = rnd or (lambda t: t)
    a = getattr(rnd, "act", None) or (lambda t: t)
    h = a(F.leaky_relu(F.conv2d(r(img), r(wn(PD, "conv_layers.0.")), PD["conv_layers.0.bias"], stride=2, padding=1),
                       0.2))
    h = a(F.leaky_relu(F.conv2d(h, r(wn(PD, "conv_layers.2.")), PD["conv_layers.2.bias"], stride=2, padding=1),
                       0.2))
    t = F.leaky_relu(F.linear(text, r(wn(PD, "text_projection.0.")), PD["text_projection.0.bias"]), 0.2)
    t = t[:, :, None, None].expand(-1, -1, h.shape[2], h.shape[3])  # :898-899
    out = F.conv2d(torch.cat([h, t], dim=1), r(wn(PD, "output_layer.0.")), PD["output_layer.0.bias"])
    return out.reshape(-1)  # :907


# ---------------------------------------------------------------------------
# Losses  (t2i_moe_gan.py:909-1000)
# ---------------------------------------------------------------------------
def d_loss(real_pred, fake_pred, mism_pred):
    return F.softplus(-real_pred).mean() + F.softplus(fake_pred).mean() + F.softplus(mism_pred).mean()


def g_loss(fake_pred):
    return F.softplus(-fake_pred).mean()


def balance_loss(probs_list, weight=0.01):
    """:951-1000 -- last layer only, unbiased std (torch.std default)."""
    p = probs_list[-1]
    E, T = p.shape[1], p.shape[0]
    frac = (p.sum(dim=0) + 1e-6) / T
    cv = frac.std() / (frac.mean() + 1e-6)
    return weight * torch.nan_to_num((E * cv).clamp(0.0, 10.0), nan=0.0)


def clip_loss(images, text, encode_image):
    """:75-119 with a caller-supplied image encoder; returns a constant (no grad)."""
    with torch.no_grad():
        im = torch.clamp(images, -1, 1)
        if im.shape[-1] != 224 or im.shape[-2] != 224:
            im = F.interpolate(im, size=(224, 224), mode="bilinear", align_corners=False)
        f = encode_image(im).float()
        f = f / f.norm(dim=-1, keepdim=True)
        tf = text / text.norm(dim=-1, keepdim=True)
        sim = torch.nan_to_num((f * tf).sum(dim=1))
        return 1.0 - sim.mean()


# ---------------------------------------------------------------------------
# One training step  (t2i_moe_gan.py:1262-1421, gradient_accumulation_steps=1)
# ---------------------------------------------------------------------------
def train_step(PG, PD, optG, optD, real, text, z, eps_dphase, eps_gphase, perm, *, r1_gamma=10.0,
               clip_w16=0.1, clip_w8=0.05, kl_weight_eff=1e-8, balance_weight=0.01, anneal=3.0,
               psi=0.7, topk=None, encode_image=None, d_clip=0.7, g_clip=0.8, acc=1, zero_grads=True,
               step_optim=True, routes_d=None, routes_g=None, full=False, d_round=None, after_d_step=None):
    """Replays one batch of the reference loop with explicit randomness.

    ``PG``/``PD`` map reference state_dict keys to leaf tensors (requires_grad
    for parameters); ``optG``/``optD`` are torch AdamW instances over them (the
    reference's own optimizer).  Gradient accumulation (:1272, :1329, :1353, :1413): ``zero_grads`` at
    the first batch of a window, ``step_optim`` at its last, losses divided by ``acc``.  The loop's loss
    guards are kept (:1315-1320 skip the batch on a NaN/Inf D loss, :1367-1376 KL clamp / NaN -> 0,
    :1396-1399 NaN/Inf G loss -> 0).  ``routes_d`` / ``routes_g``: top-k selections to replay in the
    D-phase / G-phase generator forwards (topk_route).  Returns a dict of logged scalars (``full``: also
    the images, logits and routing probabilities of the step).  ``d_round`` (floor measurements only) rounds
    the discriminator's inputs and effective weights (discriminator(rnd=...)).  ``after_d_step(PD)`` is called
    right after the discriminator's optimizer step (tests use it to continue the G phase from a given D).
    """
    D = lambda img, txt: discriminator(img, txt, PD, d_round)  # noqa: E731
    B = real.shape[0]
    if zero_grads:
        for p in PD.values():
            p.grad = None
    real = real.clone().requires_grad_(True)  # :1276
    real_pred = D(real, text)  # :1279
    g, = torch.autograd.grad(real_pred.sum(), real, create_graph=True)  # :1282-1284
    r1 = (r1_gamma / 2) * (g.reshape(B, -1).norm(2, dim=1) ** 2).mean()  # :1285-1286
    with torch.no_grad():  # :1289-1298
        f16d, f8, _, probs_d = generator(z, text, PG, eps_dphase, True, anneal, psi, topk, routes_d)
    fake_pred = D(f16d.detach(), text)  # :1299
    mism_pred = D(real.detach(), text[perm])  # :1303-1305
    dgan = d_loss(real_pred, fake_pred, mism_pred)
    dl = dgan + r1
    if not torch.isfinite(dl):  # :1315-1320 -- `continue`: no backward, no optimizer step, no G phase
        return {"d_loss_gan": float(dgan.detach()), "r1": float(r1.detach()), "skipped": True}
    (dl / acc).backward()  # :1326
    if step_optim:
        torch.nn.utils.clip_grad_norm_([p for p in PD.values() if p.requires_grad], max_norm=d_clip)  # :1336
        optD.step()
        if after_d_step is not None:
            after_d_step(PD)
    if zero_grads:
        for p in PG.values():
            p.grad = None
    f16, f8, kl, probs = generator(z, text, PG, eps_gphase, True, anneal, psi, topk, routes_g)  # :1358-1364
    if kl > 50.0:  # :1369-1370
        kl = torch.clamp(kl, max=50.0)
    if not torch.isfinite(kl):  # :1372-1376
        kl = torch.tensor(0.0, dtype=real.dtype, requires_grad=True)
    fake_pred_g = D(f16, text)
    gg = g_loss(fake_pred_g)  # :1379-1382
    if encode_image is not None:
        c16, c8 = clip_loss(f16, text, encode_image), clip_loss(f8, text, encode_image)
    else:
        c16 = c8 = torch.tensor(0.0)
    bal = balance_loss(probs, balance_weight)
    gl = gg + (clip_w16 * c16 + clip_w8 * c8) + bal  # :1393
    g_zeroed = not bool(torch.isfinite(gl))
    if g_zeroed:  # :1396-1399
        gl = torch.tensor(0.0, dtype=real.dtype, requires_grad=True)
    gl = gl + kl_weight_eff * kl  # :1402-1404
    (gl / acc).backward()  # :1410
    if step_optim:
        torch.nn.utils.clip_grad_norm_([p for p in PG.values() if p.requires_grad], max_norm=g_clip)  # :1420
        optG.step()
    out = {"d_loss_gan": float(dgan.detach()), "r1": float(r1.detach()), "g_loss_gan": float(gg.detach()),
           "kl": float(kl.detach()), "balance": float(bal.detach()), "clip16": float(c16), "clip8": float(c8),
           "r1_grad": g.detach(),
           "skipped": False, "g_zeroed": g_zeroed}
    if full:
        out.update(img16=f16.detach(), img8=f8.detach(), img16_d=f16d, probs=[p.detach() for p in probs],
                   probs_d=probs_d, real_pred=real_pred.detach(), fake_pred=fake_pred.detach(),
                   mism_pred=mism_pred.detach(), fake_pred_g=fake_pred_g.detach())
    return out
