"""Shared set-up for the step-level parity tests: the same seeded weights, inputs and router noise for the
HIP TrainStep and the CPU oracle (oracle/aurora_cpu.train_step), plus the comparison metrics."""
import numpy as np
import torch

from oracle import aurora_cpu as O
from oracle.recipe import fill_state

EPS_DIMS = [(512, 512), (256, 512), (128, 512)]  # (C, text dim) per MoE block


def make_inputs(B, E, seed=0, res=64):
    """real U(-1,1) [B,3,res,res], text / z N(0,1) [B,512], 6 router-noise triples (D phase, G phase), perm."""
    g = torch.Generator().manual_seed(seed)
    real = torch.rand(B, 3, res, res, generator=g) * 2 - 1
    text = torch.randn(B, 512, generator=g)
    z = torch.randn(B, 512, generator=g)
    eps = [tuple(torch.randn(s, generator=g) for s in ((c, 128), (t, 128), (256, E))) for c, t in EPS_DIMS * 2]
    perm = torch.randperm(B, generator=g)
    return real, text, z, eps[:3], eps[3:], perm


def oracle_models(E, lr=2e-4, seed_g=0, seed_d=50, max_res=16, dtype=torch.float32):
    """Reference-layout leaves (fp32, or fp64 for an oracle run whose own rounding must stay far below the
    device's) + the reference's AdamW (betas 0.5/0.999, wd 0.01, :1100-1102), with the clipped gradients captured
    right before each optimizer step.  ``max_res`` > 16: progressive extension."""
    from moegan_mi.layout import discriminator_shapes, frozen_rgb_prefixes, generator_shapes
    PG = {n: torch.from_numpy(v).to(dtype) for n, v in fill_state(generator_shapes(E, max_res), seed_g).items()}
    frozen = frozen_rgb_prefixes(max_res)
    PD = {n: torch.from_numpy(v).to(dtype).requires_grad_(True)
          for n, v in fill_state(discriminator_shapes(), seed_d).items()}
    for n, v in PG.items():
        # (the reference's to_rgb_8 is a leaf whose .grad stays None; the progressive extension's unused lower
        # to_rgb layers do not reach the loss at all, so they stay out of the optimizer there)
        if not n.split(".")[-1].startswith("epsilon_") and (max_res == 16 or not n.startswith(frozen)):
            v.requires_grad_(True)
    optG = torch.optim.AdamW([v for v in PG.values() if v.requires_grad], lr=lr, betas=(0.5, 0.999),
                             weight_decay=0.01)
    optD = torch.optim.AdamW(list(PD.values()), lr=lr, betas=(0.5, 0.999), weight_decay=0.01)
    return PG, PD, optG, optD, _capture(optD, optG, PD, PG)


def _capture(optD, optG, PD, PG):
    grads = {}
    for opt, which, P in ((optD, "D", PD), (optG, "G", PG)):
        def pre(o, a, k, which=which, P=P):
            grads[which] = {n: (None if t.grad is None else t.grad.clone()) for n, t in P.items() if t.requires_grad}
        opt.register_step_pre_hook(pre)
    return grads


def oracle_clone(PG, PD, optG, optD, lr=2e-4):
    """Independent copy of the oracle's current parameters and AdamW state (to run a second, perturbed step from
    the same point), with gradient capture."""
    PG2 = {n: v.detach().clone().requires_grad_(v.requires_grad) for n, v in PG.items()}
    PD2 = {n: v.detach().clone().requires_grad_(True) for n, v in PD.items()}
    optG2 = torch.optim.AdamW([v for v in PG2.values() if v.requires_grad], lr=lr, betas=(0.5, 0.999),
                              weight_decay=0.01)
    optD2 = torch.optim.AdamW(list(PD2.values()), lr=lr, betas=(0.5, 0.999), weight_decay=0.01)
    optG2.load_state_dict(optG.state_dict())
    optD2.load_state_dict(optD.state_dict())
    return PG2, PD2, optG2, optD2, _capture(optD2, optG2, PD2, PG2)


def gpu_step(E, topk, dtype, dev="cuda", seed_g=0, seed_d=50, fp8=False, max_res=16):
    from moegan_mi.layout import discriminator_shapes, generator_shapes
    from moegan_mi.step import StepConfig, TrainStep
    ts = TrainStep(StepConfig(E=E, topk=topk, dtype=dtype, fp8=fp8, max_res=max_res), dev)
    ts.gs.load_state_dict({k: torch.from_numpy(v) for k, v in
                           fill_state(generator_shapes(E, max_res), seed_g).items()})
    ts.ds.load_state_dict({k: torch.from_numpy(v) for k, v in fill_state(discriminator_shapes(), seed_d).items()})
    return ts


def cosine(a, b):
    a = a.detach().double().reshape(-1).cpu()
    b = b.detach().double().reshape(-1).cpu()
    na, nb = float(a.norm()), float(b.norm())
    if na == 0.0 and nb == 0.0:
        return 1.0
    if na == 0.0 or nb == 0.0:
        return 0.0
    return float((a @ b) / (na * nb))


def rel_norm_diff(a, b):
    a = a.detach().double().reshape(-1).cpu()
    b = b.detach().double().reshape(-1).cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


def topk_margin(probs, k):
    """log(p_(k) / p_(k+1)): the logit-space gap deciding top-k membership ([T]; +inf when k == E)."""
    E = probs.shape[1]
    if k >= E:
        return torch.full((probs.shape[0],), float("inf"))
    v = torch.topk(probs.double(), k + 1, dim=1).values
    return torch.log(v[:, k - 1]) - torch.log(v[:, k])


def routing_agreement(topi_dev, probs_dev, probs_ref, k, delta):
    """Device top-k sets vs the oracle's own top-k on its fp32 probabilities.

    Returns a dict: n tokens; ``self_mismatch`` = tokens whose device selection is not the top-k of the device's
    own probabilities (must be 0: kernel consistency); ``mismatch``; ``near`` = tokens whose oracle margin
    log(p_(k)/p_(k+1)) is below ``delta``; ``bad`` = mismatches outside the near-ties; ``drift`` = the largest
    change of that margin between oracle and device (logit units, measured on the oracle's k-th / (k+1)-th
    experts) -- the quantity ``delta`` must bound."""
    pd, pr = probs_dev.detach().float().cpu(), probs_ref.detach().float().cpu()
    dev = topi_dev.long().cpu().sort(dim=1).values
    # the device's selection must be a top-k of its own probabilities: min selected >= max unselected (value
    # based, so exact ties may resolve either way)
    sel = torch.zeros_like(pd, dtype=torch.bool).scatter_(1, topi_dev.long().cpu(), True)
    own_ok = pd.masked_fill(~sel, float("inf")).min(dim=1).values >= pd.masked_fill(sel, float("-inf")).max(dim=1).values
    ref_idx = torch.topk(pr.double(), min(k + 1, pr.shape[1]), dim=1).indices
    ref = ref_idx[:, :k].sort(dim=1).values
    mism = (ref != dev).any(dim=1)
    margin = topk_margin(pr, k)
    near = margin < delta
    drift = 0.0
    if k < pr.shape[1]:
        a, b = ref_idx[:, k - 1:k], ref_idx[:, k:k + 1]
        md = torch.log(pd.double().gather(1, a)) - torch.log(pd.double().gather(1, b))
        drift = float((md.view(-1) - margin).abs().max())
    return dict(n=int(mism.numel()), self_mismatch=int((~own_ok).sum()), mismatch=int(mism.sum()),
                near=int(near.sum()), bad=int((mism & ~near).sum()), drift=drift)


def nchw(img_nhwc_padded):
    return img_nhwc_padded[..., :3].permute(0, 3, 1, 2).float().cpu()


def np32(t):
    return np.asarray(t.detach().cpu(), dtype=np.float32)


def bf16_r1_floor(PD, real, text):
    """How far bf16 rounding ALONE moves the R1 input gradient d sum D(real) / d real (t2i_moe_gan.py:1282): the
    fp32 oracle fed the bf16-rounded image and bf16-rounded weights, vs the plain fp32 oracle (relative L2).  The
    LeakyReLU masks make this gradient ill-conditioned (a rounded pre-activation near 0 flips its slope), so a
    bf16 device cannot be held closer than this."""
    def g_of(P, x):
        x = x.clone().requires_grad_(True)
        g, = torch.autograd.grad(O.discriminator(x, text, P).sum(), x)
        return g
    bf = lambda t: t.detach().bfloat16().float()  # noqa: E731
    Pb = {k: (bf(v) if k.endswith("weight_v") else v.detach()) for k, v in PD.items()}
    P0 = {k: v.detach() for k, v in PD.items()}
    return rel_norm_diff(g_of(Pb, bf(real)), g_of(P0, real))


class Rounder:
    """Value rounding to bf16 precision (result kept in the input's dtype): round-to-nearest-even, or -- with a
    ``seed`` -- nearest-even on a rescaled grid, x -> bf16(x * s) / s with a fixed non-power-of-two s per seed.
    That is another realization of the same noise: the relative grid spacing, so the error distribution, is the
    nearest-even one, while which values round which way is independent of realization 0; equal values still round
    alike (as on the device, where an image's broadcast style, the repeated constant or a shared weight round once
    for every token).  (Stochastic rounding was measured as a poor yardstick: drawing a direction per element
    averages that coherent error away -- its floors came out 0.6x the nearest-even ones after the sqrt(2)
    variance correction.)"""

    def __init__(self, seed=None, offset_ulp=None):
        self.seed = seed
        self.noise_scale = 1.0
        self.s = 1.0 if seed is None else 2.0 ** ((seed % 7 + 1) / 8.0)  # in (1, 2): never a power of two
        # (fraction, seed): after rounding the MTM offset heads' activation (oracle.offset_act), also move that
        # fraction of its elements by one bf16 ulp (random direction) -- another valid bf16 evaluation of the same
        # activation, as two correct kernels that round a few products differently produce (see offset_ulp_move)
        self.offset_ulp = offset_ulp
        self._offset_calls = 0

    def offset_ulp_move(self, x):
        """x (fp32, already on the bf16 grid) with max(1, round(fraction * numel)) elements moved one bf16 ulp up
        or down.  The elements and directions come from a generator seeded by (seed, call index), so a realization
        is reproducible; zeros are left alone (their neighbours are denormal)."""
        frac, seed = self.offset_ulp
        self._offset_calls += 1
        g = torch.Generator().manual_seed(1000003 * seed + self._offset_calls)
        flat = x.detach().reshape(-1).bfloat16().clone()
        n = max(1, int(round(frac * flat.numel())))
        idx = torch.randperm(flat.numel(), generator=g)[:n]
        step = torch.randint(0, 2, (n,), generator=g, dtype=torch.int16) * 2 - 1
        bits = flat.view(torch.int16)
        sel = bits[idx]
        nz = (sel & 0x7FFF) != 0
        bits[idx] = torch.where(nz, sel + step, sel)
        return flat.to(x.dtype).view(x.shape)

    def __call__(self, x):
        if self.seed is None:
            return x.bfloat16().to(x.dtype)
        xd = x.detach().double()
        out = (xd * self.s).bfloat16().double() / self.s
        # the rounding offset as a constant: x's autograd graph (the R1 double backward) passes through
        return x + (out.to(x.dtype) - x.detach())

    def st(self, t):
        """Straight-through: the value rounded, the gradient passed unchanged (oracle.round_bf16_st's role)."""
        return t + (self(t.detach()) - t.detach())

    def d_round(self):
        """The discriminator's rounding for oracle.train_step(d_round=...): image and effective weights
        straight-through, the two conv activations rounded in value and gradient (the device's bf16 h0 / h1 and
        their bf16 gradients g_a0 / g_a1, engine_d.py)."""
        return _DRound(self)


class _DRound:
    def __init__(self, rounder):
        self.rounder = rounder

    def __call__(self, t):
        return self.rounder.st(t)

    def act(self, t):
        return _RoundBoth.apply(t)


_ROUNDER = [Rounder()]  # the rounding _RoundBoth applies (bf16_module_rounding sets it)


class _RoundBoth(torch.autograd.Function):
    """bf16 rounding of a value and of the gradient flowing back through it."""

    @staticmethod
    def forward(ctx, x):
        return _ROUNDER[0](x)

    @staticmethod
    def backward(ctx, g):
        return _ROUNDER[0](g)


class _RoundBothOffset(torch.autograd.Function):
    """_RoundBoth for the offset heads' activation, with the rounder's one-ulp moves (Rounder.offset_ulp) applied to
    the rounded value."""

    @staticmethod
    def forward(ctx, x):
        r = _ROUNDER[0]
        y = r(x)
        return r.offset_ulp_move(y) if r.offset_ulp is not None else y

    @staticmethod
    def backward(ctx, g):
        return _ROUNDER[0](g)


class bf16_module_rounding:
    """Context manager: the tensors the bf16 device stores in bf16 -- module outputs (modulated convs, MTMs,
    convolution / attention blocks, expert FFNs, the MoE layer's combined output, multi-head attention outputs)
    and the block-internal activations that feed its MFMA GEMMs (LayerNorm outputs, the expert FFN's GELU'd hidden
    activation) -- are rounded to bf16 in the oracle, values and the gradients flowing back through them.  With
    ``d_round=oracle.round_bf16_st`` on the discriminator this gives the bf16 FLOOR of a whole step's gradients:
    how far bf16 storage alone, in otherwise exact fp32 arithmetic, moves them.  (The LayerNorm / GELU / MHA /
    MoE-output points are the device's bf16 tensors ``n1``/``n2``/``n3``, ``Hid``, the attention output and the
    combine output, engine_g.py; the oracle computes them in fp32.)"""
    NAMES = ("modconv", "mtm", "attention_block", "expert_ffn", "conv_block", "mha", "sparse_moe", "offset_act")
    VALUE_NAMES = ("warp",)  # stored in bf16, gradient kept fp32 (the MTM's warped map; g_xw is fp32, engine_g.py)
    FUNCS = ("layer_norm", "gelu")  # torch.nn.functional, as the oracle calls them inside the blocks

    def __init__(self, attention_internals=True, rounder=None):
        self.attention_internals = attention_internals
        self.rounder = rounder or Rounder()

    def __enter__(self):
        self.prev_rounder = _ROUNDER[0]
        _ROUNDER[0] = self.rounder
        self.orig = {n: getattr(O, n) for n in self.NAMES + self.VALUE_NAMES}
        self.orig_f = {n: getattr(O.F, n) for n in self.FUNCS}
        inner = dict(self.orig)
        if self.attention_internals:  # the multi-head attention with the MFMA kernel's bf16 operands (below)
            inner["mha"] = _mha_bf16_internals

        def wrapper(f, rb=_RoundBoth):
            def wrap(*a, **k):
                r = f(*a, **k)
                return (rb.apply(r[0]),) + tuple(r[1:]) if isinstance(r, tuple) else rb.apply(r)
            return wrap
        def value_wrapper(f):
            def wrap(*a, **k):
                return self.rounder.st(f(*a, **k))
            return wrap
        for n, f in inner.items():
            setattr(O, n, value_wrapper(f) if n in self.VALUE_NAMES else
                    wrapper(f, _RoundBothOffset if n == "offset_act" else _RoundBoth))
        for n, f in self.orig_f.items():
            setattr(O.F, n, wrapper(f))
        return self

    def __exit__(self, *exc):
        for n, f in self.orig.items():
            setattr(O, n, f)
        for n, f in self.orig_f.items():
            setattr(O.F, n, f)
        _ROUNDER[0] = self.prev_rounder
        return False


_ORACLE_MHA = O.mha


def _mha_bf16_internals(q_in, kv_in, P, pre, heads=8):
    """oracle.mha (nn.MultiheadAttention forward, t2i_moe_gan.py:545-555) with the tensors the device's attention
    path stores or feeds to its MFMAs in bf16 rounded (values and gradients): the q / k / v projections, the
    softmax probabilities (the P of P @ V; their gradient stands in for the kernel's bf16 dS) and the head outputs
    before the out-projection.  The cross-attention over the single text token runs in fp32 on the device (its
    softmax is 1: the value chain text_proj -> v -> out_proj, engine_g._block_vectors), so it is left exact."""
    import math
    if kv_in.shape[1] == 1:
        return _ORACLE_MHA(q_in, kv_in, P, pre, heads)
    r = _RoundBoth.apply
    B, Tq, C = q_in.shape
    Tk = kv_in.shape[1]
    Wi, bi = P[pre + "in_proj_weight"], P[pre + "in_proj_bias"]
    q = r(O.F.linear(q_in, Wi[:C], bi[:C]))
    k = r(O.F.linear(kv_in, Wi[C:2 * C], bi[C:2 * C]))
    v = r(O.F.linear(kv_in, Wi[2 * C:], bi[2 * C:]))
    d = C // heads
    q = q.view(B, Tq, heads, d).transpose(1, 2)
    k = k.view(B, Tk, heads, d).transpose(1, 2)
    v = v.view(B, Tk, heads, d).transpose(1, 2)
    att = r(torch.softmax((q / math.sqrt(d)) @ k.transpose(-1, -2), dim=-1))
    o = r((att @ v).transpose(1, 2).reshape(B, Tq, C))
    return O.F.linear(o, P[pre + "out_proj.weight"], P[pre + "out_proj.bias"])


class bf16_weights(dict):
    """The generator's parameter dict as the bf16 device reads it: the weights its MFMA kernels take as bf16
    operands (modulated / 1x1 / to_rgb conv weights, offset-head first conv, self-attention projections, expert
    FFNs) come back rounded to bf16 (straight-through: their gradient reaches the fp32 leaf unchanged); the fp32
    prefix (mapping, text projection, styles), routers, norms, biases and the cross-attention value chain stay
    fp32, as on the device (engine_g.py).  ``values()`` / ``items()`` still give the leaves, so the oracle's
    optimizer and gradient clipping are untouched.  A weight rounding is shared by every token of every image, so
    without it the floor misses the error that adds coherently over an image's tokens."""
    SUFFIXES = ("modulated_conv.weight", "skip_proj.weight", "proj_in.weight", "proj_out.weight",
                "offset_net.0.weight", "self_attn.in_proj_weight", "self_attn.out_proj.weight")

    rounder = None  # a Rounder (None: nearest-even, oracle.round_bf16_st)

    def __getitem__(self, n):
        v = dict.__getitem__(self, n)
        if (n.endswith(self.SUFFIXES) or (n.startswith("to_rgb_") and n.endswith(".weight")) or
                (".experts." in n and n.endswith((".net.0.weight", ".net.2.weight")))):
            return O.round_bf16_st(v) if self.rounder is None else self.rounder.st(v)
        return v


def mx_quant(x, dim, s=1.0):
    """OCP MX-fp8 of ``x`` as the device's mg_quant_mx8 forms it (csrc/mg_mx8.hip): blocks of 32 consecutive
    elements along ``dim`` share one power-of-two scale 2^e with e = ceil(log2(amax / 448)) (so nothing saturates),
    each element rounded to nearest-even e4m3 at that scale; returned dequantized, in x's dtype.  ``s`` != 1 is the
    rescaled-grid realization q(x * s) / s (Rounder's construction: the same error distribution, an independent
    pattern of which values round which way)."""
    xt = x.detach().movedim(dim, -1).double() * s
    shp = xt.shape
    assert shp[-1] % 32 == 0, shp
    xb = xt.reshape(*shp[:-1], shp[-1] // 32, 32)
    amax = xb.abs().amax(-1, keepdim=True)
    m, ex = torch.frexp(amax / 448.0)  # amax / 448 = m * 2^ex, m in [0.5, 1)
    e = torch.where(m == 0.5, ex - 1, ex)
    scale = torch.where(amax > 0, torch.ldexp(torch.ones_like(amax), e), torch.ones_like(amax))
    q = (xb / scale).float().to(torch.float8_e4m3fn).double() * scale
    return (q.reshape(shp) / s).movedim(-1, dim).to(x.dtype)


def _mx8_ok(c):
    """engine_g.GeneratorEngine._mx8_ok: the MX-fp8 conv reduces over 128-channel steps inside one tap."""
    return c >= 128 and c % 128 == 0 and (c & (c - 1)) == 0


class _MXConv3(torch.autograd.Function):
    """conv2d(xs, W, padding=1) with the operands the device's MX-fp8 path quantizes (engine_g.mc_fwd / mc_bwd):
    forward x*s and the packed weight (blocks along Cin per output channel and tap) when Cin qualifies; the data
    gradient's output gradient and the flipped weight (blocks along Cout per input channel and tap) when Cout
    qualifies.  The weight gradient takes the unquantized operands (bf16 on the device)."""

    @staticmethod
    def forward(ctx, xs, W, s):
        ctx.save_for_backward(xs, W)
        ctx.s = s
        Cout, Cin = W.shape[:2]
        if _mx8_ok(Cin):
            return torch.nn.functional.conv2d(mx_quant(xs, 1, s), mx_quant(W, 1, s), padding=1)
        return torch.nn.functional.conv2d(xs, W, padding=1)

    @staticmethod
    def backward(ctx, g):
        xs, W = ctx.saved_tensors
        s = ctx.s
        if _mx8_ok(W.shape[0]):
            gx = torch.nn.grad.conv2d_input(xs.shape, mx_quant(W, 0, s), mx_quant(g, 1, s), padding=1)
        else:
            gx = torch.nn.grad.conv2d_input(xs.shape, W, g, padding=1)
        gW = torch.nn.grad.conv2d_weight(xs, W.shape, g, padding=1)
        return gx, gW, None


class mx8_modconv_rounding:
    """Context manager: oracle.modconv's 3x3 modulated convs evaluated as the MX-fp8 device path computes them --
    y = d * conv(q(x * s), q(W)) (d the demodulation, s the style), data gradient conv(q(g), q(W_flip)) -- so an
    oracle step run inside it (together with bf16_module_rounding / bf16_weights / d_round) gives the MX-fp8 step's
    FLOOR: how far the precision the device stores and multiplies in moves each gradient, in otherwise exact fp32
    arithmetic.  The factorisation (style on the activation, demodulation on the output) is the reference's math
    (t2i_moe_gan.py:158-180) regrouped; only where the quantization sits depends on it.  ``rounder``: a Rounder whose
    grid scale gives the realization (nearest-even grid for Rounder())."""

    def __init__(self, rounder=None):
        self.s = (rounder or Rounder()).s

    def __enter__(self):
        self.orig = O.modconv
        orig, s = self.orig, self.s

        def modconv(x, w, P, pre, padding=0, demod=True):
            weight = P[pre + "weight"]
            Cout, Cin, k, _ = weight.shape
            if k != 3 or padding != 1 or not demod or not (_mx8_ok(Cin) or _mx8_ok(Cout)):
                return orig(x, w, P, pre, padding, demod)
            B = x.shape[0]
            style = O.F.linear(w, P[pre + "modulation.weight"], P[pre + "modulation.bias"])  # :158
            d = torch.rsqrt((weight.unsqueeze(0) * style.view(B, 1, Cin, 1, 1)).pow(2).sum(dim=(2, 3, 4)) + 1e-8)
            y = _MXConv3.apply(x * style.view(B, Cin, 1, 1), weight, s)
            return y * d.view(B, Cout, 1, 1)
        O.modconv = modconv
        return self

    def __exit__(self, *exc):
        O.modconv = self.orig
        return False


def whole(grads, names=None):
    """One vector of every gradient in ``grads`` (dict name -> tensor or None), in a fixed name order."""
    names = sorted(n for n, v in grads.items() if v is not None) if names is None else names
    return torch.cat([grads[n].reshape(-1) for n in names]), names


# ---------------------------------------------------------------------------------------------------------------
# Router-temperature instrumentation (t2i_moe_gan.py:374-377: logits / clamp(temperature * anneal, .5, 5)).  The
# scalar gradient is a cancelling sum over tokens of -anneal / te * sum_e dL/dl[t, e] * l[t, e]; the taps below
# expose its per-token terms on both sides so a test can hold the sum to a floor derived from those terms.
# ---------------------------------------------------------------------------------------------------------------
BLOCK_OF_HW = {16: "gen_block_4", 64: "gen_block_8", 256: "gen_block_16"}


def router_temp_terms(z, topi, g_gate, coef, te, anneal, k, parts=False):
    """fp64 restatement of k_router_bwd's temperature term per token from the kernel's own inputs (scaled logits
    z [T,E], selection topi [T,k], gate gradient [T,k], balance coefficients [E] or None); returns [T] (``parts``:
    also the logit gradient dL/dz [T,E] the term contracts with z)."""
    z = z.double()
    T, E = z.shape
    s = torch.softmax(z.clamp(-20, 20), dim=1)
    q = s.clamp(1e-6, 1.0)
    Sq = q.sum(1, keepdim=True)
    p = q / Sq
    gp = torch.zeros(T, E, dtype=torch.float64)
    if coef is not None:
        gp += coef.double().view(1, E)
    ti, gg = topi.long(), g_gate.double()
    if k == E:
        gp.scatter_add_(1, ti, gg)
    else:
        psel = p.gather(1, ti)
        S = psel.sum(1, keepdim=True)
        dot = (gg * (psel / S)).sum(1, keepdim=True)
        gp.scatter_add_(1, ti, (gg - dot) / S)
    d1 = (gp * p).sum(1, keepdim=True)
    gs = torch.where((s >= 1e-6) & (s <= 1.0), (gp - d1) / Sq, torch.zeros_like(gp))
    gl = s * (gs - (gs * s).sum(1, keepdim=True))
    gl = torch.where((z >= -20) & (z <= 20), gl, torch.zeros_like(gl))
    terms = -(gl * z).sum(1) / te * anneal
    return (terms, gl) if parts else terms


class DeviceTempTap:
    """Keeps, per MoE block, the inputs of the device's router backward (ops.router_bwd) and the temperature
    gradient it writes.  References, not copies: under hipGraph capture they are the graph's static buffers, so
    ``results()`` read after a replay sees the replayed values; eagerly they are that step's tensors.  Assumes the
    temperature gradient is zeroed at the start of the G phase (gradient_accumulation_steps = 1), so after the
    step it holds exactly the router backward kernel's fold."""

    def __init__(self):
        self.rec = {}

    def __enter__(self):
        from moegan_mi import ops
        self.ops, self.orig = ops, ops.router_bwd

        def rb(probs, zlog, topi, gate, g_gate, g_probs, coef, HW, temperature, anneal, g_temp, Bn, g_logits=None):
            # the temperature as it is now (an enqueued copy: the optimizer updates the parameter later in the step)
            self.rec[BLOCK_OF_HW.get(HW, HW)] = dict(zlog=zlog, topi=topi, g_gate=g_gate, coef=coef,
                                                     temperature=temperature.detach().clone(), anneal=anneal,
                                                     g_temp=g_temp)
            return self.orig(probs, zlog, topi, gate, g_gate, g_probs, coef, HW, temperature, anneal, g_temp, Bn,
                             g_logits)
        ops.router_bwd = rb
        return self

    def __exit__(self, *exc):
        self.ops.router_bwd = self.orig
        return False

    def results(self):
        """{block: dict(terms=[T] fp64 restatement from the kernel's inputs, kernel=its fold)}."""
        torch.cuda.synchronize()
        out = {}
        for blk, r in self.rec.items():
            te = min(max(float(r["temperature"].detach().cpu()[0]) * r["anneal"], 0.5), 5.0)
            k = r["topi"].shape[1]
            z = r["zlog"].detach().cpu()
            terms, gl = router_temp_terms(z, r["topi"].detach().cpu(), r["g_gate"].detach().float().cpu(),
                                          None if r["coef"] is None else r["coef"].detach().cpu(), te, r["anneal"], k,
                                          parts=True)
            out[blk] = dict(terms=terms, kernel=float(r["g_temp"].detach().cpu()[0]), z=z.double(), gl=gl,
                            scale=-r["anneal"] / te)
        return out


class OracleTempTap:
    """Keeps the oracle router's scaled logits of the gradient-carrying (G-phase) forward of every block, so the
    per-token temperature terms can be read after the backward (``terms(block)``)."""

    def __init__(self):
        self.store = {}

    def __enter__(self):
        self.orig = O.router
        store = self.store

        def router(feature, text, P, pre, eps=None, training=True, anneal=1.0):
            wf = O.reparam(P[pre + "feature_mu"], P[pre + "feature_rho"], eps[0])
            wt = O.reparam(P[pre + "text_mu"], P[pre + "text_rho"], eps[1])
            wc = O.reparam(P[pre + "combined_mu"], P[pre + "combined_rho"], eps[2])
            t_eff = (P[pre + "temperature"] * anneal).clamp(0.5, 5.0)  # :375
            raw = (torch.cat([feature @ wf, text @ wt], dim=1) @ wc) / t_eff
            logits = raw.clamp(-20.0, 20.0)  # :378
            if logits.requires_grad:
                logits.retain_grad()
                store[pre.split(".")[0]] = dict(logits=logits, raw=raw.detach(), t_eff=float(t_eff.detach()),
                                                anneal=anneal)
            probs = torch.softmax(logits, dim=1).clamp(1e-6, 1.0)
            return probs / probs.sum(dim=1, keepdim=True), logits
        assert training_router_matches(self.orig, router)
        O.router = router
        return self

    def __exit__(self, *exc):
        O.router = self.orig
        return False

    def parts(self, block):
        """(scaled logits z [T,E] before the clamp -- the device's zlog --, the gradient dL/dz that reaches them
        [T,E], -anneal / t_eff) of the block's G-phase router.  The clamp to [-20, 20] (:378) passes no gradient
        where it is active, so there the temperature receives nothing: dL/dz is zeroed where |z| > 20 (the clamp
        output's own gradient is not)."""
        s = self.store[block]
        z = s["raw"].double()
        gl = torch.where((z >= -20.0) & (z <= 20.0), s["logits"].grad.double(), torch.zeros_like(z))
        return z, gl, -s["anneal"] / s["t_eff"]

    def terms(self, block):
        z, gl, sc = self.parts(block)
        return sc * (gl * z).sum(1)


def training_router_matches(orig, tapped):
    """The tap re-states the oracle's training router; check it agrees with the oracle on a small random case."""
    g = torch.Generator().manual_seed(5)
    C, E, T = 16, 4, 8
    P = {"r.feature_mu": torch.randn(C, 128, generator=g) * 0.1, "r.feature_rho": torch.full((C, 128), -4.0),
         "r.text_mu": torch.randn(512, 128, generator=g) * 0.1, "r.text_rho": torch.full((512, 128), -4.0),
         "r.combined_mu": torch.randn(256, E, generator=g) * 0.1, "r.combined_rho": torch.full((256, E), -4.0),
         "r.temperature": torch.tensor([1.0])}
    eps = (torch.randn(C, 128, generator=g), torch.randn(512, 128, generator=g), torch.randn(256, E, generator=g))
    f, t = torch.randn(T, C, generator=g), torch.randn(T, 512, generator=g)
    a, b = orig(f, t, P, "r.", eps, True, 3.0), tapped(f, t, P, "r.", eps, True, 3.0)
    return torch.allclose(a[0], b[0], atol=1e-6) and torch.allclose(a[1], b[1], atol=1e-5)


# ---------------------------------------------------------------------------------------------------------------
# hipGraph replay of the product step, exactly as bench.py runs it (SegmentedGraph: warm-up on the capture stream,
# capture, replay with fixed input buffers)
# ---------------------------------------------------------------------------------------------------------------
def step_state(ts):
    """Every device tensor a training step reads and updates (parameters, moments, bf16 shadow, AdamW step
    counters, the accumulation-window word)."""
    ts_ = []
    for st in (ts.gs, ts.ds):
        ts_ += [st.data, st.m, st.v, st.step_dev, st.step_dev_kl] + ([st.shadow] if st.shadow is not None else [])
    return ts_ + [ts.win]


def snapshot(ts):
    return [t.detach().clone() for t in step_state(ts)]


def restore(ts, snap):
    with torch.no_grad():
        for t, s in zip(step_state(ts), snap):
            t.copy_(s)


class ReplayedStep:
    """Captures ``ts.step`` on fixed input buffers the way bench.py does and replays it.  The warm-up step that
    sizes every lazily allocated buffer changes the model; the state from before it is restored after the
    capture, so the first replay starts where an eager step would."""

    def __init__(self, ts, real, text, z, eps_d, eps_g, perm, tap=None, **kw):
        from moegan_mi.graphs import SegmentedGraph
        self.ts = ts
        dev = ts.dev
        self.buf = dict(real=real.to(dev).clone(), text=text.to(dev).clone(), z=z.to(dev).clone(),
                        eps_d=[tuple(t.to(dev).clone() for t in e) for e in eps_d],
                        eps_g=[tuple(t.to(dev).clone() for t in e) for e in eps_g],
                        perm=perm.to(dev).int().clone())
        b = self.buf
        fn = lambda: ts.step(b["real"], b["text"], b["z"], b["eps_d"], b["eps_g"], b["perm"], **kw)  # noqa: E731
        snap = snapshot(ts)
        self.graph = SegmentedGraph()
        self.graph.run_eager(fn)
        torch.cuda.synchronize()
        if tap is not None:
            with tap:
                self.out = self.graph.capture(fn)
        else:
            self.out = self.graph.capture(fn)
        torch.cuda.synchronize()
        restore(ts, snap)

    def __call__(self, real, text, z, eps_d, eps_g, perm):
        b = self.buf
        with torch.no_grad():
            b["real"].copy_(real)
            b["text"].copy_(text)
            b["z"].copy_(z)
            for dst, src in ((b["eps_d"], eps_d), (b["eps_g"], eps_g)):
                for td, tsrc in zip(dst, src):
                    for x, y in zip(td, tsrc):
                        x.copy_(y)
            b["perm"].copy_(perm.int())
        self.graph.replay()
        torch.cuda.synchronize()
        return self.out



class lrelu_slope_replay:
    """Record the device generator's MTM pre-activation signs (GeneratorEngine.mtm_fwd calls that save for the
    backward) and replay them in the oracle (aurora_cpu.LRELU_SLOPES): the LeakyReLU kink is a discrete decision,
    replayed like the top-k routes.

        with lrelu_slope_replay() as slopes:
            ... device step (or the eager warm-up + capture of a ReplayedStep) ...
        with slopes.oracle():
            ... oracle forward/backward ...

    The recorder keeps the saved tensors themselves (the pre-activation for a residual-fused MTM, the output
    otherwise -- same sign) and reads them when ``oracle()`` is entered: after a hipGraph replay they hold that
    replay's values (held references keep the capture's allocator from reusing their memory)."""

    def __init__(self):
        self.refs = {}

    def __enter__(self):
        from moegan_mi.engine_g import GeneratorEngine
        self._cls = GeneratorEngine
        self._orig = orig = GeneratorEngine.mtm_fwd
        refs = self.refs

        def mtm_fwd(eng, pre, x, w, resid=None, save=True):
            y, sv = orig(eng, pre, x, w, resid=resid, save=save)
            if save:
                msv = sv[4]
                z, zsub, act = msv[6], msv[7], msv[8]
                assert act in (1, 2) and zsub is None, (pre, act)  # act 2: z = pre-activation; act 1: z = output
                refs[pre] = (z, tuple(x.shape[:3]), eng.P(pre + "modulated_conv.weight").shape[0])
            return y, sv
        GeneratorEngine.mtm_fwd = mtm_fwd
        return self

    def __exit__(self, *exc):
        self._cls.mtm_fwd = self._orig

    def masks(self):
        out = {}
        for pre, (z, (B, H, W), Cout) in self.refs.items():
            zz = z.reshape(B * H * W, -1)[:, :Cout].float()
            out[pre] = (zz > 0).view(B, H, W, Cout).permute(0, 3, 1, 2).cpu()
        return out

    class _Oracle:
        def __init__(self, masks):
            self.m = masks

        def __enter__(self):
            O.LRELU_SLOPES = self.m

        def __exit__(self, *exc):
            O.LRELU_SLOPES = None

    def oracle(self):
        return self._Oracle(self.masks())
