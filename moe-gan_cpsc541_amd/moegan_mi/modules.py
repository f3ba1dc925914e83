"""The reference's sub-module classes (t2i_moe_gan.py:122-666) as nn.Modules on the HIP engine.

Each class has the reference constructor signature, the reference ``state_dict`` keys and shapes (so weights
move between the two freely) and the reference forward signature and return values; its math runs on the same
GeneratorEngine code paths the fused training step uses (engine_g.py), through one torch.autograd.Function per
module: forward and backward are the engine's explicit passes, the parameter gradient comes back as the gradient
of the module's single flat parameter.

Layout: like AuroraGenerator, a module keeps its parameters in ONE flat store.  Internally the names carry a
prefix (``_IPRE``) that gives the engine the names it expects (the experts of a SparseMoE live under
``...moe.experts.*`` so the grouped expert GEMMs read them contiguously); ``state_dict`` strips it.  Children
are not separate nn.Modules (``block.conv_block`` is not an attribute) -- the keys are what checkpoints need.

Modes and limits (the reference's usage, checked): ModulatedConv demodulates, pads k // 2 and does not
upsample (the reference never instantiates anything else); multi-head attention has 8 heads; eval-mode (hard
top-1) SparseMoE / AttentionBlock / router outputs are forward-only.  Inputs are NCHW fp32 like the reference;
``dtype="bf16"`` runs the engine's bf16 storage mode.  There is no CPU path: forward needs a HIP device.
"""
from collections import OrderedDict

import torch
import torch.nn as nn

from . import _lib as L
from . import ops
from .engine_g import GeneratorEngine
from .init import init_generator
from .layout import is_buffer
from .params import ParamStore

LATENT_DIM = 512
E_ = ops.E


def _nhwc(x, dtype):
    return x.permute(0, 2, 3, 1).contiguous().to(dtype)


def _nchw(y, C):
    return y[..., :C].permute(0, 3, 1, 2).float().contiguous()


def _pad_rows(g_nchw, rows, dtype):
    B, C, H, W = g_nchw.shape
    g = torch.zeros(B, H, W, rows, device=g_nchw.device, dtype=dtype)
    g[..., :C] = g_nchw.permute(0, 2, 3, 1)
    return g


def _mc_shapes(cin, cout, k, latent, pre=""):
    return [(pre + "weight", (cout, cin, k, k)), (pre + "modulation.weight", (cin, latent)),
            (pre + "modulation.bias", (cin,))]


def _mtm_shapes(cin, cout, k, latent, offsets, pre=""):
    sh = _mc_shapes(cin, cout, k, latent, pre + "modulated_conv.")
    if offsets:
        sh += [(pre + "offset_net.0.weight", (32, cin, 3, 3)), (pre + "offset_net.0.bias", (32,)),
               (pre + "offset_net.2.weight", (2, 32, 3, 3)), (pre + "offset_net.2.bias", (2,))]
    return sh


def _router_shapes(feat, text, E, pre=""):
    return [(pre + "feature_mu", (feat, 128)), (pre + "feature_rho", (feat, 128)), (pre + "text_mu", (text, 128)),
            (pre + "text_rho", (text, 128)), (pre + "combined_mu", (256, E)), (pre + "combined_rho", (256, E)),
            (pre + "temperature", (1,)),  # parameters, then the noise buffers: torch's state_dict order
            (pre + "epsilon_f", (feat, 128)), (pre + "epsilon_t", (text, 128)), (pre + "epsilon_c", (256, E))]


def _moe_shapes(dim, text, E, pre=""):
    sh = []
    for e in range(E):
        p = f"{pre}experts.{e}.net."
        sh += [(p + "0.weight", (4 * dim, dim)), (p + "0.bias", (4 * dim,)), (p + "2.weight", (dim, 4 * dim)),
               (p + "2.bias", (dim,))]
    return sh + _router_shapes(dim, text, E, pre + "router.")


def _attn_shapes(dim, text, E, latent, pre=""):
    sh = [(pre + n + "." + w, (dim,)) for n in ("norm1", "norm2", "norm3") for w in ("weight", "bias")]
    sh += [(pre + "text_proj.weight", (dim, text)), (pre + "text_proj.bias", (dim,))]
    for a in ("self_attn", "cross_attn"):
        sh += [(pre + a + ".in_proj_weight", (3 * dim, dim)), (pre + a + ".in_proj_bias", (3 * dim,)),
               (pre + a + ".out_proj.weight", (dim, dim)), (pre + a + ".out_proj.bias", (dim,))]
    sh += _moe_shapes(dim, text, E, pre + "moe.")
    sh += _mc_shapes(dim, dim, 1, latent, pre + "proj_in.") + _mc_shapes(dim, dim, 1, latent, pre + "proj_out.")
    return sh


def _cb_shapes(cin, cout, latent, offsets, pre=""):
    sh = _mtm_shapes(cin, cout, 3, latent, offsets, pre + "mtm1.") + _mtm_shapes(cout, cout, 3, latent, offsets,
                                                                               pre + "mtm2.")
    if cin != cout:
        sh += _mc_shapes(cin, cout, 1, latent, pre + "skip_proj.")
    return sh


class _EngineModule(nn.Module):
    """Base: one flat parameter over a ParamStore with internally prefixed names; reference state_dict."""
    _IPRE = ""

    def __init__(self, shapes, E=4, topk=None, dtype="fp32", seed=0, modconvs=(), offset_nets=()):
        super().__init__()
        ip = self._IPRE
        cdt = torch.bfloat16 if dtype == "bf16" else torch.float32
        self._store = ParamStore(OrderedDict((ip + k, tuple(v)) for k, v in shapes), "cpu", shadow_dtype=cdt)
        self.flat = nn.Parameter(self._store.data)
        self._cdt = cdt
        self._E, self._topk = E, topk
        self._mc = [(ip + p, k) for p, k in modconvs]
        self._off = [ip + p for p in offset_nets]
        self._eng = None
        init_generator(self._store, seed)

    # ---- parameters / state dict in the reference's names ----
    def _apply(self, fn, recurse=True):
        super()._apply(fn, recurse)
        self._store.rebind(self.flat.data)
        return self

    def state_dict(self, *args, destination=None, prefix="", keep_vars=False):
        n = len(self._IPRE)
        sd = OrderedDict((prefix + k[n:], v) for k, v in self._store.state_dict(cpu=False).items())
        if destination is not None:
            destination.update(sd)
            return destination
        return sd

    def load_state_dict(self, state_dict, strict=True, assign=False):
        self._store.load_state_dict({self._IPRE + k: v for k, v in state_dict.items()}, strict)
        return nn.modules.module._IncompatibleKeys([], [])

    def named_reference_parameters(self):
        """(name, tensor view) pairs in the reference's parameter order (views into ``flat``)."""
        n = len(self._IPRE)
        for k in self._store.shapes:
            if not is_buffer(k):
                yield k[n:], self._store.view(k)

    # ---- engine ----
    def _engine(self):
        if not self.flat.is_cuda:
            raise RuntimeError(f"{type(self).__name__}: the MI355X path runs on a HIP device; move the module with "
                               ".to('cuda') (the CPU restatement in oracle/ is test infrastructure)")
        if self._eng is None or self._eng.st is not self._store or self._eng.dev != self._store.device:
            self._eng = GeneratorEngine(self._store, self._E, self._topk, self._cdt, modconvs=self._mc,
                                        offset_nets=self._off)
        return self._eng

    def _eps(self, router_pre):
        """Fresh router noise, drawn into the epsilon buffers as the reference does (:349-351)."""
        out = []
        for n in ("epsilon_f", "epsilon_t", "epsilon_c"):
            b = self._store.buffers[self._IPRE + router_pre + n]
            b.normal_()
            out.append(b)
        return tuple(out)

    def _grad_out(self):
        return self._store.grad.clone()


# ---------------------------------------------------------------------------
# ModulatedConv (t2i_moe_gan.py:122-186)
# ---------------------------------------------------------------------------
class _MCFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, w, mod):
        eng = mod._engine()
        eng.prep()
        y, sv = eng.mc_fwd(mod._IPRE, _nhwc(x, mod._cdt), w.float().contiguous(), act=0)
        ctx.mod, ctx.sv, ctx.rows = mod, sv, y.shape[-1]
        return _nchw(y, mod.out_channels)

    @staticmethod
    def backward(ctx, gy):
        mod, eng = ctx.mod, ctx.mod._engine()
        mod._store.zero_grad()
        x = ctx.sv[0]
        gx = torch.empty(x.shape, device=x.device, dtype=mod._cdt)
        gw = torch.zeros(x.shape[0], mod.latent_dim, device=x.device)
        eng.mc_bwd(mod._IPRE, ctx.sv, _pad_rows(gy, ctx.rows, mod._cdt), gx, gw)
        return mod._grad_out(), gx.permute(0, 3, 1, 2).float(), gw, None


class ModulatedConv(_EngineModule):
    """Reference :122-186.  y = conv(x, W * style(w) * demod) with per-sample weights, as the fused
    d * conv(x * s, W)."""

    def __init__(self, in_channels, out_channels, kernel_size, latent_dim=LATENT_DIM, stride=1, padding=0,
                 demodulate=True, upsample=False, dtype="fp32", seed=0):
        if stride != 1 or not demodulate or upsample or kernel_size not in (1, 3):
            raise NotImplementedError("ModulatedConv: 1x1 / 3x3, stride 1, demodulated, no upsampling (the reference's "
                                      "usage)")
        super().__init__(_mc_shapes(in_channels, out_channels, kernel_size, latent_dim), dtype=dtype, seed=seed,
                         modconvs=[("", kernel_size)])
        self.in_channels, self.out_channels, self.kernel_size = in_channels, out_channels, kernel_size
        self.latent_dim, self.stride, self.padding = latent_dim, stride, padding
        self.demodulate, self.upsample = demodulate, upsample

    def forward(self, x, w):
        if self.padding != self.kernel_size // 2:  # the reference's default padding=0 on a 3x3 is never used
            raise NotImplementedError("ModulatedConv: 'same' padding (kernel_size // 2), as every reference use; "
                                      f"got padding={self.padding}")
        return _MCFn.apply(self.flat, x, w, self)


# ---------------------------------------------------------------------------
# ModulatedTransformationModule (t2i_moe_gan.py:188-247)
# ---------------------------------------------------------------------------
def _mtm_fwd(eng, pre, x, w, offsets, resid=None):
    if offsets:
        return eng.mtm_fwd(pre, x, w, resid=resid)
    return eng.mc_fwd(pre + "modulated_conv.", x, w, act=1, resid=resid)


def _mtm_bwd(eng, pre, sv, gz, gx, gw, offsets, accumulate=0):
    if offsets:
        eng.mtm_bwd(pre, sv, gz, gx, gw, accumulate=accumulate)
    else:
        eng.mc_bwd(pre + "modulated_conv.", sv, gz, gx, gw, accumulate=accumulate)


class _MTMFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, w, mod):
        eng = mod._engine()
        eng.prep()
        xh = _nhwc(x, mod._cdt)
        y, sv = _mtm_fwd(eng, mod._IPRE, xh, w.float().contiguous(), mod.use_offset)
        ctx.mod, ctx.sv, ctx.xshape, ctx.rows = mod, sv, xh.shape, y.shape[-1]
        return _nchw(y, mod.out_channels)

    @staticmethod
    def backward(ctx, gy):
        mod, eng = ctx.mod, ctx.mod._engine()
        mod._store.zero_grad()
        dev = gy.device
        gx = torch.empty(ctx.xshape, device=dev, dtype=mod._cdt)
        gw = torch.zeros(ctx.xshape[0], mod.latent_dim, device=dev)
        _mtm_bwd(eng, mod._IPRE, ctx.sv, _pad_rows(gy, ctx.rows, mod._cdt), gx, gw, mod.use_offset)
        return mod._grad_out(), gx.permute(0, 3, 1, 2).float(), gw, None


class ModulatedTransformationModule(_EngineModule):
    """Reference :188-247: offsets (offset_net) -> linspace grid -> grid_sample -> modulated conv -> LeakyReLU."""

    def __init__(self, in_channels, out_channels, kernel_size=3, latent_dim=LATENT_DIM, use_offset=False,
                 resolution=None, dtype="fp32", seed=0):
        if kernel_size != 3:
            raise NotImplementedError("ModulatedTransformationModule: kernel_size 3 (the reference's usage)")
        offsets = bool(use_offset and resolution is not None and resolution <= 16)  # :199
        super().__init__(_mtm_shapes(in_channels, out_channels, 3, latent_dim, offsets), dtype=dtype, seed=seed,
                         modconvs=[("modulated_conv.", 3)], offset_nets=["offset_net.0."] if offsets else [])
        self.in_channels, self.out_channels, self.latent_dim = in_channels, out_channels, latent_dim
        self.use_offset = offsets

    def forward(self, x, w):
        return _MTMFn.apply(self.flat, x, w, self)


# ---------------------------------------------------------------------------
# SparseExpertFFN (t2i_moe_gan.py:249-263)
# ---------------------------------------------------------------------------
class _FFNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, mod):
        st = mod._store
        st.refresh_shadow()
        dim = mod.dim
        lead = x.shape[:-1]
        xt = x.reshape(-1, dim).to(mod._cdt).contiguous()
        n = xt.shape[0]
        pre = torch.empty(n, 4 * dim, device=x.device, dtype=mod._cdt)
        h = ops.linear(xt, st.cview("net.0.weight"), bias=st.view("net.0.bias"), act=L.ACT_GELU, out_pre=pre,
                       ld_pre=4 * dim)
        y = ops.linear(h, st.cview("net.2.weight"), bias=st.view("net.2.bias"))
        ctx.mod, ctx.saved_ = mod, (xt, pre, h)
        return y.float().reshape(*lead, dim)

    @staticmethod
    def backward(ctx, gy):
        mod = ctx.mod
        st = mod._store
        st.zero_grad()
        xt, pre, h = ctx.saved_
        dim, n = mod.dim, xt.shape[0]
        g = gy.reshape(-1, dim).to(mod._cdt).contiguous()
        gp = ops.gemm(g, st.cview("net.2.weight"), n, 4 * dim, dim, b_kc=False,
                      ep=E_(act=L.ACT_MUL_GELU_GRAD, aux=pre, ld_aux=4 * dim))  # d pre = (g W2) * GELU'(pre)
        ops.linear_wgrad(g, h, st.gview("net.2.weight"))
        ops.colsum(g, st.gview("net.2.bias"))
        gx = ops.linear_dgrad(gp, st.cview("net.0.weight"), out_dtype=torch.float32)
        ops.linear_wgrad(gp, xt, st.gview("net.0.weight"))
        ops.colsum(gp, st.gview("net.0.bias"))
        return mod._grad_out(), gx.reshape(gy.shape), None


class SparseExpertFFN(_EngineModule):
    """Reference :249-263: Linear(dim, 4 dim) -> exact GELU -> Linear(4 dim, dim) on MFMA GEMMs (GELU and GELU'
    fused into the GEMM epilogues)."""

    def __init__(self, dim, dtype="fp32", seed=0):
        super().__init__([("net.0.weight", (4 * dim, dim)), ("net.0.bias", (4 * dim,)),
                          ("net.2.weight", (dim, 4 * dim)), ("net.2.bias", (dim,))], dtype=dtype, seed=seed)
        self.dim = dim

    def forward(self, x):
        if not self.flat.is_cuda:
            self._engine()  # raises with the device message
        return _FFNFn.apply(self.flat, x, self)


# ---------------------------------------------------------------------------
# BayesianRouter (t2i_moe_gan.py:265-423)
# ---------------------------------------------------------------------------
class _RouterFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, feature, text, mod, sampling, anneal):
        eng = mod._engine()
        r = mod._IPRE
        feat = feature.float().contiguous()
        txt = text.float().contiguous()
        T, C = feat.shape
        E = mod.num_experts
        eps = mod._eps("") if sampling else None
        Wf, Wt, Wc = eng._router_weights(r, eps, sampling)  # reparameterised (:302-333) or the means
        Wfc = ops.gemm(Wf, Wc[:128], C, E, 128, b_kc=False)
        u = ops.gemm(txt, Wt, T, 128, txt.shape[1], b_kc=False)
        Lt = ops.gemm(u, Wc[128:], T, E, 128, b_kc=False)  # per-token text logits (HW = 1 below)
        probs, zlog, topi, gate = ops.router_fwd(feat, Wfc, Lt, E, E if sampling else 1, 1, eng.P(r + "temperature"),
                                                 anneal, eval_mode=0 if sampling else 1)
        logits = zlog.clamp(-20.0, 20.0)  # :378-381
        ctx.mod, ctx.sampling, ctx.anneal = mod, sampling, anneal
        ctx.keep = (feat, txt, Wf, Wt, Wc, Wfc, u, probs, zlog, topi, gate, eps)
        if not sampling:  # eval: one-hot of the top-1 (:392-400), forward only
            ctx.mark_non_differentiable(probs, logits)
        return probs, logits

    @staticmethod
    def backward(ctx, g_probs, g_logits):
        mod, eng = ctx.mod, ctx.mod._engine()
        if not ctx.sampling:
            raise NotImplementedError("BayesianRouter: eval-mode (hard top-1) outputs are forward-only")
        st = mod._store
        st.zero_grad()
        feat, txt, Wf, Wt, Wc, Wfc, u, probs, zlog, topi, gate, eps = ctx.keep
        T, C = feat.shape
        E = mod.num_experts
        r = mod._IPRE
        gp = None if g_probs is None else g_probs.float().contiguous()
        gl = None if g_logits is None else g_logits.float().contiguous()
        g_raw, gsum = ops.router_bwd(probs, zlog, topi, gate, None, gp, None, 1, eng.P(r + "temperature"), ctx.anneal,
                                     eng.G(r + "temperature"), T, g_logits=gl)
        g_feat = torch.empty(T, C, device=feat.device)
        ops.moe_token_grad(None, None, g_raw, Wfc, g_feat, 1)
        G1 = torch.zeros(C, E, device=feat.device)
        ops.router_feat_grad(feat, g_raw, G1)
        g_text = torch.zeros_like(txt)
        eng._router_bwd = [dict(r=r, C=C, E=E, B=T, G1=G1, gsum=gsum, Wf=Wf, Wt=Wt, Wc=Wc, u=u, w=txt, gw=g_text,
                                eps=eps, kl_coef=None)]
        eng._flush_router_bwd()
        return mod._grad_out(), g_feat, g_text, None, None, None


class _RouterKLFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, mod):
        eng = mod._engine()
        r = mod._IPRE
        kl2 = torch.empty(2, device=flat.device)
        ops.router_kl(eng.P(r + "feature_mu"), eng.P(r + "feature_rho"), eng.P(r + "text_mu"),
                      eng.P(r + "text_rho"), eng.P(r + "combined_mu"), eng.P(r + "combined_rho"), kl2)
        ctx.mod, ctx.kl2 = mod, kl2
        return kl2[0].clone()

    @staticmethod
    def backward(ctx, g):
        mod, eng = ctx.mod, ctx.mod._engine()
        st = mod._store
        st.zero_grad()
        coef = (g.float().reshape(1) * ctx.kl2[1:2]).contiguous()  # no gradient through the nan/clamp (:417-421)
        r = mod._IPRE
        for n in ("feature", "text", "combined"):
            ops.router_param_bwd(eng.P(r + n + "_mu"), eng.P(r + n + "_rho"), None, None, coef, eng.G(r + n + "_mu"),
                                 eng.G(r + n + "_rho"))
        return mod._grad_out(), None


class BayesianRouter(_EngineModule):
    """Reference :265-423: weight-uncertainty projections sampled by reparameterisation, temperature-scaled
    clamped softmax, eval-mode top-1 one-hot, closed-form KL."""

    def __init__(self, feature_dim, text_dim, num_experts=4, dtype="fp32", seed=0):
        super().__init__(_router_shapes(feature_dim, text_dim, num_experts), E=num_experts, dtype=dtype, seed=seed)
        self.feature_dim, self.text_dim, self.num_experts = feature_dim, text_dim, num_experts

    def forward(self, feature, text_embedding, sampling=True, annealing_factor=1.0):
        return _RouterFn.apply(self.flat, feature, text_embedding, self, bool(sampling), float(annealing_factor))

    def kl_divergence(self):
        return _RouterKLFn.apply(self.flat, self)


# ---------------------------------------------------------------------------
# SparseMoE (t2i_moe_gan.py:426-491)
# ---------------------------------------------------------------------------
class _MoEFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, w, mod, anneal, train):
        eng = mod._engine()
        eng.prep()
        B, C, H, W = x.shape
        tok = _nhwc(x, mod._cdt).view(B * H * W, C)
        eps = mod._eps("router.") if train else None
        eng._want_kl = True
        out, probs, kl2, topi, sv = eng.moe_fwd(mod._IPRE, tok, None, w.float().contiguous(), H * W, eps, anneal,
                                                train=train, save=train)
        ctx.mod, ctx.sv, ctx.kl2, ctx.shape = mod, sv, kl2, (B, C, H, W)
        kl = kl2[0].clone() if train else torch.zeros((), device=x.device)
        if not train:
            ctx.mark_non_differentiable(kl, probs)
        return out.view(B, H, W, C).permute(0, 3, 1, 2).float().contiguous(), kl, probs

    @staticmethod
    def backward(ctx, g_out, g_kl, g_probs):
        mod, eng = ctx.mod, ctx.mod._engine()
        if ctx.sv is None:
            raise NotImplementedError("SparseMoE: the eval-mode (hard top-1) forward is forward-only")
        st = mod._store
        st.zero_grad()
        B, C, H, W = ctx.shape
        T = B * H * W
        go = _nhwc(g_out, mod._cdt).view(T, C)
        g_tok = torch.empty(T, C, device=g_out.device, dtype=mod._cdt)
        gw = torch.zeros(B, ctx.sv["w"].shape[1], device=g_out.device)
        kl_coef = None if g_kl is None else (g_kl.float().reshape(1) * ctx.kl2[1:2]).contiguous()
        gp = None if g_probs is None else g_probs.float().contiguous()
        eng.moe_bwd(mod._IPRE, ctx.sv, go, g_tok, gw, kl_coef=kl_coef, g_probs=gp)
        eng._flush_router_bwd()
        gx = g_tok.view(B, H, W, C).permute(0, 3, 1, 2).float()
        return mod._grad_out(), gx, gw, None, None, None


class SparseMoE(_EngineModule):
    """Reference :426-491.  Training: the reference's dense soft combine over all experts (or, with ``topk`` <
    num_experts, the build's renormalised top-k dispatch); eval: hard top-1 dispatch.  Returns
    (output, kl, routing_probs)."""
    _IPRE = "m.moe."

    def __init__(self, dim, text_dim, num_experts=4, topk=None, dtype="fp32", seed=0):
        super().__init__(_moe_shapes(dim, text_dim, num_experts), E=num_experts, topk=topk, dtype=dtype, seed=seed)
        self.dim, self.num_experts, self.topk = dim, num_experts, topk

    def forward(self, x, w, annealing_factor=1.0):
        return _MoEFn.apply(self.flat, x, w, self, float(annealing_factor), self.training)


# ---------------------------------------------------------------------------
# AttentionBlock (t2i_moe_gan.py:493-576)
# ---------------------------------------------------------------------------
def _text_rows(text_seq):
    ts = text_seq
    if ts.dim() == 3:
        if ts.shape[1] != 1:
            raise NotImplementedError("AttentionBlock: a one-token text sequence (the generator's text_seq)")
        ts = ts[:, 0]
    return ts.float().contiguous()


class _AttnFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, w, text_seq, mod, anneal, train):
        eng = mod._engine()
        eng.prep()
        xh = _nhwc(x, mod._cdt)
        ts = _text_rows(text_seq)
        eps = mod._eps("moe.router.") if train else None
        eng._want_kl = True
        out, probs, kl2, topi, sv = eng.attn_fwd(mod._IPRE, xh, w.float().contiguous(), ts, eps, anneal, train,
                                                 save=train)
        ctx.mod, ctx.sv, ctx.kl2, ctx.xshape, ctx.tshape = mod, sv, kl2, xh.shape, text_seq.shape
        kl = kl2[0].clone() if train else torch.zeros((), device=x.device)
        if not train:
            ctx.mark_non_differentiable(kl, probs)
        return _nchw(out, mod.dim), probs, kl

    @staticmethod
    def backward(ctx, g_out, g_probs, g_kl):
        mod, eng = ctx.mod, ctx.mod._engine()
        if ctx.sv is None:
            raise NotImplementedError("AttentionBlock: the eval-mode (hard top-1) forward is forward-only")
        st = mod._store
        st.zero_grad()
        dev = g_out.device
        B = ctx.xshape[0]
        gx = torch.empty(ctx.xshape, device=dev, dtype=mod._cdt)
        gw = torch.zeros(B, ctx.sv["sv_moe"]["w"].shape[1], device=dev)
        g_ts = torch.zeros(B, ctx.sv["text_seq"].shape[1], device=dev)
        kl_coef = None if g_kl is None else (g_kl.float().reshape(1) * ctx.kl2[1:2]).contiguous()
        gp = None if g_probs is None else g_probs.float().contiguous()
        eng.attn_bwd(mod._IPRE, ctx.sv, _nhwc(g_out, mod._cdt), gx, gw, g_ts, kl_coef=kl_coef, g_probs=gp)
        return mod._grad_out(), gx.permute(0, 3, 1, 2).float(), gw, g_ts.view(ctx.tshape), None, None, None


class AttentionBlock(_EngineModule):
    """Reference :493-576: proj_in -> LN -> 8-head self-attention -> LN -> cross-attention against the one-token
    text sequence (collapsed algebraically: softmax over one key is 1) -> LN -> SparseMoE -> residual ->
    proj_out.  forward(x, w, text_seq, kl_losses=None, annealing_factor) -> (x_out, routing_probs); the router's
    KL is appended to ``kl_losses`` as in the reference."""
    _IPRE = "b.attn_block."

    def __init__(self, dim, text_dim=512, heads=8, num_experts=4, topk=None, latent_dim=LATENT_DIM, dtype="fp32",
                 seed=0):
        if heads != 8:
            raise NotImplementedError("AttentionBlock: 8 heads (the reference's usage)")
        super().__init__(_attn_shapes(dim, text_dim, num_experts, latent_dim), E=num_experts, topk=topk,
                         dtype=dtype, seed=seed, modconvs=[("proj_in.", 1), ("proj_out.", 1)])
        self.dim, self.heads, self.scale = dim, heads, (dim // heads) ** -0.5
        self.num_experts = num_experts

    def forward(self, x, w, text_seq, kl_losses=None, annealing_factor=1.0):
        out, probs, kl = _AttnFn.apply(self.flat, x, w, text_seq, self, float(annealing_factor), self.training)
        if kl_losses is not None:
            kl_losses.append(kl)
        return out, probs


# ---------------------------------------------------------------------------
# ConvolutionBlock (t2i_moe_gan.py:579-621) and GenerativeBlock (:622-666)
# ---------------------------------------------------------------------------
def _cb_fwd(eng, pre, x, w, offsets, has_skip):
    h1, sv1 = _mtm_fwd(eng, pre + "mtm1.", x, w, offsets)
    svs = None
    if has_skip:
        sk, svs = eng.mc_fwd(pre + "skip_proj.", x, w)
    else:
        sk = x
    out, sv2 = _mtm_fwd(eng, pre + "mtm2.", h1, w, offsets, resid=sk)
    return out, (sv1, svs, sv2, h1)


def _cb_bwd(eng, pre, sv, g_out, gx, gw, offsets):
    sv1, svs, sv2, h1 = sv
    g_h1 = torch.empty_like(h1)
    _mtm_bwd(eng, pre + "mtm2.", sv2, g_out, g_h1, gw, offsets)
    if svs is not None:
        eng.mc_bwd(pre + "skip_proj.", svs, g_out, gx, gw)
    else:
        ops.copy2d(g_out.view(-1, g_out.shape[-1]), gx.view(-1, gx.shape[-1]), g_out.numel() // g_out.shape[-1],
                   g_out.shape[-1])
    _mtm_bwd(eng, pre + "mtm1.", sv1, g_h1, gx, gw, offsets, accumulate=1)


class _CBFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, w, mod):
        eng = mod._engine()
        eng.prep()
        xh = _nhwc(x, mod._cdt)
        out, sv = _cb_fwd(eng, mod._IPRE, xh, w.float().contiguous(), mod.use_offset, mod.has_skip)
        ctx.mod, ctx.sv, ctx.xshape = mod, sv, xh.shape
        return _nchw(out, mod.out_channels)

    @staticmethod
    def backward(ctx, g_out):
        mod, eng = ctx.mod, ctx.mod._engine()
        mod._store.zero_grad()
        dev = g_out.device
        gx = torch.empty(ctx.xshape, device=dev, dtype=mod._cdt)
        gw = torch.zeros(ctx.xshape[0], mod.latent_dim, device=dev)
        _cb_bwd(eng, mod._IPRE, ctx.sv, _nhwc(g_out, mod._cdt), gx, gw, mod.use_offset)
        return mod._grad_out(), gx.permute(0, 3, 1, 2).float(), gw, None


class ConvolutionBlock(_EngineModule):
    """Reference :579-621: MTM -> MTM plus the (modulated 1x1 when Cin != Cout) skip, fused as the second MTM's
    residual epilogue."""
    _IPRE = "b.conv_block."

    def __init__(self, in_channels, out_channels, latent_dim=LATENT_DIM, resolution=None, dtype="fp32", seed=0):
        offsets = resolution is not None and resolution <= 16
        mcs = [("mtm1.modulated_conv.", 3), ("mtm2.modulated_conv.", 3)]
        if in_channels != out_channels:
            mcs.append(("skip_proj.", 1))
        super().__init__(_cb_shapes(in_channels, out_channels, latent_dim, offsets), dtype=dtype, seed=seed,
                         modconvs=mcs, offset_nets=["mtm1.offset_net.0.", "mtm2.offset_net.0."] if offsets else [])
        self.in_channels, self.out_channels, self.latent_dim = in_channels, out_channels, latent_dim
        self.use_offset, self.has_skip = offsets, in_channels != out_channels

    def forward(self, x, w):
        return _CBFn.apply(self.flat, x, w, self)


class _GBFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, flat, x, w, text_seq, mod, anneal, train):
        eng = mod._engine()
        eng.prep()
        xh = _nhwc(x, mod._cdt)
        wf = w.float().contiguous()
        if mod.upsample:
            xh = ops.upsample2x(xh)  # nn.Upsample(2, bilinear, align_corners=False), :633, :657-658
        h, cbsv = _cb_fwd(eng, "b.conv_block.", xh, wf, mod.use_offset, mod.has_skip)
        eps = mod._eps("attn_block.moe.router.") if train else None
        eng._want_kl = True
        out, probs, kl2, topi, asv = eng.attn_fwd("b.attn_block.", h, wf, _text_rows(text_seq), eps, anneal, train,
                                                  save=train)
        ctx.mod, ctx.cbsv, ctx.asv, ctx.kl2 = mod, cbsv, asv, kl2
        ctx.xshape, ctx.hshape, ctx.tshape = tuple(x.shape), h.shape, text_seq.shape
        kl = kl2[0].clone() if train else torch.zeros((), device=x.device)
        if not train:
            ctx.mark_non_differentiable(kl, probs)
        return _nchw(out, mod.out_channels), probs, kl

    @staticmethod
    def backward(ctx, g_out, g_probs, g_kl):
        mod, eng = ctx.mod, ctx.mod._engine()
        if ctx.asv is None:
            raise NotImplementedError("GenerativeBlock: the eval-mode (hard top-1) forward is forward-only")
        mod._store.zero_grad()
        dev = g_out.device
        B = ctx.hshape[0]
        g_h = torch.empty(ctx.hshape, device=dev, dtype=mod._cdt)
        gw = torch.zeros(B, mod.latent_dim, device=dev)
        g_ts = torch.zeros(B, ctx.asv["text_seq"].shape[1], device=dev)
        kl_coef = None if g_kl is None else (g_kl.float().reshape(1) * ctx.kl2[1:2]).contiguous()
        gp = None if g_probs is None else g_probs.float().contiguous()
        eng.attn_bwd("b.attn_block.", ctx.asv, _nhwc(g_out, mod._cdt), g_h, gw, g_ts, kl_coef=kl_coef, g_probs=gp)
        x_in = ctx.cbsv[0][0]  # input of mtm1 (after the upsample)
        g_in = torch.empty(x_in.shape, device=dev, dtype=mod._cdt)
        _cb_bwd(eng, "b.conv_block.", ctx.cbsv, g_h, g_in, gw, mod.use_offset)
        if mod.upsample:
            Bq, H2, W2, Cq = g_in.shape
            gprev = torch.empty(Bq, H2 // 2, W2 // 2, Cq, device=dev, dtype=mod._cdt)
            ops.upsample2x_bwd(g_in, gprev)
            g_in = gprev
        return mod._grad_out(), g_in.permute(0, 3, 1, 2).float(), gw, g_ts.view(ctx.tshape), None, None, None


class GenerativeBlock(_EngineModule):
    """Reference :622-666: optional bilinear x2 upsample -> ConvolutionBlock -> AttentionBlock.
    forward(x, w, text_seq, kl_losses=None, annealing_factor) -> (x, routing_probs)."""
    _IPRE = "b."

    def __init__(self, in_channels, out_channels, text_dim=768, upsample=False, resolution=None, num_experts=4,
                 topk=None, latent_dim=LATENT_DIM, dtype="fp32", seed=0):
        offsets = resolution is not None and resolution <= 16
        shapes = _cb_shapes(in_channels, out_channels, latent_dim, offsets, "conv_block.")
        shapes += _attn_shapes(out_channels, text_dim, num_experts, latent_dim, "attn_block.")
        mcs = [("conv_block.mtm1.modulated_conv.", 3), ("conv_block.mtm2.modulated_conv.", 3),
               ("attn_block.proj_in.", 1), ("attn_block.proj_out.", 1)]
        if in_channels != out_channels:
            mcs.append(("conv_block.skip_proj.", 1))
        offs = ["conv_block.mtm1.offset_net.0.", "conv_block.mtm2.offset_net.0."] if offsets else []
        super().__init__(shapes, E=num_experts, topk=topk, dtype=dtype, seed=seed, modconvs=mcs, offset_nets=offs)
        self.in_channels, self.out_channels, self.latent_dim = in_channels, out_channels, latent_dim
        self.upsample, self.use_offset, self.has_skip = upsample, offsets, in_channels != out_channels

    def forward(self, x, w, text_seq, kl_losses=None, annealing_factor=1.0):
        out, probs, kl = _GBFn.apply(self.flat, x, w, text_seq, self, float(annealing_factor), self.training)
        if kl_losses is not None:
            kl_losses.append(kl)
        return out, probs


# ---------------------------------------------------------------------------
# create_optimizer_for_active_blocks (t2i_moe_gan.py:1005-1026)
# ---------------------------------------------------------------------------
class FlatRangeAdamW:
    """torch.optim.AdamW semantics over named parameter ranges of a flat-parameter module (mg_adamw on each
    contiguous range of ``module.flat``).  ``step()`` reads ``module.flat.grad``; ``state_dict()`` is torch's
    format over the active parameters in order."""

    def __init__(self, module, names, lr, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01):
        st = module._store
        self.module, self.names = module, list(names)
        self.param_groups = [dict(lr=lr, betas=tuple(betas), eps=eps, weight_decay=weight_decay)]
        spans = sorted(st.offsets[n] for n in self.names)
        self.ranges = []
        for off, numel in spans:  # merge neighbours (and the alignment gaps between them) into one launch
            if self.ranges and off - (self.ranges[-1][1]) < 8:
                self.ranges[-1][1] = off + numel
            else:
                self.ranges.append([off, off + numel])
        self.m = torch.zeros_like(st.data)
        self.v = torch.zeros_like(st.data)
        self.steps = 0

    def zero_grad(self, set_to_none=True):
        self.module.zero_grad(set_to_none=set_to_none)

    @torch.no_grad()
    def step(self):
        g = self.module.flat.grad
        if g is None:
            return
        self.steps += 1
        pg = self.param_groups[0]
        p = self.module.flat.data
        if self.m.device != p.device:
            self.m, self.v = self.m.to(p.device), self.v.to(p.device)
        for lo, hi in self.ranges:
            ops.adamw(p[lo:hi], g[lo:hi], self.m[lo:hi], self.v[lo:hi], pg["lr"], pg["betas"][0], pg["betas"][1],
                      pg["eps"], pg["weight_decay"], self.steps)
        self.module._store.refresh_shadow(force=True)

    def state_dict(self):
        st = self.module._store
        state = {}
        if self.steps:
            for i, n in enumerate(self.names):
                off, numel = st.offsets[n]
                state[i] = {"step": torch.tensor(float(self.steps)),
                            "exp_avg": self.m[off:off + numel].view(st.shapes[n]).cpu().clone(),
                            "exp_avg_sq": self.v[off:off + numel].view(st.shapes[n]).cpu().clone()}
        pg = dict(self.param_groups[0], amsgrad=False, maximize=False, foreach=None, capturable=False,
                  differentiable=False, fused=None, decoupled_weight_decay=True,
                  params=list(range(len(self.names))))
        return {"state": state, "param_groups": [pg]}


def create_optimizer_for_active_blocks(generator, active_resolutions, lr, betas, weight_decay):
    """Reference :1005-1026 (dead code there: nothing calls it).  The text projection, mapping network and
    constant plus the generative blocks of ``active_resolutions``; 32 / 64 name blocks the reference generator
    does not have, which fails as it does in the reference (AttributeError)."""
    names = [n for n in generator._store.shapes if not is_buffer(n)]
    keep = [n for n in names if n.startswith(("text_projection.", "mapping.")) or n == "constant"]
    for r in active_resolutions:
        if r in (32, 64):
            raise AttributeError(f"'AuroraGenerator' object has no attribute 'gen_block_{r}'")
        keep += [n for n in names if n.startswith(f"gen_block_{r}.")]
    return FlatRangeAdamW(generator, keep, lr, betas, weight_decay=weight_decay)


__all__ = ["ModulatedConv", "ModulatedTransformationModule", "SparseExpertFFN", "BayesianRouter", "SparseMoE",
           "AttentionBlock", "ConvolutionBlock", "GenerativeBlock", "create_optimizer_for_active_blocks",
           "FlatRangeAdamW"]
