"""Explicit forward/backward of the Aurora MoE generator on the HIP kernels.

Mirrors AuroraGenerator (t2i_moe_gan.py:668-855) module by module, but as an
explicit two-pass engine: ``forward`` records exactly the activations its
``backward`` needs (no autograd graph, no tape), every contraction runs on the
MFMA GEMM core, and all activations are NHWC token rows in HBM.

Numerics: ``cdt`` is the activation / MFMA-operand dtype (fp32 = parity mode,
bf16 = the C2 bench mode).  Styles, demodulation coefficients, router logits,
LayerNorm statistics and every parameter gradient stay fp32.

Randomness is explicit: router epsilon triples, z and the mismatch
permutation are inputs (SURVEY.md §7 "Randomness parity").
"""
import os

import torch

from . import _lib as L
from . import graphs, ops
from .layout import gen_blocks, max_res_of, rgb_layers

E_ = ops.E
LRELU, GELU, RSQRT = L.ACT_LRELU, L.ACT_GELU, L.ACT_RSQRT_EPS
MUL_GELU_GRAD, MUL_LRELU_GRAD = L.ACT_MUL_GELU_GRAD, L.ACT_MUL_LRELU_GRAD


def _modconv_prefixes(max_res=16):
    out = []
    for name, cin, cout, _, _, attn in gen_blocks(max_res):
        cb = name + ".conv_block."
        out += [(cb + "mtm1.modulated_conv.", 3), (cb + "mtm2.modulated_conv.", 3)]
        if cin != cout:
            out.append((cb + "skip_proj.", 1))
        if attn:
            out += [(name + ".attn_block.proj_in.", 1), (name + ".attn_block.proj_out.", 1)]
    out += [(n + ".", 1) for n, _ in rgb_layers(max_res)[-2:]]  # intermediate + final image
    return out


def _offset_prefixes(max_res=16):
    return [f"{name}.conv_block.{m}.offset_net.0." for name, _, _, res, _, _ in gen_blocks(max_res) if res <= 16
            for m in ("mtm1", "mtm2")]


class GeneratorEngine:
    def __init__(self, store, E, topk=None, cdt=torch.float32, modconvs=None, offset_nets=None, fp8=False):
        """``modconvs`` [(prefix, k)] / ``offset_nets`` [prefix]: the modulated convs and MTM offset heads prep()
        packs -- the whole generator's by default; the sub-module API (modules.py) passes its own."""
        self.st = store
        # block list: the reference's three blocks, or the progressive extension when the store holds it
        self.max_res = max_res_of(store.offsets)
        self.blocks = gen_blocks(self.max_res)
        self.attn_blocks = [b[0] for b in self.blocks if b[5]]
        rgb = rgb_layers(self.max_res)
        self.rgb_final, self.rgb_half = rgb[-1][0] + ".", rgb[-2][0] + "."
        self.half_block = "gen_block_%d" % (self.max_res // 2)
        self.mc_list = _modconv_prefixes(self.max_res) if modconvs is None else list(modconvs)
        self.off_list = _offset_prefixes(self.max_res) if offset_nets is None else list(offset_nets)
        self.E = E
        self.k = topk or E
        self.cdt = cdt
        # operand dtype of the per-image prefix GEMMs (text projection, mapping, styles and their backward): fp32
        # even in the bf16 mode, because their rounding is shared by every token of an image and so adds up
        # coherently (measured on the router temperatures' per-image sums); MOEGAN_PREFIX_BF16=1 = bf16 operands
        self.pdt = cdt if os.environ.get("MOEGAN_PREFIX_BF16", "0") == "1" else torch.float32
        # MX-fp8 (e4m3 + per-32-channel E8M0 scales) for the 3x3 modulated-conv forward and data-gradient GEMMs
        # (BASELINE config C5); needs the bf16 compute dtype and >= 128 channels on the reduction side
        self.fp8 = bool(fp8)
        assert not self.fp8 or cdt == torch.bfloat16, "fp8 modulated convs run inside the bf16 mode"
        self.dev = store.device
        self.packs = {}
        self._ones = None
        self.style_cols = {}
        self._S = self._S2 = self._GS = None  # batched styles of the running forward / style grads of a backward
        self._D = None  # demodulation coefficients of the running forward, {prefix: [B, rows]}
        self._demod_bwd = []
        self._router_bwd, self._xattn_bwd = [], []  # per-block small backward GEMMs, batched at the end
        self._defer = False
        self._mean_latent = None
        self._want_kl = True
        self.last_klbuf = None
        self._bv = None  # per-block vectors of the running forward (_block_vectors)
        self.guard_flags = None  # the training step's loss-guard word (step.py), read by the router backward
        # called with (lo, hi) when a contiguous range of the flat gradient is final during backward (a block's
        # expert weights / biases): the data-parallel step starts that range's all-reduce right away (step.py)
        self.on_grad_final = None
        # weight gradients run on a side stream, overlapping the data-gradient chain (joined in backward)
        self.side = graphs.SideStream(self.dev, enabled=graphs.side_streams_enabled(self.dev))

    # parameter access
    def P(self, n):
        return self.st.view(n)

    def Pc(self, n):
        return self.st.cview(n)

    def G(self, n):
        return self.st.gview(n)

    def Pp(self, n):
        return self.P(n) if self.pdt == torch.float32 else self.st.cview(n)

    def _p(self, x, alpha=1.0):
        return x if (x.dtype == self.pdt and alpha == 1.0) else ops.cast(x, self.pdt, alpha=alpha)

    def _c(self, x, alpha=1.0):
        """x in the compute dtype (the mapping / text / style GEMMs run on bf16 operands in bf16 mode, as the
        reference's AMP autocast runs its Linear layers in half precision, t2i_moe_gan.py:1267)."""
        return x if (x.dtype == self.cdt and alpha == 1.0) else ops.cast(x, self.cdt, alpha=alpha)

    # ------------------------------------------------------------------
    # per-step weight preparation (after every optimizer step)
    # ------------------------------------------------------------------
    def prep(self):
        self.st.refresh_shadow()
        sb = self.st.style_block()
        self.style_cols = None
        if sb is not None:
            (o0, nrows, K, b0), cols = sb
            self.style_cols = cols
            self.style_n = nrows
            self.style_W = self.st.data[o0:o0 + nrows * K].view(nrows, K)
            self.style_Wc = (self.st.data if self.pdt == torch.float32 else self._cbuf())[o0:o0 + nrows * K].view(
                nrows, K)
            self.style_b = self.st.data[b0:b0 + nrows]
            self.style_gW = self.st.grad[o0:o0 + nrows * K].view(nrows, K)
            self.style_gb = self.st.grad[b0:b0 + nrows]
        self._mean_latent = None  # truncation centre: mapping of zeros, a function of the weights only
        pk = {}
        pb = ops.PrepBatch(self.cdt)  # every pack / demodulation sum of the generator in one launch
        for pre, k in self.mc_list:
            W = self.P(pre + "weight")
            Cout = W.shape[0]
            rows = max(Cout, 8)
            ent = {"rows": rows, "wsq": pb.wsq(W, rows=rows)}
            if k == 3:
                ent["w"] = pb.pack(W)
                ent["wflip"] = pb.pack(W, flip=True)
            elif rows != Cout:
                ent["w"] = pb.pack(W, rows=rows)
            else:
                ent["w"] = self.Pc(pre + "weight").view(Cout, -1)
            pk[pre] = ent
        for pre in self.off_list:
            W = self.P(pre + "weight")
            pk[pre] = {"w": pb.pack(W), "wflip": pb.pack(W, flip=True)}
        pb.run()
        if self.fp8:  # per-step MX-fp8 copies of the packed 3x3 weights (forward and flipped data-gradient form),
            jobs = []  # all in one launch
            for pre, k in self.mc_list:
                ent = pk[pre]
                if k == 3 and self._mx8_ok(self.P(pre + "weight").shape[1]):
                    jobs.append((ent, "wq", ent["w"]))
                if k == 3 and self._mx8_ok(ent["rows"]):
                    jobs.append((ent, "wflipq", ent["wflip"]))
            for (ent, key, _), r in zip(jobs, ops.quant_mx8_batch([w.reshape(-1, w.shape[-1]) for _, _, w in jobs])):
                ent[key] = r
        self.packs = pk

    @staticmethod
    def _mx8_ok(cin):
        """The MX-fp8 conv reduces over 128-channel steps inside one tap."""
        return cin >= 128 and cin % 128 == 0 and (cin & (cin - 1)) == 0

    # ------------------------------------------------------------------
    # ModulatedConv  (t2i_moe_gan.py:154-186), fused form
    # ------------------------------------------------------------------
    def _style(self, pre, w, Cin):
        """(s, s^2) for one modulated conv: column slices of the step's batched styles when available."""
        if self._S is not None and pre in self.style_cols:
            c = self.style_cols[pre]
            return self._S[:, c:c + Cin], self._S2[:, c:c + Cin]
        s = ops.linear(w, self.P(pre + "modulation.weight"), bias=self.P(pre + "modulation.bias"))  # :158
        return s, ops.cast(s, square=1)

    def _batched_style(self, pre, Cin):
        """The style rows s [B, Cin] of a modulated conv from the step's batched style GEMM (a column slice of S),
        or None when there is none (then mc_fwd forms x * s itself)."""
        if self._S is not None and pre in self.style_cols and Cin % 8 == 0:
            c = self.style_cols[pre]
            return self._S[:, c:c + Cin]
        return None

    def mc_fwd(self, pre, x, w, act=0, resid=None, save=True, xs=None):
        B, H, W, Cin = x.shape
        HW = H * W
        pk = self.packs[pre]
        rows = pk["rows"]
        Wt = self.P(pre + "weight")
        k = Wt.shape[-1]
        s, s2 = self._style(pre, w, Cin)
        d = self._D.get(pre) if self._D is not None else None
        if d is None:
            d = ops.gemm(s2, pk["wsq"], B, rows, Cin, ep=E_(act=RSQRT))  # demod coefficients [B, rows] (:165)
        # with a residual fused behind the LeakyReLU the backward needs the pre-activation's sign: the epilogue
        # stores it (reconstructing it as output - residual cancels: a pre-activation below the rounding of the
        # residual flips its slope -- measured ~1 % gradient error at 8x8 in fp32, far more in bf16)
        ypre = torch.empty(B * HW, rows, device=self.dev, dtype=self.cdt) if (save and resid is not None and act) \
            else None
        ep = E_(scale=d, scale_shift=ops.ilog2(HW), scale_ld=rows, act=act, resid=resid,
                ld_res=resid.shape[-1] if resid is not None else 0, out_pre=ypre, ld_pre=rows if ypre is not None else 0)
        if xs is None:  # x * style, shared by the conv and its weight gradient (the MTM warp writes it itself)
            xs = ops.scale_bc(x, s)
        if "wq" in pk:  # MX-fp8: quantize x * s per 32 channels, e4m3 x e4m3 scaled MFMA
            xq, xsc = ops.quant_mx8(xs.view(-1, Cin))
            y = ops.conv2d_mx8(xq.view(B, H, W, Cin), xsc, *pk["wq"], rows, k, k, 1, k // 2, ep=ep, out_dtype=self.cdt)
        else:
            y = ops.conv2d(xs, pk["w"], rows, k, k, 1, k // 2, ep=ep, out_dtype=self.cdt)
        if not save:
            sv = None
        elif ypre is not None:  # act 2: z holds the pre-activation itself
            sv = (x, xs, w, s, s2, d, ypre, None, 2)
        else:
            sv = (x, xs, w, s, s2, d, y, resid, act)
        return y, sv

    def mc_bwd(self, pre, sv, gz, gx, gw, accumulate=0, gx_f32=False):
        """gz: grad of the conv output (post activation / residual). Writes/accumulates gx, accumulates gw.
        ``gx_f32``: the data gradient stays fp32 up to gx (an MTM's warped-input gradient, which the offset head
        reduces over channels and pixels into cancelling sums)."""
        x, xs, w, s, s2, d, z, zsub, act = sv
        B, H, W, Cin = x.shape
        HW = H * W
        pk = self.packs[pre]
        rows = pk["rows"]
        Wt = self.P(pre + "weight")
        Cout, k = Wt.shape[0], Wt.shape[-1]
        P = B * HW
        gyt = torch.empty(P, rows, device=self.dev, dtype=self.cdt)
        gdd = torch.empty(B, rows, device=self.dev, dtype=torch.float32)
        ops.modconv_bwd_out(gz.view(P, -1), z.view(P, -1), d, B, HW, rows, act, gyt, gdd,
                            zsub=None if zsub is None else zsub.view(P, -1))
        # data gradient of the shared-weight conv
        if k == 3 and "wflipq" in pk:  # MX-fp8 data gradient (gradient rows quantized per 32 channels)
            gq, gsc = ops.quant_mx8(gyt)
            gxt = ops.conv2d_mx8(gq.view(B, H, W, rows), gsc, *pk["wflipq"], Cin, 3, 3, 1, 1, out_dtype=self.cdt)
        elif k == 3:
            gxt = ops.conv2d(gyt.view(B, H, W, rows), pk["wflip"], Cin, 3, 3, 1, 1,
                             out_dtype=torch.float32 if gx_f32 else None)
        else:
            gxt = ops.gemm(gyt, pk["w"], P, Cin, rows, b_kc=False)
        batched = self._GS is not None and pre in self.style_cols
        if batched:
            c = self.style_cols[pre]
            gs = self._GS[:, c:c + Cin]
        else:
            gs = ops.zeros(B, Cin, device=self.dev)
        ops.modconv_bwd_in(gxt.view(P, Cin), x.view(P, Cin), s, B, HW, Cin,
                           None if gx is None else gx.view(P, -1), gs, accumulate)
        # weight gradient (fp32, reference layout), on the side stream
        gW = self.G(pre + "weight")
        if rows == Cout:
            self.side.run(lambda: ops.conv2d_wgrad(gyt, xs, Cout, k, k, 1, k // 2, gW), gyt, xs)
        else:
            def wgrad_padded():
                tmp = ops.zeros(rows, Cin, k, k, device=self.dev)
                ops.conv2d_wgrad(gyt, xs, rows, k, k, 1, k // 2, tmp)
                ops.fold_add([(tmp[:Cout], gW)])  # (after tmp's own deferred slab fold)
            self.side.run(wgrad_padded, gyt, xs)
        # demodulation backward
        if batched:  # deferred: all modulated convs' demod + style backward run batched at the end
            self._demod_bwd.append((pre, gdd, s2, s, gs, Cin, rows, Cout))
            return
        gwsq = ops.gemm(gdd, s2, rows, Cin, B, a_kc=False, b_kc=False)  # [rows, Cin] = gdd^T s^2
        self.side.join()  # the side stream's conv weight gradient accumulates into the same tensor
        ops.wsq_bwd(Wt, gwsq[:Cout], self.G(pre + "weight"))
        ops.gemm(gdd, pk["wsq"], B, Cin, rows, b_kc=False, out=gs,
                 ep=E_(alpha=2.0, scale=s, scale_ld=s.stride(0), accumulate=1))  # gs += 2 s (gdd @ wsq)
        ops.linear_wgrad(gs, w, self.G(pre + "modulation.weight"))
        ops.colsum(gs, self.G(pre + "modulation.bias"), defer=True)
        ops.gemm(gs, self.P(pre + "modulation.weight"), B, w.shape[1], Cin, b_kc=False, out=gw,
                 ep=E_(accumulate=1))

    # ------------------------------------------------------------------
    # Modulated Transformation Module  (t2i_moe_gan.py:218-247)
    # ------------------------------------------------------------------
    def mtm_fwd(self, pre, x, w, resid=None, save=True):
        if (pre + "offset_net.0.") not in self.packs:  # no offset head above 16x16 (:199): modconv + LReLU
            y, msv = self.mc_fwd(pre + "modulated_conv.", x, w, act=1, resid=resid, save=save)
            return y, ((x, None, None, None, msv) if save else None)
        opk = self.packs[pre + "offset_net.0."]
        o1 = ops.conv2d(x, opk["w"], 32, 3, 3, 1, 1, out_dtype=self.cdt,
                        ep=E_(bias=self.P(pre + "offset_net.0.bias"), act=LRELU))
        s, _ = self._style(pre + "modulated_conv.", w, x.shape[-1])
        xw, samp, xs = ops.warp_fwd(x, o1, self.P(pre + "offset_net.2.weight"), self.P(pre + "offset_net.2.bias"),
                                    s=s)
        y, msv = self.mc_fwd(pre + "modulated_conv.", xw, w, act=1, resid=resid, save=save, xs=xs)
        return y, ((x, o1, samp, xw, msv) if save else None)

    def mtm_bwd(self, pre, sv, gz, gx, gw, accumulate=0):
        x, o1, samp, xw, msv = sv
        if o1 is None:  # no offset head
            self.mc_bwd(pre + "modulated_conv.", msv, gz, gx, gw, accumulate=accumulate)
            return
        B, H, W, Cin = x.shape
        P = B * H * W
        # fp32: the offset head's gradient is a sum over channels and pixels of g_xw * (neighbour differences of
        # x) that largely cancels -- a bf16 g_xw put 3-5x the whole-step bf16 floor on the head biases
        g_xw = torch.empty(P, Cin, device=self.dev, dtype=torch.float32)
        self.mc_bwd(pre + "modulated_conv.", msv, gz, g_xw, gw, gx_f32=True)
        opk = self.packs[pre + "offset_net.0."]
        if ops.mtm_bwd_fusable(x) and gx.is_contiguous():
            ga1 = torch.empty(B, H, W, 32, device=self.dev, dtype=self.cdt)
            ops.mtm_bwd_fused(g_xw, x, samp, o1, self.P(pre + "offset_net.2.weight"), gx, ga1,
                              self.G(pre + "offset_net.2.weight"), self.G(pre + "offset_net.2.bias"), accumulate)
            ops.conv2d(ga1, opk["wflip"], Cin, 3, 3, 1, 1, out=gx.view(B, H, W, Cin), ep=E_(accumulate=1))
            ops.conv2d_wgrad(ga1, x, 32, 3, 3, 1, 1, self.G(pre + "offset_net.0.weight"))
            ops.colsum(ga1.view(P, 32), self.G(pre + "offset_net.0.bias"), defer=True)
            return
        gx32 = ops.zeros(B, H, W, Cin, device=self.dev)
        goff = torch.empty(P, 2, device=self.dev, dtype=torch.float32)
        ops.warp_bwd(g_xw, x, samp, gx32, goff)
        ga1 = torch.empty(B, H, W, 32, device=self.dev, dtype=self.cdt)
        ops.offset_head_bwd(goff, o1, self.P(pre + "offset_net.2.weight"), ga1,
                            self.G(pre + "offset_net.2.weight"), self.G(pre + "offset_net.2.bias"))
        ops.conv2d(ga1, opk["wflip"], Cin, 3, 3, 1, 1, out=gx32, ep=E_(accumulate=1))
        ops.conv2d_wgrad(ga1, x, 32, 3, 3, 1, 1, self.G(pre + "offset_net.0.weight"))
        ops.colsum(ga1.view(P, 32), self.G(pre + "offset_net.0.bias"), defer=True)
        ops.copy2d(gx32.view(P, Cin), gx.view(P, Cin), P, Cin, accumulate=accumulate)

    # ------------------------------------------------------------------
    # ConvolutionBlock  (t2i_moe_gan.py:579-621)
    # ------------------------------------------------------------------
    def cb_fwd(self, pre, x, w, save=True, skip_xs=None):
        """``skip_xs``: the skip conv's input x * s when the producer of x already formed it (upsample2x)."""
        h1, sv1 = self.mtm_fwd(pre + "mtm1.", x, w, save=save)
        svs = None
        if (pre + "skip_proj.weight") in self.st.offsets:
            sk, svs = self.mc_fwd(pre + "skip_proj.", x, w, save=save, xs=skip_xs)
        else:
            sk = x
        out, sv2 = self.mtm_fwd(pre + "mtm2.", h1, w, resid=sk, save=save)
        return out, ((sv1, svs, sv2, h1) if save else None)

    def cb_bwd(self, pre, sv, g_out, gx, gw):
        sv1, svs, sv2, h1 = sv
        g_h1 = torch.empty_like(h1)
        self.mtm_bwd(pre + "mtm2.", sv2, g_out, g_h1, gw)
        if svs is not None:
            self.mc_bwd(pre + "skip_proj.", svs, g_out, gx, gw)
        else:
            ops.copy2d(g_out.view(-1, g_out.shape[-1]), gx.view(-1, gx.shape[-1]), g_out.numel() // g_out.shape[-1],
                       g_out.shape[-1])
        self.mtm_bwd(pre + "mtm1.", sv1, g_h1, gx, gw, accumulate=1)

    # ------------------------------------------------------------------
    # SparseMoE + BayesianRouter  (t2i_moe_gan.py:265-491)
    # ------------------------------------------------------------------
    def moe_fwd(self, pre, tok, resid, w, HW, eps, anneal, train=True, save=True, kl_out=None, out_style=None):
        """``out_style`` [B, C] (the next modulated conv's style rows): the combine also writes that conv's input
        x * s, returned as the sixth value (else None)."""
        r = pre + "router."
        T, C = tok.shape
        B = w.shape[0]
        E, k = self.E, (self.k if train else 1)
        bv = self._bv.get(pre) if self._bv is not None else None
        if bv is not None:  # computed for every block at once (_block_vectors)
            Wf, Wt, Wc, Wfc, u, Lt = bv["Wf"], bv["Wt"], bv["Wc"], bv["Wfc"], bv["u"], bv["Lt"]
        else:
            Wf, Wt, Wc = self._router_weights(r, eps, train)
            Wfc = ops.gemm(Wf, Wc[:128], C, E, 128, b_kc=False)  # [C, E]
            u = ops.gemm(w, Wt, B, 128, w.shape[1], b_kc=False)  # [B, 128]
            Lt = ops.gemm(u, Wc[128:], B, E, 128, b_kc=False)  # [B, E]
        probs, zlog, topi, gate = ops.router_fwd(tok, Wfc, Lt, E, k, HW, self.P(r + "temperature"), anneal,
                                                 eval_mode=0 if train else 1)
        row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
        n = T * k
        max_tiles = (n + 127) // 128 + E
        ex = pre + "experts."
        W1 = self.st.group_view(ex + "0.net.0.weight", f"{ex}{E-1}.net.0.weight", self._cbuf())
        b1 = self.st.group_view(ex + "0.net.0.bias", f"{ex}{E-1}.net.0.bias")
        W2 = self.st.group_view(ex + "0.net.2.weight", f"{ex}{E-1}.net.2.weight", self._cbuf())
        b2 = self.st.group_view(ex + "0.net.2.bias", f"{ex}{E-1}.net.2.bias")
        Hd = 4 * C
        Y = torch.empty(n, C, device=self.dev, dtype=self.cdt)
        if ops.ffn_fusable(self.cdt, C):
            # fused expert FFN: the hidden activation stays on chip; saved (pre-activation for GELU', GELU output
            # for dW2, gathered tokens for dW1) only when the backward will run
            if save:
                Xg = ops.gather_rows(tok, perm, k)
                Pre = torch.empty(n, Hd, device=self.dev, dtype=self.cdt)
                # the GELU output is recomputed from Pre by the layer-2 weight gradient's loader unless stored
                # (ops.FFN_SAVE_HID): one [rows x 4C] bf16 write less per step
                Hid = torch.empty(n, Hd, device=self.dev, dtype=self.cdt) if ops.FFN_SAVE_HID else None
                ops.moe_ffn_fwd(Xg, W1.view(E, Hd, C), b1, W2.view(E, C, Hd), b2, row_off, tile_off, max_tiles, Y,
                                pre=Pre, hid=Hid)
            else:
                Xg = Pre = Hid = None
                ops.moe_ffn_fwd(tok, W1.view(E, Hd, C), b1, W2.view(E, C, Hd), b2, row_off, tile_off, max_tiles, Y,
                                x_idx=perm, x_idx_div=k)
        else:
            # tokens in dispatch order (k copies per token), shared by the expert GEMM and its weight gradient
            Xg = ops.gather_rows(tok, perm, k)
            # the pre-activation is kept only for the backward's GELU' (a no-grad forward skips that store)
            Pre = torch.empty(n, Hd, device=self.dev, dtype=self.cdt) if save else None
            Hid = torch.empty(n, Hd, device=self.dev, dtype=self.cdt)
            ops.gemm_grouped(Xg, W1, row_off, tile_off, max_tiles, Hd, C, b_gstride=Hd * C, out=Hid, ldb=C,
                             ep=E_(bias=b1, act=GELU, out_pre=Pre, ld_pre=Hd if save else 0))
            ops.gemm_grouped(Hid, W2, row_off, tile_off, max_tiles, C, Hd, b_gstride=C * Hd, out=Y, ldb=Hd,
                             ep=E_(bias=b2))
        out = torch.empty(T, C, device=self.dev, dtype=self.cdt)
        xs_next = None
        if out_style is not None:  # x_spatial + moe_out (:571), and proj_out's x * s from the same pass
            out, xs_next = ops.moe_combine(Y, pos_of, gate, resid, out, style=out_style, HW=HW)
        else:
            ops.moe_combine(Y, pos_of, gate, resid, out)  # x_spatial + moe_out (:571)
        kl2 = None
        if train and self._want_kl:
            if kl_out is not None:  # filled by the forward's batched KL launch (ops.router_kl_batch)
                kl2 = kl_out
            else:
                kl2 = torch.empty(2, device=self.dev, dtype=torch.float32)
                ops.router_kl(self.P(r + "feature_mu"), self.P(r + "feature_rho"), self.P(r + "text_mu"),
                              self.P(r + "text_rho"), self.P(r + "combined_mu"), self.P(r + "combined_rho"), kl2)
        sv = None
        if save:
            sv = dict(tok=tok, w=w, HW=HW, eps=eps, anneal=anneal, Wf=Wf, Wt=Wt, Wc=Wc, Wfc=Wfc, u=u, probs=probs,
                      zlog=zlog, topi=topi, gate=gate, row_off=row_off, tile_off=tile_off, perm=perm, pos_of=pos_of,
                      gate_pos=gate_pos, Pre=Pre, Hid=Hid, Xg=Xg, Y=Y, W1=W1, W2=W2, max_tiles=max_tiles)
        if out_style is not None:
            return out, probs, kl2, topi, sv, xs_next
        return out, probs, kl2, topi, sv

    def _router_weights(self, r, eps, train, pb=None):
        """Reparameterised router weights (t2i_moe_gan.py:302-333) in train mode, the means in eval mode.
        With a PrepBatch ``pb`` the three reparameterisations join its launch (the caller runs it)."""
        if train:
            rp = pb.reparam if pb is not None else ops.reparam
            return (rp(self.P(r + "feature_mu"), self.P(r + "feature_rho"), eps[0]),
                    rp(self.P(r + "text_mu"), self.P(r + "text_rho"), eps[1]),
                    rp(self.P(r + "combined_mu"), self.P(r + "combined_rho"), eps[2]))
        return self.P(r + "feature_mu"), self.P(r + "text_mu"), self.P(r + "combined_mu")

    def _xattn_chain(self, text_seq):
        """The cross-attention value chain tp -> v -> out_proj of every block (t2i_moe_gan.py:549-556): a
        function of the text sequence and the weights only, so one step's D-phase and G-phase forwards share it
        (computed with the prefix); three batched launches, one per level."""
        B = text_seq.shape[0]
        dev = self.dev
        pres = [name + ".attn_block." for name in self.attn_blocks]
        Cs = [self.P(p + "text_proj.weight").shape[0] for p in pres]
        chain = {}
        src = [text_seq] * len(pres)
        for key, wname, bname, sl in (("tp", "text_proj.weight", "text_proj.bias", False),
                                      ("vv", "cross_attn.in_proj_weight", "cross_attn.in_proj_bias", True),
                                      ("ca", "cross_attn.out_proj.weight", "cross_attn.out_proj.bias", False)):
            probs, outs = [], []
            for p, C, a in zip(pres, Cs, src):
                Wm, bm = self.P(p + wname), self.P(p + bname)
                if sl:  # value rows of the packed in-projection
                    Wm, bm = Wm[2 * C:], bm[2 * C:]
                o = torch.empty(B, C, device=dev)
                probs.append(dict(A=a, B=Wm, M=B, N=C, K=a.shape[1], out=o, ep=E_(bias=bm)))
                outs.append(o)
            ops.gemm_batch(probs)
            chain[key] = outs
            src = outs
        return {p: dict(tp=chain["tp"][i], vv=chain["vv"][i], ca=chain["ca"][i]) for i, p in enumerate(pres)}

    def _block_vectors(self, w, text_seq, eps, train, xchain):
        """Everything per block that depends only on (w, text_seq, router eps): the cross-attention value chain
        (``xchain``, _xattn_chain) and the router's text logits and feature-combine matrix (:364-389) -- for all
        blocks at once in batched launches instead of eighteen GEMMs."""
        B = w.shape[0]
        dev = self.dev
        pres = [name + ".attn_block." for name in self.attn_blocks]
        Cs = [self.P(p + "text_proj.weight").shape[0] for p in pres]
        bv = {p + "moe.": {} for p in pres}
        E = self.E
        probs1, probs2 = [], []
        pb = ops.PrepBatch(torch.float32)  # the routers' reparameterisations: one launch
        for i, (p, C) in enumerate(zip(pres, Cs)):
            d = bv[p + "moe."]
            Wf, Wt, Wc = self._router_weights(p + "moe.router.", None if eps is None else eps[i], train, pb)
            d.update(Wf=Wf, Wt=Wt, Wc=Wc, Wfc=torch.empty(C, E, device=dev), u=torch.empty(B, 128, device=dev),
                     Lt=torch.empty(B, E, device=dev))
            probs1.append(dict(A=Wf, B=Wc[:128], M=C, N=E, K=128, out=d["Wfc"]))  # Wf @ Wc1
            probs1.append(dict(A=w, B=Wt, M=B, N=128, K=w.shape[1], out=d["u"]))  # w @ Wt
            probs2.append(dict(A=d["u"], B=Wc[128:], M=B, N=E, K=128, out=d["Lt"]))  # u @ Wc2
        pb.run()
        ops.gemm_batch(probs1, b_kc=False)
        ops.gemm_batch(probs2, b_kc=False)
        for p in pres:
            bv[p] = xchain[p]
        return bv

    def _flush_xattn_bwd(self):
        """Cross-attention value-chain backward of every block (t2i_moe_gan.py:549-556), level by level in
        batched launches: weight gradients (fp32 atomics), bias gradients, data gradients; the text-sequence
        gradient of all blocks accumulates with fp32 atomics."""
        items, self._xattn_bwd = self._xattn_bwd, []
        if not items:
            return
        dev = self.dev
        for q in items:
            C, pre = q["C"], q["pre"]
            q["Wo"] = self.P(pre + "cross_attn.out_proj.weight")
            q["Wv"] = self.P(pre + "cross_attn.in_proj_weight")[2 * C:]
            q["Wt"] = self.P(pre + "text_proj.weight")
            q["gWo"] = self.G(pre + "cross_attn.out_proj.weight")
            q["gWv"] = self.G(pre + "cross_attn.in_proj_weight")[2 * C:]
            q["gWt"] = self.G(pre + "text_proj.weight")
            q["gbo"] = self.G(pre + "cross_attn.out_proj.bias")
            q["gbv"] = self.G(pre + "cross_attn.in_proj_bias")[2 * C:]
            q["gbt"] = self.G(pre + "text_proj.bias")
        # (gradient in, saved input, weight, weight grad, bias grad, gradient out)
        levels = (("g_ca", "vv", "Wo", "gWo", "gbo", "g_vv"), ("g_vv", "tp", "Wv", "gWv", "gbv", "g_tp"),
                  ("g_tp", "text_seq", "Wt", "gWt", "gbt", None))
        for gin, xin, Wk, gWk, gbk, gout in levels:
            wg, dg = [], []
            for q in items:
                g, x, Wm = q[gin], q[xin], q[Wk]
                M, N = g.shape
                K = x.shape[1]
                wg.append(dict(A=g, B=x, M=N, N=K, K=M, out=q[gWk], ldc=q[gWk].stride(0), ep=E_(atomic=1)))
                if gout is None:  # d text_seq, shared by the blocks
                    dg.append(dict(A=g, B=Wm, M=M, N=Wm.shape[1], K=N, out=q["g_text_seq"], ep=E_(atomic=1)))
                else:
                    q[gout] = torch.empty(M, Wm.shape[1], device=dev)
                    dg.append(dict(A=g, B=Wm, M=M, N=Wm.shape[1], K=N, out=q[gout]))
                ops.colsum(g, q[gbk], defer=True)
            ops.gemm_batch(wg, a_kc=False, b_kc=False)
            ops.gemm_batch(dg, a_kc=True, b_kc=False)

    def _flush_router_bwd(self):
        """Router parameter backward of every block (t2i_moe_gan.py:364-389 through :302-333) in batched
        launches: dWf, dWc, dWt, d w (fp32 atomics into the shared latent gradient), then the per-parameter
        reparameterisation / KL backward."""
        items, self._router_bwd = self._router_bwd, []
        if not items:
            return
        ops.fold_flush()  # the router feature gradients G1 are folds (deferred inside a training step)
        dev = self.dev
        pa, pb, pc, pd = [], [], [], []
        for q in items:
            C, E, B, Wc = q["C"], q["E"], q["B"], q["Wc"]
            q["gWf"] = torch.empty(C, 128, device=dev)
            q["gWc"] = torch.empty(256, E, device=dev)
            q["g_u"] = torch.empty(B, 128, device=dev)
            q["gWt"] = torch.empty(q["w"].shape[1], 128, device=dev)
            pa.append(dict(A=q["G1"], B=Wc[:128], M=C, N=128, K=E, out=q["gWf"]))  # G1 @ Wc1^T
            pa.append(dict(A=q["gsum"], B=Wc[128:], M=B, N=128, K=E, out=q["g_u"]))  # gsum @ Wc2^T
            pb.append(dict(A=q["Wf"], B=q["G1"], M=128, N=E, K=C, out=q["gWc"][:128]))  # Wf^T G1
            pb.append(dict(A=q["u"], B=q["gsum"], M=128, N=E, K=B, out=q["gWc"][128:]))  # u^T gsum
            pc.append(dict(A=q["w"], B=q["g_u"], M=q["w"].shape[1], N=128, K=B, out=q["gWt"]))  # w^T g_u
            pd.append(dict(A=q["g_u"], B=q["Wt"], M=B, N=q["w"].shape[1], K=128, out=q["gw"],
                           ep=E_(atomic=1)))  # gw += g_u Wt^T
        ops.gemm_batch(pa)
        ops.gemm_batch(pb, a_kc=False, b_kc=False)
        ops.gemm_batch(pc, a_kc=False, b_kc=False)
        ops.gemm_batch(pd)
        # the reparameterisation / KL backward of every router parameter of every block: one launch
        ops.router_param_bwd_batch(
            [(self.P(q["r"] + nm + "_mu"), self.P(q["r"] + nm + "_rho"), q["eps"][epi], gWx, q["kl_coef"],
              self.G(q["r"] + nm + "_mu"), self.G(q["r"] + nm + "_rho"))
             for q in items for nm, gWx, epi in (("feature", q["gWf"], 0), ("text", q["gWt"], 1),
                                                 ("combined", q["gWc"], 2))],
            flags=self.guard_flags, mask=ops.FLAG_G_BAD)

    def _cbuf(self):
        return self.st.shadow if self.st.shadow is not None else self.st.data

    def moe_bwd(self, pre, sv, g_out, g_tok, gw, coef=None, kl_coef=None, g_probs=None, g_logits=None):
        """g_out: grad of (resid + moe) [T, C]; writes g_tok (grad of the LN3 tokens); accumulates gw."""
        r = pre + "router."
        tok, w, Y, Pre = sv["tok"], sv["w"], sv["Y"], sv["Pre"]
        T, C = tok.shape
        B = w.shape[0]
        E, k = self.E, sv["topi"].shape[1]
        n = T * k
        Hd = 4 * C
        row_off, tile_off, perm = sv["row_off"], sv["tile_off"], sv["perm"]
        ex = pre + "experts."
        g_gate = ops.moe_gate_grad(g_out, Y, sv["pos_of"], T, k)
        # gate-weighted output gradient in dispatch order: gG[r] = gate[r] * g_out[token(r)]
        gG = ops.gather_rows(g_out, perm, k, rowscale=sv["gate_pos"])
        gW2 = self.st.group_view(ex + "0.net.2.weight", f"{ex}{E-1}.net.2.weight", self.st.grad)
        gb2 = self.st.group_view(ex + "0.net.2.bias", f"{ex}{E-1}.net.2.bias", self.st.grad)
        gW1 = self.st.group_view(ex + "0.net.0.weight", f"{ex}{E-1}.net.0.weight", self.st.grad)
        gb1 = self.st.group_view(ex + "0.net.0.bias", f"{ex}{E-1}.net.0.bias", self.st.grad)
        gP = torch.empty(n, Hd, device=self.dev, dtype=self.cdt)
        gX = torch.empty(n, C, device=self.dev, dtype=self.cdt)
        fused = ops.ffn_bwd_fusable(self.cdt, C)
        Hid = sv["Hid"]
        if fused:
            # one pass per 128-row tile: gP = (gG W2_e) * GELU'(pre), gX = gP W1_e, gb1 column sums, and GELU(pre)
            # from the same erf evaluation for the W2 weight gradient (mg_moe_ffn_bwd): an 8-B store per 4 hidden
            # units instead of the GELU formed on load in that GEMM's K loop
            if Hid is None:
                Hid = torch.empty(n, Hd, device=self.dev, dtype=self.cdt)
            ops.moe_ffn_bwd(gG, Pre, sv["W1"].view(E, Hd, C), sv["W2"].view(E, C, Hd), row_off, tile_off,
                            sv["max_tiles"], gP, gX, gb1.view(E, Hd), gb2.view(E, C), hid=Hid)
        else:
            # expert layer 2: dH = gG @ W2_e, times GELU'(pre)
            ops.gemm_grouped(gG, sv["W2"], row_off, tile_off, sv["max_tiles"], Hd, C, b_kc=False, b_gstride=C * Hd,
                             out=gP, ldb=Hd, ep=E_(act=MUL_GELU_GRAD, aux=Pre, ld_aux=Hd))
        if Hid is not None:
            gw2 = lambda: ops.gemm_grouped_wgrad(gG, Hid, row_off, n, C, Hd, gW2)  # noqa: E731
        else:  # GELU(Pre) formed by the B loader (the forward kept only the pre-activation)
            gw2 = lambda: ops.gemm_grouped_wgrad(gG, Pre, row_off, n, C, Hd, gW2, b_gelu=1)  # noqa: E731
        self.side.run(lambda: (gw2(), None if fused else ops.grouped_colsum(gG, row_off, C, n, gb2)), gG)
        # expert layer 1
        if not fused:
            ops.gemm_grouped(gP, sv["W1"], row_off, tile_off, sv["max_tiles"], C, Hd, b_kc=False, b_gstride=Hd * C,
                             out=gX, ldb=C)
        self.side.run(lambda: (ops.gemm_grouped_wgrad(gP, sv["Xg"], row_off, n, Hd, C, gW1),
                               None if fused else ops.grouped_colsum(gP, row_off, Hd, n, gb1)), gP)
        if self.on_grad_final is not None:  # this block's expert parameters receive no further gradient
            ops.fold_flush()  # (a weight-gradient fold deferred on this stream lands before the bucket's all-reduce)
            lo = self.st.offsets[ex + "0.net.0.weight"][0]
            o, nl = self.st.offsets[f"{ex}{E-1}.net.2.bias"]
            self.on_grad_final(lo, o + nl)
        # router
        g_raw, gsum = ops.router_bwd(sv["probs"], sv["zlog"], sv["topi"], sv["gate"], g_gate, g_probs, coef,
                                     sv["HW"], self.P(r + "temperature"), sv["anneal"], self.G(r + "temperature"), B,
                                     g_logits=g_logits)
        ops.moe_token_grad(gX, sv["pos_of"], g_raw, sv["Wfc"], g_tok, k)
        G1 = ops.zeros(C, E, device=self.dev)
        ops.router_feat_grad(tok, g_raw, G1)
        # the router's parameter GEMMs depend only on (G1, gsum) and saved vectors: run for every block at
        # the end of the backward, batched (_flush_router_bwd)
        self._router_bwd.append(dict(r=r, C=C, E=E, B=B, G1=G1, gsum=gsum, Wf=sv["Wf"], Wt=sv["Wt"], Wc=sv["Wc"],
                                     u=sv["u"], w=w, gw=gw, eps=sv["eps"], kl_coef=kl_coef))

    # ------------------------------------------------------------------
    # AttentionBlock  (t2i_moe_gan.py:493-576)
    # ------------------------------------------------------------------
    def attn_fwd(self, pre, x, w, text_seq, eps, anneal, train=True, save=True, kl_out=None):
        B, H, W, C = x.shape
        L_ = H * W
        T = B * L_
        xf0, sv_in = self.mc_fwd(pre + "proj_in.", x, w, save=save)
        xf0 = xf0.view(T, C)
        n1, mu1, rs1 = ops.layernorm_fwd(xf0, self.P(pre + "norm1.weight"), self.P(pre + "norm1.bias"))
        qkv = ops.linear(n1, self.Pc(pre + "self_attn.in_proj_weight"), bias=self.P(pre + "self_attn.in_proj_bias"))
        att, lse = ops.attn_fwd(qkv, B, L_, C)
        # cross-attention against the single text token: softmax over one key == 1 (:553-555)
        bv = self._bv.get(pre) if self._bv is not None else None
        if bv is not None:
            tp, vv, ca = bv["tp"], bv["vv"], bv["ca"]
        else:
            ca_W = self.P(pre + "cross_attn.in_proj_weight")
            ca_b = self.P(pre + "cross_attn.in_proj_bias")
            tp = ops.linear(text_seq, self.P(pre + "text_proj.weight"), bias=self.P(pre + "text_proj.bias"))
            vv = ops.linear(tp, ca_W[2 * C:], bias=ca_b[2 * C:])
            ca = ops.linear(vv, self.P(pre + "cross_attn.out_proj.weight"),
                            bias=self.P(pre + "cross_attn.out_proj.bias"))
        xf1 = ops.linear(att, self.Pc(pre + "self_attn.out_proj.weight"), bias=self.P(pre + "self_attn.out_proj.bias"),
                         resid=xf0, ld_res=C, addvec=ca, add_shift=ops.ilog2(L_), add_ld=C)
        n3, mu3, rs3 = ops.layernorm_fwd(xf1, self.P(pre + "norm3.weight"), self.P(pre + "norm3.bias"))
        s_out = self._batched_style(pre + "proj_out.", C)
        if s_out is not None and (L_ & (L_ - 1)) == 0:  # proj_out's x * s written by the combine itself
            xpre, probs, kl2, topi, sv_moe, xs_out = self.moe_fwd(pre + "moe.", n3, xf1, w, L_, eps, anneal, train,
                                                                  save, kl_out=kl_out, out_style=s_out)
            xs_out = xs_out.view(B, H, W, C)
        else:
            xpre, probs, kl2, topi, sv_moe = self.moe_fwd(pre + "moe.", n3, xf1, w, L_, eps, anneal, train, save,
                                                          kl_out=kl_out)
            xs_out = None
        out, sv_out = self.mc_fwd(pre + "proj_out.", xpre.view(B, H, W, C), w, save=save, xs=xs_out)
        sv = None
        if save:
            sv = dict(sv_in=sv_in, xf0=xf0, n1=n1, mu1=mu1, rs1=rs1, qkv=qkv, att=att, lse=lse, tp=tp, vv=vv,
                      xf1=xf1, n3=n3, mu3=mu3, rs3=rs3, sv_moe=sv_moe, sv_out=sv_out, text_seq=text_seq, B=B, L=L_)
        return out, probs, kl2, topi, sv

    def attn_bwd(self, pre, sv, g_out, gx, gw, g_text_seq, coef=None, kl_coef=None, g_probs=None):
        B, L_ = sv["B"], sv["L"]
        T, C = sv["xf0"].shape
        g_xpre = torch.empty(T, C, device=self.dev, dtype=self.cdt)
        self.mc_bwd(pre + "proj_out.", sv["sv_out"], g_out, g_xpre, gw)
        # MoE branch -> LN3 -> residual
        g_n3 = torch.empty(T, C, device=self.dev, dtype=self.cdt)
        self.moe_bwd(pre + "moe.", sv["sv_moe"], g_xpre, g_n3, gw, coef=coef, kl_coef=kl_coef, g_probs=g_probs)
        g_xf1 = g_xpre  # residual path, accumulate LN3 backward into it
        ops.layernorm_bwd(g_n3, sv["xf1"], sv["mu3"], sv["rs3"], self.P(pre + "norm3.weight"), g_xf1,
                          self.G(pre + "norm3.weight"), self.G(pre + "norm3.bias"), accumulate=1)
        # cross-attention vector: sum over each image's tokens
        g_ca = ops.zeros(B, C, device=self.dev)
        ops.segsum(g_xf1, B, L_, C, g_ca)
        # the rest of the cross-attention chain depends only on g_ca and saved vectors: batched over the
        # blocks at the end of the backward (_flush_xattn_bwd)
        self._xattn_bwd.append(dict(pre=pre, C=C, B=B, g_ca=g_ca, vv=sv["vv"], tp=sv["tp"], text_seq=sv["text_seq"],
                                    g_text_seq=g_text_seq))
        # self-attention
        g_att = ops.linear_dgrad(g_xf1, self.Pc(pre + "self_attn.out_proj.weight"))
        ops.linear_wgrad(g_xf1, sv["att"], self.G(pre + "self_attn.out_proj.weight"))
        # out_proj bias gradient = column sums of g_xf1 = the sum over images of g_ca (deferred: g_xf1 itself is
        # accumulated into below, g_ca is not)
        ops.colsum(g_ca, self.G(pre + "self_attn.out_proj.bias"), defer=True)
        g_qkv = ops.attn_bwd(sv["qkv"], sv["att"], g_att, sv["lse"], B, L_, C)
        g_n1 = ops.linear_dgrad(g_qkv, self.Pc(pre + "self_attn.in_proj_weight"))
        gWqkv, gbqkv = self.G(pre + "self_attn.in_proj_weight"), self.G(pre + "self_attn.in_proj_bias")
        self.side.run(lambda: (ops.linear_wgrad(g_qkv, sv["n1"], gWqkv), ops.colsum(g_qkv, gbqkv, defer=True)), g_qkv)
        g_xf0 = g_xf1
        ops.layernorm_bwd(g_n1, sv["xf0"], sv["mu1"], sv["rs1"], self.P(pre + "norm1.weight"), g_xf0,
                          self.G(pre + "norm1.weight"), self.G(pre + "norm1.bias"), accumulate=1)
        self.mc_bwd(pre + "proj_in.", sv["sv_in"], g_xf0, gx, gw)
        if not self._defer:  # called on its own: complete this block's gradients now
            self._flush_router_bwd()
            self._flush_xattn_bwd()

    # ------------------------------------------------------------------
    # AuroraGenerator  (t2i_moe_gan.py:762-855)
    # ------------------------------------------------------------------
    def _mapping(self, zt, save):
        hs = [zt]
        h = zt
        for i in (0, 2, 4):
            h = ops.linear(h, self.Pp(f"mapping.{i}.weight"), bias=self.P(f"mapping.{i}.bias"), act=LRELU)
            hs.append(h)
        return h, hs

    def _prefix_fwd(self, z, text, psi, save):
        """The part of the forward that does not depend on the router samples: text projection, mapping,
        truncation, every style / demodulation, the constant and gen_block_4's convolution block.  Given the
        same z, text and weights it is identical in the D-phase and G-phase forwards of one step
        (t2i_moe_gan.py:1288-1296 and :1351-1357 feed the same z; G is not updated in between)."""
        B = z.shape[0]
        dev = self.dev
        if text.shape[0] != B and text.shape[0] == 1:
            text = text.expand(B, -1).contiguous()
        # text projection (:682-687, :790)
        text_c = self._p(text)
        t0 = ops.linear(text_c, self.Pp("text_projection.0.weight"), bias=self.P("text_projection.0.bias"),
                        out_dtype=torch.float32)
        t1, tmu, trs = ops.layernorm_fwd(t0, self.P("text_projection.1.weight"), self.P("text_projection.1.bias"),
                                         act=1)
        t1c = self._p(t1)
        text_seq = ops.linear(t1c, self.Pp("text_projection.3.weight"), bias=self.P("text_projection.3.bias"),
                              out_dtype=torch.float32)
        # mapping + truncation (:793-808).  The truncation centre mapping(0) (:802-806, no gradient) rides along as
        # an extra all-zero row B of the mapping GEMMs instead of its own chain of M = 1 launches; the backward
        # reads only rows [0, B) of the saved activations
        trunc = psi < 1.0
        zt = (ops.zeros(B + 1, z.shape[1] + text.shape[1], device=dev, dtype=self.pdt) if trunc else
              torch.empty(B, z.shape[1] + text.shape[1], device=dev, dtype=self.pdt))
        ops.copy2d(z, zt, B, z.shape[1], ldo=zt.shape[1])
        ops.copy2d(text, zt[:, z.shape[1]:], B, text.shape[1], ldo=zt.shape[1])
        h3e, hs = self._mapping(zt, save)
        h3 = h3e[:B]
        if trunc:
            # w = mean + psi (w_full - mean) = psi * h3 W6^T + beff, beff = (1 - psi) * m3 W6^T + b6 (one M = 1 GEMM)
            beff = ops.linear(h3e[B:B + 1], self.Pp("mapping.6.weight"), bias=self.P("mapping.6.bias"), alpha=1.0 - psi,
                              out_dtype=torch.float32).view(-1)
            w = ops.linear(h3, self.Pp("mapping.6.weight"), bias=beff, alpha=psi, out_dtype=torch.float32)
        else:
            w = ops.linear(h3, self.Pp("mapping.6.weight"), bias=self.P("mapping.6.bias"), out_dtype=torch.float32)
        w_c = self._p(w)
        # every modulated conv's style in one GEMM: S = w @ [W_mod ...]^T + [b_mod ...] (:158)
        S = S2 = D = None
        if self.style_cols:
            S = ops.linear(w_c, self.style_Wc, bias=self.style_b, out_dtype=torch.float32)
            S2 = ops.cast(S, square=1)
            # and every demodulation d = rsqrt(s^2 @ wsq^T + 1e-8) in batched launches (:165)
            D, probs = {}, []
            for pre, c in self.style_cols.items():
                pk = self.packs[pre]
                rows, Cin = pk["rows"], self.P(pre + "weight").shape[1]
                d = torch.empty(B, rows, device=dev)
                D[pre] = d
                probs.append(dict(A=S2[:, c:c + Cin], B=pk["wsq"], M=B, N=rows, K=Cin, out=d, ep=E_(act=RSQRT)))
            ops.gemm_batch(probs)
        self._S, self._S2, self._D = S, S2, D
        x = ops.const_fwd(self.P("constant"), B, self.cdt)
        name0, _, _, _, up0, _ = self.blocks[0]
        assert not up0
        x0, cbsv0 = self.cb_fwd(name0 + ".conv_block.", x, w, save=save)
        xchain = self._xattn_chain(text_seq) if self.attn_blocks else {}
        return dict(B=B, text=text, text_c=text_c, t0=t0, t1=t1, t1c=t1c, tmu=tmu, trs=trs, text_seq=text_seq,
                    hs=hs, h3=h3, w=w, w_c=w_c, psi=psi, S=S, S2=S2, D=D, x0=x0, cbsv0=cbsv0, save=save,
                    xchain=xchain)

    def forward(self, z, text, eps, anneal=1.0, psi=0.7, train=True, save=True, want_img8=False, want_kl=True,
                keep_prefix=False, prefix=None):
        """Returns (img [B,R,R,8] padded NHWC, the intermediate R/2 image or None, kl2 list, probs list, ctx);
        R = max_res (16: the reference generator, img16 / img8).  kl2 / probs / eps: one per attention block.
        ``want_kl=False`` skips the routers' KL terms (their kl2 entries are None).
        ``keep_prefix=True`` computes the router-independent prefix (``_prefix_fwd``) with its saved
        activations and returns it as ``self.last_prefix``; ``prefix=`` reuses such a prefix (same z, text,
        psi and weights) instead of recomputing it."""
        self._want_kl = want_kl
        if prefix is None:
            prefix = self._prefix_fwd(z, text, psi, save or keep_prefix)
        else:
            assert prefix["B"] == z.shape[0] and prefix["psi"] == psi and (prefix["save"] or not save)
            self._S, self._S2, self._D = prefix["S"], prefix["S2"], prefix["D"]
        self.last_prefix = prefix if keep_prefix else None
        B = prefix["B"]
        w, text_seq = prefix["w"], prefix["text_seq"]
        self._bv = self._block_vectors(w, text_seq, eps, train, prefix["xchain"])
        probs, kl2s, topis, blocks = [], [], [], []
        # every block's two KL terms in one [blocks, 2] buffer (no stack of per-block results afterwards)
        klbuf = (torch.empty(len(self.attn_blocks), 2, device=self.dev, dtype=torch.float32)
                 if train and self._want_kl else None)
        if klbuf is not None:  # the KL terms depend on the router parameters only: all blocks in two launches
            ops.router_kl_batch([tuple(self.P(f"{name}.attn_block.moe.router.{t}") for t in (
                "feature_mu", "feature_rho", "text_mu", "text_rho", "combined_mu", "combined_rho"))
                for (name, _, _, _, _, attn) in self.blocks if attn], klbuf)
        img8, rgb8sv = None, None
        x = None
        ai = 0
        for i, (name, cin, cout, res, up, attn) in enumerate(self.blocks):
            if i == 0:
                x, cbsv = prefix["x0"], (prefix["cbsv0"] if save else None)
            else:
                skip_xs = None
                if up:
                    s_skip = (self._batched_style(name + ".conv_block.skip_proj.", x.shape[-1])
                              if (name + ".conv_block.skip_proj.weight") in self.st.offsets else None)
                    if s_skip is not None:  # the skip conv's x * s from the upsample pass itself
                        x, skip_xs = ops.upsample2x(x, style=s_skip)
                    else:
                        x = ops.upsample2x(x)
                x, cbsv = self.cb_fwd(name + ".conv_block.", x, w, save=save, skip_xs=skip_xs)
            asv = None
            if attn:
                x, p, kl2, topi, asv = self.attn_fwd(name + ".attn_block.", x, w, text_seq,
                                                     None if eps is None else eps[ai], anneal, train, save,
                                                     kl_out=None if klbuf is None else klbuf[ai])
                ai += 1
                probs.append(p)
                kl2s.append(kl2)
                topis.append(topi)
            blocks.append((cbsv, asv, up))
            if name == self.half_block and want_img8:
                img8, rgb8sv = self.mc_fwd(self.rgb_half, x, w, save=save)
        img16, rgbsv = self.mc_fwd(self.rgb_final, x, w, save=save)
        self._S = self._S2 = self._D = None
        self._bv = None
        ctx = None
        if save:
            ctx = {k: prefix[k] for k in ("B", "text", "text_c", "t0", "t1", "t1c", "tmu", "trs", "text_seq", "hs",
                                          "h3", "w", "w_c", "psi")}
            ctx.update(z=z, blocks=blocks, rgbsv=rgbsv, rgb8sv=rgb8sv)
        self.last_klbuf = klbuf  # kl2s are its rows (TrainStep reads the buffer instead of stacking them)
        return img16, img8, kl2s, probs, topis, ctx

    def backward(self, ctx, g_img16, coef=None, kl_coef=None, want_input_grads=False, g_probs=None, g_img8=None):
        """Accumulate all generator parameter gradients for d loss / d img16 (+ balance coef on the last
        router, + KL coefficients [3] per router).  Optional: per-router d loss / d probs [T, E] (g_probs list)
        and d loss / d img8 (needs forward(..., want_img8=True, save=True)).  Returns (gz, gtext) if requested."""
        B = ctx["B"]
        dev = self.dev
        gw = ops.zeros(B, 512, device=dev)
        g_ts = ops.zeros(B, 512, device=dev)
        self._router_bwd, self._xattn_bwd = [], []
        self._defer = True  # per-block small GEMMs are batched over the blocks after the block loop
        if self.style_cols:
            self._GS = ops.zeros(B, self.style_n, device=dev)
            self._demod_bwd = []
        sv = ctx["rgbsv"]
        x_last = sv[0]
        gx = torch.empty(x_last.shape, device=dev, dtype=self.cdt)
        self.mc_bwd(self.rgb_final, sv, g_img16, gx, gw)
        na = len(self.attn_blocks)
        ai = na
        for i in reversed(range(len(self.blocks))):
            name = self.blocks[i][0]
            cbsv, asv, up = ctx["blocks"][i]
            if name == self.half_block and g_img8 is not None:
                self.mc_bwd(self.rgb_half, ctx["rgb8sv"], g_img8, gx, gw, accumulate=1)
            if asv is not None:
                ai -= 1
                g_cb = torch.empty(gx.shape, device=dev, dtype=self.cdt)
                kc = None if kl_coef is None else kl_coef[ai:ai + 1]
                self.attn_bwd(name + ".attn_block.", asv, gx, g_cb, gw, g_ts, coef=coef if ai == na - 1 else None,
                              kl_coef=kc, g_probs=None if g_probs is None else g_probs[ai])
            else:
                g_cb = gx
            x_in = cbsv[0][0]  # input of mtm1
            g_in = torch.empty(x_in.shape, device=dev, dtype=self.cdt)
            self.cb_bwd(name + ".conv_block.", cbsv, g_cb, g_in, gw)
            if up:
                Bq, H2, W2, Cq = g_in.shape
                gprev = torch.empty(Bq, H2 // 2, W2 // 2, Cq, device=dev, dtype=self.cdt)
                ops.upsample2x_bwd(g_in, gprev)
                gx = gprev
            else:
                gx = g_in
        ops.const_bwd(gx, self.G("constant"))
        self._flush_router_bwd()
        self._flush_xattn_bwd()
        self._defer = False
        self.side.join()  # every weight gradient is in place before the demodulation backward adds to it
        if self._GS is not None:  # all modulated convs' demodulation and style backward at once
            pw, pg = [], []
            for pre, gdd, s2, s, gs, Cin, rows, Cout in self._demod_bwd:
                gwsq = torch.empty(rows, Cin, device=dev)  # gdd^T s^2
                pw.append(dict(A=gdd, B=s2, M=rows, N=Cin, K=B, out=gwsq, lda=rows, ldb=s2.stride(0)))
                pg.append(dict(A=gdd, B=self.packs[pre]["wsq"], M=B, N=Cin, K=rows, out=gs, ldc=gs.stride(0),
                               ep=E_(alpha=2.0, scale=s, scale_ld=s.stride(0), accumulate=1)))  # gs += 2 s (gdd@wsq)
            ops.gemm_batch(pw, a_kc=False, b_kc=False)
            ops.gemm_batch(pg, a_kc=True, b_kc=False)
            pb = ops.PrepBatch(torch.float32)
            for (pre, _, _, _, _, Cin, rows, Cout), q in zip(self._demod_bwd, pw):
                pb.wsq_bwd(self.P(pre + "weight"), q["out"][:Cout], self.G(pre + "weight"))
            pb.run()
            self._demod_bwd = []
            GS, self._GS = self._GS, None
            GSc = self._p(GS)
            ops.linear_wgrad(GSc, ctx["w_c"], self.style_gW)
            ops.colsum(GS, self.style_gb, defer=True)
            ops.gemm(GSc, self.style_Wc, B, gw.shape[1], self.style_n, b_kc=False, out=gw, ep=E_(accumulate=1))
        # truncation: w = mean + psi (w_full - mean), mean under no_grad
        psi = ctx["psi"]
        g6 = ops.cast(gw, self.pdt, alpha=psi if psi < 1.0 else 1.0)
        hs = [h[:g6.shape[0]] for h in ctx["hs"]]  # (rows past B: the truncation centre's zero row, no gradient)
        ops.linear_wgrad(g6, hs[3], self.G("mapping.6.weight"))
        ops.colsum(g6, self.G("mapping.6.bias"), defer=True)
        # each data gradient leaves its GEMM already times lrelu'(the layer output below it) (the epilogue's
        # MUL_LRELU_GRAD; the input rows of the first layer take none)
        g = ops.linear_dgrad(g6, self.Pp("mapping.6.weight"), lrelu_out=hs[3])
        for j, i in enumerate((4, 2, 0)):
            ops.linear_wgrad(g, hs[2 - j], self.G(f"mapping.{i}.weight"))
            ops.colsum(g, self.G(f"mapping.{i}.bias"), defer=True)
            if i != 0 or want_input_grads:
                g = ops.linear_dgrad(g, self.Pp(f"mapping.{i}.weight"), lrelu_out=hs[2 - j] if i != 0 else None)
        g_zt = g if want_input_grads else None
        # text projection backward
        g_tsc = self._p(g_ts)
        ops.linear_wgrad(g_tsc, ctx["t1c"], self.G("text_projection.3.weight"))
        ops.colsum(g_ts, self.G("text_projection.3.bias"), defer=True)
        if ctx["t1"].dtype == torch.float32 and ctx["t1"].is_contiguous():
            g_t1 = ops.linear_dgrad(g_tsc, self.Pp("text_projection.3.weight"), out_dtype=torch.float32,
                                    lrelu_out=ctx["t1"])
        else:
            g_t1 = ops.linear_dgrad(g_tsc, self.Pp("text_projection.3.weight"), out_dtype=torch.float32)
            ops.lrelu_mask_mul(g_t1, ctx["t1"], g_t1)
        g_t0 = torch.empty_like(g_t1)
        ops.layernorm_bwd(g_t1, ctx["t0"], ctx["tmu"], ctx["trs"], self.P("text_projection.1.weight"), g_t0,
                          self.G("text_projection.1.weight"), self.G("text_projection.1.bias"))
        ops.linear_wgrad(self._p(g_t0), ctx["text_c"], self.G("text_projection.0.weight"))
        ops.colsum(g_t0, self.G("text_projection.0.bias"), defer=True)
        if not want_input_grads:
            return None, None
        gtext = ops.linear_dgrad(g_t0, self.P("text_projection.0.weight"))
        zd = ctx["z"].shape[1]
        gz = g_zt[:, :zd].float().contiguous()
        gtext = gtext + g_zt[:, zd:].float()
        return gz, gtext
