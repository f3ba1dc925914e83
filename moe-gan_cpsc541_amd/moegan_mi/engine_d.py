"""Explicit discriminator forward/backward, GAN losses and the R1 double backward.

AuroraDiscriminator (t2i_moe_gan.py:858-907) on the HIP kernels, NHWC:
    a0 = conv0(img) [4x4/s2/p1, 3->128]   h0 = LReLU(a0)
    a1 = conv1(h0)  [4x4/s2/p1, 128->256] h1 = LReLU(a1)
    t  = LReLU(WN-Linear(text))           out = head([h1 | tile(t)])  (4x4 valid, 384->1)
The head's 128 text channels are spatially constant, so their contribution is
a per-image scalar tb[b] = sum_c t[b,c] * sum_taps W2[256+c] (+ bias); the
mismatched-text pass therefore reuses the real pass's image features and only
re-indexes tb (t2i_moe_gan.py:1303-1305: D(real.detach(), text[perm])).

R1 (t2i_moe_gan.py:1282-1286) is computed in closed form.  With masks
m0 = LReLU'(a0), m1 = LReLU'(a1) (piecewise constant, zero second derivative):
    g_x   = C0^T m0 C1^T m1 Gh1           (Gh1 = head^T(ones), identical for every image)
    r1    = gamma/2 * mean_b ||g_x_b||^2, u = gamma/B * g_x
    dW0  += wgrad0(x=u, dy=m0 C1^T m1 Gh1)
    v1    = m1 C1(m0 C0 u)
    dW1  += wgrad1(x=m0 C0 u, dy=m1 Gh1);   dW2[:256] += head_wgrad(x=v1, dy=ones)
All weights are weight-normed (g * v / ||v||); gradients flow back to g and v.
"""
import os

import torch

from . import _lib as L
from . import graphs, ops

E_ = ops.E
MUL_LRELU_GRAD, LRELU = L.ACT_MUL_LRELU_GRAD, L.ACT_LRELU
WN_LAYERS = ("conv_layers.0.", "conv_layers.2.", "output_layer.0.", "text_projection.0.")


class DiscriminatorEngine:
    def __init__(self, store, cdt=torch.float32):
        self.st = store
        self.cdt = cdt
        # conv_layers.0 on the direct MFMA kernels (mg_d0_*) in the bf16 step; MOEGAN_D0_DIRECT=0: im2col + GEMMs
        self.direct0 = cdt == torch.bfloat16 and os.environ.get("MOEGAN_D0_DIRECT", "1") == "1"
        self.dev = store.device
        self.ones_cache = {}
        # weight gradients on a side stream, overlapping the data-gradient chain (joined before finish_grads)
        self.side = graphs.SideStream(self.dev, enabled=graphs.side_streams_enabled(self.dev))

    def _d0_ok(self, H):
        """conv_layers.0 on the direct kernels at this (square) image size: mg_d0_* take W / 2 a power of two in
        [4, 64] and H a multiple of 4; any other even size keeps the im2col + GEMM path."""
        ow = H // 2
        return self.direct0 and H % 4 == 0 and 4 <= ow <= 64 and (ow & (ow - 1)) == 0

    def _head_ok(self, Hf):
        """The per-image head kernels (mg_d_head_*): 4 <= Hf <= 32 and Hf^2 a multiple of 16."""
        return self.direct0 and 4 <= Hf <= 32 and (Hf * Hf) % 16 == 0

    def P(self, n):
        return self.st.view(n)

    def G(self, n):
        return self.st.gview(n)

    def _ones(self, n):
        if n not in self.ones_cache:
            self.ones_cache[n] = torch.ones(n, device=self.dev)
        return self.ones_cache[n]

    # ------------------------------------------------------------------
    def prep(self):
        """Weight-norm the four layers and pack them (call after every D optimizer step)."""
        outs = ops.weight_norm_fwd_batch([(self.P(pre + "weight_v"), self.P(pre + "weight_g")) for pre in WN_LAYERS])
        W = {pre: o[0] for pre, o in zip(WN_LAYERS, outs)}
        norm = {pre: o[1] for pre, o in zip(WN_LAYERS, outs)}
        self.W, self.norm = W, norm
        cdt = self.cdt
        pb = ops.PrepBatch(cdt)  # the packs in one launch
        self.W0p = pb.pack(W["conv_layers.0."])  # [128, 48] (k = tap*3 + c)
        self.W1p = pb.pack(W["conv_layers.2."])  # [256, 16*128]
        self.W1cls = pb.pack_dgrad_s2(W["conv_layers.2."])  # [4, 128, 4*256]
        pb.run()
        W2 = W["output_layer.0."].view(384, 16)
        self.W2img = W2[:256]
        # head as GEMMs: P = h1 @ W2img ([pix, 16 taps]) and g_a1 = G @ W2img^T
        self.W2img_c = ops.cast(self.W2img.contiguous(), cdt)  # [256 ch, 16 taps]  (KC B operand of g_a1)
        self.W2t_c = ops.cast(self.W2img.t().contiguous(), cdt)  # [16 taps, 256 ch] (KC B operand of P)
        self.w2sum = ops.gemm(W2[256:], self._ones(16).view(1, 16), 128, 1, 16).view(128)
        self.Wt = W["text_projection.0."]

    # ------------------------------------------------------------------
    def text_branch(self, text):
        t = ops.linear(text, self.Wt, bias=self.P("text_projection.0.bias"), act=LRELU)  # [B,128]
        tb = ops.gemm(t, self.w2sum.view(1, 128), t.shape[0], 1, 128, ep=E_(bias=self.P("output_layer.0.bias")))
        return t, tb.view(-1)

    def conv_stack(self, img, layout, B, H):
        """img: NCHW fp32 (layout 'nchw') or NHWC padded [B,H,W,ld] (layout ('nhwc', ld))."""
        if layout == "nchw":
            strides = (3 * H * H, H, 1, H * H)
        else:
            ld = layout[1]
            strides = (H * H * ld, H * ld, ld, 1)
        if self._d0_ok(H):  # direct MFMA conv (mg_d0_fwd): no im2col matrix; the backward re-gathers from the image
            cols = (img, strides)
            h0 = ops.d0_fwd(img, strides, B, H, H, self.W0p, bias=self.P("conv_layers.0.bias"))
        else:
            cols = ops.im2col_4x4s2(img, strides, B, H, H, 3, 48, self.cdt)  # [B*(H/2)^2, 48]
            h0 = ops.linear(cols, self.W0p, bias=self.P("conv_layers.0.bias"), act=LRELU).view(B, H // 2, H // 2, 128)
        h1 = ops.conv2d(h0, self.W1p, 256, 4, 4, 2, 1, ep=E_(bias=self.P("conv_layers.2.bias"), act=LRELU),
                        tag="d_conv1")
        return cols, h0, h1

    def forward(self, img, layout, text, B, H):
        cols, h0, h1 = self.conv_stack(img, layout, B, H)
        Hf = H // 4
        if self._head_ok(Hf):  # one kernel per image (mg_d_head_fwd)
            img_part = ops.d_head_fwd(h1, self.W2t_c, B, Hf)
        else:
            P = ops.gemm(h1.view(-1, 256), self.W2t_c, B * Hf * Hf, 16, 256, out_dtype=torch.float32)
            img_part = ops.disc_head_sum(P, B, Hf)  # [B, (H/4-3)^2]
        return dict(cols=cols, h0=h0, h1=h1, img_part=img_part, H=H, B=B)

    # ------------------------------------------------------------------
    def stack_backward(self, f, g_img_part, want_params=True, g_input=None):
        """Backprop d loss / d image-part logits through the conv stack.
        Accumulates dW (effective weights) into self.dW; optionally writes the image gradient."""
        B, H = f["B"], f["H"]
        Hf = H // 4
        g_a1, _ = self._head_bwd(g_img_part, g_img_part.shape[1], f["h1"], B, Hf, want_params)
        if want_params:
            dW1, gb1 = self.dW["conv_layers.2."], self.G("conv_layers.2.bias")
            self.side.run(lambda: (ops.conv2d_wgrad(g_a1, f["h0"], 256, 4, 4, 2, 1, dW1),
                                   ops.colsum(g_a1.view(-1, 256), gb1, defer=True)), g_a1, f["h0"])
        g_a0 = torch.empty(B, H // 2, H // 2, 128, device=self.dev, dtype=self.cdt)
        ops.dgrad_s2(g_a1, self.W1cls, 128, g_a0, ep=E_(act=MUL_LRELU_GRAD, aux=f["h0"], ld_aux=128))
        if want_params:
            dW0, gb0 = self.dW["conv_layers.0."].view(128, 48), self.G("conv_layers.0.bias")
            self.side.run(lambda: (self._d0_wgrad(f["cols"], g_a0, dW0),
                                   ops.colsum(g_a0.view(-1, 128), gb0, defer=True)), g_a0, f["cols"])
        if g_input is not None:
            self._d0_dgrad(g_a0, g_input)
        return g_a1, g_a0

    def _d0_wgrad(self, cols, g, dW0):
        """dW0 [128, 48] += conv_layers.0 weight gradient; ``cols`` is the im2col matrix, or (image, strides)."""
        if isinstance(cols, tuple):
            img, strides = cols
            B, OH, OW, _ = g.shape
            ops.d0_wgrad(img, strides, B, 2 * OH, 2 * OW, g, dW0)
        else:
            ops.gemm(g.view(-1, 128), cols, 128, 48, g.numel() // 128, a_kc=False, b_kc=False, out=dW0,
                     ep=E_(atomic=1), splits=0)

    def _d0_dgrad(self, g, out):
        if self._d0_ok(2 * g.shape[1]):
            ops.d0_dgrad(g, self.W0p, out)
        else:
            ops.dgrad_s2_small(g, self.W0p, 3, out)

    def _head_bwd(self, g, g_bstride, h1, B, Hf, want_w, wgrad_input=None, need_g=False):
        """g_a1 = lrelu'(a1) * (G @ W2img^T) and (optionally) dW2img += X^T G, G the tap-expanded gradient;
        X = h1 (or ``wgrad_input``, the R1 path's m1 v1)."""
        Pn = B * Hf * Hf
        h1f = h1.view(Pn, 256)
        g_a1 = torch.empty(B, Hf, Hf, 256, device=self.dev, dtype=self.cdt)
        G = None
        if want_w or need_g or not self._head_ok(Hf):
            G = ops.disc_head_gmat(g, g_bstride, B, Hf, self.cdt)
        if self._head_ok(Hf):  # G formed inside the kernel (mg_d_head_bwd)
            ops.d_head_bwd(g, g_bstride, h1, self.W2img_c, B, Hf, g_a1)
        else:
            ops.gemm(G, self.W2img_c, Pn, 256, 16, out=g_a1.view(Pn, 256),
                     ep=E_(act=MUL_LRELU_GRAD, aux=h1f, ld_aux=256))
        if want_w:
            X = h1f if wgrad_input is None else wgrad_input.view(Pn, 256)
            dW2img = self.dW["output_layer.0."].view(384, 16)[:256]
            self.side.run(lambda: ops.gemm(X, G, 256, 16, Pn, a_kc=False, b_kc=False, out=dW2img, ep=E_(atomic=1),
                                           splits=0), X, G)
        return g_a1, G

    def begin_grads(self):
        self.dW = {pre: ops.zeros(*self.W[pre].shape, device=self.dev) for pre in WN_LAYERS}

    def finish_grads(self):
        # reference weight layout: conv_layers.0 packed as [o][tap*3+c] in the GEMM -> remap to [o][c][kh][kw]
        ops.weight_norm_bwd_batch([(self.P(pre + "weight_v"), self.P(pre + "weight_g"), self.norm[pre], self.dW[pre],
                                    self.G(pre + "weight_v"), self.G(pre + "weight_g")) for pre in WN_LAYERS])

    # ------------------------------------------------------------------
    def d_phase(self, real_nchw, text, fake_img, fake_layout, perm, r1_gamma):
        """D loss + R1 and all D parameter gradients (t2i_moe_gan.py:1276-1326).
        real_nchw [B,3,H,H] fp32; fake_img: generator output (NHWC padded [B,R,R,ld]; R = 16 in the reference).
        Returns device scalars [d_loss_gan, sp_real, sp_fake, sp_mism] and r1, plus logits."""
        B = real_nchw.shape[0]
        Hr = real_nchw.shape[-1]
        dev = self.dev
        self.begin_grads()
        t, tb = self.text_branch(text)
        fr = self.forward(real_nchw, "nchw", text, B, Hr)
        ff = self.forward(fake_img, fake_layout, text, B, fake_img.shape[1])
        No = fr["img_part"].shape[1]
        out = torch.zeros(4, device=dev)
        g_img = torch.empty(B, No, device=dev)
        g_fake = torch.empty(B, ff["img_part"].shape[1], device=dev)
        g_tb = ops.zeros(B, device=dev)
        real_pred = torch.empty(B, No, device=dev)
        mism_pred = torch.empty(B, No, device=dev)
        fake_pred = torch.empty(B, ff["img_part"].shape[1], device=dev)
        ops.d_loss(fr["img_part"], ff["img_part"], tb, perm, out, g_img, g_fake, g_tb, real_pred, mism_pred,
                   fake_pred)
        # ordinary first-order backward (real + mismatched share the image features)
        self.stack_backward(fr, g_img)
        self.stack_backward(ff, g_fake)
        # text branch + head bias
        self._text_head_bwd(g_tb, t, text)
        # ---- R1 ----
        Hf = Hr // 4
        Ho = Hf - 3
        g1 = self._ones(Ho * Ho).view(1, -1)
        gA1, G1 = self._head_bwd(g1, 0, fr["h1"], B, Hf, False, need_g=True)  # m1 * Gh1 (G1: dW2's R1 term below)
        gA0 = torch.empty(B, Hr // 2, Hr // 2, 128, device=dev, dtype=self.cdt)
        ops.dgrad_s2(gA1, self.W1cls, 128, gA0, ep=E_(act=MUL_LRELU_GRAD, aux=fr["h0"], ld_aux=128))
        gx = ops.zeros(B, Hr, Hr, 4, device=dev)
        self._d0_dgrad(gA0, gx)  # d sum(real_pred) / d real  (NHWC, channel-padded)
        r1 = torch.zeros(1, device=dev)
        u = torch.empty(B, Hr, Hr, 4, device=dev, dtype=self.cdt)
        ops.r1(gx, B, r1_gamma, r1, u)
        u_strides = (Hr * Hr * 4, Hr * 4, 4, 1)
        if self._d0_ok(Hr):
            cols_u = (u, u_strides)
            m0v0 = ops.d0_fwd(u, u_strides, B, Hr, Hr, self.W0p, aux=fr["h0"])
        else:
            cols_u = ops.im2col_4x4s2(u, u_strides, B, Hr, Hr, 3, 48, self.cdt)
            m0v0 = torch.empty(B, Hr // 2, Hr // 2, 128, device=dev, dtype=self.cdt)
            ops.gemm(cols_u, self.W0p, cols_u.shape[0], 128, 48, out=m0v0.view(-1, 128),
                     ep=E_(act=MUL_LRELU_GRAD, aux=fr["h0"], ld_aux=128))
        m1v1 = ops.conv2d(m0v0, self.W1p, 256, 4, 4, 2, 1, ep=E_(act=MUL_LRELU_GRAD, aux=fr["h1"], ld_aux=256))
        dW0, dW1 = self.dW["conv_layers.0."].view(128, 48), self.dW["conv_layers.2."]
        dW2img = self.dW["output_layer.0."].view(384, 16)[:256]

        def r1_wgrads():
            self._d0_wgrad(cols_u, gA0, dW0)
            ops.conv2d_wgrad(gA1, m0v0, 256, 4, 4, 2, 1, dW1)
            ops.gemm(m1v1.view(-1, 256), G1, 256, 16, B * Hf * Hf, a_kc=False, b_kc=False, out=dW2img,
                     ep=E_(atomic=1), splits=0)
        self.side.run(r1_wgrads, gA0, cols_u, gA1, m0v0, m1v1, G1)
        self.side.join()
        self._remap_w0()
        self.finish_grads()
        if fake_pred.shape[1] == 1:  # [B] as the reference's 16x16 fakes give
            fake_pred = fake_pred.view(-1)
        return dict(losses=out, r1=r1, real_pred=real_pred, mism_pred=mism_pred, fake_pred=fake_pred, r1_grad=gx)

    def _remap_w0(self):
        """dW0 was accumulated in the GEMM layout [o][tap*3 + c]; convert to [o][c][kh][kw].  The remap and
        finish_grads read the accumulated dW: the deferred conv weight-gradient folds land first."""
        ops.fold_flush()
        g = self.dW["conv_layers.0."].view(128, 16, 3)
        self.dW["conv_layers.0."] = g.permute(0, 2, 1).contiguous().view(128, 3, 4, 4)

    # ------------------------------------------------------------------
    def g_phase(self, fake_img, fake_layout, text, scale=1.0, want_d_params=False):
        """Adversarial loss of the generator step (t2i_moe_gan.py:1379-1382) and d loss / d fake image.
        D parameter gradients are formed only when ``want_d_params``: with gradient_accumulation_steps=1 the
        reference zeroes them before they are ever used (t2i_moe_gan.py:1272 vs :1407)."""
        B = fake_img.shape[0]
        Hs = fake_img.shape[1]
        t, tb = self.text_branch(text)
        f = self.forward(fake_img, fake_layout, text, B, Hs)
        No = f["img_part"].shape[1]  # 1 for the reference's 16x16 fakes, (Hs/4-3)^2 for larger ones
        fake_pred = torch.empty(B, No, device=self.dev)
        ops.copy2d(f["img_part"], fake_pred, B, No)
        ops.copy2d(tb.view(B, 1).expand(B, No).contiguous() if No > 1 else tb.view(B, 1), fake_pred, B, No,
                   accumulate=1)
        loss = torch.empty(1, device=self.dev)  # (mg_g_loss writes it)
        g = torch.empty(B, No, device=self.dev)
        ops.g_loss(fake_pred.view(-1), loss, g.view(-1), scale)
        g_img = ops.zeros(*fake_img.shape, device=self.dev, dtype=self.cdt)
        if want_d_params:
            self.begin_grads()
        self.stack_backward(f, g, want_params=want_d_params, g_input=g_img)
        if want_d_params:
            if No > 1:
                g_tb = ops.zeros(B, device=self.dev)
                ops.segsum(g, B, No, 1, g_tb.view(B, 1), ld=1)
            else:
                g_tb = g.view(-1)
            self._text_head_bwd(g_tb, t, text)
            self.side.join()
            self._remap_w0()
            self.finish_grads()
        return loss, (fake_pred.view(-1) if No == 1 else fake_pred), g_img

    def _text_head_bwd(self, g_tb, t, text):
        B = t.shape[0]
        g_tpre = torch.empty(B, 128, device=self.dev)
        ops.d_text_bwd(g_tb, t, self.w2sum, 256, g_tpre, self.dW["output_layer.0."].view(384, 16))
        ops.colsum(g_tb.view(B, 1), self.G("output_layer.0.bias"), defer=True)
        ops.linear_wgrad(g_tpre, text, self.dW["text_projection.0."])
        ops.colsum(g_tpre, self.G("text_projection.0.bias"), defer=True)

    # ------------------------------------------------------------------
    # generic forward / backward for the module API (AuroraDiscriminator.forward)
    # ------------------------------------------------------------------
    def logits(self, img_nchw, text):
        """D(img, text) for any power-of-two H >= 16 (NCHW fp32 image) -> ([B, Ho*Ho] logits, ctx)."""
        B, _, H, _ = img_nchw.shape
        t, tb = self.text_branch(text)
        f = self.forward(img_nchw.contiguous(), "nchw", text, B, H)
        out = f["img_part"].clone()
        ops.copy2d(tb.view(B, 1).expand(B, out.shape[1]).contiguous(), out, B, out.shape[1], accumulate=1)
        return out, dict(f=f, t=t, text=text)

    def logits_backward(self, ctx, g_logits, want_input=True):
        """d loss / d logits -> D parameter gradients (accumulated) and d loss / d image (NCHW fp32)."""
        f = ctx["f"]
        B, H = f["B"], f["H"]
        g_logits = g_logits.contiguous().float()
        g_tb = ops.zeros(B, device=self.dev)
        ops.segsum(g_logits, B, g_logits.shape[1], 1, g_tb.view(B, 1), ld=1)
        self.begin_grads()
        # the image gradient is consumed inside the step (the generator backward): from the per-step zero arena
        g_img = ops.zeros(B, H, H, 4, device=self.dev) if want_input else None
        self.stack_backward(f, g_logits, want_params=True, g_input=g_img)
        self._text_head_bwd(g_tb, ctx["t"], ctx["text"])
        self.side.join()
        self._remap_w0()
        self.finish_grads()
        return None if g_img is None else g_img[..., :3].permute(0, 3, 1, 2).contiguous()
