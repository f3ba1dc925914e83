"""One G+D training step of train_aurora_gan (t2i_moe_gan.py:1262-1421) on the HIP engines.

The step keeps the reference's order and semantics with gradient_accumulation_steps=1:
  D phase: D(real) + R1, G forward under no_grad (fresh router noise), D(fake), D(real, text[perm]),
           D backward, clip_grad_norm_(D, 0.7), AdamW(D)
  G phase: G forward (fresh router noise), KL clamp at 50, D(fake) with the UPDATED D, G adversarial
           loss + CLIP terms (no gradient, :98-101) + balance loss (last layer) + annealed KL,
           G backward, clip_grad_norm_(G, 0.8), AdamW(G)
Parameters with no gradient in the reference (to_rgb_8: only feeds the gradient-free CLIP loss)
sit in the store's frozen tail and are never updated -- exactly as torch's AdamW skips a
parameter whose .grad is None.

Nothing here synchronises with the host: every loss value stays on the device until the
caller reads it, and all randomness is passed in.  Data parallelism (one process per GPU,
RCCL) all-reduces the flat D and G gradient buffers and the [E] expert-load vector.
"""
import torch

from . import graphs, ops
from .engine_d import DiscriminatorEngine
from .engine_g import GeneratorEngine
from .layout import discriminator_shapes, generator_shapes
from .params import ParamStore


class StepConfig:
    def __init__(self, E=4, topk=None, dtype="fp32", r1_gamma=10.0, clip_weight_16=0.1, clip_weight_8=0.05,
                 balance_weight=0.01, beta1=0.5, beta2=0.999, weight_decay=0.01, eps=1e-8, d_clip=0.7, g_clip=0.8,
                 psi=0.7):
        self.E, self.topk = E, topk
        self.dtype = dtype
        self.r1_gamma = r1_gamma
        self.clip_weight_16, self.clip_weight_8 = clip_weight_16, clip_weight_8
        self.balance_weight = balance_weight
        self.beta1, self.beta2, self.weight_decay, self.eps = beta1, beta2, weight_decay, eps
        self.d_clip, self.g_clip = d_clip, g_clip
        self.psi = psi


class TrainStep:
    def __init__(self, cfg, device="cuda", process_group=None, gstore=None, dstore=None):
        self.cfg = cfg
        self.dev = torch.device(device)
        self.cdt = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
        self.gs = gstore if gstore is not None else ParamStore(
            generator_shapes(cfg.E), self.dev, frozen_prefixes=("to_rgb_8.",), shadow_dtype=self.cdt)
        self.ds = dstore if dstore is not None else ParamStore(discriminator_shapes(), self.dev)
        self.ge = GeneratorEngine(self.gs, cfg.E, cfg.topk, self.cdt)
        self.de = DiscriminatorEngine(self.ds, self.cdt)
        self.pg = process_group
        self.world = 1
        if process_group is not None:
            import torch.distributed as dist
            self.world = dist.get_world_size(process_group)
        self.clip_encoder = None  # optional image encoder for the (gradient-free) CLIP loss

    # ---- data-parallel reductions ----
    # (collectives stay eager segments when the step is replayed as hipGraphs, graphs.py)
    def _allreduce_mean(self, t):
        if self.pg is None:
            return
        import torch.distributed as dist

        def run():
            dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg)
            t.mul_(1.0 / self.world)
        graphs.eager(run)

    def _allreduce_sum(self, t):
        if self.pg is None:
            return
        import torch.distributed as dist
        graphs.eager(lambda: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg))

    # ---- optimizer ----
    def _adamw(self, store, lr, max_norm, n=None, grad_scale=1.0):
        n = store.n_opt if n is None else n
        store.step_count += 1
        if grad_scale != 1.0:  # (loss / accumulation_steps) of the reference == scaling the summed gradient
            store.grad[:n].mul_(grad_scale)
        ss = torch.empty(1, device=self.dev)
        ops.opt_prologue(ss, store.step_dev)  # ss = 0, device step counter += 1 (graph-replayable)
        ops.sumsq(store.grad[:n], ss)
        c = self.cfg
        shadow = store.shadow[:n] if (store.shadow is not None and store.shadow.dtype == torch.bfloat16) else None
        ops.adamw_dev(store.data[:n], store.grad[:n], store.m[:n], store.v[:n], lr, c.beta1, c.beta2, c.eps,
                      c.weight_decay, store.step_dev, ss, max_norm, shadow=shadow)
        if shadow is not None:
            store.mark_shadow_written()
        return ss

    # ---- the step ----
    def step(self, real, text, z, eps_d, eps_g, perm, *, anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8,
             prep=True, acc=1, zero_grads=True, step_optim=True):
        """real [B,3,64,64] fp32 NCHW, text [B,512], z [B,512] fp32 (device); eps_d / eps_g: 3 triples of
        router epsilon tensors; perm [B] int32.  Returns a dict of device tensors.

        Gradient accumulation (t2i_moe_gan.py:1272, :1329, :1353, :1413): ``zero_grads`` at the first batch of
        a window, ``step_optim`` at its last; gradients are summed and scaled by 1/acc before clipping.  As in
        the reference, the generator step's loss also accumulates into the discriminator's gradients, which
        matters only when the D optimizer has not stepped yet in the window (acc > 1)."""
        c = self.cfg
        B = real.shape[0]
        ops.ARENA.begin(self.dev)
        try:
            return self._step(real, text, z, eps_d, eps_g, perm, anneal, lr_g, lr_d, eff_kl_weight, prep, acc,
                              zero_grads, step_optim)
        finally:
            ops.ARENA.end()

    def _step(self, real, text, z, eps_d, eps_g, perm, anneal, lr_g, lr_d, eff_kl_weight, prep, acc, zero_grads,
              step_optim):
        c = self.cfg
        B = real.shape[0]
        if prep:
            self.ge.prep()
            self.de.prep()
        # ------------------------- D phase -------------------------
        if zero_grads:
            self.ds.zero_grad()
        # the router-independent prefix of this forward (mapping, styles, gen_block_4's convolution block) is
        # kept with its saved activations and reused by the G-phase forward: same z / text, G not yet updated
        f16, _, _, _, _, _ = self.ge.forward(z, text, eps_d, anneal, c.psi, train=True, save=False, want_kl=False,
                                             keep_prefix=True)
        prefix, self.ge.last_prefix = self.ge.last_prefix, None
        dres = self.de.d_phase(real, text, f16, ("nhwc", 8), perm, c.r1_gamma)
        d_sumsq = None
        if step_optim:
            self._allreduce_mean(self.ds.grad)
            d_sumsq = self._adamw(self.ds, lr_d, c.d_clip, grad_scale=1.0 / acc)
            self.de.prep()
        # ------------------------- G phase -------------------------
        if zero_grads:
            self.gs.zero_grad()
        want8 = self.clip_encoder is not None
        img16, img8, kl2s, probs, _, ctx = self.ge.forward(z, text, eps_g, anneal, c.psi, train=True, save=True,
                                                           want_img8=want8, prefix=prefix)
        prefix = None
        g_gan, fake_pred, g_img = self.de.g_phase(img16, ("nhwc", 8), text, want_d_params=(acc > 1 and not step_optim))
        # balance loss on the last MoE layer, over the GLOBAL batch (t2i_moe_gan.py:951-1000)
        last = probs[-1]
        load = ops.zeros(c.E, device=self.dev)
        ops.colsum(last, load)
        self._allreduce_sum(load)
        bal = torch.zeros(1, device=self.dev)
        coef = torch.empty(c.E, device=self.dev)
        ops.balance(load, c.E, last.shape[0] * self.world, c.balance_weight, float(self.world), bal, coef)
        # KL (t2i_moe_gan.py:846, :1367-1376, :1402-1404)
        kl2 = torch.stack(kl2s)
        kl_coef = torch.empty(len(kl2s), device=self.dev)
        kl_total = torch.empty(1, device=self.dev)
        ops.kl_coefs(kl2, len(kl2s), eff_kl_weight, kl_coef, kl_total)
        self.ge.backward(ctx, g_img, coef=coef, kl_coef=kl_coef)
        g_sumsq = None
        if step_optim:
            self._allreduce_mean(self.gs.grad)
            g_sumsq = self._adamw(self.gs, lr_g, c.g_clip, grad_scale=1.0 / acc)
        out = dict(d_losses=dres["losses"], r1=dres["r1"], g_gan=g_gan, balance=bal, kl=kl_total, kl_raw=kl2,
                   d_grad_sumsq=d_sumsq, g_grad_sumsq=g_sumsq, real_pred=dres["real_pred"],
                   fake_pred=dres["fake_pred"], mism_pred=dres["mism_pred"], r1_grad=dres["r1_grad"],
                   img16=img16, img8=img8)
        return out
