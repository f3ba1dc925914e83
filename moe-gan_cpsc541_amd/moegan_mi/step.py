"""One G+D training step of train_aurora_gan (t2i_moe_gan.py:1262-1421) on the HIP engines.

The step keeps the reference's order and semantics:
  D phase: D(real) + R1, G forward under no_grad (fresh router noise), D(fake), D(real, text[perm]),
           D backward, clip_grad_norm_(D, 0.7), AdamW(D)
  G phase: G forward (fresh router noise), KL clamp at 50, D(fake) with the UPDATED D, G adversarial
           loss + CLIP terms (no gradient, :98-101) + balance loss (last layer) + annealed KL,
           G backward, clip_grad_norm_(G, 0.8), AdamW(G)
Parameters with no gradient in the reference (to_rgb_8: only feeds the gradient-free CLIP loss; with the
progressive extension every to_rgb but the final one)
sit in the store's frozen tail and are never updated -- exactly as torch's AdamW skips a
parameter whose .grad is None.

Loss guards (t2i_moe_gan.py:1315-1320, :1367-1376, :1396-1404) run on the device: a flag word per step
(``out["flags"]``) records a non-finite discriminator loss (the whole batch is skipped: no gradient is
kept, no optimizer steps, no step counters advance) or a non-finite generator loss (replaced by 0: only
the routers' KL term keeps a gradient).  A second word per accumulation window records which parameter
groups received a gradient, so the gated optimizer launches skip a group whose gradient the reference
would leave as None.  Everything stays one captured hipGraph; the host reads the flags at most once per
step.

Gradient accumulation (gradient_accumulation_steps > 1): each batch's gradients are formed in
``store.grad`` and added to the window accumulator ``store.acc`` only if the guards keep the batch.

Nothing here synchronises with the host: every loss value stays on the device until the caller reads it,
and all randomness is passed in.  Data parallelism (one process per GPU, RCCL) all-reduces the flat D and
G gradient buffers, the [E] expert-load vector and the guard word.
"""
import os

import torch
import torch.nn.functional as F

from . import graphs, ops
from .engine_d import DiscriminatorEngine
from .engine_g import GeneratorEngine
from .layout import discriminator_shapes, frozen_rgb_prefixes, generator_shapes
from .params import ParamStore

FD, FG = ops.FLAG_D_BAD, ops.FLAG_G_BAD


class StepConfig:
    def __init__(self, E=4, topk=None, dtype="fp32", r1_gamma=10.0, clip_weight_16=0.1, clip_weight_8=0.05,
                 balance_weight=0.01, beta1=0.5, beta2=0.999, weight_decay=0.01, eps=1e-8, d_clip=0.7, g_clip=0.8,
                 psi=0.7, fp8=False, max_res=16, deterministic=None):
        self.E, self.topk = E, topk
        # generator output resolution: 16 = the reference; 32 / 64 / 128 = the progressive extension (layout.py)
        self.max_res = max_res
        self.dtype = dtype
        self.fp8 = fp8  # MX-fp8 3x3 modulated convs (BASELINE config C5), inside the bf16 mode
        self.r1_gamma = r1_gamma
        self.clip_weight_16, self.clip_weight_8 = clip_weight_16, clip_weight_8
        self.balance_weight = balance_weight
        self.beta1, self.beta2, self.weight_decay, self.eps = beta1, beta2, weight_decay, eps
        self.d_clip, self.g_clip = d_clip, g_clip
        self.psi = psi
        # deterministic mode (ops.set_deterministic): None = the MOEGAN_DETERMINISTIC environment switch
        self.deterministic = (os.environ.get("MOEGAN_DETERMINISTIC", "0") == "1") if deterministic is None \
            else bool(deterministic)


def clip_loss(images_nchw, text, encode_image, images_nhwc=None):
    """CLIPLoss.forward (t2i_moe_gan.py:75-119): 1 - mean cos(CLIP(image), text), forward only (no gradient,
    :98-101).  Logging / validation only; values are parity-unpinned (CLIP weights are not available here).
    With the build's image tower (``encode_image`` a bound ``ClipImageEncoder`` method) and the generator's NHWC
    image, clamp + resize + patchify run as one kernel (``encode_generated``); any other encoder gets the NCHW
    clamp / F.interpolate input of the reference."""
    with torch.no_grad():
        tower = getattr(encode_image, "__self__", None)
        if images_nhwc is not None and hasattr(tower, "encode_generated"):
            f = tower.encode_generated(images_nhwc).float()
        else:
            im = torch.clamp(images_nchw.float(), -1, 1)
            if im.shape[-1] != 224 or im.shape[-2] != 224:
                im = F.interpolate(im, size=(224, 224), mode="bilinear", align_corners=False)
            f = encode_image(im).float()
        f = f / f.norm(dim=-1, keepdim=True)
        t = text.float() / text.float().norm(dim=-1, keepdim=True)
        sim = torch.nan_to_num((f * t).sum(dim=1))
        return (1.0 - sim.mean()).reshape(1)


class TrainStep:
    def __init__(self, cfg, device="cuda", process_group=None, gstore=None, dstore=None):
        self.cfg = cfg
        self.dev = torch.device(device)
        if getattr(cfg, "deterministic", False):
            ops.set_deterministic(True)
        self.cdt = torch.bfloat16 if cfg.dtype == "bf16" else torch.float32
        self.gs = gstore if gstore is not None else ParamStore(
            generator_shapes(cfg.E, getattr(cfg, "max_res", 16)), self.dev,
            frozen_prefixes=frozen_rgb_prefixes(getattr(cfg, "max_res", 16)), shadow_dtype=self.cdt)
        self.ds = dstore if dstore is not None else ParamStore(discriminator_shapes(), self.dev)
        self.ge = GeneratorEngine(self.gs, cfg.E, cfg.topk, self.cdt, fp8=getattr(cfg, "fp8", False))
        self.de = DiscriminatorEngine(self.ds, self.cdt)
        self.pg = process_group
        self.world = 1
        if process_group is not None:
            import torch.distributed as dist
            self.world = dist.get_world_size(process_group)
        # optional image encoder for the (gradient-free) CLIP loss terms; images are [B,3,H,W] in [-1, 1]
        self.clip_encoder = None
        self.win = torch.zeros(1, device=self.dev, dtype=torch.int32)  # accumulation-window word (mg_flag_window)

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

    def _bucketed_grad_allreduce(self, store, begin):
        """Overlapped data-parallel mean of a flat gradient: ``begin()`` arms the engine so
        every range it reports final during the backward (a block's expert parameters, ~56 % of the generator
        at E=8) starts an asynchronous RCCL all-reduce at once, overlapping the rest of the backward; the
        returned ``finish()`` all-reduces the complement of those ranges in [0, n_opt), waits for every
        bucket and scales by 1 / world.  The reductions are sums of the same per-rank gradients as the single
        collective, just split into disjoint ranges."""
        import torch.distributed as dist
        pending, done = [], []

        def on_final(lo, hi):
            t = store.grad[lo:hi]
            done.append((lo, hi))
            graphs.eager(lambda: pending.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg,
                                                                async_op=True)))
        begin(on_final)

        def finish():
            n = store.n_opt
            rest, cur = [], 0
            for lo, hi in sorted(done):
                if lo > cur:
                    rest.append((cur, lo))
                cur = max(cur, hi)
            if cur < n:
                rest.append((cur, n))
            views = [store.grad[lo:hi] for lo, hi in rest]

            def run():
                for t in views:
                    pending.append(dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.pg, async_op=True))
                for w in pending:
                    w.wait()
                pending.clear()
                store.grad[:n].mul_(1.0 / self.world)
            graphs.eager(run)
        return finish

    def _allreduce_flags(self, flags):
        """Every rank takes the same guard decision: a bit set on any rank is set on all (MAX per bit)."""
        if self.pg is None:
            return
        import torch.distributed as dist

        def run():
            bits = torch.stack([(flags & FD), (flags & FG)]).view(-1)
            dist.all_reduce(bits, op=dist.ReduceOp.MAX, group=self.pg)
            flags.copy_(bits[0:1] | bits[1:2])
        graphs.eager(run)

    def _guard(self, flags, checks, windows):
        """A phase's loss guards: the finite checks, the data-parallel agreement on the flag word, the window
        updates -- one launch (ops.guard_update) without a process group, check / all-reduce / windows with one."""
        if self.pg is None:
            ops.guard_update(flags, self.win, checks, windows)
            return
        ops.guard_update(flags, None, checks, ())
        self._allreduce_flags(flags)
        ops.guard_update(flags, self.win, (), windows)

    # ---- optimizer ----
    def _adamw(self, store, grad, lr, max_norm, flags, ranges, grad_scale=1.0):
        """clip_grad_norm_ + AdamW over ``grad[:n_opt]`` (torch semantics, :1333-1337 / :1417-1421).  ``ranges``:
        [(lo, hi, step counter, window bit)] -- each range is one gated launch with its own step counter."""
        n = store.n_opt
        if grad_scale != 1.0:  # (loss / accumulation_steps) of the reference == scaling the summed gradient
            grad[:n].mul_(grad_scale)
        ss = torch.empty(1, device=self.dev)
        live = [(lo, hi, step_dev, wbit) for lo, hi, step_dev, wbit in ranges if hi > lo]
        # the norm and every range's device step counter (+1, graph-replayable, gated) in two launches
        ops.grad_norm_steps(grad[:n], ss, [(step_dev, wbit) for _, _, step_dev, wbit in live], flags=flags,
                            skip_mask=FD, win=self.win)
        c = self.cfg
        bf16_shadow = store.shadow is not None and store.shadow.dtype == torch.bfloat16
        for lo, hi, step_dev, wbit in live:
            gate = (flags, FD, self.win, wbit)
            ops.adamw_dev(store.data[lo:hi], grad[lo:hi], store.m[lo:hi], store.v[lo:hi], lr, c.beta1, c.beta2,
                          c.eps, c.weight_decay, step_dev, ss, max_norm,
                          shadow=store.shadow[lo:hi] if bf16_shadow else None, gate=gate)
        if bf16_shadow:
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
        ops.ARENA.begin(self.dev)
        ops.COLSUMS.active = True  # bias-gradient column sums batched per backward (flushed below)
        # the library's gradient folds too: one batched launch per backward (ops.fold_flush); MOEGAN_FOLD_DEFER=0
        # folds each at its producer (same kernels, bit-identical gradients)
        ops.fold_defer(os.environ.get("MOEGAN_FOLD_DEFER", "1") == "1")
        # bf16 mode: the fp32-operand GEMMs (prefix, demodulation, router / cross-attention vectors) as split-bf16
        # products (ops.set_f32x3); the fp32 parity mode keeps exact-fp32 MFMA
        x3_prev = ops.set_f32x3(self.cdt == torch.bfloat16 and os.environ.get("MOEGAN_F32X3", "1") == "1")
        try:
            return self._step(real, text, z, eps_d, eps_g, perm, anneal, lr_g, lr_d, eff_kl_weight, prep, acc,
                              zero_grads, step_optim)
        finally:
            ops.fold_defer(False)
            ops.set_f32x3(x3_prev)
            ops.ARENA.end()
            ops.COLSUMS.active = False
            ops.COLSUMS.items = []
            self.ge.guard_flags = None

    def _step(self, real, text, z, eps_d, eps_g, perm, anneal, lr_g, lr_d, eff_kl_weight, prep, acc, zero_grads,
              step_optim):
        c = self.cfg
        accum = acc > 1
        gs, ds = self.gs, self.ds
        flags = ops.zeros(1, device=self.dev, dtype=torch.int32)  # the step's guard word (zero arena)
        self.ge.guard_flags = flags
        if prep:
            self.ge.prep()
            self.de.prep()
        if accum:
            gs.ensure_acc()
            ds.ensure_acc()
            if zero_grads:
                ds.acc.zero_()
        # ------------------------- D phase -------------------------
        if zero_grads or accum:
            ds.zero_grad()
        # the router-independent prefix of this forward (mapping, styles, gen_block_4's convolution block) is
        # kept with its saved activations and reused by the G-phase forward: same z / text, G not yet updated
        f16, _, _, probs_d, topi_d, _ = self.ge.forward(z, text, eps_d, anneal, c.psi, train=True, save=False,
                                                        want_kl=False, keep_prefix=True)
        prefix, self.ge.last_prefix = self.ge.last_prefix, None
        dres = self.de.d_phase(real, text, f16, ("nhwc", 8), perm, c.r1_gamma)
        ops.fold_flush()
        ops.COLSUMS.flush()
        # guard: NaN / Inf d_loss skips the whole batch (t2i_moe_gan.py:1315-1320)
        self._guard(flags, [(dres["losses"][:1], FD), (dres["r1"], FD)],
                    [dict(reset_bits=ops.WIN_D if zero_grads else 0, bad_mask=FD, set_bits=ops.WIN_D)])
        if accum:
            ops.gated_axpy(ds.acc, ds.grad, flags, FD)
        dgrad = ds.acc if accum else ds.grad
        d_sumsq = None
        if step_optim:
            self._allreduce_mean(dgrad)
            d_sumsq = self._adamw(ds, dgrad, lr_d, c.d_clip, flags, [(0, ds.n_opt, ds.step_dev, ops.WIN_D)],
                                  grad_scale=1.0 / acc)
            self.de.prep()
        # ------------------------- G phase -------------------------
        if accum:
            gs.zero_grad()
            if zero_grads:  # optimizer_g.zero_grad() (:1353) is never reached by a skipped batch
                ops.zero_if(gs.acc, flags, FD, when_set=False)
        elif zero_grads:
            gs.zero_grad()
        want8 = self.clip_encoder is not None
        img16, img8, kl2s, probs, topi_g, ctx = self.ge.forward(z, text, eps_g, anneal, c.psi, train=True,
                                                                save=True, want_img8=want8, prefix=prefix)
        prefix = None
        leak = accum and not step_optim  # the G loss also reaches D's gradients while D has not stepped yet
        if leak:
            ds.zero_grad()
        g_gan, fake_pred, g_img = self.de.g_phase(img16, ("nhwc", 8), text, want_d_params=leak)
        ops.fold_flush()
        ops.COLSUMS.flush()
        # balance loss on the last MoE layer, over the GLOBAL batch (t2i_moe_gan.py:951-1000)
        last = probs[-1]
        load = ops.zeros(c.E, device=self.dev)
        ops.colsum(last, load)
        self._allreduce_sum(load)
        bal = torch.empty(1, device=self.dev)  # (mg_balance writes it)
        coef = torch.empty(c.E, device=self.dev)
        ops.balance(load, c.E, last.shape[0] * self.world, c.balance_weight, float(self.world), bal, coef)
        # CLIP terms (t2i_moe_gan.py:1385-1387): forward only, they enter g_loss's value but no gradient
        clip16 = clip8 = None
        if self.clip_encoder is not None:
            clip16 = clip_loss(img16[..., :3].permute(0, 3, 1, 2), text, self.clip_encoder, images_nhwc=img16)
            clip8 = clip_loss(img8[..., :3].permute(0, 3, 1, 2), text, self.clip_encoder, images_nhwc=img8)
        # KL (t2i_moe_gan.py:846, :1367-1376, :1402-1404)
        kb = self.ge.last_klbuf  # the forward's [blocks, 2] KL buffer, whose rows kl2s are
        kl2 = kb if kb is not None and kb.shape[0] == len(kl2s) else torch.stack(kl2s)
        kl_coef = torch.empty(len(kl2s), device=self.dev)
        kl_total = torch.empty(1, device=self.dev)
        ops.kl_coefs(kl2, len(kl2s), eff_kl_weight, kl_coef, kl_total)
        # guard: NaN / Inf (GAN + CLIP + balance) generator loss -> 0, the KL term stays (:1396-1404)
        self._guard(flags, [(t, FG) for t in (g_gan, bal, clip16, clip8) if t is not None],
                    [dict(reset_bits=(ops.WIN_G_MAIN | ops.WIN_G_KL) if zero_grads else 0, keep_mask=FD, bad_mask=FD,
                          set_bits=ops.WIN_G_KL),
                     dict(bad_mask=FD | FG, set_bits=ops.WIN_G_MAIN)])
        # data parallel, one optimizer step per batch: the generator gradient is all-reduced in buckets that
        # start while the backward still runs (expert ranges first); otherwise one collective after it
        g_finish = None
        if self.pg is not None and step_optim and not accum:
            g_finish = self._bucketed_grad_allreduce(gs, lambda cb: setattr(self.ge, "on_grad_final", cb))
        try:
            self.ge.backward(ctx, g_img, coef=coef, kl_coef=kl_coef)
        finally:
            self.ge.on_grad_final = None
        ops.fold_flush()
        ops.COLSUMS.flush()
        if g_finish is not None:  # every bucket reduced and scaled before the guard below rewrites ranges
            g_finish()
        if accum:
            ops.gated_axpy(gs.acc[:gs.n_main], gs.grad[:gs.n_main], flags, FD | FG)
            ops.gated_axpy(gs.acc[gs.n_main:gs.n_opt], gs.grad[gs.n_main:gs.n_opt], flags, FD)
            if leak:
                ops.gated_axpy(ds.acc, ds.grad, flags, FD | FG)
        else:
            ops.zero_if(gs.grad[:gs.n_main], flags, FG)  # the router KL range kept only its KL term
        ggrad = gs.acc if accum else gs.grad
        g_sumsq = None
        if step_optim:
            if g_finish is None:
                self._allreduce_mean(ggrad)
            g_sumsq = self._adamw(gs, ggrad, lr_g, c.g_clip, flags,
                                  [(0, gs.n_main, gs.step_dev, ops.WIN_G_MAIN),
                                   (gs.n_main, gs.n_opt, gs.step_dev_kl, ops.WIN_G_KL)],
                                  grad_scale=1.0 / acc)
        out = dict(d_losses=dres["losses"], r1=dres["r1"], g_gan=g_gan, balance=bal, kl=kl_total, kl_raw=kl2,
                   d_grad_sumsq=d_sumsq, g_grad_sumsq=g_sumsq, real_pred=dres["real_pred"],
                   fake_pred=dres["fake_pred"], mism_pred=dres["mism_pred"], r1_grad=dres["r1_grad"],
                   img16=img16, img8=img8, probs=probs, topi=topi_g, probs_d=probs_d, topi_d=topi_d,
                   fake_img_d=f16, flags=flags, clip16=clip16, clip8=clip8, d_grad=dgrad, g_grad=ggrad)
        return out
