"""Flat, HBM-resident parameter storage in the reference state_dict naming.

Each model's parameters live in ONE fp32 buffer (plus one fp32 gradient
buffer and the two AdamW moment buffers), so the optimizer, gradient norm,
bf16 shadow cast and the data-parallel gradient all-reduce are each a single
launch / collective over a contiguous range.  Views expose every tensor under
its reference key and shape (t2i_moe_gan.py state_dict), which keeps
checkpoints drop-in (sagemaker_train.py:297-301, inference.py:34-49).

The flat ORDER is chosen for the kernels, not the reference: the E experts of
an attention block are stored back to back ([E, 4C, C] / [E, C, 4C]) so the
grouped expert GEMMs read them in place, and parameters the reference never
updates are placed in a frozen tail outside the optimizer range.
"""
import re
from collections import OrderedDict

import torch

from . import ops
from .layout import is_buffer

_EXPERT = re.compile(r"^(.*\.moe\.)experts\.(\d+)\.net\.(\d)\.(weight|bias)$")
# the routers' KL parameters (BayesianRouter mu / rho, t2i_moe_gan.py:280-300, :405-423)
_KL = re.compile(r"^.*\.router\.(feature|text|combined)_(mu|rho)$")
ALIGN = 8  # elements: keeps every view 16-byte aligned for fp32 and bf16 vector loads


def flat_order(shapes, frozen_prefixes=()):
    """Reference names reordered: the modulated convs' style weights and then their biases first (one
    [sum Cin, 512] matrix and one [sum Cin] vector: every style of a forward is ONE GEMM), experts grouped
    per (block, layer, kind), the routers' KL parameters (mu / rho) at the end of the optimised range, frozen
    names last.  The KL group is the only part of the generator that still receives a gradient when the
    loop's guard replaces a non-finite generator loss by 0 (t2i_moe_gan.py:1396-1404), so it is stepped by
    its own (gated) optimizer launch with its own step counter."""
    names = [n for n in shapes if not is_buffer(n)]
    groups = OrderedDict()
    order, frozen = [], []
    is_frozen = lambda n: any(n.startswith(p) for p in frozen_prefixes)  # noqa: E731
    style_w = [n for n in names if n.endswith("modulation.weight") and not is_frozen(n)]
    style_b = [n[:-len("weight")] + "bias" for n in style_w]
    if not all(b in shapes for b in style_b):
        style_w, style_b = [], []
    lead = set(style_w) | set(style_b)
    order.extend(style_w + style_b)
    kl_tail = []
    for n in names:
        m = _EXPERT.match(n)
        if n in lead:
            continue
        if is_frozen(n):
            frozen.append(n)
        elif _KL.match(n):
            kl_tail.append(n)
        elif m:
            key = (m.group(1), m.group(3), m.group(4))
            if key not in groups:
                groups[key] = []
                order.append(key)
            groups[key].append((int(m.group(2)), n))
        else:
            order.append(n)
    out = []
    for o in order:
        if isinstance(o, tuple):
            out.extend(n for _, n in sorted(groups[o]))
        else:
            out.append(o)
    return out + kl_tail, frozen


class ParamStore:
    def __init__(self, shapes, device, frozen_prefixes=(), shadow_dtype=None):
        self.shapes = OrderedDict((k, tuple(v)) for k, v in shapes.items())
        self.device = torch.device(device)
        order, frozen = flat_order(self.shapes, frozen_prefixes)
        self.offsets = OrderedDict()
        off = 0
        for n in order + frozen:
            numel = 1
            for s in self.shapes[n]:
                numel *= s
            if n in frozen and not any(k in frozen for k in self.offsets):
                self.n_opt = off
            self.offsets[n] = (off, numel)
            off += numel
            if not _EXPERT.match(n):
                off = (off + ALIGN - 1) // ALIGN * ALIGN
            else:
                off = off  # experts stay packed (each expert tensor is a multiple of 8 elements)
        if not frozen:
            self.n_opt = off
        # [0, n_main): parameters stepped by the main optimizer launch; [n_main, n_opt): router KL parameters
        kl = [n for n in order if _KL.match(n)]
        self.n_main = self.offsets[kl[0]][0] if kl else self.n_opt
        self.total = (off + ALIGN - 1) // ALIGN * ALIGN
        self.data = torch.zeros(self.total, device=self.device, dtype=torch.float32)
        self.grad = torch.zeros(self.total, device=self.device, dtype=torch.float32)
        self.m = torch.zeros(self.total, device=self.device, dtype=torch.float32)
        self.v = torch.zeros(self.total, device=self.device, dtype=torch.float32)
        self.step_dev = torch.zeros(1, device=self.device, dtype=torch.int32)
        self.step_dev_kl = torch.zeros(1, device=self.device, dtype=torch.int32)  # AdamW step of [n_main, n_opt)
        self.acc = None  # gradient accumulated over a window (gradient_accumulation_steps > 1), ensure_acc()
        self.buffers = OrderedDict((n, torch.zeros(s, device=self.device)) for n, s in self.shapes.items()
                                   if is_buffer(n))
        self.shadow_dtype = shadow_dtype
        self.shadow = None
        if shadow_dtype is not None and shadow_dtype != torch.float32:
            self.shadow = torch.zeros(self.total, device=self.device, dtype=shadow_dtype)

    @property
    def step_count(self):
        """Optimizer steps taken (AdamW's step of the main range): the device counter, which the gated update
        advances inside the step -- so eager steps, hipGraph replays and guard-skipped batches all count right
        (a host mirror would also count captures, which execute nothing).  Reading it synchronises."""
        return int(self.step_dev[0])

    def style_block(self):
        """(weight matrix view [sum Cin, 512], bias view [sum Cin], {prefix: column offset}) of the contiguous
        style group, or None when this store has no modulated convs."""
        ws = [n for n in self.offsets if n.endswith("modulation.weight")]
        ws = [n for n in ws if self.offsets[n][0] < self.n_opt]
        if not ws:
            return None
        o0 = self.offsets[ws[0]][0]
        K = self.shapes[ws[0]][1]
        cols, off = {}, 0
        for n in ws:
            o, numel = self.offsets[n]
            if o != o0 + off * K:
                return None
            cols[n[:-len("modulation.weight")]] = off
            off += self.shapes[n][0]
        b0 = self.offsets[ws[0][:-len("weight")] + "bias"][0]
        for n in ws:
            if self.offsets[n[:-len("weight")] + "bias"][0] != b0 + cols[n[:-len("modulation.weight")]]:
                return None
        return (o0, off, K, b0), cols

    def rebind(self, data):
        """Adopt ``data`` (the flat fp32 buffer, possibly on a new device) and move the rest with it."""
        dev = data.device
        self.data = data
        if self.grad.device != dev:
            self.grad = self.grad.to(dev)
            self.m = self.m.to(dev)
            self.v = self.v.to(dev)
            self.step_dev = self.step_dev.to(dev)
            self.step_dev_kl = self.step_dev_kl.to(dev)
            if self.acc is not None:
                self.acc = self.acc.to(dev)
            self.buffers = OrderedDict((n, b.to(dev)) for n, b in self.buffers.items())
            if self.shadow is not None:
                self.shadow = torch.zeros(self.total, device=dev, dtype=self.shadow_dtype)
        self.device = dev
        self.refresh_shadow(force=True)

    # ---- views ----
    def _v(self, buf, name):
        off, n = self.offsets[name]
        return buf[off:off + n].view(self.shapes[name])

    def view(self, name):
        return self._v(self.data, name)

    def gview(self, name):
        return self._v(self.grad, name)

    def cview(self, name):
        """Compute-dtype view (bf16 shadow if enabled, else the fp32 master)."""
        return self._v(self.shadow if self.shadow is not None else self.data, name)

    def group_view(self, first, last, buf=None):
        """Contiguous range from the start of ``first`` to the end of ``last`` (expert groups)."""
        buf = self.data if buf is None else buf
        a, _ = self.offsets[first]
        b, n = self.offsets[last]
        return buf[a:b + n]

    # ---- per-step ----
    def refresh_shadow(self, force=False):
        if self.shadow is not None and self.data.is_cuda:
            fresh = getattr(self, "_shadow_version", None) == self.data._version
            self._shadow_version = None
            if fresh and not force:  # the optimizer wrote the shadow with the parameters (mg_adamw_dev_shadow)
                return
            ops.cast(self.data, out=self.shadow)

    def mark_shadow_written(self):
        """Called after an optimizer step that also wrote the bf16 shadow of every optimised parameter.  Any
        torch-level write to the fp32 buffer afterwards (load_state_dict, copy_) bumps its version counter and
        makes the next refresh_shadow() cast again."""
        self._shadow_version = self.data._version

    def zero_grad(self):
        # the library's 16-B-store fill: torch's fill kernel ran the generator's 38.8 MB at ~1.9 TB/s (21 us per step)
        ops.zero_if(self.grad, None, 0, when_set=False) if self.grad.is_cuda else self.grad.zero_()

    def ensure_acc(self):
        """The window accumulator: with gradient accumulation each batch's gradient is formed in ``grad`` and
        added here only if the loop's guards keep that batch (t2i_moe_gan.py:1315-1320)."""
        if self.acc is None or self.acc.device != self.data.device:
            self.acc = torch.zeros(self.total, device=self.device, dtype=torch.float32)
        return self.acc

    # ---- state dict (reference layout) ----
    def state_dict(self, cpu=True):
        sd = OrderedDict()
        for n in self.shapes:
            t = self.buffers[n] if is_buffer(n) else self.view(n)
            sd[n] = t.detach().clone().cpu() if cpu else t.detach().clone()
        return sd

    def load_state_dict(self, sd, strict=True):
        missing = [n for n in self.shapes if n not in sd]
        unexpected = [n for n in sd if n not in self.shapes]
        if strict and (missing or unexpected):
            raise KeyError(f"state_dict mismatch: missing={missing[:5]} unexpected={unexpected[:5]}")
        with torch.no_grad():
            for n, t in sd.items():
                if n not in self.shapes:
                    continue
                dst = self.buffers[n] if is_buffer(n) else self.view(n)
                dst.copy_(torch.as_tensor(t).reshape(dst.shape).to(dst.device, torch.float32))
        self.refresh_shadow(force=True)
