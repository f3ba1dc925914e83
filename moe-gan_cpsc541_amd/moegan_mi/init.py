"""Reference-equivalent random initialisation for the flat parameter stores.

Follows the module constructors of t2i_moe_gan.py: ModulatedConv (kaiming_normal
fan_in / leaky_relu gain, modulation N(0, 0.02), bias 0; :142-152), nn.Linear /
nn.Conv2d defaults (kaiming_uniform(a=sqrt(5)) weights, U(+-1/sqrt(fan_in)) bias),
LayerNorm (1, 0), nn.MultiheadAttention (xavier_uniform in_proj, zero biases),
BayesianRouter (mu N(0, 0.01), rho -4, temperature 4; :279-301), the 4x4
constant N(0, 1) (:701) and weight_norm (g = ||v||) for the discriminator.
"""
import math
import re

import torch

from .layout import is_buffer

_LN = re.compile(r"(norm\d\.(weight|bias)$)|(^text_projection\.1\.(weight|bias)$)")


def _kaiming_uniform_a5(t, gen):
    fan_in = t[0].numel()
    bound = 1.0 / math.sqrt(fan_in)  # gain sqrt(2/(1+5)) * sqrt(3/fan_in)
    return t.uniform_(-bound, bound, generator=gen)


def init_generator(store, seed=0):
    gen = torch.Generator(device="cpu").manual_seed(seed)
    sd = {}
    shapes = store.shapes
    for n, shp in shapes.items():
        last = n.rsplit(".", 1)[-1]
        t = torch.empty(shp)
        if is_buffer(n):
            t.zero_()
        elif last.endswith("_rho"):
            t.fill_(-4.0)
        elif last.endswith("_mu"):
            t.normal_(0.0, 0.01, generator=gen)
        elif last == "temperature":
            t.fill_(4.0)
        elif n == "constant":
            t.normal_(0.0, 1.0, generator=gen)
        elif _LN.search(n):
            t.fill_(1.0 if last == "weight" else 0.0)
        elif n.endswith("modulation.weight"):
            t.normal_(0.0, 0.02, generator=gen)
        elif n.endswith("modulation.bias"):
            t.zero_()
        elif len(shp) == 4 and ".offset_net." not in n:  # ModulatedConv weight
            fan_in = shp[1] * shp[2] * shp[3]
            t.normal_(0.0, math.sqrt(2.0) / math.sqrt(fan_in), generator=gen)
        elif last == "in_proj_weight":
            a = math.sqrt(6.0 / (shp[0] // 3 + shp[1]))
            t.uniform_(-a, a, generator=gen)
        elif last == "in_proj_bias" or n.endswith("out_proj.bias"):
            t.zero_()
        elif len(shp) >= 2:
            _kaiming_uniform_a5(t, gen)
        else:  # bias of a Linear / Conv2d: U(+-1/sqrt(fan_in)) of its weight
            wname = n[: -len("bias")] + "weight"
            fan_in = int(torch.tensor(shapes[wname][1:]).prod()) if wname in shapes else shp[0]
            b = 1.0 / math.sqrt(fan_in)
            t.uniform_(-b, b, generator=gen)
        sd[n] = t
    store.load_state_dict(sd)


def init_discriminator(store, seed=1):
    gen = torch.Generator(device="cpu").manual_seed(seed)
    sd = {}
    for n, shp in store.shapes.items():
        if n.endswith("weight_v"):
            sd[n] = _kaiming_uniform_a5(torch.empty(shp), gen)
    for n, shp in store.shapes.items():
        if n.endswith("weight_g"):
            v = sd[n[: -1] + "v"]
            sd[n] = v.reshape(v.shape[0], -1).norm(dim=1).reshape(shp)
        elif n.endswith("bias"):
            v = sd[n[: -len("bias")] + "weight_v"]
            b = 1.0 / math.sqrt(v[0].numel())
            sd[n] = torch.empty(shp).uniform_(-b, b, generator=gen)
    store.load_state_dict(sd)
