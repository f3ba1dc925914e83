"""Name-seeded parameter recipe (TEST INFRASTRUCTURE -- see oracle/__init__.py).

Every tensor of a reference-layout state_dict is filled from
``np.random.default_rng(crc32(name) ^ seed)`` with a per-kind scale, so golden
fixtures never have to store the 28-105 M generator weights: the fixture
generator (tests/golden/make_golden.py, which runs the reference) and the
build's tests both rebuild identical weights from names alone.

Scales are chosen so that every code path is exercised with O(1) signals:
router logits are spread wide enough that top-k margins exceed 1e-5, the
router temperature sits inside its clamp window (t2i_moe_gan.py:375) so its
gradient is live, and modulation styles are O(1) so demodulation is not
degenerate (t2i_moe_gan.py:158-166).
"""
import re
import zlib

import numpy as np

_LN_RE = re.compile(r"(norm\d\.(weight|bias)$)|(^text_projection\.1\.(weight|bias)$)")


def fill_value(name, shape, seed=0):
    """Deterministic float32 array for state_dict entry ``name`` of ``shape``."""
    rng = np.random.default_rng(zlib.crc32(name.encode()) ^ seed)
    n = rng.standard_normal(shape)
    last = name.rsplit(".", 1)[-1]
    if last.endswith("_rho"):
        v = -4.0 + 0.5 * n
    elif last in ("feature_mu", "text_mu"):
        v = 0.15 * n
    elif last == "combined_mu":
        v = 0.4 * n
    elif last == "temperature":
        v = np.full(shape, 1.0)
    elif last.startswith("epsilon_"):
        v = n
    elif _LN_RE.search(name):
        v = (1.0 + 0.1 * n) if last == "weight" else 0.1 * n
    elif last == "weight_g":
        v = np.abs(1.0 + 0.2 * n)
    elif name.endswith("modulation.weight"):
        v = n / np.sqrt(shape[1])
    elif name.endswith("modulation.bias"):
        v = 1.0 + 0.1 * n
    elif last == "constant":
        v = n
    elif len(shape) >= 2:
        fan_in = int(np.prod(shape[1:]))
        v = n / np.sqrt(fan_in)
    else:
        v = 0.1 * n
    return np.asarray(v, dtype=np.float32).reshape(shape)


def fill_state(shapes, seed=0):
    """``{name: shape}`` -> ``{name: float32 ndarray}``."""
    return {k: fill_value(k, tuple(s), seed) for k, s in shapes.items()}


def input_batch(B, seed_img=0, seed_txt=1, seed_z=2, res=64):
    """Synthetic inputs of SURVEY.md §8(d): images U(-1,1), text N(0,1), z N(0,1)."""
    img = np.random.default_rng(seed_img).uniform(-1, 1, (B, 3, res, res)).astype(np.float32)
    txt = np.random.default_rng(seed_txt).standard_normal((B, 512)).astype(np.float32)
    z = np.random.default_rng(seed_z).standard_normal((B, 512)).astype(np.float32)
    return img, txt, z
