"""Helpers to read the golden fixtures and compare against them."""
import json
import os

import numpy as np
import torch

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    d = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    meta = json.loads(str(d["__meta__"]))
    return d, meta


def T(a):
    return torch.from_numpy(np.array(a, dtype=np.float32))


def close(actual, expected, rtol=1e-4, atol=1e-5, what=""):
    a = np.asarray(actual.detach().cpu().double() if torch.is_tensor(actual) else actual, dtype=np.float64)
    e = np.asarray(expected, dtype=np.float64)
    assert a.shape == e.shape, f"{what}: shape {a.shape} vs {e.shape}"
    scale = np.abs(e).max() if e.size else 0.0
    err = np.abs(a - e).max() if e.size else 0.0
    assert err <= atol + rtol * scale, f"{what}: max abs err {err:.3e} (scale {scale:.3e})"


def check_packed(d, key, actual, rtol=1e-4, atol=1e-6):
    """Compare a tensor against a fixture entry stored whole or as stats+samples."""
    a = actual.detach().cpu().double().reshape(-1).numpy()
    if key in d.files:
        e = d[key].astype(np.float64).reshape(-1)
        scale = max(np.abs(e).max(), 1e-30)
        err = np.abs(a - e).max()
        assert err <= atol + rtol * scale, f"{key}: max abs err {err:.3e} (scale {scale:.3e})"
    else:
        idx, val = d[key + "#idx"], d[key + "#val"].astype(np.float64)
        assert a.size == int(np.prod(d[key + "#shape"])), key
        scale = max(np.sqrt(float(d[key + "#sumsq"]) / a.size), 1e-30)
        err = np.abs(a[idx] - val).max()
        assert err <= atol + rtol * 10 * scale, f"{key}: sampled err {err:.3e} (rms {scale:.3e})"
    ss = float(d[key + "#sumsq"])
    assert abs((a * a).sum() - ss) <= 1e-3 * ss + atol, f"{key}: sumsq {(a*a).sum():.6e} vs {ss:.6e}"
