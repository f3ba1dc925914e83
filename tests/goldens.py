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
    """Max-abs error <= atol + rtol * max|e|, AND element-wise |a - e| <= atol + 2 rtol (|e| + rms(e)): a few
    large entries cannot hide relative errors of the typical ones."""
    a = np.asarray(actual.detach().cpu().double() if torch.is_tensor(actual) else actual, dtype=np.float64)
    e = np.asarray(expected, dtype=np.float64)
    assert a.shape == e.shape, f"{what}: shape {a.shape} vs {e.shape}"
    if not e.size:
        return
    scale = np.abs(e).max()
    d = np.abs(a - e)
    err = d.max()
    assert err <= atol + rtol * scale, f"{what}: max abs err {err:.3e} (scale {scale:.3e})"
    rms = np.sqrt((e * e).mean())
    lim = atol + 2 * rtol * (np.abs(e) + rms)
    worst = int(np.argmax(d - lim))
    assert d.flat[worst] <= lim.flat[worst], (f"{what}: element {worst}: |{a.flat[worst]:.6e} - {e.flat[worst]:.6e}| "
                                              f"> {lim.flat[worst]:.3e} (rms {rms:.3e})")


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
        rms = max(np.sqrt(float(d[key + "#sumsq"]) / a.size), 1e-30)
        dd = np.abs(a[idx] - val)
        lim = atol + 2 * rtol * (np.abs(val) + rms)  # per sampled element, as close()
        w = int(np.argmax(dd - lim))
        assert dd[w] <= lim[w], f"{key}: sample {int(idx[w])}: err {dd[w]:.3e} > {lim[w]:.3e} (rms {rms:.3e})"
    ss = float(d[key + "#sumsq"])
    assert abs((a * a).sum() - ss) <= 1e-3 * ss + atol, f"{key}: sumsq {(a*a).sum():.6e} vs {ss:.6e}"
