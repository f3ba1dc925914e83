"""Local test double for the OpenAI ``clip`` package (TEST INFRASTRUCTURE ONLY).

The reference imports ``clip`` at module top (t2i_moe_gan.py:10) and calls
``clip.load("ViT-B/32", device=..., jit=False)`` (t2i_moe_gan.py:44), which
downloads weights -- impossible offline.  The reference's CLIP loss is computed
under ``torch.no_grad()`` (t2i_moe_gan.py:98-101) and so never contributes a
gradient; this double only has to provide deterministic *values* for the
logged CLIP loss so that fixtures are reproducible.

The double is a fixed random projection of a 4x4 average-pooled image
(encode_image) and of a hashed token histogram (encode_text).  The same double
is used by the build's fixture generator (tests/golden/make_golden.py) so the plumbing of the
CLIP-loss term is pinned; real CLIP values remain "parity unpinned".
"""
import numpy as np
import torch
import torch.nn.functional as F

_EMBED = 512


def _proj(seed, rows):
    rng = np.random.default_rng(seed)
    return torch.from_numpy((rng.standard_normal((rows, _EMBED)) / np.sqrt(rows)).astype(np.float32))


class _DoubleModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.register_buffer("img_proj", _proj(1234, 3 * 4 * 4))
        self.register_buffer("txt_proj", _proj(4321, 64))

    @property
    def dtype(self):
        return torch.float32

    def encode_image(self, images):
        pooled = F.adaptive_avg_pool2d(images.float(), 4).flatten(1)
        return pooled @ self.img_proj.to(pooled.device)

    def encode_text(self, tokens):
        hist = torch.zeros(tokens.shape[0], 64, device=tokens.device)
        hist.scatter_add_(1, (tokens % 64).long(), torch.ones_like(tokens, dtype=torch.float32))
        return hist @ self.txt_proj.to(hist.device)


def load(name, device="cpu", jit=False):
    return _DoubleModel().to(device), (lambda x: x)


def tokenize(texts, context_length=77):
    if isinstance(texts, str):
        texts = [texts]
    out = torch.zeros(len(texts), context_length, dtype=torch.long)
    for i, t in enumerate(texts):
        codes = [ord(c) for c in t][:context_length]
        out[i, : len(codes)] = torch.tensor(codes, dtype=torch.long)
    return out
