"""CPU checks of the drop-in boundary: the C ABI exports, the reference state_dict layout (F9, taken
from the reference modules themselves) and the host-side module API (no device compute here)."""
import ctypes
import json
import os
import re

import pytest
import torch

from conftest import PKG, REPO

GOLD = os.path.join(REPO, "tests", "golden")


def _header_symbols():
    txt = open(os.path.join(REPO, "include", "moegan_hip.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return re.findall(r"\b(?:int|int64_t|const char\*)\s+(mg_\w+)\(", txt)


def test_library_exports_every_header_symbol():
    path = os.path.join(PKG, "moegan_mi", "libmoegan_hip.so")
    if not os.path.exists(path):
        pytest.skip("libmoegan_hip.so not built (run __graft_entry__.build())")
    lib = ctypes.CDLL(path)
    syms = _header_symbols()
    assert len(syms) >= 50
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing


def test_binding_matches_header():
    from moegan_mi import _lib as L
    assert set(L._SIGS) == set(_header_symbols())


def _f9():
    with open(os.path.join(GOLD, "F9_layout.json")) as f:
        return json.load(f)


def test_layout_matches_reference_state_dict():
    from moegan_mi.layout import discriminator_shapes, generator_shapes, is_buffer
    lay = _f9()
    for tag, shapes in (("G", generator_shapes(4)), ("D", discriminator_shapes())):
        ref = lay[tag]
        assert list(shapes.keys()) == ref["keys"], tag
        assert [list(v) for v in shapes.values()] == ref["shapes"], tag
        assert [k for k in shapes if not is_buffer(k)] == ref["params"], tag


def test_module_state_dict_is_reference_layout():
    import t2i_moe_gan as M
    lay = _f9()
    G = M.AuroraGenerator()
    D = M.AuroraDiscriminator()
    for tag, mod in (("G", G), ("D", D)):
        sd = mod.state_dict()
        assert list(sd.keys()) == lay[tag]["keys"]
        assert [list(v.shape) for v in sd.values()] == lay[tag]["shapes"]
    # round trip through a checkpoint dict, the way sagemaker_train.py / inference.py use it
    G2 = M.AuroraGenerator(seed=7)
    assert not torch.equal(G2.state_dict()["constant"], G.state_dict()["constant"])
    G2.load_state_dict(G.state_dict())
    for k, v in G.state_dict().items():
        assert torch.equal(G2.state_dict()[k], v), k
    # one flat parameter per model
    assert [n for n, _ in G.named_parameters()] == ["flat"]
    assert G.flat.numel() == G._store.total


def test_module_init_statistics():
    """Reference init: router rho -4, temperature 4, LayerNorm 1/0, weight_g = ||v||."""
    import t2i_moe_gan as M
    sd = M.AuroraGenerator().state_dict()
    r = "gen_block_8.attn_block.moe.router."
    assert torch.all(sd[r + "feature_rho"] == -4.0)
    assert torch.all(sd[r + "temperature"] == 4.0)
    assert torch.all(sd["text_projection.1.weight"] == 1.0)
    sdd = M.AuroraDiscriminator().state_dict()
    v = sdd["conv_layers.0.weight_v"]
    g = sdd["conv_layers.0.weight_g"]
    assert torch.allclose(g.view(-1), v.view(v.shape[0], -1).norm(dim=1), rtol=1e-5)


def test_forward_needs_device():
    import t2i_moe_gan as M
    G = M.AuroraGenerator()
    with pytest.raises(RuntimeError, match="HIP device"):
        G(torch.zeros(1, 512), torch.zeros(1, 512))
    D = M.AuroraDiscriminator()
    with pytest.raises(RuntimeError, match="HIP device"):
        D(torch.zeros(1, 3, 16, 16), torch.zeros(1, 512))


def test_lr_schedule_matches_reference_rules():
    """Warmup 0.1->1 linear per epoch, then CosineAnnealingLR(T_max=epochs-warmup, eta_min=5%) stepped per
    epoch on the lr the warmup left behind (t2i_moe_gan.py:1108-1118, :1149-1166, :1514-1516)."""
    import math

    import t2i_moe_gan as M
    lr, n, w = 2e-4, 10, 3
    got = M._lr_schedule(lr, n, w)
    assert got[:3] == pytest.approx([lr * 0.1, lr * 0.4, lr * 0.7])
    # closed form of torch's recursive cosine starting from the last warmup lr
    eta = 0.05 * lr
    cur = got[2]
    T = n - w
    for e in range(w, n):
        assert got[e] == pytest.approx(cur, rel=1e-6)
        k = e - w + 1
        cur = eta + (1 + math.cos(math.pi * k / T)) / (1 + math.cos(math.pi * (k - 1) / T)) * (cur - eta)


def test_train_model_cli_flags():
    """train_model.py accepts the reference CLI (moegan/train_model.py argparse flags)."""
    import subprocess
    import sys
    out = subprocess.run([sys.executable, os.path.join(PKG, "train_model.py"), "--help"], capture_output=True,
                         text=True, timeout=120)
    assert out.returncode == 0, out.stderr
    for flag in ("--data_dir", "--batch_size", "--epochs", "--lr", "--r1_gamma", "--clip_weight_64",
                 "--clip_weight_32", "--kl_weight", "--balance_weight", "--save_dir", "--log_interval",
                 "--save_interval", "--train_images", "--val_embeddings"):
        assert flag in out.stdout, flag
