"""Progressive generator extension: parameter layout and the oracle's composition on the CPU (no GPU)."""
import torch

from moegan_mi.layout import frozen_rgb_prefixes, gen_blocks, generator_shapes, max_res_of, rgb_layers
from oracle import aurora_cpu as O
from oracle.recipe import fill_state


def test_reference_layout_unchanged():
    """max_res = 16 is exactly the reference generator (F9 pins the key order / shapes separately)."""
    assert [b[:5] for b in gen_blocks(16)] == [("gen_block_4", 512, 512, 4, False), ("gen_block_8", 512, 256, 8, True),
                                               ("gen_block_16", 256, 128, 16, True)]
    assert rgb_layers(16) == (("to_rgb_8", 256), ("to_rgb_16", 128))
    assert frozen_rgb_prefixes(16) == ("to_rgb_8.",)
    assert max_res_of(generator_shapes(4)) == 16


def test_progressive_layout():
    s = generator_shapes(16, 128)
    assert max_res_of(s) == 128
    for name, cin, cout in (("gen_block_32", 128, 128), ("gen_block_64", 128, 64), ("gen_block_128", 64, 32)):
        assert s[f"{name}.conv_block.mtm1.modulated_conv.weight"] == (cout, cin, 3, 3)
        assert not any(k.startswith(name + ".attn_block.") for k in s)  # MoE / attention stays at 4 / 8 / 16
        assert not any(k.startswith(name) and "offset_net" in k for k in s)  # no offset head above 16x16 (:199)
        assert (f"{name}.conv_block.skip_proj.weight" in s) == (cin != cout)
    assert [n for n, _ in rgb_layers(128)] == ["to_rgb_8", "to_rgb_16", "to_rgb_32", "to_rgb_64", "to_rgb_128"]
    assert frozen_rgb_prefixes(128) == ("to_rgb_8.", "to_rgb_16.", "to_rgb_32.", "to_rgb_64.")
    assert s["gen_block_4.attn_block.moe.experts.15.net.0.weight"] == (2048, 512)  # E = 16 (config C4)
    # every key of the 16x16 generator is still there with the same shape
    ref = generator_shapes(16, 16)
    assert all(s[k] == v for k, v in ref.items())


def test_oracle_progressive_step_runs():
    """The oracle's train_step at 32x32 (real and fake 32x32; the D head gives 5x5 logits for both)."""
    from steputil import make_inputs, oracle_models
    torch.manual_seed(0)
    real, text, z, eps_d, eps_g, perm = make_inputs(2, 4, seed=1, res=32)
    PG, PD, optG, optD, grads = oracle_models(4, max_res=32)
    out = O.train_step(PG, PD, optG, optD, real, text, z, eps_d, eps_g, perm, full=True)
    assert out["img16"].shape == (2, 3, 32, 32) and out["img8"].shape == (2, 3, 16, 16)
    assert out["fake_pred"].shape == (2 * 25,)
    for k in ("d_loss_gan", "r1", "g_loss_gan", "balance"):
        assert torch.isfinite(torch.tensor(out[k])), k
    assert grads["G"]["to_rgb_32.weight"] is not None and grads["G"].get("to_rgb_16.weight") is None
    assert grads["G"]["gen_block_32.conv_block.mtm2.modulated_conv.weight"].abs().sum() > 0
    assert max_res_of(fill_state(generator_shapes(4, 32), 0)) == 32
