"""Reference state_dict layout of the generator / discriminator.

Names, shapes and ORDER match ``t2i_moe_gan.AuroraGenerator`` /
``AuroraDiscriminator`` (t2i_moe_gan.py:668-907) so checkpoints interchange
with the reference (``{'generator': ..., 'discriminator': ...}``,
sagemaker_train.py:297-301) and the optimizer walks parameters in the same
order.  The build generalises the hard-wired ``NUM_EXPERTS = 4``
(t2i_moe_gan.py:23) to any E.
"""
from collections import OrderedDict

LATENT = 512
TEXT = 512
# (block name, Cin, Cout, resolution, upsample) -- t2i_moe_gan.py:704-706
GEN_BLOCKS = (("gen_block_4", 512, 512, 4, False),
              ("gen_block_8", 512, 256, 8, True),
              ("gen_block_16", 256, 128, 16, True))
# Progressive extension (BASELINE config C4): the reference names gen_block_32 / _64 and
# to_rgb_32 / _64 only in dead code (create_optimizer_for_active_blocks, t2i_moe_gan.py:1005-1026) and defines
# none of them.  The build's extension blocks are GenerativeBlocks without the attention block: upsample +
# ConvolutionBlock whose MTMs have no offset head (the reference's own rule, offsets only at resolution <= 16,
# :199).  Self-attention over (2^r)^2 tokens per image would cost 4 L^2 C flops -- at 128^2 more than the rest of
# the step -- so the MoE / attention stays at 4 / 8 / 16.  (name, Cin, Cout, resolution)
EXT_BLOCKS = (("gen_block_32", 128, 128, 32), ("gen_block_64", 128, 64, 64), ("gen_block_128", 64, 32, 128))
MAX_RESOLUTIONS = (16, 32, 64, 128)


def gen_blocks(max_res=16):
    """(name, Cin, Cout, resolution, upsample, attention) of every generator block up to ``max_res``."""
    if max_res not in MAX_RESOLUTIONS:
        raise ValueError(f"max_resolution must be one of {MAX_RESOLUTIONS}, got {max_res}")
    out = [b + (True,) for b in GEN_BLOCKS]
    out += [(n, ci, co, r, True, False) for n, ci, co, r in EXT_BLOCKS if r <= max_res]
    return tuple(out)


def rgb_layers(max_res=16):
    """(name, Cin) of the to_rgb layers: one per block from 8x8 up (reference: to_rgb_8 / to_rgb_16, :708-709).
    Training reads the last (final image) and the one before it (the CLIP-only intermediate image)."""
    return tuple((f"to_rgb_{r}", co) for _, _, co, r, _, _ in gen_blocks(max_res) if r >= 8)


def max_res_of(shapes):
    """The generator resolution a state_dict / shape table describes."""
    return max(r for r in MAX_RESOLUTIONS if r == 16 or f"to_rgb_{r}.weight" in shapes)
BUFFER_SUFFIXES = ("epsilon_f", "epsilon_t", "epsilon_c")


def _modconv(d, pre, cin, cout, k):
    d[pre + "weight"] = (cout, cin, k, k)
    d[pre + "modulation.weight"] = (cin, LATENT)
    d[pre + "modulation.bias"] = (cin,)


def _mtm(d, pre, cin, cout, offsets=True):
    _modconv(d, pre + "modulated_conv.", cin, cout, 3)
    if not offsets:  # resolution > 16 (:199)
        return
    d[pre + "offset_net.0.weight"] = (32, cin, 3, 3)
    d[pre + "offset_net.0.bias"] = (32,)
    d[pre + "offset_net.2.weight"] = (2, 32, 3, 3)
    d[pre + "offset_net.2.bias"] = (2,)


def _mha(d, pre, c):
    d[pre + "in_proj_weight"] = (3 * c, c)
    d[pre + "in_proj_bias"] = (3 * c,)
    d[pre + "out_proj.weight"] = (c, c)
    d[pre + "out_proj.bias"] = (c,)


def _attn(d, pre, c, E):
    for n in ("norm1", "norm2", "norm3"):
        d[f"{pre}{n}.weight"] = (c,)
        d[f"{pre}{n}.bias"] = (c,)
    d[pre + "text_proj.weight"] = (c, TEXT)
    d[pre + "text_proj.bias"] = (c,)
    _mha(d, pre + "self_attn.", c)
    _mha(d, pre + "cross_attn.", c)
    for e in range(E):
        q = f"{pre}moe.experts.{e}.net."
        d[q + "0.weight"] = (4 * c, c)
        d[q + "0.bias"] = (4 * c,)
        d[q + "2.weight"] = (c, 4 * c)
        d[q + "2.bias"] = (c,)
    r = pre + "moe.router."
    d[r + "feature_mu"] = (c, 128)
    d[r + "feature_rho"] = (c, 128)
    d[r + "text_mu"] = (TEXT, 128)
    d[r + "text_rho"] = (TEXT, 128)
    d[r + "combined_mu"] = (256, E)
    d[r + "combined_rho"] = (256, E)
    d[r + "temperature"] = (1,)
    d[r + "epsilon_f"] = (c, 128)
    d[r + "epsilon_t"] = (TEXT, 128)
    d[r + "epsilon_c"] = (256, E)
    _modconv(d, pre + "proj_in.", c, c, 1)
    _modconv(d, pre + "proj_out.", c, c, 1)


def generator_shapes(E=4, max_res=16):
    """Ordered ``{state_dict key: shape}`` of AuroraGenerator with E experts (``max_res`` > 16: the progressive
    extension, gen_blocks)."""
    d = OrderedDict()
    d["constant"] = (1, 512, 4, 4)
    for i in (0, 3):
        if i == 3:
            d["text_projection.1.weight"] = (TEXT,)
            d["text_projection.1.bias"] = (TEXT,)
        d[f"text_projection.{i}.weight"] = (TEXT, TEXT)
        d[f"text_projection.{i}.bias"] = (TEXT,)
    d.move_to_end("text_projection.3.weight")
    d.move_to_end("text_projection.3.bias")
    d["mapping.0.weight"] = (512, LATENT + TEXT)
    d["mapping.0.bias"] = (512,)
    for i in (2, 4, 6):
        d[f"mapping.{i}.weight"] = (512, 512)
        d[f"mapping.{i}.bias"] = (512,)
    for name, cin, cout, res, _, attn in gen_blocks(max_res):
        cb = name + ".conv_block."
        _mtm(d, cb + "mtm1.", cin, cout, res <= 16)
        _mtm(d, cb + "mtm2.", cout, cout, res <= 16)
        if cin != cout:
            _modconv(d, cb + "skip_proj.", cin, cout, 1)
        if attn:
            _attn(d, name + ".attn_block.", cout, E)
    for name, cin in rgb_layers(max_res):
        _modconv(d, name + ".", cin, 3, 1)
    return d


def frozen_rgb_prefixes(max_res=16):
    """to_rgb layers that never receive a gradient in training: all but the final one (the intermediate image
    only feeds the gradient-free CLIP loss, :98-101; the lower ones are unused).  Reference: ("to_rgb_8.",)."""
    return tuple(n + "." for n, _ in rgb_layers(max_res)[:-1])


def discriminator_shapes():
    """Ordered ``{state_dict key: shape}`` of AuroraDiscriminator (old-style weight_norm g/v)."""
    d = OrderedDict()
    d["text_projection.0.bias"] = (128,)
    d["text_projection.0.weight_g"] = (128, 1)
    d["text_projection.0.weight_v"] = (128, TEXT)
    d["conv_layers.0.bias"] = (128,)
    d["conv_layers.0.weight_g"] = (128, 1, 1, 1)
    d["conv_layers.0.weight_v"] = (128, 3, 4, 4)
    d["conv_layers.2.bias"] = (256,)
    d["conv_layers.2.weight_g"] = (256, 1, 1, 1)
    d["conv_layers.2.weight_v"] = (256, 128, 4, 4)
    d["output_layer.0.bias"] = (1,)
    d["output_layer.0.weight_g"] = (1, 1, 1, 1)
    d["output_layer.0.weight_v"] = (1, 384, 4, 4)
    return d


def is_buffer(name):
    return name.rsplit(".", 1)[-1] in BUFFER_SUFFIXES
