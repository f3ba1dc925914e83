"""Forward-only CLIP image tower (ViT-B/32 layout) on the HIP kernels, for the CLIP loss terms.

The reference scores every generated image with OpenAI CLIP ``encode_image`` (``CLIPLoss``,
t2i_moe_gan.py:66-119; used for the logged G-loss terms :1385-1387 and the HPO objective ``val_clip_loss``,
:1581-1625).  Those terms carry no gradient (:98-101), so only a forward pass is needed.  The ``clip``
package and its downloaded weights are not available to this build: this module is the image tower
itself, reading the OpenAI state_dict layout (``visual.conv1.weight``, ``visual.class_embedding``,
``visual.positional_embedding``, ``visual.ln_pre.*``, ``visual.transformer.resblocks.{i}.{ln_1,attn,ln_2,
mlp.c_fc,mlp.c_proj}.*``, ``visual.ln_post.*``, ``visual.proj``) from a local file, or random-initialised
with the same shapes when no weights are given (the bench's "CLIP-loss on" config C4 measures the cost; its
values are then meaningless and parity-unpinned: CLIP weights cannot be fetched here).

Compute: the 32x32/32 patch embedding is one GEMM over unfolded patches, every Linear runs on the MFMA GEMM
core with its bias / QuickGELU / residual add in the epilogue (ACT_QUICK_GELU), LayerNorm on mg_layernorm_fwd,
and the 12-head self-attention over the 50 tokens on mg_attn_fwd.  Activations are bf16 token rows (the
reference runs CLIP in fp16 on the GPU), LayerNorm statistics and GEMM accumulation fp32.
"""
import math

import torch

from . import _lib as L
from . import ops


class ClipImageEncoder:
    def __init__(self, state_dict=None, device="cuda", width=768, layers=12, heads=None, patch=32, resolution=224,
                 output_dim=512, seed=0):
        sd = _strip_visual(state_dict) if state_dict is not None else None
        if sd is not None:  # infer the architecture from the weights
            width = sd["conv1.weight"].shape[0]
            patch = sd["conv1.weight"].shape[-1]
            layers = 1 + max(int(k.split(".")[2]) for k in sd if k.startswith("transformer.resblocks."))
            grid = int(round(math.sqrt(sd["positional_embedding"].shape[0] - 1)))
            resolution = grid * patch
            output_dim = sd["proj"].shape[1]
        self.width, self.layers, self.patch, self.resolution = width, layers, patch, resolution
        self.heads = heads or width // 64  # OpenAI ViT: 64-wide heads
        self.output_dim = output_dim
        self.grid = resolution // patch
        self.dev = torch.device(device)
        if sd is None:
            sd = random_state_dict(width, layers, patch, resolution, output_dim, seed)
        self._load(sd)

    @classmethod
    def from_file(cls, path, device="cuda"):
        """OpenAI CLIP weights saved as a plain state_dict (``torch.save(model.state_dict())``) or safetensors;
        loaded without executing anything from the file (weights_only / safetensors)."""
        if str(path).endswith(".safetensors"):
            from safetensors.torch import load_file
            sd = load_file(str(path))
        else:
            sd = torch.load(path, map_location="cpu", weights_only=True)
        return cls(sd, device=device)

    def _load(self, sd):
        dev, bf = self.dev, torch.bfloat16
        mat = lambda t: t.detach().to(dev, bf).contiguous()  # noqa: E731  (MFMA operands)
        vec = lambda t: t.detach().to(dev, torch.float32).contiguous()  # noqa: E731  (bias / LN / embeddings)
        self.W_patch = mat(sd["conv1.weight"].reshape(self.width, -1))  # [w, 3*p*p], (c, kh, kw) order
        self.cls = vec(sd["class_embedding"])
        self.pos = vec(sd["positional_embedding"])
        self.ln_pre = (vec(sd["ln_pre.weight"]), vec(sd["ln_pre.bias"]))
        self.ln_post = (vec(sd["ln_post.weight"]), vec(sd["ln_post.bias"]))
        self.proj_t = mat(sd["proj"].t())  # [out, w]
        self.blocks = []
        for i in range(self.layers):
            p = f"transformer.resblocks.{i}."
            self.blocks.append(dict(
                ln1=(vec(sd[p + "ln_1.weight"]), vec(sd[p + "ln_1.bias"])),
                W_in=mat(sd[p + "attn.in_proj_weight"]), b_in=vec(sd[p + "attn.in_proj_bias"]),
                W_out=mat(sd[p + "attn.out_proj.weight"]), b_out=vec(sd[p + "attn.out_proj.bias"]),
                ln2=(vec(sd[p + "ln_2.weight"]), vec(sd[p + "ln_2.bias"])),
                W_fc=mat(sd[p + "mlp.c_fc.weight"]), b_fc=vec(sd[p + "mlp.c_fc.bias"]),
                W_proj=mat(sd[p + "mlp.c_proj.weight"]), b_proj=vec(sd[p + "mlp.c_proj.bias"])))

    @torch.no_grad()
    def encode_image(self, img):
        """img [B, 3, res, res] (any float dtype, the caller's value range) -> image features [B, output_dim] fp32."""
        B = img.shape[0]
        p, g = self.patch, self.grid
        assert tuple(img.shape[1:]) == (3, self.resolution, self.resolution), img.shape
        patches = img.to(self.dev, torch.bfloat16).reshape(B, 3, g, p, g, p).permute(0, 2, 4, 1, 3, 5)
        return self._encode_patches(patches.reshape(B * g * g, 3 * p * p), B)

    @torch.no_grad()
    def encode_generated(self, img_nhwc):
        """CLIPLoss's input path for a generator image, NHWC [B, R, R, ld] (channels 0..2, any R): clamp, bilinear
        resize to the tower's resolution and patchify in one kernel (mg_clip_patches), then the tower."""
        patches = ops.clip_patches(img_nhwc.contiguous(), self.resolution, self.patch)
        return self._encode_patches(patches, img_nhwc.shape[0])

    def _encode_patches(self, patches, B):
        g, w = self.grid, self.width
        T = g * g + 1
        # patch embedding (conv1, stride = kernel = patch, no bias) as one GEMM over unfolded patches
        emb = ops.linear(patches, self.W_patch, out_dtype=torch.float32)
        x = torch.empty(B, T, w, device=self.dev, dtype=torch.float32)
        x[:, 0] = self.cls
        x[:, 1:] = emb.view(B, g * g, w)
        x += self.pos
        x = x.view(B * T, w)
        xb = ops.cast(ops.layernorm_fwd(x, *self.ln_pre)[0], torch.bfloat16)  # the residual stream starts here
        for blk in self.blocks:
            n1, _, _ = ops.layernorm_fwd(xb, *blk["ln1"])
            qkv = ops.linear(n1, blk["W_in"], bias=blk["b_in"])
            att, _ = ops.attn_fwd(qkv, B, T, w, heads=self.heads)
            xb = ops.linear(att, blk["W_out"], bias=blk["b_out"], resid=xb, ld_res=w)  # x + attn(ln_1(x))
            n2, _, _ = ops.layernorm_fwd(xb, *blk["ln2"])
            hid = ops.linear(n2, blk["W_fc"], bias=blk["b_fc"], act=L.ACT_QUICK_GELU)
            xb = ops.linear(hid, blk["W_proj"], bias=blk["b_proj"], resid=xb, ld_res=w)  # x + mlp(ln_2(x))
        cls_rows = xb.view(B, T, w)[:, 0].contiguous()
        c, _, _ = ops.layernorm_fwd(cls_rows, *self.ln_post)
        return ops.linear(c, self.proj_t, out_dtype=torch.float32)

    __call__ = encode_image


def _strip_visual(sd):
    """Accept a whole CLIP state_dict (``visual.*`` keys) or the image tower's own."""
    if any(k.startswith("visual.") for k in sd):
        return {k[len("visual."):]: v for k, v in sd.items() if k.startswith("visual.")}
    return dict(sd)


def random_state_dict(width=768, layers=12, patch=32, resolution=224, output_dim=512, seed=0):
    """OpenAI CLIP's VisionTransformer initialisation scales (std width^-0.5 for the embeddings and projection,
    attention / MLP weights as CLIP.initialize_parameters), in its state_dict layout."""
    gen = torch.Generator().manual_seed(seed)
    n = lambda *s, std: torch.randn(*s, generator=gen) * std  # noqa: E731
    grid = resolution // patch
    sc = width ** -0.5
    proj_std, attn_std, fc_std = sc * (2 * layers) ** -0.5, sc, (2 * width) ** -0.5
    sd = {"conv1.weight": n(width, 3, patch, patch, std=(3 * patch * patch) ** -0.5),
          "class_embedding": n(width, std=sc), "positional_embedding": n(grid * grid + 1, width, std=sc),
          "ln_pre.weight": torch.ones(width), "ln_pre.bias": torch.zeros(width),
          "ln_post.weight": torch.ones(width), "ln_post.bias": torch.zeros(width),
          "proj": n(width, output_dim, std=sc)}
    for i in range(layers):
        p = f"transformer.resblocks.{i}."
        sd.update({p + "ln_1.weight": torch.ones(width), p + "ln_1.bias": torch.zeros(width),
                   p + "ln_2.weight": torch.ones(width), p + "ln_2.bias": torch.zeros(width),
                   p + "attn.in_proj_weight": n(3 * width, width, std=attn_std),
                   p + "attn.in_proj_bias": torch.zeros(3 * width),
                   p + "attn.out_proj.weight": n(width, width, std=proj_std),
                   p + "attn.out_proj.bias": torch.zeros(width),
                   p + "mlp.c_fc.weight": n(4 * width, width, std=fc_std), p + "mlp.c_fc.bias": torch.zeros(4 * width),
                   p + "mlp.c_proj.weight": n(width, 4 * width, std=proj_std),
                   p + "mlp.c_proj.bias": torch.zeros(width)})
    return sd
