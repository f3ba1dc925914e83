"""Forward-only CLIP image tower (moegan_mi/clip_vit.py) vs a plain fp32 PyTorch restatement of OpenAI CLIP's
VisionTransformer (conv1 patchify, class token, positional embedding, ln_pre, pre-LN residual blocks with
nn.MultiheadAttention and a QuickGELU MLP, ln_post on the class token, @ proj), on the same OpenAI-layout
state_dict.  The CLIP weights themselves are not available (no download): random weights at CLIP's init scales
exercise every op; the values of the CLIP loss stay parity-unpinned against the reference (t2i_moe_gan.py:66-119).

Bar: the device runs bf16 token rows (the reference runs CLIP in fp16), so features are held to cosine >= 0.999
per image and 2e-2 relative L2 overall.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def torch_vit(sd, img, heads):
    x = F.conv2d(img, sd["conv1.weight"], stride=sd["conv1.weight"].shape[-1])
    B, w = x.shape[:2]
    x = x.reshape(B, w, -1).permute(0, 2, 1)
    x = torch.cat([sd["class_embedding"].expand(B, 1, w), x], dim=1) + sd["positional_embedding"]
    x = F.layer_norm(x, (w,), sd["ln_pre.weight"], sd["ln_pre.bias"])
    i = 0
    while f"transformer.resblocks.{i}.ln_1.weight" in sd:
        p = f"transformer.resblocks.{i}."
        h = F.layer_norm(x, (w,), sd[p + "ln_1.weight"], sd[p + "ln_1.bias"])
        a, _ = F.multi_head_attention_forward(
            h.transpose(0, 1), h.transpose(0, 1), h.transpose(0, 1), w, heads, sd[p + "attn.in_proj_weight"],
            sd[p + "attn.in_proj_bias"], None, None, False, 0.0, sd[p + "attn.out_proj.weight"],
            sd[p + "attn.out_proj.bias"], need_weights=False)
        x = x + a.transpose(0, 1)
        h = F.layer_norm(x, (w,), sd[p + "ln_2.weight"], sd[p + "ln_2.bias"])
        h = F.linear(h, sd[p + "mlp.c_fc.weight"], sd[p + "mlp.c_fc.bias"])
        h = h * torch.sigmoid(1.702 * h)
        x = x + F.linear(h, sd[p + "mlp.c_proj.weight"], sd[p + "mlp.c_proj.bias"])
        i += 1
    return F.layer_norm(x[:, 0], (w,), sd["ln_post.weight"], sd["ln_post.bias"]) @ sd["proj"]


@pytest.mark.parametrize("layers", [2, 12])
def test_clip_image_tower_vs_torch(layers):
    from moegan_mi.clip_vit import ClipImageEncoder, random_state_dict
    sd = random_state_dict(768, layers, 32, 224, 512, seed=layers)
    full = {"visual." + k: v for k, v in sd.items()}  # the whole-model key layout loads too
    full["logit_scale"] = torch.tensor(4.6)
    enc = ClipImageEncoder(full, device=DEV)
    assert (enc.width, enc.layers, enc.heads, enc.patch, enc.resolution) == (768, layers, 12, 32, 224)
    g = torch.Generator().manual_seed(1)
    img = torch.rand(3, 3, 224, 224, generator=g) * 2 - 1
    ref = torch_vit(sd, img, 12)
    got = enc.encode_image(img.to(DEV)).cpu()
    assert got.shape == (3, 512)
    cos = F.cosine_similarity(got.double(), ref.double(), dim=1)
    rel = float((got - ref).norm() / ref.norm())
    print(f"CLIP tower layers={layers}: per-image cosine {cos.tolist()}, rel L2 {rel:.3e}")
    assert float(cos.min()) >= 0.999 and rel <= 2e-2


def test_clip_loss_in_step_and_dropin():
    """TrainStep's CLIP terms and the drop-in CLIPLoss read the registered tower (no gradient, :98-101)."""
    import t2i_moe_gan as M
    from moegan_mi.clip_vit import ClipImageEncoder, random_state_dict
    from moegan_mi.step import clip_loss
    enc = ClipImageEncoder(random_state_dict(768, 2, 32, 224, 512, seed=3), device=DEV)
    g = torch.Generator().manual_seed(2)
    img16 = (torch.rand(4, 3, 16, 16, generator=g) * 2 - 1).to(DEV)
    text = torch.randn(4, 512, generator=g).to(DEV)
    v = clip_loss(img16, text, enc.encode_image)
    up = F.interpolate(img16.clamp(-1, 1), size=(224, 224), mode="bilinear", align_corners=False)
    f = enc.encode_image(up)
    exp = 1 - F.cosine_similarity(f, text, dim=1).mean()
    assert abs(float(v) - float(exp)) < 1e-4
    M.set_clip_model(enc)
    try:
        loss = M.CLIPLoss(DEV)(img16, text)
        assert abs(float(loss) - float(exp)) < 1e-4
    finally:
        M.set_clip_model(None)


@pytest.mark.parametrize("R,dtype", [(16, torch.float32), (128, torch.bfloat16), (64, torch.bfloat16)])
def test_clip_patches_match_clamp_interpolate_unfold(R, dtype):
    """mg_clip_patches (clamp + bilinear resize to 224 + conv1 patchify, from the generator's NHWC channel-padded
    image) against the reference's input path: torch.clamp, F.interpolate(bilinear, align_corners=False)
    (t2i_moe_gan.py:90-94) and the unfold, in fp32 then bf16.  Bar: one bf16 rounding step (the fp32 interpolation
    may differ in the last bit by its evaluation order)."""
    from moegan_mi import ops
    from moegan_mi.clip_vit import ClipImageEncoder, random_state_dict
    B, ld = 3, 8
    g = torch.Generator(device="cuda").manual_seed(R)
    nhwc = (torch.randn(B, R, R, ld, device="cuda", generator=g) * 0.8).to(dtype)  # some values beyond [-1, 1]
    got = ops.clip_patches(nhwc, 224, 32).float()
    im = torch.clamp(nhwc[..., :3].permute(0, 3, 1, 2).float(), -1, 1)
    im = F.interpolate(im, size=(224, 224), mode="bilinear", align_corners=False)
    ref = im.reshape(B, 3, 7, 32, 7, 32).permute(0, 2, 4, 1, 3, 5).reshape(B * 49, 3 * 1024)
    assert ((got - ref.bfloat16().float()).abs() <= ref.abs() * 2 ** -7 + 1e-6).all()
    enc = ClipImageEncoder(random_state_dict(768, 2, 32, 224, 512, seed=3), device="cuda")
    f_gen = enc.encode_generated(nhwc)
    f_ref = enc.encode_image(im)
    cos = F.cosine_similarity(f_gen.double(), f_ref.double(), dim=1)
    assert float(cos.min()) >= 0.9999
