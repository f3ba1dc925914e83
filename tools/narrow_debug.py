"""Direct vs implicit-GEMM offset-head forward on one shape: fp32 outputs against an fp64 reference (max / mean
error, where the largest errors sit in the tile), and bf16 outputs (fraction of elements that differ, largest
difference in units of the output's bf16 spacing)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV, bf = "cuda", torch.bfloat16
for B, S, C in ((8, 16, 256), (8, 16, 128), (8, 8, 256), (8, 4, 512)):
    g = torch.Generator(device=DEV).manual_seed(1)
    x = torch.randn(B, S, S, C, device=DEV, generator=g).to(bf)
    W = torch.randn(32, C, 3, 3, device=DEV, generator=g) * (9 * C) ** -0.5
    bias = torch.randn(32, device=DEV, generator=g) * 0.1
    wp = ops.pack_conv(W, bf)
    ep = ops.E(bias=bias, act=L.ACT_LRELU)
    ref = F.leaky_relu(F.conv2d(x.double().permute(0, 3, 1, 2), W.to(bf).double(), bias.double(), padding=1), 0.2)
    ref = ref.permute(0, 2, 3, 1)
    out = {}
    for mode in (0, 1):
        L.call("mg_set_tuning", 16, mode)
        for dt in (torch.float32, bf):
            out[mode, dt] = ops.conv2d(x, wp, 32, 3, 3, 1, 1, out_dtype=dt, ep=ep)
    L.call("mg_set_tuning", 16, 0)
    torch.cuda.synchronize()
    for mode, name in ((0, "direct"), (1, "generic")):
        e = (out[mode, torch.float32].double() - ref).abs()
        flat = e.view(B, S, S, 32).amax(dim=(0, 3))
        print(f"B={B} S={S} C={C} {name:7s} fp32: max {float(e.max()):.3e} mean {float(e.mean()):.3e}; "
              f"worst (row, col) {divmod(int(flat.argmax()), S)}", flush=True)
    a, b = out[0, bf].float(), out[1, bf].float()
    ulp = torch.maximum(a.abs(), b.abs()).clamp_min(1e-30)
    ulp = torch.exp2(torch.floor(torch.log2(ulp)) - 7)
    d = (a - b).abs() / ulp
    print(f"B={B} S={S} C={C} bf16 direct vs generic: {float((a != b).float().mean()) * 100:.3f}% differ, "
          f"max {float(d.max()):.1f} ulp; vs fp64: direct mean {float((a.double() - ref).abs().mean()):.3e} "
          f"generic mean {float((b.double() - ref).abs().mean()):.3e}", flush=True)
