"""Isolated timing of the discriminator's first-conv passes at the C2 shapes (B=256, 64x64 real images): the direct
kernels (mg_d0_fwd / mg_d0_wgrad / mg_d0_dgrad) against the im2col + GEMM path, HIP events over REPS launches.
Run under rocprofv3 --kernel-trace --stats for per-kernel times."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]

import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

REPS = int(os.environ.get("REPS", "20"))
B, H = int(os.environ.get("B", "256")), int(os.environ.get("H", "64"))
dev = "cuda"
g = torch.Generator(device=dev).manual_seed(0)
x = torch.rand(B, 3, H, H, device=dev, generator=g) * 2 - 1
xs = (3 * H * H, H, 1, H * H)
u = torch.zeros(B, H, H, 4, device=dev, dtype=torch.bfloat16)
u[..., :3] = x.permute(0, 2, 3, 1).bfloat16()
us = (H * H * 4, H * 4, 4, 1)
w0p = (torch.randn(128, 48, device=dev, generator=g) * 0.2).bfloat16()
bias = torch.randn(128, device=dev, generator=g) * 0.1
gy = torch.randn(B, H // 2, H // 2, 128, device=dev, generator=g).bfloat16()
dw = torch.zeros(128, 48, device=dev)
gx = torch.zeros(B, H, H, 4, device=dev)
h0 = ops.d0_fwd(x, xs, B, H, H, w0p, bias=bias)
P = B * (H // 2) ** 2


def old_fwd():
    cols = ops.im2col_4x4s2(x, xs, B, H, H, 3, 48, torch.bfloat16)
    return ops.linear(cols, w0p, bias=bias, act=L.ACT_LRELU)


def old_fwd_u():
    cols = ops.im2col_4x4s2(u, us, B, H, H, 3, 48, torch.bfloat16)
    out = torch.empty(P, 128, device=dev, dtype=torch.bfloat16)
    return ops.gemm(cols, w0p, P, 128, 48, out=out, ep=ops.E(act=L.ACT_MUL_LRELU_GRAD, aux=h0, ld_aux=128))


cols = ops.im2col_4x4s2(x, xs, B, H, H, 3, 48, torch.bfloat16)
cases = {
    "d0_fwd real (direct)": lambda: ops.d0_fwd(x, xs, B, H, H, w0p, bias=bias),
    "d0_fwd real (im2col+gemm)": old_fwd,
    "d0_fwd real (direct, staged store)": lambda: (L.call("mg_set_tuning", 13, 2),
                                                  ops.d0_fwd(x, xs, B, H, H, w0p, bias=bias),
                                                  L.call("mg_set_tuning", 13, 0)),
    "d0_fwd r1 u (direct, staged store)": lambda: (L.call("mg_set_tuning", 13, 2),
                                                  ops.d0_fwd(u, us, B, H, H, w0p, aux=h0),
                                                  L.call("mg_set_tuning", 13, 0)),
    "d0_fwd r1 u (direct)": lambda: ops.d0_fwd(u, us, B, H, H, w0p, aux=h0),
    "d0_fwd r1 u (im2col+gemm)": old_fwd_u,
    "d0_wgrad real (direct)": lambda: ops.d0_wgrad(x, xs, B, H, H, gy, dw),
    "d0_wgrad real (gemm on cols)": lambda: ops.gemm(gy.view(-1, 128), cols, 128, 48, P, a_kc=False, b_kc=False,
                                                      out=dw, ep=ops.E(atomic=1), splits=0),
    "d0_dgrad (direct)": lambda: ops.d0_dgrad(gy, w0p, gx),
    "d0_dgrad (gemm+col2im)": lambda: ops.dgrad_s2_small(gy, w0p, 3, gx),
}
mb = {"d0_fwd real": (B * H * H * 3 * 4 + P * 256) / 1e6, "d0_fwd r1 u": (B * H * H * 8 + 2 * P * 256) / 1e6,
      "d0_wgrad real": (B * H * H * 12 + P * 256) / 1e6, "d0_dgrad": (P * 256 + B * H * H * 16) / 1e6}
for name, fn in cases.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    us_ = s.elapsed_time(e) / REPS * 1e3
    key = name.split(" (")[0]
    print(f"{name:32s} {us_:8.1f} us  {mb[key] / us_:6.2f} TB/s of {mb[key]:.0f} MB algorithmic", flush=True)
