"""Isolated timing of the MTM offset-head convolutions at the C2 shapes (B=256; 16x16 / 8x8 / 4x4 maps): the direct
halo-tile kernels (csrc/mg_narrow.hip) against the implicit-GEMM path (tuning slot 16 = 1), HIP events over 20
launches, with the algorithmic HBM bytes of each call (activation read once, 32-channel side, output)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV, bf = "cuda", torch.bfloat16
B = int(os.environ.get("B", "256"))
SHAPES = [(16, 256), (16, 128), (8, 512), (8, 256), (4, 512)]
BLOCKS = [int(b) for b in os.environ.get("BLOCKS", "").split()]


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for S, C in SHAPES:
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(B, S, S, C, device=DEV, generator=g).to(bf)
    ga = torch.randn(B, S, S, 32, device=DEV, generator=g).to(bf)
    W = torch.randn(32, C, 3, 3, device=DEV, generator=g) * (9 * C) ** -0.5
    bias = torch.zeros(32, device=DEV)
    wp, wf = ops.pack_conv(W, bf), ops.pack_conv(W, bf, flip=True)
    gx = torch.zeros(B, S, S, C, device=DEV, dtype=bf)
    gw = torch.zeros(32, C, 3, 3, device=DEV)
    ep = ops.E(bias=bias, act=L.ACT_LRELU)
    P = B * S * S
    cases = {
        "fwd": (lambda: ops.conv2d(x, wp, 32, 3, 3, 1, 1, out_dtype=bf, ep=ep), P * (C + 32) * 2),
        "dgrad": (lambda: ops.conv2d(ga, wf, C, 3, 3, 1, 1, out=gx, ep=ops.E(accumulate=1)), P * (32 + 2 * C) * 2),
        "wgrad": (lambda: ops.conv2d_wgrad(ga, x, 32, 3, 3, 1, 1, gw), P * (C + 32) * 2),
    }
    for name, (fn, nbytes) in cases.items():
        L.call("mg_set_tuning", 16, 1)
        t_old = timed(fn)
        L.call("mg_set_tuning", 16, 0)
        t_new = timed(fn)
        alt = []
        for blocks in BLOCKS:  # grid-target sweep (tuning slot 17)
            L.call("mg_set_tuning", 17, blocks)
            alt.append(timed(fn))
        L.call("mg_set_tuning", 17, 0)
        sweep = "  ".join(f"{b}:{t:5.1f}" for b, t in zip(BLOCKS, alt))
        if name == "fwd":  # 256-pixel tiles (tuning slot 19 = 4)
            L.call("mg_set_tuning", 19, 4)
            sweep += f"  256px: {timed(fn):5.1f}"
            L.call("mg_set_tuning", 19, 0)
        print(f"{S:2d}x{S:<2d} C={C:3d} {name:5s} generic {t_old:6.1f} us  direct {t_new:6.1f} us  "
              f"({nbytes / 1e6:5.1f} MB: {nbytes / t_new / 1e6:.2f} TB/s)  {sweep}", flush=True)
