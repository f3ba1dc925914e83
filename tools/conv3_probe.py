"""Isolated timing of the step's 3x3 convs (modulated convs and their data gradients at B=256: 16x16 / 8x8 / 4x4
maps) under each conv tile override (tuning slot 2: 0 automatic, 64, 128, 256 = 256x128, 257 = 128x256), HIP events
over 20 launches, as TFLOP/s."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV, bf = "cuda", torch.bfloat16
SHAPES = [(16, 256, 128), (16, 128, 256), (16, 128, 128), (8, 512, 256), (8, 256, 512), (8, 256, 256),
          (4, 512, 512)]
for S, Cin, Cout in SHAPES:
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(256, S, S, Cin, device=DEV, generator=g).to(bf)
    wp = ops.pack_conv(torch.randn(Cout, Cin, 3, 3, device=DEV, generator=g) * (9 * Cin) ** -0.5, bf)
    res = []
    for tile in (0, 64, 128, 256, 257):
        L.call("mg_set_tuning", 2, tile)
        fn = lambda: ops.conv2d(x, wp, Cout, 3, 3, 1, 1, out_dtype=bf)  # noqa: E731
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            fn()
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / 20 * 1e3)
    L.call("mg_set_tuning", 2, 0)
    gf = 2.0 * 256 * S * S * Cout * 9 * Cin / 1e9
    print(f"3x3 {S:2d}x{S:<2d} {Cin:3d}->{Cout:3d}: " + "  ".join(f"{t}:{r:6.1f}" for t, r in
                                                              zip(("auto", 64, 128, 256, 257), res))
          + f" us  (best {gf / min(res) * 1e3:.0f} TF/s)", flush=True)
