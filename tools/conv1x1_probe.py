"""Isolated timing of the step's 1x1 convs (the skip projections at 16x16 / 8x8, B=256) under each conv tile
override (tuning slot 2: 0 automatic, 64, 128, 256, 257), HIP events over 20 launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV, bf = "cuda", torch.bfloat16
for S, Cin, Cout in ((16, 128, 128), (16, 256, 128), (8, 256, 256), (8, 512, 256), (16, 128, 256)):
    g = torch.Generator(device=DEV).manual_seed(0)
    x = torch.randn(256, S, S, Cin, device=DEV, generator=g).to(bf)
    wp = ops.pack_conv(torch.randn(Cout, Cin, 1, 1, device=DEV, generator=g) * Cin ** -0.5, bf)
    res = []
    for tile in (0, 64, 128, 256, 257):
        L.call("mg_set_tuning", 2, tile)
        fn = lambda: ops.conv2d(x, wp, Cout, 1, 1, 1, 0, out_dtype=bf)  # noqa: E731
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
    mb = 256 * S * S * (Cin + Cout) * 2 / 1e6
    print(f"1x1 {S}x{S} {Cin}->{Cout}: " + "  ".join(f"{t}:{r:6.1f}" for t, r in zip(("auto", 64, 128, 256, 257), res))
          + f" us ({mb:.0f} MB: {mb / min(res):.2f} TB/s best)", flush=True)
