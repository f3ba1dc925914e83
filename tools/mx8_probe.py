"""Time the MX-fp8 implicit conv against the bf16 one on the generator's 3x3 modulated-conv shapes (B=256).

    python tools/mx8_probe.py            (GPU)
Prints per shape: bf16 conv (mg_conv2d_fwd on the prescaled input) and mg_conv2d_fwd_mx8, microseconds per
launch (HIP events over 20 launches) and TF/s.
"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))
from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

SHAPES = [(256, 4, 512, 512), (256, 8, 512, 256), (256, 8, 256, 256), (256, 16, 256, 128), (256, 16, 128, 128)]


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    dev = "cuda"
    tiles = [int(t) for t in sys.argv[1:]] or [0]
    for B, H, Cin, Cout in SHAPES:
        x = torch.randn(B, H, H, Cin, device=dev).bfloat16()
        wp = (torch.randn(Cout, 9 * Cin, device=dev) / (3 * Cin ** 0.5)).bfloat16()
        wq, wsc = ops.quant_mx8(wp)
        xq, xsc = ops.quant_mx8(x.view(-1, Cin))
        xq = xq.view(B, H, H, Cin)
        y = torch.empty(B, H, H, Cout, device=dev, dtype=torch.bfloat16)
        fl = 2.0 * B * H * H * Cout * 9 * Cin
        t16 = timeit(lambda: ops.conv2d(x, wp, Cout, 3, 3, 1, 1, out=y))
        line = f"B={B} {H}x{H} {Cin}->{Cout}: bf16 {t16:7.1f} us ({fl / t16 / 1e6:6.0f} TF/s)"
        for t in tiles:
            L.call("mg_set_tuning", 2, t)
            t8 = timeit(lambda: ops.conv2d_mx8(xq, xsc, wq, wsc, Cout, 3, 3, 1, 1, out=y))
            line += f" | mx8[{t}] {t8:7.1f} us ({fl / t8 / 1e6:6.0f} TF/s)"
        L.call("mg_set_tuning", 2, 0)
        tq = timeit(lambda: ops.quant_mx8(x.view(-1, Cin)))
        print(line + f" | quant {tq:6.1f} us ({B * H * H * Cin * 3.03 / tq / 1e3:5.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
