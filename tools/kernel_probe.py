"""Run ONE hot kernel in isolation (for rocprofv3 --pmc passes and per-kernel timing).

  python tools/kernel_probe.py d_conv1 [--batch 256] [--iters 20]

d_conv1: the discriminator's conv_layers.2 forward on a 64x64 real batch (implicit GEMM
M = B*16*16, N = 256, K = 4*4*128, bf16) -- the roofline kernel reported by bench.py.
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel", choices=["d_conv1"])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    from moegan_mi import _lib as L
    from moegan_mi import ops
    dev = "cuda"
    B = a.batch
    g = torch.Generator(device=dev).manual_seed(0)
    h0 = torch.randn(B, 32, 32, 128, device=dev, generator=g).to(torch.bfloat16)
    W = torch.randn(256, 128, 4, 4, device=dev, generator=g) / 45.0
    bias = torch.randn(256, device=dev, generator=g)
    wp = ops.pack_conv(W, torch.bfloat16)
    out = torch.empty(B, 16, 16, 256, device=dev, dtype=torch.bfloat16)
    ep = ops.E(bias=bias, act=L.ACT_LRELU)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.iters)]
    for s, e in ev:
        s.record()
        ops.conv2d(h0, wp, 256, 4, 4, 2, 1, out=out, ep=ep)
        e.record()
    torch.cuda.synchronize()
    ms = sorted(s.elapsed_time(e) for s, e in ev)
    flop = 2.0 * B * 256 * 256 * 2048
    med = ms[len(ms) // 2]
    print(f"d_conv1 B={B}: median {med * 1e3:.1f} us, {flop / med / 1e9:.1f} TFLOP/s, grid {B * 256 // 128 * 2} blocks")


if __name__ == "__main__":
    main()
