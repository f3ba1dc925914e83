"""Median time of the R1 image-gradient launch (4x4/s2 data gradient to 3 channels, B=256, bf16)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))
import torch  # noqa: E402
from moegan_mi import ops  # noqa: E402

g = torch.Generator(device="cuda").manual_seed(0)
B = 256
W = torch.randn(128, 3, 4, 4, device="cuda", generator=g) / 7
gA0 = torch.randn(B, 32, 32, 128, device="cuda", generator=g).bfloat16()
wcls = ops.pack_dgrad_s2(W, torch.bfloat16, rows=3)
out = torch.zeros(B, 64, 64, 4, device="cuda")
for _ in range(3):
    ops.dgrad_s2(gA0, wcls, 3, out)
ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(20)]
for s, e in ev:
    s.record()
    ops.dgrad_s2(gA0, wcls, 3, out)
    e.record()
torch.cuda.synchronize()
ms = sorted(s.elapsed_time(e) for s, e in ev)
print("r1 image dgrad: median %.1f us" % (ms[len(ms) // 2] * 1e3))
