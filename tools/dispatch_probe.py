"""Isolated timing of mg_moe_dispatch at the C2 / C5 shapes (B=256: 16x16 / 8x8 / 4x4 token maps, top-2 of 8 and
top-4 of 32): count + scatter-with-folded-scan (default) vs count / scan / scatter (tuning slot 18 = 1), HIP
events over 50 launches."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"
for E, k, T in ((8, 2, 65536), (8, 2, 16384), (8, 2, 4096), (32, 4, 65536)):
    g = torch.Generator(device=DEV).manual_seed(0)
    topi = torch.rand(T, E, device=DEV, generator=g).topk(k, dim=1).indices.int().contiguous()
    gate = torch.rand(T, k, device=DEV, generator=g)
    res = []
    for three in (1, 0):
        L.call("mg_set_tuning", 18, three)
        for _ in range(3):
            ops.moe_dispatch(topi, gate, E)
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(50):
            ops.moe_dispatch(topi, gate, E)
        e.record()
        torch.cuda.synchronize()
        res.append(s.elapsed_time(e) / 50 * 1e3)
    L.call("mg_set_tuning", 18, 0)
    print(f"dispatch E={E:2d} k={k} T={T:6d}: three kernels {res[0]:6.1f} us  folded scan {res[1]:6.1f} us", flush=True)
