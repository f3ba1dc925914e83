"""The long-reduction weight-gradient kernel and its folds at the C2 shapes, for a rocprofv3 kernel trace (per-kernel
durations: the main kernel vs the two fold passes)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"
for M, N, K in [(128, 128, 65536), (384, 128, 65536), (256, 256, 16384)]:
    A = torch.randn(K, M, device=DEV).bfloat16()
    B = torch.randn(K, N, device=DEV).bfloat16()
    C = torch.zeros(M, N, device=DEV)
    for mode in (2, 1):
        L.call("mg_set_tuning", 15, mode)
        for _ in range(10):
            ops.gemm(A, B, M, N, K, a_kc=False, b_kc=False, out=C, ep=ops.E(atomic=1), splits=0)
        torch.cuda.synchronize()
L.call("mg_set_tuning", 15, 0)
print("ok")
