"""Device-vs-device sensitivity of the bf16 C2 step's gradients at B=8: the same step from the same state twice,
once with the offset heads' forward on the direct kernel and once on the implicit GEMM (whose bf16 outputs differ
by one rounding in ~0.02 % of elements), per-tensor relative difference of the clipped gradients (largest first)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from steputil import gpu_step, make_inputs  # noqa: E402

B, E = 8, 8
real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=100 + B)
cu = lambda t: t.to("cuda")  # noqa: E731
grads = []
for mode in (0, 2):
    L.call("mg_set_tuning", 16, mode)
    ts = gpu_step(E, 2, "bf16", "cuda")
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=0.001 * 1e-5)
    torch.cuda.synchronize()
    grads.append((out["g_grad"].clone(), ts.gs.offsets))
L.call("mg_set_tuning", 16, 0)
(g0, offs), (g1, _) = grads
rows = []
for n, (off, numel) in offs.items():
    a, b = g0[off:off + numel].double(), g1[off:off + numel].double()
    nb = float(b.norm())
    if nb > 0:
        rows.append((float((a - b).norm()) / nb, n, numel))
rows.sort(reverse=True)
for r, n, numel in rows[:12]:
    print(f"{r:.3e}  {n} ({numel})", flush=True)
print(f"median {rows[len(rows) // 2][0]:.3e} over {len(rows)} tensors", flush=True)
