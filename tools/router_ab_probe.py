"""A/B of the router kernel forms (tuning slot 24: 0 MFMA / team forms, 7 lane-FMA forms) on one MX-fp8 C5 test step
(E = 32 top-4, B = 4, the inputs of tests/test_step_fp8_gpu.py): routing, probabilities and per-tensor gradient
differences between the two forms.  Diagnostic only."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "moe-gan_cpsc541_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from steputil import gpu_step, make_inputs  # noqa: E402
from moegan_mi import _lib as L  # noqa: E402

E, topk, B = 32, 4, 4
real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=300 + E)
cu = lambda t: t.to("cuda")  # noqa: E731


def run(slot):
    L.call("mg_set_tuning", 24, slot)
    ts = gpu_step(E, topk, "bf16", "cuda", fp8=True)
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=0.001 * 1e-5)
    torch.cuda.synchronize()
    L.call("mg_set_tuning", 24, 0)
    return ts, {k: ([t.detach().cpu().clone() for t in v] if isinstance(v, (list, tuple)) else
                    v.detach().cpu().clone() if torch.is_tensor(v) else v) for k, v in out.items()}


ts, a = run(0)
_, b = run(7)
for key in ("topi_d", "topi"):
    for li, (x, y) in enumerate(zip(a[key], b[key])):
        diff = int((x.sort(1).values != y.sort(1).values).any(1).sum())
        print(f"{key} layer{li}: {diff} of {x.shape[0]} tokens route differently", flush=True)
for key in ("probs_d", "probs"):
    if key in a:
        for li, (x, y) in enumerate(zip(a[key], b[key])):
            print(f"{key} layer{li}: max |dp| {float((x - y).abs().max()):.3e}", flush=True)
ga, gb = a["g_grad"], b["g_grad"]
rows = []
for n, (off, numel) in ts.gs.offsets.items():
    x, y = ga[off:off + numel].double(), gb[off:off + numel].double()
    d = float((x - y).norm() / max(float(y.norm()), 1e-30))
    rows.append((d, n))
rows.sort(reverse=True)
print("largest per-tensor G gradient differences (relative L2):", flush=True)
for d, n in rows[:12]:
    print(f"  {d:.3e} {n}", flush=True)
