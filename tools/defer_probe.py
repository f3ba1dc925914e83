"""Deferred vs immediate gradient folds on one fp32 TrainStep: per-parameter gradient differences (diagnostic)."""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "moe-gan_cpsc541_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402
from steputil import gpu_step, make_inputs  # noqa: E402


def run(B, R, defer):
    os.environ["MOEGAN_FOLD_DEFER"] = "1" if defer else "0"
    ts = gpu_step(4, None, "fp32", "cuda:0", max_res=R)
    real, text, z, eps_d, eps_g, perm = make_inputs(B, 4, seed=7, res=64 if R == 16 else R)
    cu = lambda t: t.to("cuda:0")  # noqa: E731
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, eff_kl_weight=0.001 * 1e-5)
    torch.cuda.synchronize()
    return ts, {k: out[k].detach().cpu().clone() for k in ("g_grad", "d_grad")}


for B in (2, 4):
    ts, a = run(B, 16, False)
    _, b = run(B, 16, True)
    for key, store in (("d_grad", ts.ds), ("g_grad", ts.gs)):
        ga, gb = a[key], b[key]
        bad = []
        for name, (o, n) in store.offsets.items():
            x, y = ga[o:o + n], gb[o:o + n]
            d = (x - y).abs().max().item()
            if d > 1e-5 * max(x.abs().max().item(), 1e-30):
                bad.append((name, d, x.abs().max().item(), y.abs().max().item()))
        print(f"B={B} {key}: {len(bad)} of {len(store.offsets)} tensors differ", flush=True)
        for t in bad[:40]:
            print("   %-60s diff %.3e |imm| %.3e |def| %.3e" % t, flush=True)
