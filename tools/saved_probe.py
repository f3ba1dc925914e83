"""Saved-activation integrity probe (GPU, fp32): one progressive-stage step (R x R, E=4 dense, B=2); every MTM's
saved forward tensors are copied right after its G-phase forward and compared, bitwise, with their contents when
its backward starts -- a changed tensor means a buffer was reused while still needed."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
from steputil import gpu_step, make_inputs  # noqa: E402


def flat(sv):
    out = []
    for t in sv if isinstance(sv, (tuple, list)) else [sv]:
        if torch.is_tensor(t):
            out.append(t)
        elif isinstance(t, (tuple, list)):
            out += flat(t)
    return out


def main(R=32, B=2):
    E = 4
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=7, res=R)
    ts = gpu_step(E, None, "fp32", max_res=R)
    ge = ts.ge
    f_fwd, f_bwd, c_fwd, c_bwd = ge.mtm_fwd, ge.mtm_bwd, ge.cb_fwd, ge.cb_bwd
    snap = {}
    phase = {"save": False}

    def mtm_fwd(pre, x, w, resid=None, save=True):
        y, sv = f_fwd(pre, x, w, resid=resid, save=save)
        if save:
            torch.cuda.synchronize()
            snap[pre] = [(t, t.detach().clone()) for t in flat(sv)]
        return y, sv

    def mtm_bwd(pre, sv, gz, gx, gw, accumulate=0):
        torch.cuda.synchronize()
        bad = [i for i, (t, c) in enumerate(snap.get(pre, [])) if not torch.equal(t, c)]
        print(f"{pre:36s} saved tensors changed before backward: {bad} of {len(snap.get(pre, []))}", flush=True)
        return f_bwd(pre, sv, gz, gx, gw, accumulate)
    ge.mtm_fwd, ge.mtm_bwd = mtm_fwd, mtm_bwd
    dv = lambda trips: [tuple(t.cuda() for t in trip) for trip in trips]  # noqa: E731
    ts.step(real.cuda(), text.cuda(), z.cuda(), dv(eps_d), dv(eps_g), perm.int().cuda(), anneal=3.0, eff_kl_weight=1e-8)
    torch.cuda.synchronize()


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
