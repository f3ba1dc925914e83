"""Per-MTM gradient probe (GPU, fp32): one full G+D step at R x R (progressive stage, E=4 dense, B=2) on the
device and on the fp64 oracle; for every MTM with an offset head, the relative error of the gradient reaching
the warped input (g_xw = dL/d grid_sample output) and of the offset head's first-layer pre-activation gradient
(ga1), to locate where the device's offset-net gradient error enters."""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
from oracle import aurora_cpu as O  # noqa: E402
from steputil import gpu_step, make_inputs, oracle_models  # noqa: E402


def main(R=32, B=2):
    from moegan_mi import ops
    torch.set_num_threads(8)
    E = 4
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=7, res=R)
    ref = {}

    def mtm(x, w, P, pre, use_offset=True):
        if not use_offset or not torch.is_grad_enabled():
            return orig_mtm(x, w, P, pre, use_offset)
        Bq, C, H, W = x.shape
        o_pre = F.conv2d(x, P[pre + "offset_net.0.weight"], P[pre + "offset_net.0.bias"], padding=1)
        o_pre.retain_grad()
        o = F.leaky_relu(o_pre, 0.2)
        o = F.conv2d(o, P[pre + "offset_net.2.weight"], P[pre + "offset_net.2.bias"], padding=1)
        o.retain_grad()
        grid = (O.base_grid(H, W, dtype=x.dtype).unsqueeze(0) + o.permute(0, 2, 3, 1) * 0.05).clamp(-1, 1)
        xw = F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=False)
        xw.retain_grad()
        ref[pre] = dict(o_pre=o_pre, o=o, xw=xw)
        y = O.modconv(xw, w, P, pre + "modulated_conv.", padding=1)
        return F.leaky_relu(y, 0.2)
    orig_mtm = O.mtm
    O.mtm = mtm
    PG, PD, optG, optD, grads = oracle_models(E, max_res=R, dtype=torch.float64)
    d64 = lambda trips: [tuple(t.double() for t in trip) for trip in trips]  # noqa: E731
    O.train_step(PG, PD, optG, optD, real.double(), text.double(), z.double(), d64(eps_d), d64(eps_g), perm,
                 kl_weight_eff=1e-8)
    O.mtm = orig_mtm
    dev = []
    orig = ops.mtm_bwd_fused

    def fused(g_xw, x, samp, o1, w2, gx, ga1, gw2, gb2, accumulate):
        r = orig(g_xw, x, samp, o1, w2, gx, ga1, gw2, gb2, accumulate)
        torch.cuda.synchronize()
        dev.append(dict(shape=tuple(x.shape), g_xw=g_xw.detach().float().cpu().clone(),
                        ga1=ga1.detach().float().cpu().clone(), samp=samp.detach().cpu().clone()))
        return r
    ops.mtm_bwd_fused = fused
    ts = gpu_step(E, None, "fp32", max_res=R)
    dv = lambda trips: [tuple(t.cuda() for t in trip) for trip in trips]  # noqa: E731
    ts.step(real.cuda(), text.cuda(), z.cuda(), dv(eps_d), dv(eps_g), perm.int().cuda(), anneal=3.0, eff_kl_weight=1e-8)
    torch.cuda.synchronize()
    ops.mtm_bwd_fused = orig
    # the device's backward visits the MTMs from the last block to the first, mtm2 before mtm1
    order = []
    for name in ("gen_block_16", "gen_block_8", "gen_block_4"):
        order += [f"{name}.conv_block.mtm2.", f"{name}.conv_block.mtm1."]
    rel = lambda a, b: float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-300))  # noqa
    for pre, d in zip(order, dev):
        r = ref[pre]
        Bq, H, W, C = d["shape"]
        g_xw_ref = r["xw"].grad.permute(0, 2, 3, 1).reshape(-1, C)
        ga1_ref = r["o_pre"].grad.permute(0, 2, 3, 1)
        print(f"{pre:32s} {d['shape']}: g_xw rel err {rel(d['g_xw'].reshape(-1, C), g_xw_ref):.2e}, "
              f"ga1 rel err {rel(d['ga1'].reshape(ga1_ref.shape), ga1_ref):.2e}, "
              f"|offsets| max {float(r['o'].detach().abs().max()):.3e}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
