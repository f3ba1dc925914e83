"""Generator-only gradient probe (GPU, fp32): the upstream image gradient of a real progressive-stage step
(R x R, E=4 dense, B=2; dL/dimage from the fp64 oracle's G phase) is fed to the device generator's backward and to
the fp64 oracle generator; per MTM with an offset head, the relative error of the gradient at the warped input
(g_xw).  Separates the generator backward from the discriminator / loss path."""
import os
import sys

import torch
import torch.nn.functional as F

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
from oracle import aurora_cpu as O  # noqa: E402
from oracle.recipe import fill_state  # noqa: E402
from steputil import make_inputs, oracle_models  # noqa: E402


def main(R=32, B=2):
    from moegan_mi import ops
    from moegan_mi.engine_g import GeneratorEngine
    from moegan_mi.layout import frozen_rgb_prefixes, generator_shapes
    from moegan_mi.params import ParamStore
    torch.set_num_threads(8)
    E = 4
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=7, res=R)
    # 1. the real step's image gradient (G phase), fp64 oracle
    cap = {}
    o_gen = O.generator

    def gen(*a, **k):
        out = o_gen(*a, **k)
        if torch.is_grad_enabled():
            out[0].retain_grad()
            cap["img"] = out[0]
        return out
    O.generator = gen
    PG, PD, optG, optD, _ = oracle_models(E, max_res=R, dtype=torch.float64)
    d64 = lambda trips: [tuple(t.double() for t in trip) for trip in trips]  # noqa: E731
    O.train_step(PG, PD, optG, optD, real.double(), text.double(), z.double(), d64(eps_d), d64(eps_g), perm,
                 kl_weight_eff=1e-8, step_optim=False)
    O.generator = o_gen
    G_img = cap["img"].grad.detach()
    print(f"|dL/dimg| = {float(G_img.norm()):.3e}")
    # 2. oracle generator alone with that upstream gradient
    vals = fill_state(generator_shapes(E, R), 0)
    P = {n: torch.from_numpy(v).double().requires_grad_(not n.split(".")[-1].startswith("epsilon_"))
         for n, v in vals.items()}
    ref = {}
    o_mtm = O.mtm

    def mtm(x, w, P_, pre, use_offset=True):
        if not use_offset:
            return o_mtm(x, w, P_, pre, use_offset)
        Bq, C, H, W = x.shape
        o = F.leaky_relu(F.conv2d(x, P_[pre + "offset_net.0.weight"], P_[pre + "offset_net.0.bias"], padding=1), 0.2)
        o = F.conv2d(o, P_[pre + "offset_net.2.weight"], P_[pre + "offset_net.2.bias"], padding=1)
        grid = (O.base_grid(H, W, dtype=x.dtype).unsqueeze(0) + o.permute(0, 2, 3, 1) * 0.05).clamp(-1, 1)
        xw = F.grid_sample(x, grid, mode="bilinear", padding_mode="zeros", align_corners=False)
        xw.retain_grad()
        ref[pre] = xw
        y = O.modconv(xw, w, P_, pre + "modulated_conv.", padding=1)
        y.retain_grad()
        out = F.leaky_relu(y, 0.2)
        out.retain_grad()
        ref[pre + "y"] = y
        ref[pre + "out"] = out
        return out
    O.mtm = mtm
    img, _, kl, probs = O.generator(z.double(), text.double(), P, d64(eps_g), True, 3.0, 0.7)
    (img * G_img).sum().backward()
    O.mtm = o_mtm
    # 3. device generator, same upstream gradient
    st = ParamStore(generator_shapes(E, R), "cuda", frozen_prefixes=frozen_rgb_prefixes(R))
    st.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    ge = GeneratorEngine(st, E)
    ge.prep()
    dev = []
    last = {}
    orig = ops.mtm_bwd_fused
    orig_bo = ops.modconv_bwd_out

    def bo(gz, z, d, Bn, HW, rows, act, gyt, gdd, zsub=None):
        r = orig_bo(gz, z, d, Bn, HW, rows, act, gyt, gdd, zsub=zsub)
        last.update(gz=gz.detach().float().cpu().clone(), z=z.detach().float().cpu().clone(), act=act,
                    d=d.detach().float().cpu().clone(), gyt=gyt.detach().float().cpu().clone(), rows=rows,
                    zsub=None if zsub is None else zsub.detach().float().cpu().clone())
        return r
    ops.modconv_bwd_out = bo

    def fused(g_xw, x, *a, **k):
        dev.append((tuple(x.shape), g_xw.detach().float().cpu().clone(), dict(last)))
        return orig(g_xw, x, *a, **k)
    ops.mtm_bwd_fused = fused
    im, _, _, _, _, ctx = ge.forward(z.cuda(), text.cuda(), [tuple(t.cuda() for t in e) for e in eps_g], 3.0, 0.7,
                                     train=True, save=True)
    gpad = torch.zeros(B, R, R, 8, device="cuda")
    gpad[..., :3] = G_img.permute(0, 2, 3, 1).float().cuda()
    ge.backward(ctx, gpad)
    torch.cuda.synchronize()
    ops.mtm_bwd_fused = orig
    ops.modconv_bwd_out = orig_bo
    order = []
    for name in ("gen_block_16", "gen_block_8", "gen_block_4"):
        order += [f"{name}.conv_block.mtm2.", f"{name}.conv_block.mtm1."]
    rel = lambda a, b: float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-300))  # noqa
    print(f"image rel err {rel(im[..., :3].permute(0, 3, 1, 2).cpu(), img.detach()):.2e}")
    for pre, (shape, g, L) in zip(order, dev):
        C = shape[-1]
        r = ref[pre].grad.permute(0, 2, 3, 1).reshape(-1, C)
        Co = ref[pre + "y"].shape[1]
        nhwc = lambda t: t.detach().permute(0, 2, 3, 1).reshape(-1, Co)  # noqa: E731
        gz, z = L["gz"][:, :Co], L["z"][:, :Co]
        line = (f"{pre:32s} g_xw {rel(g.reshape(-1, C), r):.2e} | act {L['act']} zsub {L['zsub'] is not None} "
                f"g_out {rel(gz, nhwc(ref[pre + 'out'].grad)):.2e}")
        if L["act"] == 2:
            line += f" ypre {rel(z, nhwc(ref[pre + 'y'])):.2e}"
            flips = int(((z > 0) != (nhwc(ref[pre + 'y']) > 0)).sum())
            line += f" sign flips {flips}/{z.numel()}"
        else:
            line += f" z(out) {rel(z, nhwc(ref[pre + 'out'])):.2e}"
        HW = shape[1] * shape[2]
        dd = L["d"][:, :Co].repeat_interleave(HW, 0)
        line += f" g_ypre {rel(L['gyt'][:, :Co] / dd, nhwc(ref[pre + 'y'].grad)):.2e}"
        print(line)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
