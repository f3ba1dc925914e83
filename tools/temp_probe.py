"""Router-temperature gradient diagnostic (GPU): where does the bf16 step's error on the scalar
``...router.temperature`` gradient come from?

One bf16 C2-configuration step (E=8 top-2, B=4, the inputs of tests/test_step_bf16_gpu.py) on the device and the
same step on the fp32 oracle (device top-k replayed), plus the oracle's whole-step bf16 floor run.  Per MoE block
it prints the G-phase temperature gradient (t2i_moe_gan.py:374-377: logits / clamp(temperature * anneal, .5, 5))
as the sum over tokens of  -anneal / te * sum_e dL/dl[t, e] * l[t, e]  and
  * the device kernel's own value (k_router_bwd) and its fp64 host restatement from the kernel's inputs,
  * the oracle's and the floor run's value,
  * the host restatement with ONE device input swapped for the oracle's (gate gradient, logits),
so the error can be attributed to an input.

    python tools/temp_probe.py [--batch 4] [--seed 104]
"""
import argparse
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "moe-gan_cpsc541_amd"))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "tests"))

from oracle import aurora_cpu as O  # noqa: E402
from steputil import bf16_module_rounding, gpu_step, make_inputs, oracle_clone, oracle_models  # noqa: E402

BLOCK_OF_HW = {16: "gen_block_4", 64: "gen_block_8", 256: "gen_block_16"}


def host_terms(z, topi, g_gate, coef, te, anneal, k):
    """fp64 restatement of k_router_bwd's temperature term per token (softmax recomputed from the scaled logits z)."""
    z = z.double()
    T, E = z.shape
    l = z.clamp(-20, 20)
    s = torch.softmax(l, dim=1)
    q = s.clamp(1e-6, 1.0)
    Sq = q.sum(1, keepdim=True)
    p = q / Sq
    gp = torch.zeros(T, E, dtype=torch.float64)
    if coef is not None:
        gp += coef.double().view(1, E)
    ti = topi.long()
    gg = g_gate.double()
    if k == E:
        gp.scatter_add_(1, ti, gg)
    else:
        psel = p.gather(1, ti)
        S = psel.sum(1, keepdim=True)
        gate = psel / S
        dot = (gg * gate).sum(1, keepdim=True)
        gp.scatter_add_(1, ti, (gg - dot) / S)
    d1 = (gp * (q / Sq)).sum(1, keepdim=True)
    gq = (gp - d1) / Sq
    gs = torch.where((s >= 1e-6) & (s <= 1.0), gq, torch.zeros_like(gq))
    d2 = (gs * s).sum(1, keepdim=True)
    gl = s * (gs - d2)
    gl = torch.where((z >= -20) & (z <= 20), gl, torch.zeros_like(gl))
    return -(gl * z).sum(1) / te * anneal, gl


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--seed", type=int, default=None)
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    a = ap.parse_args()
    from moegan_mi import ops
    B, E, k = a.batch, a.experts, a.topk
    seed = a.seed if a.seed is not None else 100 + B
    dev = "cuda"
    torch.set_num_threads(8)

    rec_dev = {}
    orig_rb = ops.router_bwd

    def rb(probs, zlog, topi, gate, g_gate, g_probs, coef, HW, temperature, anneal, g_temp, Bn, g_logits=None):
        before = g_temp.detach().clone()
        r = orig_rb(probs, zlog, topi, gate, g_gate, g_probs, coef, HW, temperature, anneal, g_temp, Bn, g_logits)
        torch.cuda.synchronize()
        rec_dev[BLOCK_OF_HW[HW]] = dict(
            zlog=zlog.detach().cpu().clone(), topi=topi.detach().cpu().clone(),
            g_gate=g_gate.detach().float().cpu().clone(), coef=None if coef is None else coef.detach().cpu().clone(),
            temp=float(temperature.detach().cpu()[0]), anneal=anneal, dgt=float((g_temp.detach() - before).cpu()[0]),
            g_raw=r[0].detach().cpu().clone())
        return r
    ops.router_bwd = rb

    def hooks(store):
        orig_router, orig_topk = O.router, O.topk_route
        cur = {}

        def router(feature, text, P, pre, eps=None, training=True, anneal=1.0):
            probs, logits = orig_router(feature, text, P, pre, eps, training, anneal)
            return probs, logits

        def router_ret(feature, text, P, pre, eps=None, training=True, anneal=1.0):
            wf = O.reparam(P[pre + "feature_mu"], P[pre + "feature_rho"], eps[0])
            wt = O.reparam(P[pre + "text_mu"], P[pre + "text_rho"], eps[1])
            wc = O.reparam(P[pre + "combined_mu"], P[pre + "combined_rho"], eps[2])
            raw = torch.cat([feature @ wf, text @ wt], dim=1) @ wc
            t_eff = (P[pre + "temperature"] * anneal).clamp(0.5, 5.0)
            logits = (raw / t_eff).clamp(-20.0, 20.0)
            if logits.requires_grad:
                logits.retain_grad()
                cur["pre"] = pre
                store[pre] = dict(logits=logits, t_eff=float(t_eff), anneal=anneal)
            probs = torch.softmax(logits, dim=1).clamp(1e-6, 1.0)
            probs = probs / probs.sum(dim=1, keepdim=True)
            return probs, logits

        def topk_route(probs, kk, idx=None):
            g = orig_topk(probs, kk, idx)
            if g.requires_grad and "pre" in cur:
                g.retain_grad()
                store[cur.pop("pre")]["gate"] = g
            return g
        O.router, O.topk_route = router_ret, topk_route
        return lambda: (setattr(O, "router", orig_router), setattr(O, "topk_route", orig_topk))

    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=seed)
    ts = gpu_step(E, k, "bf16", dev)
    cu = lambda t: t.to(dev)  # noqa: E731
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)
    torch.cuda.synchronize()
    routes_d = [t.cpu().long() for t in out["topi_d"]]
    routes_g = [t.cpu().long() for t in out["topi"]]
    d_after = {n: ts.ds.view(n).detach().cpu().clone() for n in ts.ds.offsets}

    def use_device_d(P):
        with torch.no_grad():
            for n, t in P.items():
                t.copy_(d_after[n].view(t.shape))
    g_dev = {n: float(ts.gs.gview(n).detach().cpu()[0]) for n in ts.gs.offsets if n.endswith("router.temperature")}

    PG, PD, optG, optD, rgrads = oracle_models(E)
    runs = {}
    for tag in ("floorW", "floorD", "ref"):
        P2 = oracle_clone(PG, PD, optG, optD)
        store = {}
        undo = hooks(store)
        try:
            kw = dict(topk=k, kl_weight_eff=1e-8, routes_d=routes_d, routes_g=routes_g, after_d_step=use_device_d)
            if tag == "floorW":
                with bf16_module_rounding():
                    O.train_step(*P2[:4], real, text, z, eps_d, eps_g, perm.long(), d_round=O.round_bf16_st, **kw)
            elif tag == "floorD":
                O.train_step(*P2[:4], real, text, z, eps_d, eps_g, perm.long(), d_round=O.round_bf16_st, **kw)
            else:
                O.train_step(*P2[:4], real, text, z, eps_d, eps_g, perm.long(), **kw)
        finally:
            undo()
        runs[tag] = (store, {n: (None if t.grad is None else float(t.grad.reshape(-1)[0]))
                             for n, t in P2[0].items() if n.endswith("router.temperature")})

    for blk in ("gen_block_16", "gen_block_8", "gen_block_4"):
        pre = blk + ".attn_block.moe.router."
        d = rec_dev[blk]
        te = min(max(d["temp"] * d["anneal"], 0.5), 5.0)
        t_dev, gl_dev = host_terms(d["zlog"], d["topi"], d["g_gate"], d["coef"], te, d["anneal"], k)
        line = [f"{blk}: device kernel {d['dgt']:+.4e} (param grad {g_dev[pre + 'temperature']:+.4e}), "
                f"host restatement {float(t_dev.sum()):+.4e}"]
        for tag in ("ref", "floorD", "floorW"):
            st, tg = runs[tag]
            s = st[pre]
            lg, gr = s["logits"].detach().double(), s["logits"].grad.double()
            terms = -(gr * lg).sum(1) / s["t_eff"] * s["anneal"]
            line.append(f"  {tag}: autograd (clipped) {tg[pre + 'temperature']:+.4e}, per-token sum {float(terms.sum()):+.4e}")
            if tag == "ref":
                t_ref, gl_ref, z_ref = terms, gr, lg
                gate_grad = s["gate"].grad.double() if "gate" in s else None
        ti = d["topi"].long()
        gg_ref = gate_grad.gather(1, ti) if gate_grad is not None else None
        rel = lambda a, b: float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-30))  # noqa
        line.append(f"  per-token terms: device vs ref rel L2 {rel(t_dev, t_ref):.3e}; "
                    f"sum |ref term| {float(t_ref.abs().sum()):.4e}")
        line.append(f"  dL/dlogits: rel L2 {rel(gl_dev, gl_ref):.3e}; logits rel L2 {rel(d['zlog'], z_ref):.3e}")
        if gg_ref is not None:
            line.append(f"  gate gradient: rel L2 {rel(d['g_gate'], gg_ref):.3e}")
            sw_g, _ = host_terms(d["zlog"], d["topi"], gg_ref, d["coef"], te, d["anneal"], k)
            line.append(f"  swap gate gradient -> ref: {float(sw_g.sum()):+.4e}")
            sw_z, _ = host_terms(z_ref, d["topi"], d["g_gate"], d["coef"], te, d["anneal"], k)
            line.append(f"  swap logits -> ref: {float(sw_z.sum()):+.4e}")
            sw_b, _ = host_terms(z_ref, d["topi"], gg_ref, d["coef"], te, d["anneal"], k)
            line.append(f"  swap both -> ref (device coef only): {float(sw_b.sum()):+.4e}")
        print("\n".join(line), flush=True)


if __name__ == "__main__":
    main()
