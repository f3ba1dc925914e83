"""Attention-block gradient probe (GPU, fp32): one full G+D step (progressive stage R, E=4 dense, B=2) on the device
and the fp64 oracle; per attention block, the relative error of the gradient at its output, at the MoE output
(resid + experts), at the router/expert tokens (LN3 output), and at the block input -- to locate where the device's
fp32 error enters."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
from oracle import aurora_cpu as O  # noqa: E402
from steputil import gpu_step, make_inputs, oracle_models  # noqa: E402


def main(R=32, B=2):
    torch.set_num_threads(8)
    E = 4
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=7, res=R)
    ref = {}
    o_attn, o_moe, o_mha, o_ln = O.attention_block, O.sparse_moe, O.mha, O.F.layer_norm

    def attention_block(x, w, text_seq, P, pre, *a, **k):
        if not torch.is_grad_enabled():
            return o_attn(x, w, text_seq, P, pre, *a, **k)
        x.retain_grad()
        y, kl, probs = o_attn(x, w, text_seq, P, pre, *a, **k)
        y.retain_grad()
        ref[pre + "in"], ref[pre + "out"] = x, y
        return y, kl, probs

    def sparse_moe(x, w, P, pre, *a, **k):
        if torch.is_grad_enabled():
            x.retain_grad()
            ref[pre + "tok"] = x
        y, kl, probs = o_moe(x, w, P, pre, *a, **k)
        if torch.is_grad_enabled():
            y.retain_grad()
            ref[pre + "moe_out"] = y
        return y, kl, probs
    O.attention_block, O.sparse_moe = attention_block, sparse_moe
    PG, PD, optG, optD, grads = oracle_models(E, max_res=R, dtype=torch.float64)
    d64 = lambda trips: [tuple(t.double() for t in trip) for trip in trips]  # noqa: E731
    O.train_step(PG, PD, optG, optD, real.double(), text.double(), z.double(), d64(eps_d), d64(eps_g), perm,
                 kl_weight_eff=1e-8)
    O.attention_block, O.sparse_moe = o_attn, o_moe
    dev = {}
    ts = gpu_step(E, None, "fp32", max_res=R)
    ge = ts.ge
    a_bwd, m_bwd = ge.attn_bwd, ge.moe_bwd

    def attn_bwd(pre, sv, g_out, gx, *a, **k):
        dev[pre + "out"] = g_out.detach().float().cpu().clone()
        r = a_bwd(pre, sv, g_out, gx, *a, **k)
        torch.cuda.synchronize()
        dev[pre + "in"] = gx.detach().float().cpu().clone()
        return r

    def moe_bwd(pre, sv, g_out, g_tok, *a, **k):
        dev[pre + "moe_out"] = g_out.detach().float().cpu().clone()
        r = m_bwd(pre, sv, g_out, g_tok, *a, **k)
        torch.cuda.synchronize()
        dev[pre + "tok"] = g_tok.detach().float().cpu().clone()
        return r
    ge.attn_bwd, ge.moe_bwd = attn_bwd, moe_bwd
    dv = lambda trips: [tuple(t.cuda() for t in trip) for trip in trips]  # noqa: E731
    ts.step(real.cuda(), text.cuda(), z.cuda(), dv(eps_d), dv(eps_g), perm.int().cuda(), anneal=3.0, eff_kl_weight=1e-8)
    torch.cuda.synchronize()
    rel = lambda a, b: float((a.double() - b.double()).norm() / max(float(b.double().norm()), 1e-300))  # noqa
    for name in ("gen_block_16", "gen_block_8", "gen_block_4"):
        pre = name + ".attn_block."
        line = [f"{pre}"]
        for key, mpre in (("out", pre), ("moe_out", pre + "moe."), ("tok", pre + "moe."), ("in", pre)):
            r = ref[mpre + key].grad
            d = dev.get(pre + key if key in ("out", "in") else pre + "moe." + key)
            if d is None:
                continue
            C = r.shape[1]
            rr = r.permute(0, 2, 3, 1).reshape(-1, C)
            line.append(f"{key}: {rel(d.reshape(-1, C), rr):.2e}")
        print("  ".join(line), flush=True)


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 32)
