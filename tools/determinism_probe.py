"""Run-to-run reproducibility probe (GPU diagnostic): two identically initialised C2 steps on identical inputs,
then a per-tensor bitwise comparison of the gradients and of the step's scalar outputs.

    python tools/determinism_probe.py [--batch 256] [--tune "10=1"]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "moe-gan_cpsc541_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    ap.add_argument("--tune", default="")
    a = ap.parse_args()
    from moegan_mi import _lib as L
    from moegan_mi.init import init_discriminator, init_generator
    from moegan_mi.step import StepConfig, TrainStep
    import bench
    for kv in filter(None, a.tune.split(",")):
        k_, v_ = kv.split("=")
        L.call("mg_set_tuning", int(k_), int(v_))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    E, k, B = a.experts, a.topk, a.batch
    g = torch.Generator(device=dev).manual_seed(7)
    real = torch.rand(B, 3, 64, 64, device=dev, generator=g) * 2 - 1
    text = torch.randn(B, 512, device=dev, generator=g)
    z = torch.randn(B, 512, device=dev, generator=g)
    fd, eps_d = bench.eps_buffers(E, dev)
    fg, eps_g = bench.eps_buffers(E, dev)
    fd.normal_(generator=g)
    fg.normal_(generator=g)
    perm = torch.randperm(B, device=dev, generator=g).int()
    runs = []
    for _ in range(2):
        ts = TrainStep(StepConfig(E=E, topk=k, dtype="bf16"), dev)
        init_generator(ts.gs, seed=0)
        init_discriminator(ts.ds, seed=1)
        out = ts.step(real, text, z, eps_d, eps_g, perm, anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)
        torch.cuda.synchronize()
        scal = {n: v.detach().float().cpu().clone() for n, v in out.items() if torch.is_tensor(v) and v.numel() <= 64}
        grads = {}
        for tag, st in (("G", ts.gs), ("D", ts.ds)):
            for n in st.offsets:
                grads[f"{tag}:{n}"] = st.gview(n).detach().cpu().clone()
        runs.append((scal, grads))
        del ts
    (s0, g0), (s1, g1) = runs
    bad_s = [n for n in s0 if not torch.equal(s0[n], s1[n])]
    bad_g = [(n, float((g0[n] - g1[n]).abs().max())) for n in g0 if not torch.equal(g0[n], g1[n])]
    print(f"scalars differing: {len(bad_s)}/{len(s0)} {bad_s}")
    print(f"gradient tensors differing: {len(bad_g)}/{len(g0)}")
    for n, d in bad_g:
        print(f"  {n}  max|diff| {d:.3e}")


if __name__ == "__main__":
    main()
