"""The slowest C-ABI calls of one eager C2 (or TOP_CONFIG=C5) step, per family, with shapes (event-timed; ~3 us
event overhead each).

  python tools/top_calls.py [family ...]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402


def main():
    import bench
    from moegan_mi.init import init_discriminator, init_generator
    from moegan_mi.roofline import Attribution
    from moegan_mi.step import StepConfig, TrainStep
    dev = torch.device("cuda", 0)
    # TOP_CONFIG=C5: 32 experts top-4 with the MX-fp8 3x3 convs (bench.py --config C5)
    c5 = os.environ.get("TOP_CONFIG", "C2") == "C5"
    E, k, B = (32, 4, 256) if c5 else (8, 2, 256)
    ts = TrainStep(StepConfig(E=E, topk=k, dtype="bf16", fp8=c5), dev)
    init_generator(ts.gs, seed=0)
    init_discriminator(ts.ds, seed=1)
    g = torch.Generator(device=dev).manual_seed(1)
    real = torch.rand(B, 3, 64, 64, device=dev, generator=g) * 2 - 1
    text = torch.randn(B, 512, device=dev, generator=g)
    z = torch.randn(B, 512, device=dev, generator=g)
    _, eps_d = bench.eps_buffers(E, dev)
    _, eps_g = bench.eps_buffers(E, dev)
    for t in eps_d + eps_g:
        for x in t:
            x.normal_(generator=g)
    perm = torch.randperm(B, device=dev, generator=g).int()
    run = lambda: ts.step(real, text, z, eps_d, eps_g, perm, anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)  # noqa
    run()
    run()
    torch.cuda.synchronize()
    with Attribution(keep_args=True) as at:
        run()
    fams = sys.argv[1:] or os.environ.get("TOP_FAMILIES", "gemm,expert_gemm,conv_fwd,conv_wgrad+fold").split(",")
    top_n = int(os.environ.get("TOP_N", "60"))
    for f in fams:
        print(f"== {f}")
        calls = at.top_calls(f, 10 ** 6)
        print(f"   {len(calls)} calls, {sum(c[0] for c in calls) * 1e3:.1f} us")
        for ms, name, w, a in calls[:top_n]:
            rate = ""
            if w:
                rate = f"{w / (ms * 1e-3) / 1e12:7.1f} TF/s" if f in ("gemm", "conv_fwd", "conv_wgrad+fold",
                                                                   "expert_gemm", "conv_dgrad_s2", "attention") \
                    else f"{w / (ms * 1e-3) / 1e9:7.1f} GB/s"
            keys = {k_: v for k_, v in a.items() if k_ != "stream" and not k_.startswith("ld") and abs(v) < 1e9}
            print(f"{ms * 1e3:8.1f} us {rate} {name} {keys}")


if __name__ == "__main__":
    main()
