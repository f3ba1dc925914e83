"""Per-shape census of the plain GEMM launches (mg_gemm) of one C2 step, each re-timed in isolation.

Records every mg_gemm call of one eager step (M, N, K, orientation, atomic/accumulate epilogue, split request),
then times each distinct shape on fresh operands with HIP events and prints per-step time and TFLOP/s, heaviest
first.  Diagnostic only (GPU):  python tools/gemm_shapes.py [--config C2]
"""
import collections
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "moe-gan_cpsc541_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    from moegan_mi import ops, _lib as L
    from moegan_mi.init import init_discriminator, init_generator
    from moegan_mi.step import StepConfig, TrainStep
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    E, k, B, res = 8, 1, 256, 64
    ts = TrainStep(StepConfig(E=E, topk=k, dtype="bf16"), dev)
    init_generator(ts.gs, seed=0)
    init_discriminator(ts.ds, seed=1)
    real = torch.rand(B, 3, res, res, device=dev) * 2 - 1
    text, z = torch.randn(B, 512, device=dev), torch.randn(B, 512, device=dev)
    _, eps_d = bench.eps_buffers(E, dev)
    _, eps_g = bench.eps_buffers(E, dev)
    perm = torch.randperm(B, device=dev).int()
    seen = collections.Counter()
    real_call = ops.call

    def rec(name, *a):
        if name == "mg_gemm":
            dtype, M, N, K, _, _, akc, _, _, bkc, _, _, odt, ep, splits = a[:15]
            atomic = int(ep.atomic) if ep is not None else 0
            acc = int(ep.accumulate) if ep is not None else 0
            seen[(dtype, M, N, K, akc, bkc, odt, atomic, acc, splits)] += 1
        return real_call(name, *a)

    run = lambda: ts.step(real, text, z, eps_d, eps_g, perm, anneal=3.0, lr_g=2e-4, lr_d=2e-4,  # noqa: E731
                          eff_kl_weight=1e-8)
    run()
    torch.cuda.synchronize()
    ops.call = rec
    run()
    torch.cuda.synchronize()
    ops.call = real_call
    tdt = {0: torch.float32, 1: torch.bfloat16, 2: torch.float16}
    rows = []
    for (dtype, M, N, K, akc, bkc, odt, atomic, acc, splits), cnt in seen.items():
        A = torch.randn(M * K, device=dev).to(tdt.get(dtype, torch.bfloat16)) * 0.1
        Bm = torch.randn(N * K, device=dev).to(tdt.get(dtype, torch.bfloat16)) * 0.1
        out = torch.zeros(M * N, device=dev, dtype=tdt.get(odt, torch.float32))
        ep = L.epilogue(atomic=atomic, accumulate=acc)
        lda = K if akc else M
        ldb = K if bkc else N

        def go():
            real_call("mg_gemm", dtype, M, N, K, ops.ptr(A), lda, akc, ops.ptr(Bm), ldb, bkc, ops.ptr(out), N, odt,
                      ep, splits, ops.S())
        for _ in range(3):
            go()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(20):
            go()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / 20 * 1e3
        rows.append((us * cnt, cnt, us, 2 * M * N * K / us / 1e6, (dtype, M, N, K, akc, bkc, odt, atomic, acc, splits)))
    rows.sort(reverse=True)
    tot = sum(r[0] for r in rows)
    print(f"mg_gemm: {sum(seen.values())} launches/step, {tot:.0f} us/step isolated")
    print("  us/step  n   us/call  TFLOP/s  (dtype,M,N,K,a_kc,b_kc,out_dt,atomic,acc,splits)")
    for r in rows:
        print(f"{r[0]:8.1f} {r[1]:3d} {r[2]:8.1f} {r[3]:8.1f}  {r[4]}")


if __name__ == "__main__":
    main()
