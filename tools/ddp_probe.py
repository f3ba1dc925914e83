"""Two gloo ranks (B=2 each, cuda:0) vs one process (B=4): per-parameter generator-gradient differences (diagnostic;
the same run as tests/test_ddp_gpu.py).  MOEGAN_FOLD_DEFER is inherited by the ranks."""
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (os.path.join(ROOT, "tests"), ROOT, os.path.join(ROOT, "moe-gan_cpsc541_amd")):
    sys.path.insert(0, p)


def main():
    import socket
    import torch
    import torch.multiprocessing as mp
    from ddp_worker import run
    from steputil import gpu_step, make_inputs
    world, B, E, R = 2, 2, 4, 16
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    tmp = tempfile.mkdtemp()
    ctx = mp.get_context("spawn")
    procs = [ctx.Process(target=run, args=(r, world, port, tmp, B, E, R)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    res = [torch.load(os.path.join(tmp, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    real, text, z, eps_d, eps_g, _ = make_inputs(B * world, E, seed=7, res=64)
    perm = torch.cat([res[r]["local_perm"] + r * B for r in range(world)])
    ts = gpu_step(E, None, "fp32", "cuda", max_res=R)
    cu = lambda t: t.to("cuda")  # noqa: E731
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, eff_kl_weight=0.001 * 1e-5)
    torch.cuda.synchronize()
    for key, store in (("d_grad", ts.ds), ("g_grad", ts.gs)):
        ref = out[key].cpu()
        got = res[0][key]
        bad = []
        for name, (o, n) in store.offsets.items():
            x, y = ref[o:o + n], got[o:o + n]
            d = (x - y).abs().max().item()
            if d > 1e-3 * max(x.abs().max().item(), 1e-30):
                bad.append((name, d, x.abs().max().item(), y.abs().max().item()))
        print(f"{key}: {len(bad)} of {len(store.offsets)} tensors differ (rank 0 vs single)", flush=True)
        for t in bad[:60]:
            print("   %-60s diff %.3e |single| %.3e |rank0| %.3e" % t, flush=True)


if __name__ == "__main__":
    main()
