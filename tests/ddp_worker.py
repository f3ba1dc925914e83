"""Worker of tests/test_ddp_gpu.py: one rank of the product TrainStep under torch.distributed (gloo, every rank on
cuda:0).  Saves its losses and the averaged gradients the optimizer used to ``<out>/rank<r>.pt``."""
import os
import sys


def skew_inputs(inputs, B, world, strength):
    """Rank-skewed routing: every image of rank r's shard gets the same extra caption direction (scaled by
    ``strength``), so the routers' text term sends each rank's tokens to its own few experts and the ranks'
    per-expert loads differ (the [E] load all-reduce then carries uneven vectors)."""
    real, text, z, eps_d, eps_g, perm = inputs
    if strength:
        import torch
        g = torch.Generator().manual_seed(4242)
        dirs = torch.randn(world, text.shape[1], generator=g)
        text = text.clone()
        for r in range(world):
            text[r * B:(r + 1) * B] += strength * dirs[r]
    return real, text, z, eps_d, eps_g, perm


def run(rank, world, port, out_dir, B, E, R=16, topk=None, dtype="fp32", acc=1, skew=0.0):
    """``acc`` > 1: one gradient-accumulation window of ``acc`` batches (seeds 7, 8, ...; t2i_moe_gan.py:1272,
    :1329, :1353, :1413), the optimizers stepping after the last; gradients of the window are all-reduced once.
    ``skew``: rank-skewed routing (skew_inputs)."""
    here = os.path.dirname(os.path.abspath(__file__))
    repo = os.path.dirname(here)
    for p in (here, repo, os.path.join(repo, "moe-gan_cpsc541_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from steputil import gpu_step, make_inputs
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from moegan_mi import ops
        if dtype != "fp32":
            ops.set_deterministic(True)  # the same device numbers as the single-process reference run
        sl = slice(rank * B, (rank + 1) * B)
        ts = gpu_step(E, topk, dtype, "cuda:0", max_res=R)
        ts.pg, ts.world = dist.group.WORLD, world
        cu = lambda t: t.to("cuda:0")  # noqa: E731
        g0, d0 = ts.gs.data.cpu().clone(), ts.ds.data.cpu().clone()
        perms = []
        for i in range(acc):
            real, text, z, eps_d, eps_g, perm = skew_inputs(
                make_inputs(B * world, E, seed=7 + i, res=64 if R == 16 else R), B, world, skew)
            local_perm = torch.randperm(B, generator=torch.Generator().manual_seed(100 + rank + 10 * i))
            perms.append(local_perm)
            out = ts.step(cu(real[sl].contiguous()), cu(text[sl].contiguous()), cu(z[sl].contiguous()),
                          [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                          cu(local_perm.int()), anneal=3.0, eff_kl_weight=0.001 * 1e-5, acc=acc,
                          zero_grads=i == 0, step_optim=i == acc - 1)
        torch.cuda.synchronize()
        res = {k: out[k].detach().cpu().clone() for k in ("d_losses", "r1", "g_gan", "balance", "d_grad", "g_grad",
                                                          "d_grad_sumsq", "g_grad_sumsq", "flags")}
        res["g_data"], res["d_data"] = ts.gs.data.cpu().clone(), ts.ds.data.cpu().clone()
        res["g_before"], res["d_before"] = g0, d0
        res["local_perm"] = perms[0]
        res["local_perms"] = torch.stack(perms)
        res["topi"] = [t.detach().cpu().clone() for t in out["topi"]]  # this rank's G-phase selections
        res["world_seen"] = dist.get_world_size()
        torch.save(res, os.path.join(out_dir, f"rank{rank}.pt"))
    finally:
        dist.destroy_process_group()
