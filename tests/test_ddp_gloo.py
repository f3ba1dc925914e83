"""Data-parallel protocol of moegan_mi/step.py checked with 2 gloo ranks on the CPU.

The product's N-GPU step (TrainStep with a process group) does, per rank:
  * backprop the LOCAL mean losses,
  * all-reduce(sum) the per-expert router load of the last MoE layer, compute the balance
    loss on the GLOBAL batch (t2i_moe_gan.py:951-1000), and inject d(balance)/d(probs) scaled
    by world_size (the gradient all-reduce below averages it back),
  * all-reduce(mean) the flat gradient buffers.
This test runs that protocol with the oracle's autograd on 2 ranks x 1 image and requires
the averaged gradients to equal a single process on the 2-image batch.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from goldens import T, load
from oracle import aurora_cpu as O
from oracle.recipe import fill_state


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _params():
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "moe-gan_cpsc541_amd"))
    from moegan_mi.layout import generator_shapes
    P = {k: torch.from_numpy(v) for k, v in fill_state(generator_shapes(4), 0).items()}
    for k, v in P.items():
        if not k.split(".")[-1].startswith("epsilon_"):
            v.requires_grad_(True)
    return P


def _local_loss_and_grads(P, z, text, eps, world, dp):
    f16, f8, kl, probs = O.generator(z, text, P, eps, True, 3.0)
    g_gan = (f16 ** 2).mean()  # stand-in for the adversarial term: a per-image mean loss
    loss = g_gan + 1e-3 * kl
    last = probs[-1]
    load = last.sum(0).detach()
    T_local = last.shape[0]
    if dp:
        dist.all_reduce(load)
    T_glob = T_local * world
    ld = load.clone().requires_grad_(True)
    frac = (ld + 1e-6) / T_glob
    bal = 0.01 * torch.clamp(4 * frac.std() / (frac.mean() + 1e-6), 0, 10)
    coef, = torch.autograd.grad(bal, ld)
    loss.backward(retain_graph=True)
    last.backward(coef.expand_as(last) * world)  # d bal / d probs, scaled by world (averaged below)
    names = [k for k, v in P.items() if v.requires_grad and v.grad is not None]
    flat = torch.cat([P[k].grad.reshape(-1) for k in names])
    if dp:
        dist.all_reduce(flat)
        flat /= world
    return names, flat


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    d, _ = load("F7_generator")
    P = _params()
    eps = [tuple(T(d[f"eps{i}/{n}"]) for n in ("epsilon_f", "epsilon_t", "epsilon_c")) for i in range(3)]
    z, text = T(d["z"])[rank:rank + 1], T(d["text"])[rank:rank + 1]
    names, flat = _local_loss_and_grads(P, z, text, eps, world, True)
    if rank == 0:
        q.put(flat.numpy())
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_gradient_protocol_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    dp_flat = q.get(timeout=600)
    for p in procs:
        p.join(timeout=600)
        assert p.exitcode == 0
    d, _ = load("F7_generator")
    P = _params()
    eps = [tuple(T(d[f"eps{i}/{n}"]) for n in ("epsilon_f", "epsilon_t", "epsilon_c")) for i in range(3)]
    _, ref = _local_loss_and_grads(P, T(d["z"]), T(d["text"]), eps, 1, False)
    ref = ref.numpy()
    err = np.abs(dp_flat - ref).max() / np.abs(ref).max()
    assert err < 1e-4, err
