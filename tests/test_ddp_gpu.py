"""The product's data-parallel path on the GPU: 2 ranks (torch.distributed gloo, both on cuda:0) each run the HIP
TrainStep on half of a batch; the all-reduced (averaged) D / G gradients, the global balance loss (all-reduced
[E] expert load) and the updated parameters must equal one process stepping the whole batch (fp32).

The mismatched-text permutation stays per rank: the single-process reference uses the
block-diagonal permutation the two ranks' local permutations form.  Also rehearses bench.py's multi-rank path
(hipGraph capture with the collectives as eager segments) with 2 gloo ranks on the one GPU."""
import os
import subprocess
import sys

import pytest
import torch

from steputil import cosine, gpu_step, make_inputs, rel_norm_diff

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("R", [16, 32])
def test_two_rank_trainstep_matches_single_process(tmp_path, R):
    """R = 16: the reference generator; R = 32: the progressive extension (32x32 real and fake images, several
    fake logits per image in the D / G losses)."""
    import torch.multiprocessing as mp
    from ddp_worker import run
    world, B, E = 2, 2, 4
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=run, args=(r, world, port, str(tmp_path), B, E, R)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=240)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, p.exitcode
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    # single process, whole batch, block-diagonal permutation
    real, text, z, eps_d, eps_g, _ = make_inputs(B * world, E, seed=7, res=64 if R == 16 else R)
    perm = torch.cat([res[r]["local_perm"] + r * B for r in range(world)])
    ts = gpu_step(E, None, "fp32", "cuda", max_res=R)
    cu = lambda t: t.to("cuda")  # noqa: E731
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, eff_kl_weight=0.001 * 1e-5)
    torch.cuda.synchronize()
    # the global balance loss is identical on every rank
    for r in range(world):
        assert abs(float(res[r]["balance"][0]) - float(out["balance"][0])) <= 1e-4 * float(out["balance"][0]) + 1e-7
    # per-rank losses average to the whole-batch loss (equal shards)
    for k in ("d_losses", "r1", "g_gan"):
        avg = sum(float(res[r][k][0]) for r in range(world)) / world
        assert abs(avg - float(out[k][0])) <= 1e-4 * abs(float(out[k][0])) + 1e-6, k
    # averaged gradients == whole-batch gradients; identical updated parameters on every rank
    for key, ref in (("d_grad", out["d_grad"]), ("g_grad", out["g_grad"])):
        for r in range(world):
            got = res[r][key]
            assert cosine(got, ref) >= 0.99999 and rel_norm_diff(got, ref) <= 1e-3, (key, r)
    for key, ref in (("d_data", ts.ds.data), ("g_data", ts.gs.data)):
        assert torch.equal(res[0][key], res[1][key]), key
        assert rel_norm_diff(res[0][key], ref) <= 1e-5, key


def test_two_rank_bf16_topk_accumulation_window(tmp_path):
    """C3's routing (E=8 top-2) in the benchmarked bf16 mode under data parallelism with a gradient-accumulation
    window of two batches (reference default gradient_accumulation_steps=8, t2i_moe_gan.py:1043; accumulation
    :1272, :1329, :1353, :1413): 2 gloo ranks x B=2 per batch against one process stepping the whole batches.
    Both sides run the deterministic mode.  Checked after the window: the all-reduced window gradients (the D
    gradient includes the reference's G-phase leak of the first batch, :1272 vs :1407) against the single
    process's at the bf16 bars (cosine >= 0.999 per model), every rank's updated parameters bit-identical, and
    the AdamW update's |g|-weighted cosine with the single process's >= 0.99."""
    import torch.multiprocessing as mp
    from ddp_worker import run
    world, B, E, k, acc = 2, 2, 8, 2, 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=run, args=(r, world, port, str(tmp_path), B, E, 16, k, "bf16", acc))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, p.exitcode
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    from moegan_mi import ops
    ops.set_deterministic(True)
    try:
        ts = gpu_step(E, k, "bf16", "cuda")
        cu = lambda t: t.to("cuda")  # noqa: E731
        for i in range(acc):
            real, text, z, eps_d, eps_g, _ = make_inputs(B * world, E, seed=7 + i)
            perm = torch.cat([res[r]["local_perms"][i] + r * B for r in range(world)])
            out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d],
                          [tuple(map(cu, e)) for e in eps_g], cu(perm.int()), anneal=3.0, eff_kl_weight=0.001 * 1e-5,
                          acc=acc, zero_grads=i == 0, step_optim=i == acc - 1)
        torch.cuda.synchronize()
    finally:
        ops.set_deterministic(False)
    for r in range(world):
        assert int(res[r]["flags"][0]) == 0
        assert abs(float(res[r]["balance"][0]) - float(out["balance"][0])) <= 2e-2 * float(out["balance"][0])
    for key, ref in (("d_grad", out["d_grad"]), ("g_grad", out["g_grad"])):
        got = res[0][key]
        c = cosine(got, ref)
        print(f"{key}: window gradient cosine {c:.6f}, rel {rel_norm_diff(got, ref):.2e}")
        assert c >= 0.999, (key, c)
    for key in ("d_data", "g_data"):
        assert torch.equal(res[0][key], res[1][key]), key
    for key, before, store, g in (("d_data", "d_before", ts.ds, out["d_grad"]), ("g_data", "g_before", ts.gs,
                                                                                   out["g_grad"])):
        n = store.n_opt
        w = g[:n].abs().cpu()
        d_dp = (res[0][key][:n] - res[0][before][:n]) * w
        d_sp = (store.data[:n].cpu() - res[0][before][:n]) * w
        c = cosine(d_dp, d_sp)
        print(f"{key}: |g|-weighted update cosine {c:.6f}")
        assert c >= 0.99, (key, c)


def test_four_rank_skewed_topk_trainstep(tmp_path):
    """C3's routing (E=8 top-2) over 4 ranks whose shards route unevenly (ddp_worker.skew_inputs: each rank's
    captions share a rank-specific direction, so each rank loads its own experts): the [E] load all-reduce must
    produce the single process's global balance loss on every rank, and the bucketed G all-reduce (expert ranges
    handed over during the backward, complement at the end) the single process's gradients -- including experts
    that only some ranks touched.  fp32, 4 gloo ranks x B = 2 on cuda:0 against one process stepping all 8
    images with the block-diagonal permutation."""
    import torch.multiprocessing as mp
    from ddp_worker import run, skew_inputs
    world, B, E, k = 4, 2, 8, 2
    ctx = mp.get_context("spawn")
    port = _free_port()
    procs = [ctx.Process(target=run, args=(r, world, port, str(tmp_path), B, E, 16, k, "fp32", 1, 6.0))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(timeout=300)
    for p in procs:
        if p.is_alive():
            p.kill()
        assert p.exitcode == 0, p.exitcode
    res = [torch.load(os.path.join(tmp_path, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    assert all(res[r]["world_seen"] == world for r in range(world))
    real, text, z, eps_d, eps_g, _ = skew_inputs(make_inputs(B * world, E, seed=7), B, world, 6.0)
    perm = torch.cat([res[r]["local_perm"] + r * B for r in range(world)])
    ts = gpu_step(E, k, "fp32", "cuda")
    cu = lambda t: t.to("cuda")  # noqa: E731
    out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
                  cu(perm.int()), anneal=3.0, eff_kl_weight=0.001 * 1e-5)
    torch.cuda.synchronize()
    # the shards really are skewed: per-rank expert loads of the last MoE layer differ, and the ranks' selections
    # are the single process's rows (routing is per token)
    loads = [torch.bincount(res[r]["topi"][-1].reshape(-1).long(), minlength=E) for r in range(world)]
    print("per-rank last-layer expert loads:", [l.tolist() for l in loads])
    assert len({tuple(l.tolist()) for l in loads}) > 1
    spread = torch.stack(loads).float()
    assert float((spread.max(0).values - spread.min(0).values).max()) >= 0.25 * float(spread.sum(1).mean())
    for li in range(3):
        ref_t = out["topi"][li].cpu().sort(1).values
        n = ref_t.shape[0] // world
        for r in range(world):
            got = res[r]["topi"][li].sort(1).values
            assert torch.equal(got, ref_t[r * n:(r + 1) * n]), (li, r)
    for r in range(world):
        assert abs(float(res[r]["balance"][0]) - float(out["balance"][0])) <= 1e-4 * float(out["balance"][0]) + 1e-7
    for kk in ("d_losses", "r1", "g_gan"):
        avg = sum(float(res[r][kk][0]) for r in range(world)) / world
        assert abs(avg - float(out[kk][0])) <= 1e-4 * abs(float(out[kk][0])) + 1e-6, kk
    for key, ref in (("d_grad", out["d_grad"]), ("g_grad", out["g_grad"])):
        for r in range(world):
            got = res[r][key]
            assert cosine(got, ref) >= 0.99999 and rel_norm_diff(got, ref) <= 1e-3, (key, r)
    # expert ranges one rank never touched still carry the other ranks' gradient after the bucketed all-reduce
    for key, ref in (("d_data", ts.ds.data), ("g_data", ts.gs.data)):
        for r in range(1, world):
            assert torch.equal(res[0][key], res[r][key]), (key, r)
        assert rel_norm_diff(res[0][key], ref) <= 1e-5, key


def test_bench_two_rank_graph_replay():
    """bench.py's N>1 path (captured hipGraph segments + eager all-reduces) with 2 gloo ranks on one GPU."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "8", "--one-device", "--backend", "gloo",
           "--no-cpu-baseline"]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    p = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=REPO)
    assert p.returncode == 0, p.stderr[-3000:]
    import json
    line = [x for x in p.stdout.splitlines() if x.startswith("{")][-1]
    rec = json.loads(line)
    assert rec["n_gpus"] == 2 and rec["finite"] and rec["value"] > 0
    assert rec["config"]["world_seen"] == 2  # the rank count the process group reported
