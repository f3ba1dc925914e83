"""Benchmark: images/sec of one full G+D training step (BASELINE.json metric) on N MI355X.

Default workload = BASELINE.json configs[1] ("C2"): 64x64 real images, E=8 experts top-2,
batch 256 per GPU, bf16 activations / MFMA operands (fp32 master weights + AdamW), R1 on.
A step is the whole train_aurora_gan batch body (t2i_moe_gan.py:1262-1421): D phase with R1,
G forward x2 (fresh router noise each), G phase, both AdamW steps, clip_grad_norm_ both.
Synthetic data (no network): real ~U(-1,1), captions ~N(0,1) CLIP-like 512-d, z ~N(0,1),
router epsilon drawn on device inside the step, random-init weights (reference init).

Multi-GPU: one process per GPU (torchrun), RCCL all-reduce of the flat D/G gradients and the
[E] expert-load vector; per-GPU batch fixed ("weak" scaling).  Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "moe-gan_cpsc541_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0
MFMA_PEAK_TFLOPS = {"bf16": 2500.0, "fp32": 157.3}
# G+D step FLOPs/image = 6.810 + 0.806 * k_active GFLOP
def gflop_per_image(k_active):
    return 6.810 + 0.806 * k_active


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=256, help="per-GPU batch")
    ap.add_argument("--experts", type=int, default=8)
    ap.add_argument("--topk", type=int, default=2)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--config", default="C2", choices=["C2", "C4", "C5", "loop"],
                    help="C2 = BASELINE configs[1] (the headline line); C4 = the per-GPU slice of configs[3]: the "
                         "128x128 progressive generator, 16 experts top-2, CLIP loss on; C5 = the per-GPU slice of "
                         "configs[4]: 32 experts top-4, MX-fp8 3x3 modulated convs; loop = the C2 workload through the "
                         "drop-in train_aurora_gan loop (pinned host batches, H2D copy included)")
    ap.add_argument("--fp8", action="store_true", help="MX-fp8 3x3 modulated convs (implied by --config C5)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--secondary", default="C5,C4,loop",
                    help="comma-separated configs measured after the headline one, each in a child bench.py process "
                         "(N=1 only), reported under 'secondary' in the same JSON line; '' to skip")
    ap.add_argument("--cpu-steps", type=int, default=12, help="timed CPU-oracle steps (B=8; ~10-20 s of CPU work)")
    ap.add_argument("--eager", action="store_true",
                    help="launch every kernel from Python each step instead of replaying the captured hipGraphs")
    ap.add_argument("--backend", default="nccl", help="process-group backend for N>1 (nccl = RCCL)")
    ap.add_argument("--no-families", action="store_true",
                    help="skip the per-family roofline attribution step (one extra eager step before the capture, "
                         "outside the timed region) and with it the live roofline kernel")
    ap.add_argument("--one-device", action="store_true",
                    help="map every rank to cuda:0 (multi-rank rehearsal on a 1-GPU box, with --backend gloo)")
    args = ap.parse_args()
    args.res, args.max_res = 64, 16
    if args.config == "C5":  # BASELINE configs[4]: 64x64, 32 experts top-4, fp8 MFMA conv path, KL + balance
        args.experts, args.topk, args.fp8 = 32, 4, True
    if args.config == "C4":  # BASELINE configs[3]: 128x128 progressive stage, 16 experts top-2, CLIP loss on
        args.experts, args.topk, args.res, args.max_res = 16, 2, 128, 128
    assert not args.fp8 or args.dtype == "bf16", "the MX-fp8 convs run inside the bf16 mode"
    return args


EPS_DIMS = [(512, 512), (256, 512), (128, 512)]  # (C, text) per MoE block: eps_f [C,128], eps_t [512,128], eps_c


def eps_buffers(E, dev):
    """One flat buffer holding the router epsilons of one generator forward (3 blocks x (f, t, c)), plus views."""
    n = sum(c * 128 + t * 128 + 256 * E for c, t in EPS_DIMS)
    flat = torch.empty(n, device=dev)
    views, o = [], 0
    for c, t in EPS_DIMS:
        trip = []
        for shp in ((c, 128), (t, 128), (256, E)):
            k = shp[0] * shp[1]
            trip.append(flat[o:o + k].view(shp))
            o += k
        views.append(tuple(trip))
    return flat, views


def cpu_baseline(args, E, k):
    """Oracle (CPU restatement of the reference step) on a bounded sample: B=8, same E/top-k."""
    from oracle import aurora_cpu as O
    from moegan_mi.layout import discriminator_shapes, generator_shapes
    from moegan_mi.init import init_discriminator, init_generator  # noqa: F401
    from oracle.recipe import fill_state
    torch.set_num_threads(max(1, min(os.cpu_count() or 1, int(os.environ.get("OMP_NUM_THREADS", "16")))))
    B = 8
    PG = {n: torch.from_numpy(v) for n, v in fill_state(generator_shapes(E), 0).items()}
    PD = {n: torch.from_numpy(v).requires_grad_(True) for n, v in fill_state(discriminator_shapes(), 50).items()}
    for n, v in PG.items():
        if not n.split(".")[-1].startswith("epsilon_"):
            v.requires_grad_(True)
    optG = torch.optim.AdamW([v for v in PG.values() if v.requires_grad], lr=2e-4, betas=(0.5, 0.999),
                             weight_decay=0.01)
    optD = torch.optim.AdamW(list(PD.values()), lr=2e-4, betas=(0.5, 0.999), weight_decay=0.01)
    g = torch.Generator().manual_seed(0)
    real = torch.rand(B, 3, 64, 64, generator=g) * 2 - 1
    text = torch.randn(B, 512, generator=g)
    z = torch.randn(B, 512, generator=g)
    dims = [(512, 512), (256, 512), (128, 512)]
    mk = lambda: [tuple(torch.randn(s, generator=g) for s in ((c, 128), (t, 128), (256, E))) for c, t in dims]  # noqa
    O.train_step(PG, PD, optG, optD, real, text, z, mk(), mk(), torch.randperm(B, generator=g), topk=k)  # warm
    t0 = time.perf_counter()
    n = 0
    while n < args.cpu_steps and (n == 0 or time.perf_counter() - t0 < 20.0):
        O.train_step(PG, PD, optG, optD, real, text, z, mk(), mk(), torch.randperm(B, generator=g), topk=k)
        n += 1
        print(f"[bench] cpu baseline step {n}: {time.perf_counter() - t0:.1f} s", file=sys.stderr, flush=True)
    dt = time.perf_counter() - t0
    return {"value": round(B * n / dt, 3), "unit": "images/sec", "cores": torch.get_num_threads(),
            "kind": "port", "sample": f"oracle/aurora_cpu.train_step, B={B}, E={E} top-{k}, fp32, "
                                      f"{n} timed steps after 1 warm-up"}


def run_secondary(cfg, args):
    """Measure another BASELINE config (e.g. C5's single-GPU slice) in a child process -- its own GPU context,
    graphs and memory -- and return its JSON line (the headline line above stays C2).  The child runs in its own
    process group, which is killed after it exits, so no descendant outlives the bench."""
    import signal
    import subprocess
    cmd = [sys.executable, os.path.join(REPO, "bench.py"), "--config", cfg, "--steps", str(max(5, args.steps)),
           "--warmup", str(args.warmup), "--no-cpu-baseline", "--secondary", ""]
    print(f"[bench] secondary config {cfg}: {' '.join(cmd[1:])}", file=sys.stderr, flush=True)
    proc = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, start_new_session=True)
    try:
        out, err = proc.communicate(timeout=600)
        lines = [ln for ln in out.splitlines() if ln.startswith("{")]
        if proc.returncode != 0 or not lines:
            return {"config": cfg, "error": f"rc={proc.returncode}: {err[-300:]}"}, None
        rec = json.loads(lines[-1])
        full = dict(rec)
        full["roofline_families"] = _read_families(cfg)  # the child wrote its full table to its own file
        return compact_secondary(cfg, rec), full
    except Exception as e:  # a report, never the headline value
        return {"config": cfg, "error": repr(e)[:300]}, None
    finally:
        try:
            os.killpg(proc.pid, signal.SIGKILL)  # anything the child left in its group
        except (ProcessLookupError, PermissionError):
            pass
        proc.wait()


FAMILIES_DIR = os.path.join(REPO, "gpurun_out")  # scratch; copies worth keeping are committed under profiles/


def families_path(cfg):
    return os.path.join(FAMILIES_DIR, f"bench_families_{cfg}.json")


def _write_families(cfg, rec):
    try:
        os.makedirs(FAMILIES_DIR, exist_ok=True)
        with open(families_path(cfg), "w") as f:
            json.dump(rec, f, indent=1)
    except OSError as e:  # a report only
        print(f"[bench] could not write {families_path(cfg)}: {e}", file=sys.stderr, flush=True)


def _read_families(cfg):
    try:
        with open(families_path(cfg)) as f:
            return json.load(f).get("roofline_families")
    except (OSError, ValueError):
        return None


def compact_secondary(cfg, rec):
    """The few fields of a secondary config that go on the headline line (the driver reads a bounded stdout tail,
    so the line stays a few KB: VERDICT r3 'BENCH_r03 parsed is null')."""
    roof = rec.get("roofline") or {}
    dom = roof.get("dominant") or {}
    return {"config": cfg, "value": rec.get("value"), "ms_per_step": rec.get("ms_per_step"),
            "finite": rec.get("finite"), "dtype": rec.get("dtype"), "step_mfma_frac": rec.get("step_mfma_frac"),
            "dominant": (f"{dom.get('family')} {dom.get('frac')}" if dom else None),
            "kernel_frac": roof.get("frac")}


def loop_bench(args, dev):
    """Images/sec of the drop-in training loop itself (t2i_moe_gan.train_aurora_gan, reference :1214-1421) on the
    C2 workload: pinned host batches, each copied host -> HBM by the loop's prefetcher while the previous batch
    trains, every batch body a replayed hipGraph, the guard word / logged losses read one batch late.  Timed from
    the host seeing batch ``warmup`` done to it seeing the last batch done (steady state: the first batch of the
    epoch runs eagerly and is captured)."""
    import t2i_moe_gan as M
    B, n = args.batch, args.warmup + args.steps + 1
    g = torch.Generator().manual_seed(0)
    imgs = (torch.rand(B * n, 3, 64, 64, generator=g) * 2 - 1).pin_memory()
    text = torch.randn(B * n, 512, generator=g).pin_memory()
    loader = [(imgs[i:i + B], text[i:i + B]) for i in range(0, B * n, B)]
    marks, bad = {}, []

    def done(epoch, b, flags):
        marks[b] = time.perf_counter()
        if flags & 3:
            bad.append(b)
        if b % max(1, n // 4) == 0:
            print(f"[bench] loop batch {b + 1}/{n} done", file=sys.stderr, flush=True)
    import tempfile
    with tempfile.TemporaryDirectory() as tmp:
        M.train_aurora_gan(loader, num_epochs=1, lr=2e-4, gradient_accumulation_steps=1, checkpoint_activation=False,
                           num_experts=args.experts, topk=args.topk, dtype=args.dtype, seed=0, save_dir=tmp,
                           log_interval=10 ** 9, device=dev, use_graphs=not args.eager, on_batch_done=done)
    t0, t1 = marks[args.warmup], marks[n - 1]
    ms = (t1 - t0) / (n - 1 - args.warmup) * 1e3
    return {"metric": "images/sec (G+D step through the drop-in train_aurora_gan loop, 64x64, H2D copy included)",
            "value": round(B * 1e3 / ms, 2), "unit": "images/sec", "ms_per_step": round(ms, 3), "dtype": args.dtype,
            "finite": not bad,  # no batch raised a non-finite D / G loss guard
            "config": {"workload": f"C2 via train_aurora_gan: 64x64, {args.experts} experts top-{args.topk}, batch "
                                   f"{B}, {args.dtype}, R1 on, pinned host batches (12.6 MB) copied per batch",
                       "global_batch": B, "parallelism": "dp1",
                       "launch": "eager" if args.eager else "hipGraph replay per batch"},
            "batches_timed": n - 1 - args.warmup}


def _prof(args, B, E, name):
    """A committed rocprofv3 record of this same workload (tools/gpu.sh prof / pmc): the config's own file
    (family_time_C5.json ...) first, then the C2 one; None unless batch / dtype / experts / fp8 / res match."""
    stem, ext = os.path.splitext(name)
    for path in (os.path.join(REPO, "profiles", f"{stem}_{args.config}{ext}"), os.path.join(REPO, "profiles", name)):
        if not os.path.exists(path):
            continue
        rec = json.load(open(path))
        ok = (rec.get("batch") == B and rec.get("dtype") == args.dtype and rec.get("experts") == E and
              bool(rec.get("fp8", False)) == args.fp8 and rec.get("max_res", 16) == args.max_res)
        if ok:
            return rec
    return None


def _fam_time(f):
    """A family's time per step: the committed rocprof figure where there is one, else the live event time."""
    return f.get("rocprof_ms_per_step", f.get("event_ms_per_step", f.get("ms_per_step", 0.0)))


ROOFLINE_KERNEL_FILE = os.path.join(REPO, "profiles", "roofline_kernel.json")


def roofline_record(args, B, E, k, families, roof_call, kms, step_ms):
    """The ``roofline`` object: the dominant family (most time per step) and its largest call, timed live over the
    timed region with fence-free HIP events (``kms``: ms per launch).  ``profiles/roofline_kernel.json``
    (tools/roofline_kernel.py, from a rocprofv3 kernel trace and the PMC FETCH_SIZE / WRITE_SIZE passes of this
    same bench command, the call's dispatches found between its mg_mark kernels) supplies the rocprof duration and
    the HBM traffic of the same call where its signature and workload match."""
    roof = {}
    if families:
        dom = max((f for f in families if f["bound"] is not None), key=_fam_time, default=None)
        if dom is not None:
            roof["dominant"] = {kk: dom.get(kk) for kk in ("family", "bound", "achieved", "peak", "unit", "frac",
                                                          "launches_per_step", "gflop_per_step", "mb_per_step",
                                                          "time_source")}
            roof["dominant"].update({"ms_per_step": round(_fam_time(dom), 4),
                                     "traffic_mb_per_step": dom.get("traffic_mb_per_step"),
                                     "share_of_step": round(_fam_time(dom) / step_ms, 4)})
    if roof_call is None:
        roof.update({"bound": None, "kernel": None, "achieved": None, "peak": None, "unit": None, "frac": None,
                     "traffic": None, "note": "no attribution step (--no-families): no roofline kernel"})
        return roof
    fam = roof_call["family"]
    mfma = fam["bound"] == "mfma"
    peak = fam["peak"]
    work = roof_call["work_per_launch"] or 0.0
    avg_ms = sum(kms) / len(kms) if kms else None

    def rate(ms_):
        if not ms_:
            return None
        return work / (ms_ * 1e-3) / (1e12 if mfma else 1e9)
    ach = rate(avg_ms)
    shape = ", ".join(f"{a}={v}" for a, v in roof_call["args"].items() if a not in ("dtype",))
    roof.update({"bound": fam["bound"], "family": fam["family"],
                 "kernel": f"{roof_call['entry']}({shape}): the largest call of the dominant family {fam['family']} "
                           f"({roof_call['launches_per_step']:.0f} launches per step)",
                 "achieved": round(ach, 2) if ach else None, "peak": peak, "unit": fam["unit"],
                 "frac": round(ach / peak, 4) if ach else None,
                 "algorithmic_per_launch": work, "algorithmic_unit": "FLOP" if mfma else "bytes",
                 "algorithmic_bytes_per_launch": work if not mfma else roof_call.get("bytes_per_launch"),
                 "launches_timed": len(kms), "avg_launch_ms": round(avg_ms, 4) if avg_ms else None,
                 "time_source": "fence-free HIP events over the timed region (mg_timer_event_*)",
                 "traffic": None, "traffic_unit": "HBM bytes per launch (PMC FETCH_SIZE x2 + WRITE_SIZE)"})
    rec = None
    if os.path.exists(ROOFLINE_KERNEL_FILE):
        rec = json.load(open(ROOFLINE_KERNEL_FILE)).get(args.config)
    sig = [roof_call["signature"][0], list(roof_call["signature"][1])]
    roof["signature"] = sig
    if rec and rec.get("signature") == sig and rec.get("batch") == B and rec.get("experts") == E:
        r_ms = rec.get("rocprof_avg_ms")
        roof.update({"avg_launch_ms_rocprof": r_ms, "frac_rocprof": round(rate(r_ms) / peak, 4) if r_ms else None,
                     "traffic": rec.get("traffic_bytes_per_launch"), "rocprof_kernels": rec.get("kernels"),
                     "profile": rec.get("source")})
    return roof


def reap_children():
    """End (and report) any process this bench started that is still alive: the driver counts leftovers."""
    try:
        import psutil
    except ImportError:
        return []
    left = psutil.Process().children(recursive=True)
    for c in left:
        try:
            c.kill()
        except psutil.Error:
            pass
    psutil.wait_procs(left, timeout=10)
    return [c.pid for c in left]


def other_user_processes():
    """Processes of this user that are neither this bench nor its ancestors (stderr evidence for the driver's
    procs_at_end count: bench.py's own children are reaped above)."""
    try:
        import psutil
    except ImportError:
        return []
    me = psutil.Process()
    skip = {me.pid} | {p.pid for p in me.parents()}
    out = []
    for p in psutil.process_iter(["pid", "uids", "name", "cmdline", "create_time"]):
        try:
            if p.info["pid"] in skip or p.info["uids"] is None or p.info["uids"].real != os.getuid():
                continue
            out.append(f"{p.info['pid']}:{p.info['name']}:{' '.join(p.info['cmdline'] or [])[:80]}")
        except psutil.Error:
            pass
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.one_device:
        local = 0
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    pg = None
    world_seen = 1
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if args.backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        else:
            dist.init_process_group(args.backend, rank=rank, world_size=world)
        pg = dist.group.WORLD
        world_seen = dist.get_world_size(pg)
        assert world_seen == world, (world_seen, world)

    from moegan_mi import ops
    from moegan_mi import _lib
    from moegan_mi import roofline as roofline_mod
    from moegan_mi.graphs import SegmentedGraph
    for kv in filter(None, os.environ.get("MOEGAN_TUNE", "").split(",")):  # A/B switches: "key=value,..."
        k_, v_ = kv.split("=")
        _lib.call("mg_set_tuning", int(k_), int(v_))
    from moegan_mi.init import init_discriminator, init_generator
    from moegan_mi.step import StepConfig, TrainStep
    if args.config == "loop":
        line = loop_bench(args, dev)
        if rank == 0:
            print(json.dumps(line, separators=(",", ":")), flush=True)
        return

    E, k, B = args.experts, args.topk, args.batch
    ts = TrainStep(StepConfig(E=E, topk=k, dtype=args.dtype, fp8=args.fp8, max_res=args.max_res), dev,
                   process_group=pg)
    init_generator(ts.gs, seed=0)
    init_discriminator(ts.ds, seed=1)
    if args.config == "C4":  # CLIP loss on: the forward-only ViT-B/32 image tower (random weights: no download)
        from moegan_mi.clip_vit import ClipImageEncoder
        ts.clip_encoder = ClipImageEncoder(device=dev).encode_image
    gen = torch.Generator(device=dev).manual_seed(1000 + rank)
    real = torch.rand(B, 3, args.res, args.res, device=dev, generator=gen) * 2 - 1
    text = torch.randn(B, 512, device=dev, generator=gen)
    z = torch.randn(B, 512, device=dev, generator=gen)
    # the step's random inputs live in fixed buffers, refilled before every step (eager or replayed)
    eps_d_flat, eps_d = eps_buffers(E, dev)
    eps_g_flat, eps_g = eps_buffers(E, dev)
    perm = torch.empty(B, device=dev, dtype=torch.int32)

    draws = [0]

    def refill():
        # fresh router noise for both generator forwards (:349-351, identical on every rank) and this rank's
        # mismatched-caption permutation, one counter-based launch (mg_step_inputs)
        draws[0] += 1
        ops.step_inputs(eps_d_flat, eps_g_flat, perm, seed_eps=(3 << 32) + draws[0],
                        seed_perm=((1000 + rank) << 32) + draws[0])

    def run_step():
        return ts.step(real, text, z, eps_d, eps_g, perm, anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)

    graph = None
    if args.eager:
        refill()
        run_step()  # first-use allocations and code-object loads, before the attributed step
        torch.cuda.synchronize()
    else:
        graph = SegmentedGraph()
        refill()
        t_w = time.perf_counter()
        graph.run_eager(run_step)  # sizes every lazily allocated buffer / workspace (on the capture stream)
        t_f = time.perf_counter()  # first-step host time: allocations + first launch of every kernel (code objects)
        torch.cuda.synchronize()
        t_h = time.perf_counter()
        graph.run_eager(run_step)  # host enqueue time of one eager step (diagnostic)
        t_e = time.perf_counter()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] first eager step {(t_h - t_w) * 1e3:.1f} ms (host enqueue {(t_f - t_w) * 1e3:.1f} ms: "
                  f"first-use allocations + code-object loads); second: host enqueue {(t_e - t_h) * 1e3:.1f} ms, "
                  f"with device {(time.perf_counter() - t_h) * 1e3:.1f} ms", file=sys.stderr, flush=True)

    # per-family roofline attribution: one eager step (before capture, outside the timed region) with every C-ABI
    # call bracketed by HIP events and its algorithmic work computed from its shape arguments (moegan_mi/roofline.py).
    # It also names the roofline kernel: the largest call (signature with the most time per step) of the step's
    # dominant family, which the timed region then times live (_lib.LiveTimer).
    families = fam_meta = roof_call = None
    if not args.no_families:
        from moegan_mi.roofline import Attribution
        refill()
        with Attribution() as at:
            if graph is not None:
                graph.run_eager(run_step)
            else:
                run_step()
        families = at.summary(steps=1, peak_tflops=MFMA_PEAK_TFLOPS[args.dtype], peak_gbs=HBM_PEAK_GBS)
        if rank == 0:
            print(f"[bench] family attribution: {sum(f['ms_per_step'] for f in families):.3f} ms of call time in the "
                  f"attributed step (host_bound={at.host_bound})", file=sys.stderr, flush=True)
        ftime, ftraf = _prof(args, B, E, "family_time.json"), _prof(args, B, E, "family_traffic.json")
        for f in families:
            f["event_ms_per_step"] = f.pop("ms_per_step")  # live, includes ~3 us of event overhead per call
            t = ftime["families"].get(f["family"]) if ftime else None
            if t is not None:  # achieved rate over the rocprof kernel time (the event pairs inflate small calls)
                f["rocprof_ms_per_step"] = t["ms_per_step"]
                ms_k = t["ms_per_step"]
                work = f.get("gflop_per_step", 0) * 1e9 if f["bound"] == "mfma" else f.get("mb_per_step", 0) * 1e6
                if f["bound"] == "mfma" and ms_k > 0:
                    f["achieved"] = round(work / (ms_k * 1e-3) / 1e12, 1)
                    f["frac"] = round(f["achieved"] / f["peak"], 4)
                elif f["bound"] == "hbm" and ms_k > 0:
                    f["achieved"] = round(work / (ms_k * 1e-3) / 1e9, 1)
                    f["frac"] = round(f["achieved"] / f["peak"], 4)
                f["time_source"] = "rocprof"
            elif f["bound"] is not None:
                f["time_source"] = "hip events (live)"
            tr = ftraf["families"].get(f["family"]) if ftraf else None
            if tr is not None:
                f["traffic_mb_per_step"] = tr["mb_per_step"]
        fam_meta = {"work": "live: algorithmic FLOPs / bytes from each C-ABI call's shape arguments "
                            "(moe-gan_cpsc541_amd/moegan_mi/roofline.py)",
                    "time": ftime["source"] if ftime else "live HIP events per call",
                    "profile_busy_ms_per_step": ftime["busy_ms_per_step"] if ftime else None,
                    "traffic": ftraf["source"] if ftraf else None}
        dom = max((f for f in families if f["bound"] is not None), key=_fam_time, default=None)
        if dom is not None:
            roof_call = at.largest_call(dom["family"])
            if roof_call is not None:
                roof_call["family"] = dom
                _lib.LIVE = _lib.LiveTimer(roof_call["signature"], active=False)

    if graph is not None:
        out = graph.capture(run_step)
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] captured the step: {graph.n_graphs} graph segment(s), {len(graph.items)} items",
                  file=sys.stderr, flush=True)

    def one_step():
        refill()
        if graph is not None:
            graph.replay()
            return out
        return run_step()

    for i in range(args.warmup):
        t_w = time.perf_counter()
        one_step()
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup step {i}: {(time.perf_counter() - t_w) * 1e3:.1f} ms", file=sys.stderr, flush=True)

    if _lib.LIVE is not None:
        _lib.LIVE.active = True
    # per-step device time for the median: an event between consecutive steps on the stream the
    # steps are enqueued on (no host synchronisation inside the timed region)
    step_ev = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    if pg is not None:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    step_ev[0].record()
    for i in range(args.steps):
        out = one_step()
        step_ev[i + 1].record()
        if rank == 0 and (i + 1) % max(1, args.steps // 4) == 0:
            print(f"[bench] enqueued {i + 1}/{args.steps} steps", file=sys.stderr, flush=True)
    torch.cuda.synchronize()
    if pg is not None:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    kms = []
    if _lib.LIVE is not None:
        _lib.LIVE.active = False
        kms = _lib.LIVE.results()
    if pg is not None:
        t = torch.tensor([elapsed], device=dev)
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        elapsed = float(t)
    finite = bool(torch.isfinite(out["d_losses"]).all() and torch.isfinite(out["g_gan"]).all())
    if rank == 0:
        arena = ops.fold_arena_bytes(graph.stream if graph is not None else None)
        print(f"[bench] gradient-fold arena: {arena / 2 ** 20:.0f} MiB on the step's stream; torch allocated "
              f"{torch.cuda.memory_allocated(dev) / 2 ** 30:.2f} GiB (peak {torch.cuda.max_memory_allocated(dev) / 2 ** 30:.2f})",
              file=sys.stderr, flush=True)
    step_ms = sorted(step_ev[i].elapsed_time(step_ev[i + 1]) for i in range(args.steps))
    median_ms = step_ms[len(step_ms) // 2] if len(step_ms) % 2 else 0.5 * sum(step_ms[len(step_ms) // 2 - 1:
                                                                                      len(step_ms) // 2 + 1])

    if rank == 0:
        imgs = B * world * args.steps
        value = imgs / elapsed
        ms = elapsed / args.steps * 1e3
        peak = MFMA_PEAK_TFLOPS[args.dtype]
        roof = roofline_record(args, B, E, k, families, roof_call, kms, ms)
        if args.config == "C4":  # extension: no reference FLOP formula; the executed MFMA work (roofline.py)
            gf_step = sum(f.get("gflop_per_step", 0.0) for f in (families or []) if f["bound"] == "mfma")
            step_tflops = gf_step * world / (ms * 1e-3) / 1e3 if gf_step else 0.0
        else:
            step_tflops = gflop_per_image(k) * B * world / (ms * 1e-3) / 1e3
        step_frac = step_tflops / peak
        peak_note = f"{args.dtype} dense MFMA peak"
        fp8_gf = sum(f.get("gflop_per_step", 0.0) for f in (families or []) if f["family"] == "conv_fwd_mx8")
        if args.fp8 and fp8_gf and args.config != "C4":
            # the MX-fp8 share of the algorithmic work priced at the fp8 peak, the rest at the bf16 peak
            all_gf = gflop_per_image(k) * B
            t_peak = (all_gf - fp8_gf) / (peak * 1e3) + fp8_gf / (roofline_mod.MX8_PEAK_TFLOPS * 1e3)
            step_frac = t_peak / (ms * 1e-3)
            peak_note = (f"mixed: {fp8_gf:.0f} of {all_gf:.0f} GFLOP per step on the MX-fp8 peak "
                         f"({roofline_mod.MX8_PEAK_TFLOPS:.0f} TF/s), the rest on the bf16 peak ({peak:.0f} TF/s)")
        cpu = None
        if not args.no_cpu_baseline and world == 1 and args.config != "C4":
            try:
                cpu = cpu_baseline(args, E, k)
            except Exception as e:  # the baseline is a report, never the measured value
                cpu = {"error": repr(e)}
        metric = ("images/sec (G+D step, 64x64 MS-COCO layout)" if args.res == 64 else
                  f"images/sec (G+D step, {args.res}x{args.res} progressive stage)")
        secondary, secondary_full = [], []
        if world == 1 and args.config == "C2" and args.secondary:
            for cfg in [c for c in args.secondary.split(",") if c and c != args.config]:
                short, full = run_secondary(cfg, args)
                secondary.append(short)
                if full is not None:
                    secondary_full.append(full)
        line = {"metric": metric, "value": round(value, 2),
                "unit": "images/sec", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms, 3), "ms_per_step_median": round(median_ms, 3),
                "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
                "dtype": args.dtype + ("+mx8" if args.fp8 else ""),
                "data": "synthetic (U(-1,1) images, N(0,1) 512-d captions, random init)",
                "config": {"workload": (f"C5 single-GPU slice: 64x64, {E} experts top-{k}, batch {B}/GPU, bf16 with "
                                        "MX-fp8 (e4m3) 3x3 modulated-conv GEMMs, KL + balance, R1 on") if args.config == "C5"
                           else (f"C4 single-GPU slice: 128x128 progressive generator (extension blocks 32/64/128), "
                                 f"{E} experts top-{k}, batch {B}/GPU, {args.dtype}, CLIP loss on (ViT-B/32 image "
                                 "tower, random weights), R1 on") if args.config == "C4"
                           else f"C2: 64x64, {E} experts top-{k}, batch {B}/GPU, {args.dtype}"
                                + (" + MX-fp8 3x3 convs" if args.fp8 else "") + ", R1 on",
                           "global_batch": B * world, "experts": E, "topk": k, "parallelism": f"dp{world}",
                           "world_seen": world_seen,
                           "launch": "eager" if args.eager else "hipGraph replay"},
                "step_tflops_algorithmic": round(step_tflops, 2),
                "step_mfma_frac": round(step_frac, 4), "step_mfma_peak": peak_note, "finite": finite,
                "roofline": roof, "cpu_baseline": cpu, "secondary": secondary or None}
        if families:  # the full per-family tables go to a file; the line names it
            _write_families(args.config, dict(line, roofline_families=families, roofline_families_sources=fam_meta,
                                              secondary=secondary_full or None))
            line["roofline_families_file"] = os.path.relpath(families_path(args.config), REPO)
        text = json.dumps(line, separators=(",", ":"))
        if len(text) > 4096:  # the driver keeps a bounded tail: never let the headline line outgrow it
            line["secondary"] = [{k: s.get(k) for k in ("config", "value", "ms_per_step", "finite")}
                                 for s in secondary] or None
            line["cpu_baseline"] = {k: (cpu or {}).get(k) for k in ("value", "unit", "cores", "kind", "sample")}
            text = json.dumps(line, separators=(",", ":"))
        sys.stderr.flush()
        print(text, flush=True)
    left = reap_children()
    if left:
        print(f"[bench] ended leftover child processes {left}", file=sys.stderr, flush=True)
    if rank == 0 and args.config == "C2":
        print(f"[bench] other processes of this user at exit: {other_user_processes()}", file=sys.stderr, flush=True)
    if pg is not None:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
