"""Isolated timings of the router kernels at the C5 layer shapes (32 experts top-4; 4x4 / 8x8 / 16x16 tokens of
batch 256): router forward (MFMA vs team kernel, tuning slot 24), router backward (teams vs thread per token) and
the token gradient.  Diagnostic only; times are HIP-event averages over 50 launches (launch overhead included)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "moe-gan_cpsc541_amd"))
import torch  # noqa: E402
from moegan_mi import ops  # noqa: E402
from moegan_mi import _lib as L  # noqa: E402

DEV = "cuda"
E, k, B = 32, 4, 256


def timed(fn, n=50):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1000.0


for HW, C in ((16, 512), (64, 256), (256, 128)):
    T = B * HW
    g = torch.Generator(device=DEV).manual_seed(T)
    tok = torch.randn(T, C, device=DEV, generator=g).to(torch.bfloat16)
    Wfc = torch.randn(C, E, device=DEV, generator=g) * 0.1
    Lt = torch.randn(B, E, device=DEV, generator=g)
    temp = torch.tensor([1.0], device=DEV)
    row = {}
    for slot in (0, 1):
        L.call("mg_set_tuning", 24, slot)
        row[f"fwd{'_team' if slot else '_mfma'}"] = timed(lambda: ops.router_fwd(tok, Wfc, Lt, E, k, HW, temp, 1.0))
    L.call("mg_set_tuning", 24, 0)
    probs, zlog, topi, gate = ops.router_fwd(tok, Wfc, Lt, E, k, HW, temp, 1.0)
    g_gate = torch.randn(T, k, device=DEV, generator=g)
    gt = torch.zeros(1, device=DEV)
    for slot in (0, 2):
        L.call("mg_set_tuning", 24, slot)
        row[f"bwd{'_thread' if slot else '_team'}"] = timed(
            lambda: ops.router_bwd(probs, zlog, topi, gate, g_gate, None, None, HW, temp, 1.0, gt, B))
    L.call("mg_set_tuning", 24, 0)
    g_raw = torch.randn(T, E, device=DEV, generator=g)
    gX = torch.randn(T * k, C, device=DEV, generator=g).to(torch.bfloat16)
    pos_of = torch.randperm(T * k, device=DEV, generator=g).to(torch.int32)
    out = torch.empty(T, C, device=DEV, dtype=torch.bfloat16)
    row["token_grad"] = timed(lambda: ops.moe_token_grad(gX, pos_of, g_raw, Wfc, out, k))
    G1 = torch.zeros(C, E, device=DEV)
    row["feat_grad"] = timed(lambda: ops.router_feat_grad(tok, g_raw, G1))
    WT = Wfc.t().contiguous().to(torch.bfloat16)
    row["gemm_T_x_E"] = timed(lambda: ops.gemm(tok, WT, T, E, C))
    print(f"T={T:6d} C={C:4d}  " + "  ".join(f"{kk} {v:6.1f}us" for kk, v in row.items()), flush=True)
