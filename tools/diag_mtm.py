"""Diagnostic: MTM / ConvolutionBlock module gradients vs the oracle under large offsets (GPU)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

import t2i_moe_gan as M  # noqa: E402
from oracle import aurora_cpu as O  # noqa: E402


def params(m):
    return {k: v.detach().cpu().clone().requires_grad_(True) for k, v in m.state_dict().items()}


def run(kind, cin, cout, H, scale):
    torch.manual_seed(0)
    m = (M.ModulatedTransformationModule(cin, cout, 3, use_offset=True, resolution=H) if kind == "mtm"
         else M.ConvolutionBlock(cin, cout, resolution=H)).cuda()
    P = params(m)
    with torch.no_grad():
        for k in P:
            if k.endswith("offset_net.2.weight"):
                P[k].mul_(scale)
        m.load_state_dict({k: v.detach() for k, v in P.items()})
    x, w = torch.randn(2, cin, H, H), torch.randn(2, 512)
    xr, wr = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = O.mtm(xr, wr, P, "") if kind == "mtm" else O.conv_block(xr, wr, P, "")
    xd, wd = x.cuda().requires_grad_(True), w.cuda().requires_grad_(True)
    yd = m(xd, wd)
    gy = torch.randn(y.shape)
    (y * gy).sum().backward()
    (yd * gy.cuda()).sum().backward()
    rel = lambda a, b: float((a.cpu() - b).abs().max() / b.abs().max())  # noqa: E731
    print(f"{kind} {cin}->{cout} H={H} offsets x{scale}: y {rel(yd.detach(), y.detach()):.2e} "
          f"gx {rel(xd.grad, xr.grad):.2e} gw {rel(wd.grad, wr.grad):.2e}", flush=True)


for args in (("mtm", 256, 128, 16, 20.0), ("mtm", 128, 128, 16, 20.0), ("mtm", 256, 128, 16, 1.0),
             ("cb", 256, 128, 16, 1.0), ("cb", 256, 128, 16, 20.0), ("mtm", 512, 256, 8, 20.0),
             ("mtm", 16, 8, 16, 20.0)):
    run(*args)
