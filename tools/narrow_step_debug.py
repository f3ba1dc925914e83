"""Inside one bf16 C2 step at B=8: every 32-channel 3x3 conv call (the offset heads' forward) is run twice, on the
direct kernel and on the implicit GEMM, and their bf16 outputs compared (max difference, fraction of elements that
differ), with the input's layout (strides, alignment) printed."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "moe-gan_cpsc541_amd"), os.path.join(REPO, "tests")]
import torch  # noqa: E402

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402
from steputil import gpu_step, make_inputs  # noqa: E402

orig = ops.conv2d


def conv2d(x, wpack, Cout, KH, KW, stride=1, pad=0, **kw):
    if Cout == 32 and KH == 3 and kw.get("out") is None and kw.get("in_scale") is None:
        torch.cuda.synchronize()
        y0 = orig(x, wpack, Cout, KH, KW, stride, pad, **kw)
        L.call("mg_set_tuning", 16, 1)
        y1 = orig(x, wpack, Cout, KH, KW, stride, pad, **kw)
        L.call("mg_set_tuning", 16, 0)
        torch.cuda.synchronize()
        d = (y0.float() - y1.float()).abs()
        print(f"conv Cout=32 x{tuple(x.shape)} stride{x.stride()} contig {x.is_contiguous()} "
              f"ptr%16 {x.data_ptr() % 16} out {y0.dtype}: max diff {float(d.max()):.3e} "
              f"({float((d > 0).float().mean()) * 100:.3f}% differ), |y| max {float(y1.float().abs().max()):.3e}",
              flush=True)
        return y0
    return orig(x, wpack, Cout, KH, KW, stride, pad, **kw)


ops.conv2d = conv2d
B, E = 8, 8
ts = gpu_step(E, 2, "bf16", "cuda")
real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=100 + B)
cu = lambda t: t.to("cuda")  # noqa: E731
out = ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
              cu(perm.int()), anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=0.001 * 1e-5)
torch.cuda.synchronize()
print("step done", flush=True)
