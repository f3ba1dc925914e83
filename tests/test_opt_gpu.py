"""Vectorised AdamW with the fused bf16 parameter shadow (mg_adamw_dev_shadow) against the scalar kernel
(mg_adamw_dev, pinned by the F8 full-step fixture) followed by a cast; ragged length (tail loop)."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from moegan_mi import _lib as L  # noqa: E402
from moegan_mi import ops  # noqa: E402

DEV = "cuda"


@pytest.mark.parametrize("n", [1, 7, 4096 + 3, 1 << 20])
@pytest.mark.parametrize("clip", [0.0, 0.8])
def test_adamw_shadow_matches_scalar(n, clip):
    g = torch.Generator(device=DEV).manual_seed(n)
    p = torch.randn(n, device=DEV, generator=g)
    gr = torch.randn(n, device=DEV, generator=g)
    m = torch.randn(n, device=DEV, generator=g) * 0.1
    v = torch.rand(n, device=DEV, generator=g) * 0.01
    step = torch.tensor([3], device=DEV, dtype=torch.int32)
    ss = (gr * gr).sum().view(1)
    ref = [t.clone() for t in (p, m, v)]
    L.call("mg_adamw_dev", ops.ptr(ref[0]), ops.ptr(gr), ops.ptr(ref[1]), ops.ptr(ref[2]), n, 2e-4, 0.5, 0.999,
           1e-8, 0.01, ops.ptr(step), ops.ptr(ss) if clip else None, clip, ops.S())
    shadow = torch.empty(n, device=DEV, dtype=torch.bfloat16)
    ops.adamw_dev(p, gr, m, v, 2e-4, 0.5, 0.999, 1e-8, 0.01, step, ss if clip else None, clip, shadow=shadow)
    torch.cuda.synchronize()
    assert torch.equal(p, ref[0]) and torch.equal(m, ref[1]) and torch.equal(v, ref[2])
    assert torch.equal(shadow, ref[0].to(torch.bfloat16))
