"""mg_step_inputs (csrc/mg_rng.hip): a step's router noise and mismatched-caption permutation in one launch.
The permutation is a permutation of 0..B-1 for every B up to 4096 (ragged, powers of two, 1), depends only on its
seed and differs between seeds; the noise has N(0, 1) moments (mean, variance, the one-sigma mass, the tails) over
both buffers, is reproducible for a seed, and the two buffers do not repeat each other."""
import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("B", [1, 2, 7, 256, 1000, 4096])
def test_permutation(B):
    from moegan_mi import ops
    a = torch.empty(10, device=DEV)
    b = torch.empty(6, device=DEV)
    p1 = torch.empty(B, device=DEV, dtype=torch.int32)
    p2 = torch.empty_like(p1)
    p3 = torch.empty_like(p1)
    ops.step_inputs(a, b, p1, 1, 11)
    ops.step_inputs(a, b, p2, 2, 11)
    ops.step_inputs(a, b, p3, 1, 12)
    torch.cuda.synchronize()
    assert torch.equal(torch.sort(p1.long()).values.cpu(), torch.arange(B))
    assert torch.equal(p1, p2)  # the permutation depends on its own seed only
    if B > 2:
        assert not torch.equal(p1, p3)


def test_normals():
    from moegan_mi import ops
    na, nb = 600_001, 400_000
    a = torch.empty(na, device=DEV)
    b = torch.empty(nb, device=DEV)
    perm = torch.empty(8, device=DEV, dtype=torch.int32)
    ops.step_inputs(a, b, perm, 123, 5)
    a2, b2 = torch.empty_like(a), torch.empty_like(b)
    ops.step_inputs(a2, b2, perm, 123, 5)
    a3, b3 = torch.empty_like(a), torch.empty_like(b)
    ops.step_inputs(a3, b3, perm, 124, 5)
    torch.cuda.synchronize()
    assert torch.equal(a, a2) and torch.equal(b, b2)
    assert not torch.equal(a, a3)
    x = torch.cat([a, b]).double()
    n = x.numel()
    assert bool(torch.isfinite(x).all())
    assert abs(float(x.mean())) < 5 / math.sqrt(n)
    assert abs(float(x.var()) - 1.0) < 5 * math.sqrt(2.0 / n)
    p1 = float((x.abs() < 1).double().mean())
    assert abs(p1 - 0.682689) < 5 * math.sqrt(0.682689 * 0.317311 / n)
    p3 = float((x.abs() > 3).double().mean())
    assert abs(p3 - 0.0026998) < 5 * math.sqrt(0.0026998 / n)
    # the second buffer continues the stream, it does not restart it
    assert float((a[:1000] - b[:1000]).abs().max()) > 0.1
