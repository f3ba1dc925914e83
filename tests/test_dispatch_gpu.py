"""Expert dispatch (mg_moe_dispatch: per-expert position lists for the grouped expert GEMMs, t2i_moe_gan.py:465-470
dispatch of the top-k assignments): bit-exact against a stable sort of the assignments by expert.  Covers
E = 4 / 8 / 16 / 32 (C2: 8, C5: 32), k = 1 / 2 / 4, ragged chunk tails (the kernels work in 1024-assignment
chunks), experts that receive no assignment, the skewed routing of an early-training router, and a size whose
chunk-count table exceeds the parallel scan's LDS table (the serial scan then runs), and the largest table the parallel scan takes
(E=32, k=4, T=131072: 512 chunks x 32 = 16384 counts, ~70 KB of dynamic LDS, within gfx950's 160 KB per CU).
Both launch forms: count + scatter-with-folded-scan (default) and count / scan / scatter (tuning slot 18 = 1)."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _reference(topi, gate, E, bm):
    flat = topi.reshape(-1).long().cpu()
    perm = torch.sort(flat, stable=True).indices
    pos_of = torch.empty_like(perm)
    pos_of[perm] = torch.arange(flat.numel())
    cnt = torch.bincount(flat, minlength=E)
    row_off = torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0)])
    tiles = (cnt + bm - 1) // bm
    tile_off = torch.cat([torch.zeros(1, dtype=torch.long), tiles.cumsum(0)])
    return row_off, tile_off, perm, pos_of, gate.reshape(-1).cpu()[perm]


@pytest.mark.parametrize("E,k,T,skew", [(8, 2, 65536, False), (32, 4, 65536, False), (32, 4, 4096, True),
                                        (16, 2, 3001, False), (4, 1, 1, False), (8, 2, 5, True),
                                        (32, 4, 16384, True), (4, 4, 777, False), (32, 4, 140000, False),
                                        (32, 4, 131072, False)])
@pytest.mark.parametrize("three", [0, 1])
def test_dispatch_matches_stable_sort(E, k, T, skew, three):
    from moegan_mi import _lib as L
    from moegan_mi import ops
    g = torch.Generator(device=DEV).manual_seed(E * 1000 + k * 10 + T)
    if skew:  # a few experts take most tokens; the upper half of the experts gets none
        w = torch.zeros(E, device=DEV)
        w[: max(1, E // 2)] = torch.linspace(8.0, 1.0, max(1, E // 2), device=DEV)
        scores = torch.rand(T, E, device=DEV, generator=g) * w
    else:
        scores = torch.rand(T, E, device=DEV, generator=g)
    topi = scores.topk(k, dim=1).indices.int().contiguous()
    gate = torch.rand(T, k, device=DEV, generator=g)
    L.call("mg_set_tuning", 18, three)
    try:
        row_off, tile_off, perm, pos_of, gate_pos = ops.moe_dispatch(topi, gate, E)
        torch.cuda.synchronize()
    finally:
        L.call("mg_set_tuning", 18, 0)
    r_row, r_tile, r_perm, r_pos, r_gate = _reference(topi, gate, E, 128)
    assert torch.equal(row_off.cpu().long(), r_row)
    assert torch.equal(tile_off.cpu().long(), r_tile)
    assert torch.equal(perm.cpu().long(), r_perm)
    assert torch.equal(pos_of.cpu().long(), r_pos)
    assert torch.equal(gate_pos.cpu(), r_gate)
