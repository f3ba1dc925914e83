"""CPU: the fp64 restatement of the router backward's temperature term (steputil.router_temp_terms, the formula
k_router_bwd implements) equals autograd through the oracle router (t2i_moe_gan.py:374-389) and the top-k
combine weights, for the dense reference routing and for top-k."""
import pytest
import torch

from oracle import aurora_cpu as O
from steputil import OracleTempTap, router_temp_terms


@pytest.mark.parametrize("E,k", [(4, 4), (8, 2), (8, 8), (16, 2)])
def test_router_temp_terms_vs_autograd(E, k):
    g = torch.Generator().manual_seed(E * 10 + k)
    C, T, anneal = 32, 48, 3.0
    P = {"r.feature_mu": torch.randn(C, 128, generator=g) * 0.3, "r.feature_rho": torch.full((C, 128), -4.0),
         "r.text_mu": torch.randn(512, 128, generator=g) * 0.1, "r.text_rho": torch.full((512, 128), -4.0),
         "r.combined_mu": torch.randn(256, E, generator=g) * 0.3, "r.combined_rho": torch.full((256, E), -4.0),
         "r.temperature": torch.tensor([1.1], requires_grad=True)}
    eps = (torch.randn(C, 128, generator=g), torch.randn(512, 128, generator=g), torch.randn(256, E, generator=g))
    f, t = torch.randn(T, C, generator=g, dtype=torch.float64), torch.randn(T, 512, generator=g, dtype=torch.float64)
    P = {n: (v.double().detach().requires_grad_(v.requires_grad)) for n, v in P.items()}
    eps = tuple(e.double() for e in eps)
    R = torch.randn(T, E, generator=g, dtype=torch.float64)  # upstream gradient of the combine weights
    coef = torch.randn(E, generator=g, dtype=torch.float64) * 0.1  # e.g. the balance loss's d/dprobs
    with OracleTempTap() as tap:
        probs, logits = O.router(f, t, P, "r.", eps, True, anneal)
        tap.store["blk"] = tap.store.pop("r")
        gate = O.topk_route(probs, k)
        loss = (gate * R).sum() + (probs * coef).sum()
        loss.backward()
        auto = float(P["r.temperature"].grad)
        ti = torch.topk(probs.detach(), k, dim=1).indices
        te = min(max(float(P["r.temperature"]) * anneal, 0.5), 5.0)
        terms = router_temp_terms(logits.detach(), ti, R.gather(1, ti), coef, te, anneal, k)
        assert abs(float(terms.sum()) - auto) <= 1e-9 * max(1.0, float(terms.abs().sum())), (float(terms.sum()), auto)
        # the tap's per-token terms read from the retained logits gradient give the same sum
        assert abs(float(tap.terms("blk").sum()) - auto) <= 1e-9 * max(1.0, float(terms.abs().sum()))
