"""Which C-ABI call writes the router temperature gradients?  One bf16 C2 step (B=4) with every library call
followed by a read of the three temperature gradient slots; prints each call that changed one of them."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
from steputil import gpu_step, make_inputs  # noqa: E402


def main():
    from moegan_mi import _lib as L
    E, B, dev = 8, 4, "cuda"
    ts = gpu_step(E, 2, "bf16", dev)
    names = [n for n in ts.gs.offsets if n.endswith("router.temperature")]
    views = [ts.gs.gview(n) for n in names]
    real, text, z, eps_d, eps_g, perm = make_inputs(B, E, seed=104)
    cu = lambda t: t.to(dev)  # noqa: E731
    last = [None]
    log = []

    def hook(name, args, run):
        rc = run()
        torch.cuda.synchronize()
        cur = torch.cat([v.reshape(-1) for v in views]).cpu()
        if last[0] is not None and not torch.equal(cur, last[0]):
            d = (cur - last[0]).tolist()
            a = {n: v.value if hasattr(v, "value") else None for n, v in zip(L.ARGNAMES.get(name, []), args)}
            a = {k: v for k, v in a.items() if isinstance(v, int) and abs(v) < 1 << 40}
            log.append(f"{name} changed temperature grads by {['%.3e' % x for x in d]} args {a}")
        last[0] = cur
        return rc
    L.HOOK = hook
    ts.step(cu(real), cu(text), cu(z), [tuple(map(cu, e)) for e in eps_d], [tuple(map(cu, e)) for e in eps_g],
            cu(perm.int()), anneal=3.0, lr_g=2e-4, lr_d=2e-4, eff_kl_weight=1e-8)
    L.HOOK = None
    torch.cuda.synchronize()
    print("\n".join(log))


if __name__ == "__main__":
    main()
