"""Progressive-generator fp32 diagnostic (GPU): per-block forward outputs of the device generator vs the fp64
oracle at R x R for B = 1 and 2 (which block first departs from fp32 accuracy)."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, ".."), os.path.join(HERE, "..", "tests")]
from oracle import aurora_cpu as O  # noqa: E402
from oracle.recipe import fill_state  # noqa: E402


def main(R, B):
    from moegan_mi.engine_g import GeneratorEngine
    from moegan_mi.layout import frozen_rgb_prefixes, generator_shapes
    from moegan_mi.params import ParamStore
    E, DEV = 4, "cuda"
    shapes = generator_shapes(E, R)
    vals = fill_state(shapes, 0)
    st = ParamStore(shapes, DEV, frozen_prefixes=frozen_rgb_prefixes(R))
    st.load_state_dict({k: torch.from_numpy(v) for k, v in vals.items()})
    ge = GeneratorEngine(st, E)
    ge.prep()
    g = torch.Generator().manual_seed(R)
    z, text = torch.randn(B, 512, generator=g), torch.randn(B, 512, generator=g)
    eps = [tuple(torch.randn(s, generator=g) for s in ((c, 128), (512, 128), (256, E))) for c in (512, 256, 128)]
    P = {n: torch.from_numpy(v).double() for n, v in vals.items()}
    ref, dev = {}, {}
    orig_cb, orig_mtm = O.conv_block, O.mtm

    def cb(x, w, P_, pre):
        y = orig_cb(x, w, P_, pre)
        ref[pre] = y.detach()
        return y

    def mtm(x, w, P_, pre, use_offset=True):
        y = orig_mtm(x, w, P_, pre, use_offset)
        ref[pre] = y.detach()
        return y
    O.conv_block, O.mtm = cb, mtm
    with torch.no_grad():
        img, half, _, _ = O.generator(z.double(), text.double(), P, [tuple(t.double() for t in e) for e in eps], True,
                                      3.0, 0.7)
    O.conv_block, O.mtm = orig_cb, orig_mtm
    ocb, omtm = ge.cb_fwd, ge.mtm_fwd

    def dcb(pre, x, w, save=True):
        y, s = ocb(pre, x, w, save)
        dev[pre] = y
        return y, s

    def dmtm(pre, x, w, resid=None, save=True, **kw):
        y, s = omtm(pre, x, w, resid=resid, save=save, **kw)
        dev[pre + ("+resid" if resid is not None else "")] = y
        return y, s
    ge.cb_fwd, ge.mtm_fwd = dcb, dmtm
    im, _, _, _, _, _ = ge.forward(z.to(DEV), text.to(DEV), [tuple(t.to(DEV) for t in e) for e in eps], 3.0, 0.7,
                                   train=True, save=False)
    torch.cuda.synchronize()
    print(f"R={R} B={B}")
    for pre, y in dev.items():
        key = pre.replace("+resid", "")
        if key not in ref:
            continue
        r = ref[key]
        if "+resid" in pre:  # mtm2 with the fused residual: compare against the block output
            r = ref[key.rsplit("mtm2.", 1)[0]]
        a = y[..., :r.shape[1]].permute(0, 3, 1, 2).double().cpu()
        err = float((a - r).norm() / r.norm())
        print(f"  {pre:55s} rel err {err:.2e}  {tuple(y.shape)} {y.dtype}")
    a = im[..., :3].permute(0, 3, 1, 2).double().cpu()
    print(f"  image rel err {float((a - img).norm() / img.norm()):.2e}")


if __name__ == "__main__":
    for R_, B_ in ((128, 1), (128, 2), (64, 2)):
        main(R_, B_)
