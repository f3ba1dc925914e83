"""Check every weight pack of the generator engine's prep() against a torch restatement (GPU, fp32): the conv
pack [Cout][kh][kw][Cin], the flipped data-gradient pack [Cin][KH-1-kh][KW-1-kw][Cout] and the demodulation sums
wsq[o][ci] = sum_taps W^2, at every max_res."""
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(HERE, "..", "moe-gan_cpsc541_amd"), os.path.join(HERE, "..")]


def main():
    from moegan_mi.engine_g import GeneratorEngine
    from moegan_mi.layout import frozen_rgb_prefixes, generator_shapes
    from moegan_mi.params import ParamStore
    from oracle.recipe import fill_state
    for R in (16, 32, 64, 128):
        shapes = generator_shapes(4, R)
        st = ParamStore(shapes, "cuda", frozen_prefixes=frozen_rgb_prefixes(R))
        st.load_state_dict({k: torch.from_numpy(v) for k, v in fill_state(shapes, 0).items()})
        ge = GeneratorEngine(st, 4)
        ge.prep()
        torch.cuda.synchronize()
        bad = []
        for pre, ent in ge.packs.items():
            W = st.view(pre + "weight").float()
            Cout, Cin, KH, KW = W.shape
            if "w" in ent:
                ref = W.permute(0, 2, 3, 1).reshape(Cout, -1)
                got = ent["w"].float()[:Cout]
                if not torch.equal(got, ref):
                    bad.append((pre, "w", float((got - ref).abs().max())))
            if "wflip" in ent:
                ref = W.flip(2, 3).permute(1, 2, 3, 0).reshape(Cin, -1)
                got = ent["wflip"].float()[:Cin]
                if not torch.equal(got, ref):
                    bad.append((pre, "wflip", float((got - ref).abs().max())))
            if "wsq" in ent:
                ref = W.pow(2).sum((2, 3))
                got = ent["wsq"][:Cout]
                if not torch.allclose(got, ref, rtol=1e-5, atol=1e-7):
                    bad.append((pre, "wsq", float((got - ref).abs().max())))
        print(f"R={R}: {len(ge.packs)} packed convs, mismatches: {bad}", flush=True)


if __name__ == "__main__":
    main()
