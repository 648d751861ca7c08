"""SDF / nabla error of the HIP SDF kernel (fp32 and f16x3) against the oracle network evaluated in
float64, on uniform points in [-1, 1]^3 and on points within 0.05 of the zero level set.
Run on a GPU box; NR_LIB selects the library (tools/build_variants.py experiments)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import weightgen as wg  # noqa: E402
from helpers import neus_model  # noqa: E402
from oracle.nets import SDFNet  # noqa: E402


def main():
    sd = wg.neus_state(seed=1)
    ref = SDFNet(sd)
    ref.layers = [(W.double(), b.double()) for W, b in ref.layers]
    g = torch.Generator().manual_seed(0)
    x = torch.rand(65536, 3, generator=g, dtype=torch.float64) * 2 - 1
    s_ref, nab_ref, _ = ref.forward_with_nablas(x)
    near = x[(s_ref.abs() < 0.05)][:16384]
    sets = {'uniform': (x, s_ref, nab_ref)}
    s2, n2, _ = ref.forward_with_nablas(near)
    sets['near-surface'] = (near, s2, n2)
    for prec in ('fp32', 'f16x3'):
        m = neus_model(sd, precision=prec)
        for name, (p, sr, nr) in sets.items():
            with torch.no_grad():
                s, nab, _ = m.implicit_surface.forward_with_nablas(p.float().cuda())
            es = (s.double().cpu() - sr).abs()
            en = (nab.double().cpu() - nr).abs().max(-1).values
            print(f'{prec:6s} {name:13s} n={p.shape[0]:6d} sdf max {es.max():.3e} mean {es.mean():.3e} '
                  f'| nabla max {en.max():.3e} mean {en.mean():.3e}')


if __name__ == '__main__':
    main()
