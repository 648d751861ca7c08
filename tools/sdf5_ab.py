"""A/B of the SDF forward kernels: sdf4_kernel<false,false,0> (16x16x32 MFMA, two waves per SIMD) vs
sdf5_fwd_kernel (32x32x16 MFMA, one wave per SIMD; nr_sdf5_enable), alternated on the same points, plus
their difference and both against a float64 evaluation of the same net on a subset.

    python tools/sdf5_ab.py [--points 524288] [--iters 20] [--rounds 3]
"""
import argparse
import ctypes
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', type=int, default=524288)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--variants', default='0,1,2', help='nr_sdf5_enable values: 0 = sdf4_kernel, 1 = sdf5, 2.. experiments')
    a = ap.parse_args()
    from neurecon_amd import _lib as L
    from neurecon_amd.base import ImplicitSurface
    torch.manual_seed(0)
    s = ImplicitSurface(W=256, D=8, skips=[4], W_geo_feat=256, radius_init=0.5, embed_multires=6,
                        precision='f16x3').cuda().eval()
    x = (torch.rand(a.points, 3, device='cuda') * 2 - 1) * 0.9
    lib = L.lib()
    out = {}
    vs = [int(v) for v in a.variants.split(',')]
    times = {v: [] for v in vs}
    with torch.no_grad():
        for r in range(a.rounds):
            for v in vs:
                lib.nr_sdf5_enable(v)
                y = s.forward(x)
                torch.cuda.synchronize()
                t = time.perf_counter()
                for _ in range(a.iters):
                    s.forward(x)
                torch.cuda.synchronize()
                times[v].append((time.perf_counter() - t) / a.iters * 1e3)
                out[v] = y.clone()
    lib.nr_sdf5_enable(0)
    d = (out[1] - out[0]).abs()
    for v in vs:
        print(f'points {a.points}: variant {v} ms {["%.3f" % t for t in times[v]]}')
    print(f'|sdf5 - sdf4| max {float(d.max()):.3e} mean {float(d.mean()):.3e}; |sdf| max {float(out[0].abs().max()):.3f}')
    # float64 truth on a subset: the same net (its state_dict) through the oracle's SDFNet in float64
    # (test infrastructure, used here as the checker only)
    sys.path[:0] = [os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
    from oracle.nets import SDFNet
    n = 16384
    ref = SDFNet({'implicit_surface.' + k: v.detach().cpu() for k, v in s.state_dict().items()})
    ref.layers = [(W.double(), b.double()) for W, b in ref.layers]
    with torch.no_grad():
        sr = ref.forward(x[:n].double().cpu())
    sr = sr[0] if isinstance(sr, tuple) else sr
    for v in [u for u in vs if u <= 2]:
        e = (out[v][:n].double().cpu().reshape(-1) - sr.reshape(-1)).abs()
        print(f'variant {v}: |sdf - f64| max {float(e.max()):.3e} mean {float(e.mean()):.3e}')
    macs = 459_008  # forward without the feature rows (bench.MAC_SDF_FWD_NOFEAT)
    for v in vs:
        t = min(times[v])
        tf = a.points * macs * 2 / (t * 1e-3) / 1e12
        print(f'variant {v}: best {t:.3f} ms = {tf:.1f} TF/s = {tf / 833.3:.3f} of the f16x3 peak')


if __name__ == '__main__':
    main()
