"""Minimal driver for profiling the fused SDF MLP kernels: ImplicitSurface.forward_with_nablas on
P points (default 524288 = one config-(b) step's samples), N launches.  Used under rocprofv3."""
import argparse
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', type=int, default=524288)
    ap.add_argument('--iters', type=int, default=5)
    ap.add_argument('--precision', default='f16x3')
    ap.add_argument('--mode', default='nabla', choices=['nabla', 'nabla0', 'fwd', 'radiance'])
    ap.add_argument('--stamps', action='store_true', help='print sdf4_kernel phase totals (stamps build)')
    a = ap.parse_args()
    from neurecon_amd.base import ImplicitSurface, RadianceNet
    torch.manual_seed(0)
    s = ImplicitSurface(W=256, D=8, skips=[4], W_geo_feat=256, radius_init=0.5, embed_multires=6,
                        precision=a.precision).cuda().eval()
    x = (torch.rand(a.points, 3, device='cuda') * 2 - 1) * 0.9
    with torch.no_grad():
        if a.mode == 'radiance':
            r = RadianceNet(D=4, W=256, W_geo_feat=256, embed_multires=-1, embed_multires_view=4,
                            precision=a.precision).cuda().eval()
            _, n, h = s.forward_with_nablas(x)
            fn = lambda: r.forward(x, x, n, h)
        elif a.mode == 'nabla0':  # sdf + nablas without the geometry feature (the sample launches)
            fn = lambda: s._run(x, nabla=True, feature=False)
        elif a.mode == 'fwd':
            fn = lambda: s.forward(x)
        else:
            fn = lambda: s.forward_with_nablas(x)
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / a.iters
    print(f'{a.mode} {a.precision}: {a.points} points, {dt * 1e3:.3f} ms/launch-set')
    if a.stamps:
        import ctypes
        import numpy as np
        from neurecon_amd import _lib as L
        buf = np.zeros(2048 * 8 * 6, dtype=np.uint64)
        nw = L.lib().nr_exp_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(buf.size))
        v = buf.reshape(-1, 6)
        v = v[v[:, 4] > 0]
        tot = v[:, :4].sum(1)
        names = ['vmem issue', 'mfma loop', 'bias+vmcnt', 'barrier']
        print(f'waves {len(v)} (per WG {nw // 6}), chunk iterations/wave {v[:, 4].mean():.0f}, '
              f'clocks/iteration {tot.mean() / v[:, 4].mean():.0f}')
        for i, n in enumerate(names):
            print(f'  {n:12s} {v[:, i].mean() / v[:, 4].mean():8.0f} clk/iter  {100 * v[:, i].sum() / tot.sum():5.1f} %')


if __name__ == '__main__':
    main()
