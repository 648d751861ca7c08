"""nr_wgrad timing on the training step's main shape (P = 65536, 256 x 256, one and two pairs) vs the
split-K hipBLASLt product it replaces; run under rocprofv3 --kernel-trace --stats to split the
kernel from its reduction.  NR_WGRAD_SLICES=<S> overrides the slice count (fewer, larger slices) in the wg_slices_env variant build
(tools/build_variants.py; NR_LIB=neurecon_amd/_exp/libnrhip_wg_slices_env.so)."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', type=int, default=65536)
    ap.add_argument('--no-blas', action='store_true', help='skip the hipBLASLt comparison')
    ap.add_argument('--blocked', action='store_true',
                    help='operands read as 16 x 16 blocked (the training step layout; timing only)')
    args = ap.parse_args()
    from neurecon_amd.training import _wg, _wgrad, _wgrad2
    g = torch.Generator().manual_seed(3)
    P = args.points
    a1, b1, a2, b2 = (torch.randn(P, 256, generator=g).cuda() for _ in range(4))
    cs = torch.empty(256, device='cuda')

    def t(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3
    from neurecon_amd import _lib as L
    blk = (L.WG_BLK_A0 | L.WG_BLK_A1 | L.WG_BLK_B0 | L.WG_BLK_B1) if args.blocked else 0
    for name, fn in (('nr_wgrad 1 pair', lambda: _wg([(a1, b1)], colsum=cs, blocked=blk)),
                     ('nr_wgrad 2 pairs', lambda: _wg([(a1, b1), (a2, b2)], colsum=cs, blocked=blk)),
                     ('hipBLASLt 1 pair', lambda: _wgrad(a1, b1)),
                     ('hipBLASLt 2 pairs', lambda: _wgrad2(a1, b1, a2, b2))):
        if args.no_blas and 'BLAS' in name:
            continue
        us = t(fn)
        npairs = 2 if '2' in name else 1
        print(f'P={P}{" blocked" if blk else ""} {name}: {us:.1f} us, {npairs * 2 * P * 256 * 4 / us / 1e6:.2f} TB/s of operands '
              f'(NR_WGRAD_SLICES={os.environ.get("NR_WGRAD_SLICES", "-")})', flush=True)


if __name__ == '__main__':
    main()
