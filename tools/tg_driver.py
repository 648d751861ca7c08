"""Timing driver for the training layer GEMM (tgemm_kernel, nr_train_gemm) on the NeuS training step's
shapes: P points (default 131 072 = 512 rays x (128 samples + 127 mid-points), rounded to a tile
multiple), 16 x 16 blocked tensors, the SDF net's render pack.  Times each epilogue mode (the F1
softplus forward, the B7 nabla-chain MUL, the B7 adjoint SPADJ with the tangent term) over N launches;
with a stamps build (tools/build_variants.py stamps, NR_LIB=...) prints the per-phase shader-clock
split of one launch: tile start (input load + split), VMEM issue, MFMA loop, counted wait, epilogue
VALU, barrier.

    python tools/tg_driver.py [--points 131072] [--iters 20] [--stamps]"""
import argparse
import ctypes
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--points', type=int, default=131072)
    ap.add_argument('--iters', type=int, default=20)
    ap.add_argument('--stamps', action='store_true')
    a = ap.parse_args()
    from neurecon_amd import _lib as L
    from neurecon_amd import training as T
    from neurecon_amd.base import ImplicitSurface
    torch.manual_seed(0)
    dev = torch.device('cuda:0')
    s = ImplicitSurface(W=256, D=8, skips=[4], W_geo_feat=256, radius_init=0.5, embed_multires=6,
                        precision='f16x3').to(dev)
    desc, packed = s.nr_packed(dev)
    info = T._op_info('sdf', desc, 18)
    op = lambda i: packed.data_ptr() + info[i][0]
    shp = lambda i: (info[i][1], 0, info[i][2], 0)
    P = a.points
    st = L.stream_of(dev)
    R = lambda: torch.rand(P, 256, device=dev) * 0.5
    X, Y, Y2, S, G, ZD = R(), R(), R(), R(), R(), R()
    B = L.BLK_X1 | L.BLK_Y | L.BLK_Y2 | L.BLK_A | L.BLK_G | L.BLK_ZD
    cases = {
        'SOFTPLUS F1 (x1, y, y2)': lambda: T._tg(op(1), P, shp(1), L.TG_SOFTPLUS, X, 256, 256, Y, 256, y2=Y2, ldy2=256,
                                                stream=st, blocked=B & (L.BLK_X1 | L.BLK_Y | L.BLK_Y2)),
        'MUL B7 (x1, a, y2)': lambda: T._tg(op(9), P, shp(9), L.TG_MUL, X, 256, 256, None, 0, y2=Y2, ldy2=256, a=S,
                                           lda=256, stream=st, blocked=B & (L.BLK_X1 | L.BLK_Y2 | L.BLK_A)),
        'SPADJ B7 (x1, a, g, zd, y)': lambda: T._tg(op(9), P, shp(9), L.TG_SPADJ, X, 256, 256, Y, 256, a=S, lda=256,
                                                   g=G, ldg=256, zd=ZD, ldzd=256, g_scaled=True, stream=st,
                                                   blocked=B & (L.BLK_X1 | L.BLK_Y | L.BLK_A | L.BLK_G | L.BLK_ZD)),
    }
    for name, fn in cases.items():
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.iters
        nbytes = {'SOFTPLUS': 3, 'MUL': 3, 'SPADJ': 5}[name.split()[0]] * 1024 * P
        print(f'{name:28s} {dt * 1e6:8.1f} us/launch  {nbytes / dt / 1e12:5.2f} TB/s of tensor bytes', flush=True)
        if a.stamps:
            fn()
            torch.cuda.synchronize()
            buf = np.zeros(2048 * 8 * 6, dtype=np.uint64)
            nw = L.lib().nr_exp_stamps(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_int(buf.size))
            v = buf.reshape(-1, 6)[:min(P // 128, 256) * 8]
            tot = v.sum(1)
            names = ['VMEM issue', 'MFMA loop', 'bias + wait', 'barrier', 'tile start', 'epilogue VALU']
            order = [4, 0, 1, 2, 5, 3]
            print(f'   waves {len(v)}, clocks per wave {tot.mean():.0f}')
            for i in order:
                print(f'     {names[i]:14s} {100 * v[:, i].sum() / tot.sum():5.1f} %  ({v[:, i].mean():9.0f} clk/wave)')


if __name__ == '__main__':
    main()
