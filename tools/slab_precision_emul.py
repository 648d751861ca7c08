"""CPU emulation: nabla error of the SDF network (oracle, float64) when the backward's softplus'
(sigmoid(100 z)) is stored in 16 bits instead of the fp32 slab of sdf4_kernel.

    python tools/slab_precision_emul.py

u16: fixed-point fraction round(s' * 65535) / 65535; f16: the slab's log2 form L = softplus * 100 / ln 2
rounded to f16, s' = 1 - 2^-L; u24c (r04, the kernel's format): c = 2^-L = 1 - s' as the 24-bit code
floor(c 2^23 + 0.5), s' = 1 - code 2^-23; fp32: s' rounded to fp32 (the reference's own storage).
65 536 uniform points in [-1, 1]^3, NeuS weights (seed 1)."""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]
import weightgen as wg  # noqa: E402
from oracle.nets import SDFNet  # noqa: E402


class _Q(torch.autograd.Function):
    @staticmethod
    def forward(ctx, z, mode):
        s = torch.sigmoid(100 * z)
        if mode == 'u16':
            s = torch.round(s * 65535) / 65535
        elif mode == 'f16':
            L = (F.softplus(z, beta=100) * 100 / torch.log(torch.tensor(2., dtype=z.dtype))).half().double()
            s = 1 - 2 ** (-L)
        elif mode == 'u24c':
            c = 1 - s
            s = 1 - torch.floor(c * 2 ** 23 + 0.5) / 2 ** 23
        elif mode == 'fp32':
            s = s.float().double()
        ctx.save_for_backward(s)
        return F.softplus(z, beta=100, threshold=20)

    @staticmethod
    def backward(ctx, g):
        s, = ctx.saved_tensors
        return g * s, None


def main():
    net = SDFNet(wg.neus_state(seed=1))
    net.layers = [(W.double(), b.double()) for W, b in net.layers]
    x = torch.rand(65536, 3, generator=torch.Generator().manual_seed(0), dtype=torch.float64) * 2 - 1
    _, n0, _ = net.forward_with_nablas(x)
    for mode in ('fp32', 'u24c', 'u16', 'f16'):
        net.act = lambda z, m=mode: _Q.apply(z, m)
        _, n1, _ = net.forward_with_nablas(x)
        e = (n1 - n0).abs()
        ok = (e <= 1e-4 * n0.abs() + 1e-5).all(-1).double().mean()
        print(f'{mode}: nabla max abs {e.max():.3e} mean {e.max(-1).values.mean():.3e}, '
              f'points within 1e-4 rel + 1e-5 abs {100 * ok:.3f} %')


if __name__ == '__main__':
    main()
