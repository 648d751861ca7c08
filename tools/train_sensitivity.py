"""Sensitivity of the reference training gradients (oracle, pinned to the reference by
tests/test_oracle_golden.py) to one-ulp noise on the positional encodings, for the NeRF++ training
fixture (default) or the VolSDF one (`volsdf_train` argument): the yardstick for the GPU gradient
bar in tests/test_gpu_train.py (CPU only)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests', 'golden')]
import weightgen as wg  # noqa: E402
from oracle import nets, rays  # noqa: E402
from oracle.train import neus_train_losses, volsdf_train_losses  # noqa: E402


def run(g, noise=0.0, seed=0):
    T = lambda a: torch.from_numpy(np.asarray(a))
    volsdf = 'eik_points' in g
    st = wg.volsdf_state(seed=int(g['seed']), beta_init=float(g['beta_init'])) if volsdf else \
        wg.neus_state(seed=int(g['seed']), use_outside_nerf=True)
    sd = {k: v.clone().requires_grad_(v.is_floating_point() and k != 'implicit_surface.obj_bounding_size')
          for k, v in st.items()}
    ro, rd, _ = rays.get_rays(T(g['c2w']), T(g['K']), int(g['H']), int(g['W']))
    orig = nets.embed
    if noise:
        gen = torch.Generator().manual_seed(seed)
        nets.embed = lambda x, n: (lambda e: e * (1 + noise * (torch.rand(e.shape, generator=gen) * 2 - 1)))(orig(x, n))
    try:
        if volsdf:
            losses, _ = volsdf_train_losses(sd, ro, rd, T(g['target_rgb']), T(g['eik_points']), d_all=T(g['d_vals']))
        else:
            losses, _ = neus_train_losses(sd, ro, rd, T(g['target_rgb']), T(g['target_mask']),
                                          N_outside=int(g['N_outside']))
        losses['total'].backward()
    finally:
        nets.embed = orig
    return {k: v.grad.double() for k, v in sd.items() if v.grad is not None}


def main():
    torch.set_num_threads(8)
    name = sys.argv[1] if len(sys.argv) > 1 else 'neus_train_nerfpp'
    g = dict(np.load(os.path.join(ROOT, 'tests', 'golden', name + '.npz')))
    a = run(g)
    for seed in range(2):
        b = run(g, 1.2e-7, seed)
        worst, worst_net = {}, {}
        net_max = {}
        for k in a:
            net = k.split('.')[0]
            net_max[net] = max(net_max.get(net, 0.0), a[k].abs().max().item())
        for k in a:
            net = k.split('.')[0]
            dev = (a[k] - b[k]).abs().max().item()
            worst[net] = max(worst.get(net, 0.0), dev / (a[k].abs().max().item() + 1e-30))
            worst_net[net] = max(worst_net.get(net, 0.0), dev / (net_max[net] + 1e-30))
        print(f'seed {seed}: max deviation / tensor scale', {k: f'{v:.2e}' for k, v in worst.items()})
        print(f'seed {seed}: max deviation / network scale', {k: f'{v:.2e}' for k, v in worst_net.items()})


if __name__ == '__main__':
    main()
