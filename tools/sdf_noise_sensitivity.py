"""How often does the reference's own sampler keep identical samples when its SDF moves by rounding?
The oracle's NeuS sampler (pinned to the reference) is run on a config's rays with and without
relative noise eps * N(0, 1) on every SDF value it evaluates; the fraction of rays whose sample
(mid-point) depths stay within 1e-5 rel + 1e-6 is the reference's own sensitivity -- the floor any
implementation that is not bit-identical to its fp32 CPU arithmetic can expect.

    python tools/sdf_noise_sensitivity.py --config d --rays 2048 --eps 1e-7 --seeds 5
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='d', choices=['b', 'd'])
    ap.add_argument('--rays', type=int, default=2048)
    ap.add_argument('--eps', type=float, default=1e-7)
    ap.add_argument('--seeds', type=int, default=5)
    ap.add_argument('--abs', action='store_true', help='absolute noise eps * N(0, 1) instead of relative')
    ap.add_argument('--golden', default='', help='take the rays of tests/golden/<name>.npz (e.g. neus_b, 64 rays)')
    args = ap.parse_args()
    import torch.nn.functional as F
    import weightgen as wg
    from oracle import rays as orays
    from oracle.neus import NeuSOracle
    from oracle import rays as R
    torch.set_num_threads(8)
    H, W, f, dist = wg.CAMERAS[args.config]
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    if args.golden:
        g = np.load(os.path.join(ROOT, 'tests', 'golden', args.golden + '.npz'))
        ro, rd = torch.from_numpy(g['rays_o']), torch.from_numpy(g['rays_d'])
    elif args.rays < H * W:  # as tests/test_gpu_nerf.py: rays spread evenly over the frame
        idx = torch.linspace(0, H * W - 1, args.rays).round().long()
        ro, rd = ro[:, idx].contiguous(), rd[:, idx].contiguous()
    outside = args.config == 'd'
    sd = wg.neus_state(seed=4 if outside else 1, use_outside_nerf=outside)
    orc = NeuSOracle(sd, use_outside_nerf=outside)
    o = ro.float()
    d = F.normalize(rd.float(), dim=-1)
    near, far = R.near_far_from_sphere(o, d, r=1.0)
    clean_sdf = orc.sdf_net.sdf
    with torch.no_grad():
        base = orc.sample_depths(o, d, near, far)
    mid0 = 0.5 * (base[..., 1:] + base[..., :-1])
    fracs, tights = [], []
    for seed in range(args.seeds):
        g = torch.Generator().manual_seed(100 + seed)

        def noisy(x, _g=g):
            s = clean_sdf(x)
            n = args.eps * torch.randn(s.shape, generator=_g)
            return s + n if args.abs else s * (1 + n)
        orc.sdf_net.sdf = noisy
        with torch.no_grad():
            dn = orc.sample_depths(o, d, near, far)
        orc.sdf_net.sdf = clean_sdf
        mid = 0.5 * (dn[..., 1:] + dn[..., :-1])
        same = ((mid - mid0).abs() <= 1e-5 * mid0.abs() + 1e-6).all(-1).reshape(-1)
        fracs.append(float(same.float().mean()))
        # tests/test_gpu_parity.py::test_neus_render_vs_golden's `tight`: every depth within 1e-6 relative
        tights.append(float(((mid - mid0).abs() <= 1e-6 * mid0.abs()).all(-1).float().mean()))
        print(f'seed {seed}: identical samples on {fracs[-1] * 100:.2f}% of rays, depths within 1e-6 rel on '
              f'{tights[-1] * 100:.2f}%', file=sys.stderr, flush=True)
    print(json.dumps({'config': args.config, 'rays': int(ro.shape[1]), 'eps': args.eps, 'abs': args.abs,
                      'identical_frac': fracs, 'min': min(fracs), 'mean': float(np.mean(fracs)),
                      'tight_frac': tights, 'tight_min': min(tights)}))


if __name__ == '__main__':
    main()
