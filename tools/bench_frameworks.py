"""Timing of the VolSDF and UNISURF render paths (secondary §8 rows) on the config-(b) camera:
4096 rays, seeded random-init weights, render mode.  Prints per-kernel device time (HIP events)."""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))


def rays(dev, key='b'):
    import weightgen as wg
    from neurecon_amd import rend_util
    H, W, f, dist = wg.CAMERAS[key]
    c2w = wg.look_at_c2w(dist)[None].to(dev)
    K = wg.intrinsics(f, H, W)[None].to(dev)
    ro, rd, _ = rend_util.get_rays(c2w, K, H, W)
    return ro, rd


def mlp_roofline(ks, precision, rad_in):
    """per MLP kernel type: launches, ms, executed TFLOP/s and fraction of the matrix peak (bench.py's
    MAC counts; the radiance net's first layer has rad_in inputs)"""
    import bench as B
    peak = B.FP32_MFMA_PEAK_TFLOPS if precision == 'fp32' else B.F16X3_PEAK_TFLOPS
    mac = dict(B.KERNEL_MAC, radiance=rad_in * 256 + 3 * 256 * 256 + 3 * 256)
    out = {}
    for name, (n, ms, units) in ks.items():
        # sdf_fwd runs inside VolSDF's sampler on device-side counts: its recorded units are the
        # launch capacity, not the points evaluated, so no rate is derived for it
        if name in mac and name != 'sdf_fwd' and n and ms > 0:
            tf = units * 2.0 * mac[name] / (ms * 1e-3) / 1e12
            out[name] = {'launches': n, 'ms': round(ms, 3), 'tflops': round(tf, 1), 'frac': round(tf / peak, 4)}
    return out


def timeit(fn, steps, warmup):
    from neurecon_amd import _lib as L
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    L.profile_read()
    L.profile_enable(True)
    t = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / steps
    L.profile_enable(False)
    return dt, L.profile_read()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--steps', type=int, default=5)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--precision', default='f16x3')
    ap.add_argument('--configs', action='store_true', help='also time BASELINE configs (c), (d), (e)')
    ap.add_argument('--only', default='', help="with --configs: just these of 'c', 'd', 'e' (no framework leg)")
    args = ap.parse_args()
    if args.only:
        print(json.dumps(configs(args), default=str), flush=True)
        return
    import weightgen as wg
    from helpers import unisurf_model, volsdf_model
    dev = torch.device('cuda')
    ro, rd = rays(dev)
    out = {}
    from neurecon_amd.frameworks import unisurf, volsdf
    mv = volsdf_model(wg.volsdf_state(seed=2, beta_init=0.1), 0.1, precision=args.precision)
    kw = dict(near=0.0, far=6.0, batched=True, calc_normal=True, detailed_output=False, N_samples=128,
              N_importance=64, max_upsample_steps=6)
    with torch.no_grad():
        dt, ks = timeit(lambda: volsdf.volume_render(ro, rd, mv, **kw), args.steps, args.warmup)
        _, _, ex = volsdf.volume_render(ro, rd, mv, **dict(kw, detailed_output=True))
    it = ex['iter_usage'].flatten()
    out['volsdf'] = {'rays_per_s': ro.shape[1] / dt, 'ms': dt * 1e3, 'kernels': ks,
                     'roofline': mlp_roofline(ks, args.precision, 265),
                     'iter_usage': {str(k): int((it == k).sum()) for k in it.unique().tolist()}}
    mu = unisurf_model(wg.unisurf_state(seed=3), precision=args.precision)
    with torch.no_grad():
        dt, ks = timeit(lambda: unisurf.volume_render(ro, rd, mu, batched=True, calc_normal=True,
                                                      detailed_output=False, logit_tau=0.0), args.steps, args.warmup)
    out['unisurf'] = {'rays_per_s': ro.shape[1] / dt, 'ms': dt * 1e3, 'kernels': ks,
                      'roofline': mlp_roofline(ks, args.precision, 265)}
    print(json.dumps(out, default=str), flush=True)
    if args.configs:
        print(json.dumps(configs(args), default=str), flush=True)


def configs(args):
    """BASELINE.json configs (c), (d), (e) on one GPU: VolSDF 2048 rays x (128 + 128) error-bounded
    samples (32x64 camera); NeuS + NeRF++ full 800x600 frame (480,000 rays, 64 + 64 + 32 outside);
    UNISURF 4096 rays (64x64 camera, secant root finding)."""
    import weightgen as wg
    from helpers import neus_model, unisurf_model, volsdf_model
    from neurecon_amd.frameworks import neus, unisurf, volsdf
    dev = torch.device('cuda')
    res = {}
    want = set(args.only) if getattr(args, 'only', '') else {'c', 'd', 'e'}
    if 'c' in want:
        res.update(config_c(args, dev))
    if 'd' in want:
        res.update(config_d(args, dev))
    if 'e' in want:
        res.update(config_e(args, dev))
    return res


def config_c(args, dev):
    import weightgen as wg
    from helpers import volsdf_model
    from neurecon_amd.frameworks import volsdf
    res = {}
    ro, rd = rays(dev, 'c')
    mv = volsdf_model(wg.volsdf_state(seed=5, beta_init=1e-3), 1e-3, precision=args.precision)
    kw = dict(near=0.0, far=6.0, batched=True, calc_normal=True, detailed_output=False, N_samples=128,
              N_importance=128, max_upsample_steps=6)
    with torch.no_grad():
        dt, ks = timeit(lambda: volsdf.volume_render(ro, rd, mv, **kw), args.steps, args.warmup)
    res['c_volsdf_2048x256'] = {'rays': ro.shape[1], 'rays_per_s': ro.shape[1] / dt, 'ms': dt * 1e3,
                                'roofline': mlp_roofline(ks, args.precision, 265), 'kernels': ks}
    return res


def config_d(args, dev):
    import weightgen as wg
    from helpers import neus_model
    from neurecon_amd.frameworks import neus
    res = {}
    ro, rd = rays(dev, 'd')
    mn = neus_model(wg.neus_state(seed=4, use_outside_nerf=True), use_outside_nerf=True, precision=args.precision)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, N_samples=64,
              N_importance=64, N_outside=32)
    with torch.no_grad():
        dt, ks = timeit(lambda: neus.volume_render(ro, rd, mn, **kw), max(1, args.steps // 2), 1)
    res['d_neus_nerfpp_800x600'] = {'rays': ro.shape[1], 'rays_per_s': ro.shape[1] / dt, 'ms': dt * 1e3,
                                    'roofline': mlp_roofline(ks, args.precision, 289)}
    return res


def config_e(args, dev):
    import weightgen as wg
    from helpers import unisurf_model
    from neurecon_amd.frameworks import unisurf
    res = {}
    ro, rd = rays(dev, 'e')
    mu = unisurf_model(wg.unisurf_state(seed=3), precision=args.precision)
    with torch.no_grad():
        dt, ks = timeit(lambda: unisurf.volume_render(ro, rd, mu, batched=True, calc_normal=True,
                                                      detailed_output=False, logit_tau=0.0), args.steps, args.warmup)
    res['e_unisurf_4096'] = {'rays': ro.shape[1], 'rays_per_s': ro.shape[1] / dt, 'ms': dt * 1e3,
                             'roofline': mlp_roofline(ks, args.precision, 265)}
    return res


if __name__ == '__main__':
    main()
