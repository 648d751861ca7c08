"""Throughput of the §8f widening rows on one GPU (not the headline bench):
  * surface_render (sphere tracing, 20 iterations) of a full 800x600 frame (480,000 rays, config-(d) camera);
  * surface_render (root finding: 256-step march + secant) of the same frame, chunked and full march;
  * extract_mesh's SDF grid query at N=512 (134 M forward SDF evaluations).
Prints one JSON line per workload with per-kernel HIP-event timings from the library.

    python tools/bench_surface.py [--reps 3]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import torch  # noqa: E402

import weightgen as wg  # noqa: E402
from helpers import neus_model  # noqa: E402
from neurecon_amd import _lib as L, rend_util  # noqa: E402
from neurecon_amd.mesh_util import sdf_grid  # noqa: E402
from neurecon_amd.ray_casting import surface_render  # noqa: E402

FWD_FLOP = 2 * 524544      # SDF forward, per point
NAB_FLOP = 2 * 983552      # SDF forward + reverse pass
RAD_FLOP = 2 * 271360      # radiance MLP


def timed(fn, reps):
    fn()
    torch.cuda.synchronize()
    L.profile_enable(True)
    L.profile_read()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    prof = L.profile_read()
    L.profile_enable(False)
    return out, dt, {k: (v[0] / reps, v[1] / reps) for k, v in prof.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--grid-n', type=int, default=512)
    args = ap.parse_args()
    dev = 'cuda:0'
    m = neus_model(wg.neus_state(seed=4), precision='f16x3', device=dev)
    H, W, f, dist = wg.CAMERAS['d']
    with torch.no_grad():
        ro, rd, _ = rend_util.get_rays(wg.look_at_c2w(dist)[None].to(dev), wg.intrinsics(f, H, W)[None].to(dev), H, W)
        (rgb, depth, ex), dt, prof = timed(
            lambda: surface_render(ro, rd, m, calc_normal=True, batched=True, ray_casting_algo='sphere_tracing'),
            args.reps)
        hits = int(ex['mask_surface'].sum().item())
        print(json.dumps(dict(workload='surface_render sphere_tracing 800x600 (480000 rays, 20 iters)', rays=H * W,
                              hit_rays=hits, ms=round(dt * 1e3, 3), rays_per_s=round(H * W / dt, 1),
                              kernels={k: dict(launches=v[0], ms=round(v[1], 3)) for k, v in prof.items()})))
        # root finding (ray_casting.py:35-160): the 256-step march evaluated in chunks of 32 steps over the
        # rays without a sign change so far, against the single launch over every step (_full_march)
        for full in (True, False):
            (rgb, depth, ex), dt, prof = timed(
                lambda: surface_render(ro, rd, m, calc_normal=True, batched=True, ray_casting_algo='root_finding',
                                       ray_casting_cfgs={'_full_march': full}), args.reps)
            hits = int(ex['mask_surface'].sum().item())
            print(json.dumps(dict(workload='surface_render root_finding 800x600 (480000 rays, 256-step march + 8 '
                                           'secant steps), ' + ('full march (every step of every ray)' if full else
                                                                'chunked march (32-step chunks over rays without a '
                                                                'crossing)'),
                                  rays=H * W, hit_rays=hits, ms=round(dt * 1e3, 3), rays_per_s=round(H * W / dt, 1),
                                  kernels={k: dict(launches=v[0], ms=round(v[1], 3)) for k, v in prof.items()})))
        N = args.grid_n
        out, dt, prof = timed(lambda: sdf_grid(m.implicit_surface, 2.0, N), args.reps)
        kms = sum(v[1] for k, v in prof.items() if k.startswith('sdf'))
        print(json.dumps(dict(workload=f'extract_mesh SDF grid N={N} ({N ** 3} points)', points=N ** 3,
                              ms=round(dt * 1e3, 3), points_per_s=round(N ** 3 / dt, 1),
                              sdf_kernel_tflops=round(N ** 3 * FWD_FLOP / (kms * 1e-3) / 1e12, 2) if kms else None,
                              kernels={k: dict(launches=v[0], ms=round(v[1], 3)) for k, v in prof.items()})))


if __name__ == '__main__':
    main()
