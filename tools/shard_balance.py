"""Per-shard cost of the strong-scaled config-(d) frame on ONE GPU: the 800x600 NeuS + NeRF++ frame
(bench.py frame_d_setup) split into 8 shares the way render_sharded would deal them at world size 8
-- contiguous ranges (shard_bounds) or block-cyclic (cyclic_index) -- each share rendered alone and
timed (warm-up + median of 3, device synchronised).  Reports max/mean and the implied 8-GPU ceiling
= whole-frame time / slowest share.

    python tools/shard_balance.py [--world 8] [--block 1024]
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--world', type=int, default=8)
    ap.add_argument('--block', type=int, default=1024)
    ap.add_argument('--reps', type=int, default=3)
    ap.add_argument('--workspace-gb', type=float, default=16.0)
    args = ap.parse_args()
    import bench as B
    from neurecon_amd import dist as nd
    from neurecon_amd.frameworks.neus import NeuS, volume_render
    dev = torch.device('cuda')
    torch.manual_seed(0)
    surf = dict(use_siren=False, embed_multires=6, radius_init=0.5, geometric_init=True, D=8, W=256, skips=[4],
                precision='f16x3')
    rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=4, use_view_dirs=True, D=4, W=256, skips=[],
               precision='f16x3')
    model = NeuS(variance_init=0.05, speed_factor=10.0, W_geo_feat=256, use_outside_nerf=True, obj_bounding_radius=1.0,
                 surface_cfg=surf, radiance_cfg=rad).to(dev).eval()
    ro, rd = B.camera_for(dev, 600, 800, 800.0, 2.0)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, perturb=False,
              N_samples=64, N_importance=64, N_outside=32, upsample_algo='official_solution', N_upsample_iters=4,
              max_workspace_gb=args.workspace_gb)
    n = ro.shape[1]

    def t_render(o, d):
        with torch.no_grad():
            volume_render(o, d, model, **kw)
        torch.cuda.synchronize()
        ts = []
        for _ in range(args.reps):
            t = time.perf_counter()
            with torch.no_grad():
                volume_render(o, d, model, **kw)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return sorted(ts)[len(ts) // 2]

    frame = t_render(ro, rd)
    out = {'frame_rays': n, 'world': args.world, 'frame_ms': round(frame * 1e3, 2)}
    for layout in ('contiguous', 'cyclic'):
        ts = []
        for r in range(args.world):
            if layout == 'contiguous':
                lo, hi = nd.shard_bounds(n, r, args.world)
                o, d = ro[:, lo:hi].contiguous(), rd[:, lo:hi].contiguous()
            else:
                idx = nd.cyclic_index(n, r, args.world, args.block).to(dev)
                o, d = ro.index_select(1, idx), rd.index_select(1, idx)
            ts.append(t_render(o, d))
        mean = sum(ts) / len(ts)
        out[layout] = {'share_ms': [round(t * 1e3, 2) for t in ts], 'max_over_mean': round(max(ts) / mean, 4),
                       'sum_ms': round(sum(ts) * 1e3, 2),
                       'ceiling_speedup': round(frame / max(ts), 3)}
        print(f'{layout}: ' + ' '.join(f'{t * 1e3:.1f}' for t in ts) + f' ms; max/mean {max(ts) / mean:.3f}, '
              f'{args.world}-GPU ceiling {frame / max(ts):.2f}x', file=sys.stderr, flush=True)
    out['block'] = args.block
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
