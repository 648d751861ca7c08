"""Dump a NeuS config-(b) render (4096 rays, detailed outputs) to an .npz, or compare against one:
a bit-exactness check for schedule-only kernel changes.

    python tools/dump_neus.py save gpurun_out/neus_ref.npz
    python tools/dump_neus.py check gpurun_out/neus_ref.npz
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))
sys.path.insert(0, os.path.join(ROOT, 'tests', 'golden'))


def render():
    import weightgen as wg
    from helpers import neus_model
    from neurecon_amd import rend_util
    from neurecon_amd.frameworks.neus import volume_render
    H, W, f, dist = wg.CAMERAS['b']
    ro, rd, _ = rend_util.get_rays(wg.look_at_c2w(dist)[None].cuda(), wg.intrinsics(f, H, W)[None].cuda(), H, W)
    m = neus_model(wg.neus_state(seed=1), precision='f16x3')
    with torch.no_grad():
        rgb, depth, ex = volume_render(ro, rd, m, batched=True, calc_normal=True, detailed_output=True,
                                       N_samples=64, N_importance=64)
    out = {k: v.cpu().numpy() for k, v in ex.items() if isinstance(v, torch.Tensor)}
    return out


def main(mode, path):
    out = render()
    if mode == 'save':
        np.savez(path, **out)
        print('saved', len(out), 'arrays')
        return 0
    ref = dict(np.load(path))
    bad = [k for k in ref if not np.array_equal(ref[k], out[k], equal_nan=True)]
    print('bit-identical' if not bad else f'DIFFERENT: {bad}')
    return 1 if bad else 0


if __name__ == '__main__':
    sys.exit(main(sys.argv[1], sys.argv[2]))
