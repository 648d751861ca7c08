"""Training steps whose device kernels rocprofv3 census: the NeuS step in fp32 precision (bench.train_setup,
configs/neus.yaml, 512 rays) and the VolSDF step with configs/volsdf_siren.yaml's SIREN nets (4096 rays of a
64x64 camera, Adam), each `--steps` times after one warm-up, with the wall time per step.

    rocprofv3 --kernel-trace --stats -d out -o run -- python tools/train_census.py [--which neus32,siren32,siren16]
"""
import argparse
import os
import sys
import time
import types

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]


def siren_step(precision):
    from neurecon_amd.frameworks import volsdf as V
    from neurecon_amd.optim import Adam
    from test_gpu_siren import siren_model
    import bench
    m = siren_model(precision)
    m.train()
    tr = V.Trainer(m, device_ids=[0])
    opt = Adam(m.parameters(), lr=5e-4)
    c2w, K = bench.camera('cuda')
    g = torch.Generator().manual_seed(1)
    gt = {'rgb': torch.rand(1, 4096, 3, generator=g).cuda()}
    args = types.SimpleNamespace(data=types.SimpleNamespace(N_rays=512), model=types.SimpleNamespace(obj_bounding_radius=3.0),
                                 training=types.SimpleNamespace(w_eikonal=0.1))
    kw = dict(H=64, W=64, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, perturb=True, white_bkgd=False,
              max_upsample_steps=6, use_nerfplusplus=False, N_samples=64, N_importance=64, N_outside=0)

    def step():
        ret = tr.forward(args, None, {'intrinsics': K, 'c2w': c2w}, gt, kw, 0, device='cuda')
        opt.zero_grad()
        torch.mean(ret['losses']['total']).backward()
        opt.step()
    return step


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--which', default='neus32,siren32')
    ap.add_argument('--steps', type=int, default=10)
    a = ap.parse_args()
    import bench
    dev = torch.device('cuda:0')
    for w in a.which.split(','):
        if w == 'neus32':
            fn = bench.train_setup(dev, 'fp32', 512, 1)
        elif w == 'neus16':
            fn = bench.train_setup(dev, 'f16x3', 512, 1)
        elif w == 'nerfpp16':
            fn = bench.train_setup(dev, 'f16x3', 512, 1, nerfpp=True)
        elif w == 'siren32':
            fn = siren_step('fp32')
        elif w == 'siren16':
            fn = siren_step('f16x3')
        else:
            raise SystemExit(f'unknown step {w}')
        fn()
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.steps):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / a.steps
        print(f'{w}: {dt * 1e3:.2f} ms per step', flush=True)


if __name__ == '__main__':
    main()
