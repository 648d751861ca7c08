"""Alternated A/B of a neurecon_amd.training module flag on the NeuS training step (bench.train_setup):
    python tools/ab_train_flag.py S_CODE24 [--rounds 3] [--steps 20] [--nerfpp]
prints rays/s per round for the flag False / True (same process, same model and data)."""
import argparse
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from neurecon_amd import training as T  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('flag')
    ap.add_argument('--rounds', type=int, default=3)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--nerfpp', action='store_true')
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    step = bench.train_setup(dev, 'f16x3', 512, 1, nerfpp=args.nerfpp)
    for r in range(args.rounds):
        for val in (False, True):
            setattr(T, args.flag, val)
            for _ in range(3):
                step()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(args.steps):
                step()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.steps
            print(f'round {r} {args.flag}={val}: {512 / dt:9.1f} rays/s  {dt * 1e3:.3f} ms/step', flush=True)


if __name__ == '__main__':
    main()
