"""Host-side (Python) cost of one NeuS training step: cProfile over 20 steps of bench.py's training
workload (the GPU runs ahead; the totals are the launch path's CPU time).
    python tools/train_cprofile.py [--adam fused|foreach]"""
import cProfile
import os
import pstats
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    adam = sys.argv[sys.argv.index('--adam') + 1] if '--adam' in sys.argv else 'fused'
    dev = torch.device('cuda:0')
    step = bench.train_setup(dev, 'f16x3', 512, 1, adam)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(20):
        step()
    pr.disable()
    torch.cuda.synchronize()
    st = pstats.Stats(pr).sort_stats('tottime')
    st.print_stats(45)


if __name__ == '__main__':
    main()
