"""Where the training step's small torch kernels come from: one NeuS training step (bench.train_setup)
under torch.profiler with Python stacks; prints the aten ops that launch fills, copies and elementwise
kernels, grouped by the innermost neurecon_amd / bench frames, with their CUDA time.

    python tools/train_prof_ops.py [--nerfpp] [--top 40]"""
import argparse
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--nerfpp', action='store_true')
    ap.add_argument('--top', type=int, default=40)
    args = ap.parse_args()
    dev = torch.device('cuda:0')
    step = bench.train_setup(dev, 'f16x3', 512, 1, nerfpp=args.nerfpp)
    for _ in range(3):
        step()
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    ka = prof.key_averages(group_by_stack_n=6)
    key = 'self_device_time_total' if hasattr(next(iter(ka)), 'self_device_time_total') else 'self_cuda_time_total'
    print(ka.table(sort_by=key, row_limit=args.top, max_name_column_width=36, max_src_column_width=110))
    # the aten ops with their input shapes (where the stacks are not recorded)
    ks = prof.key_averages(group_by_input_shape=True)
    rows = [e for e in ks if e.key.startswith('aten::') and getattr(e, key, 0) > 0]
    rows.sort(key=lambda e: -getattr(e, key))
    for e in rows[:args.top]:
        print(f'{getattr(e, key):9.1f} us {e.count:4d}x {e.key:24s} {str(e.input_shapes)[:150]}')

if __name__ == '__main__':
    main()
