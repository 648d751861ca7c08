"""Where does the fp32 training step's excess gradient error (layers 0 and 4 of the SDF net, against
the float64 truth) come from?  Runs tests/test_gpu_raybatch.py's 512-ray step in fp32 mode with parts of
the GPU step swapped for float64 evaluations on the GPU (diagnostic only: torch float64 on the saved
fp32 tensors, rounded back to fp32), and prints the per-tensor errors the test prints.

    python tools/train_error_probe.py [base|wgrad64|mm64|both64]
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]


def main():
    mode = sys.argv[1] if len(sys.argv) > 1 else 'base'
    from neurecon_amd import training as T
    if mode in ('wgrad64', 'both64'):
        def wg64(pairs, out=None, scale=1.0, colsum=None, avec=None, vec=None, blocked=0, fp32=False):
            assert not blocked
            acc = sum(a.double().t() @ b.double() for a, b in pairs) * scale
            if out is None:
                out = torch.empty(acc.shape, device=acc.device)
            out.copy_(acc.float())
            if colsum is not None:
                colsum.copy_(pairs[0][0].double().sum(0).float())
            if avec is not None:
                vec.copy_((avec.double() @ pairs[0][1].double()).float())
            return out
        T._wg = wg64
        T._colsum = lambda a: a.double().sum(0).float()
    if mode in ('mm64', 'both64'):
        def mm64(a, w, bias=None, trans=False):
            r = a.double() @ (w.double().t() if trans else w.double())
            if bias is not None:
                r = r + bias.double()
            return r.float()
        T._mm = mm64
    import test_gpu_raybatch as t
    print(f'== mode {mode}')
    try:
        t.test_neus_train_step_random_batch_vs_oracle('fp32')
    except AssertionError as e:
        print('assertion:', e)


if __name__ == '__main__':
    main()
