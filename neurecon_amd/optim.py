"""torch.optim.Adam on one HIP launch (nr_adam_step, nr_train.hip): the optimizer of the reference's
train.py (torch.optim.Adam(model.parameters(), lr=args.training.lr), train.py:58-60) for fp32 parameters
on the GPU.  Same constructor, parameter groups and state_dict layout as torch.optim.Adam (state 'step' a
CPU float tensor, 'exp_avg', 'exp_avg_sq'), so the two load each other's checkpoints; the update is the
one of torch's fused Adam.  torch's fused form runs the NeuS nets' ~40 tensors in multi-tensor
launches of a few workgroups each (~45 us each, latency bound); this one launch has one workgroup per
4096 elements of every tensor (profiles/r05: 90 -> ~6 us per step).  amsgrad, maximize, sparse,
non-fp32 or CPU parameters are not supported: they raise rather than fall back."""
import torch
from torch.autograd.graph import increment_version

from . import _lib as L


class Adam(torch.optim.Optimizer):
    def __init__(self, params, lr=1e-3, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0, amsgrad=False, *,
                 maximize=False):
        if not 0.0 <= lr:
            raise ValueError(f'Invalid learning rate: {lr}')
        if not 0.0 <= eps:
            raise ValueError(f'Invalid epsilon value: {eps}')
        if not 0.0 <= betas[0] < 1.0 or not 0.0 <= betas[1] < 1.0:
            raise ValueError(f'Invalid beta parameters: {betas}')
        if not 0.0 <= weight_decay:
            raise ValueError(f'Invalid weight_decay value: {weight_decay}')
        if amsgrad or maximize:
            raise NotImplementedError('neurecon_amd.optim.Adam: amsgrad / maximize are not implemented '
                                      '(use torch.optim.Adam)')
        # the param_group keys of torch.optim.Adam, so either optimizer loads the other's state_dict
        super().__init__(params, dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, amsgrad=False,
                                      maximize=False, foreach=None, capturable=False, differentiable=False,
                                      fused=None, decoupled_weight_decay=False))

    @staticmethod
    def _check(p):
        g = p.grad
        if g.is_sparse:
            raise RuntimeError('neurecon_amd.optim.Adam does not support sparse gradients')
        if p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_cuda:
            raise RuntimeError('neurecon_amd.optim.Adam: fp32 GPU parameters only')
        if not (p.is_contiguous() and g.is_contiguous()):
            raise RuntimeError('neurecon_amd.optim.Adam: contiguous parameters and gradients only')

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        for group in self.param_groups:
            ps = [p for p in group['params'] if p.grad is not None]
            if not ps:
                continue
            by_step = {}
            for p in ps:
                self._check(p)
                st = self.state[p]
                if len(st) == 0:
                    st['step'] = torch.tensor(0.0)
                    st['exp_avg'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                    st['exp_avg_sq'] = torch.zeros_like(p, memory_format=torch.preserve_format)
                st['step'] += 1
                by_step.setdefault(int(st['step'].item()), []).append(p)
            b1, b2 = group['betas']
            for step, plist in by_step.items():
                for i in range(0, len(plist), L.ADAM_MAX):
                    part = [p for p in plist[i:i + L.ADAM_MAX] if p.numel() > 0]
                    if not part:
                        continue
                    arr = (L.NrAdamTensor * len(part))()
                    for k, p in enumerate(part):
                        st = self.state[p]
                        arr[k].param, arr[k].grad = L.ptr(p), L.ptr(p.grad)
                        arr[k].exp_avg, arr[k].exp_avg_sq = L.ptr(st['exp_avg']), L.ptr(st['exp_avg_sq'])
                        arr[k].n = p.numel()
                    L.check(L.lib().nr_adam_step(arr, len(part), step, float(group['lr']), float(b1), float(b2),
                                                 float(group['eps']), float(group['weight_decay']),
                                                 L.stream_of(part[0].device)))
                    # the launch wrote through raw pointers: bump every written tensor's version counter as
                    # torch's in-place ops do, so caches keyed on (data_ptr, _version) -- the packed weights
                    # of base._version_key -- see the update and repack
                    for p in part:
                        st = self.state[p]
                        increment_version([p, st['exp_avg'], st['exp_avg_sq']])
        return loss
