"""Ray utilities with the reference's signatures (utils/rend_util.py); compute on libnrhip.so."""
import ctypes

import numpy as np
import torch
import torch.nn.functional as F

from . import _lib as L


def get_rays(c2w, intrinsics, H, W, N_rays=-1, device_rng=False):
    """rend_util.py:112-164 (pose-matrix form).  Random pixel selection draws
    randint(H)*W + randint(W) with torch's CPU generator exactly like the reference (rend_util.py:137-138);
    device_rng=True draws them on the GPU instead (no host work per step, a different random stream)."""
    L.require_gpu(c2w, 'c2w')
    if c2w.shape[-1] == 7:
        raise NotImplementedError('quaternion camera poses (rend_util.py:114-119) are not supported')
    dev = c2w.device
    prefix = c2w.shape[:-2]
    B = int(np.prod(prefix)) if len(prefix) else 1
    m = c2w.reshape(B, 4, 4).float().contiguous()
    K = intrinsics.to(dev).reshape(-1, 4, 4).float().expand(B, 4, 4).contiguous()
    if N_rays > 0:
        N_rays = min(N_rays, H * W)
        gen_dev = dev if device_rng else None
        hs = to_device(torch.randint(0, H, size=[N_rays], device=gen_dev), dev)
        ws = to_device(torch.randint(0, W, size=[N_rays], device=gen_dev), dev)
        select_inds = (hs * W + ws).expand([*prefix, N_rays])
        sel = select_inds.reshape(B, N_rays).contiguous()
        N = N_rays
    else:
        N = H * W
        select_inds = torch.arange(N, device=dev).expand([*prefix, N])
        sel = None
    ro = torch.empty(B, N, 3, device=dev)
    rd = torch.empty(B, N, 3, device=dev)
    L.check(L.lib().nr_get_rays(L.ptr(m), L.ptr(K), B, H, W, L.ptr(sel), N, L.ptr(ro), L.ptr(rd),
                                L.stream_of(dev)))
    return ro.reshape(*prefix, N, 3), rd.reshape(*prefix, N, 3), select_inds


def gather_rays(src, select_inds):
    """Targets of a random ray batch: torch.gather(src, 1, select_inds[..., None].expand(...)) on the
    device (neus.py:432, :449): src [B, H*W, ...] (rgb, masks), select_inds [B, N] -> [B, N, ...]."""
    L.require_gpu(src, 'src')
    B, HW = src.shape[0], src.shape[1]
    idx = select_inds.to(src.device).reshape(B, -1).long().contiguous()
    N = idx.shape[1]
    s = src.contiguous()
    row_bytes = s.element_size() * int(np.prod(s.shape[2:], dtype=np.int64))
    out = torch.empty(B, N, *s.shape[2:], dtype=s.dtype, device=s.device)
    L.check(L.lib().nr_gather_rows(L.ptr(s), B, HW, row_bytes, L.ptr(idx), N, L.ptr(out), L.stream_of(s.device)))
    return out


def to_device(t, dev):
    """t.to(dev) without a host wait: a CPU draw goes up through pinned memory on the current stream
    (a pageable .to() synchronises the host with the whole queue -- once per training step it left the
    GPU idle while the host caught up)"""
    if t.device == torch.device(dev) or t.device.type != 'cpu' or torch.device(dev).type != 'cuda':
        return t.to(dev)
    return t.pin_memory().to(dev, non_blocking=True)


def uniform(shape, device=None):
    """torch.rand(shape, device=device): every perturb=True draw of the render path goes through here,
    in the reference's order, generators and shapes (tests replay recorded draws by patching it)."""
    return torch.rand(list(shape), device=device)


def near_far_from_sphere(ray_origins, ray_directions, r=1.0, keepdim=True):
    """rend_util.py:167-185 (the render kernels compute this in-kernel; kept for API users)."""
    mid = -torch.sum(ray_origins * ray_directions, dim=-1, keepdim=keepdim)
    return (mid - r).clamp_min(0.0), (mid + r).clamp_min(r)


def sample_pdf(bins, weights, N_importance, det=False, eps=1e-5):
    """rend_util.py:255-292 on the HIP kernel.  det=False draws u = torch.rand([..., N_importance],
    device=weights.device) exactly as the reference (rend_util.py:271)."""
    L.require_gpu(bins, 'bins')
    shape = bins.shape[:-1]
    Lb = bins.shape[-1]
    b = bins.reshape(-1, Lb).float().contiguous()
    w = weights.reshape(-1, Lb - 1).float().contiguous()
    if det:
        u, stride = torch.linspace(0.0, 1.0, steps=N_importance).float().to(bins.device), 0
    else:
        u = uniform(list(weights.shape[:-1]) + [N_importance], weights.device).float().reshape(-1, N_importance)
        u, stride = u.to(bins.device).contiguous(), N_importance
    out = torch.empty(b.shape[0], N_importance, device=bins.device)
    L.check(L.lib().nr_sample_pdf(L.ptr(b), L.ptr(w), b.shape[0], Lb, L.ptr(u), stride, N_importance, L.ptr(out),
                                  L.stream_of(bins.device)))
    return out.reshape(*shape, N_importance)


def lin2img(tensor, H, W, batched=False, B=None):
    """rend_util.py:237-247."""
    *_, num_samples, channels = tensor.shape
    assert num_samples == H * W
    if batched:
        if B is None:
            B = tensor.shape[0]
        else:
            tensor = tensor.view([B, num_samples // B, channels])
        return tensor.permute(0, 2, 1).view([B, channels, H, W])
    return tensor.permute(1, 0).view([channels, H, W])
