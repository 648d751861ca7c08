"""ORACLE (test infrastructure only) — surface rendering and the mesh-extraction SDF grid.

Restates models/ray_casting.py:163-263 (`sphere_tracing_surface_points`, `surface_render` with
ray_casting_algo='sphere_tracing') and utils/mesh_util.py:82-108 (`extract_mesh`'s voxel grid and
batched forward SDF) in eager fp32 PyTorch / float64 numpy on the CPU.  Pinned by
tests/golden/surface.npz (produced by the reference itself, tests/golden/gen_golden.py).
"""
import numpy as np
import torch
import torch.nn.functional as F


def sphere_trace(sdf_fn, rays_o, rays_d, near=0.0, far=6.0, N_iters=20):
    """ray_casting.py:163-182."""
    d = torch.ones(rays_o.shape[:-1]) * near
    mask = torch.ones_like(d, dtype=torch.bool)
    for _ in range(N_iters):
        pts = rays_o + rays_d * d[..., :, None]
        sv = sdf_fn(pts)
        d[mask] += sv[mask]
        mask[d > far] = False
        mask[d < 0] = False
    return d, rays_o + rays_d * d[..., :, None], mask


def root_find(sdf_fn, o, d, near=0.0, far=6.0, **cfgs):
    """ray_casting.py:35-160 with float or per-ray tensor near / far (:70-73; restated in
    oracle/unisurf.py:root_find)."""
    from .unisurf import root_find as rf
    cfgs.setdefault('fill_inf', True)
    full = lambda v: v if isinstance(v, torch.Tensor) else v * torch.ones(o.shape[:-1])
    return rf(sdf_fn, o, d, full(near), full(far), **cfgs)


def surface_render_neus(oracle, rays_o, rays_d, calc_normal=True, algo='sphere_tracing', **cfgs):
    """ray_casting.py:185-263 with a NeuS model (model.forward = neus.py:111-115), batched [B, N, 3]."""
    o = rays_o.reshape(rays_o.shape[0], -1, 3).float()
    d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).float(), dim=-1)
    if algo == 'root_finding':
        dp, pts, mask, _ = root_find(oracle.sdf_net.sdf, o, d, **cfgs)
    else:
        dp, pts, mask = sphere_trace(oracle.sdf_net.sdf, o, d, **cfgs)
    _, nab, h = oracle.sdf_net.forward_with_nablas(pts)
    color = oracle.rad_net.forward(pts, d, nab, h)
    color[~mask] = 0
    out = dict(rgb=color, depth=dp, nablas=nab, mask=mask)
    if calc_normal:
        n = F.normalize(nab, dim=-1)
        n[~mask] = 0
        out['normals'] = n
    return out


def grid_points(N, s):
    """mesh_util.py:83-100 (numpy float64, true divisions as written) -> float32 [N^3, 3]."""
    origin = [-s / 2., -s / 2., -s / 2.]
    i = np.arange(0, N ** 3, 1).astype(np.int64)
    xyz = np.zeros([N ** 3, 3])
    xyz[:, 2] = i % N
    xyz[:, 1] = (i / N) % N
    xyz[:, 0] = ((i / N) / N) % N
    xyz[:, 0] = (xyz[:, 0] * (s / (N - 1))) + origin[2]
    xyz[:, 1] = (xyz[:, 1] * (s / (N - 1))) + origin[1]
    xyz[:, 2] = (xyz[:, 2] * (s / (N - 1))) + origin[0]
    return xyz.astype(np.float32)


def sdf_grid(sdf_fn, N, s, chunk=16 * 1024):
    """mesh_util.py:102-108: batched forward SDF over the grid -> [N, N, N]."""
    pts = grid_points(N, s)
    out = [sdf_fn(torch.from_numpy(pts[i:i + chunk])).numpy() for i in range(0, pts.shape[0], chunk)]
    return np.concatenate(out).reshape(N, N, N)
