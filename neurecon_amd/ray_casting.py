"""Surface rendering: drop-in for models/ray_casting.py:163-263.

`sphere_tracing_surface_points` runs entirely in libnrhip (`nr_sphere_trace`: compacted active-ray
lists on the device, the SDF MLP launched with a device-side count each iteration), as does
`root_finding_surface_points` (`nr_root_find`: march, first crossing, secant steps); `surface_render`
chains either with the framework's own native `model.forward` (SDF + nablas +
radiance kernels) and a finish kernel (`nr_surface_finish`).  Called by tools/render_view.py
(`--use_surface_render sphere_tracing`, render_view.py:236-239).
"""
import ctypes
from collections import OrderedDict

import torch

from . import _lib as L
from .base import _no_training


def _normalize3(v):
    """F.normalize(v, dim=-1) on the device (ray_casting.py:209)."""
    L.require_gpu(v, 'vectors')
    src = v.reshape(-1, 3).float().contiguous()
    out = torch.empty_like(src)
    L.check(L.lib().nr_normalize3(L.ptr(src), src.shape[0], L.ptr(out), L.stream_of(src.device)))
    return out.reshape(v.shape)


def _per_ray(v, n, dev, name):
    """near / far: a float, or a tensor broadcast to the rays (the reference's `torch.ones * near`,
    ray_casting.py:70-73, :175) -> (scalar, per-ray device array or None)."""
    if not isinstance(v, torch.Tensor):
        return float(v), None
    t = v.to(device=dev, dtype=torch.float32)
    if t.numel() == 1:
        return float(t.reshape(-1)[0]), None
    if t.numel() != n:
        raise ValueError(f'{name}: {tuple(v.shape)} does not match {n} rays')
    return 0.0, t.reshape(-1).contiguous()


def sphere_tracing_surface_points(implicit_surface, rays_o, rays_d, near=0.0, far=6.0, batched=True,
                                  batched_info={}, N_iters=20):
    """ray_casting.py:163-182 -> (d_preds [...], pts [..., 3], mask [...] bool); near / far floats or
    per-ray tensors."""
    L.require_gpu(rays_o, 'rays_o')
    _no_training(implicit_surface)
    shape = rays_o.shape[:-1]
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd = rays_d.reshape(-1, 3).float().contiguous()
    n = ro.shape[0]
    dev = ro.device
    near, near_r = _per_ray(near, n, dev, 'near')
    far, far_r = _per_ray(far, n, dev, 'far')
    desc, packed = implicit_surface.nr_packed(dev)
    lib = L.lib()
    d = torch.empty(n, device=dev)
    pts = torch.empty(n, 3, device=dev)
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    ws_bytes = lib.nr_sphere_trace_workspace_bytes(n)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    L.check(lib.nr_sphere_trace(ctypes.byref(desc), L.ptr(packed), L.ptr(ro), L.ptr(rd), n, ctypes.c_float(near),
                                ctypes.c_float(far), L.ptr(near_r), L.ptr(far_r), int(N_iters), L.ptr(d), L.ptr(pts), L.ptr(mask), L.ptr(ws),
                                ws_bytes, L.stream_of(dev)))
    return d.reshape(shape), pts.reshape(*shape, 3), mask.view(torch.bool).reshape(shape)


def root_finding_surface_points(surface_query_fn, rays_o, rays_d, near=0.0, far=6.0, batched=True, batched_info={},
                                N_steps=256, logit_tau=0.0, method='secant', N_secant_steps=8, fill_inf=True,
                                _full_march=False):
    """ray_casting.py:35-160 -> (d_pred_out, pt_pred, mask, mask_sign_change); rays_d already
    normalised.  `surface_query_fn` must be a neurecon_amd ImplicitSurface (its forward SDF runs in
    the library); near / far floats or per-ray [(B), N_rays] tensors; a method other than 'secant'
    skips the refinement and reports depth 1 on hits (ray_casting.py:128-135).  The march runs in
    chunks of 32 steps over the rays without a sign change so far; _full_march=True evaluates every
    step of every ray (the reference's schedule, the same outputs bit for bit)."""
    from .frameworks.neus import _linspace_table
    if not hasattr(surface_query_fn, 'nr_packed'):
        raise NotImplementedError('neurecon_amd: root finding needs a neurecon_amd ImplicitSurface as surface_query_fn')
    L.require_gpu(rays_o, 'rays_o')
    _no_training(surface_query_fn)
    shape = rays_o.shape[:-1]
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd = rays_d.reshape(-1, 3).float().contiguous()
    n = ro.shape[0]
    dev = ro.device
    near, near_r = _per_ray(near, n, dev, 'near')
    far, far_r = _per_ray(far, n, dev, 'far')
    desc, packed = surface_query_fn.nr_packed(dev)
    lib = L.lib()
    t = _linspace_table(int(N_steps), dev)
    d = torch.empty(n, device=dev)
    pts = torch.empty(n, 3, device=dev)
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    msc = torch.empty(n, dtype=torch.uint8, device=dev)
    ws_bytes = lib.nr_root_find_workspace_bytes(n, int(N_steps))
    ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
    L.check(lib.nr_root_find(ctypes.byref(desc), L.ptr(packed), L.ptr(ro), L.ptr(rd), n, ctypes.c_float(near),
                             ctypes.c_float(far), L.ptr(near_r), L.ptr(far_r), int(N_steps), L.ptr(t),
                             int(N_secant_steps), int(method != 'secant'), ctypes.c_float(logit_tau), int(bool(fill_inf)),
                             int(bool(_full_march)), L.ptr(d), L.ptr(pts), L.ptr(mask), L.ptr(msc), L.ptr(ws), ws_bytes,
                             L.stream_of(dev)))
    return (d.reshape(shape), pts.reshape(*shape, 3), mask.view(torch.bool).reshape(shape),
            msc.view(torch.bool).reshape(shape))


def _couples_rays(model):
    """UNISURF's forward normalizes nablas over the points axis (unisurf.py:36): results depend on
    the chunk, so the reference's rayschunk split must be kept.  Other frameworks are per point."""
    from .frameworks.unisurf import UNISURF
    return isinstance(model, UNISURF)


def surface_render(rays_o, rays_d, model, calc_normal=True, rayschunk=8192, netchunk=1048576, batched=True,
                   use_view_dirs=True, show_progress=False, ray_casting_algo='', ray_casting_cfgs={},
                   **not_used_kwargs):
    """ray_casting.py:185-263 -> (colors, depths, extras{implicit_nablas, mask_surface[, normals_surface]})."""
    if ray_casting_algo not in ('root_finding', 'sphere_tracing'):
        raise NotImplementedError(ray_casting_algo)
    if not use_view_dirs and model.radiance_net.use_view_dirs:
        # model.forward(pts, None) (ray_casting.py:216-226) fails in the reference's embed_fn_view / cat
        raise TypeError('surface_render(use_view_dirs=False) needs a RadianceNet built with use_view_dirs=False')
    L.require_gpu(rays_o, 'rays_o')
    with torch.no_grad():
        if batched:
            DIM = 1
            flat = [rays_d.shape[0], -1, 3]
        else:
            DIM = 0
            flat = [-1, 3]
        ro = rays_o.reshape(flat).float().contiguous()
        rd = _normalize3(rays_d.reshape(flat).float())
        # ray casting is per ray: one launch sequence over every ray
        if ray_casting_algo == 'root_finding':
            d_pred, pt_pred, mask, _ = root_finding_surface_points(model.implicit_surface, ro, rd, batched=batched,
                                                                   **ray_casting_cfgs)
        else:
            d_pred, pt_pred, mask = sphere_tracing_surface_points(model.implicit_surface, ro, rd, batched=batched,
                                                                  **ray_casting_cfgs)
        n = ro.shape[DIM]
        step = rayschunk if _couples_rays(model) else max(rayschunk, 1 << 18)
        colors, nablas = [], []
        for i in range(0, n, step):
            c, _, nb = model.forward(pt_pred.narrow(DIM, i, min(step, n - i)),
                                     rd.narrow(DIM, i, min(step, n - i)) if use_view_dirs else None)
            colors.append(c)
            nablas.append(nb)
        colors = torch.cat(colors, DIM).contiguous()
        nablas = torch.cat(nablas, DIM).contiguous()
        normals = torch.empty_like(nablas) if calc_normal else None
        m8 = mask.contiguous().view(torch.uint8)
        L.check(L.lib().nr_surface_finish(L.ptr(colors), L.ptr(nablas), L.ptr(m8), m8.numel(), L.ptr(normals),
                                          L.stream_of(colors.device)))
        extras = OrderedDict([('implicit_nablas', nablas), ('mask_surface', mask)])
        if calc_normal:
            extras['normals_surface'] = normals
        return colors, d_pred, extras
