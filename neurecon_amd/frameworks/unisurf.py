"""UNISURF framework: same API as the reference's models/frameworks/unisurf.py, render path on HIP.

`volume_render(rays_o, rays_d, model, **kw) -> (rgb, depth, extras)` keeps the reference's
signature, argument meaning, output shapes and extras keys (unisurf.py:62-283).  The whole path
(256-step march + secant root finding, interval / free-space sampling, occupancy MLP with nablas,
F.normalize'd normals into the radiance net, alpha compositing) runs in libnrhip.so
(`nr_unisurf_render`).
"""
import copy
import ctypes
from collections import OrderedDict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from .. import _lib as L
from .. import rend_util
from ..base import ImplicitSurface, RadianceNet, check_view_dirs, wants_graph
from .neus import _linspace_table

N_STEPS = 256        # ray_casting.py:49 (root_finding_surface_points default)
N_SECANT_STEPS = 8   # ray_casting.py:52


class UNISURF(nn.Module):
    """unisurf.py:16-62 (parameter tree and names identical: implicit_surface.*, radiance_net.*)."""

    def __init__(self, input_ch=3, W_geo_feat=-1, surface_cfg=dict(), radiance_cfg=dict()):
        super().__init__()
        self.implicit_surface = ImplicitSurface(input_ch=input_ch, W_geo_feat=W_geo_feat, **surface_cfg)
        if W_geo_feat < 0:
            W_geo_feat = self.implicit_surface.W
        self.radiance_net = RadianceNet(W_geo_feat=W_geo_feat, **radiance_cfg)

    def forward(self, x, view_dirs):
        occ, nablas, geometry_feature = self.implicit_surface.forward_with_nablas(x)
        normals = F.normalize(nablas)  # default dim=1, exactly as unisurf.py:36
        radiances = self.radiance_net.forward(x, view_dirs, normals, geometry_feature)
        return radiances, occ, nablas

    @staticmethod
    def get_surface_from_opacity(opacity, eps=1e-4):
        if isinstance(opacity, torch.Tensor):
            opacity = torch.clamp(opacity, min=eps, max=1 - eps)
            imp_surface = torch.log(opacity / (1 - opacity))
        else:
            opacity = np.clip(opacity, a_min=eps, a_max=1 - eps)
            imp_surface = np.log(opacity / (1 - opacity))
        return (-1.) * imp_surface

    @staticmethod
    def get_opacity_from_surface(imp_surface):
        if isinstance(imp_surface, torch.Tensor):
            odds = torch.exp(-1. * imp_surface)
        else:
            odds = np.exp(-1. * imp_surface)
        return odds / (1 + odds)


def _unisurf_uniforms(B, N, batched, rayschunk, N_query, N_freespace, dev):
    """perturb=True stratification uniforms in the reference's draw order: per ray chunk the interval
    samples' torch.rand then the free-space samples' (unisurf.py:164, :193)."""
    pre = [B] if batched else []
    uq, uf = [], []
    for r0 in range(0, N, rayschunk):
        nc = min(rayschunk, N - r0)
        uq.append(rend_util.uniform([*pre, nc, N_query], dev))
        uf.append(rend_util.uniform([*pre, nc, N_freespace], dev))
    cat = lambda xs, k: torch.cat(xs, len(pre)).reshape(B * N, k).float().contiguous()
    return cat(uq, N_query), cat(uf, N_freespace)


def _window_reducer(window_ss, group=None):
    """window_reduce callback of a sharded render: all-reduce (sum) the per-window partial sums."""
    import torch.distributed as dist

    def cb(_user):
        try:
            dist.all_reduce(window_ss, op=dist.ReduceOp.SUM, group=group)
            return 0
        except Exception as e:  # reported through the library's error path
            print(f'neurecon_amd: window_reduce failed: {e!r}')
            return 1
    return L.WINDOW_REDUCE(cb)


def volume_render(rays_o, rays_d, model, batched=False, batched_info={}, calc_normal=False, logit_tau=0.0,
                  use_view_dirs=True, method='secant', rayschunk=65536, netchunk=1048576, white_bkgd=False,
                  near_bypass=None, far_bypass=None, detailed_output=True, show_progress=False,
                  radius_of_interest=4.0, perturb=False, interval=1.0, too_close_threshold=0.1, N_query=64,
                  N_freespace=32, shard=None, _sample_only=False, _full_march=False, **dummy_kwargs):
    """unisurf.py:62-283, render mode.  rays_o/rays_d: [(B,) N_rays, 3].
    shard = (ray0, row_rays, group): these rays are ranks' slice [ray0, ray0 + N) of batch rows of
    row_rays rays (neurecon_amd.dist.render_sharded); the windowed F.normalize then sums its nabla^2
    windows over all ranks (one all-reduce of B x windows x 3 doubles), so the result equals the
    single-process render of the whole batch.  _full_march=True: the root-finding march over every
    step of every ray in one launch (the reference's schedule; the same outputs bit for bit)."""
    L.require_gpu(rays_o, 'rays_o')
    if wants_graph(model) and not _sample_only:
        if shard is not None:
            raise NotImplementedError('neurecon_amd: a UNISURF training render runs on the whole batch per rank '
                                      '(DDP); shard= is for render-mode frame sharding')
        return _train_render(rays_o, rays_d, model, batched=batched, calc_normal=calc_normal, logit_tau=logit_tau,
                             use_view_dirs=use_view_dirs, method=method, rayschunk=rayschunk, netchunk=netchunk,
                             white_bkgd=white_bkgd, near_bypass=near_bypass, far_bypass=far_bypass,
                             detailed_output=detailed_output, radius_of_interest=radius_of_interest, perturb=perturb,
                             interval=interval, too_close_threshold=too_close_threshold, N_query=N_query,
                             N_freespace=N_freespace)
    check_view_dirs(model, use_view_dirs)
    dev = rays_o.device
    if batched:
        B, N = rays_d.shape[0], rays_d.reshape(rays_d.shape[0], -1, 3).shape[1]
        prefix = [B, -1]
    else:
        N = rays_d.reshape(-1, 3).shape[0]
        prefix = [-1]
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd = rays_d.reshape(-1, 3).float().contiguous()
    n = ro.shape[0]
    P = N_query + N_freespace

    sdf_desc, sdf_packed = model.implicit_surface.nr_packed(dev)
    rad_desc, rad_packed = model.radiance_net.nr_packed(dev)
    t_march = _linspace_table(N_STEPS, dev)
    # perturb: bin edges linspace(0, 1, N+1) (unisurf.py:159, :188)
    t_query = _linspace_table(N_query + (1 if perturb else 0), dev)
    t_free = _linspace_table(N_freespace + (1 if perturb else 0), dev)

    rgb = torch.empty(n, 3, device=dev) if not _sample_only else None
    depth = torch.empty(n, device=dev) if not _sample_only else None
    acc = torch.empty(n, device=dev) if not _sample_only else None
    normals = torch.empty(n, 3, device=dev) if calc_normal and not _sample_only else None
    det = {}
    if _sample_only:  # training's no-grad pass: sample depths + surface points only
        det = dict(surface_points=torch.empty(n, 3, device=dev),
                   mask_surface=torch.empty(n, dtype=torch.bool, device=dev), depth_surface=torch.empty(n, device=dev),
                   d_all=torch.empty(n, P, device=dev))
    elif detailed_output:
        det = dict(surface_points=torch.empty(n, 3, device=dev), mask_surface=torch.empty(n, dtype=torch.bool,
                                                                                           device=dev),
                   depth_surface=torch.empty(n, device=dev), radiance=torch.empty(n, P, 3, device=dev),
                   implicit_surface=torch.empty(n, P, device=dev), implicit_nablas=torch.empty(n, P, 3, device=dev),
                   alpha=torch.empty(n, P, device=dev), visibility_weights=torch.empty(n, P, device=dev))
    a = L.NrUnisurfArgs()
    a.rays_o, a.rays_d, a.n_rays, a.rays_per_batch = L.ptr(ro), L.ptr(rd), n, N
    a.sdf, a.sdf_packed = ctypes.pointer(sdf_desc), L.ptr(sdf_packed)
    a.rad, a.rad_packed = ctypes.pointer(rad_desc), L.ptr(rad_packed)
    a.logit_tau = float(logit_tau)
    a.radius_of_interest, a.interval = float(radius_of_interest), float(interval)
    a.too_close_threshold = float(too_close_threshold)
    a.near_bypass = float('nan') if near_bypass is None else float(near_bypass)
    a.far_bypass = float('nan') if far_bypass is None else float(far_bypass)
    a.N_steps, a.N_secant_steps, a.N_query, a.N_freespace = N_STEPS, N_SECANT_STEPS, N_query, N_freespace
    a.no_secant = int(method != 'secant')  # ray_casting.py:128-135: any other method reports depth 1 on hits
    # F.normalize(nablas) with dim=1: per point for [chunk, 3] inputs, per window for [B, chunk, 3]
    a.normal_mode = 1 if batched else 0
    a.rayschunk, a.netchunk = int(rayschunk), int(netchunk)
    a.calc_normal, a.white_bkgd = int(bool(calc_normal)), int(bool(white_bkgd))
    a.full_march = int(bool(_full_march))
    a.t_march, a.t_query, a.t_free = L.ptr(t_march), L.ptr(t_query), L.ptr(t_free)
    a.rgb, a.depth, a.acc, a.normals = L.ptr(rgb), L.ptr(depth), L.ptr(acc), L.ptr(normals)
    a.surface_points = L.ptr(det.get('surface_points'))
    a.mask_surface = L.ptr(det.get('mask_surface'))
    a.depth_surface = L.ptr(det.get('depth_surface'))
    a.radiance_out = L.ptr(det.get('radiance'))
    a.sdf_out = L.ptr(det.get('implicit_surface'))
    a.nablas_out = L.ptr(det.get('implicit_nablas'))
    a.alpha_out = L.ptr(det.get('alpha'))
    a.weights_out = L.ptr(det.get('visibility_weights'))
    if _sample_only:
        a.d_all_out, a.sample_only = L.ptr(det['d_all']), 1
    if perturb:
        B = rays_d.shape[0] if batched else 1
        u_q, u_f = _unisurf_uniforms(B, n // B, batched, int(rayschunk), N_query, N_freespace, dev)
        a.u_query, a.u_free = L.ptr(u_q), L.ptr(u_f)
    lib = L.lib()
    keep = None
    if shard is not None and batched:
        ray0, row_rays, group = shard
        a.shard_ray0, a.shard_row_rays = int(ray0), int(row_rays)
        B = rays_d.shape[0]
        window_ss = torch.zeros(B, max(int(lib.nr_unisurf_window_count(ctypes.byref(a))), 1), 3,
                                dtype=torch.float64, device=dev)
        keep = _window_reducer(window_ss, group)
        a.window_ss, a.window_reduce = L.ptr(window_ss), ctypes.cast(keep, ctypes.c_void_p)
    ws_bytes = lib.nr_unisurf_workspace_bytes(ctypes.byref(a))
    if ws_bytes == 0:
        raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
    ws = L.workspace(dev, ws_bytes)
    a.workspace, a.workspace_bytes = L.ptr(ws), ws_bytes
    L.check(lib.nr_unisurf_render(ctypes.byref(a), L.stream_of(dev)))
    del keep
    if _sample_only:
        return det

    ret = OrderedDict([('rgb', rgb.reshape(*prefix, 3)), ('depth_volume', depth.reshape(prefix)),
                       ('mask_volume', acc.reshape(prefix))])
    if calc_normal:
        ret['normals_volume'] = normals.reshape(*prefix, 3)
    if detailed_output:
        ret['surface_points'] = det['surface_points'].reshape(*prefix, 3)
        ret['mask_surface'] = det['mask_surface'].reshape(prefix)
        ret['depth_surface'] = det['depth_surface'].reshape(prefix)
        ret['radiance'] = det['radiance'].reshape(*prefix, P, 3)
        ret['implicit_surface'] = det['implicit_surface'].reshape(*prefix, P)
        ret['implicit_nablas'] = det['implicit_nablas'].reshape(*prefix, P, 3)
        ret['alpha'] = det['alpha'].reshape(*prefix, P)
        ret['visibility_weights'] = det['visibility_weights'].reshape(*prefix, P)
    return ret['rgb'], ret['depth_volume'], ret


def _window_normalize(nab, batched, B, rayschunk, netchunk):
    """UNISURF.forward's F.normalize(nablas) (default dim=1, unisurf.py:36) over the batchify_query
    windows it sees (train_util.py:23-71): nab [n, P, 3] ray-major.  Unbatched, the query input is
    [netchunk, 3] and dim 1 is xyz (per point); batched, it is [B, netchunk, 3] and each xyz column is
    normalised over the window's points, per batch row and per ray chunk of the render loop."""
    if not batched:
        return F.normalize(nab, dim=-1)
    P = nab.shape[1]
    x = nab.reshape(B, -1, P, 3)
    outs = []
    for r0 in range(0, x.shape[1], rayschunk):
        seg = x[:, r0:r0 + rayschunk].reshape(B, -1, 3)
        parts = [F.normalize(seg[:, i:i + netchunk], dim=1) for i in range(0, seg.shape[1], netchunk)]
        outs.append(torch.cat(parts, 1).reshape(B, -1, P, 3))
    return torch.cat(outs, 1).reshape(-1, P, 3)


def _train_render(rays_o, rays_d, model, batched, calc_normal, logit_tau, use_view_dirs, method, rayschunk, netchunk,
                  white_bkgd, near_bypass, far_bypass, detailed_output, radius_of_interest, perturb, interval,
                  too_close_threshold, N_query, N_freespace):
    """unisurf.py:62-283 with an autograd graph (training): the root finding and the interval /
    free-space samples come from the no-grad path (the reference's root finding runs under
    torch.no_grad, ray_casting.py:47; the depths carry no gradient), then occupancy + nablas + geometry
    feature at every sample (double-backward capable), the windowed F.normalize, the radiance net and
    the integration as neurecon_amd.training autograd functions.  Returns (rgb, depth, extras)."""
    from .. import training as T
    check_view_dirs(model, use_view_dirs)
    dev = rays_o.device
    B = rays_d.shape[0] if batched else 1
    prefix = [B, -1] if batched else [-1]
    P = N_query + N_freespace
    with torch.no_grad():
        ex = volume_render(rays_o, rays_d, model, batched=batched, logit_tau=logit_tau, use_view_dirs=use_view_dirs,
                           method=method, rayschunk=rayschunk, netchunk=netchunk, near_bypass=near_bypass,
                           far_bypass=far_bypass, radius_of_interest=radius_of_interest, perturb=perturb,
                           interval=interval, too_close_threshold=too_close_threshold, N_query=N_query,
                           N_freespace=N_freespace, _sample_only=True)
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd_raw = rays_d.reshape(-1, 3).float().contiguous()
    n = ro.shape[0]
    d_all = ex['d_all']
    rd = torch.empty_like(rd_raw)  # F.normalize(rays_d, dim=-1) (unisurf.py:118)
    L.check(L.lib().nr_normalize3(L.ptr(rd_raw), n, L.ptr(rd), L.stream_of(dev)))
    pts = torch.empty(n, P, 3, device=dev)
    mids = torch.empty(n, P - 1, 3, device=dev)
    dmid = torch.empty(n, P - 1, device=dev)
    L.check(L.lib().nr_neus_points(L.ptr(ro), L.ptr(rd), L.ptr(d_all), n, P, L.ptr(pts), L.ptr(mids), L.ptr(dmid),
                                   L.stream_of(dev)))
    logits, nablas, feat = T.sdf_nablas(model.implicit_surface, pts.reshape(-1, 3), True)   # unisurf.py:35
    nrm = _window_normalize(nablas.reshape(n, P, 3), batched, B, int(rayschunk), int(netchunk))
    view = rd[:, None, :].expand(n, P, 3).reshape(-1, 3).contiguous()
    rad = T.radiance(model.radiance_net, pts.reshape(-1, 3), view, nrm.reshape(-1, 3), feat)  # unisurf.py:37
    rgb, depth, acc, w, alpha = T.UnisurfComposite.apply(logits.reshape(n, P), rad.reshape(n, P, 3), d_all,
                                                         bool(white_bkgd))
    nablas = nablas.reshape(n, P, 3)
    ret = OrderedDict([('rgb', rgb.reshape(*prefix, 3)), ('depth_volume', depth.reshape(prefix)),
                       ('mask_volume', acc.reshape(prefix))])
    if calc_normal:  # unisurf.py:249-253
        nn_ = F.normalize(nablas, dim=-1)
        ret['normals_volume'] = (nn_ * w[..., None]).sum(dim=-2).reshape(*prefix, 3)
    if detailed_output:
        ret['surface_points'] = ex['surface_points'].reshape(*prefix, 3)
        ret['mask_surface'] = ex['mask_surface'].reshape(prefix)
        ret['depth_surface'] = ex['depth_surface'].reshape(prefix)
        ret['radiance'] = rad.reshape(*prefix, P, 3)
        ret['implicit_surface'] = logits.reshape(*prefix, P)
        ret['implicit_nablas'] = nablas.reshape(*prefix, P, 3)
        ret['alpha'] = alpha.reshape(*prefix, P)
        ret['visibility_weights'] = w.reshape(*prefix, P)
        ret['d_all'] = d_all.reshape(*prefix, P)
    return ret['rgb'], ret['depth_volume'], ret


def surface_perturbation(like, scale):
    """unisurf.py:335-336: (torch.rand(shape) - 0.5) * 2 * perturb_surface_pts (a module function so
    tests can replay the reference's draws)."""
    return (torch.rand(like.shape, device=like.device) - 0.5) * 2. * scale


class SingleRenderer(nn.Module):
    """unisurf.py:286-291."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, rays_o, rays_d, **kwargs):
        return volume_render(rays_o, rays_d, self.model, **kwargs)


volume_render.window_sharded = True  # render_sharded passes `shard=` (cross-rank F.normalize windows)


class Trainer(nn.Module):
    """unisurf.py:294-351: one training step's forward -- random rays of the image, the render with a
    graph (neurecon_amd.training autograd functions on libnrhip.so), L1 rgb loss and the normal
    smoothness term on the root-finding surface points.  Returns OrderedDict(losses=..., extras=...)
    like the reference; train.py calls backward() on losses['total'] (under DDP the gradient
    all-reduce runs over RCCL)."""

    def __init__(self, model, device_ids=[0], batched=True):
        super().__init__()
        self.model = model
        self.renderer = SingleRenderer(model)
        if len(device_ids) > 1:
            self.renderer = nn.DataParallel(self.renderer, device_ids=device_ids, dim=1 if batched else 0)
        self.device = device_ids[0]

    def forward(self, args, indices, model_input, ground_truth, render_kwargs_train, it, device='cuda'):
        from ..config import as_cfg
        args = as_cfg(args)
        intrinsics = model_input['intrinsics'].to(device)
        c2w = model_input['c2w'].to(device)
        rays_o, rays_d, select_inds = rend_util.get_rays(c2w, intrinsics, render_kwargs_train['H'],
                                                         render_kwargs_train['W'], N_rays=args.data.N_rays)
        target_rgb = rend_util.gather_rays(ground_truth['rgb'].to(device), select_inds)       # unisurf.py:319
        interval = max(args.training.delta_max * np.exp(-it * args.training.delta_beta), args.training.delta_min)
        rgb, depth_v, extras = self.renderer(rays_o, rays_d, interval=interval, detailed_output=True,
                                             **render_kwargs_train)
        losses = OrderedDict()
        losses['loss_img'] = F.l1_loss(rgb, target_rgb)
        losses['loss_reg'] = torch.tensor(0.).to(device)
        if args.training.w_reg > 0:                                                           # unisurf.py:331-341
            pts_surface = extras['surface_points']
            _, nablas_surface, _ = self.model.implicit_surface.forward_with_nablas(pts_surface)
            pts_neighbor = pts_surface + surface_perturbation(pts_surface, args.training.perturb_surface_pts)
            _, nablas_perturb, _ = self.model.implicit_surface.forward_with_nablas(pts_neighbor)
            losses['loss_reg'] = args.training.w_reg * F.mse_loss(F.normalize(nablas_perturb, dim=-1),
                                                                  F.normalize(nablas_surface, dim=-1))
        loss = 0
        for v in losses.values():
            loss += v
        losses['total'] = loss
        extras['scalars'] = {'interval': torch.tensor([interval]).to(device)}
        return OrderedDict([('losses', losses), ('extras', extras)])


def get_model(args):
    """unisurf.py:354-404 (same config keys and defaults)."""
    from ..config import as_cfg
    args = as_cfg(args)
    model_config = {'W_geo_feat': args.model.setdefault('W_geometry_feature', 256)}
    surface_cfg = {
        'use_siren': args.model.surface.setdefault('use_siren', args.model.setdefault('use_siren', False)),
        'embed_multires': args.model.surface.setdefault('embed_multires', 6),
        'radius_init': args.model.surface.setdefault('radius_init', 1.0),
        'geometric_init': args.model.surface.setdefault('geometric_init', True),
        'D': args.model.surface.setdefault('D', 8),
        'W': args.model.surface.setdefault('W', 256),
        'skips': args.model.surface.setdefault('skips', [4]),
    }
    radiance_cfg = {
        'use_siren': args.model.radiance.setdefault('use_siren', args.model.setdefault('use_siren', False)),
        'embed_multires': args.model.radiance.setdefault('embed_multires', -1),
        'embed_multires_view': args.model.radiance.setdefault('embed_multires_view', -1),
        'use_view_dirs': args.model.radiance.setdefault('use_view_dirs', True),
        'D': args.model.radiance.setdefault('D', 4),
        'W': args.model.radiance.setdefault('W', 256),
        'skips': args.model.radiance.setdefault('skips', []),
    }
    model_config['surface_cfg'] = surface_cfg
    model_config['radiance_cfg'] = radiance_cfg
    model = UNISURF(**model_config)
    render_kwargs_train = {
        'batched': True,
        'tau': args.model.tau,
        'perturb': args.model.get('perturb', True),
        'white_bkgd': args.model.get('white_bkgd', False),
        'logit_tau': model.get_surface_from_opacity(args.model.tau),
        'radius_of_interest': args.model.obj_bounding_radius,
    }
    render_kwargs_test = copy.deepcopy(render_kwargs_train)
    render_kwargs_test['rayschunk'] = args.data.val_rayschunk
    render_kwargs_test['perturb'] = False
    trainer = Trainer(model, device_ids=args.device_ids, batched=render_kwargs_train['batched'])
    return model, trainer, render_kwargs_train, render_kwargs_test, trainer.renderer
