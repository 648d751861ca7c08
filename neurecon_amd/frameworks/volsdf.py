"""VolSDF framework: same API as the reference's models/frameworks/volsdf.py, render path on HIP.

`volume_render(rays_o, rays_d, model, **kw) -> (rgb, depth, extras)` keeps the reference's
signature, argument meaning, output shapes and extras keys (volsdf.py:377-551).  The whole path
(error-bounded sampling with bisection on beta+, final SDF + nablas + radiance, Laplace-CDF density
compositing, builtin background sphere) runs in libnrhip.so (`nr_volsdf_render`).  With grad enabled
(training) the render builds an autograd graph (`_train_render`) and `Trainer` computes the
reference's losses (volsdf.py:564-640).
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
from ..base import ImplicitSurface, NeRF, RadianceNet, check_view_dirs, wants_graph
from .neus import _linspace_table


class VolSDF(nn.Module):
    """volsdf.py:276-327 (parameter tree and names identical: ln_beta, implicit_surface.*,
    radiance_net.*, nerf_outside.*)."""

    def __init__(self, beta_init=0.1, speed_factor=1.0, input_ch=3, W_geo_feat=-1, obj_bounding_radius=3.0,
                 use_nerfplusplus=False, surface_cfg=dict(), radiance_cfg=dict()):
        super().__init__()
        self.speed_factor = speed_factor
        ln_beta_init = np.log(beta_init) / self.speed_factor
        self.ln_beta = nn.Parameter(data=torch.Tensor([ln_beta_init]), requires_grad=True)
        self.use_sphere_bg = not use_nerfplusplus
        self.obj_bounding_radius = obj_bounding_radius
        self.implicit_surface = ImplicitSurface(W_geo_feat=W_geo_feat, input_ch=input_ch,
                                                obj_bounding_size=obj_bounding_radius, **surface_cfg)
        if W_geo_feat < 0:
            W_geo_feat = self.implicit_surface.W
        self.radiance_net = RadianceNet(W_geo_feat=W_geo_feat, **radiance_cfg)
        if use_nerfplusplus:
            self.nerf_outside = NeRF(input_ch=4, multires=10, multires_view=4, use_view_dirs=True)

    def forward_ab(self):
        beta = torch.exp(self.ln_beta * self.speed_factor)
        return 1. / beta, beta

    def forward_surface(self, x):
        """volsdf.py:310-315: min(sdf, r - |x|) with the builtin background sphere."""
        sdf = self.implicit_surface.forward(x)
        if self.use_sphere_bg:
            return torch.min(sdf, self.obj_bounding_radius - x.norm(dim=-1))
        return sdf

    def forward_surface_with_nablas(self, x):
        """volsdf.py:317-325 (nablas of the network, sdf replaced outside the background sphere)."""
        sdf, nablas, h = self.implicit_surface.forward_with_nablas(x)
        if self.use_sphere_bg:
            d_bg = self.obj_bounding_radius - x.norm(dim=-1)
            outside = d_bg < sdf
            sdf[outside] = d_bg[outside]
        return sdf, nablas, h

    def forward(self, x, view_dirs):
        sdf, nablas, geometry_feature = self.forward_surface_with_nablas(x)
        radiances = self.radiance_net.forward(x, view_dirs, nablas, geometry_feature)
        return radiances, sdf, nablas


def _host_ab(model):
    """forward_ab() evaluated exactly as the reference's CPU run (fp32 exp, fp32 reciprocal)."""
    with torch.no_grad():
        beta = torch.exp(model.ln_beta.detach().float().cpu() * model.speed_factor)
        alpha = 1. / beta
    return float(alpha.reshape(-1)[0]), float(beta.reshape(-1)[0])


def _beta_plus_init(far, n_init, eps):
    """volsdf.py:127-129: sqrt(far^2 / (4 (N-1) log(1+eps))) in fp32 on the CPU."""
    far_t = far * torch.ones([1])
    return float(torch.sqrt((far_t ** 2) / (4 * (n_init - 1) * np.log(1 + eps))).reshape(-1)[0])


def _outside_radii(n, r, device):
    """volsdf.py:452-453: r / flip(linspace(0, 1, n + 2)[1:-1]) on the CPU in fp32, uploaded."""
    t = torch.linspace(0, 1, n + 2)[..., 1:-1].float()
    return (r / torch.flip(t, dims=[-1])).contiguous().to(device)


def _volsdf_uniforms(B, N, batched, rayschunk, N_importance, N_outside, dev):
    """perturb=True uniforms per reference ray chunk: the final sample_cdf's draws (volsdf.py:102,
    rend_util.py:306), then the NeRF++ strata (volsdf.py:464).  The reference draws the sample_cdf
    uniforms per convergence event (iteration 0, 1, ..., then the unconverged rays, each a
    [rays of the event, N_importance] tensor in ray order, volsdf.py:151, :204, :266); here each ray
    gets one row of one [rays, N_importance] draw, the same distribution (independent U[0,1) rows).
    Returns u_rand [B*N, N_importance] with each row sorted ascending (the kernel's inverse-CDF walk;
    the fine depths are sorted into d_all, so a row's order never reaches the outputs) and
    u_out [B*N, N_outside] (or None)."""
    pre = [B] if batched else []
    uf, uo = [], []
    for r0 in range(0, N, rayschunk):
        nc = min(rayschunk, N - r0)
        uf.append(rend_util.uniform([(B if batched else 1) * nc, N_importance], dev).reshape(*pre, nc, N_importance))
        if N_outside > 0:
            uo.append(rend_util.uniform([*pre, nc, N_outside], dev))
    u_rand = rend_util.to_device(torch.cat(uf, len(pre)).reshape(-1, N_importance).float(), dev)
    u_rand = torch.sort(u_rand, dim=-1).values.contiguous()
    u_out = rend_util.to_device(torch.cat(uo, len(pre)).reshape(-1, N_outside).float(), dev).contiguous() if uo else None
    return u_rand, u_out


def volume_render(rays_o, rays_d, model, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=False,
                  batched_info={}, calc_normal=False, use_view_dirs=True, rayschunk=65536, netchunk=1048576,
                  white_bkgd=False, use_nerfplusplus=False, detailed_output=True, show_progress=False,
                  perturb=False, N_samples=128, N_importance=64, N_outside=32, max_upsample_steps=5,
                  max_bisection_steps=10, epsilon=0.1, _uniforms=None, **dummy_kwargs):
    """volsdf.py:377-551, render mode.  rays_o/rays_d: [(B,) N_rays, 3].  perturb=True: random final
    fine samples and NeRF++ strata (_volsdf_uniforms)."""
    L.require_gpu(rays_o, 'rays_o')
    if wants_graph(model):
        return _train_render(rays_o, rays_d, model, near=near, far=far, obj_bounding_radius=obj_bounding_radius,
                             batched=batched, calc_normal=calc_normal, use_view_dirs=use_view_dirs, rayschunk=rayschunk,
                             white_bkgd=white_bkgd, use_nerfplusplus=use_nerfplusplus, detailed_output=detailed_output,
                             perturb=perturb, N_samples=N_samples, N_importance=N_importance, N_outside=N_outside,
                             max_upsample_steps=max_upsample_steps, max_bisection_steps=max_bisection_steps,
                             epsilon=epsilon)
    check_view_dirs(model, use_view_dirs)
    dev = rays_o.device
    prefix = [rays_d.shape[0], -1] if batched else [-1]
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd = rays_d.reshape(-1, 3).float().contiguous()
    n = ro.shape[0]
    S = N_samples + N_importance
    N0 = 4 * N_samples
    No = int(N_outside) if use_nerfplusplus else 0
    M = S + No  # samples after the NeRF++ merge (volsdf.py:465-469)

    sdf_desc, sdf_packed = model.implicit_surface.nr_packed(dev)
    rad_desc, rad_packed = model.radiance_net.nr_packed(dev)
    alpha_net, beta_net = _host_ab(model)
    t_coarse = _linspace_table(N_samples, dev)
    t_init = _linspace_table(N0, dev)
    u_up = _linspace_table(N0 + 2, dev)
    u_fine = _linspace_table(N_importance, dev)

    rgb = torch.empty(n, 3, device=dev)
    depth = torch.empty(n, device=dev)
    acc = torch.empty(n, device=dev)
    normals = torch.empty(n, 3, device=dev) if calc_normal else None
    det = {}
    if detailed_output:
        det = dict(implicit_surface=torch.empty(n, S, device=dev), implicit_nablas=torch.empty(n, S, 3, device=dev),
                   radiance=torch.empty(n, M, 3, device=dev), alpha=torch.empty(n, M - 1, device=dev),
                   p_i=torch.empty(n, M - 1, device=dev), visibility_weights=torch.empty(n, M - 1, device=dev),
                   d_vals=torch.empty(n, M, device=dev), sigma=torch.empty(n, M, device=dev),
                   beta_map=torch.empty(n, device=dev), iter_usage=torch.empty(n, device=dev))
        if No > 0:
            det['sigma_out'] = torch.empty(n, No, device=dev)
            det['radiance_out'] = torch.empty(n, No, 3, device=dev)
    a = L.NrVolsdfArgs()
    a.rays_o, a.rays_d, a.n_rays = L.ptr(ro), L.ptr(rd), n
    a.sdf, a.sdf_packed = ctypes.pointer(sdf_desc), L.ptr(sdf_packed)
    a.rad, a.rad_packed = ctypes.pointer(rad_desc), L.ptr(rad_packed)
    a.alpha_net, a.beta_net = alpha_net, beta_net
    a.beta_plus_init = _beta_plus_init(far, N0, epsilon) if No == 0 else 0.0
    if No > 0:
        nerf_desc, nerf_packed = model.nerf_outside.nr_packed(dev)
        a.N_outside = No
        a.nerf, a.nerf_packed = ctypes.pointer(nerf_desc), L.ptr(nerf_packed)
        rs_out = _outside_radii(No, float(obj_bounding_radius), dev)
        a.rs_out = L.ptr(rs_out)
        a.beta_plus_k = float(np.float32(4 * (N0 - 1) * np.log(1 + epsilon)))
    a.eps = float(epsilon)
    a.near, a.far = float(near), float(far)
    # builtin background: the model's radius (volsdf.py:310-325); NeRF++: the sphere-exit far comes
    # from volume_render's own argument (volsdf.py:404), like the background radii rs_out above
    a.obj_bounding_radius = float(obj_bounding_radius) if No > 0 else float(model.obj_bounding_radius)
    a.use_sphere_bg = int(bool(model.use_sphere_bg))
    a.N_samples, a.N_importance = N_samples, N_importance
    a.max_upsample_steps, a.max_bisection_steps = max_upsample_steps, max_bisection_steps
    a.calc_normal, a.white_bkgd = int(bool(calc_normal)), int(bool(white_bkgd))
    a.t_coarse, a.t_init, a.u_up, a.u_fine = L.ptr(t_coarse), L.ptr(t_init), L.ptr(u_up), L.ptr(u_fine)
    a.rgb, a.depth, a.acc, a.normals = L.ptr(rgb), L.ptr(depth), L.ptr(acc), L.ptr(normals)
    a.d_vals = L.ptr(det.get('d_vals'))
    a.sdf_out = L.ptr(det.get('implicit_surface'))
    a.nablas_out = L.ptr(det.get('implicit_nablas'))
    a.radiance_out = L.ptr(det.get('radiance'))
    a.alpha_out = L.ptr(det.get('alpha'))
    a.p_out = L.ptr(det.get('p_i'))
    a.weights_out = L.ptr(det.get('visibility_weights'))
    a.sigma_out = L.ptr(det.get('sigma'))
    a.beta_map = L.ptr(det.get('beta_map'))
    a.iter_usage = L.ptr(det.get('iter_usage'))
    a.sigma_bg = L.ptr(det.get('sigma_out'))
    a.radiance_bg = L.ptr(det.get('radiance_out'))
    if perturb:
        if _uniforms is None:
            Bn = rays_d.shape[0] if batched else 1
            _uniforms = _volsdf_uniforms(Bn, n // Bn, batched, int(rayschunk), N_importance, No, dev)
        u_rand, u_out = _uniforms
        a.u_rand, a.u_out = L.ptr(u_rand), L.ptr(u_out)
    lib = L.lib()
    ws_bytes = lib.nr_volsdf_workspace_bytes(ctypes.byref(a))
    if ws_bytes == 0:
        raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    a.workspace, a.workspace_bytes = L.ptr(ws), ws_bytes
    L.check(lib.nr_volsdf_render(ctypes.byref(a), L.stream_of(dev)))

    ret = OrderedDict([('rgb', rgb.reshape(*prefix, 3)), ('depth_volume', depth.reshape(prefix)),
                       ('mask_volume', acc.reshape(prefix))])
    if calc_normal:
        ret['normals_volume'] = normals.reshape(*prefix, 3)
    if detailed_output:
        ret['implicit_surface'] = det['implicit_surface'].reshape(*prefix, S)
        ret['implicit_nablas'] = det['implicit_nablas'].reshape(*prefix, S, 3)
        ret['radiance'] = det['radiance'].reshape(*prefix, M, 3)
        ret['alpha'] = det['alpha'].reshape(*prefix, M - 1)
        ret['p_i'] = det['p_i'].reshape(*prefix, M - 1)
        ret['visibility_weights'] = det['visibility_weights'].reshape(*prefix, M - 1)
        ret['d_vals'] = det['d_vals'].reshape(*prefix, M)
        ret['sigma'] = det['sigma'].reshape(*prefix, M)
        ret['beta_map'] = det['beta_map'].reshape(*prefix, 1)
        ret['iter_usage'] = det['iter_usage'].reshape(prefix)
        if No > 0:
            ret['sigma_out'] = det['sigma_out'].reshape(*prefix, No)
            ret['radiance_out'] = det['radiance_out'].reshape(*prefix, No, 3)
    return ret['rgb'], ret['depth_volume'], ret


def _train_render(rays_o, rays_d, model, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=False, calc_normal=False,
                  use_view_dirs=True, rayschunk=65536, white_bkgd=False, use_nerfplusplus=False, detailed_output=True,
                  perturb=False, N_samples=128, N_importance=64, N_outside=32, max_upsample_steps=5,
                  max_bisection_steps=10, epsilon=0.1):
    """volsdf.py:377-551 with an autograd graph (training): the sample depths d_all come from the
    no-grad render path (error-bounded fine sampling, volsdf.py:420-445, the same call under
    torch.no_grad; with perturb=True both take the same uniforms), then SDF + nablas + geometry feature
    at every sample (double-backward capable), with use_nerfplusplus the background net at the
    sampler's outside depths and radii (volsdf.py:455-469),
    the radiance net and the background / sdf_to_sigma / integration as neurecon_amd.training
    autograd functions.  Gradients reach every surface, radiance (and background) parameter and
    ln_beta.  Returns
    the reference's (rgb, depth, extras)."""
    from .. import training as T
    check_view_dirs(model, use_view_dirs)
    dev = rays_o.device
    prefix = [rays_d.shape[0], -1] if batched else [-1]
    No = int(N_outside) if use_nerfplusplus else 0
    ro = rays_o.reshape(-1, 3).float().contiguous()
    rd_raw = rays_d.reshape(-1, 3).float().contiguous()
    n = ro.shape[0]
    S = N_samples + N_importance
    uni = None
    if perturb:  # drawn once: the no-grad sampler and the background radii below use the same draws
        Bn = rays_d.shape[0] if batched else 1
        uni = _volsdf_uniforms(Bn, n // Bn, batched, int(rayschunk), N_importance, No, dev)
    with torch.no_grad():
        _, _, ex = volume_render(rays_o, rays_d, model, near=near, far=far, obj_bounding_radius=obj_bounding_radius,
                                 batched=batched, calc_normal=False, use_view_dirs=use_view_dirs, rayschunk=rayschunk,
                                 white_bkgd=white_bkgd, use_nerfplusplus=use_nerfplusplus, detailed_output=True,
                                 perturb=perturb, N_samples=N_samples, N_importance=N_importance, N_outside=N_outside,
                                 max_upsample_steps=max_upsample_steps, max_bisection_steps=max_bisection_steps,
                                 epsilon=epsilon, _uniforms=uni)
    d_vals = ex['d_vals'].reshape(n, S + No)
    d_all = d_vals[:, :S].contiguous()
    rd = torch.empty_like(rd_raw)  # F.normalize(rays_d, dim=-1) (volsdf.py:386)
    L.check(L.lib().nr_normalize3(L.ptr(rd_raw), n, L.ptr(rd), L.stream_of(dev)))
    pts = torch.empty(n, S, 3, device=dev)
    mids = torch.empty(n, S - 1, 3, device=dev)
    dmid = torch.empty(n, S - 1, device=dev)
    L.check(L.lib().nr_neus_points(L.ptr(ro), L.ptr(rd), L.ptr(d_all), n, S, L.ptr(pts), L.ptr(mids), L.ptr(dmid),
                                   L.stream_of(dev)))
    sdf, nablas, feat = T.sdf_nablas(model.implicit_surface, pts.reshape(-1, 3), True)      # volsdf.py:450
    view = rd[:, None, :].expand(n, S, 3).reshape(-1, 3).contiguous()
    rad = T.radiance(model.radiance_net, pts.reshape(-1, 3), view, nablas, feat)
    _, beta = model.forward_ab()
    bg = ()
    if No > 0:  # NeRF++ background (volsdf.py:455-469) at the sampler's depths d_out and radii rs
        d_bg = d_vals[:, S:].contiguous()
        rs = _outside_radii(No, float(obj_bounding_radius), dev).expand(n, No)
        if perturb:  # volsdf.py:460-465, the draws the sampler used
            mids = .5 * (rs[..., 1:] + rs[..., :-1])
            upper = torch.cat([mids, rs[..., -1:]], -1)
            lower = torch.cat([rs[..., :1], mids], -1)
            rs = lower + (upper - lower) * uni[1].reshape(n, No)
        rs = rs.contiguous()
        x_emb = torch.empty(n * No, 84, device=dev)
        v_emb = torch.empty(n * No, 27, device=dev)
        L.check(L.lib().nr_volsdf_nerf_input(L.ptr(ro), L.ptr(rd), L.ptr(d_bg), L.ptr(rs), n, No, L.ptr(x_emb),
                                             L.ptr(v_emb), L.stream_of(dev)))
        sig_o, rad_o = T.nerf(model.nerf_outside, x_emb, v_emb)
        bg = (sig_o.reshape(n, No), rad_o.reshape(n, No, 3), d_bg)
    rgb, depth, acc, tau, sdf_bg, p_i, sigma = T.VolSDFComposite.apply(
        sdf.reshape(n, S), beta, rad.reshape(n, S, 3), pts, d_all, bool(model.use_sphere_bg),
        float(model.obj_bounding_radius), bool(white_bkgd), *bg)
    M = S + No
    nablas = nablas.reshape(n, S, 3)
    ret = OrderedDict([('rgb', rgb.reshape(*prefix, 3)), ('depth_volume', depth.reshape(prefix)),
                       ('mask_volume', acc.reshape(prefix))])
    if calc_normal:  # volsdf.py:508-512
        nrm = F.normalize(nablas, dim=-1)
        k = min(tau.shape[-1], nrm.shape[-2])
        ret['normals_volume'] = (nrm[:, :k, :] * tau[:, :k, None]).sum(dim=-2).reshape(*prefix, 3)
    if detailed_output:
        ret['implicit_surface'] = sdf_bg.reshape(*prefix, S)
        ret['implicit_nablas'] = nablas.reshape(*prefix, S, 3)
        radiances = rad.reshape(n, S, 3) if No == 0 else torch.cat([rad.reshape(n, S, 3), bg[1]], 1)
        ret['radiance'] = radiances.reshape(*prefix, M, 3)
        ret['alpha'] = (1.0 - p_i).reshape(*prefix, M - 1)
        ret['p_i'] = p_i.reshape(*prefix, M - 1)
        ret['visibility_weights'] = tau.reshape(*prefix, M - 1)
        ret['d_vals'] = d_vals.reshape(*prefix, M)
        ret['sigma'] = sigma.reshape(*prefix, M)
        ret['beta_map'] = ex['beta_map'].reshape(*prefix, 1)
        ret['iter_usage'] = ex['iter_usage'].reshape(prefix)
        if No > 0:
            ret['sigma_out'] = bg[0].reshape(*prefix, No)
            ret['radiance_out'] = bg[1].reshape(*prefix, No, 3)
    return ret['rgb'], ret['depth_volume'], ret


def eikonal_points(like, bound):
    """volsdf.py:609: torch.empty_like(nablas).uniform_(-bound, bound) (the eikonal samples of the
    training step; a module function so tests can replay the reference's draws)."""
    return torch.empty_like(like).uniform_(-bound, bound)


class SingleRenderer(nn.Module):
    """volsdf.py:555-561."""

    def __init__(self, model):
        super().__init__()
        self.model = model

    def forward(self, rays_o, rays_d, **kwargs):
        return volume_render(rays_o, rays_d, self.model, **kwargs)


class Trainer(nn.Module):
    """volsdf.py:564-640: one training step's forward -- random rays of the image, the render with a
    graph (neurecon_amd.training autograd functions on libnrhip.so), L1 rgb + eikonal losses (the
    nabla of each ray's highest-weight sample and one uniform point per ray).  Returns
    OrderedDict(losses=..., extras=...) like the reference; train.py calls backward() on
    losses['total'] (under DDP the gradient all-reduce runs over RCCL)."""

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
        H, W = render_kwargs_train['H'], render_kwargs_train['W']
        rays_o, rays_d, select_inds = rend_util.get_rays(c2w, intrinsics, H, W, N_rays=args.data.N_rays)
        target_rgb = rend_util.gather_rays(ground_truth['rgb'].to(device), select_inds)      # volsdf.py:588
        mask_ignore = rend_util.gather_rays(model_input['mask_ignore'].to(device), select_inds) \
            if 'mask_ignore' in model_input else None
        rgb, depth_v, extras = self.renderer(rays_o, rays_d, detailed_output=True, **render_kwargs_train)
        nablas = extras['implicit_nablas']
        # one point per ray: the sample of highest visibility weight (volsdf.py:604-605)
        _, ind = extras['visibility_weights'][..., :nablas.shape[-2]].max(dim=-1)
        nablas = torch.gather(nablas, dim=-2, index=ind[..., None, None].repeat([*(len(nablas.shape) - 1) * [1], 3]))
        eik = eikonal_points(nablas, args.model.obj_bounding_radius)                      # volsdf.py:607-610
        _, nablas_eik, _ = self.model.implicit_surface.forward_with_nablas(eik)
        nablas = torch.cat([nablas, nablas_eik], dim=-2)
        nablas_norm = torch.norm(nablas, dim=-1)
        losses = OrderedDict()
        losses['loss_img'] = F.l1_loss(rgb, target_rgb, reduction='none')
        losses['loss_eikonal'] = args.training.w_eikonal * F.mse_loss(
            nablas_norm, nablas_norm.new_ones(nablas_norm.shape), reduction='mean')
        if mask_ignore is not None:
            losses['loss_img'] = (losses['loss_img'] * mask_ignore[..., None].float()).sum() / (mask_ignore.sum() + 1e-10)
        else:
            losses['loss_img'] = losses['loss_img'].mean()
        loss = 0
        for k, v in losses.items():
            loss += losses[k]
        losses['total'] = loss
        extras['implicit_nablas_norm'] = nablas_norm
        alpha, beta = self.model.forward_ab()
        extras['scalars'] = {'beta': beta.data, 'alpha': alpha.data}
        extras['select_inds'] = select_inds
        return OrderedDict([('losses', losses), ('extras', extras)])


def get_model(args):
    """volsdf.py:685-750 (same config keys and defaults)."""
    from ..config import as_cfg
    args = as_cfg(args)
    model_config = {
        'use_nerfplusplus': args.model.setdefault('outside_scene', 'builtin') == 'nerf++',
        'obj_bounding_radius': args.model.obj_bounding_radius,
        'W_geo_feat': args.model.setdefault('W_geometry_feature', 256),
        'speed_factor': args.training.setdefault('speed_factor', 1.0),
        'beta_init': args.training.setdefault('beta_init', 0.1),
    }
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
    model = VolSDF(**model_config)
    render_kwargs_train = {
        'near': args.data.near,
        'far': args.data.far,
        'batched': True,
        'perturb': args.model.setdefault('perturb', True),
        'white_bkgd': args.model.setdefault('white_bkgd', False),
        'max_upsample_steps': args.model.setdefault('max_upsample_iter', 5),
        'use_nerfplusplus': model_config['use_nerfplusplus'],
        'obj_bounding_radius': args.model.obj_bounding_radius,
    }
    render_kwargs_test = copy.deepcopy(render_kwargs_train)
    render_kwargs_test['rayschunk'] = args.data.val_rayschunk
    render_kwargs_test['perturb'] = False
    trainer = Trainer(model, device_ids=args.device_ids, batched=render_kwargs_train['batched'])
    return model, trainer, render_kwargs_train, render_kwargs_test, trainer.renderer
