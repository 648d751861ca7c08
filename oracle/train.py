"""ORACLE (test infrastructure only): the NeuS training step's forward -- the render with an
autograd graph and the reference Trainer's losses -- restated from models/frameworks/neus.py:417-485
(render: :284-355; nablas with create_graph=True: models/base.py:265-282).  Parameters are the leaf
tensors of a reference-format state_dict; .backward() on the returned total gives the reference's
parameter gradients (weight_g / weight_v through weight_norm, ln_s through s = exp(ln_s * speed))."""
import torch
import torch.nn.functional as F

from . import rays as R
from .nets import NeRFNet, SDFNet, RadianceNet
from .neus import NeuSOracle, alpha_to_w, sdf_to_alpha
from .volsdf import VolSDFOracle, sdf_to_sigma


def nablas_graph(net, x):
    """ImplicitSurface.forward_with_nablas with create_graph=True (base.py:265-282)"""
    x = x.detach().requires_grad_(True)
    s, h = net.forward(x)
    g = torch.autograd.grad(s, x, torch.ones_like(s), create_graph=True, retain_graph=True, only_inputs=True)[0]
    return s, g, h


def neus_train_losses(sd, rays_o, rays_d, target_rgb, target_mask, w_eikonal=0.1, w_mask=1.0, with_mask=True,
                      d_all=None, speed_factor=10.0, obj_bounding_radius=1.0, N_samples=64, N_importance=64,
                      N_upsample_iters=4, N_outside=0, dtype=torch.float32, rad_masks=None, rad_z=None):
    """losses (neus.py:453-478) of one training render of rays [B, N, 3]; d_all [B, N, S] optional
    (the sorted sample depths; computed with the no-grad upsampling when None); N_outside > 0 adds the
    NeRF++ background (neus.py:303-343, perturb=False) with its parameters in the graph.
    dtype=torch.float64 (with a float64 state_dict and d_all given): the same function evaluated in
    float64 on the same inputs -- the truth the fp32 oracle and the GPU are both measured against.
    rad_masks / rad_z: RadianceNet.forward's masks / z_out on the mid-points [B, N, S-1] (test
    instrumentation: the radiance net's ReLU decisions pinned to the GPU's)."""
    o = rays_o.reshape(rays_o.shape[0], -1, 3).to(dtype)
    d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).to(dtype), dim=-1)
    if d_all is not None:
        d_all = d_all.to(dtype)
    near, far = R.near_far_from_sphere(o, d, r=obj_bounding_radius)
    orc = NeuSOracle({k: v.detach() for k, v in sd.items()}, speed_factor=speed_factor)
    if d_all is None:
        d_all = orc.sample_depths(o, d, near, far, N_samples, N_importance, 'official_solution', N_upsample_iters)
    sdf_net = SDFNet(sd)
    rad_net = RadianceNet(sd, multires_view=4)
    pts = o[..., None, :] + d[..., None, :] * d_all[..., :, None]          # neus.py:284
    d_mid = 0.5 * (d_all[..., 1:] + d_all[..., :-1])
    pts_mid = o[..., None, :] + d[..., None, :] * d_mid[..., :, None]
    sdf, nablas, _ = nablas_graph(sdf_net, pts)                             # neus.py:294
    s = torch.exp(sd['ln_s'] * speed_factor)
    cdf, alpha = sdf_to_alpha(sdf, s)
    _, n_m, h_m = nablas_graph(sdf_net, pts_mid)                            # neus.py:103-106, :298
    rad = rad_net.forward(pts_mid, d.unsqueeze(-2).expand_as(pts_mid), n_m, h_m, masks=rad_masks, z_out=rad_z)
    if N_outside > 0:                                                       # neus.py:303-343
        tt = torch.linspace(0, 1, N_outside + 2)[..., 1:-1].float().to(dtype)
        d_out = torch.cat([d_mid, far / torch.flip(tt, dims=[-1])], -1)
        p_out = o[..., None, :] + d[..., None, :] * d_out[..., :, None]
        r = p_out.norm(dim=-1, keepdim=True)
        x_out = torch.cat([p_out / r, 1. / r], -1)
        sigma_out, rad_out = NeRFNet(sd).forward(x_out, d.unsqueeze(-2).expand_as(x_out[..., :3]))
        dists = d_out[..., 1:] - d_out[..., :-1]
        dists = torch.cat([dists, 1e10 * torch.ones(dists[..., :1].shape, dtype=dtype)], -1)
        alpha_out = 1 - torch.exp(-F.softplus(sigma_out) * dists)
        n1 = d_mid.shape[-1]
        inside = (pts_mid.norm(dim=-1) <= obj_bounding_radius)
        alpha = torch.cat([alpha * inside.float() + alpha_out[..., :n1] * (~inside).float(), alpha_out[..., n1:]], -1)
        rad = torch.cat([rad * inside.float()[..., None] + rad_out[..., :n1, :] * (~inside).float()[..., None],
                         rad_out[..., n1:, :]], -2)
    w = alpha_to_w(alpha)
    rgb = torch.sum(w[..., None] * rad, -2)
    acc = torch.sum(w, -1)
    nablas_norm = torch.norm(nablas, dim=-1)                                # neus.py:453-478
    mask_volume = torch.clamp(acc, 1e-3, 1 - 1e-3)
    target_rgb = target_rgb.to(rgb.dtype)
    losses = {'loss_img': F.l1_loss(rgb, target_rgb, reduction='none'),
              'loss_eikonal': w_eikonal * F.mse_loss(nablas_norm, nablas_norm.new_ones(nablas_norm.shape),
                                                     reduction='mean')}
    if with_mask:
        losses['loss_mask'] = w_mask * F.binary_cross_entropy(mask_volume, target_mask.to(mask_volume.dtype),
                                                              reduction='mean')
        losses['loss_img'] = (losses['loss_img'] * target_mask[..., None].float()).sum() / (target_mask.sum() + 1e-10)
    else:
        losses['loss_img'] = losses['loss_img'].mean()
    losses['total'] = sum(losses.values())
    return losses, d_all


def volsdf_train_losses(sd, rays_o, rays_d, target_rgb, eik_points, w_eikonal=0.1, d_all=None, speed_factor=10.0,
                        obj_bounding_radius=3.0, near=0.0, far=6.0, N_samples=64, N_importance=64,
                        max_upsample_steps=6, N_outside=0, siren=False):
    """losses of one VolSDF training step (models/frameworks/volsdf.py:564-640; render :415-506 with
    a graph, builtin background sphere, or with N_outside > 0 the NeRF++ background :451-469 with its
    parameters in the graph): L1 rgb + w_eikonal * MSE(|nabla|, 1) over the highest-weight sample of
    each ray and one eikonal point per ray (eik_points [B, N, 1, 3], the reference's uniform_(-R, R)
    draws).  d_all [B, N, S (+ N_outside)] optional (the sorted sample depths, then the background
    depths; from the oracle's no-grad fine sampling when None).  perturb=False.  siren: the nets of
    configs/volsdf_siren.yaml (SirenLayers, D=5, identity embedding, view embedding 4)."""
    o = rays_o.reshape(rays_o.shape[0], -1, 3).float()
    d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).float(), dim=-1)
    if d_all is None:
        orc = VolSDFOracle({k: v.detach() for k, v in sd.items()}, speed_factor=speed_factor,
                           obj_bounding_radius=obj_bounding_radius, use_nerfplusplus=N_outside > 0, siren=siren)
        with torch.no_grad():
            d_all = orc.render(rays_o, rays_d, near=near, far=far, calc_normal=False, N_samples=N_samples,
                               N_importance=N_importance, max_upsample_steps=max_upsample_steps,
                               N_outside=max(N_outside, 1))['d_vals']
    S = N_samples + N_importance
    d_in = d_all[..., :S]
    if siren:
        sdf_net = SDFNet(sd, D=5, skips=(), multires=-1, siren=True)
        rad_net = RadianceNet(sd, D=5, multires=-1, multires_view=4, siren=True)
    else:
        sdf_net = SDFNet(sd)
        rad_net = RadianceNet(sd, multires=-1, multires_view=-1)
    pts = o[..., None, :] + d[..., None, :] * d_in[..., :, None]             # volsdf.py:446
    sdf, nablas, h = nablas_graph(sdf_net, pts)                               # volsdf.py:450, :317-325
    if N_outside == 0:
        d_bg = obj_bounding_radius - pts.norm(dim=-1)
        sdf = torch.where(d_bg < sdf, d_bg, sdf)
    rad = rad_net.forward(pts, d.unsqueeze(-2).expand_as(pts), nablas, h)
    beta = torch.exp(sd['ln_beta'] * speed_factor)                            # volsdf.py:306-308
    sigma = sdf_to_sigma(sdf, 1. / beta, beta)
    if N_outside > 0:                                                         # volsdf.py:455-469
        B, N = o.shape[:2]
        t_out = torch.linspace(0, 1, N_outside + 2)[..., 1:-1].float()
        rs = (obj_bounding_radius / torch.flip(t_out, dims=[-1])).expand([B, N, N_outside])
        d_out = d_all[..., S:]
        pts_out = o[..., None, :] + d[..., None, :] * d_out[..., :, None]
        x_out = torch.cat([pts_out / rs[..., None], 1. / rs[..., None]], dim=-1)
        sigma_out, rad_out = NeRFNet(sd).forward(x_out, d.unsqueeze(-2).expand_as(pts_out))
        sigma = torch.cat([sigma, sigma_out], -1)
        rad = torch.cat([rad, rad_out], -2)
    delta = d_all[..., 1:] - d_all[..., :-1]                                  # volsdf.py:482-495
    p = torch.exp(-F.relu(sigma[..., :-1] * delta))
    tau = (1 - p + 1e-10) * torch.cumprod(torch.cat([torch.ones_like(p[..., :1]), p], -1), -1)[..., :-1]
    rgb = torch.sum(tau[..., None] * rad[..., :-1, :], -2)
    _, ind = tau[..., :nablas.shape[-2]].max(dim=-1)                          # volsdf.py:604-610
    nab = torch.gather(nablas, dim=-2, index=ind[..., None, None].repeat([*(len(nablas.shape) - 1) * [1], 3]))
    _, nab_eik, _ = nablas_graph(sdf_net, eik_points)
    nab = torch.cat([nab, nab_eik], dim=-2)
    nablas_norm = torch.norm(nab, dim=-1)
    losses = {'loss_img': F.l1_loss(rgb, target_rgb, reduction='none').mean(),
              'loss_eikonal': w_eikonal * F.mse_loss(nablas_norm, nablas_norm.new_ones(nablas_norm.shape),
                                                     reduction='mean')}
    losses['total'] = losses['loss_img'] + losses['loss_eikonal']
    return losses, d_all


def unisurf_train_losses(sd, rays_o, rays_d, target_rgb, surf_perturb, w_reg=0.01, d_all=None, surface_points=None,
                         logit_tau=0.0, radius_of_interest=4.0, interval=1.0, N_query=64, N_freespace=32,
                         netchunk=1048576):
    """losses of one UNISURF training step (models/frameworks/unisurf.py:303-351; render :140-236 with a
    graph): L1 rgb + w_reg * MSE(normalize(nablas at surface points + surf_perturb), normalize(nablas at
    surface points)).  surf_perturb [B, N, 3] = the reference's (torch.rand - 0.5) * 2 * perturb_surface_pts
    draw.  d_all [B, N, P] / surface_points [B, N, 3] optional (from the oracle's no-grad root finding and
    sampling when None).  perturb=False, batched rays [B, N, 3] (F.normalize windows of netchunk points)."""
    from .unisurf import UNISURFOracle
    o = rays_o.reshape(rays_o.shape[0], -1, 3).float()
    d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).float(), dim=-1)
    B, N = o.shape[:2]
    if d_all is None or surface_points is None:
        orc = UNISURFOracle({k: v.detach() for k, v in sd.items()})
        with torch.no_grad():
            out = orc.render(rays_o, rays_d, logit_tau=logit_tau, radius_of_interest=radius_of_interest,
                             interval=interval, N_query=N_query, N_freespace=N_freespace, calc_normal=False)
        d_all = out['d_all'] if d_all is None else d_all
        surface_points = out['surface_points'] if surface_points is None else surface_points
    sdf_net = SDFNet(sd)
    rad_net = RadianceNet(sd, multires=-1, multires_view=-1)
    pts = o[..., None, :] + d[..., None, :] * d_all[..., :, None]              # unisurf.py:207
    P = d_all.shape[-1]
    xf = pts.flatten(1, 2)                                                      # train_util.py:23-71
    vf = d.unsqueeze(-2).expand_as(pts).flatten(1, 2)
    rad, logits = [], []
    for i in range(0, xf.shape[1], netchunk):                                   # unisurf.py:34-38
        occ, nab, h = nablas_graph(sdf_net, xf[:, i:i + netchunk])
        rad.append(rad_net.forward(xf[:, i:i + netchunk], vf[:, i:i + netchunk], F.normalize(nab), h))
        logits.append(occ)
    rad = torch.cat(rad, 1).reshape(B, N, P, 3)
    logits = torch.cat(logits, 1).reshape(B, N, P)
    odds = torch.exp(-1. * logits)                                              # unisurf.py:219-231
    alpha = odds / (1 + odds)
    Tr = torch.cumprod(torch.cat([torch.ones_like(alpha[..., :1]), 1.0 - alpha + 1e-10], -1), -1)
    w = alpha * Tr[..., :-1]
    rgb = torch.sum(w[..., None] * rad, -2)
    losses = {'loss_img': F.l1_loss(rgb, target_rgb)}
    _, nab_s, _ = nablas_graph(sdf_net, surface_points)                         # unisurf.py:331-341
    _, nab_p, _ = nablas_graph(sdf_net, surface_points + surf_perturb)
    losses['loss_reg'] = w_reg * F.mse_loss(F.normalize(nab_p, dim=-1), F.normalize(nab_s, dim=-1))
    losses['total'] = losses['loss_img'] + losses['loss_reg']
    return losses, d_all, surface_points
