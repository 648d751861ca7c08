"""ORACLE (test infrastructure only): VolSDF rendering restated from models/frameworks/volsdf.py
(render mode, builtin background sphere or NeRF++ background, perturb=False or True with torch.rand
drawn in the reference's order)."""
import numpy as np
import torch
import torch.nn.functional as F

from . import rays as R
from .nets import NeRFNet, RadianceNet, SDFNet


def sdf_to_sigma(sdf, alpha, beta):
    # volsdf.py:16-35  sigma = alpha * Psi_beta(-sdf) (Laplace CDF)
    e = 0.5 * torch.exp(-torch.abs(sdf) / beta)
    return alpha * torch.where(sdf >= 0, e, 1 - e)


def _transmittance_integral(d, sdf, alpha, beta):
    # exclusive cumsum of sigma*delta (volsdf.py:57-61, :107-112)
    sigma = sdf_to_sigma(sdf, alpha, beta)
    delta = d[..., 1:] - d[..., :-1]
    Rt = torch.cat([torch.zeros([*sdf.shape[:-1], 1]), torch.cumsum(sigma[..., :-1] * delta, -1)], -1)[..., :-1]
    return Rt, delta


def error_bound(d, sdf, alpha, beta):
    """volsdf.py:38-74: per-interval opacity error bound; NaN -> inf."""
    Rt, delta = _transmittance_integral(d, sdf, alpha, beta)
    a = torch.abs(sdf)
    dstar = torch.clamp_min(0.5 * (a[..., :-1] + a[..., 1:] - delta), 0.)
    err = alpha / (4 * beta) * (delta ** 2) * torch.exp(-dstar / beta)
    b = torch.exp(-Rt) * (torch.exp(torch.cumsum(err, -1)) - 1.)
    b[torch.isnan(b)] = np.inf
    return b


def fine_sample(sdf_fn, d_init, o, d, alpha_net, beta_net, far, eps=0.1, max_iter=5, max_bisection=10,
                N_final=64, N_up=128, perturb=False):
    """Error-bounded adaptive upsampling (volsdf.py:77-272).  Rays that are already within eps keep
    iter_usage 0; k = converged after k rounds; -1 = never (last beta+ used).  perturb: the final
    sample_cdf draws torch.rand per convergence event, in the reference's order (det=not perturb,
    volsdf.py:102)."""
    prefix = d_init.shape[:-1]
    pts = lambda dv, oo, dd: oo[..., None, :] + dd[..., None, :] * dv[..., :, None]

    def finalize(dv, sv, a, b):
        Rt, _ = _transmittance_integral(dv, sv, a, b)
        return R.sample_cdf(dv, 1 - torch.exp(-Rt), N_final, det=not perturb)

    dv = d_init
    out = torch.zeros([*prefix, N_final])
    usage = torch.zeros([*prefix])
    if not isinstance(far, torch.Tensor):
        far = far * torch.ones([*prefix, 1])
    beta = torch.sqrt((far ** 2) / (4 * (d_init.shape[-1] - 1) * np.log(1 + eps)))
    alpha = 1. / beta
    sv = sdf_fn(pts(dv, o, d))
    net_max = error_bound(dv, sv, alpha_net, beta_net).max(dim=-1).values
    mask = net_max > eps
    bm = error_bound(dv, sv, alpha, beta)[mask]
    done = torch.zeros([*prefix], dtype=torch.bool)
    if (~mask).sum() > 0:
        out[~mask] = finalize(dv[~mask], sv[~mask], alpha_net, beta_net)
        usage[~mask] = 0
    done[~mask] = True
    cur = d_init.shape[-1]
    it = 0
    while it < max_iter:
        it += 1
        if mask.sum() == 0:
            break
        up = R.sample_pdf(dv[mask], bm, N_up + 2, det=True)[..., 1:-1]
        dv = torch.cat([dv, torch.zeros([*prefix, N_up])], -1)
        sv = torch.cat([sv, torch.zeros([*prefix, N_up])], -1)
        dm, sm = dv[mask], sv[mask]
        dm[..., cur:cur + N_up] = up
        dm, order = torch.sort(dm, dim=-1)
        sm[..., cur:cur + N_up] = sdf_fn(pts(up, o[mask], d[mask]))
        sm = torch.gather(sm, -1, order)
        dv[mask], sv[mask] = dm, sm
        cur += N_up
        net_max[mask] = error_bound(dv[mask], sv[mask], alpha_net, beta_net).max(dim=-1).values
        still = net_max[mask] > eps
        conv = mask.clone()
        conv[mask] = ~still
        if conv.sum() > 0:
            done[conv] = True
            out[conv] = finalize(dv[conv], sv[conv], alpha_net, beta_net)
            usage[conv] = it
        if still.sum() == 0:
            break
        nmask = mask.clone()
        nmask[mask] = still
        br = beta[nmask]
        bl = beta_net * torch.ones_like(br)
        dt, st = dv[nmask], sv[nmask]
        for _ in range(max_bisection):                                      # volsdf.py:236-243
            bmid = 0.5 * (bl + br)
            mx = error_bound(dt, st, 1. / bmid, bmid).max(dim=-1).values
            br[mx <= eps] = bmid[mx <= eps]
            bl[mx > eps] = bmid[mx > eps]
        beta[nmask] = br
        alpha[nmask] = 1. / beta[nmask]
        bm = torch.clamp(error_bound(dt, st, alpha[nmask], beta[nmask]), 0, 1e5)
        mask = nmask
    if (~done).sum() > 0:
        bp = beta[~done]
        out[~done] = finalize(dv[~done], sv[~done], 1. / bp, bp)
        usage[~done] = -1
    beta[done] = beta_net
    return out, beta, usage


class VolSDFOracle:
    def __init__(self, sd, speed_factor=10.0, obj_bounding_radius=3.0, multires=6, use_nerfplusplus=False,
                 siren=False):
        self.sd = sd
        self.speed_factor = speed_factor
        self.R = obj_bounding_radius
        if siren:  # configs/volsdf_siren.yaml: D=5 SIREN nets, identity embedding, view embedding 4
            self.sdf_net = SDFNet(sd, D=5, skips=(), multires=-1, siren=True)
            self.rad_net = RadianceNet(sd, D=5, multires=-1, multires_view=4, siren=True)
        else:
            self.sdf_net = SDFNet(sd, multires=multires)
            self.rad_net = RadianceNet(sd, multires=-1, multires_view=-1)
        self.nerf = NeRFNet(sd) if use_nerfplusplus else None  # use_sphere_bg = not use_nerfplusplus

    def forward_ab(self):
        # volsdf.py:306-308
        beta = torch.exp(self.sd['ln_beta'] * self.speed_factor)
        return 1. / beta, beta

    def surface(self, x):
        # volsdf.py:310-315 (builtin background sphere; plain network with NeRF++)
        if self.nerf is not None:
            return self.sdf_net.sdf(x)
        return torch.min(self.sdf_net.sdf(x), self.R - x.norm(dim=-1))

    def render(self, rays_o, rays_d, near=0.0, far=6.0, calc_normal=True, N_samples=128, N_importance=64,
               max_upsample_steps=5, max_bisection_steps=10, epsilon=0.1, white_bkgd=False, N_outside=32,
               perturb=False):
        o = rays_o.reshape(rays_o.shape[0], -1, 3).float()
        d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).float(), dim=-1)
        B, N = o.shape[:2]
        nears = near * torch.ones([B, N, 1])
        if self.nerf is not None:                                              # volsdf.py:403-405
            _, fars, hit = R.sphere_intersection(o, d, r=self.R)
            assert hit.all()
        else:
            fars = far * torch.ones([B, N, 1])
        t = torch.linspace(0, 1, N_samples).float()
        d_coarse = nears * (1 - t) + fars * t                                  # volsdf.py:415-417
        alpha, beta = self.forward_ab()
        with torch.no_grad():
            t4 = torch.linspace(0, 1, N_samples * 4).float()
            d_init = nears * (1 - t4) + fars * t4
            d_fine, beta_map, usage = fine_sample(self.surface, d_init, o, d, alpha, beta, fars,
                                                  eps=epsilon, max_iter=max_upsample_steps,
                                                  max_bisection=max_bisection_steps, N_final=N_importance,
                                                  N_up=N_samples * 4, perturb=perturb)
        d_all = torch.sort(torch.cat([d_coarse, d_fine], -1), -1)[0]
        pts = o[..., None, :] + d[..., None, :] * d_all[..., :, None]
        sdf, nablas, h = self.sdf_net.forward_with_nablas(pts)
        if self.nerf is None:
            sdf = torch.min(sdf, self.R - pts.norm(dim=-1))                   # volsdf.py:317-325
        rad = self.rad_net.forward(pts, d.unsqueeze(-2).expand_as(pts), nablas, h)
        sigma = sdf_to_sigma(sdf, alpha, beta)
        extra = {}
        if self.nerf is not None:                                              # volsdf.py:451-469
            t_out = torch.linspace(0, 1, N_outside + 2)[..., 1:-1].float()
            rs = (self.R / torch.flip(t_out, dims=[-1])).expand([B, N, N_outside])
            if perturb:                                                        # volsdf.py:460-465
                mids = .5 * (rs[..., 1:] + rs[..., :-1])
                upper = torch.cat([mids, rs[..., -1:]], -1)
                lower = torch.cat([rs[..., :1], mids], -1)
                rs = lower + (upper - lower) * torch.rand(upper.shape).float()
            d_out = R.dvals_from_radius(o, d, rs)
            pts_out = o[..., None, :] + d[..., None, :] * d_out[..., :, None]
            x_out = torch.cat([pts_out / rs[..., None], 1. / rs[..., None]], dim=-1)
            sigma_out, rad_out = self.nerf.forward(x_out, d.unsqueeze(-2).expand_as(pts_out))
            d_all = torch.cat([d_all, d_out], -1)
            sigma = torch.cat([sigma, sigma_out], -1)
            rad = torch.cat([rad, rad_out], -2)
            extra = dict(sigma_out=sigma_out, radiance_out=rad_out)
        delta = d_all[..., 1:] - d_all[..., :-1]                               # volsdf.py:482-499
        p = torch.exp(-F.relu(sigma[..., :-1] * delta))
        tau = (1 - p + 1e-10) * torch.cumprod(torch.cat([torch.ones_like(p[..., :1]), p], -1), -1)[..., :-1]
        rgb = torch.sum(tau[..., None] * rad[..., :-1, :], -2)
        depth = torch.sum(tau / (tau.sum(-1, keepdim=True) + 1e-10) * d_all[..., :-1], -1)
        acc = torch.sum(tau, -1)
        if white_bkgd:
            rgb = rgb + (1.0 - acc[..., None])
        out = dict(rgb=rgb, depth_volume=depth, mask_volume=acc, implicit_surface=sdf, implicit_nablas=nablas,
                   radiance=rad, alpha=1.0 - p, p_i=p, visibility_weights=tau, d_vals=d_all, sigma=sigma,
                   beta_map=beta_map, iter_usage=usage, **extra)
        if calc_normal:
            nrm = F.normalize(nablas, dim=-1)
            n = min(tau.shape[-1], nrm.shape[-2])
            out['normals_volume'] = (nrm[..., :n, :] * tau[..., :n, None]).sum(dim=-2)
        return out
