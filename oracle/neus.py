"""ORACLE (test infrastructure only): NeuS volume rendering restated from
models/frameworks/neus.py (render mode)."""
import math
import torch
import torch.nn.functional as F

from . import rays as R
from .nets import SDFNet, RadianceNet, NeRFNet


def logistic_cdf(x, s):
    # neus.py:21-25
    return torch.sigmoid(x * s)


def sdf_to_alpha(sdf, s):
    # neus.py:28-35: alpha_i = max((c_i - c_{i+1}) / (c_i + 1e-10), 0)
    c = logistic_cdf(sdf, s)
    return c, torch.clamp_min((c[..., :-1] - c[..., 1:]) / (c[..., :-1] + 1e-10), 0)


def alpha_to_w(alpha):
    # neus.py:57-70: w_i = alpha_i * prod_{j<i}(1 - alpha_j + 1e-10)
    T = torch.cumprod(torch.cat([torch.ones_like(alpha[..., :1]), 1.0 - alpha + 1e-10], -1), -1)
    return alpha * T[..., :-1]


class NeuSOracle:
    def __init__(self, sd, speed_factor=10.0, use_outside_nerf=False, multires=6, multires_view=4, use_view_dirs=True):
        self.sd = sd
        self.speed_factor = speed_factor
        self.sdf_net = SDFNet(sd, multires=multires)
        # use_view_dirs=False: the radiance net ignores the directions it is handed (base.py:383-384)
        self.rad_net = RadianceNet(sd, multires_view=multires_view, use_view_dirs=use_view_dirs)
        self.nerf = NeRFNet(sd) if use_outside_nerf else None

    def s(self):
        # neus.py:108-109
        return torch.exp(self.sd['ln_s'] * self.speed_factor)

    def radiance(self, x, v):
        # neus.py:103-106
        _, n, h = self.sdf_net.forward_with_nablas(x)
        return self.rad_net.forward(x, v, n, h)

    def render(self, rays_o, rays_d, obj_bounding_radius=1.0, calc_normal=True, N_samples=64,
               N_importance=64, N_outside=0, upsample_algo='official_solution', N_upsample_iters=4,
               N_nograd_samples=2048, fixed_s_recp=1 / 64., white_bkgd=False, perturb=False):
        """neus.py:118-397 for one ray chunk, batched layout [B, N, 3], perturb=False."""
        assert not perturb
        o = rays_o.reshape(rays_o.shape[0], -1, 3).float()
        d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).float(), dim=-1)
        near, far = R.near_far_from_sphere(o, d, r=obj_bounding_radius)
        view = d
        d_all = self.sample_depths(o, d, near, far, N_samples, N_importance, upsample_algo, N_upsample_iters,
                                   N_nograd_samples, fixed_s_recp)
        return self.integrate(o, d, near, far, d_all, view, obj_bounding_radius, calc_normal, N_outside, white_bkgd)

    def sample_depths(self, o, d, near, far, N_samples=64, N_importance=64, upsample_algo='official_solution',
                      N_upsample_iters=4, N_nograd_samples=2048, fixed_s_recp=1 / 64.):
        """the no-grad upsampling (neus.py:206-279) -> sorted sample depths [B, N, S]"""
        pts_of = lambda dv: o.unsqueeze(-2) + dv.unsqueeze(-1) * d.unsqueeze(-2)
        t = torch.linspace(0, 1, N_samples).float()
        d_coarse = near * (1 - t) + far * t                                   # neus.py:209-210
        with torch.no_grad():
            if upsample_algo == 'direct_use':                                 # neus.py:216-229
                sdf_c = self.sdf_net.sdf(pts_of(d_coarse))
                _, a = sdf_to_alpha(sdf_c, 1. / fixed_s_recp)
                d_fine = R.sample_pdf(d_coarse, alpha_to_w(a), N_importance, det=True)
                d_all = torch.sort(torch.cat([d_coarse, d_fine], -1), -1)[0]
            elif upsample_algo == 'direct_more':                              # neus.py:233-243
                tt = torch.linspace(0, 1, N_nograd_samples).float()
                dd = near * (1 - tt) + far * tt
                _, a = sdf_to_alpha(self.sdf_net.sdf(pts_of(dd)), 1. / fixed_s_recp)
                d_fine = R.sample_pdf(dd, alpha_to_w(a), N_importance, det=True)
                d_all = torch.sort(torch.cat([d_coarse, d_fine], -1), -1)[0]
            elif upsample_algo == 'official_solution':                        # neus.py:249-277
                dv = d_coarse
                sv = self.sdf_net.sdf(pts_of(dv))
                for i in range(N_upsample_iters):
                    s0, s1 = sv[..., :-1], sv[..., 1:]
                    z0, z1 = dv[..., :-1], dv[..., 1:]
                    mid = (s0 + s1) * 0.5
                    slope = (s1 - s0) / (z1 - z0 + 1e-5)
                    prev = torch.cat([torch.zeros_like(slope[..., :1]), slope[..., :-1]], -1)
                    slope = torch.min(torch.stack([prev, slope], -1), -1)[0].clamp(-10.0, 0.0)
                    dist = z1 - z0
                    e0 = mid - slope * dist * 0.5
                    e1 = mid + slope * dist * 0.5
                    c0 = logistic_cdf(e0, 64 * (2 ** i))
                    c1 = logistic_cdf(e1, 64 * (2 ** i))
                    a = (c0 - c1 + 1e-5) / (c0 + 1e-5)
                    d_fine = R.sample_pdf(dv, alpha_to_w(a), N_importance // N_upsample_iters, det=True)
                    dv = torch.cat([dv, d_fine], -1)
                    sv = torch.cat([sv, self.sdf_net.sdf(pts_of(d_fine))], -1)
                    dv, order = torch.sort(dv, -1)
                    sv = torch.gather(sv, -1, order)
                d_all = dv
            else:
                raise NotImplementedError(upsample_algo)
        return d_all

    def integrate(self, o, d, near, far, d_all, view, obj_bounding_radius=1.0, calc_normal=True, N_outside=0,
                  white_bkgd=False):
        """neus.py:284-382 from given sample depths"""
        pts = o[..., None, :] + d[..., None, :] * d_all[..., :, None]          # neus.py:284
        d_mid = 0.5 * (d_all[..., 1:] + d_all[..., :-1])                       # neus.py:287
        pts_mid = o[..., None, :] + d[..., None, :] * d_mid[..., :, None]
        sdf, nablas, _ = self.sdf_net.forward_with_nablas(pts)                 # neus.py:294
        cdf, alpha = sdf_to_alpha(sdf, self.s())                               # neus.py:296
        radiances = self.radiance(pts_mid, view.unsqueeze(-2).expand_as(pts_mid))
        out = {}
        if N_outside > 0:                                                      # neus.py:303-343
            tt = torch.linspace(0, 1, N_outside + 2)[..., 1:-1].float()
            d_out = far / torch.flip(tt, dims=[-1])
            d_out = torch.cat([d_mid, d_out], -1)
            p_out = o[..., None, :] + d[..., None, :] * d_out[..., :, None]
            r = p_out.norm(dim=-1, keepdim=True)
            x_out = torch.cat([p_out / r, 1. / r], -1)
            with torch.no_grad():
                sigma_out, rad_out = self.nerf.forward(x_out, view.unsqueeze(-2).expand_as(x_out[..., :3]))
            dists = d_out[..., 1:] - d_out[..., :-1]
            dists = torch.cat([dists, 1e10 * torch.ones(dists[..., :1].shape)], -1)
            alpha_out = 1 - torch.exp(-F.softplus(sigma_out) * dists)
            n1 = d_mid.shape[-1]
            inside = (pts_mid.norm(dim=-1) <= obj_bounding_radius)
            a_in = alpha * inside.float() + alpha_out[..., :n1] * (~inside).float()
            alpha = torch.cat([a_in, alpha_out[..., n1:]], -1)
            r_in = radiances * inside.float()[..., None] + rad_out[..., :n1, :] * (~inside).float()[..., None]
            radiances = torch.cat([r_in, rad_out[..., n1:, :]], -2)
            d_final = d_out
            out['sigma_out'], out['radiance_out'] = sigma_out, rad_out
        else:
            d_final = d_mid
        w = alpha_to_w(alpha)                                                  # neus.py:346-352
        rgb = torch.sum(w[..., None] * radiances, -2)
        depth = torch.sum(w / (w.sum(-1, keepdim=True) + 1e-10) * d_final, -1)
        acc = torch.sum(w, -1)
        if white_bkgd:
            rgb = rgb + (1.0 - acc[..., None])
        out.update(rgb=rgb, depth_volume=depth, mask_volume=acc, implicit_nablas=nablas,
                   implicit_surface=sdf, radiance=radiances, alpha=alpha, cdf=cdf,
                   visibility_weights=w, d_final=d_final)
        if calc_normal:                                                        # neus.py:364-368
            nrm = F.normalize(nablas, dim=-1)
            n = min(w.shape[-1], nrm.shape[-2])
            out['normals_volume'] = (nrm[..., :n, :] * w[..., :n, None]).sum(dim=-2)
        return out
