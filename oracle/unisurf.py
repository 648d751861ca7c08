"""ORACLE (test infrastructure only): UNISURF rendering restated from
models/frameworks/unisurf.py and models/ray_casting.py (render mode, perturb=False)."""
import numpy as np
import torch
import torch.nn.functional as F

from . import rays as R
from .nets import SDFNet, RadianceNet


def root_find(sdf_fn, o, d, near, far, N_steps=256, logit_tau=0.0, N_secant_steps=8, fill_inf=False,
              method='secant'):
    """ray_casting.py:35-160 (batched [B, N, 3]): first outside->inside sign change on a uniform
    256-sample march, refined by 8 secant steps (ray_casting.py:11-30); any other method leaves
    depth 1 on the hits (ray_casting.py:128-135)."""
    B, N = o.shape[:2]
    t = torch.linspace(0., 1., N_steps)[None, None, :]
    dp = near[..., None] * (1 - t) + far[..., None] * t
    val = sdf_fn(o.unsqueeze(-2) + dp.unsqueeze(-1) * d.unsqueeze(-2)) - logit_tau
    first_free = val[..., 0] > 0
    sgn = torch.cat([torch.sign(val[..., :-1] * val[..., 1:]), torch.ones([B, N, 1])], -1)
    cost = sgn * torch.arange(N_steps, 0, -1).float()
    vmin, idx = torch.min(cost, -1)
    crossing = vmin < 0
    pos2neg = torch.gather(val, -1, idx[..., None])[..., 0] > 0
    hit = crossing & pos2neg & first_free
    idx1 = torch.clamp(idx + 1, max=N_steps - 1)
    g = lambda a, i: torch.gather(a, -1, i[..., None])[..., 0][hit]
    d_hi, f_hi, d_lo, f_lo = g(dp, idx), g(val, idx), g(dp, idx1), g(val, idx1)
    om, dm = o[hit], d[hit]
    if method == 'secant' and hit.sum() > 0:
        dpred = -f_lo * (d_hi - d_lo) / (f_hi - f_lo) + d_lo
        for _ in range(N_secant_steps):
            fm = sdf_fn(om + dpred.unsqueeze(-1) * dm).squeeze(-1) - logit_tau
            low = fm < 0
            d_lo[low], f_lo[low] = dpred[low], fm[low]
            d_hi[~low], f_hi[~low] = dpred[~low], fm[~low]
            dpred = -f_lo * (d_hi - d_lo) / (f_hi - f_lo) + d_lo
    else:
        dpred = torch.ones(om.shape[0])
    pt = torch.ones([B, N, 3])
    pt[hit] = om + dpred.unsqueeze(-1) * dm
    dout = torch.ones([B, N])
    dout[hit] = dpred
    dout[~hit] = np.inf if fill_inf else far[~hit]
    dout[~first_free] = 0
    return dout, pt, hit, crossing


class UNISURFOracle:
    def __init__(self, sd, multires=6, use_view_dirs=True):
        self.sdf_net = SDFNet(sd, multires=multires)
        self.rad_net = RadianceNet(sd, multires=-1, multires_view=-1, use_view_dirs=use_view_dirs)

    def forward_chunk(self, x, v):
        # unisurf.py:34-38 -- F.normalize(nablas) with the default dim=1
        occ, nab, h = self.sdf_net.forward_with_nablas(x)
        rad = self.rad_net.forward(x, v, F.normalize(nab), h)
        return rad, occ, nab

    def render(self, rays_o, rays_d, logit_tau=0.0, radius_of_interest=4.0, interval=1.0,
               too_close_threshold=0.1, N_query=64, N_freespace=32, netchunk=1048576, calc_normal=True,
               white_bkgd=False, method='secant'):
        o = rays_o.reshape(rays_o.shape[0], -1, 3).float()
        d = F.normalize(rays_d.reshape(rays_d.shape[0], -1, 3).float(), dim=-1)
        B, N = o.shape[:2]
        near, far = R.near_far_from_sphere(o, d, r=radius_of_interest, keepdim=False)
        thr = near + (far - near) * too_close_threshold
        with torch.no_grad():
            dpred, pt, hit, crossing = root_find(self.sdf_net.sdf, o, d, near, far, logit_tau=logit_tau, method=method)
        dpred = torch.max(torch.min(dpred, far), near)                        # unisurf.py:152-154
        d_up = torch.min(dpred + interval, far)
        d_lo = torch.max(dpred - interval, near)
        t = torch.linspace(0.0, 1.0, steps=N_query)
        d_int = d_lo.unsqueeze(-1) * (1 - t) + d_up.unsqueeze(-1) * t
        d_lo = torch.max(d_lo, thr)                                           # unisurf.py:177-185
        d_lo[crossing == 0] = far[crossing == 0]
        d_lo[d_lo < 1e-10] = far[d_lo < 1e-10]
        t = torch.linspace(0.0, 1.0, steps=N_freespace)
        d_free = torch.ones([B, N, 1]) * near[..., None] * (1 - t) + d_lo.unsqueeze(-1) * t
        d_all = torch.sort(torch.cat([d_free, d_int], -1), -1)[0]
        pts = o[..., None, :] + d[..., None, :] * d_all[..., :, None]
        P = d_all.shape[-1]
        # batchify_query over flattened points (train_util.py:23-71): normalization domain = netchunk
        xf = pts.flatten(1, 2)
        vf = d.unsqueeze(-2).expand_as(pts).flatten(1, 2)
        outs = [self.forward_chunk(xf[:, i:i + netchunk], vf[:, i:i + netchunk])
                for i in range(0, xf.shape[1], netchunk)]
        rad = torch.cat([a for a, _, _ in outs], 1).reshape(B, N, P, 3)
        logits = torch.cat([b for _, b, _ in outs], 1).reshape(B, N, P)
        nab = torch.cat([c for _, _, c in outs], 1).reshape(B, N, P, 3)
        odds = torch.exp(-1. * logits)                                         # unisurf.py:53-62
        alpha = odds / (1 + odds)
        T = torch.cumprod(torch.cat([torch.ones_like(alpha[..., :1]), 1.0 - alpha + 1e-10], -1), -1)
        w = alpha * T[..., :-1]
        rgb = torch.sum(w[..., None] * rad, -2)
        depth = torch.sum(w / (w.sum(-1, keepdim=True) + 1e-10) * d_all, -1)
        acc = torch.sum(w, -1)
        if white_bkgd:
            rgb = rgb + (1.0 - acc[..., None])
        out = dict(rgb=rgb, depth_volume=depth, mask_volume=acc, surface_points=pt, mask_surface=hit,
                   depth_surface=dpred, radiance=rad, implicit_surface=logits, implicit_nablas=nab,
                   alpha=alpha, visibility_weights=w, d_all=d_all)
        if calc_normal:
            nrm = F.normalize(nab, dim=-1)
            n = min(w.shape[-1], nrm.shape[-2])
            out['normals_volume'] = (nrm[..., :n, :] * w[..., :n, None]).sum(dim=-2)
        return out
