"""ORACLE (test infrastructure only): ray generation and 1-D sampling primitives restated from
utils/rend_util.py."""
import torch
import torch.nn.functional as F


def get_rays(c2w, K, H, W, select_inds=None):
    """Pixel -> ray (rend_util.py:112-164, lift :95-109).  Pixel coords are integer indices (no
    +0.5), i = column, j = row; rays_d = c2w @ [x, y, 1, 1] - cam_loc (not normalized)."""
    cam = c2w[..., :3, 3]
    B = c2w.shape[0]
    jj, ii = torch.meshgrid(torch.linspace(0, H - 1, H), torch.linspace(0, W - 1, W), indexing='ij')
    i = ii.reshape(1, H * W).expand(B, H * W)
    j = jj.reshape(1, H * W).expand(B, H * W)
    if select_inds is None:
        select_inds = torch.arange(H * W).expand(B, H * W)
    else:
        i = torch.gather(i, -1, select_inds)
        j = torch.gather(j, -1, select_inds)
    fx, fy = K[:, 0, 0, None], K[:, 1, 1, None]
    cx, cy, sk = K[:, 0, 2, None], K[:, 1, 2, None], K[:, 0, 1, None]
    z = torch.ones_like(i)
    xl = (i - cx + cy * sk / fy - sk * j / fy) / fx * z
    yl = (j - cy) / fy * z
    pc = torch.stack([xl, yl, z, torch.ones_like(z)], dim=-1).transpose(-1, -2)
    world = torch.bmm(c2w, pc).transpose(-1, -2)[..., :3]
    rays_d = world - cam[:, None, :]
    rays_o = cam[:, None, :].expand_as(rays_d)
    return rays_o, rays_d, select_inds


def near_far_from_sphere(o, d, r=1.0, keepdim=True):
    # rend_util.py:167-185
    mid = -torch.sum(o * d, dim=-1, keepdim=keepdim)
    return (mid - r).clamp_min(0.0), (mid + r).clamp_min(r)


def sphere_intersection(o, d, r=1.0):
    # rend_util.py:188-210
    on2 = torch.sum(o ** 2, dim=-1, keepdim=True)
    od = torch.sum(o * d, dim=-1, keepdim=True)
    under = od ** 2 + r ** 2 - on2
    hit = under > 0
    near = torch.zeros_like(od)
    far = torch.zeros_like(od)
    s = torch.sqrt(under[hit])
    near[hit] = -s - od[hit]
    far[hit] = s - od[hit]
    return near.clamp_min(0.0), far.clamp_min(0.0), hit


def dvals_from_radius(o, d, rs, far_end=True):
    # rend_util.py:213-234
    on2 = torch.sum(o ** 2, dim=-1, keepdim=True)
    od = torch.sum(o * d, dim=-1, keepdim=True)
    under = rs ** 2 - (on2 - od ** 2)
    assert (under > 0).all()
    s = torch.sqrt(under)
    return -od + s if far_end else torch.clamp_min(-od - s, 0.)


def _invert_cdf(bins, cdf, n, det, u=None, eps=1e-5):
    # rend_util.py:266-292 / :302-327
    if u is None:
        if det:
            u = torch.linspace(0.0, 1.0, steps=n).expand(*cdf.shape[:-1], n)
        else:
            u = torch.rand(*cdf.shape[:-1], n)
    u = u.contiguous()
    inds = torch.searchsorted(cdf, u, right=False)
    lo = torch.clamp_min(inds - 1, 0)
    hi = torch.clamp_max(inds, cdf.shape[-1] - 1)
    c0, c1 = torch.gather(cdf, -1, lo), torch.gather(cdf, -1, hi)
    b0, b1 = torch.gather(bins, -1, lo), torch.gather(bins, -1, hi)
    denom = c1 - c0
    denom = torch.where(denom < eps, torch.ones_like(denom), denom)
    t = (u - c0) / denom
    return b0 + t * (b1 - b0)


def sample_pdf(bins, weights, n, det=False, u=None):
    """Inverse-CDF sampling (rend_util.py:255-292): weights+1e-5, normalize, cumsum, prepend 0,
    searchsorted(right=False), denom<1e-5 -> 1."""
    w = weights + 1e-5
    pdf = w / torch.sum(w, -1, keepdim=True)
    cdf = torch.cat([torch.zeros_like(pdf[..., :1]), torch.cumsum(pdf, -1)], -1)
    return _invert_cdf(bins, cdf, n, det, u)


def sample_cdf(bins, cdf, n, det=False, u=None):
    # rend_util.py:294-327
    cdf = torch.cat([torch.zeros_like(cdf[..., :1]), cdf], -1)
    return _invert_cdf(bins, cdf, n, det, u)


def normalize(v, dim=-1):
    return F.normalize(v, dim=dim)
