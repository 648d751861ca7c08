"""Multi-GPU rendering: one process per GPU (torchrun), rays sharded across ranks.

The render path has no data-path exchange: rays are independent (NeuS / VolSDF), so each rank
renders a contiguous slice of the rays and, when the caller wants the whole frame on every rank,
the per-ray maps are all-gathered once (RCCL over xGMI with backend 'nccl', gloo on CPU).
UNISURF's F.normalize(nablas) couples the points of one `rayschunk` (unisurf.py:36,
train_util.py:23-71); `align` keeps shard boundaries on those chunk boundaries so the result is
identical to a single-process render.
"""
import torch
import torch.distributed as dist


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def shard_bounds(n, rank, world_size, align=1):
    """[lo, hi) ray range of `rank`: contiguous, as even as possible in units of `align` rays."""
    units = (n + align - 1) // align
    lo_u = units * rank // world_size
    hi_u = units * (rank + 1) // world_size
    return min(n, lo_u * align), min(n, hi_u * align)


def shard_rays(rays_o, rays_d, rank=None, world_size=None, align=1, dim=-2):
    """Slice [(B,) N, 3] rays along the ray dimension for this rank."""
    if rank is None:
        rank, world_size = world()
    n = rays_o.shape[dim]
    lo, hi = shard_bounds(n, rank, world_size, align)
    return rays_o.narrow(dim, lo, hi - lo), rays_d.narrow(dim, lo, hi - lo), (lo, hi)


def gather_rays(t, n_total, dim=0, align=1):
    """All-gather per-rank slices (sharded with shard_bounds) back into the full tensor on every rank."""
    rank, ws = world()
    if ws == 1:
        return t
    t = t.contiguous()
    sizes = [shard_bounds(n_total, r, ws, align) for r in range(ws)]
    cap = max(hi - lo for lo, hi in sizes)
    pad_shape = list(t.shape)
    pad_shape[dim] = cap
    buf = torch.zeros(pad_shape, dtype=t.dtype, device=t.device)
    buf.narrow(dim, 0, t.shape[dim]).copy_(t)
    parts = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(parts, buf)
    return torch.cat([p.narrow(dim, 0, hi - lo) for p, (lo, hi) in zip(parts, sizes)], dim)


def render_sharded(render_fn, rays_o, rays_d, model, gather=True, align=1, **kw):
    """Render this rank's slice of the rays with `render_fn(rays_o, rays_d, model, **kw)` (any of the
    frameworks' volume_render); with gather=True the per-ray maps (rgb, depth, every extras entry
    with a ray dimension) are all-gathered so every rank holds the full result."""
    batched = kw.get('batched', False)
    dim = 1 if batched else 0
    n = rays_o.shape[dim]
    ro, rd, _ = shard_rays(rays_o, rays_d, align=align, dim=dim)
    rgb, depth, extras = render_fn(ro, rd, model, **kw)
    if not gather:
        return rgb, depth, extras
    out = {}
    for k, v in extras.items():
        out[k] = gather_rays(v, n, dim=dim, align=align) if isinstance(v, torch.Tensor) and v.dim() > dim else v
    return out['rgb'], out['depth_volume'], out
