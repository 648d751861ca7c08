"""Multi-GPU rendering: one process per GPU (torchrun), rays sharded across ranks.

The render path has no data-path exchange: rays are independent (NeuS / VolSDF), so each rank
renders its share of the rays and, when the caller wants the whole frame on every rank, the per-ray
maps are all-gathered once (RCCL over xGMI with backend 'nccl', gloo on CPU).
Shares are dealt block-cyclically by default (blocks of `block` consecutive rays, block b to rank
b mod world): per-ray work depends on the scene (rays that miss the object skip most of the nets'
work: zero-alpha mid-points, deferred sample nablas), so contiguous row bands of a frame differ in
cost and the slowest band would bound a strong-scaled frame; dealt blocks give every rank a sample
of every band.  The gather puts each block back at its place.  layout='contiguous' keeps one
contiguous range per rank (the reference's DataParallel scatter, neus.py:413-414).
The same driver shards surface_render (sphere tracing / root finding are per ray) and
`sdf_grid_sharded` splits extract_mesh's voxel grid by contiguous index ranges.
UNISURF's F.normalize(nablas) couples the points of one `rayschunk` (unisurf.py:36,
train_util.py:23-71): its shards exchange the per-window sums of nabla^2 (3 doubles per window, one
all-reduce per render call) so the result equals a single-process render at any shard split.
"""
import math

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


BLOCK = 1024  # rays per dealt block of the cyclic layout (the largest; see cyclic_block)
MIN_BLOCKS_PER_RANK = 4


def cyclic_block(n, world_size, align=1, block=BLOCK):
    """Block size of the cyclic layout for n rays: BLOCK, shrunk so that every rank gets at least
    MIN_BLOCKS_PER_RANK blocks (4096 rays on 8 ranks: 128-ray blocks, not 4 busy ranks of 1024), a
    multiple of 16 rays (whole 16-sample tiles in the NeuS chunks) and of `align`."""
    q = 16 * align // math.gcd(16, align)
    want = -(-n // (world_size * MIN_BLOCKS_PER_RANK))
    b = min(block, max(want, 1))
    return max(q, b // q * q)


def cyclic_index(n, rank, world_size, block=BLOCK):
    """ray indices of `rank` in the block-cyclic layout, ascending: blocks rank, rank + world_size, ..."""
    nb = (n + block - 1) // block
    starts = torch.tensor(list(range(rank, nb, world_size)), dtype=torch.int64) * block
    if starts.numel() == 0:
        return torch.empty(0, dtype=torch.int64)
    idx = (starts[:, None] + torch.arange(block, dtype=torch.int64)[None, :]).reshape(-1)
    return idx[idx < n]


def cyclic_count(n, rank, world_size, block=BLOCK):
    nb = (n + block - 1) // block
    full = len(range(rank, nb, world_size)) * block
    last = nb - 1
    if nb and last % world_size == rank:
        full -= nb * block - n
    return full


def gather_cyclic(t, n_total, dim=0, block=BLOCK):
    """All-gather per-rank shares of the block-cyclic layout and put every ray back at its index."""
    rank, ws = world()
    if ws == 1:
        return t
    if t.is_cuda and dist.get_backend() == 'gloo':
        return gather_cyclic(t.cpu(), n_total, dim, block).to(t.device)
    t = t.contiguous()
    counts = [cyclic_count(n_total, r, ws, block) for r in range(ws)]
    cap = max(counts)
    pad_shape = list(t.shape)
    pad_shape[dim] = cap
    buf = torch.zeros(pad_shape, dtype=t.dtype, device=t.device)
    buf.narrow(dim, 0, t.shape[dim]).copy_(t)
    parts = [torch.empty_like(buf) for _ in range(ws)]
    dist.all_gather(parts, buf)
    out_shape = list(t.shape)
    out_shape[dim] = n_total
    out = torch.empty(out_shape, dtype=t.dtype, device=t.device)
    for r, (p, c) in enumerate(zip(parts, counts)):
        idx = cyclic_index(n_total, r, ws, block).to(t.device)
        out.index_copy_(dim, idx, p.narrow(dim, 0, c))
    return out


def gather_rays(t, n_total, dim=0, align=1):
    """All-gather per-rank slices (sharded with shard_bounds) back into the full tensor on every rank."""
    rank, ws = world()
    if ws == 1:
        return t
    if t.is_cuda and dist.get_backend() == 'gloo':  # gloo gathers host tensors only
        return gather_rays(t.cpu(), n_total, dim, align).to(t.device)
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


def render_sharded(render_fn, rays_o, rays_d, model, gather=True, align=1, group=None, layout='cyclic',
                   block=None, **kw):
    """Render this rank's share of the rays with `render_fn(rays_o, rays_d, model, **kw)` (any of the
    frameworks' volume_render); with gather=True the per-ray maps (rgb, depth, every extras entry
    with a ray dimension) are all-gathered so every rank holds the full result, each ray at its
    index.  layout 'cyclic' (default): blocks of `block` rays dealt round-robin (default
    cyclic_block(n, world, align)); 'contiguous': one range per rank (in units of `align` rays).  A
    render whose batched normalisation couples rays across shards (UNISURF, `render_fn.window_sharded`)
    needs contiguous slices: it is told its slice and reduces those sums over the ranks itself (one
    small all-reduce per call).  With gather=False the rank's own maps are returned and
    extras['ray_index'] holds the indices (along the ray dimension) of the rays it rendered."""
    batched = kw.get('batched', False)
    dim = 1 if batched else 0
    n = rays_o.shape[dim]
    rank, ws = world()
    windowed = getattr(render_fn, 'window_sharded', False) and batched and ws > 1
    if layout == 'cyclic' and not windowed and ws > 1:
        if block is None:
            block = cyclic_block(n, ws, align)
        assert block % align == 0, f'render_sharded: block {block} is not a multiple of align {align}'
        idx = cyclic_index(n, rank, ws, block).to(rays_o.device)
        ro, rd = rays_o.index_select(dim, idx), rays_d.index_select(dim, idx)
        rgb, depth, extras = render_fn(ro, rd, model, **kw)
        if not gather:
            extras['ray_index'] = idx
            return rgb, depth, extras
        g = lambda v: gather_cyclic(v, n, dim=dim, block=block)
    else:
        ro, rd, (lo, hi) = shard_rays(rays_o, rays_d, align=align, dim=dim)
        if windowed:
            kw = dict(kw, shard=(lo, n, group))
        rgb, depth, extras = render_fn(ro, rd, model, **kw)
        if not gather:
            extras['ray_index'] = torch.arange(lo, hi, device=rays_o.device)
            return rgb, depth, extras
        g = lambda v: gather_rays(v, n, dim=dim, align=align)
    rgb_all, depth_all = g(rgb), g(depth)
    out = {}
    for k, v in extras.items():
        if v is rgb:
            out[k] = rgb_all
        elif v is depth:
            out[k] = depth_all
        else:
            out[k] = g(v) if isinstance(v, torch.Tensor) and v.dim() > dim else v
    return rgb_all, depth_all, out


def sdf_grid_sharded(implicit_surface, volume_size=2.0, N=512, gather=True, grid_fn=None):
    """extract_mesh's N^3 SDF grid (mesh_util.py:82-108) split into contiguous voxel ranges, one per
    rank (`nr_sdf_grid` evaluates any [i0, i0+n) sub-range with the same coordinates as the whole
    grid); with gather=True one all_gather assembles the [N, N, N] volume on every rank, else the
    rank's flat slice and its range are returned.  `grid_fn(i0, n)` overrides the evaluator (tests)."""
    from .mesh_util import sdf_grid_range
    rank, ws = world()
    total = int(N) ** 3
    lo, hi = shard_bounds(total, rank, ws)
    if grid_fn is None:
        part = sdf_grid_range(implicit_surface, volume_size, N, lo, hi - lo)
    else:
        part = grid_fn(lo, hi - lo)
    if not gather:
        return part, (lo, hi)
    return gather_rays(part, total, dim=0).reshape(N, N, N)
