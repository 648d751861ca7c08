"""World-size-2 gloo run of the ray-sharded render driver (neurecon_amd/dist.py) on the CPU.

The render function here is a stand-in with the frameworks' calling convention (the HIP render
needs a GPU); what is checked is the sharding, the chunk alignment and the all-gather, i.e. that
a sharded render reassembles bit-for-bit into the single-process result."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from neurecon_amd import dist as nd


def _fake_render(ro, rd, model, batched=True, **kw):
    # per-ray, order-independent function of the ray, same output structure as volume_render
    rgb = torch.stack([ro.sum(-1), rd.sum(-1), (ro * rd).sum(-1)], -1)
    depth = ro.norm(dim=-1)
    return rgb, depth, {'rgb': rgb, 'depth_volume': depth, 'mask_volume': rd.norm(dim=-1),
                        'implicit_surface': ro[..., :1].expand(*ro.shape[:-1], 5).contiguous(), 'scalar': 3}


def _worker(rank, ws, port, q, align, layout='contiguous', block=nd.BLOCK):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        g = torch.Generator().manual_seed(0)
        ro = torch.randn(1, 37, 3, generator=g)
        rd = torch.randn(1, 37, 3, generator=g)
        seen = []
        fr = lambda o, d, m, **kw: (seen.append(o.shape[1]), _fake_render(o, d, m, **kw))[1]
        rgb, depth, ex = nd.render_sharded(fr, ro, rd, None, batched=True, align=align, layout=layout, block=block)
        if layout == 'cyclic':
            b = block if block is not None else nd.cyclic_block(37, ws, align)
            ok_n = seen == [nd.cyclic_count(37, rank, ws, b)]
        else:
            ok_n = True
        ref = _fake_render(ro, rd, None)
        ok = (ok_n and torch.equal(rgb, ref[0]) and torch.equal(depth, ref[1]) and
              torch.equal(ex['implicit_surface'], ref[2]['implicit_surface']) and ex['scalar'] == 3)
        # gather=False: the rank's own maps and the indices of its rays
        rgb_s, _, ex_s = nd.render_sharded(_fake_render, ro, rd, None, batched=True, align=align, layout=layout,
                                           block=block, gather=False)
        idx = ex_s['ray_index']
        ok = ok and torch.equal(rgb_s, ref[0][:, idx])
        if layout == 'cyclic':
            b = block if block is not None else nd.cyclic_block(37, ws, align)
            ok = ok and torch.equal(idx, nd.cyclic_index(37, rank, ws, b))
        lo, hi = nd.shard_bounds(37, rank, ws, align)
        q.put((rank, ok, lo, hi))
    finally:
        dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('align', [1, 8])
def test_sharded_render_reassembles_world2(align):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, align, 'contiguous')) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res)
    (_, _, lo0, hi0), (_, _, lo1, hi1) = res
    assert lo0 == 0 and hi0 == lo1 and hi1 == 37
    assert hi0 % align == 0


@pytest.mark.parametrize('ws,block', [(2, 5), (3, 4), (2, 1024), (3, None)])
def test_cyclic_sharded_render_reassembles(ws, block):
    """block-cyclic shares (the default layout): every rank renders its dealt blocks, the all-gather
    puts every ray back at its index -- bit-identical to the single-process result"""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, ws, port, q, 1, 'cyclic', block)) for r in range(ws)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res


def test_cyclic_index_partitions():
    for n in (0, 1, 5, 37, 4096, 4097, 480000):
        for ws in (1, 2, 3, 8):
            for block in (1, 5, 1024):
                parts = [nd.cyclic_index(n, r, ws, block) for r in range(ws)]
                assert [p.numel() for p in parts] == [nd.cyclic_count(n, r, ws, block) for r in range(ws)]
                allidx = torch.cat(parts).sort().values if n else torch.empty(0, dtype=torch.int64)
                assert torch.equal(allidx, torch.arange(n))
                assert all(bool((p[1:] > p[:-1]).all()) for p in parts if p.numel() > 1)


def test_cyclic_block_keeps_every_rank_busy():
    """the default block (cyclic_block) deals every rank >= MIN_BLOCKS_PER_RANK blocks on small frames,
    stays at BLOCK on large ones, and is a multiple of 16 and of align"""
    assert nd.cyclic_block(480000, 8) == nd.BLOCK
    for n in (37, 4096, 4097, 65536, 480000):
        for ws in (2, 3, 8):
            for align in (1, 8, 48):
                b = nd.cyclic_block(n, ws, align)
                assert b % 16 == 0 and b % align == 0 and b <= max(nd.BLOCK, 48)
                if n >= ws * nd.MIN_BLOCKS_PER_RANK * 48:
                    assert all(nd.cyclic_count(n, r, ws, b) > 0 for r in range(ws)), (n, ws, b)
    assert nd.cyclic_block(4096, 8) == 128   # 4096 rays on 8 ranks: 512 rays per rank


def test_shard_bounds_cover_and_align():
    for n in (1, 5, 64, 4096, 4097):
        for ws in (1, 2, 3, 8):
            for align in (1, 16, 1000):
                b = [nd.shard_bounds(n, r, ws, align) for r in range(ws)]
                assert b[0][0] == 0 and b[-1][1] == n
                assert all(b[i][1] == b[i + 1][0] for i in range(ws - 1))
                assert all(lo % align == 0 for lo, _ in b if lo < n)


def _fake_surface_render(ro, rd, model, batched=True, **kw):
    # surface_render's return convention: (colors, depths, extras without rgb/depth keys)
    c = torch.stack([ro.sum(-1), rd.sum(-1), (ro * rd).sum(-1)], -1)
    d = ro.norm(dim=-1)
    return c, d, {'implicit_nablas': rd * 2, 'mask_surface': d > 1.0}


def _fake_grid(N, s):
    from oracle.surface import grid_points
    pts = torch.from_numpy(grid_points(N, s))
    return lambda i0, n: pts[i0:i0 + n].norm(dim=-1)


def _worker_surface(rank, ws, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        g = torch.Generator().manual_seed(1)
        ro = torch.randn(1, 41, 3, generator=g)
        rd = torch.randn(1, 41, 3, generator=g)
        c, d, ex = nd.render_sharded(_fake_surface_render, ro, rd, None, batched=True)
        ref = _fake_surface_render(ro, rd, None)
        ok = (torch.equal(c, ref[0]) and torch.equal(d, ref[1]) and
              torch.equal(ex['implicit_nablas'], ref[2]['implicit_nablas']) and
              torch.equal(ex['mask_surface'], ref[2]['mask_surface']))
        N, s = 9, 2.0
        grid = nd.sdf_grid_sharded(None, s, N, grid_fn=_fake_grid(N, s))
        ok = ok and torch.equal(grid, _fake_grid(N, s)(0, N ** 3).reshape(N, N, N))
        part, (lo, hi) = nd.sdf_grid_sharded(None, s, N, gather=False, grid_fn=_fake_grid(N, s))
        ok = ok and part.numel() == hi - lo
        q.put((rank, ok, lo, hi))
    finally:
        dist.destroy_process_group()


def test_sharded_surface_render_and_grid_world2():
    """surface_render's (colors, depths, extras) convention and the voxel-range split of the mesh grid
    reassemble exactly into the single-process result."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_surface, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(ok for _, ok, _, _ in res), res
    assert res[0][2] == 0 and res[0][3] == res[1][2] and res[1][3] == 9 ** 3
