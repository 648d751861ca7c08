"""Config (d) at full size (BASELINE configs[3]): the whole 800x600 NeuS + NeRF++
frame, 480 000 rays, exactly as bench.py's strong-scaling leg renders it (bench.frame_d_inputs: the
bench's model, camera and volume_render kwargs, f16x3, the 16 GiB workspace -> ~30 deferred 16384-ray
chunks).  The reference renders a frame as a loop over `rayschunk` slices (neus.py:384-397,
tools/render_view.py:462-463), each slice independent of the others; here:

  * the one-call render of all 480 000 rays is bit-identical to the same rays rendered in 4096-ray
    calls (chunk invariance at full size: deferred chunks, the NeRF++ background compaction and the
    zero-alpha mid-point skip all run at the frame's real sizes);
  * a world-2 render_sharded(gather=True) of the same frame (two processes on the box's one GPU, gloo
    gather, block-cyclic shares) is bit-identical to it on every rank;
  * the maps are finite and in range (mask in [0, 1], |normals| <= mask).

Per-ray parity against the oracle is covered on 2048 frame rays (tests/test_gpu_nerf.py); this test
pins that nothing changes between that size and the frame's.
"""
import os
import socket
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
MAPS = ('rgb', 'depth_volume', 'mask_volume', 'normals_volume')


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _maps(ex):
    return [ex[k].detach() for k in MAPS]


def _worker(rank, ws, port, q, ref_path):
    sys.path[:0] = [HERE, ROOT]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        import bench
        from neurecon_amd import dist as nd
        from neurecon_amd.frameworks.neus import volume_render
        dev = torch.device('cuda:0')
        model, ro, rd, kw, n = bench.frame_d_inputs(dev, 'f16x3', 16.0)
        with torch.no_grad():
            _, _, ex = nd.render_sharded(volume_render, ro, rd, model, gather=True, **kw)
        torch.cuda.synchronize()
        ref = torch.load(ref_path, weights_only=True)
        diffs = {k: float((a.float() - ref[k].to(dev).float()).abs().max()) for k, a in zip(MAPS, _maps(ex))}
        q.put(('diff', rank, diffs))
        q.put(('done', rank, True))
    except Exception:
        import traceback
        q.put(('error', rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_full_frame_d_chunk_invariant_and_sharded(tmp_path):
    import time
    sys.path.insert(0, ROOT)
    import bench
    from neurecon_amd.frameworks.neus import volume_render
    dev = torch.device('cuda:0')
    model, ro, rd, kw, n = bench.frame_d_inputs(dev, 'f16x3', 16.0)
    assert n == 480000 and ro.shape == (1, n, 3)
    t0 = time.time()
    with torch.no_grad():
        _, _, ex = volume_render(ro, rd, model, **kw)
    torch.cuda.synchronize()
    t1 = time.time()
    full = _maps(ex)
    rgb, depth, mask, normals = full
    assert rgb.shape == (1, n, 3) and depth.shape == (1, n) and normals.shape == (1, n, 3)
    for t in full:
        assert bool(torch.isfinite(t).all())
    assert float(mask.min()) >= 0.0 and float(mask.max()) <= 1.0 + 1e-6
    # normals_volume = sum_i w_i n_i over unit nablas with sum_i w_i = mask <= 1 (neus.py:364-368)
    assert float((normals.norm(dim=-1) - mask).max()) <= 1e-4
    hit = float((mask > 0.5).float().mean())
    # (the bench's untrained model, variance_init 0.05: a soft surface, so most rays are mostly opaque)
    print(f'frame (d): {n} rays in one call {t1 - t0:.2f} s; mask > 0.5 on {hit:.3f} of the rays')

    # the same rays in 4096-ray calls (the reference's rayschunk loop at the bench's chunk size)
    parts = [[] for _ in MAPS]
    with torch.no_grad():
        for i in range(0, n, 4096):
            _, _, e = volume_render(ro[:, i:i + 4096], rd[:, i:i + 4096], model, **kw)
            for lst, t in zip(parts, _maps(e)):
                lst.append(t)
    torch.cuda.synchronize()
    print(f'frame (d): 4096-ray calls {time.time() - t1:.2f} s')
    for name, a, lst in zip(MAPS, full, parts):
        b = torch.cat(lst, dim=1)
        assert torch.equal(a, b), (name, float((a - b).abs().max()), int((a != b).sum()))

    # world 2: two ranks on this GPU, block-cyclic shares, maps gathered on every rank
    ref_path = str(tmp_path / 'frame_d_maps.pt')
    torch.save({k: t.cpu() for k, t in zip(MAPS, full)}, ref_path)
    del ex, full, parts, rgb, depth, mask, normals
    from neurecon_amd import _lib
    _lib._WS.clear()  # the ranks allocate their own 16 GiB workspaces
    torch.cuda.empty_cache()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, ref_path)) for r in range(2)]
    for p in ps:
        p.start()
    msgs = []
    try:
        while sum(1 for m in msgs if m[0] in ('done', 'error')) < 2:
            msgs.append(q.get(timeout=240))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = [m for m in msgs if m[0] == 'error']
    assert not errs, errs[0][2]
    for _, rank, d in (m for m in msgs if m[0] == 'diff'):
        print(f'frame (d) world 2, rank {rank}: max |sharded - one call| {d}')
        assert all(v == 0.0 for v in d.values()), (rank, d)
