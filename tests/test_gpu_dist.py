"""World-size-2 sharded render on the REAL HIP path, both ranks on the box's one GPU.

Two processes (gloo process group: RCCL refuses two ranks on one device) each render their ray
shard through neurecon_amd.dist.render_sharded with the HIP volume_render, and gather the maps.
The result must equal the single-process render of the whole batch:
  * NeuS (config b, 4096 rays) and VolSDF: rays are independent -> bit-identical;
  * UNISURF (config e, 4096 rays = ONE F.normalize window spanning both shards): each rank sums
    its nabla^2 per window, one all-reduce combines them (nr_unisurf_render's window_reduce), so
    the normals fed to the radiance net -- and every output -- match the single-process render
    (fp64 partial sums: equal up to the final fp32 rounding of the window norm).
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, ws, port, q, framework, split):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(here, 'golden'), os.path.dirname(here)]
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        import weightgen as wg
        from helpers import neus_model, unisurf_model, volsdf_model
        from neurecon_amd import dist as nd, rend_util
        from neurecon_amd.frameworks import neus, unisurf, volsdf
        key = {'neus': 'b', 'unisurf': 'e', 'volsdf': 'c'}[framework]
        H, W, f, d = wg.CAMERAS[key]
        ro, rd, _ = rend_util.get_rays(wg.look_at_c2w(d)[None].cuda(), wg.intrinsics(f, H, W)[None].cuda(), H, W)
        if framework == 'neus':
            m = neus_model(wg.neus_state(seed=1), precision='f16x3')
            fn, kw = neus.volume_render, dict(obj_bounding_radius=1.0, N_samples=64, N_importance=64)
        elif framework == 'unisurf':
            m = unisurf_model(wg.unisurf_state(seed=3), precision='f16x3')
            fn, kw = unisurf.volume_render, dict(logit_tau=0.0, N_query=64, N_freespace=32)
        else:
            m = volsdf_model(wg.volsdf_state(seed=5, beta_init=0.1), 0.1, precision='f16x3')
            fn, kw = volsdf.volume_render, dict(N_samples=64, N_importance=64, max_upsample_steps=6)
        kw.update(batched=True, calc_normal=True, detailed_output=True)
        n = ro.shape[1]
        if split != 'even':  # uneven split: rank 0 gets `split` rays (exercises an empty shard at 0)
            lo, hi = (0, int(split)) if rank == 0 else (int(split), n)
            nd.shard_bounds = lambda n_, r_, w_, a_=1: (0, int(split)) if r_ == 0 else (int(split), n_)
        with torch.no_grad():
            rgb, depth, ex = nd.render_sharded(fn, ro, rd, m, **kw)
            ok = True
            if rank == 0:
                rgb1, depth1, ex1 = fn(ro, rd, m, **kw)
                diffs = {k: float((ex[k].float() - ex1[k].float()).abs().max()) for k in
                         ('rgb', 'depth_volume', 'mask_volume', 'normals_volume')}
                q.put(('diff', framework, diffs))
        q.put(('done', rank, True))
    except Exception as e:  # surface the failure to the parent
        import traceback
        q.put(('error', rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _run(framework, split='even'):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, framework, split)) for r in range(2)]
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
    return [m[2] for m in msgs if m[0] == 'diff'][0]


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')


@pytest.mark.parametrize('framework', ['neus', 'volsdf'])
def test_sharded_render_is_bit_identical_world2(framework):
    d = _run(framework)
    print(framework, d)
    assert all(v == 0.0 for v in d.values()), d


@pytest.mark.parametrize('split', ['even', '1500', '0'])
def test_unisurf_sharded_window_normalisation_world2(split):
    """config (e): 4096 rays in ONE normalisation window split over two ranks (evenly, unevenly and
    with an empty shard on rank 0)."""
    d = _run('unisurf', split)
    print('unisurf', split, d)
    assert max(d.values()) <= 1e-6, d
