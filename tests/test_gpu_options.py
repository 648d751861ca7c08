"""GPU parity of the render options beyond the headline configs, against the reference's own outputs
(tests/golden/options.npz, gen_golden.gen_options):
  * RadianceNet(use_view_dirs=False) (config key model.radiance.use_view_dirs, base.py:334-338,
    :383-384) in NeuS and UNISURF renders, and in surface_render(use_view_dirs=False);
  * UNISURF / root finding with a method other than 'secant' (ray_casting.py:128-135: depth 1 on hits);
  * root finding and sphere tracing with per-ray near / far tensors (ray_casting.py:53-54, :70-73, :175).
Bar as everywhere: 1e-4 relative + 1e-6 absolute, normals 1e-4, masks identical.
"""
import numpy as np
import pytest
import torch

import weightgen as wg
from helpers import neus_model, report, to_gpu, unisurf_model

pytestmark = pytest.mark.gpu

RT, AT = 1e-4, 1e-6


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from neurecon_amd import _lib
    _lib.lib()


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_no_view_dirs_vs_golden(golden, precision):
    from neurecon_amd.frameworks.neus import volume_render
    g = golden('options')
    m = neus_model(wg.neus_state(seed=1, use_view_dirs=False), precision=precision, use_view_dirs=False)
    with torch.no_grad():
        rgb, depth, ex = volume_render(to_gpu(g['neus_rays_o']), to_gpu(g['neus_rays_d']), m, obj_bounding_radius=1.0,
                                       batched=True, calc_normal=True, detailed_output=True, N_samples=64,
                                       N_importance=64, upsample_algo='official_solution', N_upsample_iters=4)
    ok_d, _ = report('d_final', ex['d_final'], g['neus_d_final'], 1e-5, 1e-6)
    same = ok_d.reshape(-1, ok_d.shape[-1]).all(-1)
    ok = (report('rgb', rgb, g['neus_rgb'], RT, AT)[0].all(-1) & report('depth', depth, g['neus_depth'], RT, AT)[0]
          & report('mask', ex['mask_volume'], g['neus_mask'], RT, AT)[0]).reshape(-1)
    print(f'identical samples on {same.mean() * 100:.1f}% of rays, per-ray pass {ok.mean() * 100:.1f}%')
    assert same.mean() >= 0.6 and ok[same].all()
    assert report('normals', ex['normals_volume'], g['neus_normals'], RT, 1e-4)[0].all(-1).reshape(-1)[same].all()
    # the radiance kernel never reads the view dirs: any direction gives the same colours
    with torch.no_grad():
        rgb2, _, _ = volume_render(to_gpu(g['neus_rays_o']), to_gpu(g['neus_rays_d']) * 2.0, m, obj_bounding_radius=1.0,
                                   batched=True, N_samples=64, N_importance=64)
    assert torch.equal(rgb, rgb2)
    with pytest.raises(ValueError):  # the reference fails on the None view dirs (train_util.py:27)
        volume_render(to_gpu(g['neus_rays_o']), to_gpu(g['neus_rays_d']), m, use_view_dirs=False)


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
@pytest.mark.parametrize('tag,method', [('uni', 'secant'), ('uni_nosec', 'none')])
def test_unisurf_options_vs_golden(golden, precision, tag, method):
    from neurecon_amd.frameworks.unisurf import volume_render
    g = golden('options')
    m = unisurf_model(wg.unisurf_state(seed=3, use_view_dirs=False), precision=precision, use_view_dirs=False)
    with torch.no_grad():
        rgb, depth, ex = volume_render(to_gpu(g['uni_rays_o']), to_gpu(g['uni_rays_d']), m, batched=True,
                                       calc_normal=True, detailed_output=True, logit_tau=float(g['uni_logit_tau']),
                                       method=method, radius_of_interest=4.0, interval=1.0, N_query=64,
                                       N_freespace=32)
    assert (ex['mask_surface'].cpu().numpy() == g[tag + '_mask_surface']).all()
    assert report('depth_surface', ex['depth_surface'], g[tag + '_depth_surface'], RT, AT)[0].all()
    assert report('surface_points', ex['surface_points'], g[tag + '_surface_points'], RT, AT)[0].all()
    assert report('rgb', rgb, g[tag + '_rgb'], RT, AT)[0].all()
    assert report('depth', depth, g[tag + '_depth'], RT, AT)[0].all()
    assert report('mask', ex['mask_volume'], g[tag + '_mask'], RT, AT)[0].all()
    assert report('normals', ex['normals_volume'], g[tag + '_normals'], RT, 1e-4)[0].all()


def test_root_finding_per_ray_near_far_vs_golden(golden):
    from neurecon_amd.ray_casting import root_finding_surface_points
    g = golden('options')
    m = neus_model(wg.neus_state(seed=1), precision='f16x3')
    ro = to_gpu(g['rays_o'])
    rd = torch.nn.functional.normalize(torch.from_numpy(g['rays_d']), dim=-1).cuda()
    near, far = to_gpu(g['near']), to_gpu(g['far'])
    for tag, kw in [('rf', dict(N_secant_steps=4, fill_inf=False)), ('rfn', dict(method='none', fill_inf=True))]:
        with torch.no_grad():
            d, p, mask, msc = root_finding_surface_points(m.implicit_surface, ro, rd, near=near, far=far, N_steps=64,
                                                          **kw)
        assert (mask.cpu().numpy() == g[tag + '_mask'].astype(bool)).all()
        assert (msc.cpu().numpy() == g[tag + '_msc'].astype(bool)).all()
        dn = d.cpu().numpy()
        assert (np.isinf(dn) == np.isinf(g[tag + '_d'])).all()
        fin = ~np.isinf(g[tag + '_d'])
        assert report(tag + ' d', dn[fin], g[tag + '_d'][fin], RT, AT)[0].all()
        err = np.abs(p.cpu().numpy() - g[tag + '_pts']).max(-1)
        assert (err <= RT * np.abs(np.where(fin, g[tag + '_d'], 1.0)) + AT).all(), err.max()
    with torch.no_grad(), pytest.raises(ValueError):
        root_finding_surface_points(m.implicit_surface, ro, rd, near=near[..., :3], far=far)


def test_sphere_trace_per_ray_near_far_vs_golden(golden):
    from neurecon_amd.ray_casting import sphere_tracing_surface_points
    g = golden('options')
    m = neus_model(wg.neus_state(seed=1), precision='f16x3')
    rd = torch.nn.functional.normalize(torch.from_numpy(g['rays_d']), dim=-1).cuda()
    with torch.no_grad():
        d, p, mask = sphere_tracing_surface_points(m.implicit_surface, to_gpu(g['rays_o']), rd, near=to_gpu(g['near']),
                                                   far=to_gpu(g['far']), N_iters=10)
    assert (mask.cpu().numpy() == g['st_mask'].astype(bool)).all()
    assert report('st d', d, g['st_d'], RT, AT)[0].all()
    err = np.abs(p.cpu().numpy() - g['st_pts']).max(-1)
    assert (err <= RT * np.abs(g['st_d']) + AT).all(), err.max()


def test_surface_render_no_view_dirs():
    """surface_render(use_view_dirs=False) hands model.forward None view dirs (ray_casting.py:216-226):
    valid for a view-independent radiance net, equal to the use_view_dirs=True render; a view-dependent
    net raises as the reference's embed_fn_view does."""
    from neurecon_amd.ray_casting import surface_render
    from oracle import rays as orays
    H, W, f, dist = wg.CAMERAS['b']
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    m = neus_model(wg.neus_state(seed=1, use_view_dirs=False), precision='f16x3', use_view_dirs=False)
    with torch.no_grad():
        a = surface_render(ro.cuda(), rd.cuda(), m, ray_casting_algo='sphere_tracing', use_view_dirs=False)
        b = surface_render(ro.cuda(), rd.cuda(), m, ray_casting_algo='sphere_tracing')
    assert torch.equal(a[0], b[0]) and bool(a[2]['mask_surface'].any())
    with pytest.raises(TypeError):
        surface_render(ro.cuda(), rd.cuda(), neus_model(wg.neus_state(seed=1), precision='f16x3'),
                       ray_casting_algo='sphere_tracing', use_view_dirs=False)
