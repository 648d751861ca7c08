"""GPU parity of surface rendering (nr_sphere_trace + model.forward + nr_surface_finish) and of the
mesh-extraction SDF grid (nr_sdf_grid) vs the reference's golden vectors and the oracle.

Tolerance (north star): |gpu - ref| <= 1e-4 * |ref| + 1e-6 on rgb / depth; normals 1e-4
absolute; hit masks identical.  SDF grid values: 1e-4 relative + 1e-5 absolute (the SDF
network's fp32-level error is ~1.4e-6 absolute).
"""
import numpy as np
import pytest
import torch

import weightgen as wg
from helpers import neus_model, report, to_gpu

pytestmark = pytest.mark.gpu

RT, AT = 1e-4, 1e-6


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from neurecon_amd import _lib
    _lib.lib()


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_surface_render_vs_golden(golden, precision):
    """Two parts.  (1) Tracing: hit masks identical and depth within the bar on every ray.
    (2) Shading: rgb / nablas / normals at the GPU's own surface points vs the oracle at those
    points, every element within the bar.  End to end, rgb vs the golden is held to >= 99 % of
    elements: sphere tracing accumulates the SDF's rounding over 20 iterations and surface nablas
    move with the hit point (softplus(100 z) curvature) — the reference itself, with 1e-6 random
    noise added to its SDF, keeps 99.3-100 % of rgb and 83-95 % of nablas within 1e-4 of its own
    unperturbed output."""
    from oracle.nets import RadianceNet, SDFNet
    from neurecon_amd.ray_casting import _normalize3, sphere_tracing_surface_points, surface_render
    g = golden('surface')
    sd = wg.neus_state(seed=int(g['seed']))
    m = neus_model(sd, precision=precision)
    ro = to_gpu(g['rays_o'])
    rgb, depth, ex = surface_render(ro, to_gpu(g['rays_d']), m, calc_normal=True, batched=True,
                                    ray_casting_algo='sphere_tracing')
    torch.cuda.synchronize()
    mask = ex['mask_surface'].cpu().numpy()
    print(f'hit rays: {mask.sum()} / {mask.size}')
    assert (mask == g['mask'].astype(bool)).all()
    assert report('depth', depth, g['depth'], RT, AT)[0].all()
    ok_rgb, _ = report('rgb (end to end)', rgb, g['rgb'], RT, AT)
    assert ok_rgb.mean() >= 0.99
    # shading parity at the traced points
    with torch.no_grad():
        rdn = _normalize3(to_gpu(g['rays_d']))
        _, pts, _ = sphere_tracing_surface_points(m.implicit_surface, ro, rdn)
        p, v = pts.cpu(), rdn.cpu()
        _, nab_ref, h = SDFNet(sd).forward_with_nablas(p)
        c_ref = RadianceNet(sd).forward(p, v, nab_ref, h)
    mk = torch.from_numpy(mask)
    c_ref[~mk] = 0
    n_ref = torch.nn.functional.normalize(nab_ref, dim=-1)
    n_ref[~mk] = 0
    assert report('rgb (at traced points)', rgb, c_ref, RT, AT)[0].all()
    nab, ref = ex['implicit_nablas'].cpu().numpy(), nab_ref.numpy()
    err = np.abs(nab - ref).max(-1)
    print(f'nablas (at traced points): max abs {err.max():.3e}')
    assert (err <= 1e-4 * np.linalg.norm(ref, axis=-1) + 1e-6).all()
    assert report('normals (at traced points)', ex['normals_surface'], n_ref, RT, 1e-4)[0].all()


def test_sphere_trace_cfgs_vs_golden(golden):
    """near/far/N_iters forwarded as ray_casting_cfgs would (ray_casting.py:215-216)."""
    from neurecon_amd.ray_casting import sphere_tracing_surface_points
    g = golden('surface')
    m = neus_model(wg.neus_state(seed=int(g['seed'])), precision='f16x3')
    rd = torch.nn.functional.normalize(torch.from_numpy(g['rays_d']), dim=-1)
    with torch.no_grad():
        d, p, mask = sphere_tracing_surface_points(m.implicit_surface, to_gpu(g['rays_o']), rd.cuda(), near=0.5,
                                                   far=4.0, N_iters=5)
    assert (mask.cpu().numpy() == g['st5_mask'].astype(bool)).all()
    assert report('d', d, g['st5_d'], RT, AT)[0].all()
    # points inherit the depth error along the ray: held to 1e-4 of the depth
    err = np.abs(p.cpu().numpy() - g['st5_pts']).max(-1)
    assert (err <= RT * np.abs(g['st5_d']) + AT).all(), err.max()


def test_sphere_trace_full_camera_vs_oracle():
    """All 4096 config-(b) camera rays (unbatched layout) vs the oracle; plus the edge cases
    N_iters=0 (pts at near, every ray active) and an empty ray set."""
    from oracle.surface import sphere_trace
    from oracle.nets import SDFNet
    from oracle.rays import get_rays
    from neurecon_amd.ray_casting import sphere_tracing_surface_points
    sd = wg.neus_state(seed=1)
    H, W, f, dist = wg.CAMERAS['b']
    ro, rd, _ = get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    ro, rd = ro[0], torch.nn.functional.normalize(rd[0], dim=-1)
    net = SDFNet(sd)
    with torch.no_grad():
        d_ref, p_ref, m_ref = sphere_trace(net.sdf, ro, rd)
        m = neus_model(sd, precision='f16x3')
        d, p, mask = sphere_tracing_surface_points(m.implicit_surface, ro.cuda(), rd.cuda(), batched=False)
        agree = mask.cpu().numpy() == m_ref.numpy()
        print(f'hit {int(m_ref.sum())} / {m_ref.numel()}, mask agreement {agree.mean() * 100:.3f}%')
        assert agree.mean() >= 0.999
        ok = report('d', d, d_ref, RT, AT)[0] | ~agree
        assert ok.mean() >= 0.999
        d0, p0, m0 = sphere_tracing_surface_points(m.implicit_surface, ro.cuda(), rd.cuda(), near=0.25, N_iters=0)
        assert bool(m0.all()) and bool((d0 == 0.25).all())
        assert torch.equal(p0.cpu(), ro + rd * torch.full((ro.shape[0],), 0.25)[:, None])
        e = sphere_tracing_surface_points(m.implicit_surface, ro[:0].cuda(), rd[:0].cuda())
        assert e[0].numel() == 0


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_sdf_grid_vs_golden(golden, precision):
    from neurecon_amd.mesh_util import sdf_grid
    g = golden('surface')
    m = neus_model(wg.neus_state(seed=int(g['seed'])), precision=precision)
    for N, s in [(16, 2.0), (24, 1.5)]:
        with torch.no_grad():
            out = sdf_grid(m.implicit_surface, s, N, chunk=1000)  # ragged last chunk
        assert tuple(out.shape) == (N, N, N)
        assert report(f'grid{N}', out, g[f'grid{N}'], RT, 1e-5)[0].all()


def test_sdf_grid_512_consistency():
    """Full extract_mesh size (512^3 = 134 M points): the device grid equals ImplicitSurface.forward
    on the reference's float64 grid formula (oracle.surface.grid_points, evaluated only at sampled
    indices).  Both run the same SDF kernel on (expected) bit-identical points; the bar is the
    SDF tolerance, and the exact-match fraction is printed."""
    from neurecon_amd.mesh_util import sdf_grid
    N, s = 512, 2.0
    m = neus_model(wg.neus_state(seed=1), precision='f16x3')
    with torch.no_grad():
        out = sdf_grid(m.implicit_surface, s, N).reshape(-1)
        torch.cuda.synchronize()
        assert bool(torch.isfinite(out).all())
        rs = np.random.RandomState(0)
        i = np.concatenate([rs.randint(0, N ** 3, 4096), [0, N ** 3 - 1, N - 1, N * N - 1]]).astype(np.int64)
        step, o = s / (N - 1), -s / 2.
        xyz = np.stack([(((i / N) / N) % N) * step + o, ((i / N) % N) * step + o, (i % N) * step + o], -1)
        ref = m.implicit_surface.forward(torch.from_numpy(xyz.astype(np.float32)).cuda())
        got = out[torch.from_numpy(i).cuda()]
        print(f'grid512: exact on {(got == ref).float().mean().item() * 100:.2f}% of sampled voxels')
        assert report('grid512', got, ref.cpu(), RT, 1e-6)[0].all()


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_surface_render_root_finding_vs_golden(golden, precision):
    """surface_render(ray_casting_algo='root_finding') (ray_casting.py:35-160, 219-221): 256-step march,
    first outside->inside crossing, 8 secant steps.  Masks identical, depth within the bar on hits
    (inf on misses), shading at the traced points vs the oracle as for sphere tracing."""
    from oracle.nets import RadianceNet, SDFNet
    from neurecon_amd.ray_casting import _normalize3, root_finding_surface_points, surface_render
    g = golden('surface')
    sd = wg.neus_state(seed=int(g['seed']))
    m = neus_model(sd, precision=precision)
    ro = to_gpu(g['rays_o'])
    rgb, depth, ex = surface_render(ro, to_gpu(g['rays_d']), m, calc_normal=True, batched=True,
                                    ray_casting_algo='root_finding')
    torch.cuda.synchronize()
    mask = ex['mask_surface'].cpu().numpy()
    print(f'hit rays: {mask.sum()} / {mask.size}')
    assert (mask == g['rf_mask'].astype(bool)).all()
    dep = depth.cpu().numpy()
    assert (np.isinf(dep) == np.isinf(g['rf_depth'])).all()
    assert report('depth (hits)', dep[mask], g['rf_depth'][mask], RT, AT)[0].all()
    assert report('rgb (end to end)', rgb, g['rf_rgb'], RT, AT)[0].mean() >= 0.99
    with torch.no_grad():
        rdn = _normalize3(to_gpu(g['rays_d']))
        _, pts, _, _ = root_finding_surface_points(m.implicit_surface, ro, rdn)
        p, v = pts.cpu(), rdn.cpu()
        _, nab_ref, h = SDFNet(sd).forward_with_nablas(p)
        c_ref = RadianceNet(sd).forward(p, v, nab_ref, h)
    mk = torch.from_numpy(mask)
    c_ref[~mk] = 0
    n_ref = torch.nn.functional.normalize(nab_ref, dim=-1)
    n_ref[~mk] = 0
    assert report('rgb (at traced points)', rgb, c_ref, RT, AT)[0].all()
    assert report('normals (at traced points)', ex['normals_surface'], n_ref, RT, 1e-4)[0].all()


def test_root_finding_cfgs_vs_golden(golden):
    """root_finding_surface_points with near/far, N_steps=64, N_secant_steps=4, logit_tau=0.01,
    fill_inf=False (misses get far, occupied first samples 0)."""
    from neurecon_amd.ray_casting import root_finding_surface_points
    g = golden('surface')
    m = neus_model(wg.neus_state(seed=int(g['seed'])), precision='f16x3')
    rd = torch.nn.functional.normalize(torch.from_numpy(g['rays_d']), dim=-1)
    with torch.no_grad():
        d, p, mask, msc = root_finding_surface_points(m.implicit_surface, to_gpu(g['rays_o']), rd.cuda(), near=0.5,
                                                      far=4.0, N_steps=64, N_secant_steps=4, logit_tau=0.01,
                                                      fill_inf=False)
    mask = mask.cpu().numpy()
    assert (mask == g['rf2_mask'].astype(bool)).all()
    assert (msc.cpu().numpy() == g['rf2_msc'].astype(bool)).all()
    assert report('d', d, g['rf2_d'], RT, AT)[0].all()
    err = np.abs(p.cpu().numpy() - g['rf2_pts']).max(-1)
    assert (err <= RT * np.abs(g['rf2_d']) + AT).all(), err.max()


def test_sdf_grid_range_matches_full_grid():
    """A voxel sub-range (what one rank of dist.sdf_grid_sharded evaluates) is bit-identical to the
    same slice of the whole grid; out-of-range requests raise."""
    from neurecon_amd.mesh_util import sdf_grid, sdf_grid_range
    m = neus_model(wg.neus_state(seed=1), precision='f16x3')
    N = 24
    with torch.no_grad():
        full = sdf_grid(m.implicit_surface, 1.5, N).reshape(-1)
        part = sdf_grid_range(m.implicit_surface, 1.5, N, 1000, 5001, chunk=777)
    assert torch.equal(part, full[1000:6001])
    with pytest.raises(ValueError):
        sdf_grid_range(m.implicit_surface, 1.5, N, N ** 3 - 3, 4)


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_root_finding_chunked_march_bit_identical(precision):
    """nr_root_find's march runs in chunks of 32 steps over the rays still without a sign change
    (run_march, shared with UNISURF): d_pred / pts / mask / mask_sign_change and the surface_render
    maps equal the single-launch march over every step of every ray (_full_march=True) bit for bit,
    on a wide-angle camera where rays hit, miss and graze the surface; plus N_steps that are not a
    multiple of 32 and fewer than 32 steps."""
    from oracle.rays import get_rays
    from neurecon_amd.ray_casting import root_finding_surface_points, surface_render
    sd = wg.neus_state(seed=1)
    H, W, f, dist = 48, 64, 40.0, 2.0
    ro, rd, _ = get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    ro, rd = ro.cuda(), rd.cuda()
    rdn = torch.nn.functional.normalize(rd, dim=-1)
    m = neus_model(sd, precision=precision)
    with torch.no_grad():
        for kw in (dict(), dict(N_steps=100, N_secant_steps=4), dict(N_steps=20), dict(near=0.5, far=4.0)):
            outs = [root_finding_surface_points(m.implicit_surface, ro, rdn, _full_march=full, **kw)
                    for full in (True, False)]
            for name, a, b in zip(('d_pred', 'pts', 'mask', 'mask_sign_change'), *outs):
                assert torch.equal(a, b), (kw, name)
            print(f'[{precision}] {kw}: {int(outs[0][2].sum())} / {outs[0][2].numel()} hits, bit-identical')
        maps = [surface_render(ro, rd, m, calc_normal=True, batched=True, ray_casting_algo='root_finding',
                               ray_casting_cfgs={'_full_march': full}) for full in (True, False)]
    (c0, d0, e0), (c1, d1, e1) = maps
    assert torch.equal(c0, c1) and torch.equal(d0, d1)
    for k in e0:
        if torch.is_tensor(e0[k]):
            assert torch.equal(e0[k], e1[k]), k
