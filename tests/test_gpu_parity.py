"""GPU parity: HIP path (libnrhip.so via neurecon_amd) vs the reference's golden vectors and the
oracle.  Run on the MI355X box: `pytest -m gpu`.

Tolerance (north star): |gpu - ref| <= 1e-4 * |ref| + 1e-6 for rendered rgb / depth / mask /
normals (fp32).  Per-sample quantities behind a discrete decision (sample_pdf's `denom < eps`
switch, searchsorted ties) can legitimately move a sample when the SDF differs by rounding; those
are reported as per-ray pass rates, with rgb/depth held to the bar per ray.
"""
import numpy as np
import pytest
import torch

import weightgen as wg
from helpers import neus_model, report, to_gpu

pytestmark = pytest.mark.gpu

RT, AT = 1e-4, 1e-6
# gradient vectors are O(1): components near zero are held to 1e-5 absolute (1e-5 of the norm)
NAB_AT = 1e-5


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from neurecon_amd import _lib
    _lib.lib()  # must load: no fallback exists


def test_sdf_net_vs_golden(golden):
    g = golden('sdf_net')
    m = neus_model(wg.neus_state(seed=int(g['seed'])))
    pts = to_gpu(g['pts'])
    with torch.no_grad():
        s, h = m.implicit_surface.forward(pts, return_h=True)
        s2, n, h2 = m.implicit_surface.forward_with_nablas(pts)
    assert report('sdf (no grad)', s, g['sdf_nograd'], 1e-5, 1e-6)[0].all()
    assert report('h (no grad)', h[:64], g['h_nograd'], 1e-5, 1e-6)[0].all()
    assert report('sdf (with nablas)', s2, g['sdf'], 1e-5, 1e-6)[0].all()
    assert report('nablas', n, g['nablas'], RT, NAB_AT)[0].all()
    assert report('h (with nablas)', h2[:64], g['h'], 1e-5, 1e-6)[0].all()


def test_sdf_net_ragged_sizes():
    """P not a multiple of the 128-point workgroup tile, and P = 1, match the oracle."""
    from oracle.nets import SDFNet
    sd = wg.neus_state(seed=11)
    m = neus_model(sd)
    orc = SDFNet(sd)
    torch.manual_seed(0)
    for P in (1, 17, 129, 1000):
        x = torch.randn(P, 3) * 0.7
        ref_s, ref_n, ref_h = orc.forward_with_nablas(x)
        with torch.no_grad():
            s, n, h = m.implicit_surface.forward_with_nablas(x.cuda())
        assert report(f'sdf P={P}', s, ref_s, 1e-5, 1e-6)[0].all()
        assert report(f'nabla P={P}', n, ref_n, RT, NAB_AT)[0].all()
        assert report(f'h P={P}', h, ref_h, 1e-5, 1e-6)[0].all()


def test_sdf_forward_narrow_tiles_bit_identical():
    """launch_sdf runs forward-only launches of at most 64 points per CU on 64-point tiles (sdf4_kernel
    STAGE 3: 4 waves, one per SIMD) and larger ones on 128-point tiles: the same per-point code, so every
    point's sdf is bit-identical between the two (ragged sizes, the size limit itself, an offset slice),
    and the narrow launches meet the oracle bar"""
    from oracle.nets import SDFNet
    sd = wg.neus_state(seed=11)
    m = neus_model(sd)
    orc = SDFNet(sd)
    torch.manual_seed(1)
    lim = 64 * torch.cuda.get_device_properties(0).multi_processor_count
    x = torch.randn(lim + 4096, 3) * 0.7
    xg = x.cuda()
    with torch.no_grad():
        wide = m.implicit_surface.forward(xg)  # more than 64 points per CU: 128-point tiles
        for p0, n in ((0, 1), (5, 17), (100, 129), (1000, 1000), (0, lim), (lim - 4096, 4096)):
            narrow = m.implicit_surface.forward(xg[p0:p0 + n].contiguous())
            assert torch.equal(narrow, wide[p0:p0 + n]), (p0, n, float((narrow - wide[p0:p0 + n]).abs().max()))
        s = m.implicit_surface.forward(xg[:2000].contiguous())
    assert report('sdf narrow tiles P=2000', s, orc.sdf(x[:2000]), 1e-5, 1e-6)[0].all()


def test_radiance_vs_golden(golden):
    g = golden('radiance')
    m = neus_model(wg.neus_state(seed=int(g['seed_neus'])))
    with torch.no_grad():
        rgb = m.radiance_net.forward(to_gpu(g['x']), to_gpu(g['v']), to_gpu(g['n']), to_gpu(g['f']))
    assert report('radiance (NeuS cfg)', rgb, g['rgb_neus'], 1e-5, 1e-6)[0].all()


def test_sample_pdf_vs_golden(golden):
    from neurecon_amd import rend_util
    g = golden('sampling')
    s16 = rend_util.sample_pdf(to_gpu(g['bins']), to_gpu(g['weights']), 16, det=True)
    s66 = rend_util.sample_pdf(to_gpu(g['bins']), to_gpu(g['weights']), 66, det=True)
    assert report('sample_pdf N=16', s16, g['s16'], 1e-6, 1e-6)[0].all()
    assert report('sample_pdf N=66', s66, g['s66'], 1e-6, 1e-6)[0].all()


def test_get_rays_vs_golden(golden):
    from neurecon_amd import rend_util
    g = golden('get_rays')
    H, W = int(g['H']), int(g['W'])
    ro, rd, _ = rend_util.get_rays(to_gpu(g['c2w']), to_gpu(g['K']), H, W)
    assert report('rays_o', ro, g['rays_o'], 0, 0)[0].all()
    assert report('rays_d', rd, g['rays_d'], 1e-6, 1e-7)[0].all()


def _neus_render(m, ro, rd, **kw):
    from neurecon_amd.frameworks.neus import volume_render
    with torch.no_grad():
        return volume_render(ro, rd, m, obj_bounding_radius=1.0, batched=True, calc_normal=True,
                             detailed_output=True, perturb=False, N_samples=64, N_importance=64,
                             upsample_algo='official_solution', N_upsample_iters=4, **kw)


def _bench_render(m, ro, rd):
    """the call bench.py times: detailed_output=False, which turns the zero-alpha mid-point skip on"""
    from neurecon_amd.frameworks.neus import volume_render
    with torch.no_grad():
        return volume_render(ro, rd, m, obj_bounding_radius=1.0, batched=True, calc_normal=True,
                             detailed_output=False, perturb=False, N_samples=64, N_importance=64,
                             upsample_algo='official_solution', N_upsample_iters=4)


def _assert_bench_call_equal(detailed, bench, tag):
    """rgb / depth / mask / normals of the benchmarked call are the detailed render's, bit for bit"""
    rgb, depth, ex = detailed
    rgb_b, depth_b, ex_b = bench
    for name, a, b in [('rgb', rgb_b, rgb), ('depth', depth_b, depth), ('mask', ex_b['mask_volume'], ex['mask_volume']),
                       ('normals', ex_b['normals_volume'], ex['normals_volume'])]:
        assert torch.equal(a, b), (tag, name, float((a - b).abs().max()))
    print(f'{tag}: benchmarked call (detailed_output=False, zero-alpha skip) bit-identical to the detailed render')


def test_neus_render_vs_golden(golden):
    """64 rays of config (b) vs the reference.  rgb/depth/mask must meet the bar on every ray.
    Per-sample values are compared on the rays whose samples did not move: the upsampling's
    `denom < 1e-5` switch (rend_util.py:288) sits exactly at the flat-pdf step 1e-5/sum(w) of an
    opaque ray, so rounding-level SDF differences can move a sample there (no continuous bound)."""
    g = golden('neus_b')
    m = neus_model(wg.neus_state(seed=int(g['seed'])))
    rgb, depth, ex = _neus_render(m, to_gpu(g['rays_o']), to_gpu(g['rays_d']))
    ok_d, _ = report('d_final', ex['d_final'], g['d_final'], 1e-5, 1e-6)
    same = ok_d.reshape(ok_d.shape[-2], -1).all(-1)
    print(f'rays with identical samples: {same.sum()} / {same.size}')
    # the reference's own sensitivity on these 64 rays (tools/sdf_noise_sensitivity.py --golden neus_b,
    # 5 noise seeds, profiles/r04/sdf_noise_sensitivity.txt): with absolute SDF noise at the fp32 path's
    # mean |SDF error| vs float64 (1.2e-7; 1e-7 used) the oracle keeps identical samples on
    # 67-72 % of them; observed here: 0.70 (r02)
    assert same.mean() >= 0.65
    # per-sample values: rays whose depths agree to 1e-6 relative (d <= 3 -> |dd| <= 3e-6); the
    # sampled field moves by |grad| * |dd| <= ~5e-6 there, so sdf / radiance / weights get atol 1e-5
    dd = np.abs(ex['d_final'].cpu().numpy() - g['d_final'])
    tight = (dd <= 1e-6 * np.abs(g['d_final'])).all(-1).reshape(-1)
    print(f'rays with depths within 1e-6: {tight.sum()} / {tight.size}')
    # observed 28 / 64 (r03): the depths of an upsampled sample move by ulps wherever its sample_pdf
    # interval's cdf difference rounds differently; the oracle itself under 1e-7 absolute SDF noise keeps
    # all depths within 1e-6 on 44-50 % of these rays (same tool and table)
    assert tight.mean() >= 0.4
    sel = lambda t: (t.cpu().numpy() if isinstance(t, torch.Tensor) else t)[0][tight]
    assert report('sdf (same-sample rays)', sel(ex['implicit_surface']), sel(g['sdf']), RT, 1e-5)[0].all()
    assert report('nablas (same-sample rays)', sel(ex['implicit_nablas']), sel(g['nablas']), RT, 1e-4)[0].all()
    assert report('radiance (same-sample rays)', sel(ex['radiance']), sel(g['radiance']), RT, 1e-5)[0].all()
    assert report('weights (same-sample rays)', sel(ex['visibility_weights']), sel(g['weights']), RT, 1e-5)[0].all()
    assert report('rgb', rgb, g['rgb'], RT, AT)[0].all()
    assert report('depth', depth, g['depth'], RT, AT)[0].all()
    assert report('mask', ex['mask_volume'], g['mask'], RT, AT)[0].all()
    # normals_volume is a weighted sum of unit vectors: held to 1e-4 of unit length
    assert report('normals', ex['normals_volume'], g['normals'], RT, 1e-4)[0].all()


def test_neus_full_config_b_vs_oracle():
    """4096 rays (the BASELINE config) vs the oracle; per-ray pass rate at the 1e-4 bar."""
    from oracle.neus import NeuSOracle
    from oracle import rays as orays
    H, W, f, dist = wg.CAMERAS['b']
    c2w = wg.look_at_c2w(dist)[None]
    K = wg.intrinsics(f, H, W)[None]
    ro, rd, _ = orays.get_rays(c2w, K, H, W)
    sd = wg.neus_state(seed=1)
    torch.set_num_threads(8)
    with torch.no_grad():
        ref = NeuSOracle(sd).render(ro, rd)
    m = neus_model(sd)
    rgb, depth, ex = _neus_render(m, ro.cuda(), rd.cuda())
    _assert_bench_call_equal((rgb, depth, ex), _bench_render(m, ro.cuda(), rd.cuda()), 'fp32 config (b)')
    ok_rgb, _ = report('rgb', rgb, ref['rgb'], RT, AT)
    ok_dep, _ = report('depth', depth, ref['depth_volume'], RT, AT)
    ok_n, _ = report('normals', ex['normals_volume'], ref['normals_volume'], RT, 1e-4)
    ray_ok = ok_rgb.all(-1) & ok_dep
    d_same = (np.abs(ex['d_final'].cpu().numpy() - ref['d_final'].numpy()) <= 1e-5).all(-1)
    print(f'per-ray rgb+depth pass: {ray_ok.mean() * 100:.3f}%  rays with identical samples: '
          f'{d_same.mean() * 100:.3f}%  failing rays with identical samples: {(~ray_ok & d_same).sum()}')
    # a ray may only miss the bar if a discrete sampling decision flipped on it
    assert (~ray_ok & d_same).sum() == 0
    assert ray_ok.mean() >= 0.995


# ---------------------------------------------------------------------------------------------
# split-fp16 x3 mode (NR_PREC_F16X3, the benchmarked default): held to the SAME bars as fp32
# ---------------------------------------------------------------------------------------------
def test_f16x3_sdf_net_vs_golden(golden):
    g = golden('sdf_net')
    m = neus_model(wg.neus_state(seed=int(g['seed'])), precision='f16x3')
    pts = to_gpu(g['pts'])
    with torch.no_grad():
        s, h = m.implicit_surface.forward(pts, return_h=True)
        s2, n, h2 = m.implicit_surface.forward_with_nablas(pts)
    assert report('f16x3 sdf', s, g['sdf_nograd'], 1e-5, 1e-6)[0].all()
    assert report('f16x3 h', h[:64], g['h_nograd'], 1e-5, 1e-6)[0].all()
    assert report('f16x3 sdf (with nablas)', s2, g['sdf'], 1e-5, 1e-6)[0].all()
    assert report('f16x3 nablas', n, g['nablas'], RT, NAB_AT)[0].all()
    assert report('f16x3 h (with nablas)', h2[:64], g['h'], 1e-5, 1e-6)[0].all()


def test_f16x3_radiance_vs_golden(golden):
    g = golden('radiance')
    m = neus_model(wg.neus_state(seed=int(g['seed_neus'])), precision='f16x3')
    with torch.no_grad():
        rgb = m.radiance_net.forward(to_gpu(g['x']), to_gpu(g['v']), to_gpu(g['n']), to_gpu(g['f']))
    assert report('f16x3 radiance', rgb, g['rgb_neus'], 1e-5, 1e-6)[0].all()


def test_f16x3_neus_full_config_b_vs_oracle():
    from oracle.neus import NeuSOracle
    from oracle import rays as orays
    H, W, f, dist = wg.CAMERAS['b']
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    sd = wg.neus_state(seed=1)
    torch.set_num_threads(8)
    with torch.no_grad():
        ref = NeuSOracle(sd).render(ro, rd)
    m = neus_model(sd, precision='f16x3')
    rgb, depth, ex = _neus_render(m, ro.cuda(), rd.cuda())
    # the benchmarked call (bench.py) is the detailed render bit for bit, so the oracle check below
    # holds it too
    _assert_bench_call_equal((rgb, depth, ex), _bench_render(m, ro.cuda(), rd.cuda()), 'f16x3 config (b)')
    ok_rgb, _ = report('f16x3 rgb', rgb, ref['rgb'], RT, AT)
    ok_dep, _ = report('f16x3 depth', depth, ref['depth_volume'], RT, AT)
    ok_m, _ = report('f16x3 mask', ex['mask_volume'], ref['mask_volume'], RT, AT)
    ok_n, _ = report('f16x3 normals', ex['normals_volume'], ref['normals_volume'], RT, 1e-4)
    ray_ok = ok_rgb.all(-1) & ok_dep & ok_m
    d_same = (np.abs(ex['d_final'].cpu().numpy() - ref['d_final'].numpy()) <= 1e-5).all(-1)
    print(f'f16x3 per-ray rgb+depth+mask pass: {ray_ok.mean() * 100:.3f}%  identical samples: '
          f'{d_same.mean() * 100:.3f}%  failing rays with identical samples: {(~ray_ok & d_same).sum()}  '
          f'normals off with identical samples: {(~ok_n.all(-1) & d_same).sum()}')
    # the same invariant as fp32: only a flipped sampling decision may take a ray off the bar
    assert (~ray_ok & d_same).sum() == 0
    assert (~ok_n.all(-1) & d_same).sum() == 0
    assert ray_ok.mean() >= 0.995


@pytest.mark.parametrize('algo', ['direct_use', 'direct_more'])
def test_neus_direct_upsampling_vs_golden(golden, algo):
    """upsample_algo 'direct_use' / 'direct_more' (N_nograd_samples=512), 12 rays of config (b)."""
    g = golden('neus_algos')
    m = neus_model(wg.neus_state(seed=int(g['seed'])))
    from neurecon_amd.frameworks.neus import volume_render
    with torch.no_grad():
        rgb, depth, ex = volume_render(to_gpu(g['rays_o']), to_gpu(g['rays_d']), m, obj_bounding_radius=1.0,
                                       batched=True, calc_normal=True, detailed_output=True, perturb=False,
                                       N_samples=64, N_importance=64, upsample_algo=algo,
                                       N_nograd_samples=int(g['N_nograd_samples']))
    ok_d, _ = report(f'{algo} d_final', ex['d_final'], g[algo + '_d_final'], 1e-5, 1e-6)
    same = ok_d.reshape(ok_d.shape[-2], -1).all(-1)
    print(f'{algo}: rays with identical samples {same.sum()} / {same.size}')
    ok_rgb, _ = report(f'{algo} rgb', rgb, g[algo + '_rgb'], RT, AT)
    ok_dep, _ = report(f'{algo} depth', depth, g[algo + '_depth'], RT, AT)
    ray_ok = (ok_rgb.all(-1) & ok_dep).reshape(-1)
    assert ray_ok[same].all()
    assert same.mean() >= 0.5 and ray_ok.mean() >= 0.9


@pytest.mark.parametrize('gain', [1.0, 1.6])
def test_f16x3_sdf_net_ragged_and_scaled(gain):
    """f16x3 operand scales come from per-layer bounds (nr_mlp.hip, v3 pipeline): ragged sizes,
    far / near-origin points and weights scaled up (activations growing layer to layer) must stay
    within the f16x3 bar against the oracle -- no overflow, no lost precision."""
    from oracle.nets import SDFNet
    sd = wg.neus_state(seed=5)
    sd = {k: (v * gain if k.endswith('weight_g') else v) for k, v in sd.items()}
    m = neus_model(sd, precision='f16x3')
    orc = SDFNet(sd)
    torch.manual_seed(1)
    for P in (1, 17, 129, 1000, 5000):
        x = torch.randn(P, 3) * 0.7
        x[: P // 3] *= 4.0    # far points (large embedding arguments, large activations)
        x[-(P // 3):] *= 1e-3  # near the origin
        ref_s, ref_n, ref_h = orc.forward_with_nablas(x)
        with torch.no_grad():
            s, n, h = m.implicit_surface.forward_with_nablas(x.cuda())
            s0 = m.implicit_surface.forward(x.cuda())
        scale = float(ref_s.abs().max())
        assert report(f'f16x3 sdf P={P} gain={gain}', s, ref_s, 1e-5, 1e-6 * scale)[0].all()
        assert report(f'f16x3 sdf(no grad) P={P}', s0, ref_s, 1e-5, 1e-6 * scale)[0].all()
        # the fp32 bar, with components near zero held to 1e-5 of the largest gradient
        assert report(f'f16x3 nabla P={P}', n, ref_n, RT, NAB_AT * float(ref_n.abs().max()))[0].all()
        assert report(f'f16x3 h P={P}', h, ref_h, 1e-5, 1e-6 * float(ref_h.abs().max()))[0].all()


@pytest.mark.parametrize('framework', ['neus', 'volsdf'])
def test_multi_chunk_render_is_chunk_invariant(framework):
    """n_rays above the library's internal chunk (16384 rays) runs several chunks through the same
    workspace (NeuS: ping-pong merge buffers, evaluation slots; VolSDF: sampler lists): the result
    must be bit-identical to rendering the same rays in separate calls."""
    from helpers import volsdf_model
    from neurecon_amd.frameworks import neus, volsdf
    H, W, f, dist = wg.CAMERAS['d']
    from neurecon_amd import rend_util
    ro, rd, _ = rend_util.get_rays(wg.look_at_c2w(dist)[None].cuda(), wg.intrinsics(f, H, W)[None].cuda(), H, W)
    n = 16384 + 3000
    ro, rd = ro[:, 200000:200000 + n].contiguous(), rd[:, 200000:200000 + n].contiguous()
    if framework == 'neus':
        m = neus_model(wg.neus_state(seed=1), precision='f16x3')
        fn = lambda o, d: neus.volume_render(o, d, m, batched=True, calc_normal=True, detailed_output=False,
                                             N_samples=64, N_importance=64)
    else:
        m = volsdf_model(wg.volsdf_state(seed=2, beta_init=0.1), 0.1, precision='f16x3')
        fn = lambda o, d: volsdf.volume_render(o, d, m, batched=True, calc_normal=True, detailed_output=False,
                                               N_samples=64, N_importance=64, max_upsample_steps=6)
    with torch.no_grad():
        rgb, depth, ex = fn(ro, rd)
        parts = [fn(ro[:, a:b].contiguous(), rd[:, a:b].contiguous()) for a, b in [(0, 5000), (5000, n)]]
    assert torch.equal(rgb, torch.cat([p[0] for p in parts], 1))
    assert torch.equal(depth, torch.cat([p[1] for p in parts], 1))
    assert torch.equal(ex['normals_volume'], torch.cat([p[2]['normals_volume'] for p in parts], 1))


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
@pytest.mark.parametrize('perturb', [False, True])
def test_neus_zero_alpha_skip_bit_identical(precision, perturb):
    """The benchmarked render (detailed_output=False) sends only the mid-points whose alpha is not exactly
    0 through the SDF + radiance nets (neus_mid_compact): rgb / depth / mask / normals must equal the
    full evaluation bit for bit on the whole config-(b) workload (4096 rays; perturb=True replays the
    same uniforms in both renders)."""
    from oracle import rays as orays
    from neurecon_amd.frameworks.neus import volume_render
    H, W, f, dist = wg.CAMERAS['b']
    c2w = wg.look_at_c2w(dist)[None]
    K = wg.intrinsics(f, H, W)[None]
    ro, rd, _ = orays.get_rays(c2w, K, H, W)
    m = neus_model(wg.neus_state(seed=1), precision=precision)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, perturb=perturb,
              N_samples=64, N_importance=64, N_upsample_iters=4)
    outs = []
    for skip in (True, False):
        torch.manual_seed(7)
        with torch.no_grad():
            rgb, depth, ex = volume_render(ro.cuda(), rd.cuda(), m, skip_zero_alpha=skip, **kw)
        outs.append((rgb, depth, ex['mask_volume'], ex['normals_volume']))
    torch.cuda.synchronize()
    for name, a, b in zip(('rgb', 'depth', 'mask', 'normals'), outs[0], outs[1]):
        assert torch.equal(a, b), (name, float((a - b).abs().max()))
    print(f'{precision} perturb={perturb}: zero-alpha skip bit-identical on 4096 rays')


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
@pytest.mark.parametrize('algo,N_outside', [('direct_use', 0), ('direct_more', 0), ('official_solution', 32),
                                            ('direct_use', 32)])
def test_neus_zero_alpha_skip_algos_bit_identical(precision, algo, N_outside):
    """The mid-point skip behind the other upsamplers (neus.py:215-243) and the NeRF++ background
    (mid-points outside the bounding sphere also skip the surface nets): maps bit-identical to the
    render that evaluates every mid-point, on 1024 config-(b) rays."""
    from oracle import rays as orays
    from neurecon_amd.frameworks.neus import volume_render
    H, W, f, dist = wg.CAMERAS['b']
    c2w = wg.look_at_c2w(dist)[None]
    K = wg.intrinsics(f, H, W)[None]
    ro, rd, _ = orays.get_rays(c2w, K, H, W)
    ro, rd = ro[:, ::4].contiguous(), rd[:, ::4].contiguous()
    nerf = N_outside > 0
    m = neus_model(wg.neus_state(seed=1, use_outside_nerf=nerf), use_outside_nerf=nerf, precision=precision)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, perturb=False,
              N_samples=64, N_importance=64, N_upsample_iters=4, upsample_algo=algo, N_outside=N_outside)
    outs = []
    for skip in (True, False):
        with torch.no_grad():
            rgb, depth, ex = volume_render(ro.cuda(), rd.cuda(), m, skip_zero_alpha=skip, **kw)
        outs.append((rgb, depth, ex['mask_volume'], ex['normals_volume']))
    torch.cuda.synchronize()
    for name, a, b in zip(('rgb', 'depth', 'mask', 'normals'), outs[0], outs[1]):
        assert torch.equal(a, b), (name, float((a - b).abs().max()))
    print(f'{precision} {algo} N_outside={N_outside}: zero-alpha skip bit-identical on {rgb.shape[1]} rays')


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_ray_counts_not_multiple_of_four(precision):
    """neus_composite packs four rays per wave (16 lanes each); a block's tail lanes are dead when
    n_rays % 4 != 0.  Ray counts = 1, 2, 3 (mod 4) in one call and as separate calls: bit-identical
    maps (and the benchmarked call's skip path identical to the detailed render)."""
    from oracle import rays as orays
    H, W, f, dist = wg.CAMERAS['b']
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    ro, rd = ro[:, 1500:1500 + 1027].contiguous().cuda(), rd[:, 1500:1500 + 1027].contiguous().cuda()  # 1027 = 3 mod 4
    m = neus_model(wg.neus_state(seed=1), precision=precision)
    whole = _bench_render(m, ro, rd)
    _assert_bench_call_equal(_neus_render(m, ro, rd), whole, f'{precision} 1027 rays')
    cuts = [(0, 513), (513, 1027)]                       # 513 = 1 mod 4, 514 = 2 mod 4
    parts = [_bench_render(m, ro[:, a:b].contiguous(), rd[:, a:b].contiguous()) for a, b in cuts]
    single = [_bench_render(m, ro[:, a:a + 1].contiguous(), rd[:, a:a + 1].contiguous()) for a in (0, 700, 1026)]
    torch.cuda.synchronize()
    for name, k in [('rgb', 0), ('depth', 1)]:
        assert torch.equal(whole[k], torch.cat([p[k] for p in parts], 1)), name
        for a, p in zip((0, 700, 1026), single):
            assert torch.equal(whole[k][:, a:a + 1], p[k]), (name, a)
    for name in ('mask_volume', 'normals_volume'):
        assert torch.equal(whole[2][name], torch.cat([p[2][name] for p in parts], 1)), name
    print(f'{precision}: 1027 / 513 / 514 / 1-ray renders bit-identical')


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_many_samples_composite_fallback_vs_oracle(precision):
    """N_samples + N_importance > 455 samples per ray: the compositing runs its one-ray-per-wave variant
    (the four-rays-per-wave kernel keeps 4 x S mid-point depths in LDS).  64 config-(b) rays with
    448 + 64 samples vs the oracle, with the 'only a flipped sampling decision' invariant."""
    from oracle.neus import NeuSOracle
    from oracle import rays as orays
    from neurecon_amd.frameworks.neus import volume_render
    H, W, f, dist = wg.CAMERAS['b']
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    ro, rd = ro[:, 1000:3000:32].contiguous(), rd[:, 1000:3000:32].contiguous()
    sd = wg.neus_state(seed=1)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        ref = NeuSOracle(sd).render(ro, rd, N_samples=448, N_importance=64)
    m = neus_model(sd, precision=precision)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, perturb=False, N_samples=448, N_importance=64,
              upsample_algo='official_solution', N_upsample_iters=4)
    with torch.no_grad():
        det = volume_render(ro.cuda(), rd.cuda(), m, detailed_output=True, **kw)
        bench = volume_render(ro.cuda(), rd.cuda(), m, detailed_output=False, **kw)
    _assert_bench_call_equal(det, bench, f'{precision} S=512')
    rgb, depth, ex = det
    assert ex['d_final'].shape[-1] == 511
    ok_rgb, _ = report(f'{precision} S=512 rgb', rgb, ref['rgb'], RT, AT)
    ok_dep, _ = report(f'{precision} S=512 depth', depth, ref['depth_volume'], RT, AT)
    ok_n, _ = report(f'{precision} S=512 normals', ex['normals_volume'], ref['normals_volume'], RT, 1e-4)
    ray_ok = (ok_rgb.all(-1) & ok_dep).reshape(-1)
    d_same = (np.abs(ex['d_final'].cpu().numpy() - ref['d_final'].numpy()) <= 1e-5).all(-1).reshape(-1)
    print(f'{precision} S=512: per-ray pass {ray_ok.mean() * 100:.1f}%, identical samples {d_same.mean() * 100:.1f}%')
    assert (~ray_ok & d_same).sum() == 0
    assert (~ok_n.all(-1).reshape(-1) & d_same).sum() == 0
    assert d_same.mean() >= 0.5


@pytest.mark.parametrize('perturb', [False, True])
@pytest.mark.parametrize('calc_normal', [True, False])
@pytest.mark.parametrize('N_outside', [0, 32])
def test_neus_deferred_sample_nablas_bit_identical(perturb, calc_normal, N_outside):
    """The benchmarked f16x3 render defers the samples' reverse pass (defer_sample_nablas): sample
    launches keep per-tile slabs, and only 16-sample tiles holding a sample of non-zero alpha get
    nablas (the others are weighted by exactly 0 in normals_volume, neus.py:364-368).  With NeRF++
    (N_outside 32) a sample's weight uses the background's alpha outside the bounding sphere, and the
    last sample's the first inverted-sphere sample's, so the tiles are flagged after the background net.
    Maps must equal the render that computes every sample's nabla when drawn, bit for bit (4096 rays of
    config (b), or of the config-(d) camera fanned out so that some leave the sphere, plus an 8192-ray
    call that runs two chunks)."""
    from oracle import rays as orays
    from neurecon_amd.frameworks.neus import volume_render
    H, W, f, dist = wg.CAMERAS['b']
    if N_outside:
        dist = wg.CAMERAS['d'][3]
        f = 80.0  # a wide view: rays that miss the bounding sphere, and rays past its rim
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    sd = wg.neus_state(seed=1, use_outside_nerf=bool(N_outside))
    m = neus_model(sd, precision='f16x3', use_outside_nerf=bool(N_outside))
    for rays in (4096, 8192):
        o = ro.repeat(1, rays // 4096, 1).cuda()
        d = (rd.repeat(1, rays // 4096, 1) * torch.linspace(0.9, 1.1, rays)[None, :, None]).cuda()
        kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=calc_normal, detailed_output=False,
                  perturb=perturb, N_samples=64, N_importance=64, N_upsample_iters=4, N_outside=N_outside)
        outs = []
        for defer in (True, False):
            torch.manual_seed(3)
            with torch.no_grad():
                rgb, depth, ex = volume_render(o, d, m, defer_sample_nablas=defer, **kw)
            outs.append([rgb, depth, ex['mask_volume']] + ([ex['normals_volume']] if calc_normal else []))
        torch.cuda.synchronize()
        for name, a, b in zip(('rgb', 'depth', 'mask', 'normals'), outs[0], outs[1]):
            assert torch.equal(a, b), (rays, name, float((a - b).abs().max()))
    print(f'deferred sample nablas: bit-identical (perturb={perturb}, calc_normal={calc_normal}, N_outside={N_outside})')


@pytest.mark.parametrize('N_outside', [0, 32])
def test_neus_workspace_bound_by_rayschunk(N_outside):
    """The caller's rayschunk (neus.py:384-397: 256 for validation renders, 4096 in
    tools/render_view.py:529) is a hint floored at NR_MIN_CHUNK_RAYS (4096: a 256-ray chunk leaves the
    per-ray kernels a few CUs); the memory bound is the workspace budget, 4 GiB by default
    (NR_DEFAULT_WORKSPACE_BYTES): renders with rayschunk=256, the default, a 0.5 GiB and a 16 GiB budget
    are bit-identical, and the peak device memory of each is reported.  With an
    explicit budget set, rayschunk is honoured exactly (256-ray chunks), bit-identical too."""
    from oracle import rays as orays
    from neurecon_amd.frameworks.neus import volume_render
    from neurecon_amd import _lib
    H, W, f, dist = wg.CAMERAS['b']
    if N_outside:
        dist, f = wg.CAMERAS['d'][3], 80.0
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    sd = wg.neus_state(seed=1, use_outside_nerf=bool(N_outside))
    m = neus_model(sd, precision='f16x3', use_outside_nerf=bool(N_outside))
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=False, perturb=False,
              N_samples=64, N_importance=64, N_upsample_iters=4, N_outside=N_outside)
    o, d = ro.cuda(), rd.cuda()
    outs = []
    for name, extra in (('rayschunk=256', dict(rayschunk=256)), ('default (4 GiB)', {}),
                        ('0.5 GiB budget', dict(max_workspace_gb=0.5)), ('16 GiB budget', dict(max_workspace_gb=16)),
                        ('rayschunk=256 exact (4 GiB budget set)', dict(rayschunk=256, max_workspace_gb=4))):
        _lib._WS.clear()
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        torch.cuda.reset_peak_memory_stats()
        base = torch.cuda.memory_allocated()
        with torch.no_grad():
            rgb, depth, ex = volume_render(o, d, m, **kw, **extra)
        torch.cuda.synchronize()
        peak = (torch.cuda.max_memory_allocated() - base) / 2**30
        print(f'N_outside={N_outside} 4096-ray render, {name}: peak device memory {peak:.3f} GiB')
        if name.startswith('default') or name.startswith('rayschunk'):
            assert peak <= 4.25, peak
        if name.startswith('0.5'):
            assert peak <= 0.75, peak
        if 'exact' in name:  # 256-ray chunks: ~a sixteenth of the 4096-ray chunk's workspace
            assert peak <= 1.0, peak
        outs.append([rgb, depth, ex['mask_volume'], ex['normals_volume']])
    _lib._WS.clear()
    for other in outs[1:]:
        for nm, a, b in zip(('rgb', 'depth', 'mask', 'normals'), outs[0], other):
            assert torch.equal(a, b), (nm, float((a - b).abs().max()))
