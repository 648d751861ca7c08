"""GPU parity of the NeRF++ background (A8 NeRF MLP kernel, A13 NeuS outside sampling / merge)
vs the reference's golden vectors.  Tolerance: 1e-4 relative + 1e-6 (north star) on rgb / depth /
mask, 1e-4 absolute on normals; per-sample values on rays whose upsampled depths are unchanged."""
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


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_nerf_mlp_vs_golden(golden, precision):
    from neurecon_amd.base import NeRF
    g = golden('nerf')
    sd = wg.neus_state(seed=int(g['seed']), use_outside_nerf=True)
    net = NeRF(input_ch=4, multires=10, multires_view=4, use_view_dirs=True, precision=precision)
    net.load_state_dict({k[len('nerf_outside.'):]: v for k, v in sd.items() if k.startswith('nerf_outside.')})
    net = net.cuda().eval()
    with torch.no_grad():
        sig, rgb = net(to_gpu(g['x4']), to_gpu(g['v']))
    tol = (1e-5, 1e-6) if precision == 'fp32' else (1e-4, 1e-5)
    assert report(f'nerf sigma ({precision})', sig, g['sigma'], *tol)[0].all()
    assert report(f'nerf rgb ({precision})', rgb, g['rgb'], *tol)[0].all()


def test_neus_nerfpp_config_d_vs_golden(golden):
    g = golden('neus_d')
    m = neus_model(wg.neus_state(seed=int(g['seed']), use_outside_nerf=True), use_outside_nerf=True)
    from neurecon_amd.frameworks.neus import volume_render
    with torch.no_grad():
        rgb, depth, ex = volume_render(to_gpu(g['rays_o']), to_gpu(g['rays_d']), m, obj_bounding_radius=1.0,
                                       batched=True, calc_normal=True, detailed_output=True, perturb=False,
                                       N_samples=64, N_importance=64, N_outside=32, N_upsample_iters=4)
    S1 = g['sdf'].shape[-1] - 1  # mid-points; the last N_outside samples are far / t (A13)
    # the inverted-sphere depths do not depend on the upsampling: bit-identical on every ray
    out = lambda t: (t.cpu().numpy() if isinstance(t, torch.Tensor) else t)[..., S1:]
    assert (out(ex['d_final']) == out(g['d_final'])).all()
    report('d_final (mid-points)', ex['d_final'][..., :S1], g['d_final'][..., :S1], 1e-5, 1e-6)
    assert report('sigma_out (outside samples)', out(ex['sigma_out']), out(g['sigma_out']), RT, 1e-5)[0].all()
    assert report('radiance_out (outside samples)', out(ex['radiance_out']), out(g['radiance_out']), RT,
                  AT)[0].all()
    # alpha of sample k >= S1+1 only depends on d_k, d_k+1 and sigma_k (dist of S1 involves a mid-point)
    a1 = lambda t: (t.cpu().numpy() if isinstance(t, torch.Tensor) else t)[..., S1 + 1:]
    assert report('alpha (outside samples)', a1(ex['alpha']), a1(g['alpha']), RT, AT)[0].all()
    # mid-point samples: the NeRF input [x/r, 1/r] is encoded up to 2^9, so an ulp-level depth
    # difference from the upsampling moves sigma by ~1e-5 there -- report only
    report('sigma_out (mid-points)', ex['sigma_out'][..., :S1], g['sigma_out'][..., :S1], RT, 1e-5)
    report('weights', ex['visibility_weights'], g['weights'], RT, AT)
    ok_rgb, _ = report('rgb', rgb, g['rgb'], RT, AT)
    ok_dep, _ = report('depth', depth, g['depth'], RT, AT)
    ok_m, _ = report('mask', ex['mask_volume'], g['mask'], RT, AT)
    report('normals', ex['normals_volume'], g['normals'], RT, 1e-4)
    ray_ok = (ok_rgb.all(-1) & ok_dep & ok_m).reshape(-1)
    # per-ray dump: which rays miss and whether their upsampled (mid-point) depths moved
    dm = np.abs(ex['d_final'].cpu().numpy()[..., :S1] - g['d_final'][..., :S1]).reshape(-1, S1)
    same = (dm <= 1e-5 * np.abs(g['d_final'][..., :S1]).reshape(-1, S1) + 1e-6).all(-1)
    for i in np.nonzero(~ray_ok)[0]:
        k = int(np.argmax(dm[i]))
        print(f'  ray {i}: depth err {abs(float(depth.reshape(-1)[i]) - float(g["depth"].reshape(-1)[i])):.3e}, '
              f'max mid-point depth move {dm[i].max():.3e} at sample {k}, samples identical: {bool(same[i])}')
    print(f'per-ray rgb+depth+mask pass {ray_ok.mean() * 100:.2f}%, rays with identical samples '
          f'{same.mean() * 100:.2f}%')
    # only a flipped sampling decision may take a ray off the bar
    assert (~ray_ok & same).sum() == 0
    assert ray_ok.mean() >= 0.95


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_direct_more_with_nerfpp_vs_oracle(precision):
    """upsample_algo='direct_more' together with N_outside > 0: the 2048 no-grad weights per ray share
    the workspace with the NeRF++ sample arrays -- 32 config-(d) rays vs the oracle."""
    from oracle.neus import NeuSOracle
    from oracle import rays as orays
    H, W, f, dist = wg.CAMERAS['d']
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    idx = torch.linspace(0, H * W - 1, 32).round().long()
    ro, rd = ro[:, idx].contiguous(), rd[:, idx].contiguous()
    sd = wg.neus_state(seed=4, use_outside_nerf=True)
    with torch.no_grad():
        ref = NeuSOracle(sd, use_outside_nerf=True).render(ro, rd, N_outside=32, upsample_algo='direct_more',
                                                           N_nograd_samples=2048)
        m = neus_model(sd, use_outside_nerf=True, precision=precision)
        from neurecon_amd.frameworks.neus import volume_render
        rgb, depth, ex = volume_render(ro.cuda(), rd.cuda(), m, obj_bounding_radius=1.0, batched=True,
                                       calc_normal=True, detailed_output=True, N_samples=64, N_importance=64,
                                       N_outside=32, upsample_algo='direct_more', N_nograd_samples=2048)
    ok_d, _ = report('direct_more+nerf++ d_final', ex['d_final'], ref['d_final'], 1e-5, 1e-6)
    same = ok_d.reshape(-1, ok_d.shape[-1]).all(-1)
    ok_rgb, _ = report('direct_more+nerf++ rgb', rgb, ref['rgb'], RT, AT)
    ok_dep, _ = report('direct_more+nerf++ depth', depth, ref['depth_volume'], RT, AT)
    ray_ok = (ok_rgb.all(-1) & ok_dep).reshape(-1)
    print(f'identical samples {same.mean() * 100:.1f}%, per-ray pass {ray_ok.mean() * 100:.1f}%')
    assert (~ray_ok & same).sum() == 0
    assert same.mean() >= 0.8


@pytest.mark.parametrize('perturb', [False, True])
@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_nerfpp_compact_background_bit_identical(golden, precision, perturb):
    """Without detailed outputs the NeRF++ net runs only on the samples the compositing reads (every
    outside sample, mid-points outside the bounding sphere; neus.py:325-343): rgb / depth / mask /
    normals must be bit-identical to the render that evaluates the background at every sample, on the
    config-(d) rays plus 192 rays fanned out across the frame so that part of them leave the sphere."""
    from neurecon_amd.frameworks.neus import volume_render
    g = golden('neus_d')
    m = neus_model(wg.neus_state(seed=int(g['seed']), use_outside_nerf=True), use_outside_nerf=True,
                   precision=precision)
    ro, rd = to_gpu(g['rays_o']), to_gpu(g['rays_d'])
    gen = torch.Generator().manual_seed(3)
    rd2 = rd[:, :1].repeat(1, 192, 1) + (torch.rand(1, 192, 3, generator=gen) - 0.5).cuda() * 0.8
    ro = torch.cat([ro, ro[:, :1].repeat(1, 192, 1)], 1)
    rd = torch.cat([rd, rd2], 1)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, N_samples=64, N_importance=64,
              N_outside=32, N_upsample_iters=4, perturb=perturb)
    with torch.no_grad():  # perturb: both renders replay the same uniforms (same seed, same draws)
        torch.manual_seed(11)
        rgb_c, dep_c, ex_c = volume_render(ro, rd, m, detailed_output=False, **kw)
        torch.manual_seed(11)
        rgb_f, dep_f, ex_f = volume_render(ro, rd, m, detailed_output=True, **kw)
    torch.cuda.synchronize()
    for name, a, b in [('rgb', rgb_c, rgb_f), ('depth', dep_c, dep_f), ('mask', ex_c['mask_volume'], ex_f['mask_volume']),
                       ('normals', ex_c['normals_volume'], ex_f['normals_volume'])]:
        assert torch.equal(a, b), (name, float((a - b).abs().max()))
    print(f'{precision} perturb={perturb}: compact-background render bit-identical on {rgb_c.shape[1]} rays')


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_nerfpp_config_d_frame_vs_oracle(precision):
    """config (d) (NeuS + NeRF++, N_outside=32, official_solution) on 2048 rays spread evenly over the
    800x600 frame, so that part of them leave the bounding sphere: the benchmarked call
    (detailed_output=False: zero-alpha skip, compact background) equals the detailed render bit for
    bit, and both meet the bar against the oracle on every ray whose samples did not move."""
    from oracle.neus import NeuSOracle
    from oracle import rays as orays
    from neurecon_amd.frameworks.neus import volume_render
    H, W, f, dist = wg.CAMERAS['d']
    ro, rd, _ = orays.get_rays(wg.look_at_c2w(dist)[None], wg.intrinsics(f, H, W)[None], H, W)
    idx = torch.linspace(0, H * W - 1, 2048).round().long()
    ro, rd = ro[:, idx].contiguous(), rd[:, idx].contiguous()
    sd = wg.neus_state(seed=4, use_outside_nerf=True)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    with torch.no_grad():
        ref = NeuSOracle(sd, use_outside_nerf=True).render(ro, rd, N_outside=32)
    m = neus_model(sd, use_outside_nerf=True, precision=precision)
    kw = dict(obj_bounding_radius=1.0, batched=True, calc_normal=True, perturb=False, N_samples=64, N_importance=64,
              N_outside=32, upsample_algo='official_solution', N_upsample_iters=4)
    with torch.no_grad():
        rgb, depth, ex = volume_render(ro.cuda(), rd.cuda(), m, detailed_output=True, **kw)
        rgb_b, depth_b, ex_b = volume_render(ro.cuda(), rd.cuda(), m, detailed_output=False, **kw)
    torch.cuda.synchronize()
    for name, a, b in [('rgb', rgb_b, rgb), ('depth', depth_b, depth), ('mask', ex_b['mask_volume'], ex['mask_volume']),
                       ('normals', ex_b['normals_volume'], ex['normals_volume'])]:
        assert torch.equal(a, b), (name, float((a - b).abs().max()))
    S1 = 127
    ok_rgb, _ = report(f'[d frame {precision}] rgb', rgb, ref['rgb'], RT, AT)
    ok_dep, _ = report(f'[d frame {precision}] depth', depth, ref['depth_volume'], RT, AT)
    ok_m, _ = report(f'[d frame {precision}] mask', ex['mask_volume'], ref['mask_volume'], RT, AT)
    ok_n, _ = report(f'[d frame {precision}] normals', ex['normals_volume'], ref['normals_volume'], RT, 1e-4)
    ray_ok = (ok_rgb.all(-1) & ok_dep & ok_m).reshape(-1)
    dref = ref['d_final'].numpy()[..., :S1]
    dm = np.abs(ex['d_final'].cpu().numpy()[..., :S1] - dref).reshape(-1, S1)
    same = (dm <= 1e-5 * np.abs(dref).reshape(-1, S1) + 1e-6).all(-1)
    r = np.linalg.norm(ro[0].numpy(), axis=-1)   # all rays start at the camera
    dn = rd[0] / rd[0].norm(dim=-1, keepdim=True)
    miss = (((ro[0] * dn).sum(-1) ** 2 - (ro[0] ** 2).sum(-1) + 1.0) < 0).numpy()
    print(f'[d frame {precision}] per-ray pass {ray_ok.mean() * 100:.2f}%, identical samples {same.mean() * 100:.2f}%, '
          f'rays missing the bounding sphere {miss.mean() * 100:.1f}%, camera distance {r[0]:.2f}, '
          f'failing rays with identical samples {(~ray_ok & same).sum()}')
    assert miss.any() and (~miss).any()
    # only a flipped sampling decision may take a ray off the bar
    assert (~ray_ok & same).sum() == 0
    assert (~ok_n.all(-1).reshape(-1) & same).sum() == 0
    # Bar from the reference's own sensitivity (tools/sdf_noise_sensitivity.py, these 2048 rays, 5 noise
    # seeds, profiles/r04/sdf_noise_sensitivity.txt): the oracle's sampler with absolute SDF noise at
    # each mode's measured mean |SDF error| vs float64 (fp32 1.2e-7, f16x3 2.0e-7) keeps
    # identical samples on >= 81.7 % (1e-7) / >= 78.0 % (2e-7) of the rays.  Observed (r03): 83.7 % /
    # 84.5 %, per-ray pass 99.95 % / 99.85 %.
    floor = {'fp32': 0.81, 'f16x3': 0.78}[precision]
    assert same.mean() >= floor and ray_ok.mean() >= 0.995
