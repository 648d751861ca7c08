"""Pin the oracle (CPU restatement) against golden vectors produced by the real reference.

CPU-only.  The oracle runs the same fp32 torch CPU kernels as the reference, so agreement is at
rounding level; tolerances below are written per quantity.
"""
import numpy as np
import pytest
import torch

import weightgen as wg
from oracle import nets, rays
from oracle.neus import NeuSOracle, sdf_to_alpha, alpha_to_w
from oracle.volsdf import VolSDFOracle, error_bound, sdf_to_sigma
from oracle.unisurf import UNISURFOracle

T = lambda a: torch.from_numpy(np.asarray(a))


def close(a, b, rtol=1e-5, atol=1e-6):
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    np.testing.assert_allclose(a, np.asarray(b), rtol=rtol, atol=atol)


def test_embed(golden):
    g = golden('embed')
    close(nets.embed(T(g['x']), 6), g['emb6'], 0, 0)
    close(nets.embed(T(g['x']), 4), g['emb4'], 0, 0)
    close(nets.embed(T(g['x4']), 10), g['emb10_4d'], 0, 0)


def test_sdf_net(golden):
    g = golden('sdf_net')
    net = nets.SDFNet(wg.neus_state(seed=int(g['seed'])))
    s, h = net.forward(T(g['pts']))
    close(s, g['sdf_nograd'], 1e-6, 1e-7)
    close(h[:64], g['h_nograd'], 1e-6, 1e-7)
    s, n, h = net.forward_with_nablas(T(g['pts']))
    close(s, g['sdf'], 1e-6, 1e-7)
    close(n, g['nablas'], 1e-5, 1e-6)


def test_radiance_nets(golden):
    g = golden('radiance')
    rn = nets.RadianceNet(wg.neus_state(seed=int(g['seed_neus'])), multires_view=4)
    rv = nets.RadianceNet(wg.volsdf_state(seed=int(g['seed_volsdf'])), multires_view=-1)
    args = [T(g[k]) for k in ('x', 'v', 'n', 'f')]
    close(rn.forward(*args), g['rgb_neus'], 1e-6, 1e-7)
    close(rv.forward(*args), g['rgb_volsdf'], 1e-6, 1e-7)


def test_nerf(golden):
    g = golden('nerf')
    net = nets.NeRFNet(wg.neus_state(seed=int(g['seed']), use_outside_nerf=True))
    s, c = net.forward(T(g['x4']), T(g['v']))
    close(s, g['sigma'], 1e-6, 1e-6)
    close(c, g['rgb'], 1e-6, 1e-7)


def test_sampling(golden):
    g = golden('sampling')
    bins, w = T(g['bins']), T(g['weights'])
    close(rays.sample_pdf(bins, w, 16, det=True), g['s16'], 0, 0)
    close(rays.sample_pdf(bins, w, 66, det=True), g['s66'], 0, 0)
    close(rays.sample_pdf(bins, w, 16, det=False, u=T(g['u_rand'])), g['s_rand'], 0, 0)
    close(rays.sample_cdf(bins, T(g['cdf_in']), 24, det=True), g['s_cdf'], 0, 0)
    o, d = T(g['o']), T(g['d'])
    n, f = rays.near_far_from_sphere(o, d, 1.0)
    close(n, g['near'], 0, 0); close(f, g['far'], 0, 0)
    n, f = rays.near_far_from_sphere(o, d, 4.0, keepdim=False)
    close(n, g['near4'], 0, 0); close(f, g['far4'], 0, 0)
    n, f, m = rays.sphere_intersection(o, d, 1.0)
    close(n, g['si_near'], 0, 0); close(f, g['si_far'], 0, 0); close(m.numpy().astype(np.uint8), g['si_mask'], 0, 0)
    close(rays.dvals_from_radius(T(g['o_in']), d, T(g['rs']).expand(o.shape[0], -1)), g['dvals'], 0, 0)


def test_get_rays(golden):
    g = golden('get_rays')
    H, W = int(g['H']), int(g['W'])
    ro, rd, _ = rays.get_rays(T(g['c2w']), T(g['K']), H, W)
    close(ro, g['rays_o'], 0, 0)
    close(rd, g['rays_d'], 1e-6, 1e-7)
    ro, rd, _ = rays.get_rays(T(g['c2w']), T(g['K']), H, W, select_inds=T(g['select_inds']))
    close(rd, g['rays_d_sel'], 1e-6, 1e-7)


def test_neus_b(golden):
    g = golden('neus_b')
    orc = NeuSOracle(wg.neus_state(seed=int(g['seed'])))
    with torch.no_grad():
        out = orc.render(T(g['rays_o']), T(g['rays_d']))
    close(out['d_final'], g['d_final'], 1e-6, 1e-6)
    close(out['implicit_surface'], g['sdf'], 1e-5, 1e-6)
    close(out['implicit_nablas'], g['nablas'], 1e-5, 1e-6)
    close(out['radiance'], g['radiance'], 1e-5, 1e-6)
    close(out['visibility_weights'], g['weights'], 1e-5, 1e-6)
    close(out['rgb'], g['rgb'], 1e-5, 1e-6)
    close(out['depth_volume'], g['depth'], 1e-5, 1e-6)
    close(out['mask_volume'], g['mask'], 1e-5, 1e-6)
    close(out['normals_volume'], g['normals'], 1e-5, 1e-6)


def test_neus_upsample_variants(golden):
    g = golden('neus_algos')
    orc = NeuSOracle(wg.neus_state(seed=int(g['seed'])))
    for algo in ['direct_use', 'direct_more']:
        with torch.no_grad():
            out = orc.render(T(g['rays_o']), T(g['rays_d']), upsample_algo=algo,
                             N_nograd_samples=int(g['N_nograd_samples']))
        close(out['d_final'], g[algo + '_d_final'], 1e-6, 1e-6)
        close(out['rgb'], g[algo + '_rgb'], 1e-5, 1e-6)
        close(out['depth_volume'], g[algo + '_depth'], 1e-5, 1e-6)


def test_neus_d_nerfpp(golden):
    g = golden('neus_d')
    orc = NeuSOracle(wg.neus_state(seed=int(g['seed']), use_outside_nerf=True), use_outside_nerf=True)
    with torch.no_grad():
        out = orc.render(T(g['rays_o']), T(g['rays_d']), N_outside=32)
    close(out['d_final'], g['d_final'], 1e-6, 1e-6)
    close(out['sigma_out'], g['sigma_out'], 1e-5, 1e-5)
    close(out['radiance_out'], g['radiance_out'], 1e-5, 1e-6)
    close(out['rgb'], g['rgb'], 1e-5, 1e-6)
    close(out['depth_volume'], g['depth'], 1e-5, 1e-6)
    close(out['normals_volume'], g['normals'], 1e-5, 1e-6)


def test_volsdf_1d(golden):
    g = golden('volsdf_1d')
    x, s, beta, bp = T(g['x']), T(g['sdf']), float(g['beta']), float(g['bplus'])
    close(error_bound(x, s, 1. / beta, beta), g['bounds_net'], 1e-6, 0)
    close(error_bound(x, s, 1. / bp, bp), g['bounds_plus'], 1e-6, 0)
    close(sdf_to_sigma(s, 1. / beta, beta), g['sigma'], 0, 0)


@pytest.mark.parametrize('name,N_samples,N_importance', [('volsdf_a', 64, 64), ('volsdf_c', 128, 128)])
def test_volsdf(golden, name, N_samples, N_importance):
    g = golden(name)
    orc = VolSDFOracle(wg.volsdf_state(seed=int(g['seed']), beta_init=float(g['beta_init'])))
    with torch.no_grad():
        out = orc.render(T(g['rays_o']), T(g['rays_d']), N_samples=N_samples, N_importance=N_importance,
                         max_upsample_steps=6)
    close(out['iter_usage'], g['iter_usage'], 0, 0)
    close(out['beta_map'], g['beta_map'], 1e-6, 0)
    keep = slice(None) if name == 'volsdf_c' else slice(0, 512, 8)
    close(out['d_vals'][:, keep], g['d_vals'], 1e-6, 1e-6)
    close(out['rgb'], g['rgb'], 1e-5, 1e-6)
    close(out['depth_volume'], g['depth'], 1e-5, 1e-6)
    close(out['mask_volume'], g['mask'], 1e-5, 1e-6)
    close(out['normals_volume'], g['normals'], 1e-5, 1e-6)


def test_unisurf(golden):
    g = golden('unisurf_e')
    orc = UNISURFOracle(wg.unisurf_state(seed=int(g['seed'])))
    for tag, nc in [('', 1048576), ('_nc1000', 1000)]:
        with torch.no_grad():
            out = orc.render(T(g['rays_o']), T(g['rays_d']), logit_tau=float(g['logit_tau']), netchunk=nc)
        if tag == '':
            close(out['mask_surface'].numpy().astype(np.uint8), g['mask_surface'], 0, 0)
            close(out['depth_surface'], g['depth_surface'], 1e-6, 1e-6)
            close(out['implicit_surface'], g['sdf'], 1e-5, 1e-6)
            close(out['radiance'], g['radiance'], 1e-5, 1e-6)
        close(out['rgb'], g['rgb' + tag], 1e-5, 1e-6)
        close(out['depth_volume'], g['depth' + tag], 1e-5, 1e-6)
        close(out['normals_volume'], g['normals' + tag], 1e-5, 1e-6)


def test_surface_render_and_grid(golden):
    """oracle/surface.py vs ray_casting.surface_render / sphere tracing / extract_mesh's grid."""
    from oracle import surface
    g = golden('surface')
    orc = NeuSOracle(wg.neus_state(seed=int(g['seed'])))
    with torch.no_grad():
        out = surface.surface_render_neus(orc, T(g['rays_o']), T(g['rays_d']))
        np.testing.assert_array_equal(out['mask'].numpy(), g['mask'].astype(bool))
        close(out['depth'], g['depth'], 1e-6, 1e-6)
        close(out['rgb'], g['rgb'], 1e-5, 1e-6)
        close(out['nablas'], g['nablas'], 1e-5, 1e-6)
        close(out['normals'], g['normals'], 1e-5, 1e-6)
        d = torch.nn.functional.normalize(T(g['rays_d']), dim=-1)
        d5, p5, m5 = surface.sphere_trace(orc.sdf_net.sdf, T(g['rays_o']), d, near=0.5, far=4.0, N_iters=5)
        np.testing.assert_array_equal(m5.numpy(), g['st5_mask'].astype(bool))
        close(d5, g['st5_d'], 1e-6, 1e-6)
        close(p5, g['st5_pts'], 1e-6, 1e-6)
        for N, s in [(16, 2.0), (24, 1.5)]:
            close(surface.sdf_grid(orc.sdf_net.sdf, N, s), g[f'grid{N}'], 1e-6, 1e-7)


def test_volsdf_nerfpp(golden):
    """VolSDF + NeRF++ background (volsdf.py:400-405, 451-469) vs the reference."""
    g = golden('volsdf_nerfpp')
    orc = VolSDFOracle(wg.volsdf_state(seed=int(g['seed']), beta_init=float(g['beta_init']), use_nerfplusplus=True),
                       use_nerfplusplus=True)
    with torch.no_grad():
        out = orc.render(T(g['rays_o']), T(g['rays_d']), N_samples=64, N_importance=64, N_outside=32,
                         max_upsample_steps=6)
    np.testing.assert_array_equal(out['iter_usage'].numpy(), g['iter_usage'])
    close(out['d_vals'], g['d_vals'], 1e-6, 1e-6)
    close(out['sigma_out'], g['sigma_out'], 1e-5, 1e-6)
    close(out['radiance_out'], g['radiance_out'], 1e-5, 1e-6)
    for k, gk in [('rgb', 'rgb'), ('depth_volume', 'depth'), ('mask_volume', 'mask'), ('normals_volume', 'normals')]:
        close(out[k], g[gk], 1e-5, 1e-6)


@pytest.mark.parametrize('key', ['a', 'c', 'pp'])
def test_volsdf_perturb(golden, key):
    """oracle VolSDF perturb=True with the reference's generator state: same draws, same order."""
    g = golden('volsdf_perturb')
    nerfpp = key == 'pp'
    sd = wg.volsdf_state(seed=int(g[key + '_seed']), beta_init=float(g[key + '_beta_init']), use_nerfplusplus=nerfpp)
    orc = VolSDFOracle(sd, use_nerfplusplus=nerfpp)
    torch.manual_seed(200 + int(g[key + '_seed']))
    with torch.no_grad():
        out = orc.render(T(g[key + '_rays_o']), T(g[key + '_rays_d']), N_samples=int(g[key + '_N_samples']),
                         N_importance=int(g[key + '_N_importance']), max_upsample_steps=6, perturb=True)
    close(out['iter_usage'], g[key + '_iter_usage'], 0, 0)
    close(out['d_vals'], g[key + '_d_vals'], 1e-6, 1e-6)
    for k, gk in [('rgb', 'rgb'), ('depth_volume', 'depth'), ('mask_volume', 'mask'), ('normals_volume', 'normals')]:
        close(out[k], g[f'{key}_{gk}'], 1e-5, 1e-6)


def test_siren(golden):
    """SIREN nets (base.py:84-115) and a VolSDF render with them (configs/volsdf_siren.yaml)."""
    g = golden('siren')
    sd = wg.volsdf_siren_state(seed=int(g['seed']))
    orc = VolSDFOracle(sd, siren=True)
    s, n, h = orc.sdf_net.forward_with_nablas(T(g['pts']))
    close(s, g['sdf'], 1e-5, 1e-6)
    close(n, g['nablas'], 1e-5, 1e-5)
    close(h[:64], g['h'], 1e-5, 1e-6)
    close(orc.rad_net.forward(*[T(g[k]) for k in ('x', 'v', 'n', 'f')]), g['rgb_radiance'], 1e-5, 1e-6)
    with torch.no_grad():
        out = orc.render(T(g['rays_o']), T(g['rays_d']), N_samples=64, N_importance=64, max_upsample_steps=6)
    close(out['iter_usage'], g['iter_usage'], 0, 0)
    close(out['d_vals'], g['d_vals'], 1e-6, 1e-6)
    for k, gk in [('rgb', 'rgb'), ('depth_volume', 'depth'), ('mask_volume', 'mask'), ('normals_volume', 'normals')]:
        close(out[k], g[gk], 1e-5, 1e-6)


def test_surface_render_root_finding(golden):
    """oracle root finding vs ray_casting.surface_render(ray_casting_algo='root_finding') and
    root_finding_surface_points with non-default cfgs (fill_inf=False, logit_tau, short march)."""
    from oracle import surface
    g = golden('surface')
    orc = NeuSOracle(wg.neus_state(seed=int(g['seed'])))
    with torch.no_grad():
        out = surface.surface_render_neus(orc, T(g['rays_o']), T(g['rays_d']), algo='root_finding')
        np.testing.assert_array_equal(out['mask'].numpy(), g['rf_mask'].astype(bool))
        close(out['depth'], g['rf_depth'], 1e-6, 1e-6)
        close(out['rgb'], g['rf_rgb'], 1e-5, 1e-6)
        close(out['normals'], g['rf_normals'], 1e-5, 1e-6)
        d = torch.nn.functional.normalize(T(g['rays_d']), dim=-1)
        dp, p, m, msc = surface.root_find(orc.sdf_net.sdf, T(g['rays_o']), d, near=0.5, far=4.0, N_steps=64,
                                          N_secant_steps=4, logit_tau=0.01, fill_inf=False)
        np.testing.assert_array_equal(m.numpy(), g['rf2_mask'].astype(bool))
        np.testing.assert_array_equal(msc.numpy(), g['rf2_msc'].astype(bool))
        close(dp, g['rf2_d'], 1e-6, 1e-6)
        close(p, g['rf2_pts'], 1e-6, 1e-6)


def test_options(golden):
    """oracle vs the reference's option renders (gen_golden.gen_options): RadianceNet without view dirs
    (NeuS, UNISURF), UNISURF with a root-finding method other than 'secant', and root finding / sphere
    tracing with per-ray near / far tensors."""
    from oracle import surface
    g = golden('options')
    orc = NeuSOracle(wg.neus_state(seed=1, use_view_dirs=False), use_view_dirs=False)
    with torch.no_grad():
        out = orc.render(T(g['neus_rays_o']), T(g['neus_rays_d']))
    close(out['d_final'], g['neus_d_final'], 1e-6, 1e-6)
    close(out['radiance'], g['neus_radiance'], 1e-5, 1e-6)
    for k, gk in [('rgb', 'rgb'), ('depth_volume', 'depth'), ('mask_volume', 'mask'), ('normals_volume', 'normals')]:
        close(out[k], g['neus_' + gk], 1e-5, 1e-6)
    uo = UNISURFOracle(wg.unisurf_state(seed=3, use_view_dirs=False), use_view_dirs=False)
    for tag, method in [('uni', 'secant'), ('uni_nosec', 'none')]:
        with torch.no_grad():
            out = uo.render(T(g['uni_rays_o']), T(g['uni_rays_d']), logit_tau=float(g['uni_logit_tau']), method=method)
        np.testing.assert_array_equal(out['mask_surface'].numpy(), g[tag + '_mask_surface'].astype(bool))
        close(out['depth_surface'], g[tag + '_depth_surface'], 1e-6, 1e-6)
        for k, gk in [('rgb', 'rgb'), ('depth_volume', 'depth'), ('mask_volume', 'mask'),
                      ('normals_volume', 'normals')]:
            close(out[k], g[f'{tag}_{gk}'], 1e-5, 1e-6)
    net = nets.SDFNet(wg.neus_state(seed=1))
    o, d = T(g['rays_o']), torch.nn.functional.normalize(T(g['rays_d']), dim=-1)
    near, far = T(g['near']), T(g['far'])
    with torch.no_grad():
        for tag, kw in [('rf', dict(N_secant_steps=4, fill_inf=False)), ('rfn', dict(method='none', fill_inf=True))]:
            dp, p, m, msc = surface.root_find(net.sdf, o, d, near=near, far=far, N_steps=64, **kw)
            np.testing.assert_array_equal(m.numpy(), g[tag + '_mask'].astype(bool))
            np.testing.assert_array_equal(msc.numpy(), g[tag + '_msc'].astype(bool))
            close(dp, g[tag + '_d'], 1e-6, 1e-6)
            close(p, g[tag + '_pts'], 1e-6, 1e-6)
        dp, p, m = surface.sphere_trace(net.sdf, o, d, near=near, far=far, N_iters=10)
        np.testing.assert_array_equal(m.numpy(), g['st_mask'].astype(bool))
        close(dp, g['st_d'], 1e-6, 1e-6)
        close(p, g['st_pts'], 1e-6, 1e-6)


def train_grads_oracle(g, d_all=None):
    """oracle/train.py on the neus_train fixture: (losses, {param: grad}, d_all)"""
    from oracle.train import neus_train_losses
    No = int(g['N_outside']) if 'N_outside' in g else 0
    sd = {k: v.clone().requires_grad_(v.is_floating_point() and k != 'implicit_surface.obj_bounding_size')
          for k, v in wg.neus_state(seed=int(g['seed']), use_outside_nerf=No > 0).items()}
    H, W = int(g['H']), int(g['W'])
    ro, rd, _ = rays.get_rays(T(g['c2w']), T(g['K']), H, W)
    losses, d_all = neus_train_losses(sd, ro, rd, T(g['target_rgb']), T(g['target_mask']), d_all=d_all,
                                      N_outside=No)
    losses['total'].backward()
    return losses, {k: v.grad for k, v in sd.items() if v.grad is not None}, d_all


def check_grads(grads, g, rtol, atol_frac, report=print, net_scale=False):
    """per parameter: full gradient, or (norm, sum, 4096 sampled entries) for the big weight_v tensors;
    atol = atol_frac * max |grad| of the tensor (components near zero of a large gradient), or with
    net_scale of the tensor's whole network (first name component: implicit_surface / radiance_net /
    nerf_outside)"""
    keys = list(g.keys())
    names = sorted({k.split('/', 1)[1] for k in keys if k.startswith('g_norm/')})
    net_max = {}
    for k in names:
        net = k.split('.')[0]
        net_max[net] = max(net_max.get(net, 0.0), float(grads[k].detach().abs().max()))
    worst = 0.0
    for k in names:
        gr = grads[k].detach().reshape(-1).double().cpu().numpy()
        scale = (net_max[k.split('.')[0]] if net_scale else float(np.abs(gr).max())) + 1e-30
        if f'g_full/{k}' in keys:
            ref, mine = g[f'g_full/{k}'].astype(np.float64), gr
        else:
            ref, mine = g[f'g_val/{k}'].astype(np.float64), gr[g[f'g_idx/{k}']]
        err = np.abs(mine - ref)
        ok = err <= rtol * np.abs(ref) + atol_frac * scale
        rel_norm = abs(np.linalg.norm(gr) - float(g[f'g_norm/{k}'])) / (float(g[f'g_norm/{k}']) + 1e-30)
        worst = max(worst, float((err / scale).max()))
        report(f'{k}: max err {err.max():.3e} (scale {scale:.3e}), norm rel {rel_norm:.2e}, pass {ok.mean() * 100:.2f}%')
        assert ok.all(), k
        assert rel_norm <= rtol, k
    return worst


@pytest.mark.parametrize('name', ['neus_train', 'neus_train_nerfpp'])
def test_oracle_train_step_vs_golden(golden, name):
    """the oracle's NeuS training losses and every parameter gradient vs the reference's own
    Trainer.forward + backward (double backward through the nablas; with the NeRF++ background's
    parameters for neus_train_nerfpp)"""
    g = golden(name)
    torch.set_num_threads(8)
    losses, grads, _ = train_grads_oracle(g)
    for k in ('loss_img', 'loss_eikonal', 'loss_mask', 'total'):
        close(losses[k], g[f'loss/{k}'], 1e-5, 1e-7)
    check_grads(grads, g, 1e-4, 1e-6)


def volsdf_train_grads_oracle(g, d_all=None):
    """oracle/train.py on the volsdf_train fixture: (losses, {param: grad}, d_all)"""
    from oracle.train import volsdf_train_losses
    nerfpp = bool(g['nerfpp']) if 'nerfpp' in g else False
    siren = bool(g['siren']) if 'siren' in g else False
    state = wg.volsdf_siren_state(seed=int(g['seed'])) if siren else \
        wg.volsdf_state(seed=int(g['seed']), beta_init=float(g['beta_init']), use_nerfplusplus=nerfpp)
    sd = {k: v.clone().requires_grad_(v.is_floating_point() and k != 'implicit_surface.obj_bounding_size')
          for k, v in state.items()}
    H, W = int(g['H']), int(g['W'])
    ro, rd, _ = rays.get_rays(T(g['c2w']), T(g['K']), H, W)
    losses, d_all = volsdf_train_losses(sd, ro, rd, T(g['target_rgb']), T(g['eik_points']), d_all=d_all,
                                        N_outside=32 if nerfpp else 0, siren=siren)
    losses['total'].backward()
    return losses, {k: v.grad for k, v in sd.items() if v.grad is not None}, d_all


@pytest.mark.parametrize('name', ['volsdf_train', 'volsdf_train_nerfpp', 'volsdf_train_siren'])
def test_oracle_volsdf_train_step_vs_golden(golden, name):
    """the oracle's VolSDF training losses and every parameter gradient (surface net through the
    double backward of the nablas, radiance net, ln_beta; with the NeRF++ background its net too) vs
    the reference's own Trainer.forward + backward on the same rays, targets and eikonal points"""
    g = golden(name)
    torch.set_num_threads(8)
    losses, grads, d_all = volsdf_train_grads_oracle(g)
    close(d_all, g['d_vals'], 1e-6, 1e-6)
    for k in ('loss_img', 'loss_eikonal', 'total'):
        close(losses[k], g[f'loss/{k}'], 1e-5, 1e-7)
    check_grads(grads, g, 1e-4, 1e-6)


def unisurf_train_grads_oracle(g, d_all=None, surface_points=None):
    """oracle/train.py on the unisurf_train fixture: (losses, {param: grad}, d_all, surface_points)"""
    from oracle.train import unisurf_train_losses
    sd = {k: v.clone().requires_grad_(v.is_floating_point() and k != 'implicit_surface.obj_bounding_size')
          for k, v in wg.unisurf_state(seed=int(g['seed'])).items()}
    H, W = int(g['H']), int(g['W'])
    ro, rd, _ = rays.get_rays(T(g['c2w']), T(g['K']), H, W)
    losses, d_all, sp = unisurf_train_losses(sd, ro, rd, T(g['target_rgb']), T(g['surf_perturb']),
                                             logit_tau=float(g['logit_tau']), d_all=d_all,
                                             surface_points=surface_points)
    losses['total'].backward()
    return losses, {k: v.grad for k, v in sd.items() if v.grad is not None}, d_all, sp


def test_oracle_unisurf_train_step_vs_golden(golden):
    """the oracle's UNISURF training losses and every parameter gradient (surface net through the
    double backward of the nablas: windowed F.normalize into the radiance net and the normal
    smoothness term; radiance net) vs the reference's own Trainer.forward + backward on the same rays,
    targets and surface-point perturbation"""
    g = golden('unisurf_train')
    torch.set_num_threads(8)
    losses, grads, d_all, sp = unisurf_train_grads_oracle(g)
    close(sp, g['surface_points'], 1e-6, 1e-6)
    for k in ('loss_img', 'loss_reg', 'total'):
        close(losses[k], g[f'loss/{k}'], 1e-5, 1e-9)
    check_grads(grads, g, 1e-4, 1e-6)
