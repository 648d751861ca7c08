"""Generate golden parity vectors by running the REFERENCE implementation (this container only).

Usage (from the repo root, in the build container where /root/reference exists):
    python tests/golden/gen_golden.py

The reference is imported read-only from /root/reference with the off-path modules stubbed
(cv2/addict/imageio/skimage/torchvision are only used by data loading,
camera-matrix decomposition and logging, none of which is on the render path).  Only inputs
and outputs are written (small .npz files under tests/golden/); weights are rebuilt from seeds
by tests/golden/weightgen.py.  Nothing here is imported by the product or by the GPU tests.
"""
import os
import sys
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import weightgen as wg  # noqa: E402

REF = '/root/reference'


def _import_reference():
    for name in ['cv2', 'addict', 'imageio', 'skimage', 'skimage.transform', 'torchvision',
                 'torchvision.utils']:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules['addict'].Dict = dict
    sys.modules['skimage.transform'].rescale = None
    sys.modules['skimage'].transform = sys.modules['skimage.transform']
    sys.path.insert(0, REF)
    from models.frameworks import neus, volsdf, unisurf  # noqa
    from models import base, ray_casting  # noqa
    from utils import rend_util, train_util  # noqa
    return types.SimpleNamespace(neus=neus, volsdf=volsdf, unisurf=unisurf, base=base,
                                 ray_casting=ray_casting, rend_util=rend_util, train_util=train_util)


SURF = dict(use_siren=False, embed_multires=6, geometric_init=True, D=8, W=256, skips=[4])


def _np(d):
    out = {}
    for k, v in d.items():
        if isinstance(v, torch.Tensor):
            v = v.detach().cpu()
            out[k] = v.numpy() if v.dtype != torch.bool else v.numpy().astype(np.uint8)
        else:
            out[k] = np.asarray(v)
    return out


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **_np(arrays))
    print('wrote', path, os.path.getsize(path), 'bytes')


def camera_rays(R, key, idx=None):
    H, W, f, dist = wg.CAMERAS[key]
    c2w = wg.look_at_c2w(dist)[None]
    K = wg.intrinsics(f, H, W)[None]
    rays_o, rays_d, _ = R.rend_util.get_rays(c2w, K, H, W, N_rays=-1)
    if idx is not None:
        rays_o, rays_d = rays_o[:, idx], rays_d[:, idx]
    return rays_o.contiguous(), rays_d.contiguous()


def grid_idx(H, W, n=8, lo=0.15, hi=0.85):
    rows = np.linspace(lo * (H - 1), hi * (H - 1), n).round().astype(np.int64)
    cols = np.linspace(lo * (W - 1), hi * (W - 1), n).round().astype(np.int64)
    return torch.tensor((rows[:, None] * W + cols[None, :]).reshape(-1))


def gen_components(R):
    torch.manual_seed(123)
    # Embedders (A3)
    x = torch.randn(256, 3) * 1.5
    x4 = torch.randn(256, 4)
    e6, _ = R.base.get_embedder(6)
    e4, _ = R.base.get_embedder(4)
    e10, _ = R.base.get_embedder(10, input_dim=4)
    save('embed.npz', x=x, x4=x4, emb6=e6(x), emb4=e4(x), emb10_4d=e10(x4))

    # SDF net (A4-A6) with NeuS config
    sd = wg.neus_state(seed=11)
    surf = R.base.ImplicitSurface(W_geo_feat=256, input_ch=3, obj_bounding_size=1.0, radius_init=0.5, **SURF)
    surf.load_state_dict({k[len('implicit_surface.'):]: v for k, v in sd.items()
                          if k.startswith('implicit_surface.')})
    pts = torch.randn(512, 3) * 0.6
    with torch.no_grad():
        sdf_ng, h_ng = surf.forward(pts, return_h=True)
    sdf, nab, h = surf.forward_with_nablas(pts)
    save('sdf_net.npz', seed=11, pts=pts, sdf_nograd=sdf_ng, sdf=sdf, nablas=nab, h=h[:64], h_nograd=h_ng[:64])

    # Radiance nets (A7): NeuS cfg (view embed 4) and VolSDF cfg (identity embeds)
    rad_n = R.base.RadianceNet(W_geo_feat=256, embed_multires=-1, embed_multires_view=4, use_view_dirs=True,
                               D=4, W=256, skips=[])
    rad_n.load_state_dict({k[len('radiance_net.'):]: v for k, v in sd.items() if k.startswith('radiance_net.')})
    sdv = wg.volsdf_state(seed=12)
    rad_v = R.base.RadianceNet(W_geo_feat=256, embed_multires=-1, embed_multires_view=-1, use_view_dirs=True,
                               D=4, W=256, skips=[])
    rad_v.load_state_dict({k[len('radiance_net.'):]: v for k, v in sdv.items() if k.startswith('radiance_net.')})
    P = 256
    rx = torch.randn(P, 3) * 0.5
    rv = torch.nn.functional.normalize(torch.randn(P, 3), dim=-1)
    rn = torch.randn(P, 3)
    rf = torch.randn(P, 256) * 0.3
    with torch.no_grad():
        out_n = rad_n(rx, rv, rn, rf)
        out_v = rad_v(rx, rv, rn, rf)
    save('radiance.npz', seed_neus=11, seed_volsdf=12, x=rx, v=rv, n=rn, f=rf, rgb_neus=out_n, rgb_volsdf=out_v)

    # NeRF++ background net (A8)
    sdo = wg.neus_state(seed=13, use_outside_nerf=True)
    nerf = R.base.NeRF(input_ch=4, multires=10, multires_view=4, use_view_dirs=True)
    nerf.load_state_dict({k[len('nerf_outside.'):]: v for k, v in sdo.items() if k.startswith('nerf_outside.')})
    p = torch.randn(P, 3) * 3.0
    r = p.norm(dim=-1, keepdim=True)
    x4 = torch.cat([p / r, 1. / r], dim=-1)
    with torch.no_grad():
        sig, rgb = nerf(x4, rv)
    save('nerf.npz', seed=13, x4=x4, v=rv, sigma=sig, rgb=rgb)


def gen_sampling(R):
    torch.manual_seed(7)
    ru = R.rend_util
    # sample_pdf: random weights, plus rows with zeros, one-hot mass, ties in bins
    Rn, L = 64, 33
    bins = torch.sort(torch.rand(Rn, L) * 4.0, dim=-1).values
    bins[3, 5:9] = bins[3, 5]          # repeated bins
    w = torch.rand(Rn, L - 1)
    w[0] = 0.0                          # all-zero weights (uniform after +1e-5)
    w[1] = 0.0; w[1, 7] = 1.0           # one-hot
    w[2, :16] = 0.0                     # half empty
    w[4] = 1e-7
    s16 = ru.sample_pdf(bins, w, 16, det=True)
    s66 = ru.sample_pdf(bins, w, 66, det=True)
    u_rand = torch.rand(Rn, 16)
    # reproduce det=False with an explicit u by monkeypatching torch.rand inside the call
    orig = torch.rand
    try:
        torch.rand = lambda *a, **k: u_rand.clone()
        s_rand = ru.sample_pdf(bins, w, 16, det=False)
    finally:
        torch.rand = orig
    cdf_in = torch.cumsum(torch.rand(Rn, L - 1), -1)
    cdf_in = cdf_in / cdf_in[:, -1:]
    sc = ru.sample_cdf(bins, cdf_in, 24, det=True)
    # near/far & sphere intersections
    o = torch.randn(Rn, 3) * 2.0
    d = torch.nn.functional.normalize(torch.randn(Rn, 3), dim=-1)
    near, far = ru.near_far_from_sphere(o, d, r=1.0)
    near4, far4 = ru.near_far_from_sphere(o, d, r=4.0, keepdim=False)
    n_i, f_i, m_i = ru.get_sphere_intersection(o, d, r=1.0)
    o_in = torch.nn.functional.normalize(torch.randn(Rn, 3), dim=-1) * 0.9
    rs = 3.0 / torch.flip(torch.linspace(0, 1, 34)[1:-1], dims=[-1])
    dv = ru.get_dvals_from_radius(o_in * 2.0, d, rs.expand(Rn, 32))
    save('sampling.npz', bins=bins, weights=w, s16=s16, s66=s66, u_rand=u_rand, s_rand=s_rand,
         cdf_in=cdf_in, s_cdf=sc, o=o, d=d, near=near, far=far, near4=near4, far4=far4,
         si_near=n_i, si_far=f_i, si_mask=m_i, o_in=o_in * 2.0, rs=rs, dvals=dv)

    # get_rays: matrix and quaternion forms, plus random pixel selection
    H, W = 12, 20
    c2w = wg.look_at_c2w(2.5)[None]
    K = wg.intrinsics(25.0, H, W)[None]
    K[0, 0, 1] = 0.3   # skew
    ro, rd, si = ru.get_rays(c2w, K, H, W, N_rays=-1)
    # NOTE: the quaternion branch (rend_util.py:114-119) cannot run: quat_to_rot unpacks two prefix
    # dims (rend_util.py:77) that get_rays' bmm path cannot accept, so it is not pinned here.
    torch.manual_seed(5)
    ror, rdr, sir = ru.get_rays(c2w, K, H, W, N_rays=37)
    save('get_rays.npz', H=H, W=W, c2w=c2w, K=K, rays_o=ro, rays_d=rd,
         rays_o_sel=ror, rays_d_sel=rdr, select_inds=sir)


def _neus_model(R, sd, use_outside_nerf):
    m = R.neus.NeuS(variance_init=0.05, speed_factor=10.0, input_ch=3, W_geo_feat=256,
                    use_outside_nerf=use_outside_nerf, obj_bounding_radius=1.0,
                    surface_cfg=dict(radius_init=0.5, **SURF),
                    radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=4,
                                      use_view_dirs=True, D=4, W=256, skips=[]))
    m.load_state_dict(sd)
    return m.eval()


def gen_neus(R):
    # config (b): NeuS 64x64 camera, 64-ray sub-grid
    sd = wg.neus_state(seed=1)
    model = _neus_model(R, sd, False)
    H, W, _, _ = wg.CAMERAS['b']
    idx = grid_idx(H, W)
    ro, rd = camera_rays(R, 'b', idx)
    with torch.no_grad():
        rgb, depth, ex = R.neus.volume_render(
            ro, rd, model, obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=True,
            perturb=False, N_samples=64, N_importance=64, N_outside=0, upsample_algo='official_solution',
            N_upsample_iters=4)
    save('neus_b.npz', seed=1, rays_o=ro, rays_d=rd, idx=idx, rgb=rgb, depth=depth,
         mask=ex['mask_volume'], normals=ex['normals_volume'], d_final=ex['d_final'],
         sdf=ex['implicit_surface'], nablas=ex['implicit_nablas'], radiance=ex['radiance'],
         alpha=ex['alpha'], cdf=ex['cdf'], weights=ex['visibility_weights'])

    # NeuS direct_use / direct_more upsampling variants (12 rays)
    sub = slice(20, 32)
    outs = {}
    for algo in ['direct_use', 'direct_more']:
        with torch.no_grad():
            rgb2, depth2, ex2 = R.neus.volume_render(
                ro[:, sub], rd[:, sub], model, obj_bounding_radius=1.0, batched=True, calc_normal=True,
                detailed_output=True, perturb=False, N_samples=64, N_importance=64, upsample_algo=algo,
                N_nograd_samples=512)
        outs[algo + '_rgb'] = rgb2
        outs[algo + '_depth'] = depth2
        outs[algo + '_d_final'] = ex2['d_final']
    save('neus_algos.npz', seed=1, rays_o=ro[:, sub], rays_d=rd[:, sub], N_nograd_samples=512, **outs)

    # config (d): NeuS + NeRF++ background, 800x600 camera sub-grid
    sd = wg.neus_state(seed=4, use_outside_nerf=True)
    model = _neus_model(R, sd, True)
    H, W, _, _ = wg.CAMERAS['d']
    idx = grid_idx(H, W, n=8, lo=0.02, hi=0.98)
    ro, rd = camera_rays(R, 'd', idx)
    with torch.no_grad():
        rgb, depth, ex = R.neus.volume_render(
            ro, rd, model, obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=True,
            perturb=False, N_samples=64, N_importance=64, N_outside=32, upsample_algo='official_solution',
            N_upsample_iters=4)
    save('neus_d.npz', seed=4, rays_o=ro, rays_d=rd, idx=idx, rgb=rgb, depth=depth,
         mask=ex['mask_volume'], normals=ex['normals_volume'], d_final=ex['d_final'],
         sdf=ex['implicit_surface'], nablas=ex['implicit_nablas'], radiance=ex['radiance'],
         alpha=ex['alpha'], weights=ex['visibility_weights'], sigma_out=ex['sigma_out'],
         radiance_out=ex['radiance_out'])


def _volsdf_model(R, sd, beta_init, use_nerfplusplus=False):
    m = R.volsdf.VolSDF(beta_init=beta_init, speed_factor=10.0, input_ch=3, W_geo_feat=256,
                        obj_bounding_radius=3.0, use_nerfplusplus=use_nerfplusplus,
                        surface_cfg=dict(radius_init=1.0, **SURF),
                        radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=-1,
                                          use_view_dirs=True, D=4, W=256, skips=[]))
    m.load_state_dict(sd)
    return m.eval()


def gen_volsdf(R):
    # config (a): 16x32 camera, 512 rays, beta 0.1, 64+64
    sd = wg.volsdf_state(seed=2, beta_init=0.1)
    model = _volsdf_model(R, sd, 0.1)
    ro, rd = camera_rays(R, 'a')
    with torch.no_grad():
        rgb, depth, ex = R.volsdf.volume_render(
            ro, rd, model, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, calc_normal=True,
            detailed_output=True, perturb=False, N_samples=64, N_importance=64, max_upsample_steps=6)
    keep = slice(0, 512, 8)
    save('volsdf_a.npz', seed=2, beta_init=0.1, rays_o=ro, rays_d=rd, rgb=rgb, depth=depth,
         mask=ex['mask_volume'], normals=ex['normals_volume'], beta_map=ex['beta_map'],
         iter_usage=ex['iter_usage'], d_vals=ex['d_vals'][:, keep], sdf=ex['implicit_surface'][:, keep],
         weights=ex['visibility_weights'][:, keep], radiance=ex['radiance'][:, keep])

    # config (c): 32x64 camera sub-grid, beta 1e-3 (adaptive loop active), 128+128
    sd = wg.volsdf_state(seed=5, beta_init=1e-3)
    model = _volsdf_model(R, sd, 1e-3)
    H, W, _, _ = wg.CAMERAS['c']
    idx = grid_idx(H, W, n=8, lo=0.05, hi=0.95)
    ro, rd = camera_rays(R, 'c', idx)
    with torch.no_grad():
        rgb, depth, ex = R.volsdf.volume_render(
            ro, rd, model, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, calc_normal=True,
            detailed_output=True, perturb=False, N_samples=128, N_importance=128, max_upsample_steps=6)
    save('volsdf_c.npz', seed=5, beta_init=1e-3, rays_o=ro, rays_d=rd, idx=idx, rgb=rgb, depth=depth,
         mask=ex['mask_volume'], normals=ex['normals_volume'], beta_map=ex['beta_map'],
         iter_usage=ex['iter_usage'], d_vals=ex['d_vals'], sdf=ex['implicit_surface'],
         weights=ex['visibility_weights'])

    # error_bound / sdf_to_sigma on a 1-D analytic SDF (debug_tools/test_volsdf_algo.py:73-87 shape)
    x = torch.linspace(0, 6.0, 128)
    y1 = -x + 1.65; y2 = x - 1.55; y3 = -x + 2.05
    sdf1d = torch.where(x < 1.8, torch.where(x < 1.6, y1, y2), y3)
    beta = 0.003
    b1 = R.volsdf.error_bound(x, sdf1d, 1. / beta, beta)
    bplus = float(np.sqrt(36.0 / (4 * 127 * np.log(1.1))))
    b2 = R.volsdf.error_bound(x, sdf1d, 1. / bplus, bplus)
    sg = R.volsdf.sdf_to_sigma(sdf1d, 1. / beta, beta)
    save('volsdf_1d.npz', x=x, sdf=sdf1d, beta=beta, bplus=bplus, bounds_net=b1, bounds_plus=b2, sigma=sg)


def gen_volsdf_nerfpp(R):
    """VolSDF with the NeRF++ background (volsdf.py:400-405, 451-469): config-(a) camera (inside
    the r=3 bounding sphere, so every ray intersects it), 128 rays, 64+64 inside, 32 outside."""
    sd = wg.volsdf_state(seed=6, beta_init=0.1, use_nerfplusplus=True)
    model = _volsdf_model(R, sd, 0.1, use_nerfplusplus=True)
    H, W, _, _ = wg.CAMERAS['a']
    idx = torch.arange(0, H * W, 4)
    ro, rd = camera_rays(R, 'a', idx)
    with torch.no_grad():
        rgb, depth, ex = R.volsdf.volume_render(
            ro, rd, model, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, calc_normal=True,
            detailed_output=True, perturb=False, N_samples=64, N_importance=64, N_outside=32,
            use_nerfplusplus=True, max_upsample_steps=6)
    save('volsdf_nerfpp.npz', seed=6, beta_init=0.1, rays_o=ro, rays_d=rd, idx=idx, rgb=rgb, depth=depth,
         mask=ex['mask_volume'], normals=ex['normals_volume'], beta_map=ex['beta_map'],
         iter_usage=ex['iter_usage'], d_vals=ex['d_vals'], sigma=ex['sigma'], weights=ex['visibility_weights'],
         sigma_out=ex['sigma_out'], radiance_out=ex['radiance_out'], radiance=ex['radiance'])


def gen_unisurf(R):
    sd = wg.unisurf_state(seed=3)
    m = R.unisurf.UNISURF(W_geo_feat=256, surface_cfg=dict(radius_init=1.0, **SURF),
                          radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=-1,
                                            use_view_dirs=True, D=4, W=256, skips=[]))
    m.load_state_dict(sd)
    m.eval()
    H, W, _, _ = wg.CAMERAS['e']
    idx = grid_idx(H, W, n=8, lo=0.1, hi=0.9)
    ro, rd = camera_rays(R, 'e', idx)
    logit_tau = R.unisurf.UNISURF.get_surface_from_opacity(0.5)
    res = {}
    for tag, nc in [('', 1048576), ('_nc1000', 1000)]:
        with torch.no_grad():
            rgb, depth, ex = R.unisurf.volume_render(
                ro, rd, m, batched=True, calc_normal=True, detailed_output=True, perturb=False,
                logit_tau=logit_tau, radius_of_interest=4.0, interval=1.0, N_query=64, N_freespace=32,
                netchunk=nc)
        res.update({'rgb' + tag: rgb, 'depth' + tag: depth, 'mask' + tag: ex['mask_volume'],
                    'normals' + tag: ex['normals_volume']})
        if tag == '':
            res.update(dict(depth_surface=ex['depth_surface'], mask_surface=ex['mask_surface'],
                            surface_points=ex['surface_points'], sdf=ex['implicit_surface'],
                            nablas=ex['implicit_nablas'], radiance=ex['radiance'],
                            weights=ex['visibility_weights']))
    save('unisurf_e.npz', seed=3, logit_tau=float(logit_tau), rays_o=ro, rays_d=rd, idx=idx, **res)


def gen_surface(R):
    """surface_render / sphere tracing (ray_casting.py:163-263) and extract_mesh's SDF grid
    (mesh_util.py:82-112) on NeuS weights (seed 1), 256 rays of the config-(b) camera."""
    sd = wg.neus_state(seed=1)
    model = _neus_model(R, sd, False)
    H, W, _, _ = wg.CAMERAS['b']
    idx = grid_idx(H, W, n=16, lo=0.0, hi=1.0)
    ro, rd = camera_rays(R, 'b', idx)
    with torch.no_grad():
        rgb, depth, ex = R.ray_casting.surface_render(ro, rd, model, calc_normal=True, rayschunk=8192, batched=True,
                                                      ray_casting_algo='sphere_tracing')
        rdn = torch.nn.functional.normalize(rd, dim=-1)
        d5, p5, m5 = R.ray_casting.sphere_tracing_surface_points(model.implicit_surface, ro, rdn, near=0.5, far=4.0,
                                                                 N_iters=5)
        rgb_rf, depth_rf, ex_rf = R.ray_casting.surface_render(ro, rd, model, calc_normal=True, rayschunk=8192,
                                                               batched=True, ray_casting_algo='root_finding')
        rf = R.ray_casting.root_finding_surface_points(model.implicit_surface, ro.clone(), rdn.clone(), near=0.5,
                                                       far=4.0, N_steps=64, N_secant_steps=4, logit_tau=0.01,
                                                       fill_inf=False)
    # extract_mesh runs as shipped except for what this image lacks: numpy>=1.24 has no np.int
    # (mesh_util.py:87), there is no GPU (`.cuda()`, :104) and no scikit-image/plyfile (the
    # marching-cubes writer is replaced by a capture of the SDF volume it receives).
    for name in ['plyfile', 'skimage.measure']:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules['skimage'].measure = sys.modules['skimage.measure']
    from utils import mesh_util
    grids = {}
    np_int = getattr(np, 'int', None)
    cuda = torch.Tensor.cuda
    np.int = int
    torch.Tensor.cuda = lambda self, *a, **k: self
    saved = mesh_util.convert_sigma_samples_to_ply
    try:
        for N, s in [(16, 2.0), (24, 1.5)]:
            mesh_util.convert_sigma_samples_to_ply = lambda out, *a, _N=N, **k: grids.__setitem__(_N, out.copy())
            with torch.no_grad():
                mesh_util.extract_mesh(model.implicit_surface, volume_size=s, N=N, show_progress=False, chunk=1000)
    finally:
        mesh_util.convert_sigma_samples_to_ply = saved
        torch.Tensor.cuda = cuda
        if np_int is None:
            del np.int
    save('surface.npz', seed=1, rays_o=ro, rays_d=rd, idx=idx, rgb=rgb, depth=depth,
         nablas=ex['implicit_nablas'], mask=ex['mask_surface'], normals=ex['normals_surface'],
         st5_d=d5, st5_pts=p5, st5_mask=m5, grid16=grids[16], grid24=grids[24],
         rf_rgb=rgb_rf, rf_depth=depth_rf, rf_nablas=ex_rf['implicit_nablas'], rf_mask=ex_rf['mask_surface'],
         rf_normals=ex_rf['normals_surface'], rf2_d=rf[0], rf2_pts=rf[1], rf2_mask=rf[2], rf2_msc=rf[3])


class _RecordRand:
    """torch.rand wrapper recording every draw (in call order) of a perturb=True reference render, so
    the GPU test can replay exactly these uniforms through neurecon_amd.rend_util.uniform."""

    def __init__(self):
        self.draws = []

    def __enter__(self):
        self.orig = torch.rand

        def rand(*a, **k):
            t = self.orig(*a, **k)
            self.draws.append(t.detach().clone())
            return t
        torch.rand = rand
        return self

    def __exit__(self, *exc):
        torch.rand = self.orig


def gen_perturb(R):
    """perturb=True renders (stratified / stochastic sampling, the training-time path) of configs (b),
    (d) and (e) on 64-ray sub-grids, with the uniforms the reference drew."""
    out = {}
    for key, seed, nerfpp in [('b', 1, False), ('d', 4, True)]:
        sd = wg.neus_state(seed=seed, use_outside_nerf=nerfpp)
        model = _neus_model(R, sd, nerfpp)
        H, W, _, _ = wg.CAMERAS[key]
        idx = grid_idx(H, W) if key == 'b' else grid_idx(H, W, n=8, lo=0.02, hi=0.98)
        ro, rd = camera_rays(R, key, idx)
        torch.manual_seed(100 + seed)
        with torch.no_grad(), _RecordRand() as rec:
            rgb, depth, ex = R.neus.volume_render(
                ro, rd, model, obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=True,
                perturb=True, N_samples=64, N_importance=64, N_outside=32 if nerfpp else 0,
                upsample_algo='official_solution', N_upsample_iters=4)
        out.update({f'{key}_rays_o': ro, f'{key}_rays_d': rd, f'{key}_rgb': rgb, f'{key}_depth': depth,
                    f'{key}_mask': ex['mask_volume'], f'{key}_normals': ex['normals_volume'],
                    f'{key}_d_final': ex['d_final'], f'{key}_n_draws': len(rec.draws)})
        out.update({f'{key}_u{i}': u for i, u in enumerate(rec.draws)})
    save('neus_perturb.npz', **out)

    sd = wg.unisurf_state(seed=3)
    m = R.unisurf.UNISURF(W_geo_feat=256, surface_cfg=dict(radius_init=1.0, **SURF),
                          radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=-1,
                                            use_view_dirs=True, D=4, W=256, skips=[]))
    m.load_state_dict(sd)
    m.eval()
    H, W, _, _ = wg.CAMERAS['e']
    ro, rd = camera_rays(R, 'e', grid_idx(H, W, n=8, lo=0.1, hi=0.9))
    logit_tau = R.unisurf.UNISURF.get_surface_from_opacity(0.5)
    torch.manual_seed(103)
    with torch.no_grad(), _RecordRand() as rec:
        rgb, depth, ex = R.unisurf.volume_render(
            ro, rd, m, batched=True, calc_normal=True, detailed_output=True, perturb=True, logit_tau=logit_tau,
            radius_of_interest=4.0, interval=1.0, N_query=64, N_freespace=32)
    save('unisurf_perturb.npz', seed=3, logit_tau=float(logit_tau), rays_o=ro, rays_d=rd, rgb=rgb, depth=depth,
         mask=ex['mask_volume'], normals=ex['normals_volume'], d_vals=ex.get('d_vals', depth),
         sdf=ex['implicit_surface'], weights=ex['visibility_weights'], n_draws=len(rec.draws),
         **{f'u{i}': u for i, u in enumerate(rec.draws)})


def gen_options(R):
    """Render options beyond the headline configs, run through the reference: RadianceNet built with
    use_view_dirs=False (config key model.radiance.use_view_dirs; the render itself keeps
    use_view_dirs=True -- volume_render(use_view_dirs=False) fails inside batchify_query on the None
    view dirs, train_util.py:27) on NeuS (36 rays of the config-(b) camera) and UNISURF (36 rays of
    config (e), with 'secant' and with another root-finding method, ray_casting.py:128-135), and root finding / sphere tracing with per-ray near / far tensors
    from near_far_from_sphere (ray_casting.py:53-54, :70-73, :175)."""
    out = {}
    rad_nv = dict(use_siren=False, embed_multires=-1, embed_multires_view=4, use_view_dirs=False, D=4, W=256,
                  skips=[])
    sd = wg.neus_state(seed=1, use_view_dirs=False)
    m = R.neus.NeuS(variance_init=0.05, speed_factor=10.0, input_ch=3, W_geo_feat=256, use_outside_nerf=False,
                    obj_bounding_radius=1.0, surface_cfg=dict(radius_init=0.5, **SURF), radiance_cfg=rad_nv)
    m.load_state_dict(sd)
    m.eval()
    H, W, _, _ = wg.CAMERAS['b']
    ro, rd = camera_rays(R, 'b', grid_idx(H, W, n=6))
    with torch.no_grad():
        rgb, depth, ex = R.neus.volume_render(
            ro, rd, m, obj_bounding_radius=1.0, batched=True, calc_normal=True, detailed_output=True,
            perturb=False, N_samples=64, N_importance=64, N_outside=0,
            upsample_algo='official_solution', N_upsample_iters=4)
    out.update(neus_rays_o=ro, neus_rays_d=rd, neus_rgb=rgb, neus_depth=depth, neus_mask=ex['mask_volume'],
               neus_normals=ex['normals_volume'], neus_d_final=ex['d_final'], neus_radiance=ex['radiance'])

    sdu = wg.unisurf_state(seed=3, use_view_dirs=False)
    mu = R.unisurf.UNISURF(W_geo_feat=256, surface_cfg=dict(radius_init=1.0, **SURF),
                           radiance_cfg=dict(rad_nv, embed_multires_view=-1))
    mu.load_state_dict(sdu)
    mu.eval()
    H, W, _, _ = wg.CAMERAS['e']
    ro, rd = camera_rays(R, 'e', grid_idx(H, W, n=6, lo=0.1, hi=0.9))
    logit_tau = R.unisurf.UNISURF.get_surface_from_opacity(0.5)
    out.update(uni_rays_o=ro, uni_rays_d=rd, uni_logit_tau=float(logit_tau))
    for tag, method in [('uni', 'secant'), ('uni_nosec', 'none')]:
        with torch.no_grad():
            rgb, depth, ex = R.unisurf.volume_render(
                ro, rd, mu, batched=True, calc_normal=True, detailed_output=True, perturb=False,
                method=method, logit_tau=logit_tau, radius_of_interest=4.0, interval=1.0,
                N_query=64, N_freespace=32)
        out.update({f'{tag}_rgb': rgb, f'{tag}_depth': depth, f'{tag}_mask': ex['mask_volume'],
                    f'{tag}_normals': ex['normals_volume'], f'{tag}_depth_surface': ex['depth_surface'],
                    f'{tag}_mask_surface': ex['mask_surface'], f'{tag}_surface_points': ex['surface_points']})

    model = _neus_model(R, wg.neus_state(seed=1), False)
    H, W, _, _ = wg.CAMERAS['b']
    ro, rd = camera_rays(R, 'b', grid_idx(H, W, n=16, lo=0.0, hi=1.0))
    rdn = torch.nn.functional.normalize(rd, dim=-1)
    near, far = R.rend_util.near_far_from_sphere(ro, rdn, r=1.0, keepdim=False)
    with torch.no_grad():
        rf = R.ray_casting.root_finding_surface_points(model.implicit_surface, ro.clone(), rdn.clone(), near=near,
                                                       far=far, N_steps=64, N_secant_steps=4, fill_inf=False)
        rfn = R.ray_casting.root_finding_surface_points(model.implicit_surface, ro.clone(), rdn.clone(), near=near,
                                                        far=far, N_steps=64, method='none', fill_inf=True)
        st = R.ray_casting.sphere_tracing_surface_points(model.implicit_surface, ro, rdn, near=near, far=far,
                                                         N_iters=10)
    out.update(rays_o=ro, rays_d=rd, near=near, far=far, rf_d=rf[0], rf_pts=rf[1], rf_mask=rf[2], rf_msc=rf[3],
               rfn_d=rfn[0], rfn_pts=rfn[1], rfn_mask=rfn[2], rfn_msc=rfn[3], st_d=st[0], st_pts=st[1],
               st_mask=st[2])
    save('options.npz', **out)


def gen_volsdf_perturb(R):
    """VolSDF perturb=True renders (random final fine samples, volsdf.py:102; NeRF++ radius strata,
    :460-465) with every torch.rand draw recorded: config (a) on 64 rays (beta 0.1), config (c) on 64
    rays (beta 1e-3, several convergence rounds) and VolSDF + NeRF++ on 64 rays."""
    out = {}
    cases = [('a', 2, 0.1, False, 'a', dict(n=8), 64, 64), ('c', 5, 1e-3, False, 'c', dict(n=8, lo=0.05, hi=0.95), 128, 128),
             ('pp', 6, 0.1, True, 'a', dict(n=8, lo=0.0, hi=1.0), 64, 64)]
    for key, seed, beta_init, nerfpp, cam, gi, Ns, Ni in cases:
        sd = wg.volsdf_state(seed=seed, beta_init=beta_init, use_nerfplusplus=nerfpp)
        model = _volsdf_model(R, sd, beta_init, use_nerfplusplus=nerfpp)
        H, W, _, _ = wg.CAMERAS[cam]
        ro, rd = camera_rays(R, cam, grid_idx(H, W, **gi))
        torch.manual_seed(200 + seed)
        with torch.no_grad(), _RecordRand() as rec:
            rgb, depth, ex = R.volsdf.volume_render(
                ro, rd, model, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, calc_normal=True,
                detailed_output=True, perturb=True, N_samples=Ns, N_importance=Ni, N_outside=32,
                use_nerfplusplus=nerfpp, max_upsample_steps=6)
        out.update({f'{key}_seed': seed, f'{key}_beta_init': beta_init, f'{key}_N_samples': Ns,
                    f'{key}_N_importance': Ni, f'{key}_rays_o': ro, f'{key}_rays_d': rd, f'{key}_rgb': rgb,
                    f'{key}_depth': depth, f'{key}_mask': ex['mask_volume'], f'{key}_normals': ex['normals_volume'],
                    f'{key}_d_vals': ex['d_vals'], f'{key}_iter_usage': ex['iter_usage'],
                    f'{key}_beta_map': ex['beta_map'], f'{key}_n_draws': len(rec.draws)})
        out.update({f'{key}_u{i}': u for i, u in enumerate(rec.draws)})
    save('volsdf_perturb.npz', **out)


def gen_siren(R):
    """SIREN nets of configs/volsdf_siren.yaml (base.py:84-115): ImplicitSurface(use_siren, D=5,
    skips=[], embed_multires=-1) forward + nablas + feature on 512 points, RadianceNet(use_siren, D=5,
    embed_multires_view=4) on 256 points, and a VolSDF render with both on 64 rays of the config-(a)
    camera (64 + 64 samples; weights from weightgen.volsdf_siren_state, loaded as if pretrained)."""
    sd = wg.volsdf_siren_state(seed=7)
    surf_cfg = dict(use_siren=True, D=5, W=256, skips=[], embed_multires=-1, radius_init=1.0, geometric_init=True)
    rad_cfg = dict(use_siren=True, D=5, W=256, skips=[], embed_multires=-1, embed_multires_view=4,
                   use_view_dirs=True)
    m = R.volsdf.VolSDF(beta_init=0.1, speed_factor=10.0, input_ch=3, W_geo_feat=256, obj_bounding_radius=3.0,
                        use_nerfplusplus=False, surface_cfg=surf_cfg, radiance_cfg=rad_cfg)
    m.load_state_dict(sd)
    m.eval()
    torch.manual_seed(321)
    pts = torch.randn(512, 3) * 0.8
    sdf, nab, h = m.implicit_surface.forward_with_nablas(pts)
    P = 256
    rx = torch.randn(P, 3) * 0.5
    rv = torch.nn.functional.normalize(torch.randn(P, 3), dim=-1)
    rn = torch.randn(P, 3)
    rf = torch.randn(P, 256) * 0.3
    with torch.no_grad():
        rgb_r = m.radiance_net(rx, rv, rn, rf)
    H, W, _, _ = wg.CAMERAS['a']
    ro, rd = camera_rays(R, 'a', grid_idx(H, W, n=8, lo=0.0, hi=1.0))
    with torch.no_grad():
        rgb, depth, ex = R.volsdf.volume_render(
            ro, rd, m, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, calc_normal=True,
            detailed_output=True, perturb=False, N_samples=64, N_importance=64, max_upsample_steps=6)
    save('siren.npz', seed=7, pts=pts, sdf=sdf.detach(), nablas=nab.detach(), h=h.detach()[:64], x=rx, v=rv, n=rn,
         f=rf, rgb_radiance=rgb_r, rays_o=ro, rays_d=rd, rgb=rgb, depth=depth, mask=ex['mask_volume'],
         normals=ex['normals_volume'], beta_map=ex['beta_map'], iter_usage=ex['iter_usage'], d_vals=ex['d_vals'],
         vol_sdf=ex['implicit_surface'], vol_nablas=ex['implicit_nablas'], weights=ex['visibility_weights'])


# parameters whose full gradient is stored; the large weight_v tensors keep norm, sum and a fixed
# sample of 4096 elements (tests/test_oracle_golden.py compares those)
def _grad_summary(named):
    out = {}
    g = torch.Generator().manual_seed(7)
    for k, p in named:
        gr = p.grad.detach().reshape(-1).clone()
        out[f'g_norm/{k}'] = gr.norm()
        out[f'g_sum/{k}'] = gr.double().sum()
        if gr.numel() <= 4096:
            out[f'g_full/{k}'] = gr
        else:
            idx = torch.randperm(gr.numel(), generator=g)[:4096]
            out[f'g_idx/{k}'] = idx
            out[f'g_val/{k}'] = gr[idx]
    return out


def gen_train(R):
    """One NeuS training step's losses and parameter gradients (models/frameworks/neus.py:417-485 ->
    train.py:205 backward) on an 8x8 camera (64 rays, N_rays=-1 so no random pixels), perturb=False,
    with_mask=True, seeded random targets; and the same with the NeRF++ background (N_outside=32)."""
    _gen_train(R, 'neus_train.npz', 1, 0)
    _gen_train(R, 'neus_train_nerfpp.npz', 4, 32)


def _gen_train(R, name, seed, N_outside):
    import types as _t
    sd = wg.neus_state(seed=seed, use_outside_nerf=N_outside > 0)
    model = _neus_model(R, sd, N_outside > 0)
    model.train()
    H = W = 8
    c2w = wg.look_at_c2w(3.0)[None]
    if N_outside > 0:  # off-centre: the centre ray's mid-point samples must not hit the origin (x_out = p/|p|)
        c2w[0, 0, 3] += 0.0137
    K = wg.intrinsics(20.0, H, W)[None]
    g = torch.Generator().manual_seed(5)
    target_rgb = torch.rand(1, H * W, 3, generator=g)
    target_mask = (torch.rand(1, H * W, generator=g) > 0.4)
    args = _t.SimpleNamespace(data=_t.SimpleNamespace(N_rays=-1),
                              training=_t.SimpleNamespace(w_eikonal=0.1, w_mask=1.0, with_mask=True))
    kw = dict(H=H, W=W, upsample_algo='official_solution', N_nograd_samples=2048, N_upsample_iters=4,
              N_outside=N_outside, obj_bounding_radius=1.0, batched=True, perturb=False, white_bkgd=False)
    trainer = R.neus.Trainer(model, device_ids=[0], batched=True)
    ret = trainer.forward(args, None, {'intrinsics': K, 'c2w': c2w, 'object_mask': target_mask},
                          {'rgb': target_rgb}, kw, 0, device='cpu')
    losses = {k: torch.mean(v) for k, v in ret['losses'].items()}
    model.zero_grad()
    losses['total'].backward()
    ex = ret['extras']
    save(name, seed=seed, N_outside=N_outside, H=H, W=W, f=20.0, dist=3.0, target_rgb=target_rgb,
         target_mask=target_mask,
         c2w=c2w, K=K, **{f'loss/{k}': v.detach() for k, v in losses.items()},
         rgb=ex['rgb'].detach(), mask_volume=ex['mask_volume'].detach(), d_final=ex['d_final'].detach(),
         **_grad_summary(model.named_parameters()))


def gen_train_volsdf(R):
    """One VolSDF training step (models/frameworks/volsdf.py:564-640 -> train.py:205 backward) on an
    8x8 camera (64 rays, N_rays=-1), builtin background (volsdf_train.npz) or the NeRF++ background
    with 32 outside samples (volsdf_train_nerfpp.npz), 64 + 64 samples, 6 upsampling rounds,
    perturb=False, seeded random targets; the eikonal points (torch's uniform_(-3, 3), volsdf.py:609)
    are recorded from the reference's own call so the GPU test can replay them."""
    _gen_train_volsdf(R, 'volsdf_train.npz', 3, False, 20.0)
    # wide field of view: a third of the rays miss the surface, so the background net gets gradients
    _gen_train_volsdf(R, 'volsdf_train_nerfpp.npz', 7, True, 5.0)
    # configs/volsdf_siren.yaml's nets (SirenLayers, D=5, weights as in gen_siren)
    _gen_train_volsdf(R, 'volsdf_train_siren.npz', 7, False, 20.0, siren=True)


def _gen_train_volsdf(R, name, seed, nerfpp, f, siren=False):
    import types as _t
    if siren:
        sd = wg.volsdf_siren_state(seed=seed)
        surf_cfg = dict(use_siren=True, D=5, W=256, skips=[], embed_multires=-1, radius_init=1.0, geometric_init=True)
        rad_cfg = dict(use_siren=True, D=5, W=256, skips=[], embed_multires=-1, embed_multires_view=4,
                       use_view_dirs=True)
        model = R.volsdf.VolSDF(beta_init=0.1, speed_factor=10.0, input_ch=3, W_geo_feat=256, obj_bounding_radius=3.0,
                                use_nerfplusplus=False, surface_cfg=surf_cfg, radiance_cfg=rad_cfg)
        model.load_state_dict(sd)
    else:
        sd = wg.volsdf_state(seed=seed, beta_init=0.1, use_nerfplusplus=nerfpp)
        model = _volsdf_model(R, sd, 0.1, use_nerfplusplus=nerfpp)
    model.train()
    H = W = 8
    c2w = wg.look_at_c2w(2.7)[None]
    K = wg.intrinsics(f, H, W)[None]
    g = torch.Generator().manual_seed(6)
    target_rgb = torch.rand(1, H * W, 3, generator=g)
    seen = []
    fwn = model.implicit_surface.forward_with_nablas

    def rec(x, *a, **k):
        seen.append(x.detach().clone())
        return fwn(x, *a, **k)
    model.implicit_surface.forward_with_nablas = rec
    args = _t.SimpleNamespace(data=_t.SimpleNamespace(N_rays=-1), model=_t.SimpleNamespace(obj_bounding_radius=3.0),
                              training=_t.SimpleNamespace(w_eikonal=0.1))
    kw = dict(H=H, W=W, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, perturb=False, white_bkgd=False,
              max_upsample_steps=6, use_nerfplusplus=nerfpp, N_samples=64, N_importance=64, N_outside=32)
    trainer = R.volsdf.Trainer(model, device_ids=[0], batched=True)
    trainer.device = 'cpu'
    torch.manual_seed(9)
    ret = trainer.forward(args, None, {'intrinsics': K, 'c2w': c2w}, {'rgb': target_rgb}, kw, 0)
    losses = {k: torch.mean(v) for k, v in ret['losses'].items()}
    model.zero_grad()
    losses['total'].backward()
    ex = ret['extras']
    save(name, seed=seed, beta_init=0.1, nerfpp=nerfpp, siren=siren, H=H, W=W, f=f, dist=2.7, target_rgb=target_rgb, c2w=c2w, K=K,
         eik_points=seen[-1], **{f'loss/{k}': v.detach() for k, v in losses.items()},
         rgb=ex['rgb'].detach(), d_vals=ex['d_vals'].detach(), iter_usage=ex['iter_usage'].detach(),
         **_grad_summary(model.named_parameters()))


def gen_train_unisurf(R):
    """One UNISURF training step (models/frameworks/unisurf.py:303-351 -> train.py:205 backward) on an
    8x8 camera (64 rays, N_rays=-1), it=0 (interval = delta_max = 1), perturb=False, w_reg=0.01 with
    perturb_surface_pts=0.01, seeded random targets; the surface-point perturbation (torch.rand,
    unisurf.py:335) is recorded from the reference's own call so the GPU test can replay it."""
    import types as _t
    sd = wg.unisurf_state(seed=3)
    m = R.unisurf.UNISURF(W_geo_feat=256, surface_cfg=dict(radius_init=1.0, **SURF),
                          radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=-1,
                                            use_view_dirs=True, D=4, W=256, skips=[]))
    m.load_state_dict(sd)
    m.train()
    H = W = 8
    c2w = wg.look_at_c2w(2.7)[None]
    c2w[0, 0, 3] += 0.0137
    K = wg.intrinsics(f, H, W)[None]
    g = torch.Generator().manual_seed(8)
    target_rgb = torch.rand(1, H * W, 3, generator=g)
    args = _t.SimpleNamespace(data=_t.SimpleNamespace(N_rays=-1),
                              training=_t.SimpleNamespace(w_reg=0.01, perturb_surface_pts=0.01, delta_max=1.0,
                                                          delta_min=0.05, delta_beta=1.5e-5))
    logit_tau = float(R.unisurf.UNISURF.get_surface_from_opacity(0.5))
    kw = dict(H=H, W=W, batched=True, perturb=False, white_bkgd=False, logit_tau=logit_tau, radius_of_interest=4.0,
              N_query=64, N_freespace=32)
    trainer = R.unisurf.Trainer(m, device_ids=[0], batched=True)
    torch.manual_seed(11)
    with _RecordRand() as rr:
        ret = trainer.forward(args, None, {'intrinsics': K, 'c2w': c2w}, {'rgb': target_rgb}, kw, 0, device='cpu')
    assert len(rr.draws) == 1, len(rr.draws)
    losses = {k: torch.mean(v) for k, v in ret['losses'].items()}
    m.zero_grad()
    losses['total'].backward()
    ex = ret['extras']
    surf_perturb = (rr.draws[0] - 0.5) * 2. * 0.01
    save('unisurf_train.npz', seed=3, H=H, W=W, f=f, dist=2.7, target_rgb=target_rgb, c2w=c2w, K=K,
         logit_tau=logit_tau, rand_draw=rr.draws[0], surf_perturb=surf_perturb,
         **{f'loss/{k}': v.detach() for k, v in losses.items()}, rgb=ex['rgb'].detach(),
         surface_points=ex['surface_points'].detach(), mask_surface=ex['mask_surface'].detach(),
         depth_surface=ex['depth_surface'].detach(), **_grad_summary(m.named_parameters()))


def main():
    torch.set_num_threads(8)
    R = _import_reference()
    only = sys.argv[1:]
    gens = dict(components=gen_components, sampling=gen_sampling, neus=gen_neus, volsdf=gen_volsdf,
                unisurf=gen_unisurf, surface=gen_surface,
                volsdf_nerfpp=gen_volsdf_nerfpp, perturb=gen_perturb, train=gen_train, options=gen_options,
                volsdf_perturb=gen_volsdf_perturb, siren=gen_siren, train_volsdf=gen_train_volsdf,
                train_unisurf=gen_train_unisurf)
    for name, fn in gens.items():
        if not only or name in only:
            fn(R)


if __name__ == '__main__':
    main()
