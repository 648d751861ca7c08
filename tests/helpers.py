"""Shared test helpers: build neurecon_amd models with the fixture configs and compare arrays."""
import numpy as np
import torch

SURF = dict(use_siren=False, embed_multires=6, geometric_init=True, D=8, W=256, skips=[4])


def neus_model(sd, use_outside_nerf=False, device='cuda', precision='fp32', use_view_dirs=True):
    from neurecon_amd.frameworks.neus import NeuS
    m = NeuS(variance_init=0.05, speed_factor=10.0, input_ch=3, W_geo_feat=256, use_outside_nerf=use_outside_nerf,
             obj_bounding_radius=1.0, surface_cfg=dict(radius_init=0.5, precision=precision, **SURF),
             radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=4, use_view_dirs=use_view_dirs,
                               D=4, W=256, skips=[], precision=precision))
    m.load_state_dict(sd)
    return m.to(device).eval()


def report(name, a, b, rtol, atol):
    """max errors + fraction of elements within |a-b| <= atol + rtol*|b|."""
    a = a.detach().cpu().numpy() if isinstance(a, torch.Tensor) else np.asarray(a)
    b = np.asarray(b)
    err = np.abs(a.astype(np.float64) - b.astype(np.float64))
    ok = err <= atol + rtol * np.abs(b)
    frac = ok.mean() if ok.size else 1.0
    print(f'{name}: max abs {err.max() if err.size else 0:.3e}, pass {frac * 100:.3f}% (rtol {rtol}, atol {atol})')
    return ok, err


def per_ray_ok(ok):
    """collapse an element-wise pass mask [(B), N, ...] to per-ray"""
    ok = np.asarray(ok)
    ok = ok.reshape(-1, *ok.shape[-1:]) if ok.ndim >= 2 else ok
    return ok


def to_gpu(a):
    return torch.from_numpy(np.asarray(a)).cuda()


def volsdf_model(sd, beta_init, device='cuda', precision='fp32', use_nerfplusplus=False):
    from neurecon_amd.frameworks.volsdf import VolSDF
    m = VolSDF(beta_init=beta_init, speed_factor=10.0, input_ch=3, W_geo_feat=256, obj_bounding_radius=3.0,
               use_nerfplusplus=use_nerfplusplus, surface_cfg=dict(radius_init=1.0, precision=precision, **SURF),
               radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=-1, use_view_dirs=True,
                                 D=4, W=256, skips=[], precision=precision))
    m.load_state_dict(sd)
    return m.to(device).eval()


def unisurf_model(sd, device='cuda', precision='fp32', use_view_dirs=True):
    from neurecon_amd.frameworks.unisurf import UNISURF
    m = UNISURF(W_geo_feat=256, surface_cfg=dict(radius_init=1.0, precision=precision, **SURF),
                radiance_cfg=dict(use_siren=False, embed_multires=-1, embed_multires_view=-1,
                                  use_view_dirs=use_view_dirs, D=4, W=256, skips=[], precision=precision))
    m.load_state_dict(sd)
    return m.to(device).eval()
