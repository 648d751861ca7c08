"""Config (e) work units per library kernel for one render (nr_profile events): the SDF forward launches' points
(march, secant) against the active-ray counts the march should leave.

    python tools/e_units_probe.py"""
import sys, os, torch
sys.path[:0] = [os.getcwd()]
import bench
from neurecon_amd import _lib as L
from neurecon_amd.frameworks.unisurf import UNISURF, volume_render
dev = torch.device('cuda:0')
torch.manual_seed(0)
surf = dict(use_siren=False, embed_multires=6, radius_init=1.0, geometric_init=True, D=8, W=256, skips=[4], precision='f16x3')
rad = dict(use_siren=False, embed_multires=-1, embed_multires_view=-1, use_view_dirs=True, D=4, W=256, skips=[], precision='f16x3')
m = UNISURF(W_geo_feat=256, surface_cfg=surf, radiance_cfg=rad).to(dev).eval()
ro, rd = bench.camera_for(dev, 64, 64, 80.0, 3.0)
kw = dict(batched=True, calc_normal=True, detailed_output=False, logit_tau=0.0, radius_of_interest=4.0, method='secant', N_query=64, N_freespace=32)
with torch.no_grad():
    volume_render(ro, rd, m, **kw); torch.cuda.synchronize()
    L.profile_read(); L.profile_enable(True)
    volume_render(ro, rd, m, **kw); torch.cuda.synchronize()
    L.profile_enable(False)
    print(L.profile_read())
    _, _, ex = volume_render(ro, rd, m, **dict(kw, detailed_output=True))
    print({k: tuple(v.shape) for k, v in ex.items()})
