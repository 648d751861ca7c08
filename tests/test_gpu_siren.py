"""GPU parity of the SIREN networks (models/base.py:84-115 Sine / SirenLayer; configs/volsdf_siren.yaml:
SDF D=5, skips=[], embed_multires=-1; radiance D=5, embed_multires_view=4) against the reference's
outputs (tests/golden/siren.npz, gen_golden.gen_siren): siren_sdf_kernel (forward, nablas, geometry
feature), the sine variant of radiance_kernel, and a VolSDF render with both nets.
Bar: 1e-4 relative + 1e-6 absolute (nablas: 1e-4 of their norm + 1e-5), masks / iter_usage identical.
"""
import numpy as np
import pytest
import torch

import weightgen as wg
from helpers import report, to_gpu

pytestmark = pytest.mark.gpu

RT, AT = 1e-4, 1e-6


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from neurecon_amd import _lib
    _lib.lib()


def siren_model(precision):
    from neurecon_amd.frameworks.volsdf import VolSDF
    m = VolSDF(beta_init=0.1, speed_factor=10.0, input_ch=3, W_geo_feat=256, obj_bounding_radius=3.0,
               use_nerfplusplus=False,
               surface_cfg=dict(use_siren=True, D=5, W=256, skips=[], embed_multires=-1, radius_init=1.0,
                                geometric_init=True, precision=precision),
               radiance_cfg=dict(use_siren=True, D=5, W=256, skips=[], embed_multires=-1, embed_multires_view=4,
                                 use_view_dirs=True, precision=precision))
    m.load_state_dict(wg.volsdf_siren_state(seed=7))
    return m.cuda().eval()


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_siren_sdf_and_radiance_vs_golden(golden, precision):
    g = golden('siren')
    m = siren_model(precision)
    with torch.no_grad():
        s, n, h = m.implicit_surface.forward_with_nablas(to_gpu(g['pts']))
        s_only = m.implicit_surface.forward(to_gpu(g['pts']))
        rgb = m.radiance_net.forward(to_gpu(g['x']), to_gpu(g['v']), to_gpu(g['n']), to_gpu(g['f']))
    assert report('siren sdf', s, g['sdf'], RT, AT)[0].all()
    assert torch.equal(s, s_only)  # the forward-only launch computes the same values
    nab, ref = n.cpu().numpy(), g['nablas']
    err = np.abs(nab - ref).max(-1)
    print(f'siren nablas: max abs {err.max():.3e} (|n| up to {np.linalg.norm(ref, axis=-1).max():.2f})')
    assert (err <= 1e-4 * np.linalg.norm(ref, axis=-1) + 1e-5).all()
    assert report('siren feature', h[:64], g['h'], RT, 1e-5)[0].all()
    assert report('siren radiance', rgb, g['rgb_radiance'], RT, AT)[0].all()


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_siren_volsdf_render_vs_golden(golden, precision):
    from neurecon_amd.frameworks.volsdf import volume_render
    g = golden('siren')
    m = siren_model(precision)
    with torch.no_grad():
        rgb, depth, ex = volume_render(to_gpu(g['rays_o']), to_gpu(g['rays_d']), m, near=0.0, far=6.0,
                                       obj_bounding_radius=3.0, batched=True, calc_normal=True, detailed_output=True,
                                       N_samples=64, N_importance=64, max_upsample_steps=6)
    assert (ex['iter_usage'].cpu().numpy() == g['iter_usage']).all()
    ok_d, _ = report('siren d_vals', ex['d_vals'], g['d_vals'], 1e-5, 1e-6)
    same = ok_d.reshape(-1, ok_d.shape[-1]).all(-1)
    ok = (report('siren rgb', rgb, g['rgb'], RT, AT)[0].all(-1) & report('siren depth', depth, g['depth'], RT, AT)[0]
          & report('siren mask', ex['mask_volume'], g['mask'], RT, AT)[0]).reshape(-1)
    ok_n = report('siren normals', ex['normals_volume'], g['normals'], RT, 1e-4)[0].all(-1).reshape(-1)
    print(f'siren/{precision}: identical samples on {same.mean() * 100:.1f}% of rays, per-ray pass {ok.mean() * 100:.1f}%')
    assert ok[same].all() and ok_n[same].all()
    assert ok.mean() >= 0.95


def test_siren_pretrain_hook_vs_oracle():
    """ImplicitSurface.pretrain_hook / pretrain_siren_sdf (base.py:226-233, :284-310): the L1 sphere fit
    with Adam, its forward and gradient on the training path -- 4 steps of 2048 points vs the same
    steps on the oracle network (torch CPU autograd + Adam) from the same CPU draws: losses within
    1e-4 relative, is_pretrained set once."""
    from oracle.nets import SDFNet
    from neurecon_amd.base import pretrain_siren_sdf
    m = siren_model('fp32')
    surf = m.implicit_surface.train()
    sd = {k: v.clone().float().requires_grad_(True) for k, v in wg.volsdf_siren_state(seed=7).items()
          if k.startswith('implicit_surface.surface_fc_layers')}

    class Log:
        def __init__(self):
            self.v = []

        def add(self, a, b, val, it):
            self.v.append(val)
    log = Log()
    torch.manual_seed(5)
    pretrain_siren_sdf(surf, num_iters=4, batch_points=2048, target_radius=1.0, obj_bounding_size=3.0, logger=log)
    torch.manual_seed(5)
    opt = torch.optim.Adam(list(sd.values()), lr=1e-4)
    ref = []
    for _ in range(4):
        pts = torch.empty([2048, 3]).uniform_(-3.0, 3.0).float()
        net = SDFNet(sd, D=5, skips=(), multires=-1, siren=True)
        loss = torch.nn.functional.l1_loss(net.sdf(pts), pts.norm(dim=-1) - 1.0)
        opt.zero_grad()
        loss.backward()
        opt.step()
        ref.append(float(loss))
    print('pretrain losses gpu', log.v, 'oracle', ref)
    assert np.allclose(log.v, ref, rtol=1e-4, atol=0)
    surf.is_pretrained.fill_(False)
    assert surf.pretrain_hook({'num_iters': 1, 'batch_points': 64}) is True
    assert bool(surf.is_pretrained) and surf.pretrain_hook({'num_iters': 1}) is False
