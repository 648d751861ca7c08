"""GPU parity of the training path: the NeuS and VolSDF training steps' losses and EVERY
parameter gradient -- through the double backward of the SDF MLP's nablas -- vs the oracle's
autograd (oracle/train.py, pinned to the reference's own Trainer.forward + backward by
tests/test_oracle_golden.py::test_oracle_train_step_vs_golden) and vs that reference golden.

Bar: |grad - ref| <= 1e-4 |ref| + 1e-5 max|ref| per parameter tensor (components near zero of a
large gradient), losses 1e-5 relative.  The gradient GEMMs run in fp32 (hipBLASLt); the no-grad
sample pass runs in the model's precision -- the oracle gets the GPU's sample depths so a flipped
sampling decision cannot masquerade as a gradient error.
"""
import os
import socket
import types

import numpy as np
import pytest
import torch

import weightgen as wg
from helpers import neus_model, report, unisurf_model, volsdf_model
from test_oracle_golden import check_grads, train_grads_oracle, unisurf_train_grads_oracle, volsdf_train_grads_oracle

pytestmark = pytest.mark.gpu

RTOL, ATOL_FRAC = 1e-4, 1e-5


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from neurecon_amd import _lib
    _lib.lib()


def _args():
    return types.SimpleNamespace(data=types.SimpleNamespace(N_rays=-1),
                                 training=types.SimpleNamespace(w_eikonal=0.1, w_mask=1.0, with_mask=True))


def _kw(H, W, N_outside=0):
    return dict(H=H, W=W, upsample_algo='official_solution', N_nograd_samples=2048, N_upsample_iters=4,
                N_outside=N_outside, obj_bounding_radius=1.0, batched=True, perturb=False, white_bkgd=False)


def _n_out(g):
    return int(g['N_outside']) if 'N_outside' in g else 0


def _gpu_step(g, precision):
    from neurecon_amd.frameworks.neus import Trainer
    No = _n_out(g)
    m = neus_model(wg.neus_state(seed=int(g['seed']), use_outside_nerf=No > 0), use_outside_nerf=No > 0,
                   precision=precision)
    m.train()
    H, W = int(g['H']), int(g['W'])
    T = lambda a: torch.from_numpy(np.asarray(a)).cuda()
    trainer = Trainer(m, device_ids=[0])
    ret = trainer.forward(_args(), None, {'intrinsics': T(g['K']), 'c2w': T(g['c2w']),
                                          'object_mask': T(g['target_mask'])},
                          {'rgb': T(g['target_rgb'])}, _kw(H, W, _n_out(g)), 0, device='cuda')
    losses = {k: torch.mean(v) for k, v in ret['losses'].items()}
    m.zero_grad()
    losses['total'].backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters()}
    return m, losses, grads, ret['extras']


def _gpu_sample_depths(m, g):
    from neurecon_amd import rend_util
    from neurecon_amd.frameworks.neus import _sample_depths
    H, W = int(g['H']), int(g['W'])
    ro, rd, _ = rend_util.get_rays(torch.from_numpy(g['c2w']).cuda(), torch.from_numpy(g['K']).cuda(), H, W)
    with torch.no_grad():
        d, _ = _sample_depths(ro.reshape(-1, 3).contiguous(), rd.reshape(-1, 3).contiguous(), m, ro.device, 1.0, True,
                              1, 65536, None, None, False, 1 / 64., 64, 64, 'official_solution', 2048, 4)
    return d.reshape(1, H * W, -1).cpu()


@pytest.mark.parametrize('name', ['neus_train', 'neus_train_nerfpp'])
@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_neus_train_step_vs_oracle_and_golden(golden, precision, name):
    """neus_train_nerfpp: the same step with the NeRF++ background (N_outside=32): its 8-layer net's
    parameters get gradients through the merged compositing (neus.py:325-352).  There the absolute
    term is 3e-5 of the largest gradient of the parameter's network rather than 1e-5 of the tensor's:
    the background net's first layers get gradients 4 orders below its heads (7e-7 vs 4e-2), and the
    reference's own gradients move by up to 1.2e-5 (background net), 6.5e-5 (radiance net) and 9e-3
    (surface net) of their network's largest gradient when the encodings feeding the nets move by
    one fp32 ulp (tools/train_sensitivity.py, oracle pinned to the reference)."""
    g = golden(name)
    net_scale = name.endswith('nerfpp')
    atol_frac = 3e-5 if net_scale else ATOL_FRAC
    m, losses, grads, ex = _gpu_step(g, precision)
    d_all = _gpu_sample_depths(m, g)
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref_losses, ref_grads, d_ref = train_grads_oracle(g, d_all=d_all)
    for k in ('loss_img', 'loss_eikonal', 'loss_mask', 'total'):
        a, b = float(losses[k]), float(ref_losses[k])
        print(f'{precision} {k}: gpu {a:.8f} oracle {b:.8f} golden {float(g["loss/" + k]):.8f}')
        assert abs(a - b) <= 1e-5 * abs(b) + 1e-7
    worst = check_grads(grads, _as_golden(ref_grads, g), RTOL, atol_frac, net_scale=net_scale)
    print(f'{precision}: worst gradient error / tensor scale {worst:.3e}')
    # and straight against the reference's golden when the sample depths agree with its own
    _, _, d_own = train_grads_oracle(g)
    if torch.allclose(d_own, d_all, rtol=1e-6, atol=1e-6):
        check_grads(grads, g, RTOL, atol_frac, net_scale=net_scale)
        print(f'{precision}: sample depths match the reference (1e-6) -> gradients checked against the golden too')
    else:
        moved = ((d_own - d_all).abs() > 1e-6 * (1 + d_own.abs())).any(-1)
        print(f'{precision}: golden gradient check NOT run: the GPU sample depths differ from the reference\'s on '
              f'{int(moved.sum())} of {moved.numel()} rays (max {float((d_own - d_all).abs().max()):.3e}); the step is '
              f'held to the oracle on the GPU depths, and the oracle to the golden (test_oracle_train_step_vs_golden)')


@pytest.mark.parametrize('name', ['volsdf_train', 'volsdf_train_nerfpp', 'volsdf_train_siren'])
@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_volsdf_train_step_vs_oracle_and_golden(golden, precision, name, monkeypatch):
    """VolSDF's training step (volsdf.py:564-640): losses and every parameter gradient -- surface net
    through the double backward of the nablas, radiance net, ln_beta through sdf_to_sigma -- vs the
    oracle on the GPU's sample depths, and vs the reference's golden when the depths agree.  The
    eikonal points replay the reference's draws (volsdf.py:609).  Absolute term: 2e-4 of the largest
    gradient of the parameter's network, twice the reference's own fp32 sensitivity: its gradients
    move by up to 1.0e-5 (surface) and 1.0e-4 (radiance) of their network's largest gradient (1e-4 /
    3.7e-4 of a tensor's) when the positional encodings move by one fp32 ulp
    (tools/train_sensitivity.py volsdf_train; radiance ReLUs at their kink flip).  Measured here: 1.0e-4
    (fp32 sample pass) and 1.8e-6 (f16x3 sample pass: other depths, no ReLU near its kink)."""
    from neurecon_amd.frameworks import volsdf as V
    g = golden(name)
    nerfpp = bool(g['nerfpp']) if 'nerfpp' in g else False
    T = lambda a: torch.from_numpy(np.asarray(a)).cuda()
    eik = T(g['eik_points'])
    monkeypatch.setattr(V, 'eikonal_points', lambda like, bound: eik.reshape(like.shape).to(like.dtype))
    beta0 = float(g['beta_init'])
    if 'siren' in g and bool(g['siren']):  # configs/volsdf_siren.yaml's nets
        from test_gpu_siren import siren_model
        m = siren_model(precision)
    else:
        m = volsdf_model(wg.volsdf_state(seed=int(g['seed']), beta_init=beta0, use_nerfplusplus=nerfpp), beta0,
                         precision=precision, use_nerfplusplus=nerfpp)
    m.train()
    args = types.SimpleNamespace(data=types.SimpleNamespace(N_rays=-1),
                                 model=types.SimpleNamespace(obj_bounding_radius=3.0),
                                 training=types.SimpleNamespace(w_eikonal=0.1))
    kw = dict(H=int(g['H']), W=int(g['W']), near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, perturb=False,
              white_bkgd=False, max_upsample_steps=6, use_nerfplusplus=nerfpp, N_samples=64, N_importance=64,
              N_outside=32)
    ret = V.Trainer(m, device_ids=[0]).forward(args, None, {'intrinsics': T(g['K']), 'c2w': T(g['c2w'])},
                                               {'rgb': T(g['target_rgb'])}, kw, 0, device='cuda')
    losses = {k: torch.mean(v) for k, v in ret['losses'].items()}
    m.zero_grad()
    losses['total'].backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None}
    d_all = ret['extras']['d_vals'].detach().cpu()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref_losses, ref_grads, _ = volsdf_train_grads_oracle(g, d_all=d_all)
    for k in ('loss_img', 'loss_eikonal', 'total'):
        a, b = float(losses[k]), float(ref_losses[k])
        print(f'{precision} {k}: gpu {a:.8f} oracle {b:.8f} golden {float(g["loss/" + k]):.8f}')
        assert abs(a - b) <= 1e-5 * abs(b) + 1e-7
    worst = check_grads(grads, _as_golden(ref_grads, g), RTOL, 2e-4, net_scale=True)
    print(f'{precision}: worst gradient error / network scale {worst:.3e}')
    same = torch.allclose(d_all, torch.from_numpy(g['d_vals']), rtol=1e-6, atol=1e-6)
    print(f'{precision}: sample depths {"match" if same else "differ from"} the reference (1e-6)')
    if same:
        check_grads(grads, g, RTOL, 2e-4, net_scale=True)


@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_unisurf_train_step_vs_oracle_and_golden(golden, precision, monkeypatch):
    """UNISURF's training step (unisurf.py:303-351): losses and every parameter gradient -- surface net
    through the double backward of the nablas (windowed F.normalize into the radiance net, and the
    normal smoothness term on the root-finding surface points), radiance net -- vs the oracle on the
    GPU's sample depths and surface points, and vs the reference's golden when those agree.  The
    surface-point perturbation replays the reference's draw (unisurf.py:335)."""
    from neurecon_amd.frameworks import unisurf as U
    g = golden('unisurf_train')
    T = lambda a: torch.from_numpy(np.asarray(a)).cuda()
    sp_pert = T(g['surf_perturb'])
    monkeypatch.setattr(U, 'surface_perturbation', lambda like, scale: sp_pert.reshape(like.shape).to(like.dtype))
    m = unisurf_model(wg.unisurf_state(seed=int(g['seed'])), precision=precision)
    m.train()
    args = types.SimpleNamespace(data=types.SimpleNamespace(N_rays=-1),
                                 training=types.SimpleNamespace(w_reg=0.01, perturb_surface_pts=0.01, delta_max=1.0,
                                                                delta_min=0.05, delta_beta=1.5e-5))
    kw = dict(H=int(g['H']), W=int(g['W']), batched=True, perturb=False, white_bkgd=False,
              logit_tau=float(g['logit_tau']), radius_of_interest=4.0, N_query=64, N_freespace=32)
    ret = U.Trainer(m, device_ids=[0]).forward(args, None, {'intrinsics': T(g['K']), 'c2w': T(g['c2w'])},
                                               {'rgb': T(g['target_rgb'])}, kw, 0, device='cuda')
    losses = {k: torch.mean(v) for k, v in ret['losses'].items()}
    m.zero_grad()
    losses['total'].backward()
    torch.cuda.synchronize()
    grads = {k: p.grad.detach().cpu() for k, p in m.named_parameters() if p.grad is not None}
    d_all = ret['extras']['d_all'].detach().cpu()
    sp = ret['extras']['surface_points'].detach().cpu()
    torch.set_num_threads(max(1, min(16, torch.get_num_threads())))
    ref_losses, ref_grads, _, _ = unisurf_train_grads_oracle(g, d_all=d_all, surface_points=sp)
    for k in ('loss_img', 'loss_reg', 'total'):
        a, b = float(losses[k]), float(ref_losses[k])
        print(f'{precision} {k}: gpu {a:.8f} oracle {b:.8f} golden {float(g["loss/" + k]):.8f}')
        assert abs(a - b) <= 1e-5 * abs(b) + 1e-9
    worst = check_grads(grads, _as_golden(ref_grads, g), RTOL, 2e-4, net_scale=True)
    print(f'{precision}: worst gradient error / network scale {worst:.3e}')
    same = torch.allclose(sp, torch.from_numpy(g['surface_points']), rtol=1e-6, atol=1e-6)
    print(f'{precision}: surface points {"match" if same else "differ from"} the reference (1e-6)')
    if same:
        check_grads(grads, g, RTOL, 2e-4, net_scale=True)


def _as_golden(ref_grads, g):
    """the oracle's full gradients in the golden's summary layout (same sampled indices)"""
    out = {}
    for k in g.keys():
        if not k.startswith('g_norm/'):
            continue
        name = k.split('/', 1)[1]
        gr = ref_grads[name].detach().reshape(-1)
        out[f'g_norm/{name}'] = np.asarray(float(gr.norm()))
        if f'g_full/{name}' in g.keys():
            out[f'g_full/{name}'] = gr.numpy()
        else:
            idx = g[f'g_idx/{name}']
            out[f'g_idx/{name}'] = idx
            out[f'g_val/{name}'] = gr.numpy()[idx]
    return out


def test_sdf_double_backward_vs_autograd():
    """SdfNabla on its own: random points (ragged P), random upstream gradients for sdf, nablas and
    the geometry feature -> every SDF-net parameter gradient vs torch autograd (create_graph) on CPU."""
    from oracle.nets import SDFNet
    from oracle.train import nablas_graph
    from neurecon_amd import training as T
    sd = wg.neus_state(seed=11)
    m = neus_model(sd)
    m.train()
    torch.manual_seed(3)
    for P in (1, 130, 2000):
        x = torch.randn(P, 3) * 0.7
        gs, gn, gf = torch.randn(P), torch.randn(P, 3), torch.randn(P, 256) * 0.01
        sdp = {k: v.clone().requires_grad_(True) for k, v in sd.items() if k.startswith('implicit_surface.')
               and not k.endswith('obj_bounding_size')}
        s, n, h = nablas_graph(SDFNet(sdp), x)
        ((s * gs).sum() + (n * gn).sum() + (h * gf).sum()).backward()
        m.zero_grad()
        s2, n2, h2 = T.sdf_nablas(m.implicit_surface, x.cuda(), True)
        assert report(f'train sdf P={P}', s2, s.detach(), 1e-5, 1e-6)[0].all()
        assert report(f'train nablas P={P}', n2, n.detach(), 1e-4, 1e-5)[0].all()
        ((s2 * gs.cuda()).sum() + (n2 * gn.cuda()).sum() + (h2 * gf.cuda()).sum()).backward()
        for k, p in m.implicit_surface.named_parameters():
            ref = sdp['implicit_surface.' + k].grad
            got = p.grad.detach().cpu()
            scale = float(ref.abs().max())
            ok, _ = report(f'  d {k} P={P}', got, ref, RTOL, ATOL_FRAC * scale)
            assert ok.all(), k


def test_radiance_backward_vs_autograd():
    from oracle.nets import RadianceNet
    from neurecon_amd import training as T
    sd = wg.neus_state(seed=11)
    m = neus_model(sd)
    m.train()
    torch.manual_seed(4)
    P = 777
    x, v = torch.randn(P, 3), torch.nn.functional.normalize(torch.randn(P, 3), dim=-1)
    nrm, feat = torch.randn(P, 3).requires_grad_(True), torch.randn(P, 256).requires_grad_(True)
    gy = torch.randn(P, 3)
    rp = {k: t.clone().requires_grad_(True) for k, t in sd.items() if k.startswith('radiance_net.')}
    net = RadianceNet(rp, multires_view=4)
    # ReLU's derivative jumps at 0: a pre-activation within rounding of the kink may take either
    # side on the GPU and the CPU.  Points with such a unit get no upstream gradient (on both sides).
    from oracle.nets import embed
    with torch.no_grad():
        h = torch.cat([x, embed(v, 4), nrm, feat], -1)
        kink = torch.zeros(P, dtype=torch.bool)
        for W, b in net.layers[:-1]:
            z = torch.nn.functional.linear(h, W, b)
            kink |= (z.abs() < 2e-5).any(-1)
            h = torch.relu(z)
    print(f'points next to a ReLU kink (masked): {int(kink.sum())} / {P}')
    assert kink.float().mean() < 0.1
    gy[kink] = 0.0
    y = net.forward(x, v, nrm, feat)
    (y * gy).sum().backward()
    nrm2 = nrm.detach().cuda().requires_grad_(True)
    feat2 = feat.detach().cuda().requires_grad_(True)
    y2 = T.radiance(m.radiance_net, x.cuda(), v.cuda(), nrm2, feat2)
    assert report('train radiance', y2, y.detach(), 1e-5, 1e-6)[0].all()
    (y2 * gy.cuda()).sum().backward()
    assert report('d normals', nrm2.grad, nrm.grad, RTOL, ATOL_FRAC * float(nrm.grad.abs().max()))[0].all()
    assert report('d feature', feat2.grad, feat.grad, RTOL, ATOL_FRAC * float(feat.grad.abs().max()))[0].all()
    for k, p in m.radiance_net.named_parameters():
        ref = rp['radiance_net.' + k].grad
        assert report(f'  d {k}', p.grad, ref, RTOL, ATOL_FRAC * float(ref.abs().max()))[0].all(), k


@pytest.mark.parametrize('white_bkgd', [False, True])
def test_neus_composite_backward_vs_autograd(white_bkgd):
    """NeuSComposite vs autograd through the oracle's sdf_to_alpha / alpha_to_w / sums, with
    gradients on rgb, depth and acc and on the visibility weights."""
    from oracle.neus import alpha_to_w, sdf_to_alpha
    from neurecon_amd import training as T
    torch.manual_seed(5)
    R, S = 300, 128
    sdf = (torch.randn(R, S).cumsum(-1) * 0.05 + 0.3).requires_grad_(True)
    s = torch.tensor([20.0], requires_grad=True)
    rad = torch.rand(R, S - 1, 3).requires_grad_(True)
    dmid = torch.linspace(0.5, 3.0, S - 1).expand(R, S - 1).contiguous()
    g_rgb, g_d, g_a, g_w = torch.randn(R, 3), torch.randn(R), torch.randn(R), torch.randn(R, S - 1) * 0.1
    _, alpha = sdf_to_alpha(sdf, s)
    w = alpha_to_w(alpha)
    rgb = (w[..., None] * rad).sum(-2)
    acc = w.sum(-1)
    depth = (w / (w.sum(-1, keepdim=True) + 1e-10) * dmid).sum(-1)
    if white_bkgd:
        rgb = rgb + (1.0 - acc[..., None])
    ((rgb * g_rgb).sum() + (depth * g_d).sum() + (acc * g_a).sum() + (w * g_w).sum()).backward()
    sdf2 = sdf.detach().cuda().requires_grad_(True)
    s2 = s.detach().cuda().requires_grad_(True)
    rad2 = rad.detach().cuda().requires_grad_(True)
    rgb2, depth2, acc2, w2, _, _ = T.NeuSComposite.apply(sdf2, s2, rad2, dmid.cuda(), white_bkgd)
    assert report('composite rgb', rgb2, rgb.detach(), 1e-5, 1e-6)[0].all()
    assert report('composite depth', depth2, depth.detach(), 1e-5, 1e-6)[0].all()
    ((rgb2 * g_rgb.cuda()).sum() + (depth2 * g_d.cuda()).sum() + (acc2 * g_a.cuda()).sum() +
     (w2 * g_w.cuda()).sum()).backward()
    assert report('d sdf', sdf2.grad, sdf.grad, RTOL, ATOL_FRAC * float(sdf.grad.abs().max()))[0].all()
    assert report('d radiance', rad2.grad, rad.grad, RTOL, ATOL_FRAC * float(rad.grad.abs().max()))[0].all()
    assert report('d s', s2.grad, s.grad, RTOL, 0.0)[0].all()


# ---------------------------------------------------------------------------------------------
# DDP: the gradient all-reduce of train.py:124 over two ranks (gloo: both ranks on the one GPU)
# ---------------------------------------------------------------------------------------------
def _free_port():
    so = socket.socket()
    so.bind(('127.0.0.1', 0))
    p = so.getsockname()[1]
    so.close()
    return p


def _ddp_setup(fw):
    """(model, Trainer class, args, render kwargs, golden) of one framework's 8x8 training fixture"""
    here = os.path.dirname(os.path.abspath(__file__))
    if fw == 'neus':
        from neurecon_amd.frameworks.neus import Trainer
        g = dict(np.load(os.path.join(here, 'golden', 'neus_train.npz')))
        return neus_model(wg.neus_state(seed=1)), Trainer, _args(), _kw(8, 8), g
    if fw == 'volsdf':
        from neurecon_amd.frameworks.volsdf import Trainer
        g = dict(np.load(os.path.join(here, 'golden', 'volsdf_train.npz')))
        args = types.SimpleNamespace(data=types.SimpleNamespace(N_rays=-1),
                                     model=types.SimpleNamespace(obj_bounding_radius=3.0),
                                     training=types.SimpleNamespace(w_eikonal=0.1))
        kw = dict(H=8, W=8, near=0.0, far=6.0, obj_bounding_radius=3.0, batched=True, perturb=False,
                  white_bkgd=False, max_upsample_steps=6, use_nerfplusplus=False, N_samples=64, N_importance=64)
        return volsdf_model(wg.volsdf_state(seed=3, beta_init=0.1), 0.1), Trainer, args, kw, g
    from neurecon_amd.frameworks.unisurf import Trainer
    g = dict(np.load(os.path.join(here, 'golden', 'unisurf_train.npz')))
    args = types.SimpleNamespace(data=types.SimpleNamespace(N_rays=-1),
                                 training=types.SimpleNamespace(w_reg=0.01, perturb_surface_pts=0.01, delta_max=1.0,
                                                                delta_min=0.05, delta_beta=1.5e-5))
    kw = dict(H=8, W=8, batched=True, perturb=False, white_bkgd=False, logit_tau=float(g['logit_tau']),
              radius_of_interest=4.0, N_query=64, N_freespace=32)
    return unisurf_model(wg.unisurf_state(seed=3)), Trainer, args, kw, g


def _ddp_worker(rank, ws, port, q, fw='neus'):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path[:0] = [here, os.path.join(here, 'golden'), os.path.dirname(here)]
    import torch.distributed as dist
    from torch.nn.parallel import DistributedDataParallel as DDP
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=ws)
    try:
        m, Trainer, args, kw, g = _ddp_setup(fw)
        T = lambda a: torch.from_numpy(np.asarray(a)).cuda()
        m.train()
        trainer = DDP(Trainer(m, device_ids=[0]), device_ids=None, find_unused_parameters=False)

        def batch(r):  # per-rank image: the fixture's targets, rolled by rank
            mi = {'intrinsics': T(g['K']), 'c2w': T(g['c2w'])}
            if 'target_mask' in g:
                mi['object_mask'] = T(np.roll(g['target_mask'], 7 * r))
            torch.manual_seed(100 + r)  # the step's random draws (eikonal points, surface perturbation)
            return mi, {'rgb': T(np.roll(g['target_rgb'], 11 * r, axis=1))}
        mi, gt = batch(rank)
        ret = trainer(args, None, mi, gt, kw, 0, device='cuda')
        ret['losses']['total'].mean().backward()
        ddp_grads = {k: p.grad.detach().cpu().clone() for k, p in m.named_parameters() if p.grad is not None}
        if rank == 0:  # single-process reference: mean of both ranks' gradients
            ref = {}
            for r in range(ws):
                m.zero_grad()
                mi, gt = batch(r)
                trainer.module(args, None, mi, gt, kw, 0, device='cuda')['losses']['total'].mean().backward()
                for k, p in m.named_parameters():
                    if p.grad is not None:
                        ref[k] = ref.get(k, 0) + p.grad.detach().cpu() / ws
            worst = max(float((ddp_grads[k] - ref[k]).abs().max() / (ref[k].abs().max() + 1e-30)) for k in ref)
            q.put(('diff', worst))
        q.put(('done', rank))
    except Exception:
        import traceback
        q.put(('error', traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize('fw', ['neus', 'volsdf', 'unisurf'])
def test_ddp_gradient_allreduce_world2(fw):
    """train.py:124's DDP over two ranks (gloo, both on the one GPU): every rank's gradient after the
    all-reduce equals the mean of the two ranks' single-process gradients, for each framework's Trainer"""
    import torch.multiprocessing as mp
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_ddp_worker, args=(r, 2, port, q, fw)) for r in range(2)]
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
    assert not errs, errs[0][1]
    worst = [m[1] for m in msgs if m[0] == 'diff'][0]
    print(f'DDP-averaged vs single-process mean gradient: worst error / scale {worst:.3e}')
    assert worst <= 1e-5


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_radiance_training_strided_feature(precision):
    """A geometry feature handed over as a strided view (h[..., 1:] of a wider tensor, as a caller
    slicing the SDF net's output would) gives the same colours and gradients as a contiguous copy
    (RadianceTG / RadianceFn read raw pointers)."""
    from neurecon_amd import training as T
    m = neus_model(wg.neus_state(seed=2), precision=precision)
    m.train()
    net = m.radiance_net
    torch.manual_seed(0)
    P = 1000
    x, v, nrm = (torch.randn(P, 3, device='cuda') for _ in range(3))
    wide = torch.randn(P, 257, device='cuda')
    outs = []
    for feat in (wide[:, 1:], wide[:, 1:].contiguous()):
        f = feat.detach().requires_grad_(True)
        n = nrm.detach().requires_grad_(True)
        net.zero_grad()
        rgb = T.radiance(net, x, v, n, f)
        (rgb * torch.linspace(0.5, 1.5, 3, device='cuda')).sum().backward()
        outs.append([rgb.detach(), f.grad, n.grad] + [p.grad.clone() for p in net.parameters()])
    assert not wide[:, 1:].is_contiguous()
    for a, b in zip(*outs):
        assert torch.equal(a, b), float((a - b).abs().max())


@pytest.mark.parametrize('name', ['neus_train', 'neus_train_nerfpp'])
def test_blocked_layout_training_step_bit_identical(golden, name, monkeypatch):
    """the f16x3 SDF training path's layer tensors in the 16 x 16 blocked layout (NR_BLK_*, the default
    when P % 16 == 0) give bit-identical losses and gradients to the same step with every tensor
    row-major (NR_TRAIN_BLOCKED=0): only the addressing of the GEMM epilogues and the weight-gradient
    loaders differs"""
    g = golden(name)
    monkeypatch.setenv('NR_TRAIN_BLOCKED', '0')
    _, l_row, g_row, _ = _gpu_step(g, 'f16x3')
    monkeypatch.setenv('NR_TRAIN_BLOCKED', '1')
    _, l_blk, g_blk, _ = _gpu_step(g, 'f16x3')
    for k in l_row:
        assert torch.equal(l_row[k], l_blk[k]), k
    for k in g_row:
        assert torch.equal(g_row[k], g_blk[k]), (k, float((g_row[k] - g_blk[k]).abs().max()))


def test_merged_sample_and_midpoint_evaluation_matches_separate():
    """NeuS training evaluates its samples and mid-points in one SdfNablaTG call (feat_from: the feature
    for the mid-points only): sdf, nablas and features are per point, so they equal the two separate
    evaluations bit for bit; the weight gradients are sums over both point sets either way (checked
    against the oracle by the training-step tests)"""
    from neurecon_amd import training as T
    m = neus_model(wg.neus_state(seed=3), precision='f16x3')
    surf = m.implicit_surface
    if not T.uses_train_gemm(surf):
        pytest.skip('not on the nr_train_gemm path')
    g = torch.Generator().manual_seed(4)
    pts = (torch.rand(4096, 3, generator=g) * 2 - 1).cuda()
    mids = (torch.rand(4064, 3, generator=g) * 2 - 1).cuda()
    with torch.no_grad():
        Ws = T.effective_weights(surf)
        s1, n1, _ = T.sdf_nablas(surf, pts, False, Ws)
        _, n2, f2 = T.sdf_nablas(surf, mids, True, Ws)
        s_all, n_all, f_m = T.sdf_nablas(surf, torch.cat([pts, mids]), True, Ws, feat_from=pts.shape[0])
    torch.cuda.synchronize()
    assert torch.equal(s_all[:4096], s1) and torch.equal(n_all[:4096], n1)
    assert torch.equal(n_all[4096:], n2) and torch.equal(f_m, f2)


def test_radiance_train_fwd32_vs_fp64():
    """nr_radiance_train_fwd32 (RadianceTG's forward: the four ReLU layers chained in registers with exact
    fp32 products over the net's fp32 pack, every hidden activation stored, sigmoid head) against the
    same layers in float64 on 32 k points: hidden activations and rgb within 1e-5 of the tensor scale,
    no further from float64 than torch's fp32 GEMMs (2x + 1e-6), and ReLU masks equal to the fp32
    GEMMs' except where |z| is at fp32 rounding level; the config-(b) net (view embedding 4, normals)."""
    import ctypes
    from neurecon_amd import _lib as L
    from neurecon_amd.base import RadianceNet
    from neurecon_amd.training import _fp32_pack
    torch.manual_seed(3)
    net = RadianceNet(D=4, W=256, W_geo_feat=256, embed_multires=-1, embed_multires_view=4,
                      precision='f16x3').cuda()
    P = 32768
    x = torch.rand(P, 3, device='cuda') * 2 - 1
    v = torch.nn.functional.normalize(torch.randn(P, 3, device='cuda'), dim=-1)
    nrm = torch.randn(P, 3, device='cuda')
    feat = torch.randn(P, 256, device='cuda')
    ns = 3 + 27 + 3
    inp = torch.empty(P, ns + 256, device='cuda')
    L.check(L.lib().nr_radiance_input(L.ptr(x), L.ptr(v), L.ptr(nrm), L.ptr(feat), P, 4, 1, 256, L.ptr(inp),
                                      L.stream_of(x.device)))
    with torch.no_grad():
        Ws = [l.effective_weight() for l in net.layers]
        bs = [l.bias for l in net.layers]
        desc, pk = _fp32_pack(net, Ws, bs, x.device)
        H = [torch.empty(P, 256, device='cuda') for _ in range(4)]
        rgb = torch.empty(P, 3, device='cuda')
        L.check(L.lib().nr_radiance_train_fwd32(ctypes.byref(desc), L.ptr(pk), L.ptr(feat), L.ptr(inp), ns + 256, P,
                                                *[L.ptr(h) for h in H], L.ptr(rgb), L.stream_of(x.device)))
        h64, h32 = inp.double(), inp
        for l in range(4):
            z64 = h64 @ Ws[l].double().t() + bs[l].double()
            z32 = torch.addmm(bs[l], h32, Ws[l].t())
            h64, h32 = z64.clamp_min(0), z32.clamp_min(0)
            scale = float(h64.abs().max())
            e_hip = float((H[l].double() - h64).abs().max())
            e_32 = float((h32.double() - h64).abs().max())
            print(f'h{l}: max |hip - f64| {e_hip / scale:.2e}, |fp32 GEMM - f64| {e_32 / scale:.2e} of {scale:.3e}')
            assert e_hip <= 2 * e_32 + 1e-6 * scale and e_hip <= 1e-5 * scale, l
            flip = (H[l] > 0) != (h32 > 0)
            assert bool((z64.abs()[flip] <= 1e-5 * scale).all()), (l, int(flip.sum()))
        y64 = torch.sigmoid(h64 @ Ws[4].double().t() + bs[4].double())
        assert float((rgb.double() - y64).abs().max()) <= 1e-6


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['fp32', 'f16x3'])
def test_nerf_train32_fwd_bwd_vs_fp64(precision):
    """NeRFFn on nr_nerf_train_fwd32 / nr_nerf_train_bwd32 (the NeRF++ background net of the training
    step, base.py:426-453: one launch each way, exact fp32 products, layers chained in registers) against
    the same net in float64 on 20 000 points (not a multiple of the 128-point tile):
      forward: every stored activation, sigma and rgb within 1e-5 of the tensor scale; the ReLU decisions
        equal float64's except at |z64| <= 1e-5 of the layer scale (fp32 rounding of a z near 0);
      backward: with float64's ReLU decisions pinned to the GPU's (as the 512-ray step test pins them),
        every parameter gradient within 1e-5 (fp32 nets: exact-fp32 weight gradients) / 2e-5 (f16x3 nets:
        f16x3 weight-gradient products) of the tensor's largest entry."""
    from neurecon_amd.base import NeRF
    from neurecon_amd import training as T
    torch.manual_seed(5)
    net = NeRF(D=8, W=256, input_ch=4, input_ch_view=3, multires=10, multires_view=4, output_ch=4, skips=[4],
               use_view_dirs=True, precision=precision).cuda()
    P = 20000
    xe = (torch.rand(P, 84, device='cuda') * 2 - 1)
    ve = (torch.rand(P, 27, device='cuda') * 2 - 1)
    sigma, rgb = T.nerf(net, xe, ve)
    sv = rgb.grad_fn.saved_tensors
    hv_gpu, feat_gpu, H = sv[3], sv[4], sv[5:13]
    layers = list(net.pts_linears) + [net.feature_linear, net.views_linears[0], net.alpha_linear, net.rgb_linear]
    P64 = [p.detach().double().requires_grad_(True) for l in layers for p in (l.weight, l.bias)]

    def ref(masks=None, zs=None):
        W = P64[0::2]
        b = P64[1::2]
        x64, v64 = xe.double(), ve.double()
        h, hs = x64, []
        for i in range(8):
            z = h @ W[i].t() + b[i]
            if zs is not None:
                zs.append(z.detach())
            h = z * masks[i] if masks is not None else z.clamp_min(0)
            hs.append(h)
            if i == 4:
                h = torch.cat([x64, h], -1)
        sig = (h @ W[10].t() + b[10])[:, 0]
        feat = h @ W[8].t() + b[8]
        zv = torch.cat([feat, v64], -1) @ W[9].t() + b[9]
        hv = zv * masks[8] if masks is not None else zv.clamp_min(0)
        return sig, torch.sigmoid(hv @ W[11].t() + b[11]), hs, feat, hv

    zs = []
    with torch.no_grad():
        s64, r64, h64, f64, hv64 = ref(zs=zs)
    for name, a, b in [('sigma', sigma, s64), ('rgb', rgb, r64), ('feature', feat_gpu, f64), ('hv', hv_gpu, hv64)] + \
            [(f'h{i}', H[i], h64[i]) for i in range(8)]:
        sc = float(b.abs().max())
        e = float((a.detach().double() - b).abs().max())
        print(f'{precision} {name}: max |hip - f64| {e / sc:.2e} of {sc:.3e}')
        assert e <= 1e-5 * sc, name
    for i in range(8):
        flip = (H[i] > 0) != (zs[i] > 0)
        zd = float(zs[i].abs()[flip].max()) if bool(flip.any()) else 0.0
        assert zd <= 1e-5 * float(zs[i].abs().max()), (i, int(flip.sum()), zd)
    g_s = torch.randn(P, device='cuda')
    g_r = torch.randn(P, 3, device='cuda')
    net.zero_grad()
    ((sigma * g_s).sum() + (rgb * g_r).sum()).backward()
    masks = [(h > 0).double() for h in H] + [(hv_gpu > 0).double()]
    s64, r64, _, _, _ = ref(masks=masks)
    ((s64 * g_s.double()).sum() + (r64 * g_r.double()).sum()).backward()
    bar = 1e-5 if precision == 'fp32' else 2e-5
    names = [f'{n}.{k}' for n in [f'pts{i}' for i in range(8)] + ['feature', 'views', 'alpha', 'rgb']
             for k in ('weight', 'bias')]
    mine = [p.grad for l in layers for p in (l.weight, l.bias)]
    worst = 0.0
    for name, a, b in zip(names, mine, P64):
        sc = float(b.grad.abs().max()) + 1e-30
        e = float((a.double() - b.grad).abs().max()) / sc
        worst = max(worst, e)
        assert e <= bar, (name, e)
    print(f'{precision}: worst parameter-gradient error {worst:.2e} of the tensor scale')


def test_weight_norm_all_vs_torch():
    """training.weight_norm_all (nr_weight_norm_fwd / _bwd: every layer of a net in one launch each way)
    against torch._weight_norm and its autograd on the training nets' shapes (the SDF net's 9 layers incl.
    the 257-row output layer, the radiance net's 289-wide input layer and 3-row head): weights and the
    weight_v / weight_g gradients within 2e-6 of the tensor scale (fp32 row sums in another order)."""
    from neurecon_amd.base import WNLinear
    from neurecon_amd.training import weight_norm_all
    torch.manual_seed(11)
    shapes = [(39, 256), (256, 256), (256, 217), (256, 256), (256, 257), (289, 256), (256, 3)]
    layers = [WNLinear(i, o).cuda() for i, o in shapes]
    gw = [torch.randn(o, i, device='cuda') for i, o in shapes]
    mine = weight_norm_all(layers)
    sum((w * g).sum() for w, g in zip(mine, gw)).backward()
    got = [(l.weight_v.grad.clone(), l.weight_g.grad.clone()) for l in layers]
    for l in layers:
        l.zero_grad()
    ref = [torch._weight_norm(l.weight_v, l.weight_g, 0) for l in layers]
    sum((w * g).sum() for w, g in zip(ref, gw)).backward()
    for k, (l, a, b, (gv, gg)) in enumerate(zip(layers, mine, ref, got)):
        for name, x, y in (('w', a, b), ('grad_v', gv, l.weight_v.grad), ('grad_g', gg, l.weight_g.grad)):
            sc = float(y.abs().max()) + 1e-30
            e = float((x - y).abs().max()) / sc
            assert e <= 2e-6, (k, name, e)
    # a layer whose weight gets no gradient: zero gradients, not garbage
    w2 = weight_norm_all(layers[:2])
    for l in layers:
        l.zero_grad()
    (w2[0] * gw[0]).sum().backward()
    assert float(layers[1].weight_v.grad.abs().max()) == 0.0 and float(layers[1].weight_g.grad.abs().max()) == 0.0


@pytest.mark.parametrize('weight_decay', [0.0, 1e-2])
def test_adam_matches_torch_adam(weight_decay):
    """neurecon_amd.optim.Adam (nr_adam_step: every tensor in one launch) against torch.optim.Adam's fused
    and default forms over 6 steps on the NeuS nets' tensor shapes (incl. a scalar, a size just past a
    4096-element chunk and > 64 tensors, so two launches), two parameter groups at different lr: every
    parameter and moment within 2e-6 of its scale (fp32, the same update in another rounding order);
    the state_dicts load into each other and the run continues identically."""
    from neurecon_amd.optim import Adam
    torch.manual_seed(5)
    shapes = [(256, 39), (256,), (257, 256), (1,), (), (4097,), (3, 289)] + [(17, 5)] * 60
    init = [torch.randn(s, device='cuda') for s in shapes]
    grads = [[torch.randn(s, device='cuda') for s in shapes] for _ in range(8)]

    def run(make, steps, state=None, start=0):
        ps = [torch.nn.Parameter(t.clone()) for t in init]
        opt = make([{'params': ps[:40], 'lr': 1e-3}, {'params': ps[40:], 'lr': 3e-4}])
        if state is not None:
            for p, q in zip(ps, state[0]):
                p.data.copy_(q)
            opt.load_state_dict(state[1])
        for k in range(start, start + steps):
            for p, g in zip(ps, grads[k]):
                p.grad = g.clone()
            if k % 3 == 2:
                ps[5].grad = None  # a parameter without a gradient this step: untouched
            opt.step()
        return ps, opt

    kw = dict(betas=(0.9, 0.999), eps=1e-8, weight_decay=weight_decay)
    mine, om = run(lambda g: Adam(g, **kw), 6)
    for ref_kw in (dict(fused=True), dict(foreach=False)):
        ref, orf = run(lambda g: torch.optim.Adam(g, **kw, **ref_kw), 6)
        for i, (a, b) in enumerate(zip(mine, ref)):
            sa, sb = om.state[a], orf.state[b]
            assert float(sa['step']) == float(sb['step']), i
            for x, y in ((a, b), (sa['exp_avg'], sb['exp_avg']), (sa['exp_avg_sq'], sb['exp_avg_sq'])):
                sc = float(y.abs().max()) + 1e-30
                assert float((x - y).abs().max()) / sc <= 2e-6, (ref_kw, i)
    # checkpoint interchange: torch's state continues on nr_adam_step and vice versa
    # (deep copies: load_state_dict keeps tensors already on the parameter's device and dtype by reference)
    import copy
    ref, orf = run(lambda g: torch.optim.Adam(g, **kw), 4)
    a, _ = run(lambda g: Adam(g, **kw), 2, state=([p.detach() for p in ref], copy.deepcopy(orf.state_dict())), start=4)
    b, _ = run(lambda g: torch.optim.Adam(g, **kw), 2, state=([p.detach() for p in ref], copy.deepcopy(orf.state_dict())),
               start=4)
    for x, y in zip(a, b):
        assert float((x - y).abs().max()) / (float(y.abs().max()) + 1e-30) <= 2e-6
    # ... and the other way: nr_adam_step's state continues on torch.optim.Adam
    ref, orm = run(lambda g: Adam(g, **kw), 4)
    sd = orm.state_dict()
    assert sd['param_groups'][0].keys() == torch.optim.Adam(ref[:1]).state_dict()['param_groups'][0].keys()
    a, _ = run(lambda g: torch.optim.Adam(g, **kw), 2, state=([p.detach() for p in ref], copy.deepcopy(sd)), start=4)
    b, _ = run(lambda g: Adam(g, **kw), 2, state=([p.detach() for p in ref], copy.deepcopy(sd)), start=4)
    for x, y in zip(a, b):
        assert float((x - y).abs().max()) / (float(y.abs().max()) + 1e-30) <= 2e-6
    # the launch writes through raw pointers: every updated tensor's version counter moves, as with torch's
    # in-place update (the packed-weight caches are keyed on it)
    v0 = [p._version for p in mine]
    for p, g in zip(mine, grads[7]):
        p.grad = g.clone()
    om.step()
    assert all(p._version > v for p, v in zip(mine, v0))
    with pytest.raises(NotImplementedError):
        Adam(mine, amsgrad=True)


@pytest.mark.parametrize('precision', ['f16x3', 'fp32'])
def test_neus_training_with_nr_adam_matches_torch_adam(golden, precision):
    """Three NeuS training steps (Trainer.forward + backward + optimizer step, fixed rays) with
    neurecon_amd.optim.Adam against the same steps with torch.optim.Adam: every step's loss and the
    parameters after it agree within the two updates' rounding.  Pins that the packed-weight caches
    (render pack of the no-grad sampler, training pack, fp32 packs; keyed on the parameters' version
    counters) follow nr_adam_step's raw-pointer update: with stale packs the second and third steps'
    losses would be computed from the step-0 weights."""
    from neurecon_amd.frameworks.neus import Trainer
    from neurecon_amd.optim import Adam
    g = golden('neus_train')
    H, W = int(g['H']), int(g['W'])
    T = lambda a: torch.from_numpy(np.asarray(a)).cuda()
    results = []
    for make in (lambda ps: torch.optim.Adam(ps, lr=1e-3), lambda ps: Adam(ps, lr=1e-3)):
        m = neus_model(wg.neus_state(seed=int(g['seed'])), precision=precision)
        m.train()
        trainer = Trainer(m, device_ids=[0])
        opt = make(list(m.parameters()))
        losses = []
        for it in range(3):
            opt.zero_grad(set_to_none=True)
            ret = trainer.forward(_args(), None, {'intrinsics': T(g['K']), 'c2w': T(g['c2w']),
                                                  'object_mask': T(g['target_mask'])},
                                  {'rgb': T(g['target_rgb'])}, _kw(H, W), it, device='cuda')
            loss = torch.mean(ret['losses']['total'])
            loss.backward()
            opt.step()
            losses.append(float(loss))
        torch.cuda.synchronize()
        results.append((losses, [p.detach().clone() for p in m.parameters()]))
    (l_ref, p_ref), (l_nr, p_nr) = results
    print(precision, 'losses torch', l_ref, 'nr_adam', l_nr)
    # the steps must move the loss by far more than the tolerance, or the check would not see stale packs
    assert min(abs(l_ref[1] - l_ref[0]), abs(l_ref[2] - l_ref[1])) > 1e-3 * abs(l_ref[0]), l_ref
    for a, b in zip(l_nr, l_ref):
        assert abs(a - b) <= 2e-5 * abs(b), (l_nr, l_ref)
    # parameters: Adam moves an element by ~lr per step whatever its gradient's size, so an element whose
    # gradient is within rounding of 0 can step the other way in one run (a 2 lr difference); the bar:
    # at most 0.1 % of a tensor's elements more than 2 % of the largest displacement (3 lr) apart, and
    # 0.1 % of it on average
    lr, steps = 1e-3, 3
    for a, b in zip(p_nr, p_ref):
        d = (a - b).abs()
        far = int((d > 0.02 * lr * steps).sum())
        assert far <= max(1, 1e-3 * d.numel()) and float(d.mean()) <= 1e-3 * lr * steps, \
            (far, d.numel(), float(d.max()), float(d.mean()))
