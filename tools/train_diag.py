"""Gradient error of the NeuS training step per parameter tensor, by which nets train on nr_train_gemm.

    python tools/train_diag.py [golden name]

Variants: fp32 (hipBLASLt fp32 GEMMs), f16x3 with both nets on the f16x3 training GEMMs, and f16x3
with one of the two nets moved back to the fp32 GEMMs -- isolates which GEMM chain an error comes from.
Error = max |grad - oracle| / max |oracle| per tensor (oracle on the GPU's sample depths)."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests'), os.path.join(ROOT, 'tests', 'golden')]

import test_gpu_train as T  # noqa: E402
from neurecon_amd import training  # noqa: E402


def golden(name):
    return dict(np.load(os.path.join(ROOT, 'tests', 'golden', name + '.npz')))


def run(g, precision, tg_filter):
    orig = training.uses_train_gemm
    training.uses_train_gemm = lambda m: orig(m) and tg_filter(m)
    try:
        m, losses, grads, _ = T._gpu_step(g, precision)
        d_all = T._gpu_sample_depths(m, g)
    finally:
        training.uses_train_gemm = orig
    _, ref, _ = T.train_grads_oracle(g, d_all=d_all)
    out = {}
    for k, r in ref.items():
        if k not in grads:
            continue
        r = r.detach().double().cpu()
        e = (grads[k].double() - r).abs()
        sc = float(r.abs().max()) + 1e-30
        ok = e <= 1e-4 * r.abs() + 1e-5 * sc
        out[k] = (float(e.max()) / sc, float(ok.double().mean()))
    return out


def radiance_probe(g):
    """inputs, rgb and incoming gradient of the radiance net in the f16x3 step with the radiance net on
    the training GEMM and on the fp32 GEMMs (the SDF net on the training GEMM in both): the radiance
    parameter gradients vs a float64 autograd of RadianceNet on the recorded inputs"""
    orig_rad, orig_use = training.radiance, training.uses_train_gemm
    recs = {}
    for tag, use_tg in (('tg', True), ('fp32', False)):
        rec = {}

        def rad(net, x, v, nrm, feat, rec=rec):
            rec['in'] = [t.detach().clone() if t is not None else None for t in (x, v, nrm, feat)]
            rec['net'] = net
            y = orig_rad(net, x, v, nrm, feat)
            rec['y'] = y.detach().clone()
            y.register_hook(lambda gy: rec.__setitem__('gy', gy.detach().clone()))
            return y
        training.radiance = rad
        training.uses_train_gemm = lambda m, u=use_tg: orig_use(m) and (hasattr(m, 'surface_fc_layers') or u)
        try:
            m, _, grads, _ = T._gpu_step(g, 'f16x3')
        finally:
            training.radiance, training.uses_train_gemm = orig_rad, orig_use
        rec['grads'] = {k: v for k, v in grads.items() if k.startswith('radiance_net')}
        recs[tag] = rec
    a, b = recs['tg'], recs['fp32']
    for i, n in enumerate(('x', 'v', 'nrm', 'feat')):
        if a['in'][i] is not None:
            print(f'input {n}: max |tg - fp32| {float((a["in"][i] - b["in"][i]).abs().max()):.3e}')
    print(f'rgb: max |tg - fp32| {float((a["y"] - b["y"]).abs().max()):.3e}')
    print(f'gy:  max |tg - fp32| {float((a["gy"] - b["gy"]).abs().max()):.3e} (max |gy| {float(b["gy"].abs().max()):.3e})')
    # float64 autograd of the radiance net (base.py:372-391) on the recorded inputs and gy
    net = a['net']
    x, v, nrm, feat = [t.double() if t is not None else None for t in a['in']]
    from neurecon_amd import rend_util  # noqa: F401
    Ws = [l.effective_weight().detach().double().requires_grad_() for l in net.layers]
    bs = [l.bias.detach().double().requires_grad_() for l in net.layers]
    nf = net.embed_multires_view
    emb = [v]
    for k in range(nf):
        for fn in (torch.sin, torch.cos):
            emb.append(fn(v * 2.0 ** k))
    h = torch.cat([x, torch.cat(emb, -1), nrm, feat], -1)
    for l in range(4):
        h = torch.relu(h @ Ws[l].t() + bs[l])
    y = torch.sigmoid(h @ Ws[4].t() + bs[4])
    for tag, rec in recs.items():
        gW = torch.autograd.grad(y, Ws + bs, rec['gy'].double(), retain_graph=True)
        for l in range(5):
            for kind, gr in (('bias', gW[5 + l]),):
                mine = rec['grads'][f'radiance_net.layers.{l}.bias'].double().to(gr.device)
                print(f'{tag:5s} layer {l} bias: max err / max {float((mine - gr).abs().max() / gr.abs().max()):.3e}')


def main(name='neus_train'):
    g = golden(name)
    torch.set_num_threads(16)
    variants = {'fp32': ('fp32', lambda m: True), 'f16x3 both': ('f16x3', lambda m: True),
                'f16x3 sdf only': ('f16x3', lambda m: hasattr(m, 'surface_fc_layers')),
                'f16x3 radiance only': ('f16x3', lambda m: not hasattr(m, 'surface_fc_layers'))}
    res = {v: run(g, *a) for v, a in variants.items()}
    keys = list(res['fp32'])
    print(f'{"tensor":48s} ' + ' '.join(f'{v:>22s}' for v in res))
    for k in keys:
        print(f'{k:48s} ' + ' '.join(f'{res[v][k][0]:10.2e} {100 * res[v][k][1]:9.2f}%' for v in res))


if __name__ == '__main__':
    if len(sys.argv) > 1 and sys.argv[1] == '--probe':
        radiance_probe(golden(sys.argv[2] if len(sys.argv) > 2 else 'neus_train'))
    else:
        main(*sys.argv[1:])
