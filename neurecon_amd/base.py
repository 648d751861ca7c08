"""Network modules of the render path, state_dict-compatible with the reference (models/base.py).

Parameters keep the reference's names and shapes so reference checkpoints load unchanged
(weight_norm'ed layers store `weight_g [out,1]`, `weight_v [out,in]`, `bias [out]`;
ImplicitSurface has the `obj_bounding_size` buffer).  Forward passes run on the HIP kernels of
libnrhip.so (render mode, no autograd graph); there is no PyTorch/CPU compute fallback.
"""
import math

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _lib as L


# ---------------------------------------------------------------------------------------------
# positional encoding (models/base.py:14-81) -- API object; the kernels fuse it themselves
# ---------------------------------------------------------------------------------------------
class Embedder(nn.Module):
    def __init__(self, input_dim, max_freq_log2, N_freqs, log_sampling=True, include_input=True,
                 periodic_fns=(torch.sin, torch.cos)):
        super().__init__()
        self.input_dim = input_dim
        self.include_input = include_input
        self.periodic_fns = periodic_fns
        self.out_dim = (input_dim if include_input else 0) + input_dim * N_freqs * len(periodic_fns)
        bands = 2. ** torch.linspace(0., max_freq_log2, N_freqs) if log_sampling else \
            torch.linspace(2. ** 0., 2. ** max_freq_log2, N_freqs)
        self.freq_bands = bands.numpy().tolist()

    def forward(self, x):
        assert x.shape[-1] == self.input_dim
        parts = [x] if self.include_input else []
        for f in self.freq_bands:
            parts.extend(fn(x * f) for fn in self.periodic_fns)
        return torch.cat(parts, dim=-1)


def get_embedder(multires, input_dim=3):
    if multires < 0:
        return nn.Identity(), input_dim
    e = Embedder(input_dim, multires - 1, multires)
    return e, e.out_dim


# ---------------------------------------------------------------------------------------------
# layers
# ---------------------------------------------------------------------------------------------
class WNLinear(nn.Module):
    """Linear layer under nn.utils.weight_norm(dim=0): W = g * v / ||v||_row (base.py:226-227).
    Stores exactly the parameters weight_norm leaves on the module: weight_g, weight_v, bias."""

    def __init__(self, in_dim, out_dim, weight=None, bias=None):
        super().__init__()
        self.in_features, self.out_features = in_dim, out_dim
        if weight is None:  # nn.Linear's default init
            weight = torch.empty(out_dim, in_dim)
            nn.init.kaiming_uniform_(weight, a=math.sqrt(5))
        if bias is None:
            k = 1.0 / math.sqrt(in_dim)
            bias = torch.empty(out_dim).uniform_(-k, k)
        self.weight_v = nn.Parameter(weight.clone())
        self.weight_g = nn.Parameter(torch.norm_except_dim(weight, 2, 0).clone())
        self.bias = nn.Parameter(bias.clone())

    def effective_weight(self):
        return torch._weight_norm(self.weight_v, self.weight_g, 0)


def _siren_init(in_dim, out_dim, is_first, w0=30.0, c=6.0):
    """SirenLayer.reset_parameters (base.py:98-106): nn.Linear's init, then
    weight ~ U(-w_std, w_std), w_std = 1/in (first layer) or sqrt(c/in)/w0; bias keeps Linear's init."""
    w = torch.empty(out_dim, in_dim)
    nn.init.kaiming_uniform_(w, a=math.sqrt(5))
    k = 1.0 / math.sqrt(in_dim)
    b = torch.empty(out_dim).uniform_(-k, k)
    w_std = (1 / in_dim) if is_first else (math.sqrt(c / in_dim) / w0)
    w.uniform_(-w_std, w_std)
    return w, b


PRECISIONS = ('f16x3', 'fp32')


def default_precision():
    """GEMM arithmetic of the MLP kernels: 'f16x3' (default; split-fp16 x3 on fp16 MFMA, per-point
    power-of-two scaling -- measured at fp32-level error on the parity suite) or 'fp32' (fp32 MFMA).
    Override with NR_PRECISION or the modules' `precision=` argument."""
    import os
    p = os.environ.get('NR_PRECISION', 'f16x3')
    if p not in PRECISIONS:
        raise ValueError(f'NR_PRECISION must be one of {PRECISIONS}')
    return p


def _wn_params(layers):
    Ws, bs = [], []
    for layer in layers:
        Ws.append(layer.effective_weight().detach().float().contiguous())
        bs.append(layer.bias.detach().float().contiguous())
    return Ws, bs


_PARAM_ATTRS = ('weight_v', 'weight_g', 'weight', 'bias')


def _version_key(module, precision, device):
    """Identity of the weights a packed copy was made from: (storage, version) of every layer tensor.
    Read from the layers' attributes rather than module.parameters(): an nn.DataParallel replica
    (neus.py:413-414) holds its broadcast copies as plain attributes and has no parameters, so its key
    names its own copies and a pack made on one device is never served to another."""
    key = [str(device), precision]
    for m in module.modules():
        for name in _PARAM_ATTRS:
            t = m.__dict__.get(name, None)
            if t is None:
                t = m._parameters.get(name, None)
            if isinstance(t, torch.Tensor):
                key.append((t.data_ptr(), t._version))
    return tuple(key)


def _ptr_array(ts):
    arr = (ctypes_void_p * len(ts))(*[t.data_ptr() for t in ts])
    return arr


import ctypes  # noqa: E402
ctypes_void_p = ctypes.c_void_p


def wants_graph(*tensors_or_modules):
    """True when the call must build an autograd graph (grad mode and a parameter that needs grad)."""
    if not torch.is_grad_enabled():
        return False
    for m in tensors_or_modules:
        ps = m.parameters() if isinstance(m, nn.Module) else [m]
        if any(getattr(p, 'requires_grad', False) for p in ps):
            return True
    return False


def _no_training(*tensors_or_modules, what='this call'):
    if wants_graph(*tensors_or_modules):
        raise NotImplementedError(
            f'neurecon_amd: {what} has no native training (autograd) path; wrap it in torch.no_grad() '
            '(training runs through the NeuS / SDF / radiance autograd functions of neurecon_amd.training)')


def check_view_dirs(model, use_view_dirs):
    """View-direction independence is a property of the radiance net (RadianceNet(use_view_dirs=False),
    config key model.radiance.use_view_dirs, base.py:334-338, :383-384): the kernels then ignore the
    ray directions they are handed.  The render-level flag volume_render(use_view_dirs=False) hands
    view_dirs=None to batchify_query, which fails in the reference (train_util.py:27 flattens every
    argument; neus.py:298, volsdf.py:450, unisurf.py:214), so it raises here too."""
    if not use_view_dirs:
        raise ValueError('volume_render(use_view_dirs=False) fails in the reference (batchify_query flattens the '
                         'None view dirs, train_util.py:27); build the RadianceNet with use_view_dirs=False '
                         '(model.radiance.use_view_dirs) to drop the view dependence')


# ---------------------------------------------------------------------------------------------
# ImplicitSurface (models/base.py:131-282)
# ---------------------------------------------------------------------------------------------
class ImplicitSurface(nn.Module):
    def __init__(self, W=256, D=8, skips=[4], W_geo_feat=256, input_ch=3, radius_init=1.0, obj_bounding_size=2.0,
                 geometric_init=True, embed_multires=6, weight_norm=True, use_siren=False, precision=None):
        super().__init__()
        if not weight_norm:
            raise NotImplementedError('neurecon_amd: non-weight-normed surface nets are out of scope')
        self.radius_init = radius_init
        self.register_buffer('obj_bounding_size', torch.tensor([obj_bounding_size]).float())
        self.geometric_init = geometric_init
        self.D, self.W, self.W_geo_feat, self.skips = D, W, W_geo_feat, list(skips)
        self.use_siren = bool(use_siren)
        if use_siren:  # base.py:170-172
            assert len(skips) == 0, 'do not use skips for siren'
            self.register_buffer('is_pretrained', torch.tensor([False], dtype=torch.bool))
        self.embed_multires = embed_multires
        self.embed_fn, in_ch = get_embedder(embed_multires)
        self.input_ch = in_ch
        self.precision = default_precision() if precision is None else precision
        layers = []
        for l in range(D + 1):
            if l == D:
                out_dim = 1 + W_geo_feat if W_geo_feat > 0 else 1
            elif (l + 1) in self.skips:
                out_dim = W - in_ch
            else:
                out_dim = W
            in_dim = in_ch if l == 0 else W
            w = torch.empty(out_dim, in_dim)
            b = torch.empty(out_dim)
            if use_siren and l != D:  # SirenLayer (base.py:194-196)
                layers.append(WNLinear(in_dim, out_dim, *_siren_init(in_dim, out_dim, l == 0)))
            elif geometric_init and not use_siren:  # SAL / IDR sphere init (base.py:207-224)
                if l == D:
                    nn.init.normal_(w, mean=np.sqrt(np.pi) / np.sqrt(in_dim), std=0.0001)
                    nn.init.constant_(b, -radius_init)
                elif embed_multires > 0 and l == 0:
                    nn.init.constant_(b, 0.0)
                    nn.init.constant_(w[:, 3:], 0.0)
                    nn.init.normal_(w[:, :3], 0.0, np.sqrt(2) / np.sqrt(out_dim))
                elif embed_multires > 0 and l in self.skips:
                    nn.init.constant_(b, 0.0)
                    nn.init.normal_(w, 0.0, np.sqrt(2) / np.sqrt(out_dim))
                    nn.init.constant_(w[:, -(in_ch - 3):], 0.0)
                else:
                    nn.init.constant_(b, 0.0)
                    nn.init.normal_(w, 0.0, np.sqrt(2) / np.sqrt(out_dim))
                layers.append(WNLinear(in_dim, out_dim, w, b))
            else:
                layers.append(WNLinear(in_dim, out_dim))
        self.surface_fc_layers = nn.ModuleList(layers)
        self._nr_cache = None

    # -- native plumbing ----------------------------------------------------------------------
    def nr_desc(self):
        prec = L.PREC_FP32 if self.precision == 'fp32' else L.PREC_F16X3
        if self.use_siren:
            return L.NrSdfDesc(self.D, self.W, -1, self.embed_multires, self.W_geo_feat, prec, 1)
        if len(self.skips) != 1:
            raise NotImplementedError('neurecon_amd: SDF nets with exactly one skip layer are supported')
        return L.NrSdfDesc(self.D, self.W, self.skips[0], self.embed_multires, self.W_geo_feat, prec, 0)

    def nr_packed(self, device):
        """Effective weights folded (weight_norm) and packed into the kernel layout; cached until a
        parameter changes (tensor version counter)."""
        key = _version_key(self, self.precision, device)
        if self._nr_cache is not None and self._nr_cache[0] == key:
            return self._nr_cache[1], self._nr_cache[2]
        lib = L.lib()
        desc = self.nr_desc()
        nbytes = lib.nr_sdf_packed_bytes(ctypes.byref(desc))
        if nbytes == 0:
            raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
        with torch.no_grad():
            Ws, bs = _wn_params(self.surface_fc_layers)
            Ws = [w.to(device) for w in Ws]
            bs = [b.to(device) for b in bs]
            packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
            L.check(lib.nr_sdf_pack(ctypes.byref(desc), _ptr_array(Ws), _ptr_array(bs), L.ptr(packed),
                                    L.stream_of(device)))
        self._nr_cache = (key, desc, packed, Ws, bs)  # keep sources alive until the pack ran
        return desc, packed

    def _run(self, x, nabla, feature):
        L.require_gpu(x, 'points')
        shape = x.shape[:-1]
        if wants_graph(self):  # training: differentiable sdf / nablas / feature (double backward)
            from .training import sdf_nablas
            sdf, nab, feat = sdf_nablas(self, x, True)
            return [sdf.reshape(shape), nab.reshape(*shape, 3), feat.reshape(*shape, self.W_geo_feat)]
        pts = x.reshape(-1, 3).float().contiguous()
        P = pts.shape[0]
        dev = pts.device
        desc, packed = self.nr_packed(dev)
        sdf = torch.empty(P, device=dev)
        nab = torch.empty(P, 3, device=dev) if nabla else None
        feat = torch.empty(P, self.W_geo_feat, device=dev) if feature else None
        lib = L.lib()
        ws_bytes = lib.nr_mlp_workspace_bytes(1 if nabla else 0)
        ws = torch.empty(max(ws_bytes, 1), dtype=torch.uint8, device=dev)
        L.check(lib.nr_sdf_forward(ctypes.byref(desc), L.ptr(packed), L.ptr(pts), P, L.ptr(sdf), L.ptr(nab),
                                   L.ptr(feat), L.ptr(ws), ws_bytes, L.stream_of(dev)))
        out = [sdf.reshape(shape)]
        out.append(None if nab is None else nab.reshape(*shape, 3))
        out.append(None if feat is None else feat.reshape(*shape, self.W_geo_feat))
        return out

    # -- reference API ------------------------------------------------------------------------
    def forward(self, x, return_h=False):
        """base.py:243-263 (render mode)."""
        sdf, _, h = self._run(x, nabla=False, feature=return_h)
        return (sdf, h) if return_h else sdf

    def forward_with_nablas(self, x, has_grad_bypass=None):
        """base.py:265-282: (sdf, d sdf/d x, geometry feature); no graph is built."""
        sdf, nab, h = self._run(x, nabla=True, feature=True)
        return sdf, nab, h

    def pretrain_hook(self, configs={}):
        """base.py:226-233: a geometric-init SIREN net is pretrained to a sphere once (is_pretrained)."""
        configs['target_radius'] = self.radius_init
        configs['obj_bounding_size'] = float(self.obj_bounding_size.reshape(-1)[0])
        if self.geometric_init and self.use_siren and not bool(self.is_pretrained):
            pretrain_siren_sdf(self, **configs)
            self.is_pretrained = ~self.is_pretrained
            return True
        return False


def pretrain_siren_sdf(implicit_surface, num_iters=5000, lr=1.0e-4, batch_points=5000, target_radius=0.5,
                       obj_bounding_size=3.0, logger=None):
    """base.py:284-310: fit the SIREN SDF to |x| - target_radius (L1, Adam) on uniform points in the
    bounding cube, drawn on the CPU as the reference does; the forward and its gradient run on the
    training path's HIP kernels and hipBLASLt GEMMs (neurecon_amd.training)."""
    from torch import optim
    device = next(implicit_surface.parameters()).device
    optimizer = optim.Adam(implicit_surface.parameters(), lr=lr)
    with torch.enable_grad():
        for it in range(num_iters):
            pts = torch.empty([batch_points, 3]).uniform_(-obj_bounding_size, obj_bounding_size).float().to(device)
            sdf_gt = pts.norm(dim=-1) - target_radius
            sdf_pred = implicit_surface.forward(pts)
            loss = F.l1_loss(sdf_pred, sdf_gt, reduction='mean')
            optimizer.zero_grad()
            loss.backward()
            optimizer.step()
            if logger is not None:
                logger.add('pretrain_siren', 'loss_l1', loss.item(), it)


# ---------------------------------------------------------------------------------------------
# RadianceNet (models/base.py:312-391)
# ---------------------------------------------------------------------------------------------
class RadianceNet(nn.Module):
    """RadianceNet (base.py:312-391)."""

    def __init__(self, D=4, W=256, skips=[], W_geo_feat=256, embed_multires=6, embed_multires_view=4,
                 use_view_dirs=True, weight_norm=True, use_siren=False, precision=None):
        super().__init__()
        if not weight_norm or skips:
            raise NotImplementedError('neurecon_amd: RadianceNet needs weight_norm and no skips')
        self.D, self.W, self.skips, self.use_view_dirs = D, W, list(skips), bool(use_view_dirs)
        self.use_siren = bool(use_siren)
        self.embed_multires, self.embed_multires_view, self.W_geo_feat = embed_multires, embed_multires_view, W_geo_feat
        self.embed_fn, ch_pts = get_embedder(embed_multires)
        if use_view_dirs:  # base.py:334-338: without view dirs the input is cat([embed(x), feature])
            self.embed_fn_view, ch_view = get_embedder(embed_multires_view)
            in0 = ch_pts + ch_view + 3 + W_geo_feat
        else:
            in0 = ch_pts + W_geo_feat
        self.precision = default_precision() if precision is None else precision
        # hidden layers: DenseLayer(ReLU) or SirenLayer (base.py:357-361); head: DenseLayer(Sigmoid)
        self.layers = nn.ModuleList([
            WNLinear(in0 if l == 0 else W, W, *_siren_init(in0 if l == 0 else W, W, l == 0))
            if use_siren and l != D else WNLinear(in0 if l == 0 else W, 3 if l == D else W) for l in range(D + 1)])
        self._nr_cache = None

    def nr_desc(self):
        return L.NrRadDesc(self.D, self.W, self.embed_multires, self.embed_multires_view, self.W_geo_feat,
                           L.PREC_FP32 if self.precision == 'fp32' else L.PREC_F16X3, 0 if self.use_view_dirs else 1,
                           1 if self.use_siren else 0)

    def nr_packed(self, device):
        key = _version_key(self, self.precision, device)
        if self._nr_cache is not None and self._nr_cache[0] == key:
            return self._nr_cache[1], self._nr_cache[2]
        lib = L.lib()
        desc = self.nr_desc()
        nbytes = lib.nr_radiance_packed_bytes(ctypes.byref(desc))
        if nbytes == 0:
            raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
        with torch.no_grad():
            Ws, bs = _wn_params(self.layers)
            Ws = [w.to(device) for w in Ws]
            bs = [b.to(device) for b in bs]
            packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
            L.check(lib.nr_radiance_pack(ctypes.byref(desc), _ptr_array(Ws), _ptr_array(bs), L.ptr(packed),
                                         L.stream_of(device)))
        self._nr_cache = (key, desc, packed, Ws, bs)
        return desc, packed

    def forward(self, x, view_dirs, normals, geometry_feature):
        """base.py:372-391 (render mode; with a graph when training)."""
        L.require_gpu(x, 'points')
        shape = x.shape[:-1]
        P = x.reshape(-1, 3).shape[0]
        if self.use_view_dirs:
            if view_dirs is None:  # the reference fails in embed_fn_view / torch.cat here
                raise TypeError('RadianceNet(use_view_dirs=True) needs view_dirs')
            v = view_dirs.reshape(-1, 3).float().contiguous()
            if v.shape[0] != P:
                raise ValueError('view_dirs must have one direction per point')
            n = normals.reshape(-1, 3).float().contiguous()
        else:  # view dirs and normals are not inputs (base.py:383-384)
            v = n = None
        if wants_graph(self, normals, geometry_feature):
            from .training import radiance
            rgb = radiance(self, x.reshape(-1, 3).float(), v, n, geometry_feature.reshape(-1, self.W_geo_feat).float())
            return rgb.reshape(*shape, 3)
        dev = x.device
        xs = x.reshape(-1, 3).float().contiguous()
        f = geometry_feature.reshape(-1, self.W_geo_feat).float().contiguous()
        desc, packed = self.nr_packed(dev)
        rgb = torch.empty(P, 3, device=dev)
        L.check(L.lib().nr_radiance_forward(ctypes.byref(desc), L.ptr(packed), L.ptr(xs), L.ptr(v), 1, L.ptr(n),
                                            L.ptr(f), P, L.ptr(rgb), L.stream_of(dev)))
        return rgb.reshape(*shape, 3)


# ---------------------------------------------------------------------------------------------
# NeRF++ background (models/base.py:395-453)
# ---------------------------------------------------------------------------------------------
class NeRF(nn.Module):
    def __init__(self, D=8, W=256, input_ch=3, input_ch_view=3, multires=-1, multires_view=-1, output_ch=4,
                 skips=[4], use_view_dirs=False, precision=None):
        super().__init__()
        self.D, self.W, self.skips, self.use_view_dirs = D, W, list(skips), use_view_dirs
        self.multires, self.multires_view, self.input_ch_raw = multires, multires_view, input_ch
        self.embed_fn, input_ch = get_embedder(multires, input_dim=input_ch)
        self.embed_fn_view, input_ch_view = get_embedder(multires_view, input_dim=input_ch_view)
        self.pts_linears = nn.ModuleList(
            [nn.Linear(input_ch, W)] + [nn.Linear(W + input_ch if i in self.skips else W, W) for i in range(D - 1)])
        self.views_linears = nn.ModuleList([nn.Linear(input_ch_view + W, W // 2)])
        if use_view_dirs:
            self.feature_linear = nn.Linear(W, W)
            self.alpha_linear = nn.Linear(W, 1)
            self.rgb_linear = nn.Linear(W // 2, 3)
        else:
            self.output_linear = nn.Linear(W, output_ch)
        self.precision = default_precision() if precision is None else precision
        self._nr_cache = None

    def nr_desc(self):
        if not self.use_view_dirs or len(self.skips) != 1:
            raise NotImplementedError('neurecon_amd: only the NeRF++ background configuration is native')
        return L.NrNerfDesc(self.D, self.W, self.skips[0], self.input_ch_raw, self.multires, self.multires_view,
                            L.PREC_FP32 if self.precision == 'fp32' else L.PREC_F16X3)

    def nr_packed(self, device):
        key = _version_key(self, self.precision, device)
        if self._nr_cache is not None and self._nr_cache[0] == key:
            return self._nr_cache[1], self._nr_cache[2]
        lib = L.lib()
        desc = self.nr_desc()
        nbytes = lib.nr_nerf_packed_bytes(ctypes.byref(desc))
        if nbytes == 0:
            raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
        layers = list(self.pts_linears) + [self.feature_linear, self.views_linears[0], self.alpha_linear,
                                           self.rgb_linear]
        with torch.no_grad():
            Ws = [l.weight.detach().float().contiguous().to(device) for l in layers]
            bs = [l.bias.detach().float().contiguous().to(device) for l in layers]
            packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
            L.check(lib.nr_nerf_pack(ctypes.byref(desc), _ptr_array(Ws), _ptr_array(bs), L.ptr(packed),
                                     L.stream_of(device)))
        self._nr_cache = (key, desc, packed, Ws, bs)
        return desc, packed

    def forward(self, input_pts, input_views):
        """base.py:426-453 (render mode): returns (sigma [...], rgb [..., 3])."""
        L.require_gpu(input_pts, 'points')
        _no_training(self, what='the NeRF++ background net')
        shape = input_pts.shape[:-1]
        dev = input_pts.device
        x = input_pts.reshape(-1, 4).float().contiguous()
        P = x.shape[0]
        v = input_views.reshape(-1, 3).float().contiguous()
        if v.shape[0] != P:
            raise ValueError('input_views must have one direction per point')
        desc, packed = self.nr_packed(dev)
        sigma = torch.empty(P, device=dev)
        rgb = torch.empty(P, 3, device=dev)
        L.check(L.lib().nr_nerf_forward(ctypes.byref(desc), L.ptr(packed), L.ptr(x), L.ptr(v), 1, P, L.ptr(sigma),
                                        L.ptr(rgb), L.stream_of(dev)))
        return sigma.reshape(shape), rgb.reshape(*shape, 3)
