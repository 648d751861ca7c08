"""Deterministic synthetic weights for parity fixtures (numpy legacy RandomState => stable stream).

The fixtures under tests/golden/ store only inputs and outputs; the weights are rebuilt from a
seed by this module, both by the generator script (which loads them into the reference models)
and by the tests (which load them into the oracle and into neurecon_amd).  Shapes and state_dict
key names follow the reference's module trees:

  ImplicitSurface  models/base.py:131-231   (surface_fc_layers.{l}.{weight_g,weight_v,bias}, obj_bounding_size)
  RadianceNet      models/base.py:312-370   (layers.{l}.{weight_g,weight_v,bias})
  NeRF             models/base.py:395-424   (pts_linears.*, views_linears.0, feature/alpha/rgb_linear)
  NeuS             models/frameworks/neus.py:72-101   (ln_s)
  VolSDF           models/frameworks/volsdf.py:274-304 (ln_beta)
  UNISURF          models/frameworks/unisurf.py:16-32

Values are geometric-init-like (SAL/IDR sphere init, base.py:207-224) so that rays hit a
sphere-ish surface, but every weight is non-zero and weight_g != ||weight_v|| so that the
embedding octaves and the weight-norm fold are exercised.
"""
import math
import numpy as np
import torch


def _wn_layer(rs, out_dim, in_dim, std, mean=0.0, bstd=0.01, bias=None, small_cols=None, small_std=None):
    v = rs.normal(mean, std, size=(out_dim, in_dim))
    if small_cols is not None:
        v[:, small_cols] = rs.normal(0.0, small_std, size=(out_dim, len(range(in_dim)[small_cols])))
    nrm = np.linalg.norm(v, axis=1, keepdims=True)
    g = nrm * (1.0 + 0.05 * rs.uniform(-1.0, 1.0, size=(out_dim, 1)))
    b = rs.normal(0.0, bstd, size=(out_dim,)) if bias is None else bias
    return (torch.tensor(g, dtype=torch.float32), torch.tensor(v, dtype=torch.float32),
            torch.tensor(b, dtype=torch.float32))


def surface_dims(D=8, W=256, skips=(4,), multires=6, W_geo_feat=256):
    in_ch = 3 + 3 * 2 * multires if multires > 0 else 3
    dims = []
    for l in range(D + 1):
        if l == D:
            out_dim = 1 + W_geo_feat if W_geo_feat > 0 else 1
        elif (l + 1) in skips:
            out_dim = W - in_ch
        else:
            out_dim = W
        in_dim = in_ch if l == 0 else W
        dims.append((out_dim, in_dim))
    return dims, in_ch


def surface_state(rs, prefix, radius_init, obj_bounding_size, D=8, W=256, skips=(4,), multires=6,
                  W_geo_feat=256):
    dims, in_ch = surface_dims(D, W, skips, multires, W_geo_feat)
    sd = {}
    for l, (o, i) in enumerate(dims):
        if l == D:
            g, v, b = _wn_layer(rs, o, i, std=1e-3, mean=math.sqrt(math.pi) / math.sqrt(i))
            # feature rows: varied so the radiance net sees distinct features
            v2 = rs.normal(0.0, math.sqrt(2) / math.sqrt(i), size=(o - 1, i))
            vv = v.numpy().copy()
            vv[1:] = v2
            nrm = np.linalg.norm(vv, axis=1, keepdims=True)
            gg = nrm * (1.0 + 0.05 * rs.uniform(-1.0, 1.0, size=(o, 1)))
            bb = rs.normal(0.0, 0.01, size=(o,))
            bb[0] = -radius_init
            g = torch.tensor(gg, dtype=torch.float32)
            v = torch.tensor(vv, dtype=torch.float32)
            b = torch.tensor(bb, dtype=torch.float32)
        elif l == 0 and multires > 0:
            g, v, b = _wn_layer(rs, o, i, std=math.sqrt(2) / math.sqrt(o), small_cols=slice(3, None),
                                small_std=0.05 * math.sqrt(2) / math.sqrt(o))
        elif l in skips and multires > 0:
            g, v, b = _wn_layer(rs, o, i, std=math.sqrt(2) / math.sqrt(o),
                                small_cols=slice(i - (in_ch - 3), None),
                                small_std=0.05 * math.sqrt(2) / math.sqrt(o))
        else:
            g, v, b = _wn_layer(rs, o, i, std=math.sqrt(2) / math.sqrt(o))
        sd[f'{prefix}surface_fc_layers.{l}.weight_g'] = g
        sd[f'{prefix}surface_fc_layers.{l}.weight_v'] = v
        sd[f'{prefix}surface_fc_layers.{l}.bias'] = b
    sd[f'{prefix}obj_bounding_size'] = torch.tensor([float(obj_bounding_size)], dtype=torch.float32)
    return sd


def radiance_state(rs, prefix, in_dim0, D=4, W=256):
    sd = {}
    for l in range(D + 1):
        o = 3 if l == D else W
        i = in_dim0 if l == 0 else W
        g, v, b = _wn_layer(rs, o, i, std=math.sqrt(2.0 / i), bstd=1.0 / math.sqrt(i))
        sd[f'{prefix}layers.{l}.weight_g'] = g
        sd[f'{prefix}layers.{l}.weight_v'] = v
        sd[f'{prefix}layers.{l}.bias'] = b
    return sd


def _linear(rs, o, i):
    k = 1.0 / math.sqrt(i)
    return (torch.tensor(rs.uniform(-k, k, size=(o, i)), dtype=torch.float32),
            torch.tensor(rs.uniform(-k, k, size=(o,)), dtype=torch.float32))


def nerf_state(rs, prefix, D=8, W=256, input_ch=84, input_ch_view=27, skips=(4,)):
    sd = {}
    ins = [input_ch] + [W + input_ch if (i in skips) else W for i in range(D - 1)]
    for l, i in enumerate(ins):
        w, b = _linear(rs, W, i)
        sd[f'{prefix}pts_linears.{l}.weight'] = w
        sd[f'{prefix}pts_linears.{l}.bias'] = b
    for name, (o, i) in [('views_linears.0', (W // 2, input_ch_view + W)), ('feature_linear', (W, W)),
                         ('alpha_linear', (1, W)), ('rgb_linear', (3, W // 2))]:
        w, b = _linear(rs, o, i)
        sd[f'{prefix}{name}.weight'] = w
        sd[f'{prefix}{name}.bias'] = b
    return sd


def neus_state(seed=1, use_outside_nerf=False, variance_init=0.05, speed_factor=10.0, radius_init=0.5,
               use_view_dirs=True):
    rs = np.random.RandomState(seed)
    sd = {'ln_s': torch.tensor([-np.log(variance_init) / speed_factor], dtype=torch.float32)}
    sd.update(surface_state(rs, 'implicit_surface.', radius_init, 1.0))
    sd.update(radiance_state(rs, 'radiance_net.', 3 + 27 + 3 + 256 if use_view_dirs else 3 + 256))
    if use_outside_nerf:
        sd.update(nerf_state(rs, 'nerf_outside.'))
    return sd


def volsdf_state(seed=2, beta_init=0.1, speed_factor=10.0, obj_bounding_radius=3.0, radius_init=1.0,
                 use_nerfplusplus=False):
    rs = np.random.RandomState(seed)
    sd = {'ln_beta': torch.tensor([np.log(beta_init) / speed_factor], dtype=torch.float32)}
    sd.update(surface_state(rs, 'implicit_surface.', radius_init, obj_bounding_radius))
    sd.update(radiance_state(rs, 'radiance_net.', 3 + 3 + 3 + 256))
    if use_nerfplusplus:
        sd.update(nerf_state(rs, 'nerf_outside.'))
    return sd


def siren_layers(rs, prefix, dims, w0=30.0, c=6.0, last=None):
    """weight-normed SirenLayers (base.py:93-106 init ranges): layer l maps dims[l] -> dims[l+1];
    first layer U(+-1/in), others U(+-sqrt(c/in)/w0), bias U(+-1/sqrt(in)); `last` = (out, in) of a
    plain weight-normed Linear head with nn.Linear's ranges."""
    sd = {}
    n = len(dims) - 1
    for l in range(n):
        i, o = dims[l], dims[l + 1]
        s = (1.0 / i) if l == 0 else math.sqrt(c / i) / w0
        v = torch.tensor(rs.uniform(-s, s, size=(o, i)), dtype=torch.float32)
        b = torch.tensor(rs.uniform(-1 / math.sqrt(i), 1 / math.sqrt(i), size=(o,)), dtype=torch.float32)
        sd[f'{prefix}{l}.weight_g'] = torch.norm_except_dim(v, 2, 0)
        sd[f'{prefix}{l}.weight_v'] = v
        sd[f'{prefix}{l}.bias'] = b
    if last is not None:
        o, i = last
        k = 1 / math.sqrt(i)
        v = torch.tensor(rs.uniform(-k, k, size=(o, i)), dtype=torch.float32)
        sd[f'{prefix}{n}.weight_g'] = torch.norm_except_dim(v, 2, 0)
        sd[f'{prefix}{n}.weight_v'] = v
        sd[f'{prefix}{n}.bias'] = torch.tensor(rs.uniform(-k, k, size=(o,)), dtype=torch.float32)
    return sd


def volsdf_siren_state(seed=7, beta_init=0.1, speed_factor=10.0):
    """VolSDF with configs/volsdf_siren.yaml's nets: SIREN surface D=5 (3 -> 256 x5 -> 257) and SIREN
    radiance D=5 (3 + 27 + 3 + 256 -> 256 x5 -> 3); no pretraining (the weights are loaded as-is)."""
    rs = np.random.RandomState(seed)
    sd = {'ln_beta': torch.tensor([np.log(beta_init) / speed_factor], dtype=torch.float32),
          'implicit_surface.obj_bounding_size': torch.tensor([3.0]),
          'implicit_surface.is_pretrained': torch.tensor([True])}
    sd.update(siren_layers(rs, 'implicit_surface.surface_fc_layers.', [3] + [256] * 5, last=(257, 256)))
    sd.update(siren_layers(rs, 'radiance_net.layers.', [3 + 27 + 3 + 256] + [256] * 5, last=(3, 256)))
    return sd


def unisurf_state(seed=3, radius_init=1.0, use_view_dirs=True):
    rs = np.random.RandomState(seed)
    sd = {}
    sd.update(surface_state(rs, 'implicit_surface.', radius_init, 2.0))
    sd.update(radiance_state(rs, 'radiance_net.', 3 + 3 + 3 + 256 if use_view_dirs else 3 + 256))
    return sd


def look_at_c2w(dist):
    """Camera at (0,0,-dist) looking at the origin, OpenCV up=(0,-1,0) (rend_util.py:44-53)."""
    cam = np.array([0.0, 0.0, -dist])
    fwd = -cam / (np.linalg.norm(cam) + 1e-9)
    up = np.array([0.0, -1.0, 0.0])
    x = np.cross(up, fwd); x = x / (np.linalg.norm(x) + 1e-9)
    y = np.cross(fwd, x); y = y / (np.linalg.norm(y) + 1e-9)
    m = np.eye(4)
    m[:3, 0], m[:3, 1], m[:3, 2], m[:3, 3] = x, y, fwd, cam
    return torch.tensor(m, dtype=torch.float32)


def intrinsics(f, H, W):
    k = np.eye(4)
    k[0, 0] = f; k[1, 1] = f; k[0, 2] = W / 2.0; k[1, 2] = H / 2.0
    return torch.tensor(k, dtype=torch.float32)


# Synthetic cameras of SURVEY.md §8(d) (H, W, f, dist)
CAMERAS = {
    'a': (16, 32, 40.0, 2.7),
    'b': (64, 64, 160.0, 3.0),
    'c': (32, 64, 80.0, 2.7),
    'd': (600, 800, 800.0, 2.0),
    'e': (64, 64, 80.0, 3.0),
}
