"""ORACLE (test infrastructure only): the reference's MLPs restated as pure functions over a
reference-format state_dict (weight_g / weight_v / bias keys, models/base.py)."""
import math
import torch
import torch.nn.functional as F


def freq_bands(n_freqs):
    # models/base.py:38-44: 2**linspace(0, F-1, F), cast to python floats
    return (2. ** torch.linspace(0., n_freqs - 1, n_freqs, device='cpu')).numpy().tolist()


def embed(x, n_freqs):
    """Positional encoding [x, sin(f0 x), cos(f0 x), sin(f1 x), ...] (models/base.py:46-64);
    n_freqs < 0 => identity (models/base.py:67-69)."""
    if n_freqs < 0:
        return x
    parts = [x]
    for f in freq_bands(n_freqs):
        parts.append(torch.sin(x * f))
        parts.append(torch.cos(x * f))
    return torch.cat(parts, dim=-1)


def wn_weight(sd, prefix):
    """weight_norm(dim=0): W = g * v / ||v||_row, recomputed per forward (base.py:226-227)."""
    return torch._weight_norm(sd[prefix + '.weight_v'], sd[prefix + '.weight_g'], 0)


def softplus100(z):
    # base.py:202  nn.Softplus(beta=100) with torch's default threshold 20
    return F.softplus(z, beta=100, threshold=20)


def sine30(z):
    # base.py:84-91 Sine(w0=30): torch.sin(w0 * x)
    return torch.sin(30 * z)


class SDFNet:
    """ImplicitSurface (models/base.py:131-282) over a state_dict slice; siren=True: SirenLayer
    hidden layers (base.py:93-115, use_siren)."""

    def __init__(self, sd, prefix='implicit_surface.', D=8, skips=(4,), multires=6, W_geo_feat=256, siren=False):
        self.D, self.skips, self.multires, self.W_geo_feat = D, tuple(skips), multires, W_geo_feat
        self.act = sine30 if siren else softplus100
        self.layers = [(wn_weight(sd, f'{prefix}surface_fc_layers.{l}'), sd[f'{prefix}surface_fc_layers.{l}.bias'])
                       for l in range(D + 1)]

    def forward(self, x):
        # base.py:243-263
        xe = embed(x, self.multires)
        h = xe
        for i in range(self.D):
            if i in self.skips:
                h = torch.cat([h, xe], dim=-1) / math.sqrt(2)
            W, b = self.layers[i]
            h = self.act(F.linear(h, W, b))
        W, b = self.layers[self.D]
        out = F.linear(h, W, b)
        if self.W_geo_feat > 0:
            return out[..., 0], out[..., 1:]
        return out[..., 0], None

    def sdf(self, x):
        return self.forward(x)[0]

    def forward_with_nablas(self, x):
        # base.py:265-282 (render mode: no graph kept)
        with torch.enable_grad():
            x = x.detach().requires_grad_(True)
            s, h = self.forward(x)
            g = torch.autograd.grad(s, x, torch.ones_like(s))[0]
        return s.detach(), g.detach(), None if h is None else h.detach()


class RadianceNet:
    """RadianceNet (models/base.py:312-391)."""

    def __init__(self, sd, prefix='radiance_net.', D=4, multires=-1, multires_view=4, use_view_dirs=True, siren=False):
        self.D, self.multires, self.multires_view, self.use_view_dirs = D, multires, multires_view, use_view_dirs
        self.act = sine30 if siren else torch.relu
        self.layers = [(wn_weight(sd, f'{prefix}layers.{l}'), sd[f'{prefix}layers.{l}.bias']) for l in range(D + 1)]

    def forward(self, x, v, normals, feature, masks=None, z_out=None):
        """masks (test instrumentation, ReLU nets): per hidden layer a bool tensor [..., 256] that
        replaces relu(z) by z * mask -- the ReLU decisions pinned to another evaluation's, as the tests
        pin the sample depths; z_out: a list that receives every hidden layer's pre-activation."""
        xe = embed(x, self.multires)
        if self.use_view_dirs:
            h = torch.cat([xe, embed(v, self.multires_view), normals, feature], dim=-1)
        else:
            h = torch.cat([xe, feature], dim=-1)
        for i, (W, b) in enumerate(self.layers):
            z = F.linear(h, W, b)
            if i < self.D and z_out is not None:
                z_out.append(z.detach())
            if i == self.D:
                h = torch.sigmoid(z)
            elif masks is not None:
                h = z * masks[i].reshape(z.shape).to(z.dtype)
            else:
                h = self.act(z)
        return h


class NeRFNet:
    """NeRF++ background MLP (models/base.py:395-453), input_ch=4, multires=10, multires_view=4."""

    def __init__(self, sd, prefix='nerf_outside.', D=8, skips=(4,), multires=10, multires_view=4):
        self.D, self.skips, self.multires, self.multires_view = D, tuple(skips), multires, multires_view
        g = lambda n: (sd[f'{prefix}{n}.weight'], sd[f'{prefix}{n}.bias'])
        self.pts = [g(f'pts_linears.{i}') for i in range(D)]
        self.view = g('views_linears.0')
        self.feature = g('feature_linear')
        self.alpha = g('alpha_linear')
        self.rgb = g('rgb_linear')

    def forward(self, x, v):
        xe = embed(x, self.multires)
        ve = embed(v, self.multires_view)
        h = xe
        for i, (W, b) in enumerate(self.pts):
            h = torch.relu(F.linear(h, W, b))
            if i in self.skips:
                h = torch.cat([xe, h], dim=-1)
        sigma = F.linear(h, *self.alpha)
        feat = F.linear(h, *self.feature)
        h = torch.relu(F.linear(torch.cat([feat, ve], dim=-1), *self.view))
        rgb = torch.sigmoid(F.linear(h, *self.rgb))
        return sigma[..., 0], rgb
