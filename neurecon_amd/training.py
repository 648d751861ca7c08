"""Training path of the render hot loop: autograd Functions whose forward and
backward run on libnrhip.so.  f16x3 nets (the default precision; softplus SDF nets and ReLU D=4
radiance nets) run every layer product on the hand-written training GEMM (nr_train_gemm: f16x3 MFMA
over the render pack's weight stream, the elementwise step of the recipe fused into its epilogue);
the weight gradients run on nr_wgrad (hand-written MFMA, f16x3 products).  fp32-precision and SIREN
nets keep the reference-exact path: exact fp32 layer products on nr_gemm32 (r06, hand-written
v_mfma_f32_16x16x4_f32, k-order fmaf chains; torch.addmm / mm on hipBLASLt through r05), the elementwise
kernels of nr_train.hip between them, and nr_wgrad with exact fp32 products (fixed-order reduction) for
the weight gradients.

What the reference differentiates (models/frameworks/neus.py:284-485, models/base.py:265-282):
  * ImplicitSurface.forward_with_nablas with create_graph=True: sdf, nablas = d sdf / d x and the
    geometry feature, where the eikonal loss and the radiance net both consume the nablas -> the
    parameter gradient needs the DOUBLE backward through the SDF MLP;
  * RadianceNet on [x, embed_view(v), nablas, feature];
  * sdf_to_alpha / alpha_to_w / the rgb, depth and mask sums, and s = exp(ln_s * speed_factor).
`SdfNabla` computes the double backward as reverse mode over the (primal, tangent) network
(nr_train.hip header): the tangent seed is J_emb(x) * grad_nablas, and since the tangent's adjoint
equals the nabla chain's own gradients, one tangent sweep and one adjoint sweep give every weight
gradient: dW_l = zbar_l^T hin_l + delta_l^T hdot_in_l.
"""
import ctypes
import os
import math

import torch

from . import _lib as L

_ISQ2 = 1.0 / math.sqrt(2.0)


def _st(t):
    return L.stream_of(t.device)


def _embed(x, nfreq):
    out = torch.empty(x.shape[0], 3 + 6 * nfreq if nfreq >= 0 else 3, device=x.device)
    L.check(L.lib().nr_embed(L.ptr(x), x.shape[0], nfreq, L.ptr(out), _st(x)))
    return out


def _softplus(z):
    h = torch.empty_like(z)
    s = torch.empty_like(z)
    L.check(L.lib().nr_softplus100(L.ptr(z), z.numel(), L.ptr(h), L.ptr(s), _st(z)))
    return h, s


def _cols(a, col0, ncols, s=None, scale=1.0):
    """a[:, col0:col0+ncols] * scale (* s), contiguous"""
    out = torch.empty(a.shape[0], ncols, device=a.device)
    L.check(L.lib().nr_scale_cols(L.ptr(a), a.shape[0], a.shape[1], col0, ncols, L.ptr(s), float(scale), L.ptr(out),
                                  _st(a)))
    return out


def _sine30(z):
    h = torch.empty_like(z)
    s = torch.empty_like(z)
    L.check(L.lib().nr_sine30(L.ptr(z), z.numel(), L.ptr(h), L.ptr(s), _st(z)))
    return h, s


def _wgrad(g, h, fp32=True):
    """gᵀ h for the weight gradients of a tall batch (g [P, m], h [P, k], P ~ 65 k) on nr_wgrad: exact
    fp32 products (v_mfma_f32_16x16x4_f32) summed per row slice in order and over the slices in fixed
    order -- the fp32 nets' path (r05; r04 ran hipBLASLt's split-K batched GEMM + a sum, whose error
    was 1.4x the fp32 oracle's own on the training step's layer-0 / layer-4 weights); fp32=False: the
    f16x3 products of the default nets"""
    return _wg([(g, h)], fp32=fp32)


def _wgrad2(g1, h1, g2, h2, fp32=True):
    """g1^T h1 + g2^T h2 in one nr_wgrad launch (both sweeps of a layer)"""
    return _wg([(g1, h1), (g2, h2)], fp32=fp32)


def _wgb(g, h, fp32=True):
    """(gᵀ h, column sums of g): a layer's weight and bias gradients in one nr_wgrad launch"""
    db = torch.empty(g.shape[1], device=g.device)
    return _wg([(g, h)], colsum=db, fp32=fp32), db


def _wg(pairs, out=None, scale=1.0, colsum=None, avec=None, vec=None, blocked=0, fp32=False):
    """sum_q a_q^T b_q on the hand-written MFMA weight-gradient kernel (nr_wgrad; f16x3 products, or
    exact fp32 products on v_mfma_f32_16x16x4_f32 with fp32=True -- the fp32 nets' path): pairs of
    row-major views a [P, m], b [P, n] (unit column stride; any row stride); out [m, n] (a view with
    unit column stride, e.g. a column range of the gradient) = scale * the sum.  colsum: [m] <- the
    column sums of a_0 (the bias gradient); avec [P] / vec [n]: vec <- avec^T b_0 (an extra row).
    blocked: NR_WG_BLK_* bits of the operands stored 16 x 16 blocked (a column view [:, :n] of a
    blocked tensor keeps its pointer and leading dimension, which is all the kernel needs)."""
    a0, b0 = pairs[0]
    P, m = a0.shape
    n = b0.shape[1]
    dev = a0.device
    if out is None:
        out = torch.empty(m, n, device=dev)
    w = L.NrWgrad()
    w.P, w.npairs, w.m, w.n, w.scale = P, len(pairs), m, n, float(scale)
    for q, (a, b) in enumerate(pairs):
        assert a.shape == (P, m) and b.shape == (P, n) and a.stride(1) == 1 and b.stride(1) == 1
        w.a[q], w.lda[q], w.b[q], w.ldb[q] = a.data_ptr(), a.stride(0), b.data_ptr(), b.stride(0)
    assert out.shape == (m, n) and out.stride(1) == 1
    w.c, w.ldc = out.data_ptr(), out.stride(0)
    if colsum is not None:
        w.colsum = colsum.data_ptr()
    if avec is not None:
        w.avec, w.ldv, w.vec, w.vec_scale = avec.data_ptr(), avec.stride(0), vec.data_ptr(), 1.0
    w.blocked = blocked
    w.fp32 = int(bool(fp32))
    lib = L.lib()
    nb = lib.nr_wgrad_workspace_bytes(P, m, n, len(pairs))
    ws = L.workspace(dev, nb)
    w.workspace, w.workspace_bytes = ws.data_ptr(), nb
    L.check(lib.nr_wgrad(ctypes.byref(w), _st(a0)))
    return out


def _colsum(a):
    """a.sum(0) of a tall [P, n] gradient on the deterministic two-pass HIP reduction (nr_colsum): the
    generic column reduction took ~0.45 ms per [65536, 256] matrix, rocBLAS's GEMV ~1 ms"""
    a = a.contiguous()
    P, n = a.shape
    out = torch.empty(n, device=a.device, dtype=a.dtype)
    lib = L.lib()
    wb = lib.nr_colsum_workspace_bytes(n)
    ws = torch.empty(wb, dtype=torch.uint8, device=a.device)
    L.check(lib.nr_colsum(L.ptr(a), P, n, L.ptr(out), L.ptr(ws), wb, _st(a)))
    return out


def _mm(a, w, bias=None, trans=False, acc32=False):
    """a @ w.t() + bias (trans: nn.Linear's addmm) or a @ w on nr_gemm32: exact fp32 products accumulated
    in fp64 and rounded once (acc32: an fp32 fmaf chain in k order), the bias added last; a [P, K] with
    unit column stride (any row stride), w [N, K] (trans) or [K, N] contiguous"""
    if a.stride(1) != 1:
        a = a.contiguous()
    w = w.contiguous()
    P, K = a.shape
    N = w.shape[0] if trans else w.shape[1]
    assert w.shape[1 if trans else 0] == K
    out = torch.empty(P, N, device=a.device)
    L.check(L.lib().nr_gemm32(L.ptr(a), a.stride(0), L.ptr(w), w.stride(0), int(trans),
                              L.ptr(bias.contiguous()) if bias is not None else None, L.ptr(out), N, P, N, K, int(acc32),
                              _st(a)))
    return out


def _mul(a, b):
    out = torch.empty_like(a)
    L.check(L.lib().nr_mul(L.ptr(a), L.ptr(b), a.numel(), L.ptr(out), _st(a)))
    return out


class SdfNabla(torch.autograd.Function):
    """ImplicitSurface.forward_with_nablas with a differentiable graph (base.py:265-282,
    create_graph=True): x [P,3] (no grad) -> sdf [P], nablas [P,3], feature [P,W_geo] (or None).
    params = W_0..W_D, b_0..b_D (effective weight-normed weights, [out, in]).  Hidden activation:
    softplus(beta=100), or sin(30 z) for SirenLayers (base.py:84-115; cfg[4])."""

    @staticmethod
    def forward(ctx, x, cfg, *params):
        D, skips, nfreq, want_feat, siren = cfg
        Ws, bs = params[:D + 1], params[D + 1:]
        x = x.contiguous()
        h0 = _embed(x, nfreq)
        hin, ss = [], []
        h = h0
        for l in range(D):
            hi = torch.cat([h, h0], -1).div_(math.sqrt(2)) if l in skips else h  # base.py:250
            z = _mm(hi, Ws[l], bs[l], trans=True)
            h, s = _sine30(z) if siren else _softplus(z)
            hin.append(hi)
            ss.append(s)
        hin.append(h)
        out = _mm(h, Ws[D], bs[D], trans=True)
        sdf = out[:, 0].contiguous()
        feat = out[:, 1:].contiguous() if want_feat else None
        # nabla chain: g_l = d sdf / d h_l, delta_l = s_l * g_l
        gs, deltas = [None] * D, [None] * D
        g = Ws[D][0:1, :].expand(h.shape[0], -1)
        e_skip = None
        e_first = None
        for l in range(D - 1, -1, -1):
            gs[l] = g.contiguous()
            delta = deltas[l] = _mul(ss[l], gs[l])  # kept: the backward's tangent adjoint
            gin = _mm(delta, Ws[l])
            if l in skips:
                n_prev = Ws[l - 1].shape[0]
                e_skip = _cols(gin, n_prev, gin.shape[1] - n_prev, scale=_ISQ2)
                g = _cols(gin, 0, n_prev, scale=_ISQ2)
            elif l > 0:
                g = gin
            else:
                e_first = gin.contiguous()
        nab = torch.empty(x.shape[0], 3, device=x.device)
        L.check(L.lib().nr_embed_vjp(L.ptr(x), L.ptr(e_first), e_first.shape[1], L.ptr(e_skip),
                                     0 if e_skip is None else e_skip.shape[1], 1.0, x.shape[0], nfreq, L.ptr(nab),
                                     _st(x)))
        ctx.cfg = cfg
        ctx.save_for_backward(x, *Ws, *hin, *ss, *gs, *deltas)
        outs = (sdf, nab, feat) if want_feat else (sdf, nab)
        return outs

    @staticmethod
    def backward(ctx, g_sdf, g_nab, *rest):
        D, skips, nfreq, want_feat, siren = ctx.cfg
        saved = ctx.saved_tensors
        x = saved[0]
        Ws = saved[1:D + 2]
        hin = saved[D + 2:2 * D + 3]
        ss = saved[2 * D + 3:3 * D + 3]
        gs = saved[3 * D + 3:4 * D + 3]
        deltas = saved[4 * D + 3:5 * D + 3]
        g_feat = rest[0] if want_feat else None
        P = x.shape[0]
        dev = x.device
        lib = L.lib()
        # output-layer adjoint [d sdf, d feature]
        ob = torch.zeros(P, Ws[D].shape[0], device=dev)
        if g_sdf is not None:
            ob[:, 0] = g_sdf
        if g_feat is not None:
            ob[:, 1:] = g_feat
        # tangent sweep (forward mode along grad_nablas): hdot_0 = J_emb(x) g_nab
        tangent = g_nab is not None
        zdots, hdins = [None] * D, [None] * (D + 1)
        if tangent:
            g_nab = g_nab.contiguous()
            hd0 = torch.empty(P, 3 + 6 * nfreq if nfreq >= 0 else 3, device=dev)
            L.check(lib.nr_embed_jvp(L.ptr(x), L.ptr(g_nab), P, nfreq, L.ptr(hd0), _st(x)))
            hd = hd0
            for l in range(D):
                hdi = torch.cat([hd, hd0], -1).div_(math.sqrt(2)) if l in skips else hd
                zd = _mm(hdi, Ws[l], trans=True)
                hdins[l], zdots[l] = hdi, zd
                hd = _mul(ss[l], zd)
            hdins[D] = hd
        dW = [None] * (D + 1)
        db = [None] * (D + 1)
        dW[D] = _wgrad(ob, hin[D])
        db[D] = _colsum(ob)
        if tangent:  # d(g_nab . nabla) / d W_D[0, :] = sum_p hdot_{D-1}
            dW[D][0] += _colsum(hdins[D])
        hbar = _mm(ob, Ws[D])
        for l in range(D - 1, -1, -1):
            n = ss[l].shape[1]
            zbar = torch.empty(P, n, device=dev)
            if siren:  # layer l's output h_l = hin[l + 1] (no skips in a SIREN net)
                L.check(lib.nr_sine_adjoint(L.ptr(hbar), hbar.shape[1], L.ptr(ss[l]), L.ptr(hin[l + 1]),
                                            L.ptr(gs[l] if tangent else None), L.ptr(zdots[l]), P, n, L.ptr(zbar),
                                            _st(x)))
            else:
                L.check(lib.nr_softplus_adjoint(L.ptr(hbar), hbar.shape[1], L.ptr(ss[l]),
                                                L.ptr(gs[l] if tangent else None), L.ptr(zdots[l]), P, n, L.ptr(zbar),
                                                _st(x)))
            if tangent:  # + the tangent's adjoint (= the nabla chain's delta_l) against hdot
                dW[l] = _wgrad2(zbar, hin[l], deltas[l], hdins[l])
            else:
                dW[l] = _wgrad(zbar, hin[l])
            db[l] = _colsum(zbar)
            if l > 0:
                hb = _mm(zbar, Ws[l])
                hbar = _cols(hb, 0, Ws[l - 1].shape[0], scale=_ISQ2) if l in skips else hb
        return (None, None, *dW, *db)


class RadianceFn(torch.autograd.Function):
    """RadianceNet.forward with a graph (base.py:372-391): [x, embed_view(v), normals, feature] ->
    D x (Linear + ReLU, or SirenLayer sin(30 z)) -> Linear(3) + sigmoid.  Gradients flow to normals,
    feature and the params."""

    @staticmethod
    def forward(ctx, x, v, nrm, feat, cfg, *params):
        D, nfreq_view, view, siren = cfg
        Ws, bs = params[:D + 1], params[D + 1:]
        P = x.shape[0]
        wf = feat.shape[1]
        # without view dirs the input is cat([x, feature]) (base.py:383-384): no view / normal columns
        nv = (3 if nfreq_view < 0 else 3 + 6 * nfreq_view) if view else 0
        nn_ = 3 if view else 0
        inp = torch.empty(P, 3 + nv + nn_ + wf, device=x.device)
        L.check(L.lib().nr_radiance_input(L.ptr(x), L.ptr(v), L.ptr(nrm), L.ptr(feat), P, nfreq_view, int(view), wf,
                                          L.ptr(inp), _st(x)))
        hs = [inp]
        ss = []
        h = inp
        for l in range(D):
            h = _mm(h, Ws[l], bs[l], trans=True)
            if siren:
                h, s = _sine30(h)
                ss.append(s)
            else:
                L.check(L.lib().nr_activation(L.ptr(h), None, h.numel(), 0, _st(x)))
            hs.append(h)
        y = _mm(h, Ws[D], bs[D], trans=True)
        L.check(L.lib().nr_activation(L.ptr(y), None, y.numel(), 2, _st(x)))
        ctx.cfg = (D, nv, nn_, wf, siren)
        ctx.save_for_backward(y, *Ws, *hs, *ss)
        return y

    @staticmethod
    def backward(ctx, gy):
        D, nv, nn_, wf, siren = ctx.cfg
        saved = ctx.saved_tensors
        y = saved[0]
        Ws = saved[1:D + 2]
        hs = saved[D + 2:2 * D + 3]
        ss = saved[2 * D + 3:]
        g = gy.contiguous().clone()
        L.check(L.lib().nr_activation(L.ptr(y), L.ptr(g), g.numel(), 3, _st(g)))
        dW, db = [None] * (D + 1), [None] * (D + 1)
        for l in range(D, -1, -1):
            dW[l], db[l] = _wgb(g, hs[l])
            g = _mm(g, Ws[l])
            if l > 0:
                if siren:
                    g = _mul(ss[l - 1], g)
                else:
                    L.check(L.lib().nr_activation(L.ptr(hs[l]), L.ptr(g), g.numel(), 1, _st(g)))
        d_nrm = _cols(g, 3 + nv, 3) if nn_ else None
        d_feat = _cols(g, 3 + nv + nn_, wf)
        return (None, None, d_nrm, d_feat, None, *dW, *db)


class NeuSComposite(torch.autograd.Function):
    """sdf_to_alpha / alpha_to_w / rgb, depth, acc sums (neus.py:28-70, :346-355) with a graph:
    sdf [R,S], s [1], radiance [R,S-1,3], d_mid [R,S-1] (no grad) -> rgb [R,3], depth [R], acc [R],
    visibility weights [R,S-1] (+ alpha, cdf, not differentiable)."""

    @staticmethod
    def forward(ctx, sdf, s, rad, dmid, white_bkgd):
        R, S = sdf.shape
        dev = sdf.device
        sdf, rad, dmid, s = sdf.contiguous(), rad.contiguous(), dmid.contiguous(), s.reshape(-1)[:1].contiguous()
        rgb = torch.empty(R, 3, device=dev)
        depth = torch.empty(R, device=dev)
        acc = torch.empty(R, device=dev)
        w = torch.empty(R, S - 1, device=dev)
        alpha = torch.empty(R, S - 1, device=dev)
        cdf = torch.empty(R, S, device=dev)
        L.check(L.lib().nr_neus_composite_fwd(L.ptr(sdf), L.ptr(s), L.ptr(rad), L.ptr(dmid), R, S, int(white_bkgd),
                                              L.ptr(rgb), L.ptr(depth), L.ptr(acc), L.ptr(w), L.ptr(alpha), L.ptr(cdf),
                                              _st(sdf)))
        ctx.white = int(white_bkgd)
        ctx.save_for_backward(sdf, s, rad, dmid)
        ctx.mark_non_differentiable(alpha, cdf)
        return rgb, depth, acc, w, alpha, cdf

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_w, _ga, _gc):
        sdf, s, rad, dmid = ctx.saved_tensors
        R, S = sdf.shape
        c = lambda t: None if t is None else t.contiguous()
        d_sdf = torch.empty_like(sdf)
        d_rad = torch.empty_like(rad)
        d_s = torch.empty(R, device=sdf.device)
        lib = L.lib()
        wb = lib.nr_neus_composite_bwd_workspace_bytes(R, S)
        ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=sdf.device)
        g_rgb, g_depth, g_acc, g_w = c(g_rgb), c(g_depth), c(g_acc), c(g_w)
        L.check(lib.nr_neus_composite_bwd(L.ptr(sdf), L.ptr(s), L.ptr(rad), L.ptr(dmid), R, S, ctx.white, L.ptr(g_rgb),
                                          L.ptr(g_depth), L.ptr(g_acc), L.ptr(g_w), L.ptr(d_sdf), L.ptr(d_rad),
                                          L.ptr(d_s), L.ptr(ws), wb, _st(sdf)))
        return d_sdf, d_s.sum().reshape(1), d_rad, None, None


def _nerf_packs(net, Ws, bs, device):
    """(fp32 desc, the fp32 render pack, the training desc, the training pack) of a NeRF++ net built from
    the step's weights (12 layers: pts_linears 0..7, feature, views, alpha, rgb), cached per parameter
    version.  The forward runs on the fp32 pack whatever the net's precision (its ReLU decisions must be
    the reference's); the training pack (the backward's transposed ops) is in the net's precision: the
    backward is linear in the stored masks, so an f16x3 net runs it on f16x3 products (r06)"""
    from .base import _version_key, _ptr_array
    key = _version_key(net, 'nerf_train32', device)
    c = getattr(net, '_nr_train32_cache', None)
    if c is not None and c[0] == key:
        return c[1], c[2], c[3], c[4]
    lib = L.lib()
    desc = net.nr_desc()
    desc.precision = L.PREC_FP32
    tdesc = net.nr_desc()
    tdesc.precision = L.PREC_F16X3 if getattr(net, 'precision', 'fp32') == 'f16x3' else L.PREC_FP32
    W = [w.detach().float().contiguous() for w in Ws]
    b = [x.detach().float().contiguous() for x in bs]
    pk = torch.empty(lib.nr_nerf_packed_bytes(ctypes.byref(desc)), dtype=torch.uint8, device=device)
    L.check(lib.nr_nerf_pack(ctypes.byref(desc), _ptr_array(W), _ptr_array(b), L.ptr(pk), L.stream_of(device)))
    tp = torch.empty(lib.nr_nerf_train_packed_bytes(ctypes.byref(tdesc)), dtype=torch.uint8, device=device)
    L.check(lib.nr_nerf_train_pack(ctypes.byref(tdesc), _ptr_array(W), _ptr_array(b), L.ptr(tp), L.stream_of(device)))
    net._nr_train32_cache = (key, desc, pk, tdesc, tp, W, b)
    return desc, pk, tdesc, tp


def _ptrs(ts):
    return (ctypes.c_void_p * len(ts))(*[t.data_ptr() for t in ts])


class NeRFFn(torch.autograd.Function):
    """NeRF.forward (base.py:426-453, NeRF++ background: 8 x ReLU(256) with cat([input, h]) after the
    skip layer, alpha / feature heads, views Linear(256+27 -> 128) + ReLU, rgb Linear + sigmoid) with a
    graph.  Inputs are the embedded points x_emb [P,84] and views v_emb [P,27] (no gradient: they depend
    on the rays and the no-grad depths).  Returns sigma [P], rgb [P,3]; gradients reach every parameter.
    r05: the forward is one launch of nr_nerf_train_fwd32 (exact fp32 products, the layers chained in
    registers, every activation the backward needs stored) and the backward's data gradients one launch
    of nr_nerf_train_bwd32 (the transposed ops chained, each layer's ReLU mask applied and its
    pre-activation gradient stored; r06: f16x3 products for f16x3 nets, exact fp32 for fp32 nets), in
    place of 23 hipBLASLt GEMMs and 13 activation launches; the
    weight gradients are nr_wgrad products (exact fp32 for fp32 nets, f16x3 otherwise), the skip
    layer's and the views layer's per input column block (no [P, 340] / [P, 283] concatenations)."""

    @staticmethod
    def forward(ctx, xe, ve, net, *params):
        Ws, bs = params[:12], params[12:]
        dev = xe.device
        P = xe.shape[0]
        xe, ve = xe.contiguous(), ve.contiguous()
        if xe.data_ptr() % 16:  # a contiguous view at an unaligned offset: the kernel reads 16-B rows
            xe = xe.clone()
        desc, pk, _, _ = _nerf_packs(net, Ws, bs, dev)
        H = [torch.empty(P, 256, device=dev) for _ in range(8)]
        feat = torch.empty(P, 256, device=dev)
        hv = torch.empty(P, 128, device=dev)
        sigma = torch.empty(P, device=dev)
        rgb = torch.empty(P, 3, device=dev)
        L.check(L.lib().nr_nerf_train_fwd32(ctypes.byref(desc), L.ptr(pk), L.ptr(xe), L.ptr(ve), P, _ptrs(H),
                                            L.ptr(feat), L.ptr(hv), L.ptr(sigma), L.ptr(rgb), _st(xe)))
        ctx.net = net
        ctx.fp32 = getattr(net, 'precision', 'fp32') == 'fp32'
        ctx.save_for_backward(xe, ve, rgb, hv, feat, *H, *params)
        return sigma, rgb

    @staticmethod
    def backward(ctx, g_sigma, g_rgb):
        saved = ctx.saved_tensors
        xe, ve, rgb, hv, feat = saved[:5]
        H = saved[5:13]
        params = saved[13:]
        Ws, bs = params[:12], params[12:]
        dev = rgb.device
        P = rgb.shape[0]
        nx = xe.shape[1]
        _, _, tdesc, tp = _nerf_packs(ctx.net, Ws, bs, dev)
        g3 = torch.empty(P, 3, device=dev)
        ghv = torch.empty(P, 128, device=dev)
        g_feat = torch.empty(P, 256, device=dev)
        GZ = [torch.empty(P, 256, device=dev) for _ in range(8)]
        g_rgb = None if g_rgb is None else g_rgb.contiguous()
        gs = torch.zeros(P, device=dev) if g_sigma is None else g_sigma.reshape(P).contiguous()
        L.check(L.lib().nr_nerf_train_bwd32(ctypes.byref(tdesc), L.ptr(tp), L.ptr(rgb), L.ptr(hv), _ptrs(H),
                                            None if g_rgb is None else L.ptr(g_rgb), L.ptr(gs), P, L.ptr(g3),
                                            L.ptr(ghv), L.ptr(g_feat), _ptrs(GZ), _st(rgb)))
        f32 = ctx.fp32  # weight gradients on nr_wgrad: exact fp32 products (fp32 nets) or f16x3
        dWr, dbr = _wgb(g3, hv, f32)
        dWv = torch.empty(128, 256 + ve.shape[1], device=dev)
        dbv = torch.empty(128, device=dev)
        _wg([(ghv, feat)], out=dWv[:, :256], colsum=dbv, fp32=f32)                  # cat([feature, v_emb])
        _wg([(ghv, ve)], out=dWv[:, 256:], fp32=f32)
        dWf, dbf = _wgb(g_feat, H[7], f32)
        dWa, dba = _wgb(gs[:, None], H[7], f32)
        dW, db = [None] * 8, [None] * 8
        for i in range(8):
            db[i] = torch.empty(256, device=dev)
            if i == 0:
                dW[0] = _wg([(GZ[0], xe)], colsum=db[0], fp32=f32)
            elif i == 5:  # the skip layer's input cat([x_emb, h4]) (base.py:431-432): per column block
                dW[5] = torch.empty(256, nx + 256, device=dev)
                _wg([(GZ[5], xe)], out=dW[5][:, :nx], colsum=db[5], fp32=f32)
                _wg([(GZ[5], H[4])], out=dW[5][:, nx:], fp32=f32)
            else:
                dW[i] = _wg([(GZ[i], H[i - 1])], colsum=db[i], fp32=f32)
        # params: pts_linears W0..W7, feature, views, alpha, rgb, then the biases in the same order
        return (None, None, None, *dW, dWf, dWv, dWa, dWr, *db, dbf, dbv, dba, dbr)


class NeuSCompositeBG(torch.autograd.Function):
    """NeuSComposite with the NeRF++ background merged (neus.py:325-352): sdf [R,S], s [1], radiance
    [R,S-1,3], sigma_out [R,M], radiance_out [R,M,3]; d_out [R,M] and inside [R,S-1] (no grad) ->
    rgb, depth, acc, visibility weights [R,M] (+ alpha [R,M], cdf [R,S], not differentiable)."""

    @staticmethod
    def forward(ctx, sdf, s, rad, sig_o, rad_o, d_out, inside, white_bkgd):
        R, S = sdf.shape
        M = d_out.shape[1]
        dev = sdf.device
        sdf, rad, s = sdf.contiguous(), rad.contiguous(), s.reshape(-1)[:1].contiguous()
        sig_o, rad_o = sig_o.contiguous(), rad_o.contiguous()
        rgb = torch.empty(R, 3, device=dev)
        depth = torch.empty(R, device=dev)
        acc = torch.empty(R, device=dev)
        w = torch.empty(R, M, device=dev)
        alpha = torch.empty(R, M, device=dev)
        cdf = torch.empty(R, S, device=dev)
        L.check(L.lib().nr_neus_composite_bg_fwd(L.ptr(sdf), L.ptr(s), L.ptr(rad), L.ptr(sig_o), L.ptr(rad_o),
                                                 L.ptr(d_out), L.ptr(inside), R, S, M, int(white_bkgd), L.ptr(rgb),
                                                 L.ptr(depth), L.ptr(acc), L.ptr(w), L.ptr(alpha), L.ptr(cdf), _st(sdf)))
        ctx.white = int(white_bkgd)
        ctx.save_for_backward(sdf, s, rad, sig_o, rad_o, d_out, inside)
        ctx.mark_non_differentiable(alpha, cdf)
        return rgb, depth, acc, w, alpha, cdf

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_w, _ga, _gc):
        sdf, s, rad, sig_o, rad_o, d_out, inside = ctx.saved_tensors
        R, S = sdf.shape
        M = d_out.shape[1]
        c = lambda t: None if t is None else t.contiguous()
        d_sdf, d_rad = torch.empty_like(sdf), torch.empty_like(rad)
        d_sig, d_rad_o = torch.empty_like(sig_o), torch.empty_like(rad_o)
        d_s = torch.empty(R, device=sdf.device)
        lib = L.lib()
        wb = lib.nr_neus_composite_bg_bwd_workspace_bytes(R, S, M)
        ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=sdf.device)
        g_rgb, g_depth, g_acc, g_w = c(g_rgb), c(g_depth), c(g_acc), c(g_w)
        L.check(lib.nr_neus_composite_bg_bwd(L.ptr(sdf), L.ptr(s), L.ptr(rad), L.ptr(sig_o), L.ptr(rad_o),
                                             L.ptr(d_out), L.ptr(inside), R, S, M, ctx.white, L.ptr(g_rgb),
                                             L.ptr(g_depth), L.ptr(g_acc), L.ptr(g_w), L.ptr(d_sdf), L.ptr(d_rad),
                                             L.ptr(d_sig), L.ptr(d_rad_o), L.ptr(d_s), L.ptr(ws), wb, _st(sdf)))
        return d_sdf, d_s.sum().reshape(1), d_rad, d_sig, d_rad_o, None, None, None


class VolSDFComposite(torch.autograd.Function):
    """VolSDF's sdf_to_sigma + ray integration (volsdf.py:16-35, :480-506) with the builtin background
    (volsdf.py:317-325) or the NeRF++ background samples (volsdf.py:455-469), with a graph: sdf [R,S]
    (network values), beta [1], radiance [R,S,3]; pts [R,S,3] and d_all [R,S] (no grad); optional
    sig_bg [R,N], rad_bg [R,N,3] (the background net's outputs) and d_bg [R,N] -> rgb [R,3], depth [R],
    acc [R], visibility weights [R,M-1], sdf with the background applied [R,S] (+ p_i [R,M-1],
    sigma [R,M], not differentiable), M = S + N."""

    @staticmethod
    def forward(ctx, sdf, beta, rad, pts, d_all, use_bg, r_bg, white_bkgd, sig_bg=None, rad_bg=None, d_bg=None):
        R, S = sdf.shape
        N = 0 if sig_bg is None else sig_bg.shape[1]
        M = S + N
        dev = sdf.device
        c = lambda t: None if t is None else t.contiguous()
        sdf, rad, pts, d_all = sdf.contiguous(), rad.contiguous(), pts.contiguous(), d_all.contiguous()
        sig_bg, rad_bg, d_bg = c(sig_bg), c(rad_bg), c(d_bg)
        beta = beta.reshape(-1)[:1].float().contiguous()
        rgb = torch.empty(R, 3, device=dev)
        depth = torch.empty(R, device=dev)
        acc = torch.empty(R, device=dev)
        tau = torch.empty(R, M - 1, device=dev)
        p_i = torch.empty(R, M - 1, device=dev)
        sigma = torch.empty(R, M, device=dev)
        sdf_bg = torch.empty(R, S, device=dev)
        L.check(L.lib().nr_volsdf_composite_bg_fwd(L.ptr(sdf), L.ptr(pts), L.ptr(beta), L.ptr(rad), L.ptr(d_all), R,
                                                   S, int(use_bg), float(r_bg), int(white_bkgd), L.ptr(sig_bg),
                                                   L.ptr(rad_bg), L.ptr(d_bg), N, L.ptr(rgb), L.ptr(depth), L.ptr(acc),
                                                   L.ptr(tau), L.ptr(p_i), L.ptr(sigma), L.ptr(sdf_bg), _st(sdf)))
        ctx.cfg = (int(use_bg), float(r_bg), int(white_bkgd), N)
        ctx.save_for_backward(sdf, beta, rad, pts, d_all, sig_bg, rad_bg, d_bg)
        ctx.mark_non_differentiable(p_i, sigma)
        return rgb, depth, acc, tau, sdf_bg, p_i, sigma

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_tau, g_sdf, _gp, _gs):
        sdf, beta, rad, pts, d_all, sig_bg, rad_bg, d_bg = ctx.saved_tensors
        use_bg, r_bg, white, N = ctx.cfg
        R, S = sdf.shape
        c = lambda t: None if t is None else t.contiguous()
        d_sdf, d_rad = torch.empty_like(sdf), torch.empty_like(rad)
        d_beta = torch.empty(R, device=sdf.device)
        d_sig = torch.empty_like(sig_bg) if N else None
        d_rbg = torch.empty_like(rad_bg) if N else None
        lib = L.lib()
        wb = lib.nr_volsdf_composite_bg_bwd_workspace_bytes(R, S, N)
        ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=sdf.device)
        L.check(lib.nr_volsdf_composite_bg_bwd(L.ptr(sdf), L.ptr(pts), L.ptr(beta), L.ptr(rad), L.ptr(d_all), R, S,
                                               use_bg, r_bg, white, L.ptr(sig_bg), L.ptr(rad_bg), L.ptr(d_bg), N,
                                               L.ptr(c(g_rgb)), L.ptr(c(g_depth)), L.ptr(c(g_acc)), L.ptr(c(g_tau)),
                                               L.ptr(c(g_sdf)), L.ptr(d_sdf), L.ptr(d_rad), L.ptr(d_beta),
                                               L.ptr(d_sig), L.ptr(d_rbg), L.ptr(ws), wb, _st(sdf)))
        return (d_sdf, d_beta.sum().reshape(1), d_rad, None, None, None, None, None, d_sig, d_rbg, None)


class UnisurfComposite(torch.autograd.Function):
    """UNISURF's occupancy -> alpha and ray integration (unisurf.py:219-236, :53-62) with a graph:
    logits [R,P] (implicit_surface), radiance [R,P,3]; d_all [R,P] (no grad) -> rgb [R,3], depth [R],
    acc [R], visibility weights [R,P] (+ alpha [R,P], not differentiable)."""

    @staticmethod
    def forward(ctx, logits, rad, d_all, white_bkgd):
        R, P = logits.shape
        dev = logits.device
        logits, rad, d_all = logits.contiguous(), rad.contiguous(), d_all.contiguous()
        rgb = torch.empty(R, 3, device=dev)
        depth = torch.empty(R, device=dev)
        acc = torch.empty(R, device=dev)
        w = torch.empty(R, P, device=dev)
        alpha = torch.empty(R, P, device=dev)
        L.check(L.lib().nr_unisurf_composite_fwd(L.ptr(logits), L.ptr(rad), L.ptr(d_all), R, P, int(white_bkgd),
                                                 L.ptr(rgb), L.ptr(depth), L.ptr(acc), L.ptr(w), L.ptr(alpha),
                                                 _st(logits)))
        ctx.white = int(white_bkgd)
        ctx.save_for_backward(logits, rad, d_all)
        ctx.mark_non_differentiable(alpha)
        return rgb, depth, acc, w, alpha

    @staticmethod
    def backward(ctx, g_rgb, g_depth, g_acc, g_w, _ga):
        logits, rad, d_all = ctx.saved_tensors
        R, P = logits.shape
        c = lambda t: None if t is None else t.contiguous()
        d_lg, d_rad = torch.empty_like(logits), torch.empty_like(rad)
        lib = L.lib()
        wb = lib.nr_unisurf_composite_bwd_workspace_bytes(R, P)
        ws = torch.empty(max(wb, 1), dtype=torch.uint8, device=logits.device)
        L.check(lib.nr_unisurf_composite_bwd(L.ptr(logits), L.ptr(rad), L.ptr(d_all), R, P, ctx.white,
                                             L.ptr(c(g_rgb)), L.ptr(c(g_depth)), L.ptr(c(g_acc)), L.ptr(c(g_w)),
                                             L.ptr(d_lg), L.ptr(d_rad), L.ptr(ws), wb, _st(logits)))
        return d_lg, d_rad, None, None



# ---------------------------------------------------------------------------------------------
# f16x3 training GEMM path (nr_train_gemm)
# ---------------------------------------------------------------------------------------------
# algorithmic HBM bytes of the nr_train_gemm calls issued since the last reset (the training bench's
# roofline: these launches stream [P, <=288] fp32 activations, ~4 B per element read or written)
TG_BYTES = {'bytes': 0.0, 'calls': 0}


def _tg_bytes(P, shape, n1, n2, y, yb, y2, y3, a, g, g_row, zd, dot):
    KB, KB2, NBO, NB2 = shape
    ny, nyb = 16 * (NBO - NB2), 16 * NB2
    cols = n1 + n2                                                       # inputs
    cols += ny * ((y is not None) + (y2 is not None) + (y3 is not None)) + nyb * (yb is not None)  # outputs
    cols += ny * ((a is not None) + (g is not None and not g_row) + (zd is not None))             # epilogue inputs
    cols += dot is not None
    return 4.0 * P * cols


def _tg(op, P, shape, mode, x1, ld1, n1, y, ldy, x2=None, ld2=0, n2=0, bias=True, yscale=1.0, yb=None, ldyb=0,
        y2=None, ldy2=0, y3=None, ldy3=0, a=None, lda=0, g=None, ldg=0, zd=None, ldzd=0, g_row=False, dot=None,
        dot_bias=0.0, head=None, head_bias=None, head_out=None, stream=None, blocked=0, g_scaled=False):
    """one training layer GEMM: shape = (KB, KB2, NBO, NB2) of the packed op at device address `op`"""
    TG_BYTES['bytes'] += _tg_bytes(P, shape, n1, n2, y, yb, y2, y3, a, g, g_row, zd, dot)
    TG_BYTES['calls'] += 1
    def _p(v):  # tensor, raw device address or None
        return None if v is None else (v if isinstance(v, int) else v.data_ptr())
    t = L.NrTrainGemm()
    t.op, t.P = op, P
    t.x1, t.ld1, t.n1 = _p(x1), ld1, n1
    t.x2, t.ld2, t.n2 = _p(x2), ld2, n2
    t.use_bias, t.mode, t.yscale = int(bias), mode, float(yscale)
    t.y, t.ldy, t.yb, t.ldyb = _p(y), ldy, _p(yb), ldyb
    t.y2, t.ldy2, t.y3, t.ldy3 = _p(y2), ldy2, _p(y3), ldy3
    t.a, t.lda, t.g, t.ldg, t.zd, t.ldzd = _p(a), lda, _p(g), ldg, _p(zd), ldzd
    t.g_row, t.dot, t.dot_bias = int(g_row), _p(dot), float(dot_bias)
    t.head, t.head_bias, t.head_out = _p(head), _p(head_bias), _p(head_out)
    t.blocked, t.g_scaled = blocked, int(g_scaled)
    L.check(L.lib().nr_train_gemm(ctypes.byref(t), *shape, stream))


_OPINFO = {}


def _op_info(kind, desc, n_ops):
    """(byte offset, input blocks, output blocks) of every op of a net's render / training pack"""
    key = (kind, tuple(getattr(desc, f) for f, _ in desc._fields_))
    info = _OPINFO.get(key)
    if info is None:
        fn = L.lib().nr_sdf_op_info if kind == 'sdf' else L.lib().nr_radiance_op_info
        info = []
        for i in range(n_ops):
            off, kb, nbo = ctypes.c_int64(), ctypes.c_int(), ctypes.c_int()
            L.check(fn(ctypes.byref(desc), i, ctypes.byref(off), ctypes.byref(kb), ctypes.byref(nbo)))
            info.append((off.value, kb.value, nbo.value))
        _OPINFO[key] = info
    return info


def _train_pack(module, kind, Ws, bs, device):
    """the net's training pack (transposed ops the render pack lacks), cached per parameter version"""
    from .base import _version_key
    key = _version_key(module, 'train', device)
    c = getattr(module, '_nr_train_cache', None)
    if c is not None and c[0] == key:
        return c[1]
    lib = L.lib()
    desc = module.nr_desc()
    nbytes = (lib.nr_sdf_train_packed_bytes if kind == 'sdf' else lib.nr_radiance_train_packed_bytes)(
        ctypes.byref(desc))
    if nbytes == 0:
        raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
    from .base import _ptr_array
    W = [w.detach().float().contiguous() for w in Ws]
    b = [x.detach().float().contiguous() for x in bs]
    packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
    fn = lib.nr_sdf_train_pack if kind == 'sdf' else lib.nr_radiance_train_pack
    L.check(fn(ctypes.byref(desc), _ptr_array(W), _ptr_array(b), L.ptr(packed), L.stream_of(device)))
    module._nr_train_cache = (key, packed, W, b)
    return packed


def _fp32_pack(net, Ws, bs, device):
    """the radiance net's render pack built for exact fp32 products (the NR_PREC_FP32 layout of
    nr_radiance_pack) from the step's effective weights, cached per parameter version: the operand of
    the fp32 training forward (nr_radiance_train_fwd32)"""
    from .base import _version_key, _ptr_array
    key = _version_key(net, 'fp32pack', device)
    c = getattr(net, '_nr_fp32_cache', None)
    if c is not None and c[0] == key:
        return c[1], c[2]
    lib = L.lib()
    desc = net.nr_desc()
    desc.precision = L.PREC_FP32
    nbytes = lib.nr_radiance_packed_bytes(ctypes.byref(desc))
    if nbytes == 0:
        raise NotImplementedError('neurecon_amd: ' + lib.nr_last_error().decode())
    W = [w.detach().float().contiguous() for w in Ws]
    b = [x.detach().float().contiguous() for x in bs]
    packed = torch.empty(nbytes, dtype=torch.uint8, device=device)
    L.check(lib.nr_radiance_pack(ctypes.byref(desc), _ptr_array(W), _ptr_array(b), L.ptr(packed), L.stream_of(device)))
    net._nr_fp32_cache = (key, desc, packed, W, b)
    return desc, packed


def uses_train_gemm(module):
    """f16x3 softplus SDF nets (D=8, skip 4) and f16x3 ReLU radiance nets with D=4 train on nr_train_gemm"""
    if getattr(module, 'precision', 'fp32') != 'f16x3' or getattr(module, 'use_siren', False):
        return False
    if hasattr(module, 'surface_fc_layers'):  # the render pack's SDF shape (check_sdf_desc, nr_capi.hip)
        return (module.D == 8 and list(module.skips) == [4] and module.W == 256 and module.W_geo_feat == 256
                and module.embed_multires == 6)
    # the render pack's radiance shape (check_rad_desc) with RadianceTG's D = 4
    return (module.D == 4 and module.W == 256 and module.W_geo_feat == 256 and module.embed_multires < 0
            and module.embed_multires_view <= 7)


def _pad16(n):
    return 16 * ((n + 15) // 16)


def _blk_on(P, row0=0):
    """whether a training step stores its layer tensors 16 x 16 blocked: not when P (or a row offset
    row0 the caller addresses) is not a multiple of 16 (the blocked layout tiles whole 16-point
    blocks) or NR_TRAIN_BLOCKED=0 (row-major everywhere: the bit-identity test's reference).  Decided
    once per forward and kept on the autograd context: backward reads what forward wrote."""
    return P % 16 == 0 and row0 % 16 == 0 and os.environ.get('NR_TRAIN_BLOCKED', '1') != '0'


def _blk_bits(on):
    """NrTrainGemm.blocked bits from role names (all 0 when the layout is row-major)"""
    return lambda roles: sum(getattr(L, 'BLK_' + r) for r in roles) if on else 0


def _WG_BLK(a_blocked, b_blocked):
    """NrWgrad.blocked bits for operand pairs whose A (resp. B) operands are all blocked or all not"""
    return (L.WG_BLK_A0 | L.WG_BLK_A1) * bool(a_blocked) | (L.WG_BLK_B0 | L.WG_BLK_B1) * bool(b_blocked)


class SdfNablaTG(torch.autograd.Function):
    """SdfNabla on nr_train_gemm (f16x3 softplus nets, D=8, skip at layer 4, W=256): the same recipe
    (nr_train.hip header) with every layer product an op of the render pack (F0..F8 forward, B7..B0
    transposed) or the training pack (B8 = W8^T), and the elementwise steps in the GEMM epilogues:
      primal   F_l: h_l, s_l = softplus100 / softplus'(W_l hin_l + b_l); F7 also delta_7 = s_7 W8[0, :]
               and sdf = h_7 . W8[0, :] + b8;  F8: feature
      nabla    B_l: g_{l-1} = W_l^T delta_l, delta_{l-1} = s_{l-1} g_{l-1} (only delta stored); B4 splits
               [g_3 ; e_skip];
               B0: e_first;  nabla = J_emb^T (e_first + e_skip)
      tangent  F_l (no bias): zdot_l = W_l hdot_in_l, hdot_l = s_l zdot_l
      adjoint  B8 then B7..B1: zbar_{l-1} = (W_l^T zbar_l) s_{l-1} + delta_{l-1} zdot_{l-1} 100 (1 - s)
               (= g zdot 100 s (1 - s), torch's softplus double backward)
    Activations are [P, 16-column blocks] (217-wide layer-3 tensors padded to 224, the embedding to
    64); the layer tensors (H, S, delta, G, ZD, HD, Z) are stored 16 x 16 blocked when P % 16 == 0
    (include/neurecon_hip.h NR_BLK_*: one contiguous 1 KB run per wave-instruction of the GEMM epilogues
    and the weight-gradient loaders, instead of 16 rows x 64 B), the embedding tensors, the feature and
    hdot_7 (a torch-side column sum) row-major.  Weight gradients: dW_l = zbar_l^T hin_l + delta_l^T
    hdot_in_l (nr_wgrad)."""

    @staticmethod
    def forward(ctx, x, surface, want_feat, feat_from, *params):
        D = 8
        Ws, bs = params[:D + 1], params[D + 1:]
        dev = x.device
        st = L.stream_of(dev)
        x = x.contiguous()
        P = x.shape[0]
        assert 0 <= feat_from <= P or not want_feat
        desc, packed = surface.nr_packed(dev)
        info = _op_info('sdf', desc, 18)
        base = packed.data_ptr()
        op = lambda i: base + info[i][0]
        shp = lambda i, kb2=0, nb2=0: (info[i][1], kb2, info[i][2], nb2)
        nf = surface.input_ch                      # 39
        h0 = torch.empty(P, 64, device=dev)
        L.check(L.lib().nr_embed_padded(L.ptr(x), P, surface.embed_multires, L.ptr(h0), 64, st))
        wd = [256, 256, 256, 224, 256, 256, 256, 256]   # padded widths of the layer outputs h_l
        nv = [256, 256, 256, 217, 256, 256, 256, 256]
        H = [torch.empty(P, wd[l], device=dev) for l in range(D)]
        S = [torch.empty(P, wd[l], device=dev) for l in range(D)]
        sdf = torch.empty(P, device=dev)
        delta = [None] * D
        delta[7] = torch.empty(P, 256, device=dev)
        ctx.blk_on = _blk_on(P, feat_from)
        bk = _blk_bits(ctx.blk_on)
        for l in range(D):                                                 # F0..F7
            if l == 0:
                xin = dict(x1=h0, ld1=64, n1=nf)
            elif l == 4:
                xin = dict(x1=H[3], ld1=224, n1=217, x2=h0, ld2=64, n2=nf)
            else:
                xin = dict(x1=H[l - 1], ld1=wd[l - 1], n1=nv[l - 1])
            extra = dict(y3=delta[7], ldy3=256, dot=sdf) if l == 7 else {}
            _tg(op(l), P, shp(l, 4 if l == 4 else 0), L.TG_SOFTPLUS, y=H[l], ldy=wd[l], y2=S[l], ldy2=wd[l],
                stream=st, blocked=bk(('X1',) * (l > 0) + ('Y', 'Y2') + ('Y3',) * (l == 7)), **xin, **extra)
        sdf.add_(bs[D].detach()[0])                                        # + b8 (no host sync)
        feat = None
        if want_feat:                                                      # F8 on points [feat_from, P)
            feat = torch.empty(P - feat_from, 256, device=dev)
            _tg(op(8), P - feat_from, shp(8), L.TG_NONE, H[7].data_ptr() + feat_from * 256 * 4, 256, 256, feat, 256,
                stream=st, blocked=bk(('X1',)))  # a row offset of a multiple of 16: the same in both layouts
        # g_l = d sdf / d h_l (l < 7) is not stored: only delta_l = s_l g_l is, and the adjoint's
        # g zdot s' term reads delta (NrTrainGemm.g_scaled: s' / s = 100 (1 - s))
        for l in range(D - 1, 0, -1):                                      # B7..B1: op index 16 - l
            i = 16 - l
            delta[l - 1] = torch.empty(P, wd[l - 1], device=dev)
            if l == 4:  # [g_3 (14 blocks, not stored) ; e_skip (4 blocks)]
                e_skip = torch.empty(P, 64, device=dev)
                _tg(op(i), P, shp(i, 0, 4), L.TG_MUL, delta[4], 256, 256, None, 0, yb=e_skip, ldyb=64,
                    y2=delta[3], ldy2=224, a=S[3], lda=224, stream=st, blocked=bk(('X1', 'Y2', 'A')))
            else:
                _tg(op(i), P, shp(i), L.TG_MUL, delta[l], wd[l], nv[l], None, 0, y2=delta[l - 1],
                    ldy2=wd[l - 1], a=S[l - 1], lda=wd[l - 1], stream=st, blocked=bk(('X1', 'Y2', 'A')))
        e_first = torch.empty(P, 64, device=dev)                           # B0
        _tg(op(16), P, shp(16), L.TG_NONE, delta[0], 256, 256, e_first, 64, stream=st, blocked=bk(('X1',)))
        nab = torch.empty(P, 3, device=dev)
        L.check(L.lib().nr_embed_vjp(L.ptr(x), L.ptr(e_first), 64, L.ptr(e_skip), 64, 1.0, P, surface.embed_multires,
                                     L.ptr(nab), st))
        ctx.surface = surface
        ctx.want_feat = want_feat
        ctx.feat_from = feat_from
        ctx.save_for_backward(x, h0, *H, *S, *delta, *Ws, *bs)
        return (sdf, nab, feat) if want_feat else (sdf, nab)

    @staticmethod
    def backward(ctx, g_sdf, g_nab, *rest):
        D = 8
        saved = ctx.saved_tensors
        x, h0 = saved[0], saved[1]
        H = saved[2:2 + D]
        S = saved[2 + D:2 + 2 * D]
        delta = saved[2 + 2 * D:2 + 3 * D]
        Ws = saved[2 + 3 * D:2 + 3 * D + D + 1]
        surface = ctx.surface
        g_feat = rest[0] if ctx.want_feat else None
        dev = x.device
        st = L.stream_of(dev)
        P = x.shape[0]
        desc, packed = surface.nr_packed(dev)
        info = _op_info('sdf', desc, 18)
        base = packed.data_ptr()
        op = lambda i: base + info[i][0]
        shp = lambda i, kb2=0, nb2=0: (info[i][1], kb2, info[i][2], nb2)
        nf = surface.input_ch
        wd = [256, 256, 256, 224, 256, 256, 256, 256]
        nv = [256, 256, 256, 217, 256, 256, 256, 256]
        tangent = g_nab is not None
        bk = _blk_bits(ctx.blk_on)  # the layout forward wrote
        wb = _WG_BLK if bk(('Y',)) else (lambda a, b: 0)
        ZD = [None] * D
        HD = [None] * D                                                   # hdot_l = s_l zdot_l
        hd0 = None
        if tangent:
            hd0 = torch.empty(P, 64, device=dev)
            L.check(L.lib().nr_embed_jvp_padded(L.ptr(x), L.ptr(g_nab.contiguous()), P, surface.embed_multires,
                                                L.ptr(hd0), 64, st))
            for l in range(D):
                if l == 0:
                    xin = dict(x1=hd0, ld1=64, n1=nf)
                elif l == 4:
                    xin = dict(x1=HD[3], ld1=224, n1=217, x2=hd0, ld2=64, n2=nf)
                else:
                    xin = dict(x1=HD[l - 1], ld1=wd[l - 1], n1=nv[l - 1])
                ZD[l] = torch.empty(P, wd[l], device=dev)
                HD[l] = torch.empty(P, wd[l], device=dev)
                # hdot_7 stays row-major: its consumer is the torch-side column sum of dW8[0]
                _tg(op(l), P, shp(l, 4 if l == 4 else 0), L.TG_MUL, y=ZD[l], ldy=wd[l], y2=HD[l], ldy2=wd[l],
                    a=S[l], lda=wd[l], bias=False, stream=st,
                    blocked=bk(('X1',) * (l > 0) + ('Y', 'A') + ('Y2',) * (l < 7)), **xin)
        # output-layer adjoint ob = [d sdf, d feature] -> zbar_7 through B8 = W8^T (training pack)
        Wl = [surface.surface_fc_layers[i] for i in range(D + 1)]
        tp = _train_pack(surface, 'sdf', Ws, [l.bias for l in Wl], dev)  # the forward's effective weights
        gs = torch.zeros(P, device=dev) if g_sdf is None else g_sdf.contiguous()
        if g_feat is None:
            gf = torch.zeros(P, 256, device=dev)
        elif ctx.feat_from:  # no feature (zero gradient) on the points before feat_from
            gf = torch.empty(P, 256, device=dev)
            gf[:ctx.feat_from].zero_()
            gf[ctx.feat_from:].copy_(g_feat)
        else:
            gf = g_feat.contiguous()
        Z = [None] * D
        Z[7] = torch.empty(P, 256, device=dev)
        _tg(tp.data_ptr() + info[17][0], P, (18, 2, 16, 0), L.TG_SPADJ, gf, 256, 256, Z[7], 256, x2=gs, ld2=1, n2=1,
            a=S[7], lda=256, zd=ZD[7], ldzd=256, g_row=tangent, stream=st,
            blocked=bk(('Y', 'A') + ('ZD',) * tangent))
        for l in range(D - 1, 0, -1):                                      # B7..B1 -> zbar_{l-1}
            i = 16 - l
            Z[l - 1] = torch.empty(P, wd[l - 1], device=dev)
            gz = dict(g=delta[l - 1], ldg=wd[l - 1], g_scaled=True, zd=ZD[l - 1], ldzd=wd[l - 1]) if tangent else {}
            _tg(op(i), P, shp(i, 0, 4 if l == 4 else 0), L.TG_SPADJ, Z[l], wd[l], nv[l], Z[l - 1], wd[l - 1],
                a=S[l - 1], lda=wd[l - 1], stream=st, blocked=bk(('X1', 'Y', 'A') + ('G', 'ZD') * tangent), **gz)
        # weight gradients on nr_wgrad (f16x3 MFMA): dW_l = zbar_l^T hin_l + delta_l^T hdot_in_l (one
        # launch for both sweeps), db_l = sum_p zbar_l fused into it
        dW, db = [None] * (D + 1), [None] * (D + 1)
        dW[D] = torch.empty(257, 256, device=dev)  # rows [d sdf ; d feature] x h7
        db[D] = torch.empty(257, device=dev)
        if g_feat is not None:
            _wg([(gf, H[7])], out=dW[D][1:], colsum=db[D][1:], avec=gs, vec=dW[D][0], blocked=wb(False, True))
        else:  # no feature gradient: only the sdf row
            dW[D][1:].zero_()
            db[D][1:].zero_()
            _wg([(gs[:, None], H[7])], out=dW[D][:1], blocked=wb(False, True))
        db[D][:1] = _colsum(gs[:, None])
        if tangent:
            dW[D][0] += _colsum(HD[7])
        for l in range(D):
            zb = Z[l][:, :nv[l]]
            db[l] = torch.empty(nv[l], device=dev)
            if l == 0:
                pr = [(zb, h0[:, :nf])] + ([(delta[0][:, :nv[0]], hd0[:, :nf])] if tangent else [])
                dW[0] = _wg(pr, colsum=db[0], blocked=wb(True, False))
            elif l == 4:  # the skip layer's input cat([h3, embed(x)]) / sqrt(2) (base.py:250): per column block
                dW[4] = torch.empty(256, 217 + nf, device=dev)
                _wg([(zb, H[3][:, :217])] + ([(delta[4][:, :nv[4]], HD[3][:, :217])] if tangent else []),
                    out=dW[4][:, :217], scale=_ISQ2, colsum=db[4], blocked=wb(True, True))
                _wg([(zb, h0[:, :nf])] + ([(delta[4][:, :nv[4]], hd0[:, :nf])] if tangent else []),
                    out=dW[4][:, 217:], scale=_ISQ2, blocked=wb(True, False))
            else:
                hin = H[l - 1][:, :nv[l - 1]]
                pr = [(zb, hin)] + ([(delta[l][:, :nv[l]], HD[l - 1][:, :nv[l - 1]])] if tangent else [])
                dW[l] = _wg(pr, colsum=db[l], blocked=wb(True, True))
        return (None, None, None, None, *dW, *db)


class RadianceTG(torch.autograd.Function):
    """RadianceFn with the backward on nr_train_gemm (f16x3 ReLU nets, D=4): head^T and W3^T..W1^T of
    the training pack with the ReLU mask in the epilogue, W0^T split into d feature / d small inputs
    (-> d normals); weight gradients on nr_wgrad.  The forward keeps exact fp32 products: ReLU'(z) is
    a step, and the f16x3 forward's ~5e-7 relative error in z flips a few masks per step against the
    reference's fp32 z -- each flip moves one point's whole contribution to the gradients of every
    earlier layer (measured: layer-2 bias gradient 3.8e-4 off the float64 truth with the f16x3
    forward, 9e-8 with the fp32 one; tools/train_diag.py --probe).  r05: that fp32 forward is one
    launch of nr_radiance_train_fwd32 (the four layers chained in registers on v_mfma_f32_16x16x4_f32
    over the net's fp32 pack, every h_l stored, sigmoid head) instead of four hipBLASLt GEMMs, their
    ReLU launches and the head.  The backward has no such decision."""

    @staticmethod
    def forward(ctx, x, v, nrm, feat, net, *params):
        Ws, bs = params[:5], params[5:]
        P = x.shape[0]
        view = net.use_view_dirs
        nfv = net.embed_multires_view
        nvw = (3 if nfv < 0 else 3 + 6 * nfv) if view else 0
        ns = 3 + nvw + (3 if view else 0)
        inp = torch.empty(P, ns + 256, device=x.device)  # [x, embed_view(v), normals, feature] (base.py:383-386)
        L.check(L.lib().nr_radiance_input(L.ptr(x), L.ptr(v), L.ptr(nrm), L.ptr(feat), P, nfv, int(view), 256,
                                          L.ptr(inp), _st(x)))
        desc32, pk32 = _fp32_pack(net, Ws, bs, x.device)
        H = [torch.empty(P, 256, device=x.device) for _ in range(4)]
        rgb = torch.empty(P, 3, device=x.device)
        feat = feat.contiguous()
        L.check(L.lib().nr_radiance_train_fwd32(ctypes.byref(desc32), L.ptr(pk32), L.ptr(feat), L.ptr(inp), ns + 256, P,
                                                *[L.ptr(h) for h in H], L.ptr(rgb), _st(x)))
        ctx.net = net
        ctx.cfg = (ns, nvw, view)
        ctx.save_for_backward(rgb, inp, *H, *Ws)
        return rgb

    @staticmethod
    def backward(ctx, gy):
        ns, nvw, view = ctx.cfg
        net = ctx.net
        saved = ctx.saved_tensors
        rgb, inp = saved[:2]
        H = saved[2:6]
        dev = rgb.device
        st = L.stream_of(dev)
        P = rgb.shape[0]
        desc = net.nr_desc()  # the layout only (no render pack)
        info = _op_info('rad', desc, 10)
        tp = _train_pack(net, 'rad', saved[6:11], [l.bias for l in net.layers], dev)  # the forward's effective weights
        tb = tp.data_ptr()
        g = gy.contiguous().clone()
        L.check(L.lib().nr_activation(L.ptr(rgb), L.ptr(g), g.numel(), 3, st))  # sigmoid'
        dW, db = [None] * 5, [None] * 5
        db[4] = torch.empty(3, device=dev)
        dW[4] = _wg([(g, H[3])], colsum=db[4])      # weight gradients on nr_wgrad (bias gradient fused)
        # the pre-activation adjoints gz stay inside this function: 16 x 16 blocked (SdfNablaTG's note)
        bk = _blk_bits(_blk_on(P))  # gz is written and read inside this backward
        wb = _WG_BLK if bk(('Y',)) else (lambda a, b: 0)
        gz = torch.empty(P, 256, device=dev)
        _tg(tb + info[5][0], P, (2, 0, 16, 0), L.TG_RELUMASK, g, 3, 3, gz, 256, bias=False, a=H[3], lda=256, stream=st,
            blocked=bk(('Y',)))
        for l in range(3, 0, -1):  # gz = d z_l  ->  d z_{l-1} through W_l^T (training ops 6, 7, 8)
            db[l] = torch.empty(256, device=dev)
            dW[l] = _wg([(gz, H[l - 1])], colsum=db[l], blocked=wb(True, False))
            gn = torch.empty(P, 256, device=dev)
            _tg(tb + info[5 + (4 - l)][0], P, (16, 0, 16, 0), L.TG_RELUMASK, gz, 256, 256, gn, 256, bias=False,
                a=H[l - 1], lda=256, stream=st, blocked=bk(('X1', 'Y')))
            gz = gn
        db[0] = torch.empty(256, device=dev)
        dW[0] = _wg([(gz, inp)], colsum=db[0], blocked=wb(True, False))  # W0 columns [small | feature], as inp
        nbo0 = info[9][2]
        d_feat = torch.empty(P, 256, device=dev)
        d_small = torch.empty(P, 16 * (nbo0 - 16), device=dev)
        _tg(tb + info[9][0], P, (16, 0, nbo0, nbo0 - 16), L.TG_NONE, gz, 256, 256, d_feat, 256, bias=False,
            yb=d_small, ldyb=16 * (nbo0 - 16), stream=st, blocked=bk(('X1',)))
        d_nrm = d_small[:, 3 + nvw:3 + nvw + 3].contiguous() if view else None
        return (None, None, d_nrm, d_feat, None, *dW, *db)


def nerf(net, x_emb, v_emb):
    """Differentiable (sigma [P], rgb [P,3]) of a neurecon_amd NeRF background net (the NeRF++
    configuration, NeRF.nr_desc)."""
    layers = list(net.pts_linears) + [net.feature_linear, net.views_linears[0], net.alpha_linear, net.rgb_linear]
    return NeRFFn.apply(x_emb, v_emb, net, *[l.weight for l in layers], *[l.bias for l in layers])


class _WeightNormAll(torch.autograd.Function):
    """torch._weight_norm(v, g, 0) (base.py:118-129, 226-227) of a net's layers in one nr_weight_norm_fwd
    launch, the backward in one nr_weight_norm_bwd launch (torch: one weight_norm_fwd / _bwd_first_dim
    launch per layer, ~5 us each; 28 per NeuS training step)"""

    @staticmethod
    def forward(ctx, n, *vg):
        vs = [v.contiguous() for v in vg[:n]]
        gs = [g.contiguous() for g in vg[n:]]
        dev = vs[0].device
        ws = [torch.empty_like(v) for v in vs]
        norms = [torch.empty(v.shape[0], device=dev) for v in vs]
        arr = (L.NrWnLayer * n)()
        for i in range(n):
            arr[i].v, arr[i].g, arr[i].w, arr[i].norm = L.ptr(vs[i]), L.ptr(gs[i]), L.ptr(ws[i]), L.ptr(norms[i])
            arr[i].rows, arr[i].cols = vs[i].shape
        L.check(L.lib().nr_weight_norm_fwd(arr, n, _st(vs[0])))
        ctx.n = n
        ctx.save_for_backward(*vs, *gs, *norms)
        return tuple(ws)

    @staticmethod
    def backward(ctx, *gws):
        n = ctx.n
        sv = ctx.saved_tensors
        vs, gs, norms = sv[:n], sv[n:2 * n], sv[2 * n:]
        gv = [torch.empty_like(v) for v in vs]
        gg = [torch.empty_like(g) for g in gs]
        gw = [None if t is None else t.contiguous() for t in gws]
        arr = (L.NrWnLayer * n)()
        for i in range(n):
            arr[i].v, arr[i].g, arr[i].norm = L.ptr(vs[i]), L.ptr(gs[i]), L.ptr(norms[i])
            arr[i].grad_w = None if gw[i] is None else L.ptr(gw[i])
            arr[i].grad_v, arr[i].grad_g = L.ptr(gv[i]), L.ptr(gg[i])
            arr[i].rows, arr[i].cols = vs[i].shape
        L.check(L.lib().nr_weight_norm_bwd(arr, n, _st(vs[0])))
        return (None, *gv, *gg)


def weight_norm_all(layers):
    """[l.effective_weight() for l in layers] (weight-normed WNLinear layers) with one launch each way"""
    ls = list(layers)
    if len(ls) > L.WN_MAX:
        return [l.effective_weight() for l in ls]
    return list(_WeightNormAll.apply(len(ls), *[l.weight_v for l in ls], *[l.weight_g for l in ls]))


def effective_weights(surface):
    """The SDF layers' weight-normed weights (differentiable), to share between evaluations of one step"""
    return weight_norm_all(surface.surface_fc_layers)


def sdf_nablas(surface, x, want_feat, Ws=None, feat_from=0):
    """Differentiable (sdf, nablas, feature) of a neurecon_amd ImplicitSurface at points x [P,3]
    (Ws: effective_weights(surface) of this step, computed here when not given).  feat_from (the
    nr_train_gemm path only): the feature is computed for points [feat_from, P) only, so one call can
    evaluate two point sets that need it and do not (NeuS's samples and mid-points)."""
    if Ws is None:
        Ws = effective_weights(surface)
    bs = [l.bias for l in surface.surface_fc_layers]
    if uses_train_gemm(surface):
        out = SdfNablaTG.apply(x.reshape(-1, 3).float().contiguous(), surface, bool(want_feat), int(feat_from),
                               *Ws, *bs)
        return out if want_feat else (out[0], out[1], None)
    assert feat_from == 0, 'feat_from: nr_train_gemm path only'
    cfg = (surface.D, tuple(surface.skips), surface.embed_multires, bool(want_feat), bool(surface.use_siren))
    out = SdfNabla.apply(x.reshape(-1, 3).float().contiguous(), cfg, *Ws, *bs)
    return out if want_feat else (out[0], out[1], None)


def radiance(net, x, v, nrm, feat):
    Ws = weight_norm_all(net.layers)
    bs = [l.bias for l in net.layers]
    view = net.use_view_dirs
    if uses_train_gemm(net):
        return RadianceTG.apply(x.contiguous(), v.contiguous() if view else None, nrm.contiguous() if view else None,
                                feat.contiguous(), net, *Ws, *bs)
    return RadianceFn.apply(x.contiguous(), v.contiguous() if view else None, nrm.contiguous() if view else None,
                            feat.contiguous(), (net.D, net.embed_multires_view, view, bool(net.use_siren)), *Ws, *bs)
