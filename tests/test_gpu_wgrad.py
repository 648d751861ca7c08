"""GPU parity of the training step's weight-gradient kernel (nr_wgrad, f16x3 MFMA): the DenseLayer
weight gradients autograd forms as mm(grad_out^T, input) (models/base.py:118-129 under the double
backward of base.py:265-282, train.py:205), on the shapes the NeuS training step hands it -- aligned
256 x 256 layers, both sweeps of a layer in one call, the 217-wide layer and the 39-wide embedding in
padded buffers, the 3-row colour head, the 289-column radiance input (unaligned rows), an extra
vector row (the sdf row of the output layer), the fused bias gradient, ragged P.

Bar: element-wise |hip - f64| <= |torch fp32 - f64| + 2e-6 max|f64| (the kernel is no further from
the float64 truth than the fp32 GEMM, up to 2e-6 of the output's scale), bias gradients and the vector
row 1e-5 relative; results are bit-identical across calls (fixed-order reduction)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    from neurecon_amd import _lib
    _lib.lib()


def _mk(P, cols, ld, g, scale=1.0, heavy=False):
    t = torch.randn(P, ld, generator=g) * scale
    if heavy:  # gradients of a training step: a few large entries over many small ones
        t = t * torch.exp(2.0 * torch.randn(P, ld, generator=g))
    return t.cuda()[:, :cols]


CASES = {
    # name: (P, m, lda, n, ldb, npairs)
    'layer_256x256': (65536, 256, 256, 256, 256, 1),
    'layer_two_sweeps': (65536, 256, 256, 256, 256, 2),
    'layer3_217': (65536, 217, 224, 256, 256, 2),
    'skip_h3_217': (65536, 256, 256, 217, 224, 2),
    'first_embed_39': (65536, 256, 256, 39, 64, 2),
    'head_3': (65024, 3, 3, 256, 256, 1),
    'radiance_in_289': (65024, 256, 256, 289, 289, 1),
    'ragged_P': (1000, 256, 256, 256, 256, 2),
    'tiny_P': (33, 17, 17, 5, 5, 1),
}


@pytest.mark.parametrize('fp32', [False, True], ids=['f16x3', 'fp32'])
@pytest.mark.parametrize('name', list(CASES))
def test_wgrad_vs_float64(name, fp32):
    """both product modes: f16x3 (the default nets) and exact fp32 products (NrWgrad.fp32, the fp32 nets'
    training path in place of hipBLASLt's split-K GEMMs)"""
    from neurecon_amd.training import _wg
    P, m, lda, n, ldb, npairs = CASES[name]
    g = torch.Generator().manual_seed(sum(map(ord, name)))
    pairs = [(_mk(P, m, lda, g, heavy=True), _mk(P, n, ldb, g, scale=0.3)) for _ in range(npairs)]
    cs = torch.empty(m, device='cuda')
    out = _wg(pairs, colsum=cs, scale=0.5, fp32=fp32)
    out2 = _wg(pairs, colsum=torch.empty(m, device='cuda'), scale=0.5, fp32=fp32)
    torch.cuda.synchronize()
    assert torch.equal(out, out2), 'not deterministic'
    ref64 = sum(a.double().t() @ b.double() for a, b in pairs) * 0.5
    ref32 = sum(a.t() @ b for a, b in pairs) * 0.5
    scale = float(ref64.abs().max())
    e_hip = (out.double() - ref64).abs()
    e_32 = (ref32.double() - ref64).abs()
    print(f'{name} [{"fp32" if fp32 else "f16x3"}]: max |hip - f64| {float(e_hip.max()) / scale:.2e}, max |fp32 GEMM - f64| '
          f'{float(e_32.max()) / scale:.2e} (of max |C| = {scale:.3e})')
    assert bool((e_hip <= e_32 + 2e-6 * scale).all()), float((e_hip - e_32).max()) / scale
    cref = pairs[0][0].double().sum(0)
    assert torch.allclose(cs.double(), cref, rtol=1e-5, atol=1e-5 * float(cref.abs().max())), 'column sums'


def test_wgrad_vector_row_and_views():
    """the output layer's [d sdf ; d feature] x h7: the sdf row through the vector option, the feature
    rows written into a row range of the gradient; the skip layer's two column blocks scaled 1/sqrt(2)
    written into column ranges of one output"""
    from neurecon_amd.training import _wg
    g = torch.Generator().manual_seed(7)
    P = 65536
    gs, gf, h7 = _mk(P, 1, 1, g, heavy=True)[:, 0].contiguous(), _mk(P, 256, 256, g, heavy=True), _mk(P, 256, 256, g)
    dW = torch.full((257, 256), float('nan'), device='cuda')
    db = torch.empty(257, device='cuda')
    _wg([(gf, h7)], out=dW[1:], colsum=db[1:], avec=gs, vec=dW[0])
    ref = torch.cat([gs[:, None], gf], 1).double().t() @ h7.double()
    sc = float(ref.abs().max())
    assert float((dW.double() - ref).abs().max()) <= 1e-5 * sc
    assert torch.allclose(db[1:].double(), gf.double().sum(0), rtol=1e-5, atol=1e-5 * float(gf.abs().sum(0).max()))
    zb, h3, h0 = _mk(P, 256, 256, g, heavy=True), _mk(P, 217, 224, g), _mk(P, 39, 64, g)
    out = torch.full((256, 256), float('nan'), device='cuda')
    _wg([(zb, h3)], out=out[:, :217], scale=0.5 ** 0.5)
    _wg([(zb, h0)], out=out[:, 217:], scale=0.5 ** 0.5)
    ref = (zb.double().t() @ torch.cat([h3, h0], 1).double()) * 0.5 ** 0.5
    assert not torch.isnan(out).any()
    assert float((out.double() - ref).abs().max()) <= 1e-5 * float(ref.abs().max())


def test_wgrad_timing_vs_hipblaslt():
    """device time of one 65536 x 256 x 256 weight gradient (both sweeps) on nr_wgrad vs the split-K
    fp32 batched GEMM + sum it replaces (hipBLASLt)"""
    from neurecon_amd.training import _wg, _wgrad, _wgrad2
    g = torch.Generator().manual_seed(3)
    P = 65536
    a1, b1, a2, b2 = (_mk(P, 256, 256, g) for _ in range(4))
    cs = torch.empty(256, device='cuda')

    def t(fn, reps=20):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps * 1e3
    us_hip = t(lambda: _wg([(a1, b1), (a2, b2)], colsum=cs))
    us_blas = t(lambda: _wgrad2(a1, b1, a2, b2))
    us_hip1 = t(lambda: _wg([(a1, b1)], colsum=cs))
    us_blas1 = t(lambda: _wgrad(a1, b1))
    gb = 4 * P * 256 * 4 / 1e9
    print(f'weight gradient, 2 x [65536, 256]^T [65536, 256]: nr_wgrad {us_hip:.1f} us ({gb / us_hip * 1e6 / 1e3:.2f} TB/s '
          f'of operands, bias gradient fused), hipBLASLt split-K bmm + sum {us_blas:.1f} us; one pair: nr_wgrad '
          f'{us_hip1:.1f} us, hipBLASLt {us_blas1:.1f} us')


def test_wgrad_tiny_and_zero_quads():
    """column quads whose values are all zero, tiny (1e-30, below the scale cap) or denormal in some
    32-row blocks (adjoints of points the loss does not see): finite results equal to the float64 product
    up to the tiny values' share"""
    from neurecon_amd.training import _wg
    g = torch.Generator().manual_seed(11)
    P = 4096
    a = torch.randn(P, 256, generator=g)
    b = torch.randn(P, 256, generator=g)
    a[:, 4:8] = 0.0                      # a zero quad
    a[:64, 8:12] *= 1e-30                # tiny in two k-steps, normal elsewhere
    a[:, 12:16] = 1e-40                  # denormal everywhere
    b[32:96, 16:20] = 0.0
    b[:, 20:24] *= 1e-35
    a, b = a.cuda(), b.cuda()
    out = _wg([(a, b)])
    torch.cuda.synchronize()
    assert torch.isfinite(out).all()
    ref = a.double().t() @ b.double()
    sc = float(ref.abs().max())
    assert float((out.double() - ref).abs().max()) <= 1e-5 * sc


def _blocked(t):
    """the 16 x 16 blocked storage (include/neurecon_hip.h NR_BLK_*) of a row-major [P, C] tensor, as a
    [P, C]-shaped tensor whose memory is in blocked order"""
    P, C = t.shape
    return t.reshape(P // 16, 16, C // 16, 16).permute(0, 2, 1, 3).contiguous().reshape(P, C)


@pytest.mark.parametrize('m, lda, n, ldb, npairs', [(256, 256, 256, 256, 2), (217, 224, 256, 256, 2),
                                                    (256, 256, 217, 224, 1), (256, 256, 39, 64, 2)])
def test_wgrad_blocked_operands_bit_identical(m, lda, n, ldb, npairs):
    """operands in the 16 x 16 blocked layout give bit-identical results to the same operands
    row-major (only the addressing differs), A and B blocked independently; column views [:, :n] of a
    blocked tensor keep the pointer and leading dimension the kernel needs"""
    from neurecon_amd import _lib as L
    from neurecon_amd.training import _wg
    g = torch.Generator().manual_seed(m + n)
    P = 4096 + 48
    A = [_mk(P, lda, lda, g, heavy=True) for _ in range(npairs)]
    B = [_mk(P, ldb, ldb, g) for _ in range(npairs)]
    ref = _wg([(a[:, :m], b[:, :n]) for a, b in zip(A, B)], colsum=(cs0 := torch.empty(m, device='cuda')))
    for ba, bb in ((True, False), (False, True), (True, True)):
        AA = [_blocked(a) if ba else a for a in A]
        BB = [_blocked(b) if bb else b for b in B]
        bits = (L.WG_BLK_A0 | L.WG_BLK_A1) * ba | (L.WG_BLK_B0 | L.WG_BLK_B1) * bb
        cs = torch.empty(m, device='cuda')
        out = _wg([(a[:, :m], b[:, :n]) for a, b in zip(AA, BB)], colsum=cs, blocked=bits)
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (ba, bb, float((out - ref).abs().max()))
        assert torch.equal(cs, cs0), (ba, bb)
