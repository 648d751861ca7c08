"""nr_gemm32: the layer products of the fp32 / SIREN nets' training step (nn.Linear's addmm and its
autograd's mm, models/base.py:118-129, 243-282), against float64.

Default mode: exact fp32 products accumulated in fp64 (v_mfma_f64_16x16x4_f64) and rounded once, then
the bias added: every element within one rounding of the float64 dot product plus the bias addition's
(2^-24 (|dot| + |C|) element-wise), i.e. at least as close to float64 as any fp32 GEMM.  acc32 mode: an
fp32 fmaf chain over k in order (v_mfma_f32_16x16x4_f32), held to the fp32 dot-product bound
K u sum_k |a_k b_k| (u = 2^-24) and to within 3x (max) / 2x (mean) of torch's fp32 product's error.
Shapes: the training step's (P = 65 k rows, K in {39, 217, 256, 257, 289}, N in {3, 39, 217, 256,
257}), ragged tiles, row strides wider than K (column views of a wider tensor), with and without bias,
both operand orientations."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module', autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')


def _check(a, w, bias, trans, tag):
    from neurecon_amd.training import _mm
    wt = w.t() if trans else w
    dot64 = a.double() @ wt.double()
    ref64 = dot64 + (bias.double() if bias is not None else 0.0)
    ref32 = torch.addmm(bias, a, wt) if bias is not None else a @ wt
    e32 = (ref32.double() - ref64).abs()
    # default: fp64 accumulation, one rounding of the dot product (+ one of the bias addition)
    got = _mm(a, w, bias, trans=trans)
    e = (got.double() - ref64).abs()
    bound = 2.0 ** -24 * (dot64.abs() + ref64.abs()) + 1e-38
    print(f'{tag}: max |gemm32 - f64| {float(e.max()):.3e} (torch fp32 {float(e32.max()):.3e}), mean '
          f'{float(e.mean()):.3e} ({float(e32.mean()):.3e}), max error / one-rounding bound {float((e / bound).max()):.3f}')
    assert bool((e <= bound).all()), tag
    # acc32: the fp32 fmaf chain
    got32 = _mm(a, w, bias, trans=trans, acc32=True)
    e = (got32.double() - ref64).abs()
    bound = a.shape[1] * 2.0 ** -24 * (a.double().abs() @ wt.double().abs()) + (
        bias.double().abs() * 2.0 ** -24 if bias is not None else 0.0) + 1e-30
    print(f'{tag} acc32: max {float(e.max()):.3e} mean {float(e.mean()):.3e}, max error / bound {float((e / bound).max()):.3f}')
    assert bool((e <= bound).all()), tag
    assert float(e.max()) <= 3 * float(e32.max()) + 1e-30 and float(e.mean()) <= 2 * float(e32.mean()) + 1e-30, tag
    return got


@pytest.mark.parametrize('M,K,N', [(65536, 256, 256), (65536, 39, 256), (65536, 256, 217), (65536, 217, 256),
                                   (65536, 256, 257), (65536, 257, 256), (65536, 289, 256), (65536, 256, 3),
                                   (65536, 256, 39), (1, 5, 1), (129, 33, 65), (1000, 300, 130)])
def test_gemm32_vs_f64(M, K, N):
    g = torch.Generator(device='cuda').manual_seed(M + 7 * K + 13 * N)
    a = torch.randn(M, K, device='cuda', generator=g)
    w_nt = torch.randn(N, K, device='cuda', generator=g) / K ** 0.5
    w_nn = torch.randn(K, N, device='cuda', generator=g) / K ** 0.5
    bias = torch.randn(N, device='cuda', generator=g)
    _check(a, w_nt, bias, True, f'A W^T + b  M={M} K={K} N={N}')
    _check(a, w_nt, None, True, f'A W^T      M={M} K={K} N={N}')
    _check(a, w_nn, None, False, f'A W        M={M} K={K} N={N}')


def test_gemm32_strided_rows_and_repeatable():
    """A as a column view [:, :K] of a wider tensor (row stride > K), and two launches bit-identical."""
    from neurecon_amd.training import _mm
    g = torch.Generator(device='cuda').manual_seed(3)
    big = torch.randn(20000, 300, device='cuda', generator=g)
    a = big[:, :257]
    w = torch.randn(256, 257, device='cuda', generator=g)
    b = torch.randn(256, device='cuda', generator=g)
    got = _check(a, w, b, True, 'strided A')
    assert torch.equal(got, _mm(a, w, b, trans=True))
    assert torch.equal(got, _mm(a.contiguous(), w, b, trans=True))
