"""Timing / accuracy probe: the training step's weight gradient gᵀh ([P, m]ᵀ [P, k], P = 65536) as
(a) the fp32 split-K batched GEMM the training path runs (training._wgrad) and
(b) f16 hi/lo operands on hipBLASLt with fp32 accumulation (torch.bmm(..., out_dtype=float32)):
    gᵀh ≈ ghᵀhh + ghᵀhl + glᵀhh, g scaled by a power of two into f16's range.
    python tools/wgrad_probe.py"""
import torch


def split(x, scale):
    xs = x * scale
    hi = xs.half()
    lo = (xs - hi.float()).half()
    return hi, lo


def time_it(fn, n=50):
    for _ in range(5):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def main():
    torch.manual_seed(0)
    dev = 'cuda'
    P, m, k, C = 65536, 256, 256, 16
    g = (torch.randn(P, m, device=dev) * 1e-6) * torch.rand(P, 1, device=dev)
    h = torch.nn.functional.softplus(torch.randn(P, k, device=dev), beta=100)
    ref = (g.double().t() @ h.double())

    def fp32():
        return torch.bmm(g.view(C, P // C, m).transpose(1, 2), h.view(C, P // C, k)).sum(0)

    sg = 2.0 ** (14 - torch.ceil(torch.log2(g.abs().max())).item())
    gh, gl = split(g, sg)
    hh, hl = split(h, 1.0)
    # [P, 2k]: hi | lo per row, so gh^T [hh | hl] is one GEMM
    hcat = torch.cat([hh, hl], 1)
    gcat = torch.cat([gh, gl], 1)

    def f16_2():
        a = torch.bmm(gh.view(C, P // C, m).transpose(1, 2), hcat.view(C, P // C, 2 * k), out_dtype=torch.float32)
        b = torch.bmm(gl.view(C, P // C, m).transpose(1, 2), hh.view(C, P // C, k), out_dtype=torch.float32)
        return (a[:, :, :k].sum(0) + a[:, :, k:].sum(0) + b.sum(0)) / sg

    def f16_k3():
        # K-concatenated: [gh; gh; gl]^T [hh; hl; hh]
        A = torch.cat([gh, gh, gl], 0).view(3 * C, P // C, m)
        B = torch.cat([hh, hl, hh], 0).view(3 * C, P // C, k)
        return torch.bmm(A.transpose(1, 2), B, out_dtype=torch.float32).sum(0) / sg

    A3 = torch.cat([gh, gh, gl], 0).view(3 * C, P // C, m)
    B3 = torch.cat([hh, hl, hh], 0).view(3 * C, P // C, k)

    def f16_k3_pre():
        return torch.bmm(A3.transpose(1, 2), B3, out_dtype=torch.float32).sum(0) / sg

    def f16_k3_pre_bmm_only():
        return torch.bmm(A3.transpose(1, 2), B3, out_dtype=torch.float32)

    for C2 in (4, 8, 16):
        A4 = A3.view(3 * C2, -1, m)
        B4 = B3.view(3 * C2, -1, k)
        t = time_it(lambda: torch.bmm(A4.transpose(1, 2), B4, out_dtype=torch.float32))
        print(f'f16 K3 bmm only, {3 * C2} slabs: {t:.1f} us')
    for name, fn in [('fp32 split-K (current)', fp32), ('f16 two GEMMs', f16_2), ('f16 K-concat incl. cat', f16_k3),
                     ('f16 K-concat pre-cat', f16_k3_pre), ('f16 K-concat bmm only', f16_k3_pre_bmm_only)]:
        t = time_it(fn)
        out = fn()
        if out.dim() == 2:
            err = ((out.double() - ref).abs().max() / ref.abs().max()).item()
        else:
            err = float('nan')
        print(f'{name:28s} {t:8.1f} us   max err / max|ref| {err:.3e}')
    t = time_it(lambda: split(g, sg))
    print(f'split g (torch ops) {t:.1f} us')
    gg = torch.randn(P, 512, device=dev)
    t = time_it(lambda: gg.clone())
    print(f'copy 128 MB: {t:.1f} us')


if __name__ == '__main__':
    main()
