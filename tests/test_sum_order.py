"""The render kernels reproduce ATen's CPU float row-sum association order (nr_common.h
`aten_row_sum`) for normalisers that feed a discrete decision (sample_pdf).  This CPU test pins
that algorithm against torch.sum on this machine: a Python transcription of the device function
must agree with torch.sum bit for bit."""
import numpy as np
import torch

f32 = np.float32


def aten_row_sum(x, V=8):
    """Python transcription of nr_common.h aten_row_sum (same association order)."""
    n = len(x)
    if n < V:
        p = [f32(0)] * 4
        si = n // 4
        for i in range(si):
            for k in range(4):
                p[k] = f32(p[k] + x[4 * i + k])
        for t in range(si * 4, n):
            p[0] = f32(p[0] + x[t])
        return f32(f32(f32(p[0] + p[1]) + p[2]) + p[3])
    vec_size, size_ilp = n // V, (n // V) // 4
    acc = np.zeros((4, 4, V), f32)
    cl2 = 1
    if size_ilp > 2:
        cl2 = 0
        while (1 << cl2) < size_ilp:
            cl2 += 1
    lp = max(4, cl2 // 4)
    step, mask = 1 << lp, (1 << lp) - 1
    vec = lambda t: x[t * V:(t + 1) * V].astype(f32)
    i = 0
    while i + step <= size_ilp:
        for _ in range(step):
            for k in range(4):
                acc[0][k] = (acc[0][k] + vec(4 * i + k)).astype(f32)
            i += 1
        for j in range(1, 4):
            acc[j] = (acc[j] + acc[j - 1]).astype(f32)
            acc[j - 1] = 0
            if (i & (mask << (j * lp))) != 0:
                break
    while i < size_ilp:
        for k in range(4):
            acc[0][k] = (acc[0][k] + vec(4 * i + k)).astype(f32)
        i += 1
    for j in range(1, 4):
        acc[0] = (acc[0] + acc[j]).astype(f32)
    for t in range(size_ilp * 4, vec_size):
        acc[0][0] = (acc[0][0] + vec(t)).astype(f32)
    for k in range(1, 4):
        acc[0][0] = (acc[0][0] + acc[0][k]).astype(f32)
    fa = f32(0)
    for t in range(vec_size * V, n):
        fa = f32(fa + x[t])
    for l in range(V):
        fa = f32(fa + acc[0][0][l])
    return fa


def test_row_sum_order_matches_torch():
    rng = np.random.RandomState(0)
    sizes = list(range(1, 130)) + [255, 511, 512, 513, 1023, 2047, 2559, 3583]
    for n in sizes:
        for trial in range(6):
            x = (rng.rand(n) * rng.choice([1e-5, 1.0, 100.0])).astype(f32)
            if trial % 2:
                x[rng.randint(n)] = 1.0
            ref = torch.sum(torch.from_numpy(x).reshape(1, n), -1, keepdim=True).numpy()[0, 0]
            assert aten_row_sum(x) == ref, (n, trial)


def test_norm3_matches_torch_fma_order():
    """nr_common.h norm3_ref: torch's CPU x.norm(dim=-1) of 3-vectors == sqrt(fma(z,z,fma(y,y,x*x)))."""
    torch.manual_seed(0)
    x = (torch.randn(200000, 3) * 3).float()
    ref = x.norm(dim=-1).numpy()
    d = x.numpy().astype(np.float64)
    fma = lambda p, q, r: (p * q + r).astype(np.float32).astype(np.float64)  # exact product, one rounding
    sq = (d[:, 0] * d[:, 0]).astype(np.float32).astype(np.float64)
    got = np.sqrt(fma(d[:, 2], d[:, 2], fma(d[:, 1], d[:, 1], sq))).astype(np.float32)
    assert (got == ref).all()
