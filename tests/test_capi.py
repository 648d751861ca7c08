"""CPU-side checks of the C-ABI boundary: the library loads (no GPU needed) and exports every
function include/neurecon_hip.h declares; struct layouts agree with the ctypes mirror."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    src = open(os.path.join(ROOT, 'include', 'neurecon_hip.h')).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'\b(nr_[a-z0-9_]+)\s*\(', src)))


@pytest.fixture(scope='module')
def lib():
    from neurecon_amd import build, _lib
    if not os.path.exists(_lib.LIB_PATH):
        build.build()
    return _lib.lib()


def test_exports_every_declared_symbol(lib):
    names = _declared()
    assert len(names) >= 12
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing


def test_ctypes_mirror_covers_header(lib):
    from neurecon_amd import _lib
    assert sorted(_lib.EXPORTED) == _declared()


def test_version_and_error_text(lib):
    assert lib.nr_version() >= 1
    assert isinstance(lib.nr_last_error(), bytes)


def test_descriptor_validation_without_gpu(lib):
    from neurecon_amd import _lib
    bad = _lib.NrSdfDesc(8, 128, 4, 6, 256, 0)
    assert lib.nr_sdf_packed_bytes(ctypes.byref(bad)) == 0
    assert b'W=256' in lib.nr_last_error()
    good = _lib.NrSdfDesc(8, 256, 4, 6, 256, 0)
    assert lib.nr_sdf_packed_bytes(ctypes.byref(good)) > 4 * 1024 * 1024
    rad = _lib.NrRadDesc(4, 256, -1, 4, 256, 0)
    assert lib.nr_radiance_packed_bytes(ctypes.byref(rad)) > 0


def test_struct_sizes(lib):
    from neurecon_amd import _lib
    assert ctypes.sizeof(_lib.NrSdfDesc) == 28
    assert ctypes.sizeof(_lib.NrRadDesc) == 32
    assert ctypes.sizeof(_lib.NrNerfDesc) == 28


def test_cpu_tensors_are_rejected():
    import torch
    from neurecon_amd.frameworks.neus import volume_render
    import weightgen as wg
    from helpers import neus_model
    from neurecon_amd.frameworks.neus import NeuS
    with pytest.raises(RuntimeError, match='GPU'):
        volume_render(torch.zeros(1, 4, 3), torch.ones(1, 4, 3), None)


def test_struct_layouts_match_the_c_compiler(tmp_path):
    """Every ctypes mirror struct has the size and field offsets gcc computes from the header."""
    import subprocess
    from neurecon_amd import _lib
    structs = [getattr(_lib, n) for n in dir(_lib) if n.startswith('Nr') and isinstance(getattr(_lib, n), type)
               and issubclass(getattr(_lib, n), ctypes.Structure)]
    assert len(structs) >= 7  # 3 descriptors, 3 render-argument blocks, kernel stats
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "neurecon_hip.h"', 'int main(void) {']
    for S in structs:
        lines.append(f'printf("{S.__name__} %zu\\n", sizeof({S.__name__}));')
        for f, _ in S._fields_:
            lines.append(f'printf("{S.__name__}.{f} %zu\\n", offsetof({S.__name__}, {f}));')
    lines.append('return 0; }')
    src = tmp_path / 'layout.c'
    src.write_text('\n'.join(lines))
    exe = tmp_path / 'layout'
    subprocess.check_call(['gcc', '-I', os.path.join(ROOT, 'include'), str(src), '-o', str(exe)])
    got = dict(l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for S in structs:
        assert int(got[S.__name__]) == ctypes.sizeof(S), S.__name__
        for f, _ in S._fields_:
            assert int(got[f'{S.__name__}.{f}']) == getattr(S, f).offset, (S.__name__, f)


def _wgrad_args(P=1000, m=256, n=256, npairs=1, ld=None):
    from neurecon_amd import _lib
    w = _lib.NrWgrad()
    w.P, w.npairs, w.m, w.n, w.scale = P, npairs, m, n, 1.0
    for q in range(2):  # fake non-null device pointers: argument checks run before any HIP call
        w.a[q], w.b[q] = 0x1000, 0x2000
        w.lda[q], w.ldb[q] = ld or m, ld or n
    w.c, w.ldc = 0x3000, n
    w.workspace = 0x4000
    w.workspace_bytes = 1 << 40
    return w


@pytest.mark.parametrize('case, code, text', [
    ('npairs', -1, 'npairs'),
    ('lda', -1, 'leading dimension'),
    ('null_out', -1, 'null output'),
    ('vec_without_avec', -1, 'avec'),
    ('operand_2gib', -1, '2 GiB'),
    ('workspace', -4, 'workspace'),
])
def test_wgrad_rejects_bad_arguments(lib, case, code, text):
    """nr_wgrad's argument checks (include/neurecon_hip.h NrWgrad) fail loudly before touching the GPU"""
    w = _wgrad_args()
    if case == 'npairs':
        w.npairs = 3
    elif case == 'lda':
        w.lda[0] = 100
    elif case == 'null_out':
        w.c = 0
    elif case == 'vec_without_avec':
        w.vec = 0x5000
    elif case == 'operand_2gib':
        w = _wgrad_args(P=1 << 22, m=256, n=256)  # 4 M rows x 256 x 4 B = 4 GiB
    elif case == 'workspace':
        w.workspace_bytes = 16
    rc = lib.nr_wgrad(ctypes.byref(w), None)
    assert rc == code, (rc, lib.nr_last_error())
    assert text in lib.nr_last_error().decode()


def test_wgrad_workspace_sizes(lib):
    """partials [S][n tiles x 128][m tiles x 256] + column-sum / vector partials, S ~ 256 / tiles"""
    one = lib.nr_wgrad_workspace_bytes(65536, 256, 256, 1)
    assert one >= 256 * 256 * 4 * 8
    assert lib.nr_wgrad_workspace_bytes(65536, 3, 256, 1) <= one
    assert lib.nr_wgrad_workspace_bytes(33, 17, 5, 1) > 0


def test_r05_training_entries_reject_bad_arguments(lib):
    """nr_weight_norm_*, nr_nerf_train_* and nr_radiance_train_fwd32 check their arguments before any HIP
    call (fake device pointers: nothing is dereferenced on the error paths)"""
    from neurecon_amd import _lib
    P = ctypes.c_void_p
    # weight norm: layer count, shapes, outputs
    assert lib.nr_weight_norm_fwd(None, 0, None) == -1 and 'NR_WN_MAX' in lib.nr_last_error().decode()
    arr = (_lib.NrWnLayer * 17)()
    assert lib.nr_weight_norm_fwd(arr, 17, None) == -1
    one = (_lib.NrWnLayer * 1)()
    one[0].v, one[0].g, one[0].norm, one[0].w, one[0].rows, one[0].cols = 0x1000, 0x2000, 0x3000, 0x4000, 0, 8
    assert lib.nr_weight_norm_fwd(one, 1, None) == -1 and 'bad layer' in lib.nr_last_error().decode()
    one[0].rows = 4
    assert lib.nr_weight_norm_bwd(one, 1, None) == -1 and 'null output' in lib.nr_last_error().decode()
    # NeRF++ training: the forward needs the fp32 pack and an aligned embedding; the backward every pointer
    nd = _lib.NrNerfDesc(8, 256, 4, 4, 10, 4, _lib.PREC_F16X3)
    assert lib.nr_nerf_train_packed_bytes(ctypes.byref(nd)) > 8 * 8 * 33 * 1024  # 8 ops of 8 x 33 KB chunks + views^T
    h8 = (P * 8)(*([0x10000] * 8))
    rc = lib.nr_nerf_train_fwd32(ctypes.byref(nd), 0x1000, 0x2000, 0x3000, 64, h8, 0x4000, 0x5000, 0x6000, 0x7000, None)
    assert rc == -1 and 'NR_PREC_FP32' in lib.nr_last_error().decode()
    nd.precision = _lib.PREC_FP32
    rc = lib.nr_nerf_train_fwd32(ctypes.byref(nd), 0x1000, 0x2004, 0x3000, 64, h8, 0x4000, 0x5000, 0x6000, 0x7000, None)
    assert rc == -1 and '16-byte' in lib.nr_last_error().decode()
    gz = (P * 8)(*([0x20000] * 7 + [0]))
    rc = lib.nr_nerf_train_bwd32(ctypes.byref(nd), 0x1000, 0x2000, 0x3000, h8, None, None, 64, 0x4000, 0x5000, 0x6000,
                                 gz, None)
    assert rc == -1 and 'null layer pointer' in lib.nr_last_error().decode()
    # the radiance training forward: the small-input stride covers the small inputs
    rd = _lib.NrRadDesc(4, 256, -1, 4, 256, _lib.PREC_FP32)
    rc = lib.nr_radiance_train_fwd32(ctypes.byref(rd), 0x1000, 0x2000, 0x3000, 8, 64, 0x4000, 0x5000, 0x6000, 0x7000,
                                     0x8000, None)
    assert rc == -1 and 'ld_small' in lib.nr_last_error().decode()


def _lib_env_int(name):
    from neurecon_amd import _lib
    return _lib._env_int(name)


def test_r06_entries_reject_bad_arguments(lib):
    """nr_gemm32 checks its sizes and leading dimensions before any HIP call (fake device pointers);
    nr_sdf5_enable refuses without NR_SDF5 at load (the packs would lack the 32x32x16 layout)"""
    A, B, C = 0x1000, 0x2000, 0x3000
    assert lib.nr_gemm32(None, 8, B, 8, 0, None, C, 8, 16, 8, 8, 0, None) == -1
    assert 'null argument' in lib.nr_last_error().decode()
    assert lib.nr_gemm32(A, 4, B, 8, 0, None, C, 8, 16, 8, 8, 0, None) == -1      # lda < K
    assert 'leading dimension' in lib.nr_last_error().decode()
    assert lib.nr_gemm32(A, 8, B, 4, 1, None, C, 8, 16, 8, 8, 0, None) == -1      # transposed B: ldb < K
    assert lib.nr_gemm32(A, 8, B, 8, 0, None, C, 4, 16, 8, 8, 0, None) == -1      # ldc < N
    assert lib.nr_gemm32(A, 0, B, 8, 0, None, C, 8, 16, 8, 0, 0, None) == -1      # K = 0
    assert 'K must be positive' in lib.nr_last_error().decode()
    assert lib.nr_gemm32(A, 8, B, 8, 0, None, C, 8, 128 * 65536, 8, 8, 0, None) == -1
    assert 'row tiles' in lib.nr_last_error().decode()
    assert lib.nr_gemm32(A, 8, B, 8, 0, None, C, 8, 0, 8, 8, 0, None) == 0        # empty: no launch
    if not _lib_env_int('NR_SDF5'):
        assert lib.nr_sdf5_enable(1) == -1 and 'NR_SDF5' in lib.nr_last_error().decode()
        assert lib.nr_sdf5_enable(0) == 0


def test_adam_step_rejects_bad_arguments(lib):
    """nr_adam_step checks its table and hyper-parameters before any HIP call"""
    from neurecon_amd import _lib
    assert lib.nr_adam_step(None, 0, 1, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1
    assert 'NR_ADAM_MAX' in lib.nr_last_error().decode()
    arr = (_lib.NrAdamTensor * 1)()
    arr[0].param, arr[0].grad, arr[0].exp_avg, arr[0].exp_avg_sq, arr[0].n = 0x1000, 0x2000, 0x3000, 0x4000, 0
    assert lib.nr_adam_step(arr, 1, 1, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1
    assert 'bad tensor' in lib.nr_last_error().decode()
    arr[0].n = 10
    assert lib.nr_adam_step(arr, 1, 0, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1      # step counts from 1
    assert lib.nr_adam_step(arr, 1, 1, 1e-3, 1.0, 0.999, 1e-8, 0.0, None) == -1      # beta1 < 1
    assert 'hyper-parameter' in lib.nr_last_error().decode()
    assert lib.nr_adam_step(arr, _lib.ADAM_MAX + 1, 1, 1e-3, 0.9, 0.999, 1e-8, 0.0, None) == -1


def test_adam_optimizer_rejects_cpu_parameters():
    """neurecon_amd.optim.Adam has no CPU path: a CPU parameter raises instead of falling back"""
    import torch
    from neurecon_amd.optim import Adam
    p = torch.nn.Parameter(torch.zeros(4))
    p.grad = torch.ones(4)
    with pytest.raises(RuntimeError, match='GPU'):
        Adam([p]).step()
