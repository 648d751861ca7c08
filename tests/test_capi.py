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
    # NrNeusArgs: 7 pointers+i64, 4 floats, 5 ints (+pad), 2 table ptrs, 11 output ptrs, ws ptr + size
    assert ctypes.sizeof(_lib.NrSdfDesc) == 24
    assert ctypes.sizeof(_lib.NrRadDesc) == 24
    assert ctypes.sizeof(_lib.NrNeusArgs) == 7 * 8 + 4 * 4 + 5 * 4 + 4 + 2 * 8 + 11 * 8 + 2 * 8


def test_cpu_tensors_are_rejected():
    import torch
    from neurecon_amd.frameworks.neus import volume_render
    import weightgen as wg
    from helpers import neus_model
    from neurecon_amd.frameworks.neus import NeuS
    with pytest.raises(RuntimeError, match='GPU'):
        volume_render(torch.zeros(1, 4, 3), torch.ones(1, 4, 3), None)
