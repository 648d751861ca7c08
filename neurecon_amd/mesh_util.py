"""Mesh extraction: drop-in for utils/mesh_util.py:82-112.

The hot part — the N^3 SDF grid query (134 M forward SDF evaluations at N=512) — runs in
libnrhip (`nr_sdf_grid`: voxel coordinates generated on the device with the reference's float64
formula, then the forward SDF kernel), with no host point array and no per-chunk host copies.
Marching cubes + PLY writing stay on the host exactly as in the reference (scikit-image and
plyfile; neither is installed in this image, so `convert_sigma_samples_to_ply` raises ImportError
and callers use `sdf_grid` directly).

Note: the reference computes the voxel y / x indices with true division (`(i / N) % N`,
`((i / N) / N) % N`, mesh_util.py:92-93), i.e. with fractional parts z/N and y/N + z/N^2 of a
voxel; the grid reproduces that bit for bit (tests/test_gpu_surface.py), it does not "fix" it.
"""
import ctypes

import numpy as np
import torch

from . import _lib as L

_GRID_CHUNK = 1 << 22  # points per native launch (48 MB of coordinates in the workspace)


def sdf_grid_range(implicit_surface, volume_size, N, start, count, chunk=None, device=None):
    """SDF at flat voxel indices [start, start+count) of extract_mesh's N^3 grid -> device tensor [count].
    Inference only, like the reference (`.data`, mesh_util.py:104): no graph, also under grad mode."""
    N, start, count = int(N), int(start), int(count)
    if start < 0 or count < 0 or start + count > N ** 3:
        raise ValueError(f'voxel range [{start}, {start + count}) outside the {N}^3 grid')
    dev = torch.device(device) if device is not None else next(implicit_surface.parameters()).device
    if dev.type != 'cuda':
        raise RuntimeError('neurecon_amd: sdf_grid needs the model on a GPU (ROCm) device; the path is HIP-only')
    with torch.no_grad():
        return _grid_range(implicit_surface, volume_size, N, start, count, chunk, dev)


def _grid_range(implicit_surface, volume_size, N, start, count, chunk, dev):
    out = torch.empty(count, device=dev)
    if count == 0:
        return out
    chunk = min(int(chunk or _GRID_CHUNK), count)
    desc, packed = implicit_surface.nr_packed(dev)
    lib = L.lib()
    ws_bytes = lib.nr_sdf_grid_workspace_bytes(chunk)
    ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
    st = L.stream_of(dev)
    for j in range(0, count, chunk):
        n = min(chunk, count - j)
        L.check(lib.nr_sdf_grid(ctypes.byref(desc), L.ptr(packed), ctypes.c_double(float(volume_size)), N,
                                start + j, n, ctypes.c_void_p(out.data_ptr() + 4 * j), L.ptr(ws), ws_bytes, st))
    return out


def sdf_grid(implicit_surface, volume_size=2.0, N=512, chunk=None, device=None):
    """SDF of extract_mesh's N^3 grid (mesh_util.py:82-108) as a device tensor [N, N, N]."""
    N = int(N)
    return sdf_grid_range(implicit_surface, volume_size, N, 0, N ** 3, chunk, device).reshape(N, N, N)


def convert_sigma_samples_to_ply(input_3d_sigma_array, voxel_grid_origin, volume_size, ply_filename_out, level=5.0,
                                 offset=None, scale=None):
    """mesh_util.py:13-79 (host-side marching cubes + PLY)."""
    try:
        import skimage.measure
        import plyfile
    except ImportError as e:  # not in this image
        raise ImportError('neurecon_amd.mesh_util: marching cubes needs scikit-image and plyfile; '
                          'use sdf_grid() for the SDF volume') from e
    verts, faces, _, _ = skimage.measure.marching_cubes(input_3d_sigma_array, level=level, spacing=volume_size)
    pts = np.asarray(verts, dtype=np.float64) + np.asarray(voxel_grid_origin, dtype=np.float64)[None]
    if scale is not None:
        pts = pts / scale
    if offset is not None:
        pts = pts - offset
    v = np.zeros((pts.shape[0],), dtype=[('x', 'f4'), ('y', 'f4'), ('z', 'f4')])
    v['x'], v['y'], v['z'] = pts[:, 0], pts[:, 1], pts[:, 2]
    f = np.zeros((faces.shape[0],), dtype=[('vertex_indices', 'i4', (3,))])
    f['vertex_indices'] = faces
    plyfile.PlyData([plyfile.PlyElement.describe(v, 'vertex'),
                     plyfile.PlyElement.describe(f, 'face')]).write(ply_filename_out)


def extract_mesh(implicit_surface, volume_size=2.0, level=0.0, N=512, filepath='./surface.ply', show_progress=True,
                 chunk=16 * 1024):
    """mesh_util.py:82-112; `chunk` is accepted for API compatibility (the device grid uses larger launches)."""
    s = volume_size
    out = sdf_grid(implicit_surface, s, N).cpu().numpy()
    convert_sigma_samples_to_ply(out, [-s / 2., -s / 2., -s / 2.], [float(s) / N] * 3, filepath, level=level)
