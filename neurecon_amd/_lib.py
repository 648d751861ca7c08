"""ctypes binding of libnrhip.so (include/neurecon_hip.h).

The library is the product: there is no fallback.  `lib()` raises if the shared object is
missing or cannot be loaded, and every wrapper raises on a non-zero status code.
"""
import ctypes
import os
import threading

import torch  # noqa: F401  (loads the HIP runtime that libnrhip.so binds to by SONAME)

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('NR_LIB', os.path.join(HERE, 'libnrhip.so'))

PREC_FP32 = 0
PREC_F16X3 = 1
UPSAMPLE = {'official_solution': 0, 'direct_use': 1, 'direct_more': 2}

_c_p = ctypes.c_void_p
_c_i = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_c_d = ctypes.c_double
_c_sz = ctypes.c_size_t


class NrSdfDesc(ctypes.Structure):
    _fields_ = [('D', _c_i), ('W', _c_i), ('skip', _c_i), ('multires', _c_i), ('W_geo_feat', _c_i),
                ('precision', _c_i), ('siren', _c_i)]


class NrRadDesc(ctypes.Structure):
    _fields_ = [('D', _c_i), ('W', _c_i), ('multires', _c_i), ('multires_view', _c_i), ('W_geo_feat', _c_i),
                ('precision', _c_i), ('no_view_dirs', _c_i), ('siren', _c_i)]


class NrNerfDesc(ctypes.Structure):
    _fields_ = [('D', _c_i), ('W', _c_i), ('skip', _c_i), ('input_ch', _c_i), ('multires', _c_i),
                ('multires_view', _c_i), ('precision', _c_i)]


class NrNeusArgs(ctypes.Structure):
    _fields_ = [
        ('rays_o', _c_p), ('rays_d', _c_p), ('n_rays', _c_i64),
        ('sdf', ctypes.POINTER(NrSdfDesc)), ('sdf_packed', _c_p),
        ('rad', ctypes.POINTER(NrRadDesc)), ('rad_packed', _c_p),
        ('s', _c_f), ('obj_bounding_radius', _c_f), ('near_bypass', _c_f), ('far_bypass', _c_f),
        ('N_samples', _c_i), ('N_importance', _c_i), ('N_upsample_iters', _c_i), ('calc_normal', _c_i),
        ('white_bkgd', _c_i),
        ('t_coarse', _c_p), ('u_fine', _c_p),
        ('rgb', _c_p), ('depth', _c_p), ('acc', _c_p), ('normals', _c_p),
        ('d_final', _c_p), ('sdf_out', _c_p), ('nablas_out', _c_p), ('radiance_out', _c_p),
        ('alpha_out', _c_p), ('cdf_out', _c_p), ('weights_out', _c_p),
        ('nerf', ctypes.POINTER(NrNerfDesc)), ('nerf_packed', _c_p), ('N_outside', _c_i), ('t_outside', _c_p),
        ('sigma_out', _c_p), ('radiance_bg_out', _c_p),
        ('upsample_algo', _c_i), ('fixed_s', _c_f), ('N_nograd_samples', _c_i), ('t_nograd', _c_p),
        ('workspace', _c_p), ('workspace_bytes', _c_sz),
        ('u_rand', _c_p), ('t_out_rand', _c_p), ('s_dev', _c_p), ('sample_only', _c_i), ('d_all_out', _c_p),
        ('no_mid_skip', _c_i), ('no_defer', _c_i), ('max_chunk_rays', _c_i64), ('max_workspace_bytes', _c_sz),
    ]


class NrVolsdfArgs(ctypes.Structure):
    _fields_ = [
        ('rays_o', _c_p), ('rays_d', _c_p), ('n_rays', _c_i64),
        ('sdf', ctypes.POINTER(NrSdfDesc)), ('sdf_packed', _c_p),
        ('rad', ctypes.POINTER(NrRadDesc)), ('rad_packed', _c_p),
        ('alpha_net', _c_f), ('beta_net', _c_f), ('beta_plus_init', _c_f), ('eps', _c_f),
        ('near', _c_f), ('far', _c_f), ('obj_bounding_radius', _c_f), ('use_sphere_bg', _c_i),
        ('N_samples', _c_i), ('N_importance', _c_i), ('max_upsample_steps', _c_i), ('max_bisection_steps', _c_i),
        ('calc_normal', _c_i), ('white_bkgd', _c_i),
        ('t_coarse', _c_p), ('t_init', _c_p), ('u_up', _c_p), ('u_fine', _c_p),
        ('rgb', _c_p), ('depth', _c_p), ('acc', _c_p), ('normals', _c_p),
        ('d_vals', _c_p), ('sdf_out', _c_p), ('nablas_out', _c_p), ('radiance_out', _c_p),
        ('alpha_out', _c_p), ('p_out', _c_p), ('weights_out', _c_p), ('sigma_out', _c_p),
        ('beta_map', _c_p), ('iter_usage', _c_p),
        ('workspace', _c_p), ('workspace_bytes', _c_sz),
        ('N_outside', _c_i), ('nerf', ctypes.POINTER(NrNerfDesc)), ('nerf_packed', _c_p), ('rs_out', _c_p),
        ('beta_plus_k', _c_f), ('sigma_bg', _c_p), ('radiance_bg', _c_p), ('u_rand', _c_p), ('u_out', _c_p),
    ]


class NrUnisurfArgs(ctypes.Structure):
    _fields_ = [
        ('rays_o', _c_p), ('rays_d', _c_p), ('n_rays', _c_i64), ('rays_per_batch', _c_i64),
        ('sdf', ctypes.POINTER(NrSdfDesc)), ('sdf_packed', _c_p),
        ('rad', ctypes.POINTER(NrRadDesc)), ('rad_packed', _c_p),
        ('logit_tau', _c_f), ('radius_of_interest', _c_f), ('interval', _c_f), ('too_close_threshold', _c_f),
        ('near_bypass', _c_f), ('far_bypass', _c_f),
        ('N_steps', _c_i), ('N_secant_steps', _c_i), ('N_query', _c_i), ('N_freespace', _c_i),
        ('normal_mode', _c_i), ('rayschunk', _c_i64), ('netchunk', _c_i64),
        ('calc_normal', _c_i), ('white_bkgd', _c_i),
        ('t_march', _c_p), ('t_query', _c_p), ('t_free', _c_p),
        ('rgb', _c_p), ('depth', _c_p), ('acc', _c_p), ('normals', _c_p),
        ('surface_points', _c_p), ('mask_surface', _c_p), ('depth_surface', _c_p),
        ('radiance_out', _c_p), ('sdf_out', _c_p), ('nablas_out', _c_p), ('alpha_out', _c_p), ('weights_out', _c_p),
        ('workspace', _c_p), ('workspace_bytes', _c_sz),
        ('u_query', _c_p), ('u_free', _c_p),
        ('shard_ray0', _c_i64), ('shard_row_rays', _c_i64), ('window_ss', _c_p), ('window_reduce', _c_p),
        ('window_user', _c_p), ('no_secant', _c_i), ('d_all_out', _c_p), ('sample_only', _c_i),
        ('full_march', _c_i),
    ]


WINDOW_REDUCE = ctypes.CFUNCTYPE(_c_i, _c_p)

TG_NONE, TG_SOFTPLUS, TG_MUL, TG_SPADJ, TG_RELUMASK = 0, 1, 3, 4, 5
# NrTrainGemm.blocked / NrWgrad.blocked bits (include/neurecon_hip.h: 16 x 16 blocked tensors)
BLK_X1, BLK_X2, BLK_Y, BLK_YB, BLK_Y2, BLK_Y3, BLK_A, BLK_G, BLK_ZD = 1, 2, 4, 8, 16, 32, 64, 128, 256
WG_BLK_A0, WG_BLK_A1, WG_BLK_B0, WG_BLK_B1 = 1, 2, 4, 8
WN_MAX = 16  # NR_WN_MAX: layers per nr_weight_norm_* call
ADAM_MAX = 64  # NR_ADAM_MAX: tensors per nr_adam_step call


class NrTrainGemm(ctypes.Structure):
    _fields_ = [
        ('op', _c_p), ('P', _c_i64),
        ('x1', _c_p), ('ld1', _c_i64), ('n1', _c_i),
        ('x2', _c_p), ('ld2', _c_i64), ('n2', _c_i),
        ('use_bias', _c_i), ('mode', _c_i), ('yscale', _c_f),
        ('y', _c_p), ('ldy', _c_i64), ('yb', _c_p), ('ldyb', _c_i64),
        ('y2', _c_p), ('ldy2', _c_i64), ('y3', _c_p), ('ldy3', _c_i64),
        ('a', _c_p), ('lda', _c_i64), ('g', _c_p), ('ldg', _c_i64), ('zd', _c_p), ('ldzd', _c_i64),
        ('g_row', _c_i), ('dot', _c_p), ('dot_bias', _c_f),
        ('head', _c_p), ('head_bias', _c_p), ('head_out', _c_p), ('blocked', _c_i),
        ('g_scaled', _c_i),
    ]


class NrWgrad(ctypes.Structure):
    _fields_ = [
        ('P', _c_i64), ('npairs', _c_i), ('a', _c_p * 2), ('lda', _c_i64 * 2), ('b', _c_p * 2), ('ldb', _c_i64 * 2),
        ('m', _c_i), ('n', _c_i), ('scale', _c_f), ('c', _c_p), ('ldc', _c_i64), ('colsum', _c_p),
        ('avec', _c_p), ('ldv', _c_i64), ('vec', _c_p), ('vec_scale', _c_f), ('workspace', _c_p),
        ('workspace_bytes', _c_sz), ('blocked', _c_i), ('fp32', _c_i),
    ]


class NrWnLayer(ctypes.Structure):
    _fields_ = [('v', _c_p), ('g', _c_p), ('w', _c_p), ('norm', _c_p), ('grad_w', _c_p), ('grad_v', _c_p),
                ('grad_g', _c_p), ('rows', _c_i), ('cols', _c_i)]


class NrAdamTensor(ctypes.Structure):
    _fields_ = [('param', _c_p), ('grad', _c_p), ('exp_avg', _c_p), ('exp_avg_sq', _c_p), ('n', _c_i64)]


class NrKernelStat(ctypes.Structure):
    _fields_ = [('name', ctypes.c_char * 32), ('launches', _c_i64), ('ms', ctypes.c_double),
                ('units', ctypes.c_double)]


_SIGS = {
    'nr_version': (_c_i, []),
    'nr_last_error': (ctypes.c_char_p, []),
    'nr_build_id': (ctypes.c_char_p, []),
    'nr_sdf_packed_bytes': (_c_sz, [ctypes.POINTER(NrSdfDesc)]),
    'nr_sdf_pack': (_c_i, [ctypes.POINTER(NrSdfDesc), ctypes.POINTER(_c_p), ctypes.POINTER(_c_p), _c_p, _c_p]),
    'nr_mlp_workspace_bytes': (_c_sz, [_c_i]),
    'nr_sdf_forward': (_c_i, [ctypes.POINTER(NrSdfDesc), _c_p, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    'nr_radiance_packed_bytes': (_c_sz, [ctypes.POINTER(NrRadDesc)]),
    'nr_radiance_pack': (_c_i, [ctypes.POINTER(NrRadDesc), ctypes.POINTER(_c_p), ctypes.POINTER(_c_p), _c_p, _c_p]),
    'nr_radiance_forward': (_c_i, [ctypes.POINTER(NrRadDesc), _c_p, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_i64, _c_p,
                                   _c_p]),
    'nr_nerf_packed_bytes': (_c_sz, [ctypes.POINTER(NrNerfDesc)]),
    'nr_nerf_pack': (_c_i, [ctypes.POINTER(NrNerfDesc), ctypes.POINTER(_c_p), ctypes.POINTER(_c_p), _c_p, _c_p]),
    'nr_nerf_forward': (_c_i, [ctypes.POINTER(NrNerfDesc), _c_p, _c_p, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_p]),
    'nr_nerf_train_fwd32': (_c_i, [ctypes.POINTER(NrNerfDesc), _c_p, _c_p, _c_p, _c_i64, ctypes.POINTER(_c_p), _c_p,
                                   _c_p, _c_p, _c_p, _c_p]),
    'nr_nerf_train_packed_bytes': (_c_sz, [ctypes.POINTER(NrNerfDesc)]),
    'nr_weight_norm_fwd': (_c_i, [ctypes.POINTER(NrWnLayer), _c_i, _c_p]),
    'nr_weight_norm_bwd': (_c_i, [ctypes.POINTER(NrWnLayer), _c_i, _c_p]),
    'nr_adam_step': (_c_i, [ctypes.POINTER(NrAdamTensor), _c_i, _c_i64, _c_d, _c_d, _c_d, _c_d, _c_d, _c_p]),
    'nr_nerf_train_pack': (_c_i, [ctypes.POINTER(NrNerfDesc), ctypes.POINTER(_c_p), ctypes.POINTER(_c_p), _c_p, _c_p]),
    'nr_nerf_train_bwd32': (_c_i, [ctypes.POINTER(NrNerfDesc), _c_p, _c_p, _c_p, ctypes.POINTER(_c_p), _c_p, _c_p,
                                   _c_i64, _c_p, _c_p, _c_p, ctypes.POINTER(_c_p), _c_p]),
    'nr_neus_workspace_bytes': (_c_sz, [ctypes.POINTER(NrNeusArgs)]),
    'nr_neus_render': (_c_i, [ctypes.POINTER(NrNeusArgs), _c_p]),
    'nr_volsdf_workspace_bytes': (_c_sz, [ctypes.POINTER(NrVolsdfArgs)]),
    'nr_volsdf_render': (_c_i, [ctypes.POINTER(NrVolsdfArgs), _c_p]),
    'nr_unisurf_workspace_bytes': (_c_sz, [ctypes.POINTER(NrUnisurfArgs)]),
    'nr_unisurf_render': (_c_i, [ctypes.POINTER(NrUnisurfArgs), _c_p]),
    'nr_unisurf_window_count': (_c_i64, [ctypes.POINTER(NrUnisurfArgs)]),
    'nr_sample_pdf': (_c_i, [_c_p, _c_p, _c_i64, _c_i, _c_p, _c_i64, _c_i, _c_p, _c_p]),
    'nr_get_rays': (_c_i, [_c_p, _c_p, _c_i, _c_i, _c_i, _c_p, _c_i64, _c_p, _c_p, _c_p]),
    'nr_gather_rows': (_c_i, [_c_p, _c_i64, _c_i64, _c_i64, _c_p, _c_i64, _c_p, _c_p]),
    'nr_sphere_trace_workspace_bytes': (_c_sz, [_c_i64]),
    'nr_sphere_trace': (_c_i, [ctypes.POINTER(NrSdfDesc), _c_p, _c_p, _c_p, _c_i64, ctypes.c_float, ctypes.c_float,
                               _c_p, _c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    'nr_radiance_train_fwd32': (_c_i, [ctypes.POINTER(NrRadDesc), _c_p, _c_p, _c_p, _c_i64, _c_i64, _c_p, _c_p, _c_p,
                                        _c_p, _c_p, _c_p]),
    'nr_root_find_workspace_bytes': (_c_sz, [_c_i64, _c_i]),
    'nr_root_find': (_c_i, [ctypes.POINTER(NrSdfDesc), _c_p, _c_p, _c_p, _c_i64, ctypes.c_float, ctypes.c_float, _c_p,
                            _c_p, _c_i, _c_p, _c_i, _c_i, ctypes.c_float, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p,
                            _c_sz, _c_p]),
    'nr_normalize3': (_c_i, [_c_p, _c_i64, _c_p, _c_p]),
    'nr_surface_finish': (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_p, _c_p]),
    'nr_sdf_grid_workspace_bytes': (_c_sz, [_c_i64]),
    'nr_sdf_grid': (_c_i, [ctypes.POINTER(NrSdfDesc), _c_p, ctypes.c_double, _c_i64, _c_i64, _c_i64, _c_p, _c_p,
                           _c_sz, _c_p]),
    # training path (nr_train.hip)
    'nr_embed': (_c_i, [_c_p, _c_i64, _c_i, _c_p, _c_p]),
    'nr_embed_jvp': (_c_i, [_c_p, _c_p, _c_i64, _c_i, _c_p, _c_p]),
    'nr_embed_vjp': (_c_i, [_c_p, _c_p, _c_i, _c_p, _c_i, _c_f, _c_i64, _c_i, _c_p, _c_p]),
    'nr_embed_padded': (_c_i, [_c_p, _c_i64, _c_i, _c_p, _c_i, _c_p]),
    'nr_embed_jvp_padded': (_c_i, [_c_p, _c_p, _c_i64, _c_i, _c_p, _c_i, _c_p]),
    # training layer GEMMs (nr_mlp.hip tgemm_kernel)
    'nr_train_gemm': (_c_i, [ctypes.POINTER(NrTrainGemm), _c_i, _c_i, _c_i, _c_i, _c_p]),
    'nr_sdf_op_info': (_c_i, [ctypes.POINTER(NrSdfDesc), _c_i, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i),
                              ctypes.POINTER(_c_i)]),
    'nr_sdf_train_packed_bytes': (_c_sz, [ctypes.POINTER(NrSdfDesc)]),
    'nr_sdf_train_pack': (_c_i, [ctypes.POINTER(NrSdfDesc), ctypes.POINTER(_c_p), ctypes.POINTER(_c_p), _c_p, _c_p]),
    'nr_radiance_op_info': (_c_i, [ctypes.POINTER(NrRadDesc), _c_i, ctypes.POINTER(_c_i64), ctypes.POINTER(_c_i),
                                   ctypes.POINTER(_c_i)]),
    'nr_radiance_train_packed_bytes': (_c_sz, [ctypes.POINTER(NrRadDesc)]),
    'nr_radiance_train_pack': (_c_i, [ctypes.POINTER(NrRadDesc), ctypes.POINTER(_c_p), ctypes.POINTER(_c_p), _c_p,
                                      _c_p]),
    'nr_softplus100': (_c_i, [_c_p, _c_i64, _c_p, _c_p, _c_p]),
    'nr_scale_cols': (_c_i, [_c_p, _c_i64, _c_i, _c_i, _c_i, _c_p, _c_f, _c_p, _c_p]),
    'nr_softplus_adjoint': (_c_i, [_c_p, _c_i, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_p, _c_p]),
    'nr_colsum_workspace_bytes': (_c_sz, [_c_i]),
    'nr_colsum': (_c_i, [_c_p, _c_i64, _c_i, _c_p, _c_p, _c_sz, _c_p]),
    'nr_sine30': (_c_i, [_c_p, _c_i64, _c_p, _c_p, _c_p]),
    'nr_sine_adjoint': (_c_i, [_c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_p, _c_p]),
    'nr_mul': (_c_i, [_c_p, _c_p, _c_i64, _c_p, _c_p]),
    'nr_activation': (_c_i, [_c_p, _c_p, _c_i64, _c_i, _c_p]),
    'nr_radiance_input': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_i, _c_p, _c_p]),
    'nr_neus_points': (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i, _c_p, _c_p, _c_p, _c_p]),
    'nr_neus_composite_fwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                     _c_p]),
    'nr_neus_composite_bwd_workspace_bytes': (_c_sz, [_c_i64, _c_i]),
    'nr_neus_composite_bwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                     _c_p, _c_p, _c_sz, _c_p]),
    'nr_nerf_train_input': (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, ctypes.c_float, _c_p, _c_p, _c_p, _c_p]),
    'nr_neus_composite_bg_fwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_i, _c_p, _c_p,
                                        _c_p, _c_p, _c_p, _c_p, _c_p]),
    'nr_neus_composite_bg_bwd_workspace_bytes': (_c_sz, [_c_i64, _c_i, _c_i]),
    'nr_neus_composite_bg_bwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_i, _c_p, _c_p,
                                        _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    'nr_unisurf_composite_fwd': (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    'nr_unisurf_composite_bwd_workspace_bytes': (_c_sz, [_c_i64, _c_i]),
    'nr_unisurf_composite_bwd': (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                        _c_sz, _c_p]),
    'nr_volsdf_composite_bg_fwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_f, _c_i, _c_p, _c_p,
                                          _c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p]),
    'nr_volsdf_composite_bg_bwd_workspace_bytes': (_c_sz, [_c_i64, _c_i, _c_i]),
    'nr_volsdf_composite_bg_bwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_f, _c_i, _c_p, _c_p,
                                          _c_p, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p,
                                          _c_sz, _c_p]),
    'nr_volsdf_nerf_input': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_p, _c_p, _c_p]),
    'nr_volsdf_composite_fwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_f, _c_i, _c_p, _c_p, _c_p,
                                       _c_p, _c_p, _c_p, _c_p, _c_p]),
    'nr_volsdf_composite_bwd_workspace_bytes': (_c_sz, [_c_i64, _c_i]),
    'nr_volsdf_composite_bwd': (_c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, _c_i, _c_i, _c_f, _c_i, _c_p, _c_p, _c_p,
                                       _c_p, _c_p, _c_p, _c_p, _c_p, _c_p, _c_sz, _c_p]),
    'nr_wgrad_workspace_bytes': (_c_sz, [_c_i64, _c_i, _c_i, _c_i]),
    'nr_wgrad': (_c_i, [ctypes.POINTER(NrWgrad), _c_p]),
    'nr_profile_enable': (_c_i, [_c_i]),
    'nr_gemm32': (_c_i, [_c_p, _c_i64, _c_p, _c_i64, _c_i, _c_p, _c_p, _c_i64, _c_i64, _c_i, _c_i, _c_i, _c_p]),
    'nr_sdf5_enable': (_c_i, [_c_i]),
    'nr_profile_filter': (_c_i, [ctypes.c_char_p]),
    'nr_profile_read': (_c_i, [ctypes.POINTER(NrKernelStat), _c_i, ctypes.POINTER(_c_i)]),
}

EXPORTED = tuple(_SIGS)

_lock = threading.Lock()
_lib = None


class NrError(RuntimeError):
    pass



def _env_int(name):
    """integer value of an environment switch (unset, empty or not a number: 0)"""
    try:
        return int(os.environ.get(name, '') or 0)
    except ValueError:
        return 0

def lib():
    """Load libnrhip.so (raises if absent: the HIP path is the only path)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(f'neurecon_amd: {LIB_PATH} not found; build it with `python -m neurecon_amd.build`')
            L = ctypes.CDLL(LIB_PATH)
            for name, (res, args) in _SIGS.items():
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            if _env_int('NR_SDF5'):  # kernel selection (nr_sdf5_enable), for A/B runs
                L.nr_sdf5_enable(_env_int('NR_SDF5'))
            _lib = L
    return _lib


def build_id():
    """the source hash compiled into the loaded library (neurecon_amd/build.py source_hash)"""
    return lib().nr_build_id().decode()


def check(rc):
    if rc != 0:
        raise NrError(f'libnrhip error {rc}: {lib().nr_last_error().decode()}')


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream_of(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def profile_enable(on=True, prefix=''):
    """library kernel timing on/off; prefix: only kernels whose name starts with it get events"""
    check(lib().nr_profile_filter(prefix.encode()))
    check(lib().nr_profile_enable(1 if on else 0))


def profile_read():
    """{kernel: (launches, total_ms, total_units)} since the last read (waits for the events)."""
    buf = (NrKernelStat * 64)()
    n = ctypes.c_int(0)
    check(lib().nr_profile_read(buf, 64, ctypes.byref(n)))
    return {buf[i].name.decode(): (buf[i].launches, buf[i].ms, buf[i].units) for i in range(n.value)}


_WS = {}
_BUDGET = [None]


def set_workspace_budget(gib):
    """Module-wide cap (GiB) on one render call's workspace; None: $NR_MAX_WORKSPACE_GB, else the
    library's default (NR_DEFAULT_WORKSPACE_BYTES, 4 GiB).  Renders are chunked to fit it."""
    _BUDGET[0] = gib


def workspace_budget_bytes(override_gib=None):
    """bytes for NrNeusArgs.max_workspace_bytes (0 = the library's default)"""
    g = override_gib if override_gib is not None else _BUDGET[0]
    if g is None:
        g = os.environ.get('NR_MAX_WORKSPACE_GB')
    return 0 if g in (None, '') else int(float(g) * (1 << 30))


def workspace(device, nbytes):
    """Scratch for one library call, reused across calls (grow-only) on the same device AND stream:
    calls enqueued on one stream are ordered, so they can share one buffer; a render on another stream
    (e.g. a side-stream validation render beside training) gets its own.  A buffer outgrown on its
    stream is freed through the caching allocator, which reuses the block only in that stream's order.
    DataParallel replica threads run on their own devices' streams, so they never share a buffer."""
    dev = torch.device(device)
    key = (str(dev), torch.cuda.current_stream(dev).cuda_stream)
    buf = _WS.get(key)
    if buf is None or buf.numel() < nbytes:
        _WS.pop(key, None)
        buf = torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=dev)
        _WS[key] = buf
    return buf


def require_gpu(t, what='input'):
    if not (isinstance(t, torch.Tensor) and t.is_cuda):
        raise RuntimeError(f'neurecon_amd: {what} must be a GPU (ROCm) tensor; the render path is HIP-only')
