/*
 * neurecon_hip.h — C-ABI of the MI355X (gfx950) render library `libnrhip.so`.
 *
 * Drop-in boundary for neurecon's ray-marched SDF volume renderer.  The reference is pure
 * Python/PyTorch (no FFI), so each entry point below replaces a Python-level operator of the
 * reference (file:line cited per function, paths relative to SuwoongHeo/neurecon):
 *
 *   nr_sdf_forward          ImplicitSurface.forward / forward_with_nablas   models/base.py:243-282
 *   nr_radiance_forward     RadianceNet.forward                              models/base.py:372-391
 *   nr_nerf_forward         NeRF.forward (NeRF++ background)                models/base.py:426-453
 *   nr_neus_render          neus.volume_render (one ray chunk, render mode) models/frameworks/neus.py:118-397
 *   nr_volsdf_render        volsdf.volume_render (render mode)             models/frameworks/volsdf.py:16-551
 *   nr_unisurf_render       unisurf.volume_render (render mode)            models/frameworks/unisurf.py:62-283,
 *                           + root_finding_surface_points (secant)         models/ray_casting.py:11-160
 *   nr_sample_pdf           rend_util.sample_pdf                             utils/rend_util.py:255-292
 *   nr_get_rays             rend_util.get_rays (+ lift)                      utils/rend_util.py:95-164
 *
 * Conventions
 *   - all pointers are DEVICE pointers (fp32 unless stated) owned by the caller;
 *   - `stream` is a hipStream_t (PyTorch's current stream) passed as void*;
 *   - no hidden allocation: scratch lives in a caller-provided workspace whose size is given by
 *     the matching *_workspace_bytes() query;
 *   - weights are passed as *effective* fp32 matrices (weight_norm folded: W = g * v / ||v||,
 *     models/base.py:226-227) and packed once by *_pack() into the kernels' tile layout;
 *   - every call returns 0 on success or a negative NR_ERR_* code; nr_last_error() gives text.
 *   - no global mutable state besides the thread-local error string: entry points are reentrant.
 */
#ifndef NEURECON_HIP_H
#define NEURECON_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NR_OK 0
#define NR_ERR_ARG (-1)
#define NR_ERR_UNSUPPORTED (-2)
#define NR_ERR_HIP (-3)
#define NR_ERR_WORKSPACE (-4)

/* arithmetic mode of the MLP GEMMs (fp32 accumulate in both) */
#define NR_PREC_FP32 0  /* v_mfma_f32_16x16x4_f32: exact fp32 products                        */
#define NR_PREC_F16X3 1 /* split-fp16 x3 on v_mfma_f32_16x16x32_f16 (hi*hi + hi*lo + lo*hi)     */

/* NeuS upsampling algorithms (models/frameworks/neus.py:213-279) */
#define NR_UPSAMPLE_OFFICIAL 0
#define NR_UPSAMPLE_DIRECT_USE 1
#define NR_UPSAMPLE_DIRECT_MORE 2

int nr_version(void);
const char* nr_last_error(void);
/* 16 hex digits: sha256 of the library's sources and flags at build time (neurecon_amd/build.py
 * source_hash), so a caller can check that the loaded binary is the tree it was built from */
const char* nr_build_id(void);

/* ------------------------------------------------------------------------------------------
 * NeRF++ background MLP (NeRF, models/base.py:395-453) as used by NeuS / VolSDF outside scenes:
 * input_ch=4 ([x/r, 1/r]), multires=10, multires_view=4, use_view_dirs=True, D=8, W=256,
 * skips=[4]; plain nn.Linear layers (no weight norm).  Output: raw sigma and sigmoid rgb.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int D;             /* 8   */
  int W;             /* 256 */
  int skip;          /* 4   */
  int input_ch;      /* 4   */
  int multires;      /* 10  */
  int multires_view; /* 4   */
  int precision;     /* NR_PREC_* */
} NrNerfDesc;

size_t nr_nerf_packed_bytes(const NrNerfDesc* d);
/* W/b: pts_linears[0..7], feature_linear, views_linears[0], alpha_linear, rgb_linear (12 layers,
 * PyTorch [out, in] row-major weights, device pointers) */
int nr_nerf_pack(const NrNerfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream);
/* x4 [P, 4], view dirs [P / vdir_div, 3] -> sigma [P], rgb [P, 3].  Replaces base.py:426-453. */
int nr_nerf_forward(const NrNerfDesc* d, const void* packed, const float* x4, const float* vdir, int64_t vdir_div,
                    int64_t P, float* sigma, float* rgb, void* stream);

/* ------------------------------------------------------------------------------------------
 * SDF MLP  (ImplicitSurface, models/base.py:131-282)
 * D+1 weight-normed linear layers, Softplus(beta=100) hidden activation, skip connection
 * cat([h, embed(x)]) / sqrt(2) before layer `skip`; output row 0 = sdf, rows 1..W_geo_feat =
 * geometry feature.  Supported: D=8, W=256, skip=4, multires in [1,10], W_geo_feat=256.
 * siren != 0: SirenLayer hidden layers h = sin(30 (W h + b)) (base.py:84-115, use_siren, as in
 * configs/volsdf_siren.yaml): D=5, W=256, no skip (skip = -1), identity embedding (multires = -1),
 * W_geo_feat=256.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int D;          /* 8   (5 with siren) */
  int W;          /* 256 */
  int skip;       /* 4   (-1 with siren) */
  int multires;   /* 6   (-1 with siren) */
  int W_geo_feat; /* 256 */
  int precision;  /* NR_PREC_* */
  int siren;      /* 0: Softplus(beta=100) layers */
} NrSdfDesc;

size_t nr_sdf_packed_bytes(const NrSdfDesc* d);
/* W[l]: [out_l, in_l] row-major effective weights, b[l]: [out_l], l = 0..D (device pointers) */
int nr_sdf_pack(const NrSdfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream);
size_t nr_mlp_workspace_bytes(int with_backward);
/* pts [P,3] -> sdf [P]; nabla [P,3] (= d sdf / d x, NULL to skip the backward pass);
 * feature [P, W_geo_feat] (NULL to skip).  Replaces base.py:243-263 / :265-282. */
int nr_sdf_forward(const NrSdfDesc* d, const void* packed, const float* pts, int64_t P, float* sdf, float* nabla,
                   float* feature, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Radiance MLP (RadianceNet, models/base.py:312-391)
 * input cat([embed(x), embed_view(v), normals, feature]) -> D x (Linear+ReLU, W) -> Linear(3)+Sigmoid;
 * with no_view_dirs (use_view_dirs=False, base.py:334-338, :383-384) the input is cat([embed(x),
 * feature]) and view dirs / normals are not read.
 * Supported: D=4 or 5, W=256, multires=-1 (identity on x), view_multires in {-1..7}, W_geo_feat=256,
 * ReLU or (siren) sine hidden layers.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int D;             /* 4   */
  int W;             /* 256 */
  int multires;      /* -1  */
  int multires_view; /* 4 (NeuS) or -1 (VolSDF/UNISURF) */
  int W_geo_feat;    /* 256 */
  int precision;
  int no_view_dirs;  /* 0: use_view_dirs=True (default) */
  int siren;         /* hidden layers sin(30 (W h + b)) instead of ReLU (base.py:357-361); D = 4 or 5 */
} NrRadDesc;

size_t nr_radiance_packed_bytes(const NrRadDesc* d);
int nr_radiance_pack(const NrRadDesc* d, const float* const* W, const float* const* b, void* packed, void* stream);
/* x [P,3], view dirs: vdir[(p / vdir_div) * 3 + c] (vdir_div = samples per ray, or 1),
 * normals [P,3], feature [P,W_geo_feat] -> rgb [P,3]; vdir / normals may be NULL with no_view_dirs */
int nr_radiance_forward(const NrRadDesc* d, const void* packed, const float* x, const float* vdir, int64_t vdir_div,
                        const float* normals, const float* feature, int64_t P, float* rgb, void* stream);

/* ------------------------------------------------------------------------------------------
 * NeuS render, one ray chunk, render mode (neus.py:118-397 with perturb=False,
 * upsample_algo='official_solution').  Rays are [n_rays, 3]; rays_d need not be normalized.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  const float* rays_o;
  const float* rays_d;
  int64_t n_rays;
  const NrSdfDesc* sdf;
  const void* sdf_packed;
  const NrRadDesc* rad;
  const void* rad_packed;
  float s;                   /* exp(ln_s * speed_factor)  (neus.py:108-109)        */
  float obj_bounding_radius; /* near/far sphere radius    (rend_util.py:167-185)   */
  float near_bypass;         /* NaN = unused (neus.py:185-188) */
  float far_bypass;          /* NaN = unused */
  int N_samples;             /* coarse samples, <= 64+... (N_samples + N_importance <= 256) */
  int N_importance;
  int N_upsample_iters;
  int calc_normal;
  int white_bkgd;
  const float* t_coarse; /* torch.linspace(0,1,N_samples) as computed by the host        */
  const float* u_fine;   /* torch.linspace(0,1,N_importance/N_upsample_iters)              */
  /* outputs [n_rays]-major */
  float* rgb;     /* [n_rays,3] */
  float* depth;   /* [n_rays]   */
  float* acc;     /* [n_rays]   */
  float* normals; /* [n_rays,3] (if calc_normal) */
  /* optional per-sample outputs (NULL to skip), ray-major; S = N_samples+N_importance */
  float* d_final;     /* [n_rays, S-1] */
  float* sdf_out;     /* [n_rays, S]   */
  float* nablas_out;  /* [n_rays, S, 3] */
  float* radiance_out;/* [n_rays, S-1, 3] */
  float* alpha_out;   /* [n_rays, S-1] */
  float* cdf_out;     /* [n_rays, S]   */
  float* weights_out; /* [n_rays, S-1] */
  /* NeRF++ background (neus.py:303-343), N_outside = 0 disables it.  With N_outside > 0 the
   * per-sample outputs d_final / radiance_out / alpha_out / weights_out have M = S-1+N_outside
   * entries per ray (mid-points then the inverted-sphere samples). */
  const NrNerfDesc* nerf;
  const void* nerf_packed;
  int N_outside;
  const float* t_outside; /* torch.linspace(0, 1, N_outside + 2) */
  float* sigma_out;       /* [n_rays, M]    raw NeRF sigma ('sigma_out')      */
  float* radiance_bg_out; /* [n_rays, M, 3] NeRF radiance  ('radiance_out')  */
  /* upsampling algorithm (neus.py:213-279): NR_UPSAMPLE_OFFICIAL (N_upsample_iters rounds of
   * N_importance/N_upsample_iters, u_fine = linspace(0,1,N_importance/N_upsample_iters)), or
   * DIRECT_USE / DIRECT_MORE (one sample_pdf of N_importance over the coarse / N_nograd_samples
   * uniform depths with s = 1/fixed_s_recp, u_fine = linspace(0,1,N_importance)) */
  int upsample_algo;
  float fixed_s;          /* 1 / fixed_s_recp (direct algorithms)     */
  int N_nograd_samples;   /* direct_more                               */
  const float* t_nograd;  /* torch.linspace(0, 1, N_nograd_samples)  */
  void* workspace;
  size_t workspace_bytes;
  /* perturb=True (training) uniforms, drawn by the caller exactly as the reference draws them
   * (rend_util.py:271 in sample_pdf, neus.py:306-311 for NeRF++); NULL = deterministic:
   * u_rand: official_solution [N_upsample_iters][n_rays][N_importance/N_upsample_iters],
   *         direct_use / direct_more [n_rays][N_importance] (replace u_fine's linspace);
   * t_out_rand: [n_rays][N_outside] stratification of the inverted-sphere depths. */
  const float* u_rand;
  const float* t_out_rand;
  const float* s_dev; /* optional device scalar s (overrides `s`): no host round trip per call */
  /* sample_only = 1 (training, neus.py:206-279 under torch.no_grad): stop after the upsampling and
   * write the sorted sample depths d_all_out [n_rays, S]; rgb / depth / acc and rad_packed (the radiance
   * net is not evaluated; `rad` still describes it) may then be NULL.  The
   * differentiable part of the step (SDF + nablas, radiance, compositing) runs through the
   * nr_train entry points below. */
  int sample_only;
  float* d_all_out;
  /* Mid-points whose alpha is exactly 0 (the SDF does not decrease from sample i to i+1, neus.py:28-35)
   * contribute w = 0 to every map (with NeRF++, mid-points outside the bounding sphere take the
   * background's colour instead); without the radiance output these skip the SDF and radiance nets
   * (rgb / depth / mask / normals bit-identical).  no_mid_skip != 0: evaluate every
   * mid-point, as the reference does. */
  int no_mid_skip;
  /* Deferred sample nablas (official_solution render without the per-sample nablas / radiance outputs,
   * f16x3 softplus net, chunks of a multiple of 16 rays; with NeRF++ too, flagged after the background
   * net): the sample launches leave their reverse-pass state per 16-sample tile and only the samples
   * of non-zero interval weight run the reverse pass (listed one by one); the other samples' nablas are
   * weighted by exactly 0 in normals_volume (neus.py:364-368).  Maps bit-identical; the workspace then
   * holds 8 KB per sample of a chunk (sized by max_workspace_bytes below).  no_defer != 0: nablas at
   * every sample when drawn. */
  int no_defer;
  /* Memory bound of the render (neus.py:384-397: the reference's `rayschunk` loop is the caller's
   * memory bound).  With max_workspace_bytes 0, rays per internal chunk <= max(max_chunk_rays,
   * NR_MIN_CHUNK_RAYS) (the caller's rayschunk is a hint: a 256-ray validation chunk would leave the
   * per-ray kernels a few CUs); with an explicit max_workspace_bytes, <= max_chunk_rays exactly
   * (<= 0: no bound).  Either way the chunk is sized so that nr_neus_workspace_bytes() <=
   * max_workspace_bytes (0: NR_DEFAULT_WORKSPACE_BYTES), down to one 16-ray chunk. */
  int64_t max_chunk_rays;
  size_t max_workspace_bytes;
} NrNeusArgs;

#define NR_DEFAULT_WORKSPACE_BYTES ((size_t)4 << 30) /* 4 GiB */
#define NR_MIN_CHUNK_RAYS 4096 /* floor of max_chunk_rays when max_workspace_bytes is 0 */

size_t nr_neus_workspace_bytes(const NrNeusArgs* a);
int nr_neus_render(const NrNeusArgs* a, void* stream);

/* ------------------------------------------------------------------------------------------
 * VolSDF rendering (models/frameworks/volsdf.py:377-551, render mode: perturb=False, builtin
 * background sphere or NeRF++ background).  Error-bounded sampling (volsdf.py:77-272) over 4*N_samples initial depths,
 * up to max_upsample_steps rounds of 4*N_samples new depths with max_bisection_steps bisection
 * steps on beta+, then N_importance final depths merged with N_samples uniform ones.
 * Outputs are ray-major; detailed outputs (NULL to skip) have S = N_samples + N_importance
 * samples (S-1 for alpha / p_i / weights).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  const float* rays_o; /* [n_rays, 3] */
  const float* rays_d; /* [n_rays, 3], normalised inside (volsdf.py:388) */
  int64_t n_rays;
  const NrSdfDesc* sdf;
  const void* sdf_packed;
  const NrRadDesc* rad;
  const void* rad_packed;
  float alpha_net, beta_net; /* VolSDF.forward_ab() (volsdf.py:306-308) */
  float beta_plus_init;      /* sqrt(far^2 / (4 (4 N_samples - 1) log(1 + eps))) (volsdf.py:128) */
  float eps;                 /* epsilon, compared in fp32 like the reference */
  float near, far;           /* constant near / far (volsdf.py:408-413) */
  float obj_bounding_radius; /* background sphere radius (volsdf.py:310-325) */
  int use_sphere_bg;
  int N_samples, N_importance, max_upsample_steps, max_bisection_steps;
  int calc_normal, white_bkgd;
  const float* t_coarse; /* torch.linspace(0, 1, N_samples)     (CPU values) */
  const float* t_init;   /* torch.linspace(0, 1, 4 N_samples)   */
  const float* u_up;     /* torch.linspace(0, 1, 4 N_samples + 2) */
  const float* u_fine;   /* torch.linspace(0, 1, N_importance)  */
  float* rgb;            /* [n_rays, 3] */
  float* depth;          /* [n_rays]    */
  float* acc;            /* [n_rays]    */
  float* normals;        /* [n_rays, 3] (calc_normal) */
  float* d_vals;         /* [n_rays, S]   */
  float* sdf_out;        /* [n_rays, S]   implicit_surface */
  float* nablas_out;     /* [n_rays, S, 3] */
  float* radiance_out;   /* [n_rays, S, 3] */
  float* alpha_out;      /* [n_rays, S-1] */
  float* p_out;          /* [n_rays, S-1] p_i */
  float* weights_out;    /* [n_rays, S-1] visibility_weights */
  float* sigma_out;      /* [n_rays, S]   */
  float* beta_map;       /* [n_rays]      */
  float* iter_usage;     /* [n_rays]      */
  void* workspace;
  size_t workspace_bytes;
  /* NeRF++ background (volsdf.py:400-405, 451-469), N_outside > 0 (requires use_sphere_bg = 0):
   * far per ray = exit of the sphere of radius obj_bounding_radius (rend_util.py:188-210; `far`
   * above is then unused), beta+ init per ray = sqrt(far^2 / beta_plus_k) (volsdf.py:127-129),
   * N_outside background samples on the spheres of radii rs_out (rend_util.py:213-234) through the
   * NeRF MLP, composited after the S inside samples.  With N_outside > 0 the detailed outputs
   * d_vals / sigma_out / radiance_out hold M = S + N_outside samples and alpha / p / weights M-1. */
  int N_outside;
  const NrNerfDesc* nerf;
  const void* nerf_packed;
  const float* rs_out;   /* [N_outside] obj_bounding_radius / flip(linspace(0,1,N_outside+2)[1:-1]) (CPU values) */
  float beta_plus_k;     /* float32(4 (4 N_samples - 1) log(1 + eps)) */
  float* sigma_bg;       /* [n_rays, N_outside] sigma_out (detailed, NULL to skip) */
  float* radiance_bg;    /* [n_rays, N_outside, 3] radiance_out (detailed) */
  /* perturb=True (volsdf.py:102 det=not perturb, :460-465), NULL for the deterministic render:
   * u_rand [n_rays, N_importance]: the uniforms of each ray's final sample_cdf (rend_util.py:302-306),
   *   each row sorted ascending (sample_cdf is elementwise in u and the fine depths are sorted into
   *   d_all, volsdf.py:445-446, so a row's order does not reach the outputs);
   * u_out [n_rays, N_outside]: the NeRF++ radius strata uniforms (volsdf.py:460-465). */
  const float* u_rand;
  const float* u_out;
} NrVolsdfArgs;

size_t nr_volsdf_workspace_bytes(const NrVolsdfArgs* a);
int nr_volsdf_render(const NrVolsdfArgs* a, void* stream);

/* ------------------------------------------------------------------------------------------
 * UNISURF rendering (models/frameworks/unisurf.py:62-283, render mode: perturb=False, secant
 * root finding of ray_casting.py:11-160).  P = N_query + N_freespace samples per ray.
 * normal_mode selects what the reference's F.normalize(nablas) (default dim=1, unisurf.py:36)
 * normalises over: 0 = the xyz components of each point (unbatched call, [chunk, 3] tensors),
 * 1 = each component over a batchify_query window of `netchunk` points of one batch row's
 * ray chunk of `rayschunk` rays (batched call, [B, chunk, 3] tensors).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  const float* rays_o; /* [n_rays, 3] */
  const float* rays_d; /* [n_rays, 3], normalised inside (unisurf.py:112) */
  int64_t n_rays;
  int64_t rays_per_batch; /* rays of one batch row (n_rays = B * rays_per_batch); <= 0: n_rays */
  const NrSdfDesc* sdf;
  const void* sdf_packed;
  const NrRadDesc* rad;
  const void* rad_packed;
  float logit_tau;
  float radius_of_interest;
  float interval;
  float too_close_threshold;
  float near_bypass, far_bypass; /* NaN = none */
  int N_steps, N_secant_steps, N_query, N_freespace;
  int normal_mode;
  int64_t rayschunk, netchunk;
  int calc_normal, white_bkgd;
  const float* t_march; /* torch.linspace(0, 1, N_steps)     (CPU values) */
  const float* t_query; /* torch.linspace(0, 1, N_query)     */
  const float* t_free;  /* torch.linspace(0, 1, N_freespace) */
  float* rgb;            /* [n_rays, 3] */
  float* depth;          /* [n_rays]    */
  float* acc;            /* [n_rays]    */
  float* normals;        /* [n_rays, 3] (calc_normal) */
  float* surface_points; /* [n_rays, 3] */
  uint8_t* mask_surface; /* [n_rays] (bool) */
  float* depth_surface;  /* [n_rays]    */
  float* radiance_out;   /* [n_rays, P, 3] */
  float* sdf_out;        /* [n_rays, P] implicit_surface (logits) */
  float* nablas_out;     /* [n_rays, P, 3] */
  float* alpha_out;      /* [n_rays, P] */
  float* weights_out;    /* [n_rays, P] visibility_weights */
  void* workspace;
  size_t workspace_bytes;
  /* perturb=True (unisurf.py:158-165, :187-194): the caller's stratification uniforms (torch.rand
   * in the reference's order), u_query [n_rays, N_query], u_free [n_rays, N_freespace]; t_query /
   * t_free then hold the N+1 bin edges linspace(0, 1, N+1).  NULL = deterministic. */
  const float* u_query;
  const float* u_free;
  /* Multi-GPU ray shard with normal_mode 1: the reference's F.normalize windows span
   * the whole batch (unisurf.py:36, train_util.py:23-71), so every rank computes its partial sums of
   * nabla^2 per window into window_ss ([B][nr_unisurf_window_count][3] fp64, zeroed by the caller),
   * then the library calls window_reduce(window_user) exactly once per nr_unisurf_render call (an
   * all-reduce over the ranks, enqueued on `stream`) and normalises with the totals.  rays are this
   * rank's [B, n_rays / B] slice starting at row-relative ray shard_ray0 of rows of shard_row_rays
   * rays; the shard must be <= 65536 rays.  shard_row_rays = 0: not sharded. */
  int64_t shard_ray0;
  int64_t shard_row_rays;
  double* window_ss;
  int (*window_reduce)(void* user);
  void* window_user;
  /* root finding method (unisurf.py:76 `method`, ray_casting.py:128): 0 = 'secant'; any other method
   * skips the secant refinement and reports depth 1 on hits, as the reference does */
  int no_secant;
  /* training (unisurf.py:140-211 under torch.no_grad in neurecon_amd's training render): d_all_out
   * [n_rays, P] receives each ray's sorted sample depths d_all (unisurf.py:201); sample_only != 0 stops
   * after the sampling (root finding + interval / free-space samples; surface_points / mask_surface /
   * depth_surface are still written when given) -- rgb / depth / acc and rad_packed may then be NULL */
  float* d_all_out;
  int sample_only;
  /* full_march != 0: the root-finding march evaluates every step of every ray in one launch (the
   * reference's schedule, ray_casting.py:88-101; bit-identical outputs, slower).  0 (default): in
   * chunks of 32 steps over the rays still without a sign change */
  int full_march;
} NrUnisurfArgs;

size_t nr_unisurf_workspace_bytes(const NrUnisurfArgs* a);
int nr_unisurf_render(const NrUnisurfArgs* a, void* stream);
/* F.normalize windows per batch row of the whole batch (normal_mode 1), for sizing window_ss */
int64_t nr_unisurf_window_count(const NrUnisurfArgs* a);

/* ------------------------------------------------------------------------------------------
 * Inverse-CDF sampling (rend_util.sample_pdf, utils/rend_util.py:255-292): bins [R, L],
 * weights [R, L-1] -> samples [R, N].  det=True: u [N] shared and ascending (u_stride = 0);
 * det=False: the caller's uniforms u[r * u_stride + k] (any order), e.g. torch.rand([R, N]).
 * ------------------------------------------------------------------------------------------ */
int nr_sample_pdf(const float* bins, const float* weights, int64_t R, int L, const float* u, int64_t u_stride, int N,
                  float* out, void* stream);

/* ------------------------------------------------------------------------------------------
 * Pixel -> ray (rend_util.get_rays, pose-matrix form): c2w [B,4,4], K [B,4,4] (row-major),
 * select_inds [B,N] int64 pixel indices (row*W+col) or NULL for all N = H*W pixels in order.
 * rays_o, rays_d [B,N,3]; rays_d is NOT normalized (rend_util.py:159-162).
 * ------------------------------------------------------------------------------------------ */
int nr_get_rays(const float* c2w, const float* K, int B, int H, int W, const int64_t* select_inds, int64_t N,
                float* rays_o, float* rays_d, void* stream);
/* training targets of a random ray batch (neus.py:432 torch.gather of ground_truth['rgb'], :449 of
 * the object mask): out[b, n] = src[b, idx[b, n]] for rows of row_bytes bytes, src [B, HW, ...] */
int nr_gather_rows(const void* src, int64_t B, int64_t HW, int64_t row_bytes, const int64_t* idx, int64_t N, void* out,
                   void* stream);

/* ------------------------------------------------------------------------------------------
 * Surface rendering (models/ray_casting.py:163-263).
 * nr_sphere_trace replaces `sphere_tracing_surface_points` (ray_casting.py:163-182): from d = near,
 * n_iters times d += sdf(o + d*dir) on rays still inside [0, far]; near / far scalars, or per-ray [R]
 * device arrays near_rays / far_rays when non-null (the reference broadcasts tensor near/far,
 * :175, :180); rays_d as given (surface_render normalizes first, ray_casting.py:209).  Outputs d_pred [R], pts [R,3] (= o + d*dir), mask [R]
 * (u8).  Only still-active rays are evaluated (compacted on device).  Workspace:
 * nr_sphere_trace_workspace_bytes(R).
 * nr_normalize3: F.normalize(v, dim=-1) of [n,3] (ray_casting.py:209).
 * nr_surface_finish: surface_render's tail (ray_casting.py:226, 255-258): rgb[~mask] = 0 in place;
 * normals (optional) = F.normalize(nablas) with normals[~mask] = 0.
 * ------------------------------------------------------------------------------------------ */
size_t nr_sphere_trace_workspace_bytes(int64_t n_rays);
int nr_sphere_trace(const NrSdfDesc* d, const void* packed, const float* rays_o, const float* rays_d, int64_t n_rays,
                    float near, float far, const float* near_rays, const float* far_rays, int n_iters, float* d_pred,
                    float* pts, uint8_t* mask, void* workspace, size_t workspace_bytes, void* stream);
/* nr_root_find replaces `root_finding_surface_points` (ray_casting.py:35-160): N_steps march samples
 * at near*(1-t)+far*t (t_march = torch.linspace(0,1,N_steps), CPU values), first sign change of
 * sdf - logit_tau, N_secant_steps secant refinements on rays entering the surface from outside with
 * a free first sample (no_secant != 0: method != 'secant', ray_casting.py:128-135 -- no refinement,
 * depth 1 on hits).  near / far: scalars, or per-ray [R] device arrays near_rays / far_rays when
 * non-null (the reference's tensor near/far, :53-54, :70-73).  Outputs d_pred [R] (inf if fill_inf,
 * else far, on misses; 0 when the first sample is occupied), pts [R,3] (1 on misses), mask [R],
 * mask_sign_change [R] (u8, optional).  rays_d as given (already normalised).  The march runs in
 * chunks of 32 steps over the rays still without a sign change (a ray's march is read only up to its
 * first crossing: bit-identical outputs); full_march != 0 evaluates every step of every ray in one
 * launch (the reference's schedule).  Workspace: nr_root_find_workspace_bytes. */
size_t nr_root_find_workspace_bytes(int64_t n_rays, int N_steps);
int nr_root_find(const NrSdfDesc* d, const void* packed, const float* rays_o, const float* rays_d, int64_t n_rays,
                 float near, float far, const float* near_rays, const float* far_rays, int N_steps,
                 const float* t_march, int N_secant_steps, int no_secant, float logit_tau, int fill_inf,
                 int full_march, float* d_pred, float* pts, uint8_t* mask, uint8_t* mask_sign_change, void* workspace,
                 size_t workspace_bytes, void* stream);
int nr_normalize3(const float* v, int64_t n, float* out, void* stream);
int nr_surface_finish(float* rgb, const float* nablas, const uint8_t* mask, int64_t n, float* normals, void* stream);

/* ------------------------------------------------------------------------------------------
 * Mesh-extraction SDF grid (utils/mesh_util.py:82-112 `extract_mesh`): points
 * [i0, i0+n) of the N^3 voxel grid of edge `volume_size` centred at the origin, generated on the
 * device with the reference's float64 formula (:87-100, including its true divisions), then the
 * forward SDF (ImplicitSurface.forward) -> sdf [n].  Workspace: nr_sdf_grid_workspace_bytes(n).
 * ------------------------------------------------------------------------------------------ */
size_t nr_sdf_grid_workspace_bytes(int64_t n_points);
int nr_sdf_grid(const NrSdfDesc* d, const void* packed, double volume_size, int64_t N, int64_t i0, int64_t n,
                float* sdf, void* workspace, size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Training path (models/frameworks/neus.py:417-485, models/base.py:265-282 with
 * create_graph=True).  The host runs the step layer by layer: the dense [P, K] x [K, N] layer
 * products go to hipBLASLt, every per-point / per-ray step between them is one of these kernels.
 * The double backward through the nablas is reverse mode over the (primal, tangent) network (see
 * nr_train.hip): tangent seed J_emb(x) grad_nabla, adjoint zbar = hbar s + g zdot s'.
 *   nr_embed          Embedder.forward (base.py:46-64): [P,3] -> [P, 3+6F]
 *   nr_embed_jvp      J_emb(x) v                      (tangent seed)
 *   nr_embed_vjp      J_emb(x)^T (e0 + s1 e1) -> [P,3] (nablas; autograd.grad through the encoding)
 *   nr_softplus100    Softplus(beta=100, threshold=20) (base.py:202) and softplus_backward's factor
 *   nr_scale_cols     out = a[:, col0:col0+n] * scale (* s)  (skip-connection split, delta = s * g)
 *   nr_softplus_adjoint  zbar = hbar * s + g * zdot * 100 s (1 - s)  (softplus_double_backward)
 *   nr_mul / nr_activation  elementwise product; ReLU / sigmoid forward (in place) and backward
 *   nr_radiance_input cat([x, embed_view(v), normals, feature]) (base.py:379-384), or cat([x, feature])
 *                     when use_view_dirs = 0 (v / nrm unused); wfeat = 0: without the feature (feat unused)
 *   nr_neus_points    pts / d_mid / pts_mid of the sorted sample depths (neus.py:284-288)
 *   nr_neus_composite_fwd/bwd  sdf_to_alpha, alpha_to_w, rgb / depth / acc (neus.py:28-70, 346-355)
 *                      and their gradient w.r.t. sdf, radiance and s (per-ray partials of d s)
 * ------------------------------------------------------------------------------------------ */
int nr_embed(const float* x, int64_t P, int nfreq, float* out, void* stream);
int nr_embed_jvp(const float* x, const float* v, int64_t P, int nfreq, float* out, void* stream);
/* the same into rows of ldo >= 3+6F floats, zero beyond the features (the training GEMMs' 16-column blocks) */
int nr_embed_padded(const float* x, int64_t P, int nfreq, float* out, int ldo, void* stream);
int nr_embed_jvp_padded(const float* x, const float* v, int64_t P, int nfreq, float* out, int ldo, void* stream);
int nr_embed_vjp(const float* x, const float* e0, int ld0, const float* e1, int ld1, float s1, int64_t P, int nfreq,
                 float* out, void* stream);
int nr_softplus100(const float* z, int64_t n, float* h, float* s, void* stream);
int nr_scale_cols(const float* a, int64_t P, int lda, int col0, int ncols, const float* s, float scale, float* out,
                  void* stream);
int nr_softplus_adjoint(const float* hbar, int ldh, const float* s, const float* g, const float* zdot, int64_t P,
                        int n, float* zbar, void* stream);
/* column sums of a row-major [P, n] fp32 matrix (the training path's bias gradients), deterministic
 * two-pass reduction; workspace nr_colsum_workspace_bytes(n) */
size_t nr_colsum_workspace_bytes(int n);
int nr_colsum(const float* a, int64_t P, int n, float* out, void* workspace, size_t workspace_bytes, void* stream);
/* SirenLayer activation (base.py:84-115) in the training path: h = sin(30 z), s = 30 cos(30 z); and
 * the layer's adjoint in the double backward, zbar = hbar * s + g * zdot * (-900 h) (g / zdot optional,
 * as nr_softplus_adjoint) */
int nr_sine30(const float* z, int64_t n, float* h, float* s, void* stream);
int nr_sine_adjoint(const float* hbar, int ldh, const float* s, const float* h, const float* g, const float* zdot,
                    int64_t P, int n, float* zbar, void* stream);
int nr_mul(const float* a, const float* b, int64_t n, float* out, void* stream);
/* mode 0: y = relu(y); 1: g *= (y > 0); 2: y = sigmoid(y); 3: g *= y (1 - y) */
int nr_activation(float* y, float* g, int64_t n, int mode, void* stream);
/* weight_norm(dim=0) of up to NR_WN_MAX layers in one launch (torch._weight_norm, models/base.py:118-129,
 * 226-227): w = v * (g / ||v_row||), norm[row] saved for the backward; backward (torch's
 * weight_norm_bwd_first_dim): dot = sum grad_w * v per row, grad_g = dot / norm, grad_v = (g / norm) *
 * (grad_w - v * dot / norm^2).  v / w / grad_w / grad_v [rows][cols] row-major, g / norm / grad_g [rows];
 * a null grad_w is a zero gradient.  One 64-lane wave per row, fp32 sums in a fixed order. */
#define NR_WN_MAX 16
typedef struct {
  const float* v;
  const float* g;
  float* w;          /* forward output */
  float* norm;       /* forward output / backward input */
  const float* grad_w;
  float* grad_v;
  float* grad_g;
  int rows;
  int cols;
} NrWnLayer;
int nr_weight_norm_fwd(const NrWnLayer* layers, int n, void* stream);
int nr_weight_norm_bwd(const NrWnLayer* layers, int n, void* stream);
/* One torch.optim.Adam step (train.py:main's optimizer; amsgrad = maximize = False) over up to
 * NR_ADAM_MAX fp32 parameter tensors in one launch, in place: g += weight_decay * p; m = b1 m + (1 - b1) g;
 * v = b2 v + (1 - b2) g^2; p -= lr / (1 - b1^step) * m / (sqrt(v) / sqrt(1 - b2^step) + eps) -- the
 * update of torch's fused Adam (replaces its multi-tensor launches, ~45 us each for the NeuS nets).
 * step = the step count after this update (>= 1), shared by every tensor of the call.  The hyper-parameters
 * are doubles (as torch passes them): 1 - beta and the bias corrections are formed in double, then rounded. */
#define NR_ADAM_MAX 64
typedef struct {
  float* param;
  const float* grad;
  float* exp_avg;
  float* exp_avg_sq;
  int64_t n;
} NrAdamTensor;
int nr_adam_step(const NrAdamTensor* tensors, int n, int64_t step, double lr, double beta1, double beta2, double eps,
                 double weight_decay, void* stream);
int nr_radiance_input(const float* x, const float* v, const float* nrm, const float* feat, int64_t P, int nfreq_view,
                      int use_view_dirs, int wfeat, float* out, void* stream);
int nr_neus_points(const float* rays_o, const float* rays_d, const float* d_all, int64_t R, int S, float* pts,
                   float* mids, float* dmid, void* stream);
int nr_neus_composite_fwd(const float* sdf, const float* s_dev, const float* rad, const float* dmid, int64_t R, int S,
                          int white_bkgd, float* rgb, float* depth, float* acc, float* weights, float* alpha,
                          float* cdf, void* stream);
size_t nr_neus_composite_bwd_workspace_bytes(int64_t R, int S);
int nr_neus_composite_bwd(const float* sdf, const float* s_dev, const float* rad, const float* dmid, int64_t R, int S,
                          int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc,
                          const float* g_weights, float* d_sdf, float* d_rad, float* d_s, void* workspace,
                          size_t workspace_bytes, void* stream);
/* NeRF++ background in the training step (neus.py:303-343):
 *   nr_nerf_train_input  x_emb [R*M, 84] = Embedder(4, 10)([p/|p|, 1/|p|]), p = o + d_out*dir;
 *                        v_emb [R*M, 27] = Embedder(3, 4)(dir); inside [R, n_mid] = |p_k| <= r_obj
 *                        for the first n_mid (= S-1 mid-point) depths
 *   nr_neus_composite_bg_fwd / _bwd  the compositing with the background merged (neus.py:325-352):
 *                        sdf [R,S], radiance [R,S-1,3] of the surface net, sigma_out [R,M] and
 *                        radiance_out [R,M,3] of the background net at d_out [R,M] (M = S-1+N_outside);
 *                        weights / alpha [R,M]; backward also -> d sigma_out, d radiance_out */
int nr_nerf_train_input(const float* rays_o, const float* rays_d, const float* d_out, int64_t R, int M, int n_mid,
                        float r_obj, float* x_emb, float* v_emb, uint8_t* inside, void* stream);
int nr_neus_composite_bg_fwd(const float* sdf, const float* s_dev, const float* rad, const float* sigma_out,
                             const float* rad_out, const float* d_out, const uint8_t* inside, int64_t R, int S, int M,
                             int white_bkgd, float* rgb, float* depth, float* acc, float* weights, float* alpha,
                             float* cdf, void* stream);
size_t nr_neus_composite_bg_bwd_workspace_bytes(int64_t R, int S, int M);
int nr_neus_composite_bg_bwd(const float* sdf, const float* s_dev, const float* rad, const float* sigma_out,
                             const float* rad_out, const float* d_out, const uint8_t* inside, int64_t R, int S, int M,
                             int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc,
                             const float* g_weights, float* d_sdf, float* d_rad, float* d_sigma_out,
                             float* d_rad_out, float* d_s, void* workspace, size_t workspace_bytes, void* stream);

/* VolSDF training compositing (replaces the autograd graph of volsdf.py:449-506 with the builtin
 * background of volsdf.py:317-325 and sdf_to_sigma volsdf.py:16-35).  sdf [R,S] network values at
 * pts [R,S,3], beta_dev [1] = exp(ln_beta * speed_factor), radiance [R,S,3] (the first S-1 rows are
 * composited), d_all [R,S] sorted depths.  use_bg: min(sdf, r_bg - |x|).  Outputs rgb [R,3], depth [R],
 * acc [R], tau [R,S-1] (visibility weights), optional p_i [R,S-1], sigma [R,S], sdf_out [R,S]
 * (background applied).  The backward takes the output gradients (each may be NULL) and returns
 * d sdf [R,S] (0 where the background value was taken), d radiance [R,S,3] and d beta per ray [R]. */
int nr_volsdf_composite_fwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                            const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd, float* rgb,
                            float* depth, float* acc, float* tau, float* p_i, float* sigma, float* sdf_out,
                            void* stream);
size_t nr_volsdf_composite_bwd_workspace_bytes(int64_t R, int S);
int nr_volsdf_composite_bwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                            const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd,
                            const float* g_rgb, const float* g_depth, const float* g_acc, const float* g_tau,
                            const float* g_sdf, float* d_sdf, float* d_rad, float* d_beta, void* workspace,
                            size_t workspace_bytes, void* stream);
/* the same with VolSDF's NeRF++ background (volsdf.py:455-469): N background samples after the S inner
 * ones, sigma_bg [R,N] (the background net's raw sigma), radiance_bg [R,N,3], d_bg [R,N]; tau / p_i
 * [R,S+N-1], sigma [R,S+N]; the backward adds d sigma_bg [R,N] and d radiance_bg [R,N,3]. */
int nr_volsdf_composite_bg_fwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                               const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd,
                               const float* sigma_bg, const float* rad_bg, const float* d_bg, int N, float* rgb,
                               float* depth, float* acc, float* tau, float* p_i, float* sigma, float* sdf_out,
                               void* stream);
size_t nr_volsdf_composite_bg_bwd_workspace_bytes(int64_t R, int S, int N);
int nr_volsdf_composite_bg_bwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                               const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd,
                               const float* sigma_bg, const float* rad_bg, const float* d_bg, int N,
                               const float* g_rgb, const float* g_depth, const float* g_acc, const float* g_tau,
                               const float* g_sdf, float* d_sdf, float* d_rad, float* d_beta, float* d_sigma_bg,
                               float* d_rad_bg, void* workspace, size_t workspace_bytes, void* stream);
/* inputs of VolSDF's NeRF++ background net in the training step (volsdf.py:456-467): p = o + d_bg*dir,
 * x_emb [R*N, 84] = Embedder(4, 10)([p / rs, 1 / rs]) at the sample radii rs [R,N], v_emb [R*N, 27] =
 * Embedder(3, 4)(dir) */
int nr_volsdf_nerf_input(const float* rays_o, const float* rays_d, const float* d_bg, const float* rs, int64_t R,
                         int N, float* x_emb, float* v_emb, void* stream);

/* UNISURF compositing with a graph (unisurf.py:219-236, get_opacity_from_surface :53-62): logits [R,P]
 * (implicit_surface), radiance [R,P,3], d_all [R,P].  alpha = exp(-l) / (1 + exp(-l)), visibility weights
 * w = alpha * cumprod(1 - alpha + 1e-10) (exclusive); outputs rgb [R,3], depth [R], acc [R], w [R,P],
 * optional alpha [R,P].  The backward takes the output gradients (each may be NULL) and returns
 * d logits [R,P] and d radiance [R,P,3]. */
int nr_unisurf_composite_fwd(const float* logits, const float* rad, const float* d_all, int64_t R, int P,
                             int white_bkgd, float* rgb, float* depth, float* acc, float* weights, float* alpha,
                             void* stream);
size_t nr_unisurf_composite_bwd_workspace_bytes(int64_t R, int P);
int nr_unisurf_composite_bwd(const float* logits, const float* rad, const float* d_all, int64_t R, int P,
                             int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc,
                             const float* g_weights, float* d_logits, float* d_rad, void* workspace,
                             size_t workspace_bytes, void* stream);

/* ------------------------------------------------------------------------------------------
 * Training layer GEMMs (f16x3 MFMA; the dense layer products of the training step together with the
 * elementwise step that follows each -- base.py:245-282 forward / nablas with create_graph=True,
 * base.py:372-391 radiance -- replacing an addmm / mm on hipBLASLt plus one to three elementwise
 * launches).  One call applies one packed op of a weight stream to a row-major [P, K] activation:
 *   Y[p, o] = epi( sum_i X[p, i] M[o, i] (+ bias[o]) ),   M = W (forward ops) or W^T (backward ops)
 * X = [x1 (KB - KB2 blocks of 16 columns) ; x2 (KB2 blocks)], Y = [y (NBO - NB2 blocks) ; yb (NB2)].
 * epi (mode):
 *   NR_TG_NONE      y = z * yscale
 *   NR_TG_SOFTPLUS  y = softplus100(z), y2 = softplus'(z), y3 = y2 * rowvec, dot = y . rowvec + dot_bias
 *                   (rowvec: the op's per-row vector, e.g. W8[0, :] riding F7: delta_7 and the sdf)
 *   (2: reserved -- the radiance forward stays on fp32 GEMMs, whose ReLU masks match the reference's;
 *    the head / head_bias / head_out fields are unused)
 *   NR_TG_MUL       y = z * yscale, y2 = a * y            (nabla chain delta = s * g, tangent hdot = s * zdot)
 *   NR_TG_SPADJ     y = hbar s + g zdot 100 s (1 - s), hbar = z * yscale, s = a, g = g (or rowvec with g_row)
 *   NR_TG_RELUMASK  y = z where a > 0, else 0             (ReLU backward on the saved activation)
 * Ops come from the render pack (nr_sdf_pack / nr_radiance_pack: forward ops and the SDF net's
 * transposed ops) and the training pack (nr_sdf_train_pack: W8^T with W8[0, :] as its row vector;
 * nr_radiance_train_pack: the radiance net's transposed ops); nr_*_op_info give an op's byte offset
 * in its buffer, input blocks and output blocks.  Supported (KB, KB2, NBO, NB2, mode) shapes are the
 * training path's own (NR_ERR_UNSUPPORTED otherwise).
 * ------------------------------------------------------------------------------------------ */
#define NR_TG_NONE 0
#define NR_TG_SOFTPLUS 1
#define NR_TG_MUL 3
#define NR_TG_SPADJ 4
#define NR_TG_RELUMASK 5

typedef struct {
  const char* op;        /* packed op */
  int64_t P;
  const float* x1;       /* x1[p * ld1 + col], n1 valid columns (the rest of its blocks read as 0) */
  int64_t ld1;
  int n1;
  const float* x2;
  int64_t ld2;
  int n2;
  int use_bias;
  int mode;
  float yscale;
  float* y;              /* NULL: those blocks are not stored (at least one output must be given) */
  int64_t ldy;
  float* yb;             /* NULL: those blocks are not stored */
  int64_t ldyb;
  float* y2;
  int64_t ldy2;
  float* y3;
  int64_t ldy3;
  const float* a;
  int64_t lda;
  const float* g;
  int64_t ldg;
  const float* zd;
  int64_t ldzd;
  int g_row;
  float* dot;
  float dot_bias;
  const float* head;     /* [3][256] */
  const float* head_bias;
  float* head_out;       /* [P][3] */
  int blocked;           /* NR_BLK_* bits: those tensors are 16 x 16 blocked (below), the rest row-major */
  int g_scaled;          /* NR_TG_SPADJ: g holds s * g (the nabla chain's delta) and the g zdot term uses
                            100 (1 - s) -- the nabla sweep then need not store g at all */
} NrTrainGemm;

/* 16 x 16 blocked layout of a [P, ld] tensor (ld and P multiples of 16): element (p, c) at float
 * ((p / 16) * (ld / 16) + c / 16) * 256 + (p % 16) * 16 + c % 16 -- a 16-point x 16-column block is one
 * contiguous 1 KB run, which is what one wave-instruction of the training GEMMs' epilogues and of
 * nr_wgrad's loaders reads or writes (row-major: 16 rows x 64 B).  Same size as the row-major tensor. */
#define NR_BLK_X1 1
#define NR_BLK_X2 2
#define NR_BLK_Y 4
#define NR_BLK_YB 8
#define NR_BLK_Y2 16
#define NR_BLK_Y3 32
#define NR_BLK_A 64
#define NR_BLK_G 128
#define NR_BLK_ZD 256

int nr_train_gemm(const NrTrainGemm* a, int KB, int KB2, int NBO, int NB2, void* stream);
/* SDF ops: 0..16 = F0..F8, B7..B0 of the render pack (nr_sdf_pack), 17 = B8 of the training pack */
int nr_sdf_op_info(const NrSdfDesc* d, int op, int64_t* offset, int* kb, int* nbo);
size_t nr_sdf_train_packed_bytes(const NrSdfDesc* d);
int nr_sdf_train_pack(const NrSdfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream);
/* radiance ops: 0..D-1 = forward ops of the render pack (op 0: [feature ; small inputs]), D = head
 * offset ([3][256] then [3] bias; kb = nbo = 0); training pack: D+1 = head^T, D+2.. = W_{D-1}^T .. W_1^T,
 * 2D+1 = W_0^T (output blocks [feature ; small inputs]) */
int nr_radiance_op_info(const NrRadDesc* d, int op, int64_t* offset, int* kb, int* nbo);
/* Training forward of a ReLU D=4 radiance net (RadianceNet.forward with a graph, base.py:372-391) with
 * exact fp32 products: `packed` is the net's pack for a desc with precision NR_PREC_FP32 (nr_radiance_pack),
 * feat [P][256], small[p * ld_small + f] the small inputs [x, embed_view(v), normals] (nr_radiance_input's
 * first columns); outputs the hidden activations h0..h3 [P][256] (after the ReLU, for the backward) and
 * rgb [P][3] (sigmoid).  The layers chain in registers in one launch; the ReLU masks come from fp32
 * pre-activations as the reference's.  NR_ERR_UNSUPPORTED for SIREN / D != 4 / f16x3 packs. */
int nr_radiance_train_fwd32(const NrRadDesc* d, const void* packed, const float* feat, const float* small,
                            int64_t ld_small, int64_t P, float* h0, float* h1, float* h2, float* h3, float* rgb,
                            void* stream);
/* NeRF++ background net in the training step (NeRF.forward with a graph, base.py:426-453), exact fp32
 * products, replacing NeRFFn's hipBLASLt GEMMs (neurecon_amd/training.py):
 *   nr_nerf_train_fwd32  `packed` = nr_nerf_pack for a desc with precision NR_PREC_FP32; x_emb [P][84]
 *                        (16-byte aligned) and v_emb [P][27] from nr_nerf_train_input; outputs the 8 ReLU
 *                        activations h[0..7] [P][256], the feature [P][256], the view branch's ReLU output
 *                        hv [P][128], sigma [P] and rgb [P][3] in one launch
 *   nr_nerf_train_pack   the backward's transposed ops (views^T, feature^T, W7^T .. W1^T) and the rgb /
 *                        alpha rows, in d->precision (r06: NR_PREC_F16X3 packs them for the f16x3
 *                        products below); W / b as nr_nerf_pack's 12 layers (biases unused)
 *   nr_nerf_train_bwd32  the data gradients in one launch: g3 = g_rgb * sigmoid' [P][3], ghv = (g3 Wr) *
 *                        [hv > 0] [P][128], g_feat = Wv[:, :256]^T ghv [P][256], gz[7] = (Wf^T g_feat +
 *                        g_sigma Wa) * [h7 > 0], gz[i-1] = (W_i^T gz[i])[h columns] * [h_{i-1} > 0]; g_rgb /
 *                        g_sigma may be null (zero).  The products are exact fp32 for d->precision
 *                        NR_PREC_FP32, f16x3 for NR_PREC_F16X3 (the backward is linear in the forward's
 *                        stored ReLU masks, so no decision depends on their rounding); `train_packed` must
 *                        come from nr_nerf_train_pack with the same precision.  The weight gradients are
 *                        nr_wgrad products of these. */
int nr_nerf_train_fwd32(const NrNerfDesc* d, const void* packed, const float* x_emb, const float* v_emb, int64_t P,
                        float* const* h, float* feat, float* hv, float* sigma, float* rgb, void* stream);
size_t nr_nerf_train_packed_bytes(const NrNerfDesc* d);
int nr_nerf_train_pack(const NrNerfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream);
int nr_nerf_train_bwd32(const NrNerfDesc* d, const void* train_packed, const float* rgb, const float* hv,
                        const float* const* h, const float* g_rgb, const float* g_sigma, int64_t P, float* g3,
                        float* ghv, float* g_feat, float* const* gz, void* stream);
size_t nr_radiance_train_packed_bytes(const NrRadDesc* d);
int nr_radiance_train_pack(const NrRadDesc* d, const float* const* W, const float* const* b, void* packed,
                           void* stream);

/* ------------------------------------------------------------------------------------------
 * Weight gradients of the training step (f16x3 MFMA, nr_wgrad.hip): the DenseLayer weight gradients
 * of models/base.py:118-129 under the double backward (base.py:265-282, train.py:205) -- autograd's
 * mm(grad_out^T, input) over the sample points -- as
 *   c[i * ldc + j] = scale * sum_q sum_p a_q[p * lda_q + i] * b_q[p * ldb_q + j]   (i < m, j < n)
 * for one or two (a, b) pairs (the primal and tangent sweeps of one layer); optional:
 *   colsum[i] = sum_p a_0[p * lda_0 + i]                  (the bias gradient),
 *   vec[j]    = vec_scale * sum_p avec[p * ldv] b_0[p * ldb_0 + j]   (one extra output row).
 * Deterministic (fixed-order slice reduction).  Workspace: nr_wgrad_workspace_bytes(P, m, n, npairs).
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  int64_t P;
  int npairs;
  const float* a[2];
  int64_t lda[2];
  const float* b[2];
  int64_t ldb[2];
  int m, n;
  float scale;
  float* c;
  int64_t ldc;
  float* colsum;      /* [m] or NULL */
  const float* avec;  /* [P] (stride ldv) or NULL */
  int64_t ldv;
  float* vec;         /* [n] or NULL */
  float vec_scale;
  void* workspace;
  size_t workspace_bytes;
  int blocked;        /* NR_WG_BLK_* bits: those operands are 16 x 16 blocked (NR_BLK_* comment above:
                         lda / ldb and P multiples of 16), the rest row-major */
  int fp32;           /* 0: f16x3 products (hi*hi + hi*lo + lo*hi, running per-quad exponents);
                         1: exact fp32 products (v_mfma_f32_16x16x4_f32), the fp32-precision nets' path */
} NrWgrad;
#define NR_WG_BLK_A0 1
#define NR_WG_BLK_A1 2
#define NR_WG_BLK_B0 4
#define NR_WG_BLK_B1 8

size_t nr_wgrad_workspace_bytes(int64_t P, int m, int n, int npairs);
int nr_wgrad(const NrWgrad* w, void* stream);

/* Layer products of the fp32 / SIREN nets' training step (nn.Linear forward, models/base.py:118-129,
 * 243-263, SirenLayer base.py:84-115, RadianceNet base.py:372-391, and their autograd -- torch.addmm /
 * mm in the reference): C[M, N] (row stride ldc) = A[M, K] (lda) op(B) (+ bias[N], may be NULL),
 * op(B) = B^T for B [N, K] (ldb) with trans_b != 0 (A W^T), else B [K, N] (ldb); K > 0.  Exact fp32
 * products accumulated in fp64 (v_mfma_f64_16x16x4_f64) and rounded once, the bias added last; acc32
 * != 0: accumulated in fp32 in k order instead (v_mfma_f32_16x16x4_f32, an fmaf chain per element). */
int nr_gemm32(const float* A, int64_t lda, const float* B, int64_t ldb, int trans_b, const float* bias, float* C,
              int64_t ldc, int64_t M, int N, int K, int acc32, void* stream);

/* ------------------------------------------------------------------------------------------
 * Opt-in kernel timing (diagnostics / bench roofline).  While enabled, every kernel launch of
 * the library is bracketed by hipEvents on its stream; nr_profile_read() waits for them and
 * returns per-kernel totals (launches, milliseconds, work units: points or rays), then clears.
 * ------------------------------------------------------------------------------------------ */
typedef struct {
  char name[32];
  int64_t launches;
  double ms;
  double units;
} NrKernelStat;

int nr_profile_enable(int on);
/* record only the launches whose kernel name starts with prefix (NULL or "": every launch); each
 * recorded launch costs two event markers (and, for compacted launches, a count copy) on the stream */
int nr_profile_filter(const char* prefix);
int nr_profile_read(NrKernelStat* out, int max, int* n_out);

/* Kernel selection experiment (no reference counterpart): on != 0 routes the f16x3
 * softplus SDF nets' forward-only evaluations (nr_sdf_forward without nablas or feature, the UNISURF /
 * root-finding march, sphere tracing, the mesh grid, VolSDF's no-grad sampling) to the
 * v_mfma_f32_32x32x16_f16 kernel (one wave per SIMD, nr_sdf5.hip) instead of the 16x16x32 one; both
 * meet the same bars, their results differ by rounding.  Measured 3 % slower, so off by default.
 * Needs the process started with $NR_SDF5 set to a nonzero integer (the packs then carry the 32x32x16 layout as well;
 * nr_sdf_packed_bytes grows): returns -1 otherwise, else the previous setting. */
int nr_sdf5_enable(int on);

#ifdef __cplusplus
}
#endif
#endif /* NEURECON_HIP_H */
