// neurecon_amd — UNISURF render path internals (models/frameworks/unisurf.py, models/ray_casting.py).
#pragma once
#include "nr_common.h"

namespace nr {

// Device views of one ray chunk.  Per-ray arrays are sample-major ([sample][ray]) for the
// one-thread-per-ray kernels; the MLP kernels see flat point lists p = sample * R + ray.
struct UniChunk {
  int R;             // rays in this chunk
  int N_steps;       // root-finding march samples
  int N_query, N_free, P;  // P = N_query + N_free
  float logit_tau, interval, too_close;
  float near_bypass, far_bypass;  // NaN = none
  float r_interest;
  float* ro; float* rd; float* near; float* far; float* thr;
  float* pts_m;      // [N_steps][R][3] march points
  float* sm;         // [N_steps][R] march sdf
  float* sec;        // [R][8]: d_lo, f_lo, d_hi, f_hi, d_pred, hit, crossing, first_free
  float* pts_s;      // [R][3] secant points
  float* ss;         // [R] secant sdf
  float* d_all;      // [P][R]
  float* pts_f;      // [P][R][3]
  float* sdf_f; float* nab_f; float* feat_f; float* nrm_f; float* rad_f;
  double* wss;       // [windows][3] sum of squares of the nablas per normalisation window
  int64_t netchunk;  // points per F.normalize window (normal_mode 1)
  const float* t_march; const float* t_query; const float* t_free;
};

struct UniOut {
  int64_t ray0;
  float* rgb; float* depth; float* acc; float* normals;
  float* surface_points; uint8_t* mask_surface; float* depth_surface;
  float* radiance; float* sdf; float* nablas; float* alpha; float* weights;
};

struct UniPlan {
  int64_t Rc;
  size_t o_ro, o_rd, o_near, o_far, o_thr, o_ptsm, o_sm, o_sec, o_ptss, o_ss, o_dall, o_ptsf, o_sdff, o_nabf;
  size_t o_featf, o_nrmf, o_radf, o_wss, o_mlp;
  size_t total;
  int64_t max_windows;
};

UniPlan unisurf_plan(const NrUnisurfArgs& a, int64_t Rc);
int64_t unisurf_chunk_rays(const NrUnisurfArgs& a);

__global__ void uni_prologue(UniChunk c, const float* rays_o, const float* rays_d);
__global__ void uni_root(UniChunk c);
__global__ void rf_prologue(UniChunk c, const float* rays_o, const float* rays_d, float near, float far);
__global__ void rf_finish(UniChunk c, int64_t ray0, float* d_out, float* pts, uint8_t* mask, uint8_t* msc,
                          int fill_inf);
__global__ void uni_secant(UniChunk c, int last);
__global__ void uni_samples(UniChunk c, UniOut o);
__global__ void uni_window_ss(UniChunk c);
__global__ void uni_normalize(UniChunk c, int mode);
__global__ void uni_composite(UniChunk c, UniOut o, int calc_normal, int white_bkgd);

}  // namespace nr
