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
  int no_secant;     // method != 'secant' (ray_casting.py:128-135): depth 1 on hits, no refinement
  float* ro; float* rd; float* near; float* far; float* thr;
  float* pts_m;      // [N_steps][R][3] march points
  float* sm;         // [N_steps][R] march sdf
  float* sec;        // [R][8]: d_lo, f_lo, d_hi, f_hi, d_pred, hit, crossing, first_free
  float* pts_s;      // [R][3] secant points
  float* ss;         // [R] secant sdf
  float* d_all;      // [P][R]
  float* pts_f;      // [P][R][3]
  float* sdf_f; float* nab_f; float* feat_f; float* nrm_f; float* rad_f;
  // F.normalize windows (normal_mode 1): window w of a batch row covers points q in
  // [j*netchunk, (j+1)*netchunk) of reference ray chunk k = w / nw_full (j = w % nw_full), q = ray-major
  // index (ray - k*rc_rays) * P + s inside that chunk.  The chunk's R rays are `rows` batch rows of
  // nloc rays each, starting at row-relative ray row_ray0 (a multi-GPU shard, or an internal chunk).
  double* wss;       // [rows][nw_row][3] sum of squares of the nablas per window
  double* wsp;       // [rows][nw_row][kWinSlices][3] partial sums (uni_window_ss_part)
  int64_t netchunk;  // points per F.normalize window
  int64_t rc_rays;   // the reference's rayschunk (clipped to the row)
  int64_t row_rays;  // rays per batch row of the whole (unsharded) batch
  int64_t row_ray0;  // row-relative index of this chunk's first ray
  int64_t nw_full;   // windows per full reference ray chunk
  int64_t nw_row;    // windows per batch row (row stride of wss)
  int nloc;          // rays per batch row in this chunk (R = rows * nloc)
  const float* t_march; const float* t_query; const float* t_free;
  // perturb (unisurf.py:158-165, :187-194): per-ray stratification uniforms of this chunk, rows of
  // N_query / N_free (null: deterministic linspace; else t_query / t_free hold N+1 bin edges)
  const float* u_q; const float* u_f;
};

struct UniOut {
  int64_t ray0;
  float* rgb; float* depth; float* acc; float* normals;
  float* surface_points; uint8_t* mask_surface; float* depth_surface;
  float* radiance; float* sdf; float* nablas; float* alpha; float* weights;
};

// The root-finding march evaluates its steps in chunks of kMarchK: a ray leaves the march at its first
// sign change (uni_root only reads up to there), so later chunks run on the device-compacted rays
// still without one.  Same values at every step uni_root reads: the maps are bit-identical.
constexpr int kMarchK = 32;
constexpr int kWinSlices = 64;  // blocks per F.normalize window in its sum of squares

struct UniPlan {
  int64_t Rc;
  size_t o_ro, o_rd, o_near, o_far, o_thr, o_ptsm, o_sm, o_sec, o_ptss, o_ss, o_dall, o_ptsf, o_sdff, o_nabf;
  size_t o_featf, o_nrmf, o_radf, o_wss, o_wsp, o_mlp;
  size_t o_act0, o_act1, o_acnt, o_ptsc, o_sc;  // chunked march: active lists, counts, compacted points / sdf
  size_t total;
  int64_t max_windows;
};

UniPlan unisurf_plan(const NrUnisurfArgs& a, int64_t Rc);
int64_t unisurf_chunk_rays(const NrUnisurfArgs& a);
// window geometry of one batch row of the whole batch: (rayschunk clipped, windows per full chunk,
// windows per row)
void unisurf_windows(const NrUnisurfArgs& a, int64_t& rc_rays, int64_t& nw_full, int64_t& nw_row);

__global__ void uni_prologue(UniChunk c, const float* rays_o, const float* rays_d);
__global__ void uni_root(UniChunk c);
__global__ void uni_march_scan(UniChunk c, int s0, int s1, const int* act_in, const int* n_in, int* act_out,
                               int* n_out);
__global__ void uni_march_gather(UniChunk c, int s0, int K, const int* act, const int* n, float* pts);
__global__ void uni_march_scatter(UniChunk c, int s0, int K, const int* act, const int* n, const float* v);
// The root-finding march of one chunk (ray_casting.py:88-101) into c.sm: steps [0, kMarchK) of every ray,
// then chunks of kMarchK steps over the rays still without a sign change (full: every step of every
// ray in one launch).  act0 / act1: [R] ints, cnt: 2 ints, ptsc: [kMarchK R, 3], sc: [kMarchK R] floats
// of workspace.  Used by UNISURF's render and by nr_root_find.
struct SdfLayout;
int run_march(const SdfLayout& SL, const void* packed, int multires, const UniChunk& c, bool full, int* act0,
              int* act1, int* cnt, float* ptsc, float* sc, hipStream_t st);
__global__ void rf_prologue(UniChunk c, const float* rays_o, const float* rays_d, float near, float far,
                            const float* near_rays, const float* far_rays);
__global__ void rf_finish(UniChunk c, int64_t ray0, float* d_out, float* pts, uint8_t* mask, uint8_t* msc,
                          int fill_inf);
__global__ void uni_secant(UniChunk c, int last);
__global__ void uni_samples(UniChunk c, UniOut o);
__global__ void uni_window_ss_part(UniChunk c);  // grid (nw_row, rows, kWinSlices), 256 threads
__global__ void uni_window_ss_sum(UniChunk c);   // grid (nw_row, rows), 64 threads
__global__ void uni_normalize(UniChunk c, int mode);
__global__ void uni_composite(UniChunk c, UniOut o, int calc_normal, int white_bkgd);

}  // namespace nr
