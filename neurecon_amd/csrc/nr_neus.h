// neurecon_amd — NeuS render path internals.
#pragma once
#include "nr_common.h"

namespace nr {

constexpr int kMaxUp = 32;  // max new samples per upsampling round

// device views of one ray chunk's workspace (sample-major [s][r] arrays)
struct NeusChunk {
  int R;          // rays in this chunk
  int N_samples;  // coarse samples
  int n_up;       // new samples per round
  int n_iters;    // upsampling rounds
  int S;          // total samples = N_samples + n_iters * n_up
  float* ro; float* rd; float* near; float* far;
  float* dv; float* sv; float* wtmp; float* dnew; float* snew;
  float* pts; float* mids; float* dmid;
  float* sdf_f; float* nab_f;
  // official_solution: SDF + nablas computed when a sample is first evaluated.  nraw [S][R][3]
  // holds the nablas in evaluation order (coarse samples, then each round's new ones); the merges
  // carry each sample's evaluation slot in idv [S][R] (parallel to dv / sv), and neus_points
  // gathers the sorted nablas once.  idv == NULL: not fused.
  float* nraw; int* idv;
  // deferred sample nablas (official_solution, no detailed outputs): the sample launches leave each
  // 16-slot tile's slabs in `slabs` (sdf4_kernel STAGE 1); the tiles holding a sample whose interval
  // weight can be non-zero are flagged (tflag), listed (tiles / tcnt) and get their nablas in one
  // reverse-pass launch (STAGE 2); the rest of nraw stays 0 (those samples are weighted by exactly 0).
  // tshift 0: the flags are per sample slot, the list (neus_point_list) holds the flagged slots in
  // 16-aligned segments, and the reverse pass runs on the listed samples alone (STAGE 4, sdf4_kernel);
  // 4: flags and list per 16-slot tile (STAGE 2)
  float4* slabs; int* tflag; int* tiles; int* tcnt; int tshift;
  float* sdf_m; float* nab_m; float* feat_m; float* rad_m;
  // NeRF++ background (N_out = 0: none); M = S-1+N_out samples, sample-major
  int N_out;
  float r_obj;
  const float* t_out;
  float* d_out; float* x4; float* sig_o; float* rad_o;
  // direct_use / direct_more upsampling
  int n_imp;      // N_importance drawn in one sample_pdf
  int n_nog;      // N_nograd_samples (direct_more)
  float fixed_s;
  const float* t_nog;
  float* pts_nog; float* s_nog;
};

// outputs (ray-major); ray0 = index of the chunk's first ray in the full batch
struct NeusOut {
  int64_t ray0;
  float* rgb; float* depth; float* acc; float* normals;
  float* d_final; float* sdf; float* nablas; float* radiance; float* alpha; float* cdf; float* weights;
  float* sigma_out; float* radiance_bg;
};

struct NeusPlan {
  int64_t Rc;
  size_t o_ro, o_rd, o_near, o_far, o_dv, o_sv, o_wtmp, o_dnew, o_snew, o_pts, o_mids, o_dmid;
  size_t o_sdf_f, o_nab_f, o_sdf_m, o_nab_m, o_feat_m, o_rad_m, o_dout, o_x4, o_sigo, o_rado, o_ptsn, o_sn, o_mlp;
  size_t o_idv, o_nsort, o_dv2, o_sv2, o_idv2;
  size_t o_slot, o_x4c, o_vdc, o_sigc, o_radc, o_cnt;  // NeRF++: compacted background points
  size_t o_mslot, o_midc, o_mvd, o_mrad, o_mcnt;        // mid-points of non-zero alpha (compacted)
  size_t o_slabs, o_tflag, o_tiles, o_tcnt;             // deferred sample nablas
  size_t total;
};

NeusPlan neus_plan(const NrNeusArgs& a, int64_t Rc);
// the sample launches defer their reverse pass (see NeusChunk::slabs) for this chunk of R rays
bool neus_deferred(const NrNeusArgs& a, int64_t R);
int neus_total_samples(const NrNeusArgs& a);
__global__ void neus_sample_need(NeusChunk c, const float* s_dev, float s_val);
__global__ void neus_tile_list(NeusChunk c, int64_t n_tiles);
__global__ void neus_point_list(NeusChunk c, int64_t n_slots);
__global__ void neus_sample_need_outside(NeusChunk c, const float* s_dev, float s_val);
__global__ void neus_gather_nablas(NeusChunk c);

__global__ void neus_prologue(NeusChunk c, const float* rays_o, const float* rays_d, const float* t_coarse,
                              float r_obj, float near_bypass, float far_bypass);
template <int RPW>
__global__ void neus_upsample(NeusChunk c, int it, const float* u, int64_t u_stride);
__global__ void neus_merge(NeusChunk c, int L, float* dv2, float* sv2, int* idv2);
__global__ void neus_expand(NeusChunk c, int gather);
template <int RPW>
__global__ void neus_composite(NeusChunk c, NeusOut o, const float* s_dev, float s_val, int calc_normal, int white_bkgd);
__global__ void neus_outside_points(NeusChunk c, const float* t_rand);
__global__ void neus_outside_compact(NeusChunk c, int* count, int* slot, float* x4c, float* vdc);
__global__ void neus_mid_compact(NeusChunk c, const float* s_dev, float s_val, int* count, int* slot, float* midc,
                                 float* vdc);
__global__ void neus_mid_scatter(const int* slot, const float* radc, int64_t n, float* rad_m);
__global__ void neus_outside_scatter(const int* slot, const float* sigc, const float* radc, int64_t n, float* sig_o,
                                     float* rad_o);
__global__ void neus_nograd_points(NeusChunk c);
__global__ void neus_direct_upsample(NeusChunk c, int more, const float* u, int64_t u_stride);
__global__ void neus_composite_outside(NeusChunk c, NeusOut o, const float* s_dev, float s_val, int calc_normal,
                                       int white_bkgd);
template <int RPW>
__global__ void neus_composite_outside_w(NeusChunk c, NeusOut o, const float* s_dev, float s_val, int calc_normal,
                                         int white_bkgd);
__global__ void neus_write_dall(const float* dv, int64_t R, int S, int64_t ray0, float* out);
__global__ void sample_pdf_kernel(const float* bins, const float* weights, int64_t R, int L, const float* u,
                                  int64_t u_stride, int N, float* out);

}  // namespace nr
