// neurecon_amd — C-ABI entry points (include/neurecon_hip.h): argument checking, packed-weight
// layouts, and the host-side orchestration of one NeuS ray chunk.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <string>

#include "nr_common.h"
#include <cstdlib>
#include "nr_mlp.h"
#include "nr_tgemm.h"
#include "nr_neus.h"
#include "nr_volsdf.h"
#include "nr_unisurf.h"

namespace nr {

static thread_local std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }

static size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }
static int64_t chunk_bytes_host(int KB) { return (int64_t)(2 * KB + 1) * 1024; }

// ---------------------------------------------------------------------------------------------
// descriptors
// ---------------------------------------------------------------------------------------------
int check_sdf_desc(const NrSdfDesc* d) {
  NR_REQUIRE(d, NR_ERR_ARG, "null NrSdfDesc");
  if (d->siren) {
    NR_REQUIRE(d->D == 5 && d->W == 256 && d->skip < 0 && d->multires < 0 && d->W_geo_feat == 256,
               NR_ERR_UNSUPPORTED,
               "SIREN SDF net: only D=5, W=256, skips=[], embed_multires=-1, W_geo_feat=256 (configs/volsdf_siren.yaml)");
    NR_REQUIRE(d->precision == NR_PREC_FP32 || d->precision == NR_PREC_F16X3, NR_ERR_UNSUPPORTED,
               "SDF net: unknown precision mode");
    return NR_OK;
  }
  NR_REQUIRE(d->D == 8 && d->W == 256 && d->skip == 4 && d->multires == 6 && d->W_geo_feat == 256,
             NR_ERR_UNSUPPORTED,
             "SDF net: only D=8, W=256, skips=[4], embed_multires=6, W_geo_feat=256 are implemented");
  NR_REQUIRE(d->precision == NR_PREC_FP32 || d->precision == NR_PREC_F16X3, NR_ERR_UNSUPPORTED,
             "SDF net: unknown precision mode");
  return NR_OK;
}

int check_rad_desc(const NrRadDesc* d) {
  NR_REQUIRE(d, NR_ERR_ARG, "null NrRadDesc");
  NR_REQUIRE((d->D == 4 || d->D == 5) && d->W == 256 && d->multires < 0 && d->W_geo_feat == 256 &&
                 d->multires_view <= 7,
             NR_ERR_UNSUPPORTED,
             "radiance net: only D=4 or 5, W=256, embed_multires=-1, embed_multires_view<=7, W_geo_feat=256");
  NR_REQUIRE(d->precision == NR_PREC_FP32 || d->precision == NR_PREC_F16X3, NR_ERR_UNSUPPORTED,
             "radiance net: unknown precision mode");
  return NR_OK;
}


SdfLayout sdf_layout(const NrSdfDesc& d) {
  SdfLayout L{};
  L.prec = d.precision;
  L.siren = d.siren ? 1 : 0;
  const int nops = L.siren ? kSirenOps : kSdfOps;
  const int* KB = L.siren ? kSirenKB : kSdfKB;
  const int* NBO = L.siren ? kSirenNBO : kSdfNBO;
  size_t off = 0;
  for (int i = 0; i < nops; ++i) {
    L.op_bytes[i] = (2 * KB[i] + 1) * 1024;
    L.op_off[i] = (uint32_t)off;
    off += (size_t)(NBO[i] / 2) * L.op_bytes[i];
  }
  static_assert(sdf_op_off(kSdfOps - 1) + (kSdfNBO[kSdfOps - 1] / 2) * (2 * kSdfKB[kSdfOps - 1] + 1) * 1024 > 0, "");
  L.scale_off = (uint32_t)off;
  off = align256(off + kSdfOps * 4);
  L.bound_off = (uint32_t)off;
  off = align256(off + kSdfOps * 8);
  L.w8row0_off = (uint32_t)off;
  off = align256(off + 256 * 4);
  L.misc_off = (uint32_t)off;
  off = align256(off + 16);
  if (g_sdf5_pack && L.prec == NR_PREC_F16X3 && !L.siren) {  // the ops again in the 32x32x16 layout (nr_sdf5.hip)
    L.l32_off = (uint32_t)off;
    off = align256(off + L.scale_off);
  }
  L.total = (uint32_t)off;
  return L;
}

// small input columns of layer 0 ahead of the feature: x, then (use_view_dirs) embed_view(v), normals
static int rad_small(const NrRadDesc& d) {
  return d.no_view_dirs ? 3 : 3 + (d.multires_view < 0 ? 3 : 3 + 6 * d.multires_view) + 3;
}

RadLayout rad_layout(const NrRadDesc& d) {
  RadLayout L{};
  L.prec = d.precision;
  L.n_small = rad_small(d);
  L.view = d.no_view_dirs ? 0 : 1;
  L.D = d.D;
  L.siren = d.siren ? 1 : 0;
  L.kbs = L.n_small <= 32 ? 2 : 4;
  size_t off = 0;
  for (int i = 0; i < L.D; ++i) {
    const int kb = i == 0 ? 16 + L.kbs : 16;
    L.op_bytes[i] = (2 * kb + 1) * 1024;
    L.op_off[i] = (uint32_t)off;
    off += 8 * (size_t)L.op_bytes[i];
  }
  L.scale_off = (uint32_t)off;
  off = align256(off + 5 * 4);
  L.bound_off = (uint32_t)off;
  off = align256(off + 5 * 2 * 4);
  L.head_off = (uint32_t)off;
  off = align256(off + (3 * 256 + 4) * 4);
  L.total = (uint32_t)off;
  return L;
}

int check_nerf_desc(const NrNerfDesc* d) {
  NR_REQUIRE(d, NR_ERR_ARG, "null NrNerfDesc");
  NR_REQUIRE(d->D == 8 && d->W == 256 && d->skip == 4 && d->input_ch == 4 && d->multires == 10 &&
                 d->multires_view == 4,
             NR_ERR_UNSUPPORTED,
             "NeRF net: only the NeRF++ background configuration (D=8, W=256, skips=[4], input_ch=4, "
             "multires=10, multires_view=4, use_view_dirs) is implemented");
  NR_REQUIRE(d->precision == NR_PREC_FP32 || d->precision == NR_PREC_F16X3, NR_ERR_UNSUPPORTED,
             "NeRF net: unknown precision mode");
  return NR_OK;
}

// (input blocks, output blocks) of each NeRF GEMM op: N0..N7, feature, views
static const int kNerfKB[kNerfOps] = {6, 16, 16, 16, 16, 22, 16, 16, 16, 18};
static const int kNerfNBO[kNerfOps] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 8};

// output blocks of NeRF op i: f16x3's NF also carries alpha_linear (blocks 16-17, row 0 = sigma)
static int nerf_nbo(int i, int prec) { return (i == NF && prec == NR_PREC_F16X3) ? 18 : kNerfNBO[i]; }

NerfLayout nerf_layout(const NrNerfDesc& d) {
  NerfLayout L{};
  L.prec = d.precision;
  size_t off = 0;
  for (int i = 0; i < kNerfOps; ++i) {
    L.op_bytes[i] = (2 * kNerfKB[i] + 1) * 1024;
    L.op_off[i] = (uint32_t)off;
    off += (size_t)(nerf_nbo(i, d.precision) / 2) * L.op_bytes[i];
  }
  L.scale_off = (uint32_t)off;
  off = align256(off + kNerfOps * 4);
  L.bound_off = (uint32_t)off;
  off = align256(off + kNerfOps * 2 * 4);
  L.alpha_off = (uint32_t)off;
  off = align256(off + 257 * 4);
  L.rgb_off = (uint32_t)off;
  off = align256(off + (3 * 128 + 3) * 4);
  L.total = (uint32_t)off;
  return L;
}

static PackSeg seg(int nblk, int off, int nvalid) { return PackSeg{nblk, off, nvalid}; }
static PackOp mkop(const float* W, const float* bias, int rows, int ld, int tr, PackSeg o0, PackSeg o1, PackSeg i0,
                   PackSeg i1, float scale, int prec, float* wmax) {
  PackOp op{};
  op.W = W; op.bias = bias; op.wn = (int64_t)rows * ld; op.ld = ld; op.transpose = tr;
  op.out[0] = o0; op.out[1] = o1; op.in[0] = i0; op.in[1] = i1;
  op.scale = scale; op.prec = prec; op.wmax = wmax;
  return op;
}
static PackSeg none() { return PackSeg{0, 0, 0}; }

static size_t scratch_bytes() {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  return (size_t)cus * kScratchPerWG;
}

// ---------------------------------------------------------------------------------------------
// NeuS chunk orchestration
// ---------------------------------------------------------------------------------------------
static int neus_chunk(const NrNeusArgs& a, const NeusPlan& pl, int64_t ray0, int R, hipStream_t st) {
  char* ws = (char*)a.workspace;
  const bool direct = a.upsample_algo != NR_UPSAMPLE_OFFICIAL;
  const int n_up = direct ? 0 : (a.N_upsample_iters > 0 ? a.N_importance / a.N_upsample_iters : 0);
  NeusChunk c{};
  c.R = R;
  c.N_samples = a.N_samples;
  c.n_up = n_up;
  c.n_iters = direct ? 0 : a.N_upsample_iters;
  c.S = direct ? a.N_samples + a.N_importance : a.N_samples + a.N_upsample_iters * n_up;
  c.n_imp = a.N_importance;
  c.n_nog = a.upsample_algo == NR_UPSAMPLE_DIRECT_MORE ? a.N_nograd_samples : 0;
  c.fixed_s = a.fixed_s;
  c.t_nog = a.t_nograd;
  auto F = [&](size_t o) { return (float*)(ws + o); };
  c.ro = F(pl.o_ro); c.rd = F(pl.o_rd); c.near = F(pl.o_near); c.far = F(pl.o_far);
  c.dv = F(pl.o_dv); c.sv = F(pl.o_sv); c.wtmp = F(pl.o_wtmp); c.dnew = F(pl.o_dnew); c.snew = F(pl.o_snew);
  c.pts = F(pl.o_pts); c.mids = F(pl.o_mids); c.dmid = F(pl.o_dmid);
  c.sdf_f = F(pl.o_sdf_f); c.nab_f = F(pl.o_nab_f);
  c.sdf_m = F(pl.o_sdf_m); c.nab_m = F(pl.o_nab_m); c.feat_m = F(pl.o_feat_m); c.rad_m = F(pl.o_rad_m);
  c.N_out = a.N_outside;
  c.r_obj = a.obj_bounding_radius;
  c.t_out = a.t_outside;
  c.d_out = F(pl.o_dout); c.x4 = F(pl.o_x4); c.sig_o = F(pl.o_sigo); c.rad_o = F(pl.o_rado);
  c.pts_nog = F(pl.o_ptsn); c.s_nog = F(pl.o_sn);
  // official_solution evaluates every final sample exactly once, when it is drawn: the coarse and
  // upsampled points are bit-identical to the final `pts` (neus.py:284 recomputes o + d*dir from
  // the same depths), so one SDF+nabla launch per round replaces the forward-only round launches
  // plus the reference's second pass over all samples (neus.py:294).  sdf rides along the sorted
  // merges (sv); nablas stay in evaluation order (nraw) and are gathered once by neus_points.
  const bool fused = !direct && !a.sample_only;  // the sample pass needs no nablas
  c.nraw = fused ? c.nab_f : nullptr;
  c.idv = fused ? (int*)(ws + pl.o_idv) : nullptr;
  if (fused) {
    c.sdf_f = c.sv;
    c.nab_f = F(pl.o_nsort);
  }
  // deferred sample nablas (NeusChunk::slabs): sample launches leave per-tile slabs, the reverse pass
  // runs after the sampling on the tiles of non-zero weight
  const bool defer = fused && neus_deferred(a, R);
  if (defer) {
    c.slabs = (float4*)(ws + pl.o_slabs);
    c.tflag = (int*)(ws + pl.o_tflag);
    c.tiles = (int*)(ws + pl.o_tiles);
    c.tcnt = (int*)(ws + pl.o_tcnt);
  }
  void* mlp_ws = ws + pl.o_mlp;
  const size_t mlp_bytes = a.workspace_bytes - pl.o_mlp;
  const SdfLayout SL = sdf_layout(*a.sdf);
  const RadLayout RL = rad_layout(*a.rad);
  // SDF of P sample points at evaluation slot slot0 (coarse: 0; round it: (N_samples + it n_up) R)
  auto sample_sdf = [&](const float* pts, int64_t P, float* sdf_out, int64_t slot0) -> int {
    if (defer)
      return launch_sdf_deferred(SL, a.sdf_packed, pts, P, sdf_out, nullptr, a.sdf->multires,
                                 (float4*)((char*)c.slabs + (size_t)(slot0 / 16) * kSlabColBytes), nullptr, nullptr,
                                 1, st);
    return launch_sdf(SL, a.sdf_packed, pts, P, sdf_out, fused ? c.nraw + slot0 * 3 : nullptr, nullptr,
                      a.sdf->multires, fused ? mlp_ws : nullptr, fused ? mlp_bytes : 0, st);
  };
  const dim3 blk(64), grd((R + 63) / 64);  // one wave per block: a 4096-ray chunk spreads over 64 CUs
  int rc;

  {
  ProfScope prof("neus_prologue", (double)R, st);
  hipLaunchKernelGGL(neus_prologue, grd, blk, 0, st, c, a.rays_o + ray0 * 3, a.rays_d + ray0 * 3, a.t_coarse,
                     a.obj_bounding_radius, a.near_bypass, a.far_bypass);
  }
  NR_HIP_CHECK(hipGetLastError());
  // coarse SDF (no grad, neus.py:220 / :251); direct_more uses its own uniform depths instead
  if (a.upsample_algo != NR_UPSAMPLE_DIRECT_MORE && (rc = sample_sdf(c.pts, (int64_t)a.N_samples * R, c.sv, 0)))
    return rc;
  if (a.upsample_algo == NR_UPSAMPLE_DIRECT_MORE) {  // SDF at N_nograd_samples uniform depths
    hipLaunchKernelGGL(neus_nograd_points, grd, blk, 0, st, c);
    NR_HIP_CHECK(hipGetLastError());
    if ((rc = launch_sdf(SL, a.sdf_packed, c.pts_nog, (int64_t)c.n_nog * R, c.s_nog, nullptr, nullptr,
                         a.sdf->multires, nullptr, 0, st)))
      return rc;
  }
  if (direct) {
    ProfScope prof("neus_upsample", (double)R, st);
    // perturb: this chunk's rows of the caller's [n_rays][N_importance] uniforms
    const float* u = a.u_rand ? a.u_rand + ray0 * a.N_importance : a.u_fine;
    hipLaunchKernelGGL(neus_direct_upsample, grd, blk, 0, st, c, (int)(a.upsample_algo == NR_UPSAMPLE_DIRECT_MORE), u,
                       (int64_t)(a.u_rand ? a.N_importance : 0));
  }
  NR_HIP_CHECK(hipGetLastError());
  // sorted sample lists ping-pong between two buffers; each merge writes the other one
  float* dvb[2] = {c.dv, F(pl.o_dv2)};
  float* svb[2] = {c.sv, F(pl.o_sv2)};
  int* idb[2] = {c.idv, fused ? (int*)(ws + pl.o_idv2) : nullptr};
  int cur = 0;
  auto merge = [&](int L) -> int {
    ProfScope prof("neus_merge", (double)R, st);
    const int64_t nt = (int64_t)(L + n_up) * R;
    hipLaunchKernelGGL(neus_merge, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, st, c, L, dvb[cur ^ 1],
                       svb[cur ^ 1], idb[cur ^ 1]);
    cur ^= 1;
    c.dv = dvb[cur];
    c.sv = svb[cur];
    c.idv = idb[cur];
    if (fused) c.sdf_f = c.sv;
    NR_HIP_CHECK(hipGetLastError());
    return NR_OK;
  };
  for (int it = 0; it < c.n_iters; ++it) {
    if (it > 0 && (rc = merge(a.N_samples + (it - 1) * n_up))) return rc;
    const int64_t slot0 = (int64_t)(a.N_samples + it * n_up) * R;
    // deferred: every round's points stay at their evaluation slots (the reverse pass reads them)
    NeusChunk cu = c;
    if (defer) cu.pts = c.pts + slot0 * 3;
    {
      ProfScope prof("neus_upsample", (double)R, st);
      // perturb: round it's [n_rays][n_up] block of the caller's uniforms
      const float* u = a.u_rand ? a.u_rand + ((int64_t)it * a.n_rays + ray0) * n_up : a.u_fine;
      const size_t lds1 = (5 * (size_t)c.S + 1) * sizeof(float);  // four rays per wave when their staging fits
      if (4 * lds1 <= 65536)
        hipLaunchKernelGGL((neus_upsample<4>), dim3((unsigned)((R + 3) / 4)), dim3(64), 4 * lds1, st, cu, it, u,
                           (int64_t)(a.u_rand ? n_up : 0));
      else
        hipLaunchKernelGGL((neus_upsample<1>), dim3((unsigned)R), dim3(64), lds1, st, cu, it, u,
                           (int64_t)(a.u_rand ? n_up : 0));
    }
    NR_HIP_CHECK(hipGetLastError());
    if ((rc = sample_sdf(cu.pts, (int64_t)n_up * R, c.snew, slot0))) return rc;
  }
  if (c.n_iters > 0 && (rc = merge(c.S - n_up))) return rc;
  if (defer) {  // nablas of the tiles holding a sample of non-zero interval weight; the rest stay 0
    const int64_t nslot = (int64_t)c.S * R;
    c.tshift = 0;  // flags per sample slot, the reverse pass on the listed samples (sdf4_kernel STAGE 4)
    NR_HIP_CHECK(hipMemsetAsync(c.nraw, 0, (size_t)nslot * 3 * sizeof(float), st));
    if (a.calc_normal && a.N_outside == 0) {  // normals_volume is the only reader of the sample nablas here
      // (with NeRF++ the flags need the background's alphas: after the background net, below)
      NR_HIP_CHECK(hipMemsetAsync(c.tflag, 0, (size_t)nslot * sizeof(int), st));
      NR_HIP_CHECK(hipMemsetAsync(c.tcnt, 0, sizeof(int), st));
      const int64_t nq = (int64_t)(c.S - 1) * R;
      hipLaunchKernelGGL(neus_sample_need, dim3((unsigned)((nq + 255) / 256)), dim3(256), 0, st, c, a.s_dev, a.s);
      NR_HIP_CHECK(hipGetLastError());
      hipLaunchKernelGGL(neus_point_list, dim3((unsigned)((nslot + 1023) / 1024)), dim3(1024), 0, st, c, nslot);
      NR_HIP_CHECK(hipGetLastError());
      if ((rc = launch_sdf_deferred(SL, a.sdf_packed, c.pts, nslot, nullptr, c.nraw, a.sdf->multires, c.slabs, c.tiles,
                                    c.tcnt, 4, st)))
        return rc;
    }
  }
  if (a.sample_only) {  // training: the sorted depths are the whole output (neus.py:279)
    hipLaunchKernelGGL(neus_write_dall, dim3((unsigned)(((int64_t)c.S * R + 255) / 256)), dim3(256), 0, st, c.dv,
                       (int64_t)R, c.S, ray0, a.d_all_out);
    NR_HIP_CHECK(hipGetLastError());
    return NR_OK;
  }
  {
    ProfScope prof("neus_points", (double)R, st);
    hipLaunchKernelGGL(neus_expand, dim3((unsigned)(((int64_t)c.S * R + 255) / 256)), dim3(256), 0, st, c,
                       (int)!(defer && a.N_outside > 0));
  }
  NR_HIP_CHECK(hipGetLastError());
  // SDF + nablas at the samples (neus.py:294); already in sv / nv on the fused path
  if (!fused && (rc = launch_sdf(SL, a.sdf_packed, c.pts, (int64_t)c.S * R, c.sdf_f, c.nab_f, nullptr,
                                 a.sdf->multires, mlp_ws, mlp_bytes, st)))
    return rc;
  // SDF + nablas + geometry feature at the mid-points, then the radiance net (neus.py:103-106, :298)
  const int64_t Pm = (int64_t)(c.S - 1) * R;
  if (a.radiance_out || a.no_mid_skip) {  // every mid-point, as the reference
    if ((rc = launch_sdf(SL, a.sdf_packed, c.mids, Pm, c.sdf_m, c.nab_m, c.feat_m, a.sdf->multires, mlp_ws, mlp_bytes,
                         st)))
      return rc;
    if ((rc = launch_radiance(RL, a.rad_packed, c.mids, c.rd, 1, R, c.nab_m, c.feat_m, Pm, c.rad_m,
                              a.rad->multires_view, st)))
      return rc;
  } else {  // only the mid-points whose alpha is not exactly 0 (neus_mid_compact); bit-identical maps
    char* wsb = (char*)a.workspace;
    int* cnt = (int*)(wsb + pl.o_mcnt);
    int* slot = (int*)(wsb + pl.o_mslot);
    float* midc = (float*)(wsb + pl.o_midc);
    float* vdc = (float*)(wsb + pl.o_mvd);
    float* radc = (float*)(wsb + pl.o_mrad);
    NR_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int), st));
    const dim3 g1((unsigned)((Pm + 255) / 256));
    hipLaunchKernelGGL(neus_mid_compact, dim3((unsigned)((Pm + 1023) / 1024)), dim3(1024), 0, st, c, a.s_dev, a.s, cnt,
                       slot, midc, vdc);
    NR_HIP_CHECK(hipGetLastError());
    if ((rc = launch_sdf(SL, a.sdf_packed, midc, Pm, c.sdf_m, c.nab_m, c.feat_m, a.sdf->multires, mlp_ws, mlp_bytes,
                         st, cnt, 1)))
      return rc;
    if ((rc = launch_radiance(RL, a.rad_packed, midc, vdc, 1, INT64_MAX, c.nab_m, c.feat_m, Pm, radc,
                              a.rad->multires_view, st, cnt)))
      return rc;
    hipLaunchKernelGGL(neus_mid_scatter, g1, dim3(256), 0, st, slot, radc, Pm, c.rad_m);
    NR_HIP_CHECK(hipGetLastError());
  }
  NeusOut o{ray0, a.rgb, a.depth, a.acc, a.normals, a.d_final, a.sdf_out, a.nablas_out,
            a.radiance_out, a.alpha_out, a.cdf_out, a.weights_out, a.sigma_out, a.radiance_bg_out};
  if (a.N_outside > 0) {  // NeRF++ background on [mid-points ; inverted-sphere samples]
    hipLaunchKernelGGL(neus_outside_points, grd, blk, 0, st, c,
                       a.t_out_rand ? a.t_out_rand + ray0 * a.N_outside : (const float*)nullptr);
    NR_HIP_CHECK(hipGetLastError());
    const int64_t Po = (int64_t)(c.S - 1 + a.N_outside) * R;
    if (a.sigma_out || a.radiance_bg_out) {  // detailed outputs: the background at every sample, as the reference
      if ((rc = launch_nerf(nerf_layout(*a.nerf), a.nerf_packed, c.x4, c.rd, 1, R, Po, c.sig_o, c.rad_o, st)))
        return rc;
    } else {  // only the background values the compositing reads (neus_outside_compact)
      char* wsb = (char*)a.workspace;
      int* cnt = (int*)(wsb + pl.o_cnt);
      int* slot = (int*)(wsb + pl.o_slot);
      float* x4c = (float*)(wsb + pl.o_x4c);
      float* vdc = (float*)(wsb + pl.o_vdc);
      float* sigc = (float*)(wsb + pl.o_sigc);
      float* radc = (float*)(wsb + pl.o_radc);
      NR_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int), st));
      const dim3 g1((unsigned)((Po + 255) / 256));
      hipLaunchKernelGGL(neus_outside_compact, dim3((unsigned)((Po + 1023) / 1024)), dim3(1024), 0, st, c, cnt, slot,
                         x4c, vdc);
      NR_HIP_CHECK(hipGetLastError());
      if ((rc = launch_nerf(nerf_layout(*a.nerf), a.nerf_packed, x4c, vdc, 1, INT64_MAX, Po, sigc, radc, st, cnt)))
        return rc;
      hipLaunchKernelGGL(neus_outside_scatter, g1, dim3(256), 0, st, slot, sigc, radc, Po, c.sig_o, c.rad_o);
      NR_HIP_CHECK(hipGetLastError());
    }
    if (defer) {  // deferred sample nablas: samples (or tiles) whose (inside or background) alpha != 0
      const int64_t nslot = (int64_t)c.S * R;
      c.tshift = 0;
      if (a.calc_normal) {
        NR_HIP_CHECK(hipMemsetAsync(c.tflag, 0, (size_t)nslot * sizeof(int), st));
        NR_HIP_CHECK(hipMemsetAsync(c.tcnt, 0, sizeof(int), st));
        hipLaunchKernelGGL(neus_sample_need_outside, dim3((unsigned)((nslot + 255) / 256)), dim3(256), 0, st, c,
                           a.s_dev, a.s);
        NR_HIP_CHECK(hipGetLastError());
        hipLaunchKernelGGL(neus_point_list, dim3((unsigned)((nslot + 1023) / 1024)), dim3(1024), 0, st, c, nslot);
        NR_HIP_CHECK(hipGetLastError());
        if ((rc = launch_sdf_deferred(SL, a.sdf_packed, c.pts, nslot, nullptr, c.nraw, a.sdf->multires, c.slabs,
                                      c.tiles, c.tcnt, 4, st)))
          return rc;
      }
      hipLaunchKernelGGL(neus_gather_nablas, dim3((unsigned)((nslot + 255) / 256)), dim3(256), 0, st, c);
      NR_HIP_CHECK(hipGetLastError());
    }
    ProfScope prof("neus_composite", (double)R, st);
    const int M = c.S - 1 + a.N_outside;
    const size_t lds1 = (6 * (size_t)M + 4 * (size_t)c.S) * sizeof(float);  // wave-per-ray staging of one ray
    if (4 * lds1 <= 65536)
      hipLaunchKernelGGL((neus_composite_outside_w<4>), dim3((unsigned)((R + 3) / 4)), dim3(64), 4 * lds1, st, c, o,
                         a.s_dev, a.s, a.calc_normal, a.white_bkgd);
    else if (lds1 <= 65536)
      hipLaunchKernelGGL((neus_composite_outside_w<1>), dim3((unsigned)R), dim3(64), lds1, st, c, o, a.s_dev, a.s,
                         a.calc_normal, a.white_bkgd);
    else
      hipLaunchKernelGGL(neus_composite_outside, grd, blk, 0, st, c, o, a.s_dev, a.s, a.calc_normal, a.white_bkgd);
  } else {
    ProfScope prof("neus_composite", (double)R, st);
    const size_t lds1 = 9 * (size_t)c.S * sizeof(float);  // four rays per wave when four rays' staging fits
    if (4 * lds1 <= 65536)  // the dynamic-LDS limit per workgroup (nr_neus_render checks lds1 against it)
      hipLaunchKernelGGL((neus_composite<4>), dim3((unsigned)((R + 3) / 4)), dim3(64), 4 * lds1, st, c, o, a.s_dev, a.s,
                         a.calc_normal, a.white_bkgd);
    else
      hipLaunchKernelGGL((neus_composite<1>), dim3((unsigned)R), dim3(64), lds1, st, c, o, a.s_dev, a.s, a.calc_normal,
                         a.white_bkgd);
  }
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

// rays per chunk: at most 16384, the caller's max_chunk_rays (its rayschunk) -- with no explicit
// workspace budget a hint floored at NR_MIN_CHUNK_RAYS (the reference's validation rayschunk of 256
// would leave the per-ray kernels a few CUs; memory is bounded by the default budget), exact when the
// caller also set max_workspace_bytes -- and as many as keep the workspace within
// max_workspace_bytes (the plan is affine in the chunk's ray count); deferred chunks (8 KB of slabs
// per sample) are a multiple of 16 rays, so that every launch starts a tile
static int64_t neus_chunk_rays(const NrNeusArgs* a) {
  const int64_t n = a->n_rays > 0 ? a->n_rays : 1;
  int64_t cap = 16384;
  // the floor applies to a caller that left the memory bound to the library (max_workspace_bytes 0); one
  // that set a workspace budget gets its max_chunk_rays exactly, as the reference's rayschunk loop
  if (a->max_chunk_rays > 0)
    cap = std::min(cap, a->max_workspace_bytes ? a->max_chunk_rays : std::max<int64_t>(a->max_chunk_rays, NR_MIN_CHUNK_RAYS));
  const size_t budget = a->max_workspace_bytes ? a->max_workspace_bytes : NR_DEFAULT_WORKSPACE_BYTES;
  const bool defer = neus_deferred(*a, 16);
  NrNeusArgs q = *a;  // plan sizes with deferral decided as for a 16-ray-multiple chunk
  const size_t t1 = neus_plan(q, 1024).total, t2 = neus_plan(q, 2048).total;
  const size_t per_ray = (t2 - t1) / 1024 + 1, fixed = t1 > 1024 * per_ray ? t1 - 1024 * per_ray : 0;
  const int64_t fit = budget > fixed ? (int64_t)((budget - fixed) / per_ray) : 0;
  cap = std::min(cap, std::max<int64_t>(fit, 16));
  // deferred chunks tile exactly: a ray count that is not a multiple of 16 renders as 16-multiple
  // chunks (deferred) plus a < 16-ray tail (nablas when drawn)
  if (defer && n > 16 && n % 16) cap = std::min(cap, n / 16 * 16);
  if (n <= cap) return n;
  if (defer && cap >= 16) cap = cap / 16 * 16;
  return std::max<int64_t>(cap, 1);
}

// ---------------------------------------------------------------------------------------------
// VolSDF chunk orchestration (volsdf.py:394-551): prologue -> SDF(4 N_samples) -> first check ->
// [SDF(active x N_up, device count) -> round it] x max_iter -> points -> SDF+nablas+feature ->
// radiance -> composite.  No host synchronisation inside a chunk.
// ---------------------------------------------------------------------------------------------
static int volsdf_chunk(const NrVolsdfArgs& a, const VolPlan& pl, int64_t ray0, int R, hipStream_t st) {
  char* ws = (char*)a.workspace;
  auto F = [&](size_t o) { return (float*)(ws + o); };
  VolChunk c{};
  c.R = R;
  c.N0 = 4 * a.N_samples;
  c.N_up = 4 * a.N_samples;
  c.cap = c.N0 + a.max_upsample_steps * c.N_up;
  c.N_samples = a.N_samples;
  c.N_imp = a.N_importance;
  c.S = a.N_samples + a.N_importance;
  c.max_iter = a.max_upsample_steps;
  c.max_bisect = a.max_bisection_steps;
  c.alpha_net = a.alpha_net;
  c.beta_net = a.beta_net;
  c.beta_plus0 = a.beta_plus_init;
  c.eps = a.eps;
  c.near = a.near;
  c.far = a.far;
  c.r_bg = a.obj_bounding_radius;
  c.use_bg = a.use_sphere_bg;
  c.ro = F(pl.o_ro); c.rd = F(pl.o_rd);
  c.Ld[0] = F(pl.o_Ld0); c.Ld[1] = F(pl.o_Ld1); c.Ls[0] = F(pl.o_Ls0); c.Ls[1] = F(pl.o_Ls1);
  c.dnew[0] = F(pl.o_dn0); c.dnew[1] = F(pl.o_dn1);
  c.pts = F(pl.o_pts); c.sraw = F(pl.o_sraw);
  c.act[0] = (int*)(ws + pl.o_act0); c.act[1] = (int*)(ws + pl.o_act1); c.cnt = (int*)(ws + pl.o_cnt);
  c.beta = F(pl.o_beta); c.fine = F(pl.o_fine); c.usage = F(pl.o_usage); c.bmap = F(pl.o_bmap);
  c.d_all = F(pl.o_dall); c.pts_f = F(pl.o_ptsf); c.sdf_f = F(pl.o_sdff); c.nab_f = F(pl.o_nabf);
  c.feat_f = F(pl.o_featf); c.rad_f = F(pl.o_radf);
  c.t_coarse = a.t_coarse; c.t_init = a.t_init; c.u_up = a.u_up; c.u_fine = a.u_fine;
  c.N_out = a.N_outside > 0 ? a.N_outside : 0;
  c.u_rand = a.u_rand ? a.u_rand + ray0 * a.N_importance : nullptr;
  c.u_out = a.u_out && c.N_out > 0 ? a.u_out + ray0 * c.N_out : nullptr;
  c.beta_k = a.beta_plus_k;
  c.farr = F(pl.o_farr); c.bp0 = F(pl.o_bp0); c.rs_out = a.rs_out; c.d_out = F(pl.o_dout);
  c.x4 = F(pl.o_x4); c.sig_o = F(pl.o_sigo); c.rad_o = F(pl.o_rado);
  void* mlp_ws = ws + pl.o_mlp;
  const size_t mlp_bytes = a.workspace_bytes - pl.o_mlp;
  const SdfLayout SL = sdf_layout(*a.sdf);
  const RadLayout RL = rad_layout(*a.rad);
  const unsigned lds = (unsigned)pl.lds_bytes;
  const dim3 blk(64), grd((unsigned)R);
  int rc;
  NR_HIP_CHECK(hipMemsetAsync(c.cnt, 0, sizeof(int) * (a.max_upsample_steps + 1), st));
  {
    ProfScope prof("volsdf_prologue", (double)R, st);
    hipLaunchKernelGGL(volsdf_prologue, grd, blk, 0, st, c, a.rays_o + ray0 * 3, a.rays_d + ray0 * 3);
  }
  NR_HIP_CHECK(hipGetLastError());
  if ((rc = launch_sdf(SL, a.sdf_packed, c.pts, (int64_t)c.N0 * R, c.sraw, nullptr, nullptr, a.sdf->multires,
                       nullptr, 0, st)))
    return rc;
  {
    ProfScope prof("volsdf_first", (double)R, st);
    hipLaunchKernelGGL(volsdf_first, grd, blk, lds, st, c);
  }
  NR_HIP_CHECK(hipGetLastError());
  for (int it = 1; it <= a.max_upsample_steps; ++it) {
    if ((rc = launch_sdf(SL, a.sdf_packed, c.pts, (int64_t)c.N_up * R, c.sraw, nullptr, nullptr, a.sdf->multires,
                         nullptr, 0, st, c.cnt + (it - 1), c.N_up)))
      return rc;
    {
      ProfScope prof("volsdf_iter", (double)R, st);
      hipLaunchKernelGGL(volsdf_iter, grd, blk, lds, st, c, it);
    }
    NR_HIP_CHECK(hipGetLastError());
  }
  {
    ProfScope prof("volsdf_points", (double)R, st);
    hipLaunchKernelGGL(volsdf_points, grd, blk, lds, st, c);
  }
  NR_HIP_CHECK(hipGetLastError());
  const int64_t P = (int64_t)c.S * R;
  if ((rc = launch_sdf(SL, a.sdf_packed, c.pts_f, P, c.sdf_f, c.nab_f, c.feat_f, a.sdf->multires, mlp_ws, mlp_bytes,
                       st)))
    return rc;
  if ((rc = launch_radiance(RL, a.rad_packed, c.pts_f, c.rd, c.S, INT64_MAX, c.nab_f, c.feat_f, P, c.rad_f,
                            a.rad->multires_view, st)))
    return rc;
  if (c.N_out > 0) {
    {
      ProfScope prof("volsdf_outside", (double)R, st);
      hipLaunchKernelGGL(volsdf_outside, grd, blk, 0, st, c);
    }
    NR_HIP_CHECK(hipGetLastError());
    if ((rc = launch_nerf(nerf_layout(*a.nerf), a.nerf_packed, c.x4, c.rd, c.N_out, INT64_MAX,
                          (int64_t)c.N_out * R, c.sig_o, c.rad_o, st)))
      return rc;
  }
  VolOut o{ray0, a.rgb, a.depth, a.acc, a.normals, a.d_vals, a.sdf_out, a.nablas_out, a.radiance_out,
           a.alpha_out, a.p_out, a.weights_out, a.sigma_out, a.beta_map, a.iter_usage, a.sigma_bg, a.radiance_bg};
  {
    ProfScope prof("volsdf_composite", (double)R, st);
    hipLaunchKernelGGL(volsdf_composite, grd, blk, lds, st, c, o, a.calc_normal, a.white_bkgd);
  }
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

static int64_t volsdf_chunk_rays(const NrVolsdfArgs* a) {
  const int64_t cap = 16384;
  return a->n_rays < cap ? (a->n_rays > 0 ? a->n_rays : 1) : cap;
}

static int check_volsdf(const NrVolsdfArgs* a) {
  NR_REQUIRE(a, NR_ERR_ARG, "nr_volsdf_render: null args");
  int rc = check_sdf_desc(a->sdf);
  if (rc) return rc;
  if ((rc = check_rad_desc(a->rad))) return rc;
  // an empty shard (multi-GPU ray sharding) may pass null ray / output pointers
  NR_REQUIRE(a->n_rays <= 0 || (a->rays_o && a->rays_d && a->rgb && a->depth && a->acc), NR_ERR_ARG,
             "nr_volsdf_render: null ray or output pointer");
  NR_REQUIRE(a->sdf_packed && a->rad_packed && a->t_coarse && a->t_init && a->u_up && a->u_fine, NR_ERR_ARG,
             "nr_volsdf_render: null argument");
  NR_REQUIRE(a->n_rays <= 0 || !a->calc_normal || a->normals, NR_ERR_ARG,
             "nr_volsdf_render: calc_normal needs normals output");
  NR_REQUIRE(a->N_samples >= 1 && a->N_importance >= 1 && a->max_upsample_steps >= 0 && a->max_bisection_steps >= 0,
             NR_ERR_ARG, "nr_volsdf_render: bad sample counts");
  NR_REQUIRE(4 * a->N_samples <= 1024 && a->N_importance <= 1024, NR_ERR_UNSUPPORTED,
             "nr_volsdf_render: 4*N_samples and N_importance must be <= 1024");
  NR_REQUIRE(a->beta_net > 0.f && (a->N_outside > 0 || a->beta_plus_init > 0.f), NR_ERR_ARG,
             "nr_volsdf_render: beta must be positive");
  if (a->N_outside > 0) {
    NR_REQUIRE(!a->use_sphere_bg, NR_ERR_ARG, "nr_volsdf_render: NeRF++ background excludes the builtin sphere");
    NR_REQUIRE(a->nerf && a->nerf_packed && a->rs_out && a->beta_plus_k > 0.f, NR_ERR_ARG,
               "nr_volsdf_render: N_outside > 0 needs nerf, nerf_packed, rs_out and beta_plus_k");
    if ((rc = check_nerf_desc(a->nerf))) return rc;
  }
  return NR_OK;
}

// ---------------------------------------------------------------------------------------------
// UNISURF chunk orchestration (unisurf.py:118-244): prologue -> SDF(march) -> root -> [SDF(secant
// point) -> secant] x N_secant_steps -> samples -> SDF+nablas+feature -> F.normalize -> radiance
// -> composite.
// ---------------------------------------------------------------------------------------------
// rays [ray0, ray0 + R) of the call = `R / nloc` batch rows of nloc rays, starting at row-relative
// ray row_ray0 (internal chunks: one row; a multi-GPU shard: all of its rows in one chunk)
static int unisurf_chunk(const NrUnisurfArgs& a, const UniPlan& pl, int64_t ray0, int R, int64_t row_ray0, int nloc,
                         hipStream_t st) {
  char* ws = (char*)a.workspace;
  auto F = [&](size_t o) { return (float*)(ws + o); };
  UniChunk c{};
  c.R = R;
  c.N_steps = a.N_steps;
  c.N_query = a.N_query;
  c.N_free = a.N_freespace;
  c.P = a.N_query + a.N_freespace;
  c.logit_tau = a.logit_tau;
  c.interval = a.interval;
  c.too_close = a.too_close_threshold;
  c.near_bypass = a.near_bypass;
  c.far_bypass = a.far_bypass;
  c.r_interest = a.radius_of_interest;
  c.ro = F(pl.o_ro); c.rd = F(pl.o_rd); c.near = F(pl.o_near); c.far = F(pl.o_far); c.thr = F(pl.o_thr);
  c.pts_m = F(pl.o_ptsm); c.sm = F(pl.o_sm); c.sec = F(pl.o_sec); c.pts_s = F(pl.o_ptss); c.ss = F(pl.o_ss);
  c.d_all = F(pl.o_dall); c.pts_f = F(pl.o_ptsf); c.sdf_f = F(pl.o_sdff); c.nab_f = F(pl.o_nabf);
  c.feat_f = F(pl.o_featf); c.nrm_f = F(pl.o_nrmf); c.rad_f = F(pl.o_radf); c.wss = (double*)(ws + pl.o_wss);
  c.wsp = (double*)(ws + pl.o_wsp);
  c.netchunk = a.netchunk;
  const bool sharded = a.normal_mode == 1 && a.shard_row_rays > 0;
  if (a.normal_mode == 1) {
    unisurf_windows(a, c.rc_rays, c.nw_full, c.nw_row);
    c.row_rays = sharded ? a.shard_row_rays : (a.rays_per_batch > 0 ? a.rays_per_batch : a.n_rays);
    c.row_ray0 = row_ray0;
    c.nloc = nloc;
    if (sharded) c.wss = a.window_ss;  // the caller's [B][nw_row][3], all-reduced by window_reduce
  }
  c.t_march = a.t_march; c.t_query = a.t_query; c.t_free = a.t_free;
  c.no_secant = a.no_secant;
  c.u_q = a.u_query ? a.u_query + ray0 * a.N_query : nullptr;
  c.u_f = a.u_free ? a.u_free + ray0 * a.N_freespace : nullptr;
  void* mlp_ws = ws + pl.o_mlp;
  const size_t mlp_bytes = a.workspace_bytes - pl.o_mlp;
  const SdfLayout SL = sdf_layout(*a.sdf);
  const RadLayout RL = rad_layout(*a.rad);
  const dim3 blk(64), grd((R + 63) / 64);  // one wave per block: a 4096-ray chunk spreads over 64 CUs
  const int64_t P = (int64_t)c.P * R;
  int rc;
  {
    ProfScope prof("unisurf_prologue", (double)R, st);
    hipLaunchKernelGGL(uni_prologue, grd, blk, 0, st, c, a.rays_o + ray0 * 3, a.rays_d + ray0 * 3);
  }
  NR_HIP_CHECK(hipGetLastError());
  // the march (ray_casting.py:88-101) in chunks of kMarchK steps over the rays still without a crossing
  // (full_march: every step of every ray in one launch, the bit-identity test's reference)
  if ((rc = run_march(SL, a.sdf_packed, a.sdf->multires, c, a.full_march != 0, (int*)(ws + pl.o_act0),
                      (int*)(ws + pl.o_act1), (int*)(ws + pl.o_acnt), F(pl.o_ptsc), F(pl.o_sc), st)))
    return rc;
  hipLaunchKernelGGL(uni_root, grd, blk, 0, st, c);
  NR_HIP_CHECK(hipGetLastError());
  for (int i = 0; i < (a.no_secant ? 0 : a.N_secant_steps); ++i) {
    if ((rc = launch_sdf(SL, a.sdf_packed, c.pts_s, R, c.ss, nullptr, nullptr, a.sdf->multires, nullptr, 0, st)))
      return rc;
    hipLaunchKernelGGL(uni_secant, grd, blk, 0, st, c, (int)(i == a.N_secant_steps - 1));
    NR_HIP_CHECK(hipGetLastError());
  }
  UniOut o{ray0, a.rgb, a.depth, a.acc, a.normals, a.surface_points, a.mask_surface, a.depth_surface,
           a.radiance_out, a.sdf_out, a.nablas_out, a.alpha_out, a.weights_out};
  hipLaunchKernelGGL(uni_samples, grd, blk, 0, st, c, o);
  NR_HIP_CHECK(hipGetLastError());
  if (a.d_all_out) {  // training: the sorted sample depths, ray-major (unisurf.py:201)
    hipLaunchKernelGGL(neus_write_dall, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, c.d_all, (int64_t)R, c.P,
                       ray0, a.d_all_out);
    NR_HIP_CHECK(hipGetLastError());
  }
  if (a.sample_only) return NR_OK;
  if ((rc = launch_sdf(SL, a.sdf_packed, c.pts_f, P, c.sdf_f, c.nab_f, c.feat_f, a.sdf->multires, mlp_ws, mlp_bytes,
                       st)))
    return rc;
  if (a.normal_mode == 1) {
    hipLaunchKernelGGL(uni_window_ss_part, dim3((unsigned)c.nw_row, (unsigned)(R / nloc), kWinSlices), dim3(256), 0,
                       st, c);
    NR_HIP_CHECK(hipGetLastError());
    hipLaunchKernelGGL(uni_window_ss_sum, dim3((unsigned)c.nw_row, (unsigned)(R / nloc)), dim3(64), 0, st, c);
    NR_HIP_CHECK(hipGetLastError());
    if (sharded) {  // every rank's partial sums -> the sums of the whole batch (collective, stream-ordered)
      const int rr = a.window_reduce(a.window_user);
      NR_REQUIRE(rr == 0, NR_ERR_ARG, "nr_unisurf_render: window_reduce callback failed");
    }
  }
  hipLaunchKernelGGL(uni_normalize, dim3((unsigned)((P + 255) / 256)), dim3(256), 0, st, c, a.normal_mode);
  NR_HIP_CHECK(hipGetLastError());
  if ((rc = launch_radiance(RL, a.rad_packed, c.pts_f, c.rd, 1, R, c.nrm_f, c.feat_f, P, c.rad_f,
                            a.rad->multires_view, st)))
    return rc;
  {
    ProfScope prof("unisurf_composite", (double)R, st);
    hipLaunchKernelGGL(uni_composite, grd, blk, 0, st, c, o, a.calc_normal, a.white_bkgd);
  }
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

static int check_unisurf(const NrUnisurfArgs* a) {
  NR_REQUIRE(a, NR_ERR_ARG, "nr_unisurf_render: null args");
  int rc = check_sdf_desc(a->sdf);
  if (rc) return rc;
  if ((rc = check_rad_desc(a->rad))) return rc;
  NR_REQUIRE(a->n_rays <= 0 || (a->rays_o && a->rays_d && (a->sample_only ? a->d_all_out != nullptr
                                                                            : (a->rgb && a->depth && a->acc))),
             NR_ERR_ARG, "nr_unisurf_render: null ray or output pointer");
  NR_REQUIRE(!a->sample_only || a->shard_row_rays <= 0, NR_ERR_ARG,
             "nr_unisurf_render: sample_only is not a sharded render");
  NR_REQUIRE(a->sdf_packed && a->rad && (a->rad_packed || a->sample_only) && a->t_march && a->t_query && a->t_free,
             NR_ERR_ARG, "nr_unisurf_render: null argument");
  NR_REQUIRE(a->n_rays <= 0 || a->sample_only || !a->calc_normal || a->normals, NR_ERR_ARG,
             "nr_unisurf_render: calc_normal needs normals output");
  NR_REQUIRE(a->N_steps >= 2 && a->N_secant_steps >= 0 && a->N_query >= 1 && a->N_freespace >= 1, NR_ERR_ARG,
             "nr_unisurf_render: bad sample counts");
  NR_REQUIRE(a->normal_mode == 0 || a->normal_mode == 1, NR_ERR_ARG, "nr_unisurf_render: normal_mode must be 0|1");
  NR_REQUIRE(!a->u_query == !a->u_free, NR_ERR_ARG, "nr_unisurf_render: u_query and u_free go together");
  NR_REQUIRE(a->normal_mode == 0 || (a->rayschunk > 0 && a->netchunk > 0), NR_ERR_ARG,
             "nr_unisurf_render: rayschunk/netchunk must be positive");
  if (a->rays_per_batch > 0)
    NR_REQUIRE(a->n_rays % a->rays_per_batch == 0, NR_ERR_ARG, "nr_unisurf_render: n_rays % rays_per_batch != 0");
  NR_REQUIRE(unisurf_chunk_rays(*a) > 0, NR_ERR_UNSUPPORTED,
             "nr_unisurf_render: rayschunk too large for windowed normalisation unless netchunk % P == 0");
  if (a->shard_row_rays > 0) {
    NR_REQUIRE(a->normal_mode == 1 && a->window_ss && a->window_reduce, NR_ERR_ARG,
               "nr_unisurf_render: a sharded render needs normal_mode 1, window_ss and window_reduce");
    const int64_t nloc = a->rays_per_batch > 0 ? a->rays_per_batch : a->n_rays;
    NR_REQUIRE(a->shard_ray0 >= 0 && a->shard_ray0 + nloc <= a->shard_row_rays, NR_ERR_ARG,
               "nr_unisurf_render: shard outside its batch row");
  }
  return NR_OK;
}

}  // namespace nr

using namespace nr;

extern "C" {

int nr_version(void) { return 1; }
#ifndef NR_BUILD_ID
#define NR_BUILD_ID "unknown-source00"
#endif
// the marker lets neurecon_amd/build.py read the ID from the file without loading it
__attribute__((used)) static const char kBuildIdMarker[] = "NR_BUILD_ID=" NR_BUILD_ID;
const char* nr_build_id(void) { return kBuildIdMarker + 12; }
const char* nr_last_error(void) { return g_err.c_str(); }

size_t nr_sdf_packed_bytes(const NrSdfDesc* d) {
  if (check_sdf_desc(d)) return 0;
  return sdf_layout(*d).total;
}

int nr_sdf_pack(const NrSdfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream) {
  int rc = check_sdf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(W && b && packed, NR_ERR_ARG, "nr_sdf_pack: null argument");
  for (int l = 0; l <= d->D; ++l) NR_REQUIRE(W[l] && b[l], NR_ERR_ARG, "nr_sdf_pack: null layer pointer");
  hipStream_t st = (hipStream_t)stream;
  const SdfLayout L = sdf_layout(*d);
  char* P = (char*)packed;
  if (L.siren) {  // S0..S4, SF, SB4..SB0 (nr_mlp.h SirenOp); layer 5 = Linear(256 -> 257)
    const int prec = d->precision;
    float* wmax = (float*)(P + L.scale_off);
    float* bound = (float*)(P + L.bound_off);
    PackOp ops[kSirenOps];
    ops[S0] = mkop(W[0], b[0], 256, 3, 0, seg(16, 0, 256), none(), seg(4, 0, 3), none(), 1.0f, prec, wmax + S0);
    for (int l = 1; l < 5; ++l)
      ops[S0 + l] = mkop(W[l], b[l], 256, 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec,
                         wmax + S0 + l);
    ops[SF] = mkop(W[5], b[5], 257, 256, 0, seg(16, 1, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + SF);
    for (int l = 4; l >= 1; --l)
      ops[SB4 + (4 - l)] = mkop(W[l], nullptr, 256, 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f,
                                prec, wmax + SB4 + (4 - l));
    ops[SB0] = mkop(W[0], nullptr, 256, 3, 1, seg(4, 0, 3), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + SB0);
    char* dst[kSirenOps];
    for (int i = 0; i < kSirenOps; ++i) {
      ops[i].bound = bound + 2 * i;
      dst[i] = P + L.op_off[i];
    }
    if ((rc = launch_pack_ops(ops, dst, kSirenOps, st))) return rc;
    if ((rc = launch_pack_vec(W[5], 0, 256, 256, P + L.w8row0_off, st))) return rc;
    return launch_pack_vec(b[5], 0, 1, 4, P + L.misc_off, st);
  }
  const int in0 = 39, n3 = 217;
  const float isq2 = 1.0f / 1.41421356237309504880f;
  const int prec = d->precision;
  float* wmax = (float*)(P + L.scale_off);
  auto ROWS = [&](int l) { return l == 3 ? n3 : (l == 8 ? 257 : 256); };
  PackOp ops[kSdfOps];
  // forward
  ops[F0] = mkop(W[0], b[0], ROWS(0), in0, 0, seg(16, 0, 256), none(), seg(4, 0, in0), none(), 1.0f, prec, wmax + F0);
  ops[F1] = mkop(W[1], b[1], ROWS(1), 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F1);
  ops[F2] = mkop(W[2], b[2], ROWS(2), 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F2);
  ops[F3] = mkop(W[3], b[3], ROWS(3), 256, 0, seg(14, 0, n3), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F3);
  ops[F4] = mkop(W[4], b[4], ROWS(4), 256, 0, seg(16, 0, 256), none(), seg(14, 0, n3), seg(4, n3, in0), isq2, prec, wmax + F4);
  ops[F5] = mkop(W[5], b[5], ROWS(5), 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F5);
  ops[F6] = mkop(W[6], b[6], ROWS(6), 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F6);
  ops[F7] = mkop(W[7], b[7], ROWS(7), 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F7);
  ops[F8] = mkop(W[8], b[8], ROWS(8), 256, 0, seg(16, 1, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + F8);
  // backward (transposed)
  ops[B7] = mkop(W[7], nullptr, ROWS(7), 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + B7);
  ops[B6] = mkop(W[6], nullptr, ROWS(6), 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + B6);
  ops[B5] = mkop(W[5], nullptr, ROWS(5), 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + B5);
  ops[B4] = mkop(W[4], nullptr, ROWS(4), 256, 1, seg(14, 0, n3), seg(4, n3, in0), seg(16, 0, 256), none(), isq2, prec, wmax + B4);
  ops[B3] = mkop(W[3], nullptr, ROWS(3), 256, 1, seg(16, 0, 256), none(), seg(14, 0, n3), none(), 1.0f, prec, wmax + B3);
  ops[B2] = mkop(W[2], nullptr, ROWS(2), 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + B2);
  ops[B1] = mkop(W[1], nullptr, ROWS(1), 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + B1);
  ops[B0] = mkop(W[0], nullptr, ROWS(0), in0, 1, seg(4, 0, in0), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + B0);
  float* bound = (float*)(P + L.bound_off);
  for (int i = 0; i < kSdfOps; ++i) ops[i].bound = bound + 2 * i;
  ops[F7].aux = W[8];  // sdf row W8[0, :] rides with F7's chunks (v2 pipeline's running dot product)
  char* dst[kSdfOps];
  for (int i = 0; i < kSdfOps; ++i) dst[i] = P + L.op_off[i];
  if ((rc = launch_pack_ops(ops, dst, kSdfOps, st))) return rc;
  if (L.l32_off) {  // the 32x32x16 copy of the forward ops (same scales and bounds, rewritten identically)
    for (int i = 0; i <= F8; ++i) {
      ops[i].l32 = 1;
      dst[i] = P + L.l32_off + L.op_off[i];
    }
    if ((rc = launch_pack_ops(ops, dst, F8 + 1, st))) return rc;
  }
  if ((rc = launch_pack_vec(W[8], 0, 256, 256, P + L.w8row0_off, st))) return rc;
  if ((rc = launch_pack_vec(b[8], 0, 1, 4, P + L.misc_off, st))) return rc;
  return NR_OK;
}

size_t nr_mlp_workspace_bytes(int with_backward) { return with_backward ? scratch_bytes() : 0; }

int nr_sdf_forward(const NrSdfDesc* d, const void* packed, const float* pts, int64_t P, float* sdf, float* nabla,
                   float* feature, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_sdf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(packed && pts && sdf && P >= 0, NR_ERR_ARG, "nr_sdf_forward: null argument");
  return launch_sdf(sdf_layout(*d), packed, pts, P, sdf, nabla, feature, d->multires, workspace, workspace_bytes,
                    (hipStream_t)stream);
}

size_t nr_nerf_packed_bytes(const NrNerfDesc* d) {
  if (check_nerf_desc(d)) return 0;
  return nerf_layout(*d).total;
}

int nr_nerf_pack(const NrNerfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream) {
  int rc = check_nerf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(W && b && packed, NR_ERR_ARG, "nr_nerf_pack: null argument");
  for (int l = 0; l < 12; ++l) NR_REQUIRE(W[l] && b[l], NR_ERR_ARG, "nr_nerf_pack: null layer pointer");
  hipStream_t st = (hipStream_t)stream;
  const NerfLayout L = nerf_layout(*d);
  char* P = (char*)packed;
  const int prec = d->precision;
  float* wmax = (float*)(P + L.scale_off);
  const int in0 = 84, inv = 27;
  PackOp ops[kNerfOps];
  ops[N0] = mkop(W[0], b[0], 256, in0, 0, seg(16, 0, 256), none(), seg(6, 0, in0), none(), 1.0f, prec, wmax + N0);
  for (int i = 1; i < 8; ++i) {
    if (i == 5)  // Linear(W + input_ch, W): columns [input_pts(84) | h(256)] -> K blocks [h ; input_pts]
      ops[i] = mkop(W[i], b[i], 256, 256 + in0, 0, seg(16, 0, 256), none(), seg(16, in0, 256), seg(6, 0, in0), 1.0f,
                    prec, wmax + i);
    else
      ops[i] = mkop(W[i], b[i], 256, 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + i);
  }
  if (prec == NR_PREC_F16X3) {  // [feature_linear; alpha_linear]: sigma = row 0 of output block 16
    ops[NF] = mkop(W[8], b[8], 256, 256, 0, seg(16, 0, 256), seg(2, 0, 1), seg(16, 0, 256), none(), 1.0f, prec,
                   wmax + NF);
    ops[NF].W2 = W[10];
    ops[NF].bias2 = b[10];
    ops[NF].wn2 = 256;
    ops[NF].ld2 = 256;
  } else {
    ops[NF] = mkop(W[8], b[8], 256, 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + NF);
  }
  ops[NV] = mkop(W[9], b[9], 128, 256 + inv, 0, seg(8, 0, 128), none(), seg(16, 0, 256), seg(2, 256, inv), 1.0f, prec,
                 wmax + NV);
  float* bound = (float*)(P + L.bound_off);
  char* dst[kNerfOps];
  for (int i = 0; i < kNerfOps; ++i) {
    ops[i].bound = bound + 2 * i;
    dst[i] = P + L.op_off[i];
  }
  if ((rc = launch_pack_ops(ops, dst, kNerfOps, st))) return rc;
  if ((rc = launch_pack_vec(W[10], 0, 256, 256, P + L.alpha_off, st))) return rc;
  if ((rc = launch_pack_vec(b[10], 0, 1, 1, P + L.alpha_off + 256 * 4, st))) return rc;
  if ((rc = launch_pack_vec(W[11], 0, 384, 384, P + L.rgb_off, st))) return rc;
  if ((rc = launch_pack_vec(b[11], 0, 3, 3, P + L.rgb_off + 384 * 4, st))) return rc;
  return NR_OK;
}

int nr_nerf_forward(const NrNerfDesc* d, const void* packed, const float* x4, const float* vdir, int64_t vdir_div,
                    int64_t P, float* sigma, float* rgb, void* stream) {
  int rc = check_nerf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(packed && x4 && vdir && sigma && rgb && vdir_div > 0 && P >= 0, NR_ERR_ARG,
             "nr_nerf_forward: bad argument");
  return launch_nerf(nerf_layout(*d), packed, x4, vdir, vdir_div, INT64_MAX, P, sigma, rgb, (hipStream_t)stream);
}

size_t nr_radiance_packed_bytes(const NrRadDesc* d) {
  if (check_rad_desc(d)) return 0;
  return rad_layout(*d).total;
}

int nr_radiance_pack(const NrRadDesc* d, const float* const* W, const float* const* b, void* packed, void* stream) {
  int rc = check_rad_desc(d);
  if (rc) return rc;
  NR_REQUIRE(W && b && packed, NR_ERR_ARG, "nr_radiance_pack: null argument");
  for (int l = 0; l <= d->D; ++l) NR_REQUIRE(W[l] && b[l], NR_ERR_ARG, "nr_radiance_pack: null layer pointer");
  hipStream_t st = (hipStream_t)stream;
  const RadLayout L = rad_layout(*d);
  char* P = (char*)packed;
  const int ns = L.n_small, ld0 = ns + 256;
  PackOp ops[5];
  const int prec = d->precision;
  float* wmax = (float*)(P + L.scale_off);
  ops[0] = mkop(W[0], b[0], 256, ld0, 0, seg(16, 0, 256), none(), seg(16, ns, 256), seg(L.kbs, 0, ns), 1.0f, prec, wmax);
  for (int i = 1; i < L.D; ++i)
    ops[i] = mkop(W[i], b[i], 256, 256, 0, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + i);
  float* bound = (float*)(P + L.bound_off);
  char* dst[5];
  for (int i = 0; i < L.D; ++i) {
    ops[i].bound = bound + 2 * i;
    dst[i] = P + L.op_off[i];
  }
  if ((rc = launch_pack_ops(ops, dst, L.D, st))) return rc;
  if ((rc = launch_pack_vec(W[L.D], 0, 768, 768, P + L.head_off, st))) return rc;
  if ((rc = launch_pack_vec(b[L.D], 0, 3, 4, P + L.head_off + 768 * 4, st))) return rc;
  return NR_OK;
}

int nr_radiance_forward(const NrRadDesc* d, const void* packed, const float* x, const float* vdir, int64_t vdir_div,
                        const float* normals, const float* feature, int64_t P, float* rgb, void* stream) {
  int rc = check_rad_desc(d);
  if (rc) return rc;
  NR_REQUIRE(packed && x && (d->no_view_dirs || (vdir && normals)) && feature && rgb && vdir_div > 0, NR_ERR_ARG,
             "nr_radiance_forward: bad argument");
  return launch_radiance(rad_layout(*d), packed, x, vdir, vdir_div, INT64_MAX, normals, feature, P, rgb,
                         d->multires_view, (hipStream_t)stream);
}

int nr_radiance_train_fwd32(const NrRadDesc* d, const void* packed, const float* feat, const float* small,
                            int64_t ld_small, int64_t P, float* h0, float* h1, float* h2, float* h3, float* rgb,
                            void* stream) {
  int rc = check_rad_desc(d);
  if (rc) return rc;
  NR_REQUIRE(P >= 0, NR_ERR_ARG, "nr_radiance_train_fwd32: negative P");
  if (P == 0) return NR_OK;
  NR_REQUIRE(packed && feat && small && h0 && h1 && h2 && h3 && rgb, NR_ERR_ARG,
             "nr_radiance_train_fwd32: null argument");
  const RadLayout L = rad_layout(*d);
  NR_REQUIRE(ld_small >= L.n_small, NR_ERR_ARG, "nr_radiance_train_fwd32: ld_small below the small-input count");
  float* const h[4] = {h0, h1, h2, h3};
  return launch_radiance_train32(L, packed, feat, small, ld_small, L.n_small, P, h, rgb, (hipStream_t)stream);
}

// ---- NeRF++ net in the training step (nr_mlp.hip nerf_train32_*_kernel) ---------------------------
static NerfBwdLayout nerf_bwd_layout() {
  NerfBwdLayout B{};
  size_t off = 0;
  for (int i = 0; i < kNerfBwdOps; ++i) {
    B.op_bytes[i] = (2 * (i == NBV ? 8 : 16) + 1) * 1024;
    B.op_off[i] = (uint32_t)off;
    off += 8 * (size_t)B.op_bytes[i];  // 16 output blocks = 8 chunks
  }
  B.scale_off = (uint32_t)off;
  off = align256(off + kNerfBwdOps * 4);
  B.wr_off = (uint32_t)off;
  off = align256(off + 3 * 128 * 4);
  B.wa_off = (uint32_t)off;
  off = align256(off + 256 * 4);
  B.total = (uint32_t)off;
  return B;
}

size_t nr_nerf_train_packed_bytes(const NrNerfDesc* d) {
  if (check_nerf_desc(d)) return 0;
  return nerf_bwd_layout().total;
}

int nr_nerf_train_pack(const NrNerfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream) {
  int rc = check_nerf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(W && b && packed, NR_ERR_ARG, "nr_nerf_train_pack: null argument");
  for (int l = 0; l < 12; ++l) NR_REQUIRE(W[l], NR_ERR_ARG, "nr_nerf_train_pack: null layer pointer");
  hipStream_t st = (hipStream_t)stream;
  const NerfBwdLayout B = nerf_bwd_layout();
  char* P = (char*)packed;
  float* wmax = (float*)(P + B.scale_off);
  const int prec = d->precision == NR_PREC_F16X3 ? NR_PREC_F16X3 : NR_PREC_FP32, in0 = 84, inv = 27;
  PackOp ops[kNerfBwdOps];
  // views_linears[0]^T restricted to the feature columns: [128][256 + 27] -> out 256 (feature), in 128
  ops[NBV] = mkop(W[9], nullptr, 128, 256 + inv, 1, seg(16, 0, 256), none(), seg(8, 0, 128), none(), 1.0f, prec,
                  wmax + NBV);
  ops[NBF] = mkop(W[8], nullptr, 256, 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec,
                  wmax + NBF);
  for (int i = 7; i >= 1; --i) {
    const int o = NB7 + (7 - i);
    if (i == 5)  // input cat([x_emb(84), h4(256)]): the h4 columns 84..339
      ops[o] = mkop(W[5], nullptr, 256, 256 + in0, 1, seg(16, in0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec,
                    wmax + o);
    else
      ops[o] = mkop(W[i], nullptr, 256, 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f, prec, wmax + o);
  }
  char* dst[kNerfBwdOps];
  for (int i = 0; i < kNerfBwdOps; ++i) dst[i] = P + B.op_off[i];
  if ((rc = launch_pack_ops(ops, dst, kNerfBwdOps, st))) return rc;
  if ((rc = launch_pack_vec(W[11], 0, 384, 384, P + B.wr_off, st))) return rc;
  if ((rc = launch_pack_vec(W[10], 0, 256, 256, P + B.wa_off, st))) return rc;
  return NR_OK;
}

int nr_nerf_train_fwd32(const NrNerfDesc* d, const void* packed, const float* x_emb, const float* v_emb, int64_t P,
                        float* const* h, float* feat, float* hv, float* sigma, float* rgb, void* stream) {
  int rc = check_nerf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(d->precision == NR_PREC_FP32, NR_ERR_ARG, "nr_nerf_train_fwd32: the desc / pack must be NR_PREC_FP32");
  NR_REQUIRE(P >= 0, NR_ERR_ARG, "nr_nerf_train_fwd32: negative P");
  if (P == 0) return NR_OK;
  NR_REQUIRE(packed && x_emb && v_emb && h && feat && hv && sigma && rgb, NR_ERR_ARG,
             "nr_nerf_train_fwd32: null argument");
  for (int i = 0; i < 8; ++i) NR_REQUIRE(h[i], NR_ERR_ARG, "nr_nerf_train_fwd32: null activation pointer");
  NR_REQUIRE(((uintptr_t)x_emb & 15) == 0, NR_ERR_ARG, "nr_nerf_train_fwd32: x_emb must be 16-byte aligned");
  return launch_nerf_train32_fwd(nerf_layout(*d), packed, x_emb, v_emb, P, h, feat, hv, sigma, rgb,
                                 (hipStream_t)stream);
}

int nr_nerf_train_bwd32(const NrNerfDesc* d, const void* train_packed, const float* rgb, const float* hv,
                        const float* const* h, const float* g_rgb, const float* g_sigma, int64_t P, float* g3,
                        float* ghv, float* g_feat, float* const* gz, void* stream) {
  int rc = check_nerf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(P >= 0, NR_ERR_ARG, "nr_nerf_train_bwd32: negative P");
  if (P == 0) return NR_OK;
  NR_REQUIRE(train_packed && rgb && hv && h && g3 && ghv && g_feat && gz, NR_ERR_ARG,
             "nr_nerf_train_bwd32: null argument");
  for (int i = 0; i < 8; ++i) NR_REQUIRE(h[i] && gz[i], NR_ERR_ARG, "nr_nerf_train_bwd32: null layer pointer");
  return launch_nerf_train32_bwd(nerf_bwd_layout(), train_packed, rgb, hv, h, g_rgb, g_sigma, P, g3, ghv, g_feat, gz,
                                 (hipStream_t)stream, d->precision == NR_PREC_F16X3);
}

// ---- training layer GEMMs (nr_mlp.hip tgemm_kernel) ---------------------------------------------
int nr_train_gemm(const NrTrainGemm* a, int KB, int KB2, int NBO, int NB2, void* stream) {
  NR_REQUIRE(a, NR_ERR_ARG, "nr_train_gemm: null argument");
  return launch_tgemm(*a, KB, KB2, NBO, NB2, (hipStream_t)stream);
}

static int softplus_net(const NrSdfDesc* d) {
  int rc = check_sdf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(!d->siren && d->precision == NR_PREC_F16X3, NR_ERR_UNSUPPORTED,
             "training GEMMs: f16x3 softplus SDF nets only (SIREN / fp32 nets train on nr_gemm32)");
  return NR_OK;
}

int nr_sdf_op_info(const NrSdfDesc* d, int op, int64_t* offset, int* kb, int* nbo) {
  int rc = softplus_net(d);
  if (rc) return rc;
  NR_REQUIRE(offset && kb && nbo && op >= 0 && op <= kSdfOps, NR_ERR_ARG, "nr_sdf_op_info: bad argument");
  if (op == kSdfOps) {  // B8 = W8^T of the training pack
    *offset = 0; *kb = 18; *nbo = 16;
    return NR_OK;
  }
  const SdfLayout L = sdf_layout(*d);
  *offset = L.op_off[op]; *kb = kSdfKB[op]; *nbo = kSdfNBO[op];
  return NR_OK;
}

size_t nr_sdf_train_packed_bytes(const NrSdfDesc* d) {
  if (softplus_net(d)) return 0;
  return align256((size_t)8 * chunk_bytes_host(18) + 4) + 256;
}

// W8^T [256 x 257]: output rows = the 256 inputs of layer 8 (h7), input blocks [feature rows (16) ;
// sdf row (2 blocks, 1 valid)]; per-row vector W8[0, :] (g_7 of the nabla chain, nr_train.hip)
int nr_sdf_train_pack(const NrSdfDesc* d, const float* const* W, const float* const* b, void* packed, void* stream) {
  int rc = softplus_net(d);
  if (rc) return rc;
  NR_REQUIRE(W && b && packed && W[8], NR_ERR_ARG, "nr_sdf_train_pack: null argument");
  char* P = (char*)packed;
  float* wmax = (float*)(P + (size_t)8 * chunk_bytes_host(18));
  PackOp op = mkop(W[8], nullptr, 257, 256, 1, seg(16, 0, 256), none(), seg(16, 1, 256), seg(2, 0, 1), 1.0f,
                   NR_PREC_F16X3, wmax);
  op.aux = W[8];
  return launch_pack_op(op, P, (hipStream_t)stream);
}

static int train_radiance(const NrRadDesc* d) {
  int rc = check_rad_desc(d);
  if (rc) return rc;
  NR_REQUIRE(!d->siren && d->D == 4 && d->precision == NR_PREC_F16X3, NR_ERR_UNSUPPORTED,
             "training GEMMs: f16x3 ReLU radiance nets with D = 4 only");
  return NR_OK;
}

// training pack of a radiance net: head^T (KB 2), W3^T, W2^T, W1^T (16 x 16), W0^T (out 16 + kbs)
static void rad_train_layout(const RadLayout& L, int64_t (&off)[5], int (&kb)[5], int (&nbo)[5], int64_t& total) {
  const int KBs[5] = {2, 16, 16, 16, 16};
  const int NBOs[5] = {16, 16, 16, 16, 16 + L.kbs};
  int64_t o = 0;
  for (int i = 0; i < 5; ++i) {
    off[i] = o; kb[i] = KBs[i]; nbo[i] = NBOs[i];
    o += (int64_t)(NBOs[i] / 2) * chunk_bytes_host(KBs[i]);
  }
  total = o;
}

int nr_radiance_op_info(const NrRadDesc* d, int op, int64_t* offset, int* kb, int* nbo) {
  int rc = train_radiance(d);
  if (rc) return rc;
  NR_REQUIRE(offset && kb && nbo && op >= 0 && op <= 2 * d->D + 1, NR_ERR_ARG, "nr_radiance_op_info: bad argument");
  const RadLayout L = rad_layout(*d);
  if (op < d->D) {
    *offset = L.op_off[op]; *kb = op == 0 ? 16 + L.kbs : 16; *nbo = 16;
  } else if (op == d->D) {
    *offset = L.head_off; *kb = 0; *nbo = 0;
  } else {
    int64_t off[5], total;
    int kbs[5], nbos[5];
    rad_train_layout(L, off, kbs, nbos, total);
    const int i = op - d->D - 1;
    *offset = off[i]; *kb = kbs[i]; *nbo = nbos[i];
  }
  return NR_OK;
}

size_t nr_radiance_train_packed_bytes(const NrRadDesc* d) {
  if (train_radiance(d)) return 0;
  int64_t off[5], total;
  int kb[5], nbo[5];
  rad_train_layout(rad_layout(*d), off, kb, nbo, total);
  return align256((size_t)total + 5 * 4) + 256;
}

int nr_radiance_train_pack(const NrRadDesc* d, const float* const* W, const float* const* b, void* packed,
                           void* stream) {
  int rc = train_radiance(d);
  if (rc) return rc;
  NR_REQUIRE(W && b && packed, NR_ERR_ARG, "nr_radiance_train_pack: null argument");
  for (int l = 0; l <= d->D; ++l) NR_REQUIRE(W[l], NR_ERR_ARG, "nr_radiance_train_pack: null layer pointer");
  hipStream_t st = (hipStream_t)stream;
  const RadLayout L = rad_layout(*d);
  int64_t off[5], total;
  int kb[5], nbo[5];
  rad_train_layout(L, off, kb, nbo, total);
  char* P = (char*)packed;
  float* wmax = (float*)(P + total);
  const int ns = L.n_small, ld0 = ns + 256;
  PackOp ops[5];
  ops[0] = mkop(W[4], nullptr, 3, 256, 1, seg(16, 0, 256), none(), seg(2, 0, 3), none(), 1.0f, NR_PREC_F16X3, wmax);
  for (int i = 1; i <= 3; ++i)  // W3^T, W2^T, W1^T
    ops[i] = mkop(W[4 - i], nullptr, 256, 256, 1, seg(16, 0, 256), none(), seg(16, 0, 256), none(), 1.0f,
                  NR_PREC_F16X3, wmax + i);
  ops[4] = mkop(W[0], nullptr, 256, ld0, 1, seg(16, ns, 256), seg(L.kbs, 0, ns), seg(16, 0, 256), none(), 1.0f,
                NR_PREC_F16X3, wmax + 4);
  char* dst[5];
  for (int i = 0; i < 5; ++i) dst[i] = P + off[i];
  if ((rc = launch_pack_ops(ops, dst, 5, st))) return rc;
  return NR_OK;
}

size_t nr_neus_workspace_bytes(const NrNeusArgs* a) {
  if (!a) return 0;
  return neus_plan(*a, neus_chunk_rays(a)).total;
}

int nr_neus_render(const NrNeusArgs* a, void* stream) {
  NR_REQUIRE(a, NR_ERR_ARG, "nr_neus_render: null args");
  int rc = check_sdf_desc(a->sdf);
  if (rc) return rc;
  if ((rc = check_rad_desc(a->rad))) return rc;
  // an empty shard (multi-GPU ray sharding) may pass null ray / output pointers
  NR_REQUIRE(a->n_rays <= 0 || (a->rays_o && a->rays_d && (a->sample_only ? a->d_all_out != nullptr
                                                                            : (a->rgb && a->depth && a->acc))),
             NR_ERR_ARG, "nr_neus_render: null ray or output pointer");
  NR_REQUIRE(a->sdf_packed && a->rad && (a->rad_packed || a->sample_only) && a->t_coarse, NR_ERR_ARG,
             "nr_neus_render: null argument");
  NR_REQUIRE(a->N_samples >= 2, NR_ERR_ARG, "nr_neus_render: N_samples must be >= 2");
  NR_REQUIRE(a->n_rays <= 0 || a->sample_only || !a->calc_normal || a->normals, NR_ERR_ARG,
             "nr_neus_render: calc_normal needs normals output");
  NR_REQUIRE(a->N_outside >= 0, NR_ERR_ARG, "nr_neus_render: N_outside must be >= 0");
  if (a->N_outside > 0) {
    if ((rc = check_nerf_desc(a->nerf))) return rc;
    NR_REQUIRE(a->nerf_packed && a->t_outside, NR_ERR_ARG, "nr_neus_render: N_outside > 0 needs the NeRF++ net");
  }
  NR_REQUIRE(a->upsample_algo >= NR_UPSAMPLE_OFFICIAL && a->upsample_algo <= NR_UPSAMPLE_DIRECT_MORE, NR_ERR_ARG,
             "nr_neus_render: unknown upsample_algo");
  if (a->upsample_algo != NR_UPSAMPLE_OFFICIAL) {
    NR_REQUIRE(a->N_importance >= 1 && a->u_fine && a->fixed_s > 0.f, NR_ERR_ARG,
               "nr_neus_render: direct upsampling needs N_importance >= 1, u_fine and fixed_s > 0");
    NR_REQUIRE(a->upsample_algo != NR_UPSAMPLE_DIRECT_MORE || (a->N_nograd_samples >= 2 && a->t_nograd), NR_ERR_ARG,
               "nr_neus_render: direct_more needs N_nograd_samples >= 2 and t_nograd");
  } else if (a->N_upsample_iters > 0) {
    const int n_up = a->N_importance / a->N_upsample_iters;
    NR_REQUIRE(n_up >= 1 && n_up <= kMaxUp && a->u_fine, NR_ERR_UNSUPPORTED,
               "nr_neus_render: N_importance/N_upsample_iters must be in [1, 32]");
  }
  if (a->n_rays <= 0) return NR_OK;
  const int64_t Rc = neus_chunk_rays(a);
  const NeusPlan pl = neus_plan(*a, Rc);
  NR_REQUIRE(a->workspace && a->workspace_bytes >= pl.total, NR_ERR_WORKSPACE, "nr_neus_render: workspace too small");
  {  // the wave-per-ray upsampling / compositing kernels stage S samples per ray in LDS
    const bool direct = a->upsample_algo != NR_UPSAMPLE_OFFICIAL;
    const int S = direct ? a->N_samples + a->N_importance
                         : a->N_samples + a->N_upsample_iters * (a->N_upsample_iters > 0 ? a->N_importance / a->N_upsample_iters : 0);
    int dev = 0, lds_max = 65536;
    NR_HIP_CHECK(hipGetDevice(&dev));
    NR_HIP_CHECK(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
    NR_REQUIRE((size_t)9 * S * sizeof(float) <= (size_t)lds_max, NR_ERR_UNSUPPORTED,
               "nr_neus_render: N_samples + N_importance too large for the per-ray LDS staging of the compositing");
  }
  for (int64_t r0 = 0; r0 < a->n_rays; r0 += Rc) {
    const int R = (int)((a->n_rays - r0) < Rc ? (a->n_rays - r0) : Rc);
    if ((rc = neus_chunk(*a, pl, r0, R, (hipStream_t)stream))) return rc;
  }
  return NR_OK;
}

size_t nr_volsdf_workspace_bytes(const NrVolsdfArgs* a) {
  if (!a || check_volsdf(a)) return 0;
  return volsdf_plan(*a, volsdf_chunk_rays(a)).total;
}

int nr_volsdf_render(const NrVolsdfArgs* a, void* stream) {
  int rc = check_volsdf(a);
  if (rc) return rc;
  if (a->n_rays <= 0) return NR_OK;
  const int64_t Rc = volsdf_chunk_rays(a);
  const VolPlan pl = volsdf_plan(*a, Rc);
  NR_REQUIRE(a->workspace && a->workspace_bytes >= pl.total, NR_ERR_WORKSPACE,
             "nr_volsdf_render: workspace too small");
  int dev = 0, lds_max = 65536;
  NR_HIP_CHECK(hipGetDevice(&dev));
  NR_HIP_CHECK(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerBlock, dev));
  NR_REQUIRE(pl.lds_bytes <= (size_t)lds_max, NR_ERR_UNSUPPORTED,
             "nr_volsdf_render: per-ray sample list does not fit in LDS (reduce N_samples or max_upsample_steps)");
  for (int64_t r0 = 0; r0 < a->n_rays; r0 += Rc) {
    const int R = (int)((a->n_rays - r0) < Rc ? (a->n_rays - r0) : Rc);
    if ((rc = volsdf_chunk(*a, pl, r0, R, (hipStream_t)stream))) return rc;
  }
  return NR_OK;
}

size_t nr_unisurf_workspace_bytes(const NrUnisurfArgs* a) {
  if (!a || check_unisurf(a)) return 0;
  return unisurf_plan(*a, unisurf_chunk_rays(*a)).total;
}

int64_t nr_unisurf_window_count(const NrUnisurfArgs* a) {
  if (!a || a->normal_mode != 1) return 0;
  int64_t rc_rays, nw_full, nw_row;
  unisurf_windows(*a, rc_rays, nw_full, nw_row);
  return nw_row;
}

int nr_unisurf_render(const NrUnisurfArgs* a, void* stream) {
  int rc = check_unisurf(a);
  if (rc) return rc;
  const bool sharded = a->shard_row_rays > 0;
  if (a->n_rays <= 0) {  // an empty shard still joins the collective
    if (sharded) NR_REQUIRE(a->window_reduce(a->window_user) == 0, NR_ERR_ARG, "nr_unisurf_render: window_reduce failed");
    return NR_OK;
  }
  const int64_t Rc = unisurf_chunk_rays(*a);
  const UniPlan pl = unisurf_plan(*a, Rc);
  NR_REQUIRE(a->workspace && a->workspace_bytes >= pl.total, NR_ERR_WORKSPACE,
             "nr_unisurf_render: workspace too small");
  if (sharded)  // the whole shard (every batch row) is one chunk: one window reduction per call
    return unisurf_chunk(*a, pl, 0, (int)a->n_rays, a->shard_ray0,
                         (int)(a->rays_per_batch > 0 ? a->rays_per_batch : a->n_rays), (hipStream_t)stream);
  const int64_t per_b = (a->normal_mode == 1 && a->rays_per_batch > 0) ? a->rays_per_batch : a->n_rays;
  // window mode: chunks restart at every batch row and at every reference ray chunk
  const int64_t span = a->normal_mode == 1 ? (a->rayschunk < per_b ? a->rayschunk : per_b) : per_b;
  for (int64_t b0 = 0; b0 < a->n_rays; b0 += per_b) {
    const int64_t b1 = b0 + per_b < a->n_rays ? b0 + per_b : a->n_rays;
    for (int64_t c0 = b0; c0 < b1; c0 += span) {
      const int64_t c1 = c0 + span < b1 ? c0 + span : b1;
      for (int64_t r0 = c0; r0 < c1; r0 += Rc) {
        const int R = (int)((c1 - r0) < Rc ? (c1 - r0) : Rc);
        if ((rc = unisurf_chunk(*a, pl, r0, R, r0 - b0, R, (hipStream_t)stream))) return rc;
      }
    }
  }
  return NR_OK;
}

int nr_sample_pdf(const float* bins, const float* weights, int64_t R, int L, const float* u, int64_t u_stride, int N,
                  float* out, void* stream) {
  NR_REQUIRE(bins && weights && u && out && L >= 2 && N >= 1 && u_stride >= 0, NR_ERR_ARG,
             "nr_sample_pdf: bad argument");
  if (R <= 0) return NR_OK;
  hipLaunchKernelGGL(sample_pdf_kernel, dim3((unsigned)((R + 255) / 256)), dim3(256), 0, (hipStream_t)stream, bins,
                     weights, R, L, u, u_stride, N, out);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

}  // extern "C"
