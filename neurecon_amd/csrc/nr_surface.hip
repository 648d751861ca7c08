// neurecon_amd — surface rendering and SDF grid queries:
//   * sphere tracing (models/ray_casting.py:163-182 `sphere_tracing_surface_points`) with the
//     active rays compacted between iterations, so the SDF MLP only runs on rays still marching;
//   * surface_render's per-ray finish (ray_casting.py:219-262: black colour and zero normal off
//     the surface, F.normalize(nablas));
//   * root finding (ray_casting.py:35-160 `root_finding_surface_points`): the UNISURF march /
//     first-crossing / secant kernels driven with scalar or per-ray near / far on caller-normalised
//     rays;
//   * the mesh-extraction grid (utils/mesh_util.py:82-112 `extract_mesh`): voxel coordinates
//     generated on the device with the reference's own float64 formula, then the forward SDF.
#include "nr_common.h"
#include "nr_mlp.h"
#include "nr_unisurf.h"

namespace nr {

int check_sdf_desc(const NrSdfDesc* d);

// F.normalize(v, dim=-1) of one 3-vector: v / max(||v||, 1e-12)
__device__ __forceinline__ void normalize3s(float& x, float& y, float& z) {
  const float d = fmaxf(norm3_ref(x, y, z), 1e-12f);
  x = fdiv(x, d);
  y = fdiv(y, d);
  z = fdiv(z, d);
}

// pts = rays_o + rays_d * d (ray_casting.py:178,181): one rounding for the product, one for the sum
__device__ __forceinline__ void ray_point(const float* ro, const float* rd, int64_t r, float d, float* out) {
#pragma unroll
  for (int c = 0; c < 3; ++c) out[c] = fadd(ro[r * 3 + c], fmul(rd[r * 3 + c], d));
}

__global__ void normalize3_kernel(const float* __restrict__ v, int64_t n, float* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  float x = v[t * 3], y = v[t * 3 + 1], z = v[t * 3 + 2];
  normalize3s(x, y, z);
  out[t * 3] = x;
  out[t * 3 + 1] = y;
  out[t * 3 + 2] = z;
}

// iteration 0: every ray active at d = near (ray_casting.py:175-176)
__global__ void trace_init(const float* __restrict__ ro, const float* __restrict__ rd, int64_t R, float near_s,
                           const float* __restrict__ near_rays, float* __restrict__ d, uint8_t* __restrict__ mask,
                           int* __restrict__ idx, float* __restrict__ pts) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= R) return;
  const float near = near_rays ? near_rays[t] : near_s;
  d[t] = near;
  mask[t] = 1;
  idx[t] = (int)t;
  ray_point(ro, rd, t, near, pts + t * 3);
}

// one sphere-tracing update over the compacted active list (ray_casting.py:179-180):
// d += sdf; rays leaving [0, far] drop out; survivors are appended (wave-aggregated atomic) to
// the next list together with their next query point.  NaN depths stay active, as in the
// reference (both comparisons are false).
__global__ void trace_step(const float* __restrict__ ro, const float* __restrict__ rd, const int* __restrict__ cnt_in,
                           const int* __restrict__ idx_in, const float* __restrict__ sv, float far_s,
                           const float* __restrict__ far_rays, float* __restrict__ d, uint8_t* __restrict__ mask, int* __restrict__ cnt_out,
                           int* __restrict__ idx_out, float* __restrict__ pts_out, int append) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int n = *cnt_in;
  bool alive = false;
  int r = 0;
  float nd = 0.f;
  if (t < n) {
    r = idx_in[t];
    nd = fadd(d[r], sv[t]);
    d[r] = nd;
    const float far = far_rays ? far_rays[r] : far_s;
    alive = !(nd > far) && !(nd < 0.f);
    if (!alive) mask[r] = 0;
  }
  if (!append) return;
  const unsigned long long b = __ballot(alive);
  if (b == 0ull) return;
  const int lane = threadIdx.x & 63;
  const int first = __ffsll((long long)b) - 1;
  int base = 0;
  if (lane == first) base = atomicAdd(cnt_out, __popcll(b));
  base = __shfl(base, first);
  if (alive) {
    const int slot = base + __popcll(b & ((1ull << lane) - 1ull));
    idx_out[slot] = r;
    ray_point(ro, rd, r, nd, pts_out + (int64_t)slot * 3);
  }
}

// final surface points for every ray (ray_casting.py:181)
__global__ void trace_final(const float* __restrict__ ro, const float* __restrict__ rd, int64_t R,
                            const float* __restrict__ d, float* __restrict__ pts) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= R) return;
  ray_point(ro, rd, t, d[t], pts + t * 3);
}

// surface_render finish (ray_casting.py:226, 255-258): rgb[~mask] = 0; normals = F.normalize(nablas),
// normals[~mask] = 0
__global__ void surface_finish(float* __restrict__ rgb, const float* __restrict__ nab,
                               const uint8_t* __restrict__ mask, int64_t n, float* __restrict__ normals) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const bool on = mask[t] != 0;
  if (!on) {
    rgb[t * 3] = 0.f;
    rgb[t * 3 + 1] = 0.f;
    rgb[t * 3 + 2] = 0.f;
  }
  if (normals) {
    float x = nab[t * 3], y = nab[t * 3 + 1], z = nab[t * 3 + 2];
    normalize3s(x, y, z);
    normals[t * 3] = on ? x : 0.f;
    normals[t * 3 + 1] = on ? y : 0.f;
    normals[t * 3 + 2] = on ? z : 0.f;
  }
}

// extract_mesh voxel coordinates (mesh_util.py:87-100), float64 exactly as numpy evaluates them —
// including the reference's true divisions: x = ((i/N)/N) % N, y = (i/N) % N, z = i % N — then
// coordinate = index * (s/(N-1)) + origin (no FMA), cast to float32 (`.float()`, :104).
__global__ void grid_points_kernel(int64_t N, double step, double origin, int64_t i0, int64_t n,
                                   float* __restrict__ pts) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n) return;
  const int64_t i = i0 + t;
  const double Nd = (double)N;
  const double qi = __ddiv_rn((double)i, Nd);
  const double z = (double)(i % N);
  const double y = fmod(qi, Nd);
  const double x = fmod(__ddiv_rn(qi, Nd), Nd);
  pts[t * 3 + 0] = (float)__dadd_rn(__dmul_rn(x, step), origin);
  pts[t * 3 + 1] = (float)__dadd_rn(__dmul_rn(y, step), origin);
  pts[t * 3 + 2] = (float)__dadd_rn(__dmul_rn(z, step), origin);
}

static size_t a256(size_t x) { return (x + 255) & ~(size_t)255; }

struct TracePlan {
  size_t o_idx0, o_idx1, o_pts, o_sv, o_cnt, total;
};

static TracePlan trace_plan(int64_t R) {
  TracePlan p{};
  size_t o = 0;
  p.o_idx0 = o; o += a256((size_t)R * 4);
  p.o_idx1 = o; o += a256((size_t)R * 4);
  p.o_pts = o; o += a256((size_t)R * 12);
  p.o_sv = o; o += a256((size_t)R * 4);
  p.o_cnt = o; o += 256;
  p.total = o;
  return p;
}

static dim3 grid1(int64_t n) { return dim3((unsigned)((n + 255) / 256)); }

constexpr int64_t kRootChunk = 65536;  // rays per chunk: 16.7 M march points at N_steps = 256
constexpr int kSecFloats = 8;          // per-ray secant state (nr_unisurf.hip kSec)

struct RootPlan {
  int64_t Rc;
  size_t o_ro, o_rd, o_near, o_far, o_ptsm, o_sm, o_sec, o_ptss, o_ss;
  size_t o_act0, o_act1, o_acnt, o_ptsc, o_sc;  // chunked march (run_march): active lists, counts, compacted points
  size_t total;
};

static RootPlan root_plan(int64_t n_rays, int N_steps) {
  RootPlan p{};
  p.Rc = n_rays < kRootChunk ? (n_rays > 0 ? n_rays : 1) : kRootChunk;
  const size_t R = (size_t)p.Rc;
  size_t o = 0;
  p.o_ro = o; o += a256(R * 12);
  p.o_rd = o; o += a256(R * 12);
  p.o_near = o; o += a256(R * 4);
  p.o_far = o; o += a256(R * 4);
  p.o_ptsm = o; o += a256(R * (size_t)N_steps * 12);
  p.o_sm = o; o += a256(R * (size_t)N_steps * 4);
  p.o_sec = o; o += a256(R * kSecFloats * 4);
  p.o_ptss = o; o += a256(R * 12);
  p.o_ss = o; o += a256(R * 4);
  p.o_act0 = o; o += a256(R * 4);
  p.o_act1 = o; o += a256(R * 4);
  p.o_acnt = o; o += a256(2 * 4);
  p.o_ptsc = o; o += a256(R * (size_t)kMarchK * 12);
  p.o_sc = o; o += a256(R * (size_t)kMarchK * 4);
  p.total = o;
  return p;
}

}  // namespace nr

using namespace nr;

extern "C" {

size_t nr_sphere_trace_workspace_bytes(int64_t n_rays) { return n_rays > 0 ? trace_plan(n_rays).total : 256; }

int nr_sphere_trace(const NrSdfDesc* d, const void* packed, const float* rays_o, const float* rays_d, int64_t n_rays,
                    float near, float far, const float* near_rays, const float* far_rays, int n_iters, float* d_pred,
                    float* pts, uint8_t* mask, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_sdf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(n_rays >= 0 && n_iters >= 0, NR_ERR_ARG, "nr_sphere_trace: negative n_rays / n_iters");
  if (n_rays == 0) return NR_OK;  // empty tensors may carry null data pointers
  NR_REQUIRE(packed && rays_o && rays_d && d_pred && pts && mask, NR_ERR_ARG, "nr_sphere_trace: null argument");
  NR_REQUIRE(n_rays < (int64_t)1 << 31, NR_ERR_UNSUPPORTED, "nr_sphere_trace: n_rays must be < 2^31");
  const TracePlan pl = trace_plan(n_rays);
  NR_REQUIRE(workspace && workspace_bytes >= pl.total, NR_ERR_WORKSPACE, "nr_sphere_trace: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  int* idx[2] = {(int*)(ws + pl.o_idx0), (int*)(ws + pl.o_idx1)};
  float* qp = (float*)(ws + pl.o_pts);
  float* sv = (float*)(ws + pl.o_sv);
  int* cnt = (int*)(ws + pl.o_cnt);  // cnt[0], cnt[1]: active counts of the two lists
  const SdfLayout SL = sdf_layout(*d);
  {
    ProfScope prof("trace_init", (double)n_rays, st);
    hipLaunchKernelGGL(trace_init, grid1(n_rays), dim3(256), 0, st, rays_o, rays_d, n_rays, near, near_rays, d_pred,
                       mask, idx[0], qp);
  }
  NR_HIP_CHECK(hipGetLastError());
  NR_HIP_CHECK(hipMemsetD32Async((hipDeviceptr_t)cnt, (int)n_rays, 1, st));
  for (int it = 0; it < n_iters; ++it) {
    const int cur = it & 1, nxt = cur ^ 1;
    // the query points of list `cur` are contiguous in qp[0, cnt[cur]); the MLP reads the count on device
    if ((rc = launch_sdf(SL, packed, qp, n_rays, sv, nullptr, nullptr, d->multires, nullptr, 0, st, cnt + cur, 1)))
      return rc;
    const int append = it + 1 < n_iters;
    NR_HIP_CHECK(hipMemsetAsync(cnt + nxt, 0, sizeof(int), st));
    {
      ProfScope prof("trace_step", (double)n_rays, st);
      hipLaunchKernelGGL(trace_step, grid1(n_rays), dim3(256), 0, st, rays_o, rays_d, cnt + cur, idx[cur], sv, far,
                         far_rays, d_pred, mask, cnt + nxt, idx[nxt], qp, append);
    }
    NR_HIP_CHECK(hipGetLastError());
  }
  hipLaunchKernelGGL(trace_final, grid1(n_rays), dim3(256), 0, st, rays_o, rays_d, n_rays, d_pred, pts);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

int nr_normalize3(const float* v, int64_t n, float* out, void* stream) {
  NR_REQUIRE(n >= 0, NR_ERR_ARG, "nr_normalize3: negative n");
  if (n == 0) return NR_OK;
  NR_REQUIRE(v && out, NR_ERR_ARG, "nr_normalize3: null argument");
  hipLaunchKernelGGL(normalize3_kernel, grid1(n), dim3(256), 0, (hipStream_t)stream, v, n, out);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

int nr_surface_finish(float* rgb, const float* nablas, const uint8_t* mask, int64_t n, float* normals, void* stream) {
  NR_REQUIRE(n >= 0, NR_ERR_ARG, "nr_surface_finish: negative n");
  if (n == 0) return NR_OK;
  NR_REQUIRE(rgb && nablas && mask, NR_ERR_ARG, "nr_surface_finish: null argument");
  hipLaunchKernelGGL(surface_finish, grid1(n), dim3(256), 0, (hipStream_t)stream, rgb, nablas, mask, n, normals);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

size_t nr_root_find_workspace_bytes(int64_t n_rays, int N_steps) {
  return N_steps >= 2 ? root_plan(n_rays, N_steps).total : 0;
}

int nr_root_find(const NrSdfDesc* d, const void* packed, const float* rays_o, const float* rays_d, int64_t n_rays,
                 float near, float far, const float* near_rays, const float* far_rays, int N_steps,
                 const float* t_march, int N_secant_steps, int no_secant, float logit_tau, int fill_inf,
                 int full_march, float* d_pred, float* pts, uint8_t* mask, uint8_t* mask_sign_change, void* workspace,
                 size_t workspace_bytes, void* stream) {
  int rc = check_sdf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(n_rays >= 0 && N_steps >= 2 && N_secant_steps >= 0, NR_ERR_ARG,
             "nr_root_find: need n_rays >= 0, N_steps >= 2, N_secant_steps >= 0");
  if (n_rays == 0) return NR_OK;
  NR_REQUIRE(packed && rays_o && rays_d && t_march && d_pred && pts && mask, NR_ERR_ARG, "nr_root_find: null argument");
  const RootPlan pl = root_plan(n_rays, N_steps);
  NR_REQUIRE(workspace && workspace_bytes >= pl.total, NR_ERR_WORKSPACE, "nr_root_find: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)workspace;
  auto F = [&](size_t o) { return (float*)(ws + o); };
  const SdfLayout SL = sdf_layout(*d);
  for (int64_t r0 = 0; r0 < n_rays; r0 += pl.Rc) {
    const int R = (int)((n_rays - r0) < pl.Rc ? (n_rays - r0) : pl.Rc);
    UniChunk c{};
    c.R = R;
    c.N_steps = N_steps;
    c.logit_tau = logit_tau;
    c.no_secant = no_secant;
    c.ro = F(pl.o_ro); c.rd = F(pl.o_rd); c.near = F(pl.o_near); c.far = F(pl.o_far);
    c.pts_m = F(pl.o_ptsm); c.sm = F(pl.o_sm); c.sec = F(pl.o_sec); c.pts_s = F(pl.o_ptss); c.ss = F(pl.o_ss);
    c.t_march = t_march;
    const dim3 blk(64), grd((R + 63) / 64);
    {
      ProfScope prof("root_prologue", (double)R, st);
      hipLaunchKernelGGL(rf_prologue, grd, blk, 0, st, c, rays_o + r0 * 3, rays_d + r0 * 3, near, far,
                         near_rays ? near_rays + r0 : nullptr, far_rays ? far_rays + r0 : nullptr);
    }
    NR_HIP_CHECK(hipGetLastError());
    // the march in chunks of kMarchK steps over the rays still without a sign change (uni_root reads a
    // ray's march only up to its first crossing); full_march: every step of every ray in one launch
    if ((rc = run_march(SL, packed, d->multires, c, full_march != 0, (int*)(ws + pl.o_act0), (int*)(ws + pl.o_act1),
                        (int*)(ws + pl.o_acnt), F(pl.o_ptsc), F(pl.o_sc), st)))
      return rc;
    hipLaunchKernelGGL(uni_root, grd, blk, 0, st, c);
    NR_HIP_CHECK(hipGetLastError());
    for (int i = 0; i < (no_secant ? 0 : N_secant_steps); ++i) {
      if ((rc = launch_sdf(SL, packed, c.pts_s, R, c.ss, nullptr, nullptr, d->multires, nullptr, 0, st))) return rc;
      hipLaunchKernelGGL(uni_secant, grd, blk, 0, st, c, (int)(i == N_secant_steps - 1));
      NR_HIP_CHECK(hipGetLastError());
    }
    hipLaunchKernelGGL(rf_finish, grd, blk, 0, st, c, r0, d_pred, pts, mask, mask_sign_change, fill_inf);
    NR_HIP_CHECK(hipGetLastError());
  }
  return NR_OK;
}

size_t nr_sdf_grid_workspace_bytes(int64_t n_points) { return a256((size_t)(n_points > 0 ? n_points : 1) * 12); }

int nr_sdf_grid(const NrSdfDesc* d, const void* packed, double volume_size, int64_t N, int64_t i0, int64_t n,
                float* sdf, void* workspace, size_t workspace_bytes, void* stream) {
  int rc = check_sdf_desc(d);
  if (rc) return rc;
  NR_REQUIRE(N >= 2 && N <= 2097151 && i0 >= 0 && n >= 0 && i0 + n <= N * N * N, NR_ERR_ARG,
             "nr_sdf_grid: bad argument (need 2 <= N < 2^21 and [i0, i0+n) inside the N^3 grid)");
  if (n == 0) return NR_OK;
  NR_REQUIRE(packed && sdf, NR_ERR_ARG, "nr_sdf_grid: null argument");
  NR_REQUIRE(workspace && workspace_bytes >= (size_t)n * 12, NR_ERR_WORKSPACE, "nr_sdf_grid: workspace too small");
  hipStream_t st = (hipStream_t)stream;
  float* pts = (float*)workspace;
  const double step = volume_size / (double)(N - 1), origin = -volume_size / 2.0;
  {
    ProfScope prof("grid_points", (double)n, st);
    hipLaunchKernelGGL(grid_points_kernel, grid1(n), dim3(256), 0, st, N, step, origin, i0, n, pts);
  }
  NR_HIP_CHECK(hipGetLastError());
  return launch_sdf(sdf_layout(*d), packed, pts, n, sdf, nullptr, nullptr, d->multires, nullptr, 0, st);
}

}  // extern "C"
