// neurecon_amd — UNISURF render path for gfx950 (models/frameworks/unisurf.py:62-283 and
// models/ray_casting.py:11-160, render mode: perturb=False, secant root finding).
//
// One thread per ray for the march / secant / sampling / compositing steps (sample-major state,
// coalesced); the SDF and radiance MLPs run in the fused MFMA kernels.  The reference feeds
// F.normalize(nablas) with torch's default dim=1 to the radiance net (unisurf.py:36): for batched
// renders that normalises each gradient component over a whole batchify_query chunk of points
// (train_util.py:23-71), which is reproduced here with a per-window fp64 reduction.
#include "nr_common.h"
#include "nr_mlp.h"
#include "nr_unisurf.h"

namespace nr {
namespace {

__device__ __forceinline__ float norm3f(float x, float y, float z) {
  return norm3_ref(x, y, z);
}

// d_proposal = near * (1 - t) + far * t (ray_casting.py:79)
__device__ __forceinline__ float lerp_ref(float a, float b, float t) { return fadd(fmul(a, fsub(1.0f, t)), fmul(b, t)); }

// d_pred = -f_low * (d_high - d_low) / (f_high - f_low) + d_low (ray_casting.py:15, :29)
__device__ __forceinline__ float secant(float d_lo, float f_lo, float d_hi, float f_hi) {
  return fadd(fdiv(fmul(-f_lo, fsub(d_hi, d_lo)), fsub(f_hi, f_lo)), d_lo);
}

enum { kDLo, kFLo, kDHi, kFHi, kDPred, kHit, kCross, kFree, kSec };

}  // namespace

// normalised directions, near/far on the sphere of interest (rend_util.py:167-185), the too-close
// threshold (unisurf.py:128) and the N_steps march points (ray_casting.py:74-83)
__global__ void uni_prologue(UniChunk c, const float* __restrict__ rays_o, const float* __restrict__ rays_d) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const float ox = rays_o[r * 3 + 0], oy = rays_o[r * 3 + 1], oz = rays_o[r * 3 + 2];
  float dx = rays_d[r * 3 + 0], dy = rays_d[r * 3 + 1], dz = rays_d[r * 3 + 2];
  const float nn = fmaxf(norm3f(dx, dy, dz), 1e-12f);
  dx = fdiv(dx, nn);
  dy = fdiv(dy, nn);
  dz = fdiv(dz, nn);
  c.ro[r * 3 + 0] = ox; c.ro[r * 3 + 1] = oy; c.ro[r * 3 + 2] = oz;
  c.rd[r * 3 + 0] = dx; c.rd[r * 3 + 1] = dy; c.rd[r * 3 + 2] = dz;
  const float mid = -fadd(fadd(fmul(ox, dx), fmul(oy, dy)), fmul(oz, dz));
  float nr = fmaxf(fsub(mid, c.r_interest), 0.0f);
  float fr = fmaxf(fadd(mid, c.r_interest), c.r_interest);
  if (!__builtin_isnan(c.near_bypass)) nr = c.near_bypass;
  if (!__builtin_isnan(c.far_bypass)) fr = c.far_bypass;
  c.near[r] = nr;
  c.far[r] = fr;
  c.thr[r] = fadd(nr, fmul(fsub(fr, nr), c.too_close));
  for (int i = 0; i < c.N_steps; ++i) {
    const float d = lerp_ref(nr, fr, c.t_march[i]);
    const int64_t q = (int64_t)i * c.R + r;
    c.pts_m[q * 3 + 0] = fadd(ox, fmul(d, dx));
    c.pts_m[q * 3 + 1] = fadd(oy, fmul(d, dy));
    c.pts_m[q * 3 + 2] = fadd(oz, fmul(d, dz));
  }
}

// standalone root_finding_surface_points (ray_casting.py:35-160, used by surface_render): rays as
// given (already normalised by the caller), scalar or per-ray near / far (:70-73), march points
// sample-major
__global__ void rf_prologue(UniChunk c, const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                            float near_s, float far_s, const float* __restrict__ near_rays,
                            const float* __restrict__ far_rays) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const float near = near_rays ? near_rays[r] : near_s, far = far_rays ? far_rays[r] : far_s;
  const float ox = rays_o[r * 3 + 0], oy = rays_o[r * 3 + 1], oz = rays_o[r * 3 + 2];
  const float dx = rays_d[r * 3 + 0], dy = rays_d[r * 3 + 1], dz = rays_d[r * 3 + 2];
  c.ro[r * 3 + 0] = ox; c.ro[r * 3 + 1] = oy; c.ro[r * 3 + 2] = oz;
  c.rd[r * 3 + 0] = dx; c.rd[r * 3 + 1] = dy; c.rd[r * 3 + 2] = dz;
  c.near[r] = near;
  c.far[r] = far;
  for (int i = 0; i < c.N_steps; ++i) {
    const float d = lerp_ref(near, far, c.t_march[i]);
    const int64_t q = (int64_t)i * c.R + r;
    // p_proposal = rays_o + d_proposal * rays_d (ray_casting.py:82)
    c.pts_m[q * 3 + 0] = fadd(ox, fmul(d, dx));
    c.pts_m[q * 3 + 1] = fadd(oy, fmul(d, dy));
    c.pts_m[q * 3 + 2] = fadd(oz, fmul(d, dz));
  }
}

// outputs of root_finding_surface_points (ray_casting.py:142-160): d = secant estimate on hits,
// inf (fill_inf) or far elsewhere, 0 when the first sample is occupied; points o + d*dir on hits, 1
// elsewhere; mask = hit; mask_sign_change = any crossing
__global__ void rf_finish(UniChunk c, int64_t ray0, float* __restrict__ d_out, float* __restrict__ pts,
                          uint8_t* __restrict__ mask, uint8_t* __restrict__ msc, int fill_inf) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const float* s = c.sec + (int64_t)r * kSec;
  const bool hit = s[kHit] != 0.0f;
  const float dp = s[kDPred];
  float d = hit ? dp : (fill_inf ? __builtin_inff() : c.far[r]);
  if (s[kFree] == 0.0f) d = 0.0f;
  const int64_t o = ray0 + r;
  d_out[o] = d;
#pragma unroll
  for (int k = 0; k < 3; ++k) pts[o * 3 + k] = hit ? fadd(c.ro[r * 3 + k], fmul(dp, c.rd[r * 3 + k])) : 1.0f;
  mask[o] = hit ? 1 : 0;
  if (msc) msc[o] = s[kCross] != 0.0f ? 1 : 0;
}

// first sign change of the march (ray_casting.py:89-131) and the first secant estimate
__global__ void uni_root(UniChunk c) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const int N = c.N_steps;
  const float tau = c.logit_tau;
  float v0 = fsub(c.sm[r], tau);
  const bool first_free = v0 > 0.0f;
  int idx = -1;
  float vi = v0, vn = 0.0f;
  for (int i = 0; i + 1 < N; ++i) {
    vn = fsub(c.sm[(int64_t)(i + 1) * c.R + r], tau);
    if (fmul(vi, vn) < 0.0f) {  // torch.sign(v_i * v_{i+1}) == -1: the earliest one wins the min
      idx = i;
      break;
    }
    vi = vn;
  }
  const bool crossing = idx >= 0;
  const bool hit = crossing && vi > 0.0f && first_free;
  float* s = c.sec + (int64_t)r * kSec;
  s[kHit] = hit ? 1.0f : 0.0f;
  s[kCross] = crossing ? 1.0f : 0.0f;
  s[kFree] = first_free ? 1.0f : 0.0f;
  float dp = 1.0f;
  if (hit) {
    const float nr = c.near[r], fr = c.far[r];
    const int i1 = idx + 1 < N ? idx + 1 : N - 1;
    const float d_hi = lerp_ref(nr, fr, c.t_march[idx]), f_hi = vi;
    const float d_lo = lerp_ref(nr, fr, c.t_march[i1]), f_lo = vn;
    s[kDLo] = d_lo; s[kFLo] = f_lo; s[kDHi] = d_hi; s[kFHi] = f_hi;
    if (!c.no_secant) dp = secant(d_lo, f_lo, d_hi, f_hi);
  }
  s[kDPred] = dp;
  c.pts_s[r * 3 + 0] = fadd(c.ro[r * 3 + 0], fmul(dp, c.rd[r * 3 + 0]));
  c.pts_s[r * 3 + 1] = fadd(c.ro[r * 3 + 1], fmul(dp, c.rd[r * 3 + 1]));
  c.pts_s[r * 3 + 2] = fadd(c.ro[r * 3 + 2], fmul(dp, c.rd[r * 3 + 2]));
}

// chunked march (kMarchK): after steps [s0, s1) are evaluated, the rays without a sign change among the
// pairs (i, i + 1) with i + 1 in [max(s0, 1), s1) -- uni_root's test, in its order -- and steps left
// are appended to act_out (order free: each ray's points go back to its own slots)
__global__ void uni_march_scan(UniChunk c, int s0, int s1, const int* __restrict__ act_in,
                               const int* __restrict__ n_in, int* __restrict__ act_out, int* __restrict__ n_out) {
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  const int n = act_in ? *n_in : c.R;
  if (j >= n) return;
  const int r = act_in ? act_in[j] : j;
  const float tau = c.logit_tau;
  const int i0 = s0 > 0 ? s0 - 1 : 0;
  float vi = fsub(c.sm[(int64_t)i0 * c.R + r], tau);
  for (int i = i0; i + 1 < s1; ++i) {
    const float vn = fsub(c.sm[(int64_t)(i + 1) * c.R + r], tau);
    if (fmul(vi, vn) < 0.0f) return;  // its first crossing: uni_root stops here
    vi = vn;
  }
  if (s1 < c.N_steps) act_out[atomicAdd(n_out, 1)] = r;
}

// steps [s0, s0 + K) of the active rays -> compacted points q = j K + t
__global__ void uni_march_gather(UniChunk c, int s0, int K, const int* __restrict__ act, const int* __restrict__ n,
                                 float* __restrict__ pts) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)*n * K) return;
  const int j = (int)(q / K), t = (int)(q - (int64_t)j * K);
  const int64_t src = (int64_t)(s0 + t) * c.R + act[j];
  pts[q * 3 + 0] = c.pts_m[src * 3 + 0];
  pts[q * 3 + 1] = c.pts_m[src * 3 + 1];
  pts[q * 3 + 2] = c.pts_m[src * 3 + 2];
}

// ... and their sdf back into the march array
__global__ void uni_march_scatter(UniChunk c, int s0, int K, const int* __restrict__ act, const int* __restrict__ n,
                                  const float* __restrict__ v) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)*n * K) return;
  const int j = (int)(q / K), t = (int)(q - (int64_t)j * K);
  c.sm[(int64_t)(s0 + t) * c.R + act[j]] = v[q];
}

// one secant step (ray_casting.py:17-29) given f at the current estimate
__global__ void uni_secant(UniChunk c, int last) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  float* s = c.sec + (int64_t)r * kSec;
  if (s[kHit] == 0.0f) return;
  const float dp = s[kDPred];
  const float fm = fsub(c.ss[r], c.logit_tau);
  if (fm < 0.0f) {
    s[kDLo] = dp;
    s[kFLo] = fm;
  } else {
    s[kDHi] = dp;
    s[kFHi] = fm;
  }
  const float dn = secant(s[kDLo], s[kFLo], s[kDHi], s[kFHi]);
  s[kDPred] = dn;
  if (!last) {
    c.pts_s[r * 3 + 0] = fadd(c.ro[r * 3 + 0], fmul(dn, c.rd[r * 3 + 0]));
    c.pts_s[r * 3 + 1] = fadd(c.ro[r * 3 + 1], fmul(dn, c.rd[r * 3 + 1]));
    c.pts_s[r * 3 + 2] = fadd(c.ro[r * 3 + 2], fmul(dn, c.rd[r * 3 + 2]));
  }
}

// surface outputs, interval + free-space samples, sorted (unisurf.py:135-203)
__global__ void uni_samples(UniChunk c, UniOut o) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const float* s = c.sec + (int64_t)r * kSec;
  const bool hit = s[kHit] != 0.0f, crossing = s[kCross] != 0.0f, first_free = s[kFree] != 0.0f;
  const float dpred = s[kDPred];
  const float nr = c.near[r], fr = c.far[r];
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  float dout = hit ? dpred : fr;  // fill_inf=False (unisurf.py:143)
  if (!first_free) dout = 0.0f;
  const int64_t rg = o.ray0 + r;
  if (o.surface_points) {
    o.surface_points[rg * 3 + 0] = hit ? fadd(ox, fmul(dpred, dx)) : 1.0f;
    o.surface_points[rg * 3 + 1] = hit ? fadd(oy, fmul(dpred, dy)) : 1.0f;
    o.surface_points[rg * 3 + 2] = hit ? fadd(oz, fmul(dpred, dz)) : 1.0f;
  }
  if (o.mask_surface) o.mask_surface[rg] = hit ? 1 : 0;
  const float dc = fmaxf(fminf(dout, fr), nr);
  if (o.depth_surface) o.depth_surface[rg] = dc;
  const float d_up = fminf(fadd(dc, c.interval), fr);
  const float d_lo = fmaxf(fsub(dc, c.interval), nr);
  float d_lo2 = fmaxf(d_lo, c.thr[r]);
  if (!crossing) d_lo2 = fr;
  if (d_lo2 < 1e-10f) d_lo2 = fr;
  // merge the two (ascending) runs; an insertion pass below repairs rounding-level disorder
  const int nf = c.N_free, nq = c.N_query, P = c.P;
  const int64_t R = c.R;
  float* da = c.d_all + r;
  int jf = 0, jq = 0;
  // sample j of a run on [a, b]: the linspace point, or (perturb) lower + (upper - lower) * u with the
  // bin edges of linspace(0, 1, n+1); both runs stay ascending
  auto run = [&](float a, float b, const float* t, const float* u, int j) {
    const float lo = lerp_ref(a, b, t[j]);
    if (!u) return lo;
    const float hi = lerp_ref(a, b, t[j + 1]);
    return fadd(lo, fmul(fsub(hi, lo), u[j]));
  };
  const float* uq = c.u_q ? c.u_q + (int64_t)r * nq : nullptr;
  const float* uf = c.u_f ? c.u_f + (int64_t)r * nf : nullptr;
  float vf = nf > 0 ? run(nr, d_lo2, c.t_free, uf, 0) : 0.0f;
  float vq = nq > 0 ? run(d_lo, d_up, c.t_query, uq, 0) : 0.0f;
  for (int k = 0; k < P; ++k) {
    const bool take_f = jq >= nq || (jf < nf && vf <= vq);
    if (take_f) {
      da[k * R] = vf;
      ++jf;
      if (jf < nf) vf = run(nr, d_lo2, c.t_free, uf, jf);
    } else {
      da[k * R] = vq;
      ++jq;
      if (jq < nq) vq = run(d_lo, d_up, c.t_query, uq, jq);
    }
  }
  for (int k = 1; k < P; ++k) {
    const float v = da[k * R];
    int j = k - 1;
    while (j >= 0 && da[j * R] > v) {
      da[(j + 1) * R] = da[j * R];
      --j;
    }
    da[(j + 1) * R] = v;
  }
  for (int k = 0; k < P; ++k) {
    const float d = da[k * R];
    const int64_t q = k * R + r;
    c.pts_f[q * 3 + 0] = fadd(ox, fmul(dx, d));
    c.pts_f[q * 3 + 1] = fadd(oy, fmul(dy, d));
    c.pts_f[q * 3 + 2] = fadd(oz, fmul(dz, d));
  }
}

// window of the point (row-relative ray rg, sample s)
__device__ __forceinline__ int64_t uni_window(const UniChunk& c, int64_t rg, int64_t s) {
  const int64_t k = rg / c.rc_rays;
  return k * c.nw_full + ((rg - k * c.rc_rays) * c.P + s) / c.netchunk;
}

// sum of squares of every nabla component over the part of each F.normalize window that lies in
// this chunk, in two deterministic stages (r06; r05 ran one 256-thread block per window, 0.55 ms for
// config (e)'s single 393 k-point window): uni_window_ss_part sums slice g of the window's points in each
// of kWinSlices blocks (grid: windows x rows x slices; a block tree-reduces its threads' fp64 sums),
// uni_window_ss_sum adds the slices' partials in slice order.  Windows the chunk does not touch get
// zeros.
__device__ __forceinline__ void uni_window_range(const UniChunk& c, int64_t w, int64_t& k0, int64_t& q0, int64_t& q1) {
  const int64_t P = c.P, k = w / c.nw_full, j = w % c.nw_full;
  k0 = k * c.rc_rays;  // first ray of reference chunk k
  const int64_t rays_k = min(c.rc_rays, c.row_rays - k0);
  q0 = j * c.netchunk;
  q1 = min((j + 1) * c.netchunk, rays_k * P);
  q0 = max(q0, (c.row_ray0 - k0) * P);           // points of this chunk's rays only
  q1 = min(q1, (c.row_ray0 + c.nloc - k0) * P);
}
__global__ void uni_window_ss_part(UniChunk c) {
  __shared__ double red[3][256];
  const int64_t w = blockIdx.x, b = blockIdx.y, g = blockIdx.z, t = threadIdx.x;
  const int64_t P = c.P;
  int64_t k0, q0, q1;
  uni_window_range(c, w, k0, q0, q1);
  const int64_t len = q1 > q0 ? q1 - q0 : 0;
  const int64_t qa = q0 + len * g / kWinSlices, qb = q0 + len * (g + 1) / kWinSlices;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0;
  for (int64_t q = qa + t; q < qb; q += blockDim.x) {
    const int64_t rl = k0 + q / P - c.row_ray0, s = q % P;  // ray within this chunk's row
    const int64_t p = s * c.R + b * c.nloc + rl;            // sample-major point index
    const double x = c.nab_f[p * 3 + 0], y = c.nab_f[p * 3 + 1], z = c.nab_f[p * 3 + 2];
    a0 += x * x;
    a1 += y * y;
    a2 += z * z;
  }
  red[0][t] = a0;
  red[1][t] = a1;
  red[2][t] = a2;
  __syncthreads();
  for (int o = blockDim.x / 2; o > 0; o >>= 1) {
    if (t < o) {
      red[0][t] += red[0][t + o];
      red[1][t] += red[1][t + o];
      red[2][t] += red[2][t + o];
    }
    __syncthreads();
  }
  if (t == 0) {
    double* o = c.wsp + ((b * c.nw_row + w) * kWinSlices + g) * 3;
    o[0] = red[0][0];
    o[1] = red[1][0];
    o[2] = red[2][0];
  }
}
__global__ void uni_window_ss_sum(UniChunk c) {
  const int64_t w = blockIdx.x, b = blockIdx.y;
  const int t = threadIdx.x;
  if (t >= 3) return;
  const double* pp = c.wsp + (b * c.nw_row + w) * kWinSlices * 3 + t;
  double acc = 0.0;
  for (int g = 0; g < kWinSlices; ++g) acc += pp[g * 3];
  c.wss[(b * c.nw_row + w) * 3 + t] = acc;
}

// normals fed to the radiance net: F.normalize(nablas) (unisurf.py:36). mode 0: per point (an
// unbatched call normalises over the xyz dim); mode 1: per window and component.
__global__ void uni_normalize(UniChunk c, int mode) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t n = (int64_t)c.R * c.P;
  if (p >= n) return;
  const float x = c.nab_f[p * 3 + 0], y = c.nab_f[p * 3 + 1], z = c.nab_f[p * 3 + 2];
  if (mode == 0) {
    const float d = fmaxf(norm3f(x, y, z), 1e-12f);
    c.nrm_f[p * 3 + 0] = fdiv(x, d);
    c.nrm_f[p * 3 + 1] = fdiv(y, d);
    c.nrm_f[p * 3 + 2] = fdiv(z, d);
  } else {
    const int64_t rf = p % c.R, s = p / c.R;
    const int64_t b = rf / c.nloc, rg = c.row_ray0 + rf % c.nloc;
    const double* ws = c.wss + (b * c.nw_row + uni_window(c, rg, s)) * 3;
    c.nrm_f[p * 3 + 0] = fdiv(x, fmaxf((float)sqrt(ws[0]), 1e-12f));
    c.nrm_f[p * 3 + 1] = fdiv(y, fmaxf((float)sqrt(ws[1]), 1e-12f));
    c.nrm_f[p * 3 + 2] = fdiv(z, fmaxf((float)sqrt(ws[2]), 1e-12f));
  }
}

// occupancy-logit alpha compositing (unisurf.py:53-62, :206-244)
__global__ void uni_composite(UniChunk c, UniOut o, int calc_normal, int white_bkgd) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const int P = c.P;
  const int64_t R = c.R;
  const int64_t rg = o.ray0 + r;
  double T = 1.0, a_acc = 0.0, a0 = 0.0, a1 = 0.0, a2 = 0.0, n0 = 0.0, n1 = 0.0, n2 = 0.0;
  for (int i = 0; i < P; ++i) {
    const int64_t q = i * R + r;
    const float lg = c.sdf_f[q];
    const float odds = expf(-lg);
    const float alpha = fdiv(odds, fadd(1.0f, odds));
    const float w = fmul(alpha, (float)T);
    T *= (double)fadd(fsub(1.0f, alpha), 1e-10f);
    a0 += (double)fmul(w, c.rad_f[q * 3 + 0]);
    a1 += (double)fmul(w, c.rad_f[q * 3 + 1]);
    a2 += (double)fmul(w, c.rad_f[q * 3 + 2]);
    a_acc += (double)w;
    const float nx = c.nab_f[q * 3 + 0], ny = c.nab_f[q * 3 + 1], nz = c.nab_f[q * 3 + 2];
    if (calc_normal) {
      const float d = fmaxf(norm3f(nx, ny, nz), 1e-12f);
      n0 += (double)fmul(fdiv(nx, d), w);
      n1 += (double)fmul(fdiv(ny, d), w);
      n2 += (double)fmul(fdiv(nz, d), w);
    }
    if (o.alpha) o.alpha[rg * P + i] = alpha;
    if (o.weights) o.weights[rg * P + i] = w;
    if (o.sdf) o.sdf[rg * P + i] = lg;
    if (o.nablas) {
      o.nablas[(rg * P + i) * 3 + 0] = nx;
      o.nablas[(rg * P + i) * 3 + 1] = ny;
      o.nablas[(rg * P + i) * 3 + 2] = nz;
    }
    if (o.radiance) {
      o.radiance[(rg * P + i) * 3 + 0] = c.rad_f[q * 3 + 0];
      o.radiance[(rg * P + i) * 3 + 1] = c.rad_f[q * 3 + 1];
      o.radiance[(rg * P + i) * 3 + 2] = c.rad_f[q * 3 + 2];
    }
  }
  const float accf = (float)a_acc;
  const float denom = fadd(accf, 1e-10f);
  double dep = 0.0;
  T = 1.0;
  for (int i = 0; i < P; ++i) {  // second pass: weights normalised by their float sum
    const int64_t q = i * R + r;
    const float odds = expf(-c.sdf_f[q]);
    const float alpha = fdiv(odds, fadd(1.0f, odds));
    const float w = fmul(alpha, (float)T);
    T *= (double)fadd(fsub(1.0f, alpha), 1e-10f);
    dep += (double)fmul(fdiv(w, denom), c.d_all[q]);
  }
  float q0 = (float)a0, q1 = (float)a1, q2 = (float)a2;
  if (white_bkgd) {
    const float bg = fsub(1.0f, accf);
    q0 = fadd(q0, bg); q1 = fadd(q1, bg); q2 = fadd(q2, bg);
  }
  o.rgb[rg * 3 + 0] = q0;
  o.rgb[rg * 3 + 1] = q1;
  o.rgb[rg * 3 + 2] = q2;
  o.depth[rg] = (float)dep;
  o.acc[rg] = accf;
  if (calc_normal && o.normals) {
    o.normals[rg * 3 + 0] = (float)n0;
    o.normals[rg * 3 + 1] = (float)n1;
    o.normals[rg * 3 + 2] = (float)n2;
  }
}

// ---------------------------------------------------------------------------------------------
// workspace plan and chunking
// ---------------------------------------------------------------------------------------------
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

static constexpr int64_t kUniMaxChunk = 65536;

// rays per internal chunk: in window mode (batched call) a chunk never straddles a normalisation
// window, i.e. it is the reference's ray chunk (rayschunk) or a whole number of windows of it
int64_t unisurf_chunk_rays(const NrUnisurfArgs& a) {
  const int64_t P = a.N_query + a.N_freespace;
  if (a.normal_mode == 1 && a.shard_row_rays > 0)  // a multi-GPU shard is one chunk
    return a.n_rays <= kUniMaxChunk ? (a.n_rays > 0 ? a.n_rays : 1) : -1;
  const int64_t per_b = a.rays_per_batch > 0 ? a.rays_per_batch : a.n_rays;
  if (a.normal_mode == 1) {
    const int64_t rc = a.rayschunk < per_b ? a.rayschunk : per_b;
    if (rc <= kUniMaxChunk) return rc > 0 ? rc : 1;
    if (a.netchunk % P != 0) return -1;
    const int64_t rw = a.netchunk / P;  // rays per window
    const int64_t k = kUniMaxChunk / rw;
    return k > 0 ? k * rw : -1;
  }
  return a.n_rays < kUniMaxChunk ? (a.n_rays > 0 ? a.n_rays : 1) : kUniMaxChunk;
}

void unisurf_windows(const NrUnisurfArgs& a, int64_t& rc_rays, int64_t& nw_full, int64_t& nw_row) {
  const int64_t P = a.N_query + a.N_freespace;
  const int64_t row = a.shard_row_rays > 0 ? a.shard_row_rays : (a.rays_per_batch > 0 ? a.rays_per_batch : a.n_rays);
  const int64_t nc = a.netchunk > 0 ? a.netchunk : 1;
  rc_rays = a.rayschunk > 0 ? (a.rayschunk < row ? a.rayschunk : row) : (row > 0 ? row : 1);
  if (rc_rays < 1) rc_rays = 1;
  nw_full = (rc_rays * P + nc - 1) / nc;
  nw_row = ((row + rc_rays - 1) / rc_rays) * nw_full;
  if (nw_row < 1) nw_row = 1;
}

UniPlan unisurf_plan(const NrUnisurfArgs& a, int64_t Rc) {
  UniPlan p{};
  const int P = a.N_query + a.N_freespace;
  p.Rc = Rc;
  int64_t rc_rays = 1, nw_full = 1, nw_row = 1;
  if (a.normal_mode == 1) unisurf_windows(a, rc_rays, nw_full, nw_row);
  p.max_windows = nw_row;  // one batch row's windows (internal chunks never span rows)
  size_t off = 0;
  auto take = [&](size_t words) { size_t o = off; off = align_up(off + words * 4); return o; };
  p.o_ro = take(Rc * 3);
  p.o_rd = take(Rc * 3);
  p.o_near = take(Rc);
  p.o_far = take(Rc);
  p.o_thr = take(Rc);
  p.o_ptsm = take((size_t)a.N_steps * Rc * 3);
  p.o_sm = take((size_t)a.N_steps * Rc);
  p.o_sec = take((size_t)Rc * 9);
  p.o_ptss = take(Rc * 3);
  p.o_ss = take(Rc);
  p.o_dall = take((size_t)P * Rc);
  p.o_ptsf = take((size_t)P * Rc * 3);
  p.o_sdff = take((size_t)P * Rc);
  p.o_nabf = take((size_t)P * Rc * 3);
  p.o_featf = take((size_t)P * Rc * 256);
  p.o_nrmf = take((size_t)P * Rc * 3);
  p.o_radf = take((size_t)P * Rc * 3);
  p.o_wss = take((size_t)p.max_windows * 6);
  // a multi-GPU shard renders all its batch rows in one chunk (nr_unisurf_render), internal chunks one row
  const int64_t nloc = a.rays_per_batch > 0 ? a.rays_per_batch : (a.n_rays > 0 ? a.n_rays : 1);
  const int64_t rows = (a.normal_mode == 1 && a.shard_row_rays > 0) ? (a.n_rays + nloc - 1) / nloc : 1;
  p.o_wsp = take((size_t)(rows > 0 ? rows : 1) * p.max_windows * kWinSlices * 6);
  p.o_act0 = take(Rc);
  p.o_act1 = take(Rc);
  p.o_acnt = take(2);
  p.o_ptsc = take((size_t)kMarchK * Rc * 3);
  p.o_sc = take((size_t)kMarchK * Rc);
  p.o_mlp = off;
  p.total = off + nr_mlp_workspace_bytes(1);
  return p;
}

int run_march(const SdfLayout& SL, const void* packed, int multires, const UniChunk& c, bool full, int* act0,
              int* act1, int* cnt, float* ptsc, float* sc, hipStream_t st) {
  const int R = c.R;
  const dim3 blk(64), grd((R + 63) / 64);
  const int N = c.N_steps, K0 = (full || N < kMarchK) ? N : kMarchK;
  int rc;
  if ((rc = launch_sdf(SL, packed, c.pts_m, (int64_t)K0 * R, c.sm, nullptr, nullptr, multires, nullptr, 0, st)))
    return rc;
  if (K0 == N) return NR_OK;
  int* act[2] = {act0, act1};
  NR_HIP_CHECK(hipMemsetAsync(cnt, 0, 2 * sizeof(int), st));
  hipLaunchKernelGGL(uni_march_scan, grd, blk, 0, st, c, 0, K0, nullptr, nullptr, act[0], cnt);
  NR_HIP_CHECK(hipGetLastError());
  int cur = 0;
  for (int s0 = K0; s0 < N; s0 += kMarchK) {
    const int Kc = N - s0 < kMarchK ? N - s0 : kMarchK;
    const dim3 gq((unsigned)(((int64_t)Kc * R + 255) / 256));
    hipLaunchKernelGGL(uni_march_gather, gq, dim3(256), 0, st, c, s0, Kc, act[cur], cnt + cur, ptsc);
    NR_HIP_CHECK(hipGetLastError());
    if ((rc = launch_sdf(SL, packed, ptsc, (int64_t)Kc * R, sc, nullptr, nullptr, multires, nullptr, 0, st, cnt + cur,
                         Kc)))
      return rc;
    hipLaunchKernelGGL(uni_march_scatter, gq, dim3(256), 0, st, c, s0, Kc, act[cur], cnt + cur, sc);
    NR_HIP_CHECK(hipGetLastError());
    NR_HIP_CHECK(hipMemsetAsync(cnt + (cur ^ 1), 0, sizeof(int), st));
    hipLaunchKernelGGL(uni_march_scan, grd, blk, 0, st, c, s0, s0 + Kc, act[cur], cnt + cur, act[cur ^ 1],
                       cnt + (cur ^ 1));
    NR_HIP_CHECK(hipGetLastError());
    cur ^= 1;
  }
  return NR_OK;
}

}  // namespace nr
