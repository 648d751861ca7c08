// neurecon_amd — VolSDF render path for gfx950 (models/frameworks/volsdf.py:16-551, render mode,
// builtin background sphere).
//
// The error-bounded sampler (volsdf.py:77-272) works on per-ray sample lists of up to
// 4*N_samples*(1 + max_iter) entries.  Each list is handled by ONE wave (a 64-thread workgroup)
// with the list resident in LDS: every pass over it (error bound, bisection, inverse CDF) is a
// strided loop with wave-wide fp64 prefix scans, so the scans round like ATen's CPU cumsum
// (accumulate in double, round each prefix to float).  Only rays that are still refining stay
// in the active list, and the SDF MLP launches read the active count from device memory, so no
// host synchronisation is needed between rounds.
#include "nr_common.h"
#include "nr_mlp.h"
#include "nr_volsdf.h"

namespace nr {
namespace {

constexpr int kMaxPerLane = 16;  // N_up, N_importance <= 1024

__device__ __forceinline__ double wave_scan_add(double v) {
  const int l = threadIdx.x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o);
    if (l >= o) v += t;
  }
  return v;
}

__device__ __forceinline__ double wave_scan_mul(double v) {
  const int l = threadIdx.x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double t = __shfl_up(v, o);
    if (l >= o) v *= t;
  }
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// first index with A[idx] >= x / > x (A sorted ascending, LDS)
__device__ __forceinline__ int lower_bound(const float* A, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (A[m] < x) lo = m + 1; else hi = m;
  }
  return lo;
}
__device__ __forceinline__ int upper_bound(const float* A, int n, float x) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if (A[m] <= x) lo = m + 1; else hi = m;
  }
  return lo;
}

// #{k : u[k] <= x} for the (host-computed) torch.linspace(0, 1, N) table u
__device__ __forceinline__ int count_le(const float* __restrict__ u, int N, float x) {
  if (!(x >= u[0])) return 0;
  int g = (int)(fminf(x, 2.0f) * (float)(N - 1)) + 1;
  g = g < 1 ? 1 : (g > N ? N : g);
  while (g < N && u[g] <= x) ++g;
  while (g > 1 && u[g - 1] > x) --g;
  return g;
}

// sdf_to_sigma (volsdf.py:16-35): alpha * (sdf >= 0 ? 0.5 exp(-|sdf|/beta) : 1 - 0.5 exp(-|sdf|/beta))
__device__ __forceinline__ float vs_sigma(float s, float alpha, float beta) {
  const float e = fmul(0.5f, expf(fdiv(-fabsf(s), beta)));
  return fmul(alpha, s >= 0.0f ? e : fsub(1.0f, e));
}

__device__ __forceinline__ void point_at(const VolChunk& c, int r, float d, float& x, float& y, float& z) {
  x = fadd(c.ro[r * 3 + 0], fmul(c.rd[r * 3 + 0], d));
  y = fadd(c.ro[r * 3 + 1], fmul(c.rd[r * 3 + 1], d));
  z = fadd(c.ro[r * 3 + 2], fmul(c.rd[r * 3 + 2], d));
}

__device__ __forceinline__ float norm3(float x, float y, float z) {
  return norm3_ref(x, y, z);
}

// VolSDF.forward_surface (volsdf.py:310-315): min(sdf, r_bg - |x|) with the builtin background
__device__ __forceinline__ float surface_sdf(const VolChunk& c, int r, float d, float s) {
  if (!c.use_bg) return s;
  float x, y, z;
  point_at(c, r, d, x, y, z);
  return fminf(s, fsub(c.r_bg, norm3(x, y, z)));
}

// One error-bound pass (volsdf.py:38-74) over the LDS list (D, S)[0..n): for every interval i the
// callback receives (i, valid, bound_i (NaN -> inf), R_t[i]) -- all 64 lanes call it together.
template <class Fn>
__device__ __forceinline__ void vs_bounds(const float* D, const float* S, int n, float alpha, float beta, Fn&& fn) {
  const int l = threadIdx.x;
  const float c4 = fdiv(alpha, fmul(4.0f, beta));
  double carR = 0.0, carE = 0.0;
  for (int base = 0; base < n - 1; base += 64) {
    const int i = base + l;
    const bool v = i < n - 1;
    float x = 0.0f, err = 0.0f;
    if (v) {
      const float d0 = D[i], d1 = D[i + 1], s0 = S[i], s1 = S[i + 1];
      const float delta = fsub(d1, d0);
      x = fmul(vs_sigma(s0, alpha, beta), delta);
      const float dstar = fmaxf(fmul(0.5f, fsub(fadd(fabsf(s0), fabsf(s1)), delta)), 0.0f);
      err = fmul(fmul(c4, fmul(delta, delta)), expf(fdiv(-dstar, beta)));
    }
    const double sx = wave_scan_add((double)x), se = wave_scan_add((double)err);
    double ex = __shfl_up(sx, 1);
    if (l == 0) ex = 0.0;
    const float Rt = (float)(carR + ex);
    const float E = (float)(carE + se);
    float b = fmul(expf(-Rt), fsub(expf(E), 1.0f));
    if (b != b) b = __builtin_inff();
    fn(i, v, b, Rt);
    carR += __shfl(sx, 63);
    carE += __shfl(se, 63);
    __syncthreads();
  }
}

__device__ float vs_bound_max(const float* D, const float* S, int n, float alpha, float beta) {
  float m = -__builtin_inff();
  vs_bounds(D, S, n, alpha, beta, [&](int, bool v, float b, float) {
    if (v) m = fmaxf(m, b);
  });
  return wave_max(m);
}

// inverse-CDF emission (rend_util.py:266-292 / :302-327): searchsorted(cdf, u, right=False) maps
// u in (cdf_i, cdf_{i+1}] to interval i -> lane-local; u <= cdf_0 and u > cdf_{n-1} clamp.
template <class Emit>
__device__ __forceinline__ void emit_range(const float* __restrict__ u, int k0, int k1, float c0, float c1, float b0,
                                           float b1, Emit& em) {
  for (int k = k0; k < k1; ++k) em(k, invert_one(u[k], c0, c1, b0, b1));
}

// opacity_invert_cdf_sample (volsdf.py:104-117): cdf = [0, 1 - exp(-R_t)], sample_cdf(d, cdf, N)
template <class Emit>
__device__ void vs_finalize(const float* D, const float* S, int n, float alpha, float beta, const float* u, int N,
                            Emit& em) {
  const int l = threadIdx.x;
  if (l == 0) emit_range(u, 0, count_le(u, N, 0.0f), 0.0f, 0.0f, D[0], D[0], em);
  float carry = 0.0f;  // cdf_0
  vs_bounds(D, S, n, alpha, beta, [&](int i, bool v, float, float Rt) {
    const float c1 = fsub(1.0f, expf(-Rt));
    float c0 = __shfl_up(c1, 1);
    if (l == 0) c0 = carry;
    if (v) {
      const float b0 = D[i], b1 = D[i + 1];
      emit_range(u, count_le(u, N, c0), count_le(u, N, c1), c0, c1, b0, b1, em);
      if (i == n - 2) emit_range(u, count_le(u, N, c1), N, c1, c1, b1, b1, em);
    }
    carry = __shfl(c1, 63);
  });
}

// sample_pdf(d, bounds, N, det=True) (rend_util.py:255-292) with bounds from error_bound(alpha, beta)
// (clamped to [0, 1e5] after a bisection, volsdf.py:248-249).  Destroys S (holds the weights).
template <class Emit>
__device__ void vs_sample_pdf(const float* D, float* S, int n, float alpha, float beta, bool clamp, const float* u,
                              int N, float* red, Emit& em) {
  const int l = threadIdx.x;
  vs_bounds(D, S, n, alpha, beta, [&](int i, bool v, float b, float) {
    if (clamp) b = fminf(fmaxf(b, 0.0f), 1e5f);
    __syncthreads();  // every lane has read S[i], S[i+1] of this block
    if (v) S[i] = fadd(b, 1e-5f);
  });
  __syncthreads();
  if (l == 0) *red = aten_row_sum(n - 1, [&](int i) { return S[i]; });
  __syncthreads();
  const float total = *red;
  if (l == 0) emit_range(u, 0, count_le(u, N, 0.0f), 0.0f, 0.0f, D[0], D[0], em);
  double car = 0.0;
  float carry = 0.0f;
  for (int base = 0; base < n - 1; base += 64) {
    const int i = base + l;
    const bool v = i < n - 1;
    const float pdf = v ? fdiv(S[i], total) : 0.0f;
    const double inc = wave_scan_add((double)pdf);
    const float c1 = (float)(car + inc);
    float c0 = __shfl_up(c1, 1);
    if (l == 0) c0 = carry;
    if (v) {
      const float b0 = D[i], b1 = D[i + 1];
      emit_range(u, count_le(u, N, c0), count_le(u, N, c1), c0, c1, b0, b1, em);
      if (i == n - 2) emit_range(u, count_le(u, N, c1), N, c1, c1, b1, b1, em);
    }
    carry = __shfl(c1, 63);
    car += __shfl(inc, 63);
  }
}

// Merge m new samples (Nw, Ns; any order) into the sorted list (D, S)[0..n_old) in place, like
// torch.sort(cat([old, new])) + gather (volsdf.py:193-200).  Needs D/S capacity n_old + m.
__device__ void vs_merge(float* D, float* S, int n_old, float* Nw, float* Ns, int m) {
  const int l = threadIdx.x;
  bool bad = false;
  for (int j = l; j + 1 < m; j += 64) bad |= Nw[j] > Nw[j + 1];
  if (__ballot(bad) != 0) {  // rare: rounding made the new depths non-monotone -> rank sort
    for (int j = l; j < m; j += 64) {
      const float v = Nw[j];
      int r = 0;
      for (int k = 0; k < m; ++k) {
        const float w = Nw[k];
        r += (w < v) || (w == v && k < j);
      }
      D[n_old + r] = v;
      S[n_old + r] = Ns[j];
    }
    __syncthreads();
    for (int j = l; j < m; j += 64) {
      Nw[j] = D[n_old + j];
      Ns[j] = S[n_old + j];
    }
    __syncthreads();
  }
  int posn[kMaxPerLane];
#pragma unroll
  for (int t = 0; t < kMaxPerLane; ++t) {
    const int j = l + 64 * t;
    posn[t] = j < m ? j + upper_bound(D, n_old, Nw[j]) : 0;
  }
  __syncthreads();
  // old elements only move up: shift blocks from the top so nothing unread is overwritten
  for (int base = ((n_old - 1) >> 6) << 6; base >= 0; base -= 64) {
    const int i = base + l;
    float dv = 0.0f, sv = 0.0f;
    int p = 0;
    if (i < n_old) {
      dv = D[i];
      sv = S[i];
      p = i + lower_bound(Nw, m, dv);
    }
    __syncthreads();
    if (i < n_old) {
      D[p] = dv;
      S[p] = sv;
    }
    __syncthreads();
  }
#pragma unroll
  for (int t = 0; t < kMaxPerLane; ++t) {
    const int j = l + 64 * t;
    if (j < m) {
      D[posn[t]] = Nw[j];
      S[posn[t]] = Ns[j];
    }
  }
  __syncthreads();
}

struct Lds {
  float* D; float* S; float* Nw; float* Ns; float* red;
};

__device__ __forceinline__ Lds lds_views(const VolChunk& c) {
  extern __shared__ float lds[];
  const int M = c.S + c.N_out;
  const int big = c.cap > M ? c.cap : M;
  const int small = c.N_up > c.N_imp ? c.N_up : c.N_imp;
  return Lds{lds, lds + big, lds + 2 * big, lds + 2 * big + small, lds + 2 * big + 2 * small};
}

// Decision step shared by the first pass and every refinement round `it` (volsdf.py:134-270):
// converged -> final samples with the network's beta; otherwise bisect beta+, then either sample
// the next round (ray stays active) or, after the last round, sample with the final beta+.
__device__ void vs_decide(const VolChunk& c, int r, int it, int n, Lds& s) {
  const int l = threadIdx.x;
  float* fine = c.fine + (int64_t)r * c.N_imp;
  auto emit_fine = [&](int k, float v) { fine[k] = v; };
  const float* uf = c.u_rand ? c.u_rand + (int64_t)r * c.N_imp : c.u_fine;  // perturb: this ray's draws
  const float mnet = vs_bound_max(s.D, s.S, n, c.alpha_net, c.beta_net);
  if (!(mnet > c.eps)) {
    vs_finalize(s.D, s.S, n, c.alpha_net, c.beta_net, uf, c.N_imp, emit_fine);
    if (l == 0) {
      c.usage[r] = (float)it;
      c.bmap[r] = c.beta_net;
    }
    return;
  }
  float beta = c.N_out > 0 ? c.bp0[r] : c.beta_plus0;
  if (it > 0) {  // bisection on beta+ (volsdf.py:228-244)
    float br = c.beta[r], bl = c.beta_net;
    for (int b = 0; b < c.max_bisect; ++b) {
      const float bt = fmul(0.5f, fadd(bl, br));
      const float mx = vs_bound_max(s.D, s.S, n, fdiv(1.0f, bt), bt);
      if (mx <= c.eps) br = bt; else bl = bt;
    }
    beta = br;
  }
  const float alpha = fdiv(1.0f, beta);
  if (it == c.max_iter) {  // never converged: sample with the last beta+ (volsdf.py:259-268)
    vs_finalize(s.D, s.S, n, alpha, beta, uf, c.N_imp, emit_fine);
    if (l == 0) {
      c.usage[r] = -1.0f;
      c.bmap[r] = beta;
    }
    return;
  }
  // stays active for round it+1
  int slot = 0;
  if (l == 0) {
    slot = atomicAdd(c.cnt + it, 1);
    c.act[it & 1][slot] = r;
    c.beta[r] = beta;
  }
  slot = __shfl(slot, 0);
  if (it > 0) {  // persist the merged list for the next round (round 0's list is already there)
    float* gd = c.Ld[it & 1] + (int64_t)r * c.cap;
    float* gs = c.Ls[it & 1] + (int64_t)r * c.cap;
    for (int j = l; j < n; j += 64) {
      gd[j] = s.D[j];
      gs[j] = s.S[j];
    }
  }
  float* dn = c.dnew[it & 1] + (int64_t)slot * c.N_up;
  float* pp = c.pts + (int64_t)slot * c.N_up * 3;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  const int N_up = c.N_up;
  auto emit_up = [&](int k, float v) {  // sample_pdf(..., N_up + 2)[..., 1:-1]
    if (k >= 1 && k <= N_up) {
      const int q = k - 1;
      dn[q] = v;
      pp[q * 3 + 0] = fadd(ox, fmul(dx, v));
      pp[q * 3 + 1] = fadd(oy, fmul(dy, v));
      pp[q * 3 + 2] = fadd(oz, fmul(dz, v));
    }
  };
  vs_sample_pdf(s.D, s.S, n, alpha, beta, it > 0, c.u_up, N_up + 2, s.red, emit_up);
}

}  // namespace

// torch.sum(a * b, dim=-1) of two 3-vectors on the CPU: products rounded, then summed in order
__device__ __forceinline__ float ray_dot(float ax, float ay, float az, float bx, float by, float bz) {
  return fadd(fadd(fmul(ax, bx), fmul(ay, by)), fmul(az, bz));
}

// ---------------------------------------------------------------------------------------------
// kernels (one 64-thread workgroup = one wave per ray or active slot)
// ---------------------------------------------------------------------------------------------

// normalised directions (volsdf.py:388), d_init = near*(1-t)+far*t over 4*N_samples (volsdf.py:421-423)
__global__ __launch_bounds__(64) void volsdf_prologue(VolChunk c, const float* __restrict__ rays_o,
                                                       const float* __restrict__ rays_d) {
  const int r = blockIdx.x, l = threadIdx.x;
  const float ox = rays_o[r * 3 + 0], oy = rays_o[r * 3 + 1], oz = rays_o[r * 3 + 2];
  float dx = rays_d[r * 3 + 0], dy = rays_d[r * 3 + 1], dz = rays_d[r * 3 + 2];
  const float nn = fmaxf(norm3(dx, dy, dz), 1e-12f);
  dx = fdiv(dx, nn);
  dy = fdiv(dy, nn);
  dz = fdiv(dz, nn);
  float far = c.far;
  if (c.N_out > 0) {
    // rend_util.get_sphere_intersection (rend_util.py:188-210), far end, clamp_min(0); rays that
    // miss keep far = 0 (the reference asserts they do not occur, volsdf.py:405)
    const float dot = ray_dot(ox, oy, oz, dx, dy, dz);
    const float under = fsub(fadd(fmul(dot, dot), fmul(c.r_bg, c.r_bg)), ray_dot(ox, oy, oz, ox, oy, oz));
    far = under > 0.f ? fmaxf(fsub(sqrtf(under), dot), 0.f) : 0.f;
    if (l == 0) {
      c.farr[r] = far;
      c.bp0[r] = sqrtf(fdiv(fmul(far, far), c.beta_k));  // volsdf.py:129 with a per-ray far
    }
  }
  if (l == 0) {
    c.ro[r * 3 + 0] = ox; c.ro[r * 3 + 1] = oy; c.ro[r * 3 + 2] = oz;
    c.rd[r * 3 + 0] = dx; c.rd[r * 3 + 1] = dy; c.rd[r * 3 + 2] = dz;
  }
  float* gd = c.Ld[0] + (int64_t)r * c.cap;
  float* pp = c.pts + (int64_t)r * c.N0 * 3;
  for (int j = l; j < c.N0; j += 64) {
    const float t = c.t_init[j];
    const float d = fadd(fmul(c.near, fsub(1.0f, t)), fmul(far, t));
    gd[j] = d;
    pp[j * 3 + 0] = fadd(ox, fmul(dx, d));
    pp[j * 3 + 1] = fadd(oy, fmul(dy, d));
    pp[j * 3 + 2] = fadd(oz, fmul(dz, d));
  }
}

// first bound check with the network's beta, beta+ sampling for round 1 (volsdf.py:134-160)
__global__ __launch_bounds__(64) void volsdf_first(VolChunk c) {
  const int r = blockIdx.x, l = threadIdx.x;
  Lds s = lds_views(c);
  const float* gd = c.Ld[0] + (int64_t)r * c.cap;
  float* gs = c.Ls[0] + (int64_t)r * c.cap;
  const float* sr = c.sraw + (int64_t)r * c.N0;
  for (int j = l; j < c.N0; j += 64) {
    const float d = gd[j];
    const float v = surface_sdf(c, r, d, sr[j]);
    s.D[j] = d;
    s.S[j] = v;
    gs[j] = v;
  }
  __syncthreads();
  vs_decide(c, r, 0, c.N0, s);
}

// refinement round it >= 1 for the rays still active after round it-1 (volsdf.py:167-252)
__global__ __launch_bounds__(64) void volsdf_iter(VolChunk c, int it) {
  const int slot = blockIdx.x, l = threadIdx.x;
  if (slot >= c.cnt[it - 1]) return;
  const int p = (it - 1) & 1;
  const int r = c.act[p][slot];
  Lds s = lds_views(c);
  const int n_old = c.N0 + (it - 1) * c.N_up;
  const float* gd = c.Ld[p] + (int64_t)r * c.cap;
  const float* gs = c.Ls[p] + (int64_t)r * c.cap;
  for (int j = l; j < n_old; j += 64) {
    s.D[j] = gd[j];
    s.S[j] = gs[j];
  }
  const float* dn = c.dnew[p] + (int64_t)slot * c.N_up;
  const float* sr = c.sraw + (int64_t)slot * c.N_up;
  for (int j = l; j < c.N_up; j += 64) {
    const float d = dn[j];
    s.Nw[j] = d;
    s.Ns[j] = surface_sdf(c, r, d, sr[j]);
  }
  __syncthreads();
  vs_merge(s.D, s.S, n_old, s.Nw, s.Ns, c.N_up);
  vs_decide(c, r, it, n_old + c.N_up, s);
}

// d_all = sort(cat([d_coarse, d_fine])) and its points (volsdf.py:445-448)
__global__ __launch_bounds__(64) void volsdf_points(VolChunk c) {
  const int r = blockIdx.x, l = threadIdx.x;
  Lds s = lds_views(c);
  const float far = c.N_out > 0 ? c.farr[r] : c.far;
  for (int j = l; j < c.N_samples; j += 64) {
    const float t = c.t_coarse[j];
    s.D[j] = fadd(fmul(c.near, fsub(1.0f, t)), fmul(far, t));
    s.S[j] = 0.0f;
  }
  const float* fine = c.fine + (int64_t)r * c.N_imp;
  for (int j = l; j < c.N_imp; j += 64) {
    s.Nw[j] = fine[j];
    s.Ns[j] = 0.0f;
  }
  __syncthreads();
  vs_merge(s.D, s.S, c.N_samples, s.Nw, s.Ns, c.N_imp);
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  float* da = c.d_all + (int64_t)r * c.S;
  float* pp = c.pts_f + (int64_t)r * c.S * 3;
  for (int j = l; j < c.S; j += 64) {
    const float d = s.D[j];
    da[j] = d;
    pp[j * 3 + 0] = fadd(ox, fmul(dx, d));
    pp[j * 3 + 1] = fadd(oy, fmul(dy, d));
    pp[j * 3 + 2] = fadd(oz, fmul(dz, d));
  }
}

// NeRF++ background samples (volsdf.py:451-463): d_out = get_dvals_from_radius(o, d, rs)
// (rend_util.py:213-234, far end), x_out = [p_out / rs, 1 / rs]; perturb stratifies rs per ray
__global__ __launch_bounds__(64) void volsdf_outside(VolChunk c) {
  const int r = blockIdx.x, l = threadIdx.x;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  const float nsq = ray_dot(ox, oy, oz, ox, oy, oz);
  const float dot = ray_dot(ox, oy, oz, dx, dy, dz);
  const float q = fsub(nsq, fmul(dot, dot));
  const float* ur = c.u_out ? c.u_out + (int64_t)r * c.N_out : nullptr;
  for (int k = l; k < c.N_out; k += 64) {
    float rs = c.rs_out[k];
    if (ur) {  // perturb (volsdf.py:460-465): mids of neighbouring radii, the end radii kept
      const float lo = k > 0 ? fmul(0.5f, fadd(c.rs_out[k], c.rs_out[k - 1])) : c.rs_out[0];
      const float hi = k + 1 < c.N_out ? fmul(0.5f, fadd(c.rs_out[k + 1], c.rs_out[k])) : c.rs_out[c.N_out - 1];
      rs = fadd(lo, fmul(fsub(hi, lo), ur[k]));
    }
    const float d = fadd(-dot, sqrtf(fsub(fmul(rs, rs), q)));
    const int64_t i = (int64_t)r * c.N_out + k;
    c.d_out[i] = d;
    c.x4[i * 4 + 0] = fdiv(fadd(ox, fmul(dx, d)), rs);
    c.x4[i * 4 + 1] = fdiv(fadd(oy, fmul(dy, d)), rs);
    c.x4[i * 4 + 2] = fdiv(fadd(oz, fmul(dz, d)), rs);
    c.x4[i * 4 + 3] = fdiv(1.0f, rs);
  }
}

// background replacement (volsdf.py:317-325), sigma, p_i, tau_i and the maps (volsdf.py:449-528);
// with NeRF++ the N_out background samples follow the S inside ones (volsdf.py:465-469)
__global__ __launch_bounds__(64) void volsdf_composite(VolChunk c, VolOut o, int calc_normal, int white_bkgd) {
  const int r = blockIdx.x, l = threadIdx.x;
  Lds s = lds_views(c);
  const int S = c.S, No = c.N_out, M = S + No;
  const int64_t ro = o.ray0 + r;
  const float* da = c.d_all + (int64_t)r * S;
  const float* sf = c.sdf_f + (int64_t)r * S;
  const float* nb = c.nab_f + (int64_t)r * S * 3;
  const float* rad = c.rad_f + (int64_t)r * S * 3;
  const float* pp = c.pts_f + (int64_t)r * S * 3;
  const float* rado = c.rad_o + (int64_t)r * No * 3;
  // s.D: depths, s.S: sigma (inside: from the sdf; outside: the NeRF's raw sigma)
  for (int j = l; j < S; j += 64) {
    const float d = da[j];
    float v = sf[j];
    if (c.use_bg) {
      const float dbg = fsub(c.r_bg, norm3(pp[j * 3], pp[j * 3 + 1], pp[j * 3 + 2]));
      if (dbg < v) v = dbg;
    }
    const float sg = vs_sigma(v, c.alpha_net, c.beta_net);
    s.D[j] = d;
    s.S[j] = sg;
    if (o.sdf) o.sdf[ro * S + j] = v;
    if (o.d_vals) o.d_vals[ro * M + j] = d;
    if (o.sigma) o.sigma[ro * M + j] = sg;
    if (o.nablas) {
      o.nablas[(ro * S + j) * 3 + 0] = nb[j * 3 + 0];
      o.nablas[(ro * S + j) * 3 + 1] = nb[j * 3 + 1];
      o.nablas[(ro * S + j) * 3 + 2] = nb[j * 3 + 2];
    }
    if (o.radiance) {
      o.radiance[(ro * M + j) * 3 + 0] = rad[j * 3 + 0];
      o.radiance[(ro * M + j) * 3 + 1] = rad[j * 3 + 1];
      o.radiance[(ro * M + j) * 3 + 2] = rad[j * 3 + 2];
    }
  }
  for (int k = l; k < No; k += 64) {
    const int64_t i = (int64_t)r * No + k;
    const float d = c.d_out[i], sg = c.sig_o[i];
    s.D[S + k] = d;
    s.S[S + k] = sg;
    if (o.d_vals) o.d_vals[ro * M + S + k] = d;
    if (o.sigma) o.sigma[ro * M + S + k] = sg;
    if (o.sigma_bg) o.sigma_bg[ro * No + k] = sg;
#pragma unroll
    for (int q = 0; q < 3; ++q) {
      if (o.radiance) o.radiance[(ro * M + S + k) * 3 + q] = rado[k * 3 + q];
      if (o.radiance_bg) o.radiance_bg[(ro * No + k) * 3 + q] = rado[k * 3 + q];
    }
  }
  __syncthreads();
  // normals use the first min(#tau, #nablas) samples (volsdf.py:509-511)
  const int Nn = M - 1 < S ? M - 1 : S;
  double T = 1.0, a_rgb0 = 0.0, a_rgb1 = 0.0, a_rgb2 = 0.0, a_acc = 0.0, a_n0 = 0.0, a_n1 = 0.0, a_n2 = 0.0;
  for (int base = 0; base < M - 1; base += 64) {
    const int i = base + l;
    const bool v = i < M - 1;
    float p = 1.0f;
    if (v) p = expf(-fmaxf(fmul(s.S[i], fsub(s.D[i + 1], s.D[i])), 0.0f));
    const double inc = wave_scan_mul((double)p);
    double ex = __shfl_up(inc, 1);
    if (l == 0) ex = 1.0;
    const float Ti = (float)(T * ex);
    T *= __shfl(inc, 63);
    if (v) {
      const float tau = fmul(fadd(fsub(1.0f, p), 1e-10f), Ti);
      const float* rr = i < S ? rad + i * 3 : rado + (i - S) * 3;
      a_rgb0 += (double)fmul(tau, rr[0]);
      a_rgb1 += (double)fmul(tau, rr[1]);
      a_rgb2 += (double)fmul(tau, rr[2]);
      a_acc += (double)tau;
      if (calc_normal && i < Nn) {
        float x = nb[i * 3 + 0], y = nb[i * 3 + 1], z = nb[i * 3 + 2];
        const float nn = fmaxf(norm3(x, y, z), 1e-12f);
        a_n0 += (double)fmul(fdiv(x, nn), tau);
        a_n1 += (double)fmul(fdiv(y, nn), tau);
        a_n2 += (double)fmul(fdiv(z, nn), tau);
      }
      if (o.alpha) o.alpha[ro * (M - 1) + i] = fsub(1.0f, p);
      if (o.p_i) o.p_i[ro * (M - 1) + i] = p;
      if (o.weights) o.weights[ro * (M - 1) + i] = tau;
      s.S[i] = tau;  // sigma of sample i is only read by this lane, above
    }
    __syncthreads();
  }
  const float accf = (float)wave_sum(a_acc);
  const float denom = fadd(accf, 1e-10f);
  double a_dep = 0.0;
  for (int i = l; i < M - 1; i += 64) a_dep += (double)fmul(fdiv(s.S[i], denom), s.D[i]);
  const float depth = (float)wave_sum(a_dep);
  const float r0 = (float)wave_sum(a_rgb0), r1 = (float)wave_sum(a_rgb1), r2 = (float)wave_sum(a_rgb2);
  float n0 = 0.f, n1 = 0.f, n2 = 0.f;
  if (calc_normal) {
    n0 = (float)wave_sum(a_n0);
    n1 = (float)wave_sum(a_n1);
    n2 = (float)wave_sum(a_n2);
  }
  if (l == 0) {
    float q0 = r0, q1 = r1, q2 = r2;
    if (white_bkgd) {
      const float bg = fsub(1.0f, accf);
      q0 = fadd(q0, bg); q1 = fadd(q1, bg); q2 = fadd(q2, bg);
    }
    o.rgb[ro * 3 + 0] = q0;
    o.rgb[ro * 3 + 1] = q1;
    o.rgb[ro * 3 + 2] = q2;
    o.depth[ro] = depth;
    o.acc[ro] = accf;
    if (calc_normal && o.normals) {
      o.normals[ro * 3 + 0] = n0;
      o.normals[ro * 3 + 1] = n1;
      o.normals[ro * 3 + 2] = n2;
    }
    if (o.beta_map) o.beta_map[ro] = c.bmap[r];
    if (o.iter_usage) o.iter_usage[ro] = c.usage[r];
  }
}

// ---------------------------------------------------------------------------------------------
// workspace plan
// ---------------------------------------------------------------------------------------------
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

VolPlan volsdf_plan(const NrVolsdfArgs& a, int64_t Rc) {
  VolPlan p{};
  const int N0 = 4 * a.N_samples, N_up = 4 * a.N_samples;
  const int cap = N0 + a.max_upsample_steps * N_up;
  const int S = a.N_samples + a.N_importance;
  const int nq = N0 > N_up ? N0 : N_up;
  p.Rc = Rc;
  size_t off = 0;
  auto take = [&](size_t words) { size_t o = off; off = align_up(off + words * 4); return o; };
  p.o_ro = take(Rc * 3);
  p.o_rd = take(Rc * 3);
  p.o_Ld0 = take((size_t)Rc * cap);
  p.o_Ld1 = take((size_t)Rc * cap);
  p.o_Ls0 = take((size_t)Rc * cap);
  p.o_Ls1 = take((size_t)Rc * cap);
  p.o_dn0 = take((size_t)Rc * N_up);
  p.o_dn1 = take((size_t)Rc * N_up);
  p.o_pts = take((size_t)Rc * nq * 3);
  p.o_sraw = take((size_t)Rc * nq);
  p.o_act0 = take(Rc);
  p.o_act1 = take(Rc);
  p.o_cnt = take(a.max_upsample_steps + 1);
  p.o_beta = take(Rc);
  p.o_fine = take((size_t)Rc * a.N_importance);
  p.o_usage = take(Rc);
  p.o_bmap = take(Rc);
  p.o_dall = take((size_t)Rc * S);
  p.o_ptsf = take((size_t)Rc * S * 3);
  p.o_sdff = take((size_t)Rc * S);
  p.o_nabf = take((size_t)Rc * S * 3);
  p.o_featf = take((size_t)Rc * S * 256);
  p.o_radf = take((size_t)Rc * S * 3);
  const int No = a.N_outside > 0 ? a.N_outside : 0;
  p.o_farr = take(Rc);
  p.o_bp0 = take(Rc);
  p.o_dout = take((size_t)Rc * No + 1);
  p.o_x4 = take((size_t)Rc * No * 4 + 1);
  p.o_sigo = take((size_t)Rc * No + 1);
  p.o_rado = take((size_t)Rc * No * 3 + 1);
  p.o_mlp = off;
  p.total = off + nr_mlp_workspace_bytes(1);
  const int big = cap > S + No ? cap : S + No;
  const int small = N_up > a.N_importance ? N_up : a.N_importance;
  p.lds_bytes = (size_t)(2 * big + 2 * small + 4) * 4;
  return p;
}

}  // namespace nr
