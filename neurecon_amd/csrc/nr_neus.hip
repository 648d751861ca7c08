// neurecon_amd — NeuS render path for gfx950: per-ray sampling / compositing kernels and the
// orchestration of one ray chunk (models/frameworks/neus.py:118-397, render mode).
//
// Per-ray state is stored sample-major ([sample][ray]) so the one-thread-per-ray kernels read
// and write coalesced lines; the MLP kernels see a flat point list p = sample * Rc + ray.
// Scans (cumsum / cumprod) accumulate in fp64 exactly like ATen's CPU kernels
// (acc_type<float, is_cuda=false> = double), each prefix rounded to fp32.
#include "nr_common.h"
#include "nr_mlp.h"
#include "nr_neus.h"

namespace nr {

__device__ __forceinline__ float4 load3(const float* p) { return make_float4(p[0], p[1], p[2], 0.f); }

// F.normalize(v, dim=-1): v / max(||v||_2, 1e-12)
__device__ __forceinline__ void normalize3(float& x, float& y, float& z) {
  const float n = norm3_ref(x, y, z);
  const float d = fmaxf(n, 1e-12f);
  x = fdiv(x, d);
  y = fdiv(y, d);
  z = fdiv(z, d);
}

// ---------------------------------------------------------------------------------------------
// prologue: normalize rays_d (neus.py:169-172), near/far (rend_util.py:167-185), coarse depths
// (neus.py:209-210) and their points (neus.py:251)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void neus_prologue(NeusChunk c, const float* __restrict__ rays_o, const float* __restrict__ rays_d,
                              const float* __restrict__ t_coarse, float r_obj, float near_bypass, float far_bypass) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const float ox = rays_o[r * 3 + 0], oy = rays_o[r * 3 + 1], oz = rays_o[r * 3 + 2];
  float dx = rays_d[r * 3 + 0], dy = rays_d[r * 3 + 1], dz = rays_d[r * 3 + 2];
  normalize3(dx, dy, dz);
  c.ro[r * 3 + 0] = ox; c.ro[r * 3 + 1] = oy; c.ro[r * 3 + 2] = oz;
  c.rd[r * 3 + 0] = dx; c.rd[r * 3 + 1] = dy; c.rd[r * 3 + 2] = dz;
  const float mid = -fadd(fadd(fmul(ox, dx), fmul(oy, dy)), fmul(oz, dz));
  float nr = fmaxf(fsub(mid, r_obj), 0.0f);
  float fr = fmaxf(fadd(mid, r_obj), r_obj);
  if (!__builtin_isnan(near_bypass)) nr = near_bypass;
  if (!__builtin_isnan(far_bypass)) fr = far_bypass;
  c.near[r] = nr;
  c.far[r] = fr;
  for (int s = 0; s < c.N_samples; ++s) {
    const float t = t_coarse[s];
    const float d = fadd(fmul(nr, fsub(1.0f, t)), fmul(fr, t));
    const int64_t q = (int64_t)s * c.R + r;
    c.dv[q] = d;
    if (c.idv) c.idv[q] = s;
    c.pts[q * 3 + 0] = fadd(ox, fmul(dx, d));
    c.pts[q * 3 + 1] = fadd(oy, fmul(dy, d));
    c.pts[q * 3 + 2] = fadd(oz, fmul(dz, d));
  }
}

// sample_pdf(bins=dv[0..L), weights=wtmp[0..L-1) (already +1e-5), N=n, u) -> out[k*R + r]
// total = sum of the (+1e-5) weights.  rend_util.py:255-292.
__device__ void sample_pdf_ray(const float* __restrict__ bins, const float* __restrict__ w, int64_t stride, int L,
                               float total, const float* __restrict__ u, int n, float* __restrict__ out,
                               int64_t out_stride) {
  // w[i] are the raw weights; the +1e-5 of rend_util.py:259 is applied on the fly
  int k = 0;
  const float b_first = bins[0];
  while (k < n && u[k] <= 0.0f) {  // searchsorted -> 0: below = above = 0
    out[k * out_stride] = invert_one(u[k], 0.0f, 0.0f, b_first, b_first);
    ++k;
  }
  double acc = 0.0;
  float c_prev = 0.0f, b_prev = b_first;
  for (int i = 0; i < L - 1 && k < n; ++i) {
    acc += (double)fdiv(fadd(w[i * stride], 1e-5f), total);
    const float c_next = (float)acc;
    const float b_next = bins[(i + 1) * stride];
    while (k < n && u[k] <= c_next) {
      out[k * out_stride] = invert_one(u[k], c_prev, c_next, b_prev, b_next);
      ++k;
    }
    c_prev = c_next;
    b_prev = b_next;
  }
  // u above every cdf value: searchsorted -> L, below = above = L-1 (c_prev = cdf[L-1] here)
  for (; k < n; ++k) out[k * out_stride] = invert_one(u[k], c_prev, c_prev, b_prev, b_prev);
}

// sample_pdf with det=False (rend_util.py:268-290): the caller's uniforms u[0..n) are in any order,
// so each draw does its own searchsorted(cdf, u, right=False).  The cdf overwrites the weights in
// place (w[i] <- cdf[i+1], same fp64 running sum as above) and is binary-searched per draw.
__device__ void sample_pdf_ray_rand(const float* __restrict__ bins, float* __restrict__ w, int64_t stride, int L,
                                    float total, const float* __restrict__ u, int n, float* __restrict__ out,
                                    int64_t out_stride) {
  double acc = 0.0;
  for (int i = 0; i < L - 1; ++i) {
    acc += (double)fdiv(fadd(w[i * stride], 1e-5f), total);
    w[i * stride] = (float)acc;
  }
  auto cdf = [&](int j) { return j == 0 ? 0.0f : w[(int64_t)(j - 1) * stride]; };
  for (int k = 0; k < n; ++k) {
    const float uk = u[k];
    int lo = 0, hi = L;  // first j in [0, L) with cdf[j] >= uk, L if none
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (cdf(m) >= uk) hi = m; else lo = m + 1;
    }
    const int below = lo > 0 ? lo - 1 : 0, above = lo < L - 1 ? lo : L - 1;
    out[k * out_stride] = invert_one(uk, cdf(below), cdf(above), bins[below * stride], bins[above * stride]);
  }
}

// one "official_solution" upsampling round (neus.py:252-276): RPW rays per wave (64 / RPW lanes each).  The per-interval
// work (slopes, logistic CDFs, alpha) runs across the lanes; the three order-sensitive scans
// (transmittance cumprod, the ATen-order weight sum, the CDF cumsum) run on lane 0 over LDS with
// exactly the arithmetic of the per-ray version; the n_up inverse-CDF draws run across lanes.
// u: the round's uniforms, u[r * u_stride + k] (u_stride 0: the shared deterministic linspace)
template <int RPW>
__global__ __launch_bounds__(64) void neus_upsample(NeusChunk c, int it, const float* __restrict__ u, int64_t u_stride) {
  extern __shared__ float lds[];
  constexpr int NL = 64 / RPW;  // lanes per ray
  const int r = blockIdx.x * RPW + (int)threadIdx.x / NL, l = (int)threadIdx.x % NL;
  const int L = c.N_samples + it * c.n_up;  // last round's samples were merged by neus_merge
  const int64_t R = c.R;
  const bool live = r < R;
  const int Ll = live ? L : 0;  // a ray past the chunk's end only joins the barriers
  float* sz = lds + ((int)threadIdx.x / NL) * (5 * c.S + 1);  // depths [L]
  float* ss = sz + c.S;      // sdf [L]
  float* sa = ss + c.S;      // alpha, then weights [L-1]
  float* scdf = sa + c.S;    // (1 - alpha + 1e-10) factors [L-1], then the cdf [L]
  float* sq = scdf + c.S;    // normalised weights [L-1]
  float* stot = sq + c.S;    // [1] weight total
  for (int i = l; i < Ll; i += NL) {
    sz[i] = c.dv[i * R + r];
    ss[i] = c.sv[i * R + r];
  }
  __syncthreads();
  const float S = (float)(64 << it);  // 64 * 2**i
  for (int i = l; i < Ll - 1; i += NL) {
    const float s0 = ss[i], s1 = ss[i + 1], z0 = sz[i], z1 = sz[i + 1];
    const float mid = fmul(fadd(s0, s1), 0.5f);
    const float slope = fdiv(fsub(s1, s0), fadd(fsub(z1, z0), 1e-5f));
    const float prev_slope = i > 0 ? fdiv(fsub(s0, ss[i - 1]), fadd(fsub(z0, sz[i - 1]), 1e-5f)) : 0.0f;
    float m = fminf(prev_slope, slope);
    m = fminf(fmaxf(m, -10.0f), 0.0f);
    const float dist = fsub(z1, z0);
    const float md = fmul(fmul(m, dist), 0.5f);
    const float c0 = sigmoidf_ref(fmul(fsub(mid, md), S));
    const float c1 = sigmoidf_ref(fmul(fadd(mid, md), S));
    const float alpha = fdiv(fadd(fsub(c0, c1), 1e-5f), fadd(c0, 1e-5f));
    sa[i] = alpha;
    scdf[i] = fadd(fsub(1.0f, alpha), 1e-10f);  // the transmittance factor, off the serial chain
  }
  __syncthreads();
  if (l == 0 && live) {
    double T = 1.0;
    for (int i = 0; i < L - 1; ++i) {
      sa[i] = fmul(sa[i], (float)T);
      T *= (double)scdf[i];
    }
    stot[0] = aten_row_sum(L - 1, [&](int i) { return fadd(sa[i], 1e-5f); });
  }
  __syncthreads();
  {  // sample_pdf's normalised weights (rend_util.py:259-264) across the lanes
    const float total = stot[0];
    for (int i = l; i < Ll - 1; i += NL) sq[i] = fdiv(fadd(sa[i], 1e-5f), total);
  }
  __syncthreads();
  if (l == 0 && live) {  // ... and their fp64 running sum
    double acc = 0.0;
    scdf[0] = 0.0f;
    for (int i = 0; i < L - 1; ++i) {
      acc += (double)sq[i];
      scdf[i + 1] = (float)acc;
    }
  }
  __syncthreads();
  if (!live) return;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  for (int k = l; k < c.n_up; k += NL) {
    const float uk = u[r * u_stride + k];
    float d;
    if (uk <= 0.0f) {  // searchsorted -> 0: below = above = 0
      d = invert_one(uk, 0.0f, 0.0f, sz[0], sz[0]);
    } else {
      int lo = 0, hi = L - 1;  // first interval i with uk <= cdf[i+1]
      while (lo < hi) {
        const int mm = (lo + hi) >> 1;
        if (uk <= scdf[mm + 1]) hi = mm; else lo = mm + 1;
      }
      d = lo < L - 1 ? invert_one(uk, scdf[lo], scdf[lo + 1], sz[lo], sz[lo + 1])
                     : invert_one(uk, scdf[L - 1], scdf[L - 1], sz[L - 1], sz[L - 1]);  // above every cdf
    }
    const int64_t q = k * R + r;
    c.dnew[q] = d;
    c.pts[q * 3 + 0] = fadd(ox, fmul(dx, d));
    c.pts[q * 3 + 1] = fadd(oy, fmul(dy, d));
    c.pts[q * 3 + 2] = fadd(oz, fmul(dz, d));
  }
}

template __global__ void neus_upsample<1>(NeusChunk, int, const float*, int64_t);
template __global__ void neus_upsample<4>(NeusChunk, int, const float*, int64_t);

// merge (neus.py:276: cat + sort + gather) of the sorted list (dv, sv, idv)[0..L) with the n_up new
// samples (dnew, snew) into (dv2, sv2, idv2)[0..L+n_up), one thread per (output element, ray):
// old element i lands at i + #(new < d_i), new element j at rank_j + #(old <= d_j) (stable; ties put
// new after old) — the order of a stable sort of the concatenation.
// sort key: NaN after everything (torch.sort order), so positions stay a permutation for any input
__device__ __forceinline__ float merge_key(float v) { return v != v ? __builtin_inff() : v; }

__global__ void neus_merge(NeusChunk c, int L, float* __restrict__ dv2, float* __restrict__ sv2,
                           int* __restrict__ idv2) {
  const int64_t R = c.R;
  const int n = c.n_up;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)(L + n) * R) return;
  const int64_t e = t / R, r = t - e * R;
  if (e < L) {
    const int64_t q = e * R + r;
    const float d = c.dv[q], kd = merge_key(d);
    int cnt = 0;
    for (int k = 0; k < n; ++k) cnt += merge_key(c.dnew[k * R + r]) < kd ? 1 : 0;
    const int64_t qo = (e + cnt) * R + r;
    dv2[qo] = d;
    sv2[qo] = c.sv[q];
    if (idv2) idv2[qo] = c.idv[q];
  } else {
    const int j = (int)(e - L);
    const float d = c.dnew[j * R + r], kd = merge_key(d);
    int rank = 0;
    for (int k = 0; k < n; ++k) {
      const float v = merge_key(c.dnew[k * R + r]);
      rank += (v < kd || (v == kd && k < j)) ? 1 : 0;
    }
    int lo = 0, hi = L;  // upper bound of d in the sorted old list
    while (lo < hi) {
      const int m = (lo + hi) >> 1;
      if (merge_key(c.dv[m * R + r]) <= kd) lo = m + 1; else hi = m;
    }
    const int64_t qo = (int64_t)(rank + lo) * R + r;
    dv2[qo] = d;
    sv2[qo] = c.snew[j * R + r];
    if (idv2) idv2[qo] = L + j;  // new samples were evaluated in slots L .. L+n-1
  }
}

// per (sample, ray) after the final merge: sample points (or, fused, the sorted nablas) and the
// S-1 mid-points d_mid = (d_s + d_{s-1}) / 2 (neus.py:284-288); sample-major, fully parallel
// gather = 0: the fused path's nablas are gathered later (neus_gather_nablas: the deferred reverse
// pass of a NeRF++ render runs after the background net)
__global__ void neus_expand(NeusChunk c, int gather) {
  const int64_t R = c.R;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)c.S * R) return;
  const int64_t s = q / R, r = q - s * R;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  const float d = c.dv[q];
  if (c.idv) {  // fused: nablas of the sorted samples from their evaluation slots
    if (gather) {
      const int64_t qs = (int64_t)c.idv[q] * R + r;
#pragma unroll
      for (int e = 0; e < 3; ++e) c.nab_f[q * 3 + e] = c.nraw[qs * 3 + e];
    }
  } else {
    c.pts[q * 3 + 0] = fadd(ox, fmul(dx, d));
    c.pts[q * 3 + 1] = fadd(oy, fmul(dy, d));
    c.pts[q * 3 + 2] = fadd(oz, fmul(dz, d));
  }
  if (s > 0) {
    const float dm = fmul(0.5f, fadd(d, c.dv[q - R]));
    const int64_t qm = q - R;
    c.dmid[qm] = dm;
    c.mids[qm * 3 + 0] = fadd(ox, fmul(dx, dm));
    c.mids[qm * 3 + 1] = fadd(oy, fmul(dy, dm));
    c.mids[qm * 3 + 2] = fadd(oz, fmul(dz, dm));
  }
}

// the fused path's sample nablas into sorted order (neus_expand's gather, run on its own)
__global__ void neus_gather_nablas(NeusChunk c) {
  const int64_t R = c.R;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)c.S * R) return;
  const int64_t r = q - (q / R) * R;
  const int64_t qs = (int64_t)c.idv[q] * R + r;
#pragma unroll
  for (int e = 0; e < 3; ++e) c.nab_f[q * 3 + e] = c.nraw[qs * 3 + e];
}

// compositing (neus.py:296, :346-380), RPW rays per wave (64 / RPW lanes each): logistic CDFs,
// alpha, radiance and unit normals per sample across the ray's lanes (LDS); the transmittance product
// and the fp64 rgb / acc / normal / depth accumulations on the ray's first lane in sample order,
// exactly as the per-ray version did.  RPW 4: the serial scans of four rays share one wave's issue.
// s = exp(ln_s * speed_factor) (neus.py:108-109): *s_dev when given (device scalar, no host sync), else s_val
template <int RPW>
__global__ __launch_bounds__(64) void neus_composite(NeusChunk c, NeusOut o, const float* __restrict__ s_dev,
                                                     float s_val, int calc_normal, int white_bkgd) {
  extern __shared__ float lds[];
  constexpr int NL = 64 / RPW;  // lanes per ray
  const float s_inv = s_dev ? *s_dev : s_val;
  const int r = blockIdx.x * RPW + (int)threadIdx.x / NL, l = (int)threadIdx.x % NL;
  const int S = c.S;
  const int64_t R = c.R;
  const bool live = r < R;
  const int Sl = live ? S : 0;    // a ray past the chunk's end only joins the barriers
  const int64_t ro = o.ray0 + r;  // global ray index for outputs
  float* scdf = lds + ((int)threadIdx.x / NL) * 9 * S;  // [S]
  float* sal = scdf + S;      // [S-1] alpha, then weights
  float* srad = sal + S;      // [S-1][3]
  float* snrm = srad + 3 * S; // [S-1][3] unit nablas
  float* sdm = snrm + 3 * S;  // [S-1] mid-point depths (the serial depth sum reads LDS, not HBM)
  for (int i = l; i < Sl; i += NL) {
    const float cdf = sigmoidf_ref(fmul(c.sdf_f[i * R + r], s_inv));
    scdf[i] = cdf;
    if (o.cdf) o.cdf[ro * S + i] = cdf;
  }
  __syncthreads();
  for (int i = l; i < Sl - 1; i += NL) {
    const float cp = scdf[i], cn = scdf[i + 1];
    const float alpha = fmaxf(fdiv(fsub(cp, cn), fadd(cp, 1e-10f)), 0.0f);
    sal[i] = alpha;
    if (o.alpha) o.alpha[ro * (S - 1) + i] = alpha;
    const int64_t q = i * R + r;
    sdm[i] = c.dmid[q];
#pragma unroll
    for (int e = 0; e < 3; ++e) srad[i * 3 + e] = c.rad_m[q * 3 + e];
    if (calc_normal) {
      float x = c.nab_f[q * 3 + 0], y = c.nab_f[q * 3 + 1], z = c.nab_f[q * 3 + 2];
      normalize3(x, y, z);
      snrm[i * 3 + 0] = x;
      snrm[i * 3 + 1] = y;
      snrm[i * 3 + 2] = z;
    }
  }
  __syncthreads();
  double rgb0 = 0.0, rgb1 = 0.0, rgb2 = 0.0, n0 = 0.0, n1 = 0.0, n2 = 0.0;
  float accf = 0.0f;
  if (l == 0 && live) {
    double T = 1.0, acc = 0.0;
    for (int i = 0; i < S - 1; ++i) {
      const float alpha = sal[i];
      const float w = fmul(alpha, (float)T);
      T *= (double)fadd(fsub(1.0f, alpha), 1e-10f);
      rgb0 += (double)fmul(w, srad[i * 3 + 0]);
      rgb1 += (double)fmul(w, srad[i * 3 + 1]);
      rgb2 += (double)fmul(w, srad[i * 3 + 2]);
      acc += (double)w;
      if (calc_normal) {
        n0 += (double)fmul(snrm[i * 3 + 0], w);
        n1 += (double)fmul(snrm[i * 3 + 1], w);
        n2 += (double)fmul(snrm[i * 3 + 2], w);
      }
      sal[i] = w;
    }
    accf = (float)acc;
    scdf[0] = fadd(accf, 1e-10f);  // the depth normaliser for the ray's lanes (the cdf is no longer read)
  }
  __syncthreads();
  // depth terms w_i / (acc + 1e-10) * d_mid_i across the ray's lanes, into scdf[1 ..] (the CDFs
  // are no longer read; scdf[0] holds the normaliser)
  {
    const float denom = scdf[0];
    __syncthreads();  // every lane has its normaliser before scdf[1 ..] is overwritten
    for (int i = l; i < Sl - 1; i += NL) scdf[i + 1] = fmul(fdiv(sal[i], denom), sdm[i]);
  }
  __syncthreads();
  if (l == 0 && live) {
    double depth = 0.0;
    for (int i = 0; i < S - 1; ++i) depth += (double)scdf[i + 1];
    float r0 = (float)rgb0, r1 = (float)rgb1, r2 = (float)rgb2;
    if (white_bkgd) {
      const float bg = fsub(1.0f, accf);
      r0 = fadd(r0, bg); r1 = fadd(r1, bg); r2 = fadd(r2, bg);
    }
    o.rgb[ro * 3 + 0] = r0;
    o.rgb[ro * 3 + 1] = r1;
    o.rgb[ro * 3 + 2] = r2;
    o.depth[ro] = (float)depth;
    o.acc[ro] = accf;
    if (calc_normal && o.normals) {
      o.normals[ro * 3 + 0] = (float)n0;
      o.normals[ro * 3 + 1] = (float)n1;
      o.normals[ro * 3 + 2] = (float)n2;
    }
  }
  __syncthreads();
  // detailed per-sample outputs, ray-major
  for (int i = l; i < Sl; i += NL) {
    const int64_t q = i * R + r;
    if (o.sdf) o.sdf[ro * S + i] = c.sdf_f[q];
    if (o.nablas) {
      o.nablas[(ro * S + i) * 3 + 0] = c.nab_f[q * 3 + 0];
      o.nablas[(ro * S + i) * 3 + 1] = c.nab_f[q * 3 + 1];
      o.nablas[(ro * S + i) * 3 + 2] = c.nab_f[q * 3 + 2];
    }
    if (i < S - 1) {
      if (o.weights) o.weights[ro * (S - 1) + i] = sal[i];
      if (o.d_final) o.d_final[ro * (S - 1) + i] = c.dmid[q];
      if (o.radiance) {
        o.radiance[(ro * (S - 1) + i) * 3 + 0] = srad[i * 3 + 0];
        o.radiance[(ro * (S - 1) + i) * 3 + 1] = srad[i * 3 + 1];
        o.radiance[(ro * (S - 1) + i) * 3 + 2] = srad[i * 3 + 2];
      }
    }
  }
}

template __global__ void neus_composite<1>(NeusChunk, NeusOut, const float*, float, int, int);
template __global__ void neus_composite<4>(NeusChunk, NeusOut, const float*, float, int, int);

// ---------------------------------------------------------------------------------------------
// 'direct_use' / 'direct_more' upsampling (neus.py:215-243): one sample_pdf of N_importance over
// the visibility weights of the coarse (or N_nograd_samples uniform) depths, s = 1/fixed_s_recp
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64) void neus_nograd_points(NeusChunk c) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const int64_t R = c.R;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  const float nr = c.near[r], fr = c.far[r];
  for (int k = 0; k < c.n_nog; ++k) {
    const float t = c.t_nog[k];
    const float d = fadd(fmul(nr, fsub(1.0f, t)), fmul(fr, t));
    const int64_t q = (int64_t)k * R + r;
    c.pts_nog[q * 3 + 0] = fadd(ox, fmul(d, dx));
    c.pts_nog[q * 3 + 1] = fadd(oy, fmul(d, dy));
    c.pts_nog[q * 3 + 2] = fadd(oz, fmul(d, dz));
  }
}

__global__ __launch_bounds__(64) void neus_direct_upsample(NeusChunk c, int more, const float* __restrict__ u,
                                                         int64_t u_stride) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const int64_t R = c.R;
  const int L = more ? c.n_nog : c.N_samples;
  const float nr = c.near[r], fr = c.far[r];
  // bins: the coarse depths (dv) or the nograd depths (recomputed, never stored)
  float* bins = c.dv + r;
  if (more) {
    bins = c.d_out + r;  // scratch column of >= n_nog floats
    for (int k = 0; k < L; ++k) {
      const float t = c.t_nog[k];
      bins[(int64_t)k * R] = fadd(fmul(nr, fsub(1.0f, t)), fmul(fr, t));
    }
  }
  const float* sdf = more ? c.s_nog + r : c.sv + r;
  // sdf_to_w (neus.py:37-70): logistic cdf, alpha = max((c_i - c_i+1)/(c_i + 1e-10), 0), cumprod
  double T = 1.0;
  float cprev = sigmoidf_ref(fmul(sdf[0], c.fixed_s));
  for (int i = 0; i < L - 1; ++i) {
    const float cn = sigmoidf_ref(fmul(sdf[(int64_t)(i + 1) * R], c.fixed_s));
    const float alpha = fmaxf(fdiv(fsub(cprev, cn), fadd(cprev, 1e-10f)), 0.0f);
    c.wtmp[(int64_t)i * R + r] = fmul(alpha, (float)T);
    T *= (double)fadd(fsub(1.0f, alpha), 1e-10f);
    cprev = cn;
  }
  float* wr = c.wtmp + r;
  const float total = aten_row_sum(L - 1, [&](int i) { return fadd(wr[(int64_t)i * R], 1e-5f); });
  float* dn = c.dnew + r;
  if (u_stride) sample_pdf_ray_rand(bins, wr, R, L, total, u + r * u_stride, c.n_imp, dn, R);
  else sample_pdf_ray(bins, wr, R, L, total, u, c.n_imp, dn, R);
  // sort(cat([d_coarse, d_fine])) (neus.py:227-228): insertion-sort the new column, merge in place
  const int n = c.n_imp;
  for (int k = 1; k < n; ++k) {
    const float v = dn[(int64_t)k * R];
    int j = k - 1;
    while (j >= 0 && dn[(int64_t)j * R] > v) {
      dn[(int64_t)(j + 1) * R] = dn[(int64_t)j * R];
      --j;
    }
    dn[(int64_t)(j + 1) * R] = v;
  }
  int i = c.N_samples - 1, j = n - 1;
  for (int k = c.N_samples + n - 1; k >= 0 && j >= 0; --k) {
    const float di = i >= 0 ? c.dv[(int64_t)i * R + r] : 0.f;
    const float dj = dn[(int64_t)j * R];
    if (i >= 0 && di > dj) {
      c.dv[(int64_t)k * R + r] = di;
      --i;
    } else {
      c.dv[(int64_t)k * R + r] = dj;
      --j;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// NeRF++ background (neus.py:303-343)
// ---------------------------------------------------------------------------------------------
// d_vals_out = cat([d_mid, far / flip(linspace(0,1,N_out+2)[1:-1])]); x_out = [p / |p|, 1 / |p|]
// perturb (neus.py:306-311): d_k = lower_k + (upper_k - lower_k) * t_rand[r][k] with the mid-point
// brackets of the deterministic inverted-sphere depths (t_rand: the caller's uniforms, or null)
__global__ __launch_bounds__(64) void neus_outside_points(NeusChunk c, const float* __restrict__ t_rand) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const int64_t R = c.R;
  const int S1 = c.S - 1, M = S1 + c.N_out;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  const float fr = c.far[r];
  const int No = c.N_out;
  auto dvo = [&](int j) { return fdiv(fr, c.t_out[No - j]); };  // far / flip(linspace(0,1,No+2)[1:-1])[j]
  for (int k = 0; k < M; ++k) {
    float d;
    if (k < S1) {
      d = c.dmid[(int64_t)k * R + r];
    } else {
      const int j = k - S1;
      d = dvo(j);
      if (t_rand) {
        const float lower = j > 0 ? fmul(0.5f, fadd(dvo(j), dvo(j - 1))) : dvo(0);
        const float upper = j + 1 < No ? fmul(0.5f, fadd(dvo(j + 1), dvo(j))) : dvo(No - 1);
        d = fadd(lower, fmul(fsub(upper, lower), t_rand[(int64_t)r * No + j]));
      }
    }
    const int64_t q = (int64_t)k * R + r;
    c.d_out[q] = d;
    const float px = fadd(ox, fmul(dx, d)), py = fadd(oy, fmul(dy, d)), pz = fadd(oz, fmul(dz, d));
    const float rr = norm3_ref(px, py, pz);
    *(float4*)(c.x4 + q * 4) = make_float4(fdiv(px, rr), fdiv(py, rr), fdiv(pz, rr), fdiv(1.0f, rr));
  }
}

// Workgroup-aggregated append (blockDim.x a multiple of 64, at most 1024): one atomicAdd per
// workgroup instead of one per wave -- the per-wave atomics on the one counter serialised (~8 ns
// each, 8 k of them per config-(b) mid-point pass).  Returns the lane's compact index when need.
// Every thread of the block must call it (barriers inside).
__device__ __forceinline__ int64_t block_append(bool need, int* __restrict__ count) {
  __shared__ int wcnt[16];
  __shared__ int bbase;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t bal = __ballot(need);
  if (lane == 0) wcnt[w] = __popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
    for (int i = 0; i < nw; ++i) {
      const int v = wcnt[i];
      wcnt[i] = t;
      t += v;
    }
    bbase = t ? atomicAdd(count, t) : 0;
  }
  __syncthreads();
  return (int64_t)bbase + wcnt[w] + __popcll(bal & ((1ull << lane) - 1ull));
}

// The background values the compositing reads (neus.py:325-343): every inverted-sphere sample, and the
// mid-points outside the bounding sphere -- the ones inside take the SDF's alpha and radiance, so the
// reference's background evaluation there is discarded.  Without detailed outputs only these points
// go through the NeRF++ net: appended (one atomic per workgroup) to x4c / vdc, slot[q] = compact index or
// -1; the inside test is the compositing's own (norm3_ref(o + d dm) <= r_obj).
__global__ void neus_outside_compact(NeusChunk c, int* __restrict__ count, int* __restrict__ slot,
                                     float* __restrict__ x4c, float* __restrict__ vdc) {
  const int64_t R = c.R;
  const int S1 = c.S - 1, M = S1 + c.N_out;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in_range = q < (int64_t)M * R;
  int64_t r = 0;
  bool need = false;
  if (in_range) {
    const int k = (int)(q / R);
    r = q - (int64_t)k * R;
    if (k >= S1) {
      need = true;
    } else {
      const float dm = c.dmid[q];
      const float px = fadd(c.ro[r * 3], fmul(c.rd[r * 3], dm)), py = fadd(c.ro[r * 3 + 1], fmul(c.rd[r * 3 + 1], dm)),
                  pz = fadd(c.ro[r * 3 + 2], fmul(c.rd[r * 3 + 2], dm));
      need = !(norm3_ref(px, py, pz) <= c.r_obj);
    }
  }
  const int64_t ja = block_append(need, count);
  if (!in_range) return;
  if (need) {
    const int j = (int)ja;
    slot[q] = j;
    *(float4*)(x4c + (int64_t)j * 4) = *(const float4*)(c.x4 + q * 4);
    vdc[(int64_t)j * 3 + 0] = c.rd[r * 3 + 0];
    vdc[(int64_t)j * 3 + 1] = c.rd[r * 3 + 1];
    vdc[(int64_t)j * 3 + 2] = c.rd[r * 3 + 2];
  } else {
    slot[q] = -1;
  }
}

// Mid-point i of a ray contributes w_i * radiance_i with w_i = alpha_i T_i, and alpha_i = max((c_i -
// c_{i+1}) / (c_i + 1e-10), 0) is exactly 0 wherever the SDF does not decrease from sample i to i+1
// (neus.py:28-35): there the radiance (and the mid-point's SDF, nablas and feature that feed it) is
// multiplied by an exact zero.  Without detailed outputs only the mid-points with alpha != 0 (the
// compositing's own arithmetic) go through the SDF + radiance nets; the others get radiance 0.
__global__ void neus_mid_compact(NeusChunk c, const float* __restrict__ s_dev, float s_val, int* __restrict__ count,
                                 int* __restrict__ slot, float* __restrict__ midc, float* __restrict__ vdc) {
  const int64_t R = c.R;
  const int S1 = c.S - 1;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool in_range = q < (int64_t)S1 * R;
  int64_t r = 0;
  bool need = false;
  if (in_range) {
    const float s_inv = s_dev ? *s_dev : s_val;
    const int i = (int)(q / R);
    r = q - (int64_t)i * R;
    const float cp = sigmoidf_ref(fmul(c.sdf_f[(int64_t)i * R + r], s_inv));
    const float cn = sigmoidf_ref(fmul(c.sdf_f[(int64_t)(i + 1) * R + r], s_inv));
    const float alpha = fmaxf(fdiv(fsub(cp, cn), fadd(cp, 1e-10f)), 0.0f);
    need = !(alpha == 0.0f);
    if (need && c.N_out > 0) {  // NeRF++: a mid-point outside the bounding sphere takes the background's
      const float dm = c.dmid[q];  // alpha and colour (neus_composite_outside's own inside test)
      const float px = fadd(c.ro[r * 3], fmul(c.rd[r * 3], dm)), py = fadd(c.ro[r * 3 + 1], fmul(c.rd[r * 3 + 1], dm)),
                  pz = fadd(c.ro[r * 3 + 2], fmul(c.rd[r * 3 + 2], dm));
      need = norm3_ref(px, py, pz) <= c.r_obj;
    }
  }
  const int64_t j = block_append(need, count);
  if (!in_range) return;
  if (need) {
    slot[q] = (int)j;
#pragma unroll
    for (int e = 0; e < 3; ++e) {
      midc[j * 3 + e] = c.mids[q * 3 + e];
      vdc[j * 3 + e] = c.rd[r * 3 + e];
    }
  } else {
    slot[q] = -1;
  }
}

// F.softplus (beta 1, threshold 20)
__device__ __forceinline__ float softplus1(float x) { return x > 20.0f ? x : log1pf(expf(x)); }

// deferred sample nablas: flag the 16-slot tile (evaluation order) of every sorted sample i < S-1 whose
// interval alpha is not exactly 0 -- neus_composite weights sample i's unit nabla by w_i = alpha_i T_i
// (neus.py:364-368), so the others contribute exactly 0 (their nablas stay 0, normalize(0) = 0).
// Same alpha arithmetic as neus_mid_compact / the compositing.
__global__ void neus_sample_need(NeusChunk c, const float* __restrict__ s_dev, float s_val) {
  const int64_t R = c.R;
  const int S1 = c.S - 1;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)S1 * R) return;
  const float s_inv = s_dev ? *s_dev : s_val;
  const int i = (int)(q / R);
  const int64_t r = q - (int64_t)i * R;
  const float cp = sigmoidf_ref(fmul(c.sdf_f[(int64_t)i * R + r], s_inv));
  const float cn = sigmoidf_ref(fmul(c.sdf_f[(int64_t)(i + 1) * R + r], s_inv));
  const float alpha = fmaxf(fdiv(fsub(cp, cn), fadd(cp, 1e-10f)), 0.0f);
  if (!(alpha == 0.0f)) c.tflag[((int64_t)c.idv[q] * R + r) >> c.tshift] = 1;
}

// the same with the NeRF++ background (neus_composite_outside): sample k < S weights its unit nabla by
// w_k = alpha_k T_k, alpha_k the SDF alpha of interval k if mid-point k is inside the bounding sphere,
// else the background's 1 - exp(-softplus(sigma) dist) -- also for k = S-1, whose weight is the first
// inverted-sphere sample's (neus.py:364-366 pairs min(#weights, #nablas) = S of them).  Runs after the
// background net (sig_o) with the compositing's own arithmetic; a tile is flagged if any alpha != 0.
__global__ void neus_sample_need_outside(NeusChunk c, const float* __restrict__ s_dev, float s_val) {
  const int64_t R = c.R;
  const int S = c.S, S1 = S - 1, M = S1 + c.N_out;
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)S * R) return;
  const int k = (int)(q / R);
  const int64_t r = q - (int64_t)k * R;
  bool inside = false;
  float alpha = 0.0f;
  if (k < S1) {
    const float s_inv = s_dev ? *s_dev : s_val;
    const float cp = sigmoidf_ref(fmul(c.sdf_f[(int64_t)k * R + r], s_inv));
    const float cn = sigmoidf_ref(fmul(c.sdf_f[(int64_t)(k + 1) * R + r], s_inv));
    alpha = fmaxf(fdiv(fsub(cp, cn), fadd(cp, 1e-10f)), 0.0f);
    const float dm = c.dmid[q];
    const float px = fadd(c.ro[r * 3], fmul(c.rd[r * 3], dm)), py = fadd(c.ro[r * 3 + 1], fmul(c.rd[r * 3 + 1], dm)),
                pz = fadd(c.ro[r * 3 + 2], fmul(c.rd[r * 3 + 2], dm));
    inside = norm3_ref(px, py, pz) <= c.r_obj;
  }
  if (!inside) {
    const float dk = c.d_out[q];
    const float dist = k + 1 < M ? fsub(c.d_out[q + R], dk) : 1e10f;
    alpha = fsub(1.0f, expf(fmul(-softplus1(c.sig_o[q]), dist)));
  }
  if (!(alpha == 0.0f)) c.tflag[((int64_t)c.idv[q] * R + r) >> c.tshift] = 1;
}

// flagged sample slots -> list for the compacted reverse pass (sdf4_kernel STAGE 4): each 1024-slot
// workgroup appends its flagged slots in slot order as one segment padded with -1 to a multiple of 16
// entries (one atomic per workgroup), so the 16 entries a wave takes come from one 1024-slot range:
// within 64 tiles of the segment's first entry (the kernel's per-lane slab offsets stay small)
__global__ __launch_bounds__(1024) void neus_point_list(NeusChunk c, int64_t n_slots) {
  __shared__ int wcnt[16];
  __shared__ int bbase, btot;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool need = t < n_slots && c.tflag[t] != 0;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const uint64_t bal = __ballot(need);
  if (lane == 0) wcnt[w] = __popcll(bal);
  __syncthreads();
  if (threadIdx.x == 0) {
    int s = 0;
    for (int i = 0; i < nw; ++i) {
      const int v = wcnt[i];
      wcnt[i] = s;
      s += v;
    }
    btot = s;
    bbase = s ? atomicAdd(c.tcnt, (s + 15) & ~15) : 0;
  }
  __syncthreads();
  if (need) c.tiles[(int64_t)bbase + wcnt[w] + __popcll(bal & ((1ull << lane) - 1ull))] = (int)t;
  const int pad = ((btot + 15) & ~15) - btot;
  if ((int)threadIdx.x < pad) c.tiles[(int64_t)bbase + btot + threadIdx.x] = -1;
}

// flagged tiles -> list (any order: each tile's nablas depend on that tile alone)
__global__ void neus_tile_list(NeusChunk c, int64_t n_tiles) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool need = t < n_tiles && c.tflag[t] != 0;
  const int64_t j = block_append(need, c.tcnt);
  if (need) c.tiles[j] = (int)t;
}

__global__ void neus_mid_scatter(const int* __restrict__ slot, const float* __restrict__ radc, int64_t n,
                                 float* __restrict__ rad_m) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int j = slot[q];
#pragma unroll
  for (int e = 0; e < 3; ++e) rad_m[q * 3 + e] = j < 0 ? 0.0f : radc[(int64_t)j * 3 + e];
}

__global__ void neus_outside_scatter(const int* __restrict__ slot, const float* __restrict__ sigc,
                                     const float* __restrict__ radc, int64_t n, float* __restrict__ sig_o,
                                     float* __restrict__ rad_o) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= n) return;
  const int j = slot[q];
  if (j < 0) return;
  sig_o[q] = sigc[j];
  rad_o[q * 3 + 0] = radc[(int64_t)j * 3 + 0];
  rad_o[q * 3 + 1] = radc[(int64_t)j * 3 + 1];
  rad_o[q * 3 + 2] = radc[(int64_t)j * 3 + 2];
}


// compositing with the background merged in, RPW rays per wave (neus_composite's structure): the
// per-sample CDFs, the inside test, the inside / background alphas, radiance and unit nablas across the
// ray's lanes into LDS; the transmittance product and the fp64 sums on the ray's first lane in sample
// order with the per-ray version's arithmetic (bit-identical maps; that version, one thread per ray,
// remains the fallback when the LDS staging does not fit).  LDS per ray: 6 M + 4 S floats.
template <int RPW>
__global__ __launch_bounds__(64) void neus_composite_outside_w(NeusChunk c, NeusOut o, const float* __restrict__ s_dev,
                                                               float s_val, int calc_normal, int white_bkgd) {
  extern __shared__ float lds[];
  constexpr int NL = 64 / RPW;
  const float s_inv = s_dev ? *s_dev : s_val;
  const int r = blockIdx.x * RPW + (int)threadIdx.x / NL, l = (int)threadIdx.x % NL;
  const int S = c.S, S1 = S - 1, M = S1 + c.N_out;
  const int Nn = M < S ? M : S;  // normals use min(#weights, #nablas) samples (neus.py:364-366)
  const int64_t R = c.R;
  const bool live = r < R;
  const int Sl = live ? S : 0, Ml = live ? M : 0, Nl = live ? Nn : 0;
  const int64_t ro = o.ray0 + r;
  float* scdf = lds + ((int)threadIdx.x / NL) * (6 * M + 4 * S);  // [S]
  float* sal = scdf + S;       // [M] alpha, then weights
  float* srad = sal + M;       // [M][3]
  float* sdo = srad + 3 * M;   // [M] d_out
  float* dum = sdo + M;        // [M] (pad)
  float* snrm = dum + M;       // [S][3] unit nablas
  for (int i = l; i < Sl; i += NL) {
    const float cdf = sigmoidf_ref(fmul(c.sdf_f[(int64_t)i * R + r], s_inv));
    scdf[i] = cdf;
    if (o.cdf) o.cdf[ro * S + i] = cdf;
  }
  __syncthreads();
  for (int k = l; k < Ml; k += NL) {
    const int64_t q = (int64_t)k * R + r;
    const float dk = c.d_out[q];
    sdo[k] = dk;
    bool inside = false;
    float a_in = 0.0f;
    if (k < S1) {
      const float cp = scdf[k], cn = scdf[k + 1];
      a_in = fmaxf(fdiv(fsub(cp, cn), fadd(cp, 1e-10f)), 0.0f);
      const float dm = c.dmid[q];
      const float px = fadd(c.ro[r * 3], fmul(c.rd[r * 3], dm)), py = fadd(c.ro[r * 3 + 1], fmul(c.rd[r * 3 + 1], dm)),
                  pz = fadd(c.ro[r * 3 + 2], fmul(c.rd[r * 3 + 2], dm));
      inside = norm3_ref(px, py, pz) <= c.r_obj;
    }
    float alpha;
    if (inside) {
      alpha = a_in;
#pragma unroll
      for (int e = 0; e < 3; ++e) srad[k * 3 + e] = c.rad_m[q * 3 + e];
    } else {
      const float dist = k + 1 < M ? fsub(c.d_out[q + R], dk) : 1e10f;
      alpha = fsub(1.0f, expf(fmul(-softplus1(c.sig_o[q]), dist)));
#pragma unroll
      for (int e = 0; e < 3; ++e) srad[k * 3 + e] = c.rad_o[q * 3 + e];
    }
    sal[k] = alpha;
    if (o.alpha) o.alpha[ro * M + k] = alpha;
  }
  if (calc_normal) {
    for (int k = l; k < Nl; k += NL) {
      const int64_t q = (int64_t)k * R + r;
      float x = c.nab_f[q * 3 + 0], y = c.nab_f[q * 3 + 1], z = c.nab_f[q * 3 + 2];
      normalize3(x, y, z);
      snrm[k * 3 + 0] = x;
      snrm[k * 3 + 1] = y;
      snrm[k * 3 + 2] = z;
    }
  }
  __syncthreads();
  if (l == 0 && live) {
    double T = 1.0, acc = 0.0, rgb0 = 0.0, rgb1 = 0.0, rgb2 = 0.0, n0 = 0.0, n1 = 0.0, n2 = 0.0;
    for (int k = 0; k < M; ++k) {
      const float alpha = sal[k];
      const float w = fmul(alpha, (float)T);
      T *= (double)fadd(fsub(1.0f, alpha), 1e-10f);
      rgb0 += (double)fmul(w, srad[k * 3 + 0]);
      rgb1 += (double)fmul(w, srad[k * 3 + 1]);
      rgb2 += (double)fmul(w, srad[k * 3 + 2]);
      acc += (double)w;
      if (calc_normal && k < Nn) {
        n0 += (double)fmul(snrm[k * 3 + 0], w);
        n1 += (double)fmul(snrm[k * 3 + 1], w);
        n2 += (double)fmul(snrm[k * 3 + 2], w);
      }
      sal[k] = w;
    }
    const float accf = (float)acc;
    const float denom = fadd(accf, 1e-10f);
    double depth = 0.0;
    for (int k = 0; k < M; ++k) depth += (double)fmul(fdiv(sal[k], denom), sdo[k]);
    float q0 = (float)rgb0, q1 = (float)rgb1, q2 = (float)rgb2;
    if (white_bkgd) {
      const float bg = fsub(1.0f, accf);
      q0 = fadd(q0, bg); q1 = fadd(q1, bg); q2 = fadd(q2, bg);
    }
    o.rgb[ro * 3 + 0] = q0;
    o.rgb[ro * 3 + 1] = q1;
    o.rgb[ro * 3 + 2] = q2;
    o.depth[ro] = (float)depth;
    o.acc[ro] = accf;
    if (calc_normal && o.normals) {
      o.normals[ro * 3 + 0] = (float)n0;
      o.normals[ro * 3 + 1] = (float)n1;
      o.normals[ro * 3 + 2] = (float)n2;
    }
  }
  __syncthreads();
  // detailed per-sample outputs, ray-major
  for (int k = l; k < Ml; k += NL) {
    const int64_t q = (int64_t)k * R + r;
    if (o.weights) o.weights[ro * M + k] = sal[k];
    if (o.d_final) o.d_final[ro * M + k] = sdo[k];
    if (o.radiance) {
      o.radiance[(ro * M + k) * 3 + 0] = srad[k * 3 + 0];
      o.radiance[(ro * M + k) * 3 + 1] = srad[k * 3 + 1];
      o.radiance[(ro * M + k) * 3 + 2] = srad[k * 3 + 2];
    }
    if (o.sigma_out) o.sigma_out[ro * M + k] = c.sig_o[q];
    if (o.radiance_bg) {
      o.radiance_bg[(ro * M + k) * 3 + 0] = c.rad_o[q * 3 + 0];
      o.radiance_bg[(ro * M + k) * 3 + 1] = c.rad_o[q * 3 + 1];
      o.radiance_bg[(ro * M + k) * 3 + 2] = c.rad_o[q * 3 + 2];
    }
  }
  for (int i = l; i < Sl; i += NL) {
    const int64_t q = (int64_t)i * R + r;
    if (o.sdf) o.sdf[ro * S + i] = c.sdf_f[q];
    if (o.nablas) {
      o.nablas[(ro * S + i) * 3 + 0] = c.nab_f[q * 3 + 0];
      o.nablas[(ro * S + i) * 3 + 1] = c.nab_f[q * 3 + 1];
      o.nablas[(ro * S + i) * 3 + 2] = c.nab_f[q * 3 + 2];
    }
  }
}

template __global__ void neus_composite_outside_w<1>(NeusChunk, NeusOut, const float*, float, int, int);
template __global__ void neus_composite_outside_w<4>(NeusChunk, NeusOut, const float*, float, int, int);

// compositing with the background merged in (neus.py:325-343, :346-380)
__global__ __launch_bounds__(64) void neus_composite_outside(NeusChunk c, NeusOut o, const float* __restrict__ s_dev,
                                                             float s_val, int calc_normal, int white_bkgd) {
  const float s_inv = s_dev ? *s_dev : s_val;
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= c.R) return;
  const int S = c.S, S1 = S - 1, M = S1 + c.N_out;
  const int64_t R = c.R;
  const int64_t ro = o.ray0 + r;
  const float ox = c.ro[r * 3], oy = c.ro[r * 3 + 1], oz = c.ro[r * 3 + 2];
  const float dx = c.rd[r * 3], dy = c.rd[r * 3 + 1], dz = c.rd[r * 3 + 2];
  double T = 1.0, acc = 0.0, rgb0 = 0.0, rgb1 = 0.0, rgb2 = 0.0, n0 = 0.0, n1 = 0.0, n2 = 0.0;
  float cprev = sigmoidf_ref(fmul(c.sdf_f[r], s_inv));
  if (o.cdf) o.cdf[ro * S] = cprev;
  const int Nn = M < S ? M : S;  // normals use min(#weights, #nablas) samples (neus.py:364-366)
  for (int k = 0; k < M; ++k) {
    const int64_t q = (int64_t)k * R + r;
    const float dk = c.d_out[q];
    const float dist = k + 1 < M ? fsub(c.d_out[q + R], dk) : 1e10f;
    const float a_out = fsub(1.0f, expf(fmul(-softplus1(c.sig_o[q]), dist)));
    float alpha, r0, r1, r2;
    bool inside = false;
    float a_in = 0.f;
    if (k < S1) {
      const float cn = sigmoidf_ref(fmul(c.sdf_f[(int64_t)(k + 1) * R + r], s_inv));
      a_in = fmaxf(fdiv(fsub(cprev, cn), fadd(cprev, 1e-10f)), 0.0f);
      if (o.cdf) o.cdf[ro * S + k + 1] = cn;
      cprev = cn;
      const float dm = c.dmid[q];
      const float px = fadd(ox, fmul(dx, dm)), py = fadd(oy, fmul(dy, dm)), pz = fadd(oz, fmul(dz, dm));
      inside = norm3_ref(px, py, pz) <= c.r_obj;
    }
    if (inside) {
      alpha = a_in;
      r0 = c.rad_m[q * 3 + 0]; r1 = c.rad_m[q * 3 + 1]; r2 = c.rad_m[q * 3 + 2];
    } else {
      alpha = a_out;
      r0 = c.rad_o[q * 3 + 0]; r1 = c.rad_o[q * 3 + 1]; r2 = c.rad_o[q * 3 + 2];
    }
    const float w = fmul(alpha, (float)T);
    T *= (double)fadd(fsub(1.0f, alpha), 1e-10f);
    rgb0 += (double)fmul(w, r0);
    rgb1 += (double)fmul(w, r1);
    rgb2 += (double)fmul(w, r2);
    acc += (double)w;
    if (calc_normal && k < Nn) {
      float x = c.nab_f[(int64_t)k * R * 3 + r * 3 + 0], y = c.nab_f[(int64_t)k * R * 3 + r * 3 + 1],
            z = c.nab_f[(int64_t)k * R * 3 + r * 3 + 2];
      normalize3(x, y, z);
      n0 += (double)fmul(x, w);
      n1 += (double)fmul(y, w);
      n2 += (double)fmul(z, w);
    }
    c.wtmp[q] = w;
    if (o.alpha) o.alpha[ro * M + k] = alpha;
    if (o.weights) o.weights[ro * M + k] = w;
    if (o.d_final) o.d_final[ro * M + k] = dk;
    if (o.radiance) {
      o.radiance[(ro * M + k) * 3 + 0] = r0;
      o.radiance[(ro * M + k) * 3 + 1] = r1;
      o.radiance[(ro * M + k) * 3 + 2] = r2;
    }
    if (o.sigma_out) o.sigma_out[ro * M + k] = c.sig_o[q];
    if (o.radiance_bg) {
      o.radiance_bg[(ro * M + k) * 3 + 0] = c.rad_o[q * 3 + 0];
      o.radiance_bg[(ro * M + k) * 3 + 1] = c.rad_o[q * 3 + 1];
      o.radiance_bg[(ro * M + k) * 3 + 2] = c.rad_o[q * 3 + 2];
    }
  }
  const float accf = (float)acc;
  const float denom = fadd(accf, 1e-10f);
  double depth = 0.0;
  for (int k = 0; k < M; ++k) {
    const int64_t q = (int64_t)k * R + r;
    depth += (double)fmul(fdiv(c.wtmp[q], denom), c.d_out[q]);
  }
  float q0 = (float)rgb0, q1 = (float)rgb1, q2 = (float)rgb2;
  if (white_bkgd) {
    const float bg = fsub(1.0f, accf);
    q0 = fadd(q0, bg); q1 = fadd(q1, bg); q2 = fadd(q2, bg);
  }
  o.rgb[ro * 3 + 0] = q0;
  o.rgb[ro * 3 + 1] = q1;
  o.rgb[ro * 3 + 2] = q2;
  o.depth[ro] = (float)depth;
  o.acc[ro] = accf;
  if (calc_normal && o.normals) {
    o.normals[ro * 3 + 0] = (float)n0;
    o.normals[ro * 3 + 1] = (float)n1;
    o.normals[ro * 3 + 2] = (float)n2;
  }
  for (int i = 0; i < S; ++i) {
    const int64_t q = (int64_t)i * R + r;
    if (o.sdf) o.sdf[ro * S + i] = c.sdf_f[q];
    if (o.nablas) {
      o.nablas[(ro * S + i) * 3 + 0] = c.nab_f[q * 3 + 0];
      o.nablas[(ro * S + i) * 3 + 1] = c.nab_f[q * 3 + 1];
      o.nablas[(ro * S + i) * 3 + 2] = c.nab_f[q * 3 + 2];
    }
  }
}

// sorted sample depths, sample-major [S][R] -> ray-major rows of the output (training sample pass)
__global__ void neus_write_dall(const float* __restrict__ dv, int64_t R, int S, int64_t ray0, float* __restrict__ out) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= (int64_t)S * R) return;
  const int64_t s = q / R, r = q - s * R;
  out[(ray0 + r) * S + s] = dv[q];
}

// ---------------------------------------------------------------------------------------------
// generic sample_pdf entry (rend_util.py:255-292), bins/weights ray-major [R][L], u [N]
// ---------------------------------------------------------------------------------------------
// u: shared sorted uniforms (u_stride 0, det=True) or per-row uniforms u[r * u_stride + k] in any
// order (det=False): each of those is inverted by its own cumsum walk (weights stay read-only)
__global__ void sample_pdf_kernel(const float* __restrict__ bins, const float* __restrict__ weights, int64_t R, int L,
                                  const float* __restrict__ u, int64_t u_stride, int N, float* __restrict__ out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const float* wr = weights + r * (L - 1);
  const float total = aten_row_sum(L - 1, [&](int i) { return fadd(wr[i], 1e-5f); });
  if (!u_stride) {
    sample_pdf_ray(bins + r * L, wr, 1, L, total, u, N, out + r * N, 1);
    return;
  }
  const float* br = bins + r * L;
  for (int k = 0; k < N; ++k) {
    const float uk = u[r * u_stride + k];
    sample_pdf_ray(br, wr, 1, L, total, &uk, 1, out + r * N + k, 1);
  }
}

// ---------------------------------------------------------------------------------------------
// host orchestration
// ---------------------------------------------------------------------------------------------
static size_t align_up(size_t x) { return (x + 255) & ~(size_t)255; }

NeusPlan neus_plan(const NrNeusArgs& a, int64_t Rc) {
  NeusPlan p{};
  const bool direct = a.upsample_algo != NR_UPSAMPLE_OFFICIAL;
  const int n_up0 = a.N_upsample_iters > 0 ? a.N_importance / a.N_upsample_iters : 0;
  const int S = direct ? a.N_samples + a.N_importance : a.N_samples + a.N_upsample_iters * n_up0;
  const int n_nog = a.upsample_algo == NR_UPSAMPLE_DIRECT_MORE ? a.N_nograd_samples : 0;
  p.Rc = Rc;
  size_t off = 0;
  auto take = [&](size_t floats) { size_t o = off; off = align_up(off + floats * 4); return o; };
  p.o_ro = take(Rc * 3);
  p.o_rd = take(Rc * 3);
  p.o_near = take(Rc);
  p.o_far = take(Rc);
  p.o_dv = take((size_t)S * Rc);
  p.o_sv = take((size_t)S * Rc);
  p.o_wtmp = take((size_t)(S > n_nog ? S : n_nog) * Rc);
  const int n_up = direct ? a.N_importance : (a.N_upsample_iters > 0 ? a.N_importance / a.N_upsample_iters : 0);
  p.o_dnew = take((size_t)(n_up > 0 ? n_up : 1) * Rc);
  p.o_snew = take((size_t)(n_up > 0 ? n_up : 1) * Rc);
  p.o_pts = take((size_t)S * Rc * 3);
  p.o_mids = take((size_t)(S - 1) * Rc * 3);
  p.o_dmid = take((size_t)(S - 1) * Rc);
  p.o_sdf_f = take((size_t)S * Rc);
  p.o_nab_f = take((size_t)S * Rc * 3);
  p.o_sdf_m = take((size_t)(S - 1) * Rc);
  p.o_nab_m = take((size_t)(S - 1) * Rc * 3);
  p.o_feat_m = take((size_t)(S - 1) * Rc * 256);
  p.o_rad_m = take((size_t)(S - 1) * Rc * 3);
  const int M = S - 1 + a.N_outside;
  // weights of all M samples; direct_more also writes its n_nog-1 no-grad weights here first
  p.o_wtmp = a.N_outside > 0 ? take((size_t)(M > n_nog ? M : n_nog) * Rc) : p.o_wtmp;
  p.o_dout = take((size_t)(a.N_outside > 0 ? (M > n_nog ? M : n_nog) : (n_nog > 0 ? n_nog : 1)) * Rc);
  p.o_x4 = take((size_t)(a.N_outside > 0 ? M : 1) * Rc * 4);
  p.o_sigo = take((size_t)(a.N_outside > 0 ? M : 1) * Rc);
  p.o_rado = take((size_t)(a.N_outside > 0 ? M : 1) * Rc * 3);
  const size_t Mo = (size_t)(a.N_outside > 0 ? M : 1) * Rc;
  p.o_slot = take(Mo);
  p.o_x4c = take(Mo * 4);
  p.o_vdc = take(Mo * 3);
  p.o_sigc = take(Mo);
  p.o_radc = take(Mo * 3);
  p.o_cnt = take(1);
  const size_t Mm = (size_t)(S - 1) * Rc;
  p.o_mslot = take(Mm);
  p.o_midc = take(Mm * 3);
  p.o_mvd = take(Mm * 3);
  p.o_mrad = take(Mm * 3);
  p.o_mcnt = take(1);
  p.o_ptsn = take((size_t)(n_nog > 0 ? n_nog : 1) * Rc * 3);
  p.o_sn = take((size_t)(n_nog > 0 ? n_nog : 1) * Rc);
  p.o_idv = take((size_t)S * Rc);
  p.o_nsort = take((size_t)S * Rc * 3);
  p.o_dv2 = take((size_t)S * Rc);  // merge ping-pong buffers
  p.o_sv2 = take((size_t)S * Rc);
  p.o_idv2 = take((size_t)S * Rc);
  const size_t tiles = neus_deferred(a, Rc) ? ((size_t)S * Rc + 15) / 16 : 1;
  p.o_slabs = take(neus_deferred(a, Rc) ? tiles * (kSlabColBytes / 4) : 1);  // 100 KB per 16-slot tile
  // flags per sample slot; the list (neus_point_list) pads each 1024-slot segment to 16 entries
  const size_t slots = neus_deferred(a, Rc) ? (size_t)S * Rc : 1;
  p.o_tflag = take(slots);
  p.o_tiles = take(slots + 16 * ((slots + 1023) / 1024));
  p.o_tcnt = take(1);
  p.o_mlp = off;
  p.total = off + nr_mlp_workspace_bytes(1);
  return p;
}

int neus_total_samples(const NrNeusArgs& a) {
  const bool direct = a.upsample_algo != NR_UPSAMPLE_OFFICIAL;
  const int n_up0 = a.N_upsample_iters > 0 ? a.N_importance / a.N_upsample_iters : 0;
  return direct ? a.N_samples + a.N_importance : a.N_samples + a.N_upsample_iters * n_up0;
}

// official_solution, render mode without the per-sample nablas (detailed outputs), the f16x3 softplus
// net, and slots that tile exactly (R % 16 == 0: every launch starts a tile).  With NeRF++ the tiles
// are flagged after the background net (neus_sample_need_outside); not with its detailed outputs.
bool neus_deferred(const NrNeusArgs& a, int64_t R) {
  return a.upsample_algo == NR_UPSAMPLE_OFFICIAL && !a.sample_only && !a.nablas_out && !a.no_mid_skip &&
         !a.no_defer && !(a.N_outside > 0 && (a.sigma_out || a.radiance_bg_out || a.radiance_out)) && a.sdf &&
         a.sdf->precision == NR_PREC_F16X3 && !a.sdf->siren && R > 0 && R % 16 == 0;
}

}  // namespace nr
