// neurecon_amd — training path kernels: the per-point / per-ray arithmetic of
// the NeuS training step's forward and backward, between the layer GEMMs (plain [P, K] x [K, N]
// products issued to hipBLASLt by the host).
//
// What the reference computes (models/frameworks/neus.py:417-485, models/base.py:265-282): the SDF
// net's nablas with create_graph=True, so the eikonal loss and the radiance net (which eats the
// nablas) differentiate THROUGH the input gradient -- a double backward.  The host formulates it as
// reverse mode over the (primal, tangent) network:
//   primal   z_l = W_l hin_l + b_l,  h_l = softplus100(z_l),  s_l = softplus100'(z_l)
//   nabla    g_l = W_{l+1}^T delta_{l+1} (skip-split at layer 4),  delta_l = s_l * g_l,
//            nabla = J_emb(x)^T (W_0^T delta_0 + skip part)
//   tangent  hdot_0 = J_emb(x) grad_nabla,  zdot_l = W_l hdot_in_l,  hdot_l = s_l * zdot_l
//   adjoint  zbar_l = hbar_l * s_l + g_l * zdot_l * s'_l   (s'_l = 100 s_l (1 - s_l), 0 on torch's
//            linear branch: softplus_double_backward), dW_l = zbar_l^T hin_l + delta_l^T hdot_in_l
// This file holds every elementwise step of that recipe plus the NeuS compositing forward/backward.
#include <cmath>

#include "nr_common.h"

namespace nr {
namespace {

constexpr int kBlk = 256;

inline dim3 grid1(int64_t n) { return dim3((unsigned)((n + kBlk - 1) / kBlk)); }

// positional encoding feature f of [x, sin(2^0 x), cos(2^0 x), ..., sin(2^{F-1} x), cos(2^{F-1} x)]
// (models/base.py:14-64; F < 0: identity, 3 features)
__device__ float emb_f(int f, const float (&x)[3], int nfreq) {
  if (f < 3) return x[f];
  const int fp = f - 3, band = fp / 6, m = fp - band * 6, c = m % 3;
  const float v = fmul(x[c], (float)(1 << band));
  return m < 3 ? sinf(v) : cosf(v);
}

// The embedding kernels run one 64-lane wave per point, a lane per feature (r05: one thread per
// element indexed p = i / ldo paid a 64-bit division per element, one thread per point for the vjp
// walked its row serially: 23 / 31 / 46 us per 131 k-point training step)
constexpr int kEmbPts = 4;  // points (waves) per 256-thread block
// grid-stride over points: ~2 k workgroups, each wave walking its points (one wave per point as a
// launch was wave-dispatch bound)
inline dim3 emb_grid(int64_t P) { return dim3((unsigned)std::min<int64_t>((P + kEmbPts - 1) / kEmbPts, 2048)); }
__device__ __forceinline__ float emb_wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// out[p * ldo + f]: features f < nf, zeros up to ldo (ldo >= nf; the training GEMMs' padded blocks)
__global__ __launch_bounds__(256) void embed_kernel(const float* __restrict__ x, int64_t P, int nfreq,
                                                    float* __restrict__ out, int ldo) {
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  const int lane = threadIdx.x & 63;
  for (int64_t p = (int64_t)blockIdx.x * kEmbPts + (threadIdx.x >> 6); p < P; p += (int64_t)gridDim.x * kEmbPts) {
    const float xs[3] = {x[p * 3], x[p * 3 + 1], x[p * 3 + 2]};
    for (int f = lane; f < ldo; f += 64) out[p * ldo + f] = f < nf ? emb_f(f, xs, nfreq) : 0.0f;
  }
}

// J_emb(x) v: d/dt embed(x + t v) (the tangent seed of the double backward)
__global__ __launch_bounds__(256) void embed_jvp_kernel(const float* __restrict__ x, const float* __restrict__ v,
                                                        int64_t P, int nfreq, float* __restrict__ out, int ldo) {
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  const int lane = threadIdx.x & 63;
  for (int64_t p = (int64_t)blockIdx.x * kEmbPts + (threadIdx.x >> 6); p < P; p += (int64_t)gridDim.x * kEmbPts)
  for (int f = lane; f < ldo; f += 64) {
    float o = 0.0f;
    if (f < 3) {
      o = v[p * 3 + f];
    } else if (f < nf) {
      const int fp = f - 3, band = fp / 6, m = fp - band * 6, c = m % 3;
      const float freq = (float)(1 << band);
      const float a = fmul(x[p * 3 + c], freq);
      const float d = m < 3 ? cosf(a) : -sinf(a);
      o = fmul(fmul(v[p * 3 + c], d), freq);
    }
    out[p * ldo + f] = o;
  }
}

// J_emb(x)^T (e0 + s1 e1) -> [P, 3] (autograd's Sin/Cos backward then the Mul by the frequency): each
// lane forms its feature's contribution, the three components are summed over the wave by a fixed
// butterfly
__device__ __forceinline__ void embed_vjp_acc(int f, float gf, const float (&xp)[3], float (&n)[3]) {
  if (f < 3) {
    n[f] = fadd(n[f], gf);
    return;
  }
  const int fp = f - 3, band = fp / 6, m = fp - band * 6, c = m % 3;
  const float freq = (float)(1 << band);
  const float a = fmul(xp[c], freq);
  const float contrib = m < 3 ? fmul(fmul(gf, cosf(a)), freq) : fmul(fmul(gf, -sinf(a)), freq);
  n[c] = fadd(n[c], contrib);
}

__global__ __launch_bounds__(256) void embed_vjp_kernel(const float* __restrict__ x, const float* __restrict__ e0,
                                                        int ld0, const float* __restrict__ e1, int ld1, float s1,
                                                        int64_t P, int nfreq, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  for (int64_t p = (int64_t)blockIdx.x * kEmbPts + (threadIdx.x >> 6); p < P; p += (int64_t)gridDim.x * kEmbPts) {
  const float xp[3] = {x[p * 3], x[p * 3 + 1], x[p * 3 + 2]};
  float n[3] = {0.f, 0.f, 0.f};
  for (int f = lane; f < nf; f += 64) {
    float gf = e0[p * ld0 + f];
    if (e1) gf = fadd(gf, fmul(e1[p * ld1 + f], s1));
    embed_vjp_acc(f, gf, xp, n);
  }
  n[0] = emb_wave_sum(n[0]);
  n[1] = emb_wave_sum(n[1]);
  n[2] = emb_wave_sum(n[2]);
  if (lane == 0) {
    out[p * 3 + 0] = n[0];
    out[p * 3 + 1] = n[1];
    out[p * 3 + 2] = n[2];
  }
  }
}

// Softplus(beta=100, threshold=20) (base.py:202) and torch's softplus_backward factor
// e / (e + 1), e = exp(100 z) (1 on the linear branch)
__global__ void softplus100_kernel(const float* __restrict__ z, int64_t n, float* __restrict__ h,
                                   float* __restrict__ s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float zi = z[i];
  const float t = fmul(zi, 100.0f);
  if (t > 20.0f) {
    h[i] = zi;
    s[i] = 1.0f;
  } else {
    const float e = expf(t);
    h[i] = fdiv(log1pf(e), 100.0f);
    s[i] = fdiv(e, fadd(e, 1.0f));
  }
}

// out[p, j] = a[p, col0 + j] * scale (* s[p, j])
__global__ void scale_cols_kernel(const float* __restrict__ a, int64_t P, int lda, int col0, int ncols,
                                  const float* __restrict__ s, float scale, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * ncols) return;
  const int64_t p = i / ncols;
  const int j = (int)(i - p * ncols);
  float v = a[p * lda + col0 + j];
  if (scale != 1.0f) v = fmul(v, scale);
  if (s) v = fmul(v, s[i]);
  out[i] = v;
}

// zbar = hbar * s + g * zdot * 100 s (1 - s)   (hbar rows of stride ldh; the rest [P, n] dense)
__global__ void softplus_adjoint_kernel(const float* __restrict__ hbar, int ldh, const float* __restrict__ s,
                                        const float* __restrict__ g, const float* __restrict__ zdot, int64_t P, int n,
                                        float* __restrict__ zbar) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * n) return;
  const int64_t p = i / n;
  const int j = (int)(i - p * n);
  const float si = s[i];
  const float d2 = fmul(fmul(si, fsub(1.0f, si)), 100.0f);  // sigmoid_backward * beta; 0 where s == 1
  float v = fmul(hbar[p * ldh + j], si);
  if (g) v = fadd(v, fmul(fmul(g[i], zdot[i]), d2));
  zbar[i] = v;
}

// column sums of a row-major [P, n] gradient (bias gradients): block b sums its slab of rows per column
// (threads across columns: coalesced rows), then one thread per column sums the kColBlocks partials
constexpr int kColBlocks = 1024;
__global__ void colsum_partial_kernel(const float* __restrict__ a, int64_t P, int n, float* __restrict__ part) {
  const int64_t rows = (P + kColBlocks - 1) / kColBlocks;
  const int64_t r0 = (int64_t)blockIdx.x * rows, r1 = r0 + rows < P ? r0 + rows : P;
  for (int c = threadIdx.x; c < n; c += blockDim.x) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};  // 8 loads in flight per thread
    int64_t r = r0;
    for (; r + 8 <= r1; r += 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += a[(r + k) * n + c];
    for (; r < r1; ++r) acc[0] += a[r * n + c];
    part[(int64_t)blockIdx.x * n + c] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  }
}
// 1024 threads per 64 columns: 16 partial-row groups per column (64 partials each, 8 loads in
// flight), combined through LDS in a fixed order
__global__ void colsum_final_kernel(const float* __restrict__ part, int n, float* __restrict__ out) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, grp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if (c < n)
    for (int b = grp * (kColBlocks / 16); b < (grp + 1) * (kColBlocks / 16); b += 8)
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += part[(int64_t)(b + k) * n + c];
  red[grp][cl] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
  __syncthreads();
  if (grp == 0 && c < n) {
    float t = 0.0f;
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    out[c] = t;
  }
}

// SirenLayer activation (base.py:84-115): h = sin(30 z), s = dh/dz = 30 cos(30 z)
__global__ void sine30_kernel(const float* __restrict__ z, int64_t n, float* __restrict__ h, float* __restrict__ s) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const float a = fmul(30.0f, z[i]);
  h[i] = sinf(a);
  s[i] = fmul(30.0f, cosf(a));
}

// the softplus_adjoint_kernel of a sine layer: d2 = ds/dz = -900 sin(30 z) = -900 h
__global__ void sine_adjoint_kernel(const float* __restrict__ hbar, int ldh, const float* __restrict__ s,
                                    const float* __restrict__ h, const float* __restrict__ g,
                                    const float* __restrict__ zdot, int64_t P, int n, float* __restrict__ zbar) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * n) return;
  const int64_t p = i / n;
  const int j = (int)(i - p * n);
  float v = fmul(hbar[p * ldh + j], s[i]);
  if (g) v = fadd(v, fmul(fmul(g[i], zdot[i]), fmul(-900.0f, h[i])));
  zbar[i] = v;
}

__global__ void mul_kernel(const float* __restrict__ a, const float* __restrict__ b, int64_t n, float* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) out[i] = fmul(a[i], b[i]);
}

// y = relu(y) in place (mode 0), g *= (y > 0) (mode 1), y = sigmoid(y) in place (mode 2),
// g *= y (1 - y) (mode 3)
__global__ void act_kernel(float* __restrict__ y, float* __restrict__ g, int64_t n, int mode) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  switch (mode) {
    case 0: y[i] = fmaxf(y[i], 0.0f); break;
    case 1: if (!(y[i] > 0.0f)) g[i] = 0.0f; break;
    case 2: y[i] = sigmoidf_ref(y[i]); break;
    default: g[i] = fmul(g[i], fmul(y[i], fsub(1.0f, y[i]))); break;
  }
}

// weight_norm(dim=0) of a batch of layers: one wave per row (rows of all layers concatenated)
struct WnBatch {
  NrWnLayer l[NR_WN_MAX];
  int row0[NR_WN_MAX + 1];
  int n;
};
__device__ __forceinline__ int wn_layer(const WnBatch& b, int row) {
  int i = 0;
  while (i + 1 < b.n && row >= b.row0[i + 1]) ++i;
  return i;
}
// lane-strided sum, then a fixed butterfly over the wave
__device__ __forceinline__ float wave_sum64(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__global__ __launch_bounds__(256) void weight_norm_fwd_kernel(WnBatch b) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= b.row0[b.n]) return;
  const int li = wn_layer(b, row);
  const NrWnLayer& L = b.l[li];
  const int r = row - b.row0[li];
  const float* v = L.v + (int64_t)r * L.cols;
  float ss = 0.0f;
  for (int c = lane; c < L.cols; c += 64) ss = fmaf(v[c], v[c], ss);
  const float nrm = __fsqrt_rn(wave_sum64(ss));
  const float s = fdiv(L.g[r], nrm);
  float* w = L.w + (int64_t)r * L.cols;
  for (int c = lane; c < L.cols; c += 64) w[c] = fmul(v[c], s);
  if (lane == 0) L.norm[r] = nrm;
}
__global__ __launch_bounds__(256) void weight_norm_bwd_kernel(WnBatch b) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (row >= b.row0[b.n]) return;
  const int li = wn_layer(b, row);
  const NrWnLayer& L = b.l[li];
  const int r = row - b.row0[li];
  const float* v = L.v + (int64_t)r * L.cols;
  float* gv = L.grad_v + (int64_t)r * L.cols;
  if (!L.grad_w) {
    for (int c = lane; c < L.cols; c += 64) gv[c] = 0.0f;
    if (lane == 0) L.grad_g[r] = 0.0f;
    return;
  }
  const float* gw = L.grad_w + (int64_t)r * L.cols;
  float dot = 0.0f;
  for (int c = lane; c < L.cols; c += 64) dot = fmaf(gw[c], v[c], dot);
  dot = wave_sum64(dot);
  const float nrm = L.norm[r];
  const float a = fdiv(L.g[r], nrm), bcoef = fdiv(dot, fmul(nrm, nrm));
  for (int c = lane; c < L.cols; c += 64) gv[c] = fmul(a, fsub(gw[c], fmul(v[c], bcoef)));
  if (lane == 0) L.grad_g[r] = fdiv(dot, nrm);
}

// Adam over a batch of parameter tensors: each workgroup owns kAdamChunk consecutive elements of one
// tensor (chunk0[i] = first chunk of tensor i), thread t updates elements t, t + 256, ... of the chunk
// (coalesced), the update in the order of torch's fused Adam (FusedAdamKernel, ADAM_MODE::ORIGINAL)
constexpr int kAdamChunk = 4096;
struct AdamBatch {
  NrAdamTensor t[NR_ADAM_MAX];
  int chunk0[NR_ADAM_MAX + 1];
  int n;
  float beta1, beta2, omb1, omb2, eps, wd, step_size, bc2_sqrt;  // omb = 1 - beta, formed in double as torch
};
__global__ __launch_bounds__(256) void adam_kernel(AdamBatch b) {
  const int c = blockIdx.x;
  int i = 0;
  while (i + 1 < b.n && c >= b.chunk0[i + 1]) ++i;
  const NrAdamTensor& T = b.t[i];
  const int64_t e0 = (int64_t)(c - b.chunk0[i]) * kAdamChunk;
  const int64_t e1 = e0 + kAdamChunk < T.n ? e0 + kAdamChunk : T.n;
  for (int64_t e = e0 + threadIdx.x; e < e1; e += 256) {
    const float p = T.param[e];
    float g = T.grad[e];
    if (b.wd != 0.0f) g = fadd(g, fmul(b.wd, p));
    const float m = fadd(fmul(b.beta1, T.exp_avg[e]), fmul(b.omb1, g));
    const float v = fadd(fmul(b.beta2, T.exp_avg_sq[e]), fmul(fmul(b.omb2, g), g));
    const float denom = fadd(fdiv(__fsqrt_rn(v), b.bc2_sqrt), b.eps);
    T.exp_avg[e] = m;
    T.exp_avg_sq[e] = v;
    T.param[e] = fsub(p, fdiv(fmul(b.step_size, m), denom));
  }
}

// RadianceNet input cat([x, embed_view(v), normals, feature]) (base.py:379-384), one row per point;
// v is indexed per point.  Without view dirs (view = 0): cat([x, feature]) (base.py:383-384)
__global__ void radiance_input_kernel(const float* __restrict__ x, const float* __restrict__ v,
                                      const float* __restrict__ nrm, const float* __restrict__ feat, int64_t P,
                                      int nfreq_view, int view, int wfeat, float* __restrict__ out) {
  const int nv = view ? (nfreq_view < 0 ? 3 : 3 + 6 * nfreq_view) : 0;
  const int nn = view ? 3 : 0;
  const int ld = 3 + nv + nn + wfeat;
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= P * ld) return;
  const int64_t p = i / ld;
  int f = (int)(i - p * ld);
  float val;
  if (f < 3) {
    val = x[p * 3 + f];
  } else if ((f -= 3) < nv) {
    const float vs[3] = {v[p * 3], v[p * 3 + 1], v[p * 3 + 2]};
    val = emb_f(f, vs, nfreq_view);
  } else if ((f -= nv) < nn) {
    val = nrm[p * 3 + f];
  } else {
    val = feat[p * wfeat + f - nn];
  }
  out[i] = val;
}

// training sample points (neus.py:284-288): pts = o + d t_s, d_mid = (t_s + t_{s-1}) / 2, pts_mid
__global__ void neus_points_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                   const float* __restrict__ d_all, int64_t R, int S, float* __restrict__ pts,
                                   float* __restrict__ mids, float* __restrict__ dmid) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * S) return;
  const int64_t r = i / S;
  const int s = (int)(i - r * S);
  const float t = d_all[i];
#pragma unroll
  for (int k = 0; k < 3; ++k) pts[i * 3 + k] = fadd(ro[r * 3 + k], fmul(rd[r * 3 + k], t));
  if (s + 1 < S) {
    const int64_t m = r * (S - 1) + s;
    const float tm = fmul(0.5f, fadd(d_all[i + 1], t));
    dmid[m] = tm;
#pragma unroll
    for (int k = 0; k < 3; ++k) mids[m * 3 + k] = fadd(ro[r * 3 + k], fmul(rd[r * 3 + k], tm));
  }
}

// NeuS compositing with a differentiable graph (neus.py:28-70, :346-355), one thread per ray.
// sdf [R,S], radiance [R,S-1,3], dmid [R,S-1]; s from the device.  fp64 prefix products / sums
// rounded per element, as in the render kernels.
// One ray per 64-lane wave, everything across the lanes (r05; r03-r04 ran the scans on lane 0: 26 + 78
// us per 512-ray step): the transmittance T_i = prod_{j<i} (1 - alpha_j + 1e-10) is a wave prefix
// product in fp64 over 64-sample segments with a carried running product, the colour / opacity / depth
// sums are per-lane fp64 partials reduced by a fixed butterfly; the backward's suffix sums likewise.
// The association of the fp64 products and sums differs from a sequential walk (relative 1e-16, below
// the per-element fp32 rounding).  LDS: fwd 2 S floats, bwd S doubles + 5 S floats.
__device__ __forceinline__ double wave_incl_prod(double x, int l) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double t = __shfl_up(x, d);
    if (l >= d) x *= t;
  }
  return x;
}
__device__ __forceinline__ double wave_incl_sum_rev(double x, int l) {  // sum over lanes >= l
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const double t = __shfl_down(x, d);
    if (l + d < 64) x += t;
  }
  return x;
}
__device__ __forceinline__ double wave_sum_d(double x) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

__global__ __launch_bounds__(64) void neus_composite_fwd_kernel(const float* __restrict__ sdf, const float* __restrict__ s_dev,
                                          const float* __restrict__ rad, const float* __restrict__ dmid, int64_t R,
                                          int S, int white_bkgd, float* __restrict__ rgb, float* __restrict__ depth,
                                          float* __restrict__ acc, float* __restrict__ w_out,
                                          float* __restrict__ alpha_out, float* __restrict__ cdf_out) {
  extern __shared__ float lds[];
  const int64_t r = blockIdx.x;
  const int l = threadIdx.x, S1 = S - 1;
  const float s = *s_dev;
  const float* sd = sdf + r * S;
  float* lc = lds;      // [S] cdf
  float* lw = lc + S;   // [S] weights
  for (int i = l; i < S; i += 64) {
    const float c = sigmoidf_ref(fmul(sd[i], s));
    lc[i] = c;
    if (cdf_out) cdf_out[r * S + i] = c;
  }
  __syncthreads();
  double Tc = 1.0, c0 = 0.0, c1 = 0.0, c2 = 0.0, a_acc = 0.0;
  for (int b = 0; b < S1; b += 64) {
    const int i = b + l;
    const bool ok = i < S1;
    const int64_t q = r * S1 + (ok ? i : 0);
    const float al = ok ? fmaxf(fdiv(fsub(lc[i], lc[i + 1]), fadd(lc[i], 1e-10f)), 0.0f) : 0.0f;
    const double u = ok ? (double)fadd(fsub(1.0f, al), 1e-10f) : 1.0;
    const double incl = wave_incl_prod(u, l);
    const double excl = __shfl_up(incl, 1);
    const double T = Tc * (l == 0 ? 1.0 : excl);
    const float w = fmul(al, (float)T);
    if (ok) {
      lw[i] = w;
      if (alpha_out) alpha_out[q] = al;
      c0 += (double)fmul(w, rad[q * 3 + 0]);
      c1 += (double)fmul(w, rad[q * 3 + 1]);
      c2 += (double)fmul(w, rad[q * 3 + 2]);
      a_acc += (double)w;
    }
    Tc *= __shfl(incl, 63);
  }
  c0 = wave_sum_d(c0);
  c1 = wave_sum_d(c1);
  c2 = wave_sum_d(c2);
  a_acc = wave_sum_d(a_acc);
  __syncthreads();
  const float accf = (float)a_acc;
  const float den = fadd(accf, 1e-10f);
  double dep = 0.0;
  for (int i = l; i < S1; i += 64) {
    dep += (double)fmul(fdiv(lw[i], den), dmid[r * S1 + i]);
    w_out[r * S1 + i] = lw[i];
  }
  dep = wave_sum_d(dep);
  if (l == 0) {
    float o0 = (float)c0, o1 = (float)c1, o2 = (float)c2;
    if (white_bkgd) {
      const float bg = fsub(1.0f, accf);
      o0 = fadd(o0, bg); o1 = fadd(o1, bg); o2 = fadd(o2, bg);
    }
    rgb[r * 3 + 0] = o0;
    rgb[r * 3 + 1] = o1;
    rgb[r * 3 + 2] = o2;
    depth[r] = (float)dep;
    acc[r] = accf;
  }
}

// backward of the above: grads of rgb [R,3], depth [R], acc [R] and (optional) the visibility
// weights [R,S-1] -> d sdf [R,S], d radiance [R,S-1,3], d s per ray [R] (summed by the host).
// alpha_i = max((c_i - c_{i+1}) / (c_i + 1e-10), 0) (clamp_min passes the gradient where >= 0);
// T = exclusive cumprod of (1 - alpha + 1e-10) (cumprod_backward: suffix sums / input):
//   alpha-bar_i = wbar_i T_i - (sum_{k > i} wbar_k alpha_k T_k) / u_i, then c_i and c_{i+1} receive the
//   quotient rule's terms; c_{i+1}'s total is cn_bar_i + ci_bar_{i+1} (rounded to fp32 as before).
__global__ __launch_bounds__(64) void neus_composite_bwd_kernel(const float* __restrict__ sdf, const float* __restrict__ s_dev,
                                          const float* __restrict__ rad, const float* __restrict__ dmid, int64_t R,
                                          int S, int white_bkgd, const float* __restrict__ g_rgb,
                                          const float* __restrict__ g_depth, const float* __restrict__ g_acc,
                                          const float* __restrict__ g_w, float* __restrict__ d_sdf,
                                          float* __restrict__ d_rad, float* __restrict__ d_s) {
  extern __shared__ double ldsd[];
  const int64_t r = blockIdx.x;
  const int l = threadIdx.x, S1 = S - 1;
  const float s = *s_dev;
  const float* sd = sdf + r * S;
  double* cnb = ldsd;     // [S] cn_bar_{k-1} at k (fp64, as the sequential walk adds it)
  float* c = (float*)(cnb + S);  // [S] cdf
  float* al = c + S;      // [S] alpha
  float* Tt = al + S;     // [S] T (fp32, as the weights use it)
  float* wb = Tt + S;     // [S] weight adjoints
  float* cib = wb + S;    // [S] ci_bar (fp32)
  for (int i = l; i < S; i += 64) c[i] = sigmoidf_ref(fmul(sd[i], s));
  __syncthreads();
  // forward recompute: alpha, T, weights; acc and sum w d
  double Tc = 1.0, a_acc = 0.0, wd = 0.0;
  for (int b = 0; b < S1; b += 64) {
    const int i = b + l;
    const bool ok = i < S1;
    const float a = ok ? fmaxf(fdiv(fsub(c[i], c[i + 1]), fadd(c[i], 1e-10f)), 0.0f) : 0.0f;
    const double u = ok ? (double)fadd(fsub(1.0f, a), 1e-10f) : 1.0;
    const double incl = wave_incl_prod(u, l);
    const double excl = __shfl_up(incl, 1);
    const float T = (float)(Tc * (l == 0 ? 1.0 : excl));
    if (ok) {
      al[i] = a;
      Tt[i] = T;
      const float w = fmul(a, T);
      a_acc += (double)w;
      wd += (double)w * (double)dmid[r * S1 + i];
    }
    Tc *= __shfl(incl, 63);
  }
  a_acc = wave_sum_d(a_acc);
  wd = wave_sum_d(wd);
  const double A = (double)fadd((float)a_acc, 1e-10f);
  const float gr0 = g_rgb ? g_rgb[r * 3 + 0] : 0.f, gr1 = g_rgb ? g_rgb[r * 3 + 1] : 0.f,
              gr2 = g_rgb ? g_rgb[r * 3 + 2] : 0.f;
  const double gd = g_depth ? (double)g_depth[r] : 0.0;
  // white_bkgd: rgb += 1 - acc -> acc receives -sum(g_rgb)
  const double ga = (g_acc ? (double)g_acc[r] : 0.0) - (white_bkgd ? (double)gr0 + gr1 + gr2 : 0.0);
  __syncthreads();
  for (int i = l; i < S1; i += 64) {
    const int64_t q = r * S1 + i;
    const float w = fmul(al[i], Tt[i]);
    double v = (double)gr0 * rad[q * 3 + 0] + (double)gr1 * rad[q * 3 + 1] + (double)gr2 * rad[q * 3 + 2] + ga;
    v += gd * ((double)dmid[q] / A - wd / (A * A));
    if (g_w) v += (double)g_w[q];
    wb[i] = (float)v;
    d_rad[q * 3 + 0] = fmul(w, gr0);
    d_rad[q * 3 + 1] = fmul(w, gr1);
    d_rad[q * 3 + 2] = fmul(w, gr2);
  }
  __syncthreads();
  // alpha-bar from the reverse suffix sums (segments from the end, carried), then the quotient rule
  double carry = 0.0;  // sum over the later segments
  double sbar = 0.0;
  const int nseg = (S1 + 63) / 64;
  for (int sg = nseg - 1; sg >= 0; --sg) {
    const int i = sg * 64 + l;
    const bool ok = i < S1;
    const double t = ok ? (double)wb[i] * al[i] * Tt[i] : 0.0;
    const double incl = wave_incl_sum_rev(t, l);          // sum over lanes >= l of this segment
    const double suffix = carry + (incl - t);              // sum_{k > i}
    if (ok) {
      const double u = (double)fadd(fsub(1.0f, al[i]), 1e-10f);
      const double abar = (double)wb[i] * Tt[i] - suffix / u;
      const float num = fsub(c[i], c[i + 1]), den = fadd(c[i], 1e-10f);
      double ci_bar = 0.0, cn_bar = 0.0;
      if (fdiv(num, den) >= 0.0f) {
        ci_bar = abar / den - abar * num / ((double)den * den);
        cn_bar = -abar / den;
      }
      cib[i] = (float)ci_bar;
      cnb[i + 1] = cn_bar;  // c_{i+1}'s term from alpha_i (completed below)
    }
    carry += __shfl(incl, 0);
  }
  __syncthreads();
  // c_{i+1} collects cn_bar_i plus ci_bar_{i+1} (rounded to fp32); c_0 only ci_bar_0
  for (int k = l; k < S; k += 64) {
    double cb;
    if (k == 0) cb = (double)cib[0];
    else cb = cnb[k] + (k < S1 ? (double)cib[k] : 0.0);
    const float cc = c[k];
    const double g = cb * cc * (1.0 - cc);
    d_sdf[r * S + k] = (float)(g * s);
    sbar += g * sd[k];
  }
  sbar = wave_sum_d(sbar);
  if (l == 0) d_s[r] = (float)sbar;
}

// ---- VolSDF compositing with a graph (volsdf.py:449-506) ----------------------------------------------
// One thread per ray.  sdf [R,S] are the network's values at pts [R,S,3]; with the builtin background
// sphere (volsdf.py:317-325) a sample whose r_bg - |x| is smaller takes that value instead (and then
// passes no gradient to the network).  sigma = sdf_to_sigma(sdf, 1/beta, beta) (volsdf.py:16-35),
// p_i = exp(-relu(sigma_i delta_i)), tau_i = (1 - p_i + 1e-10) prod_{j<i} p_j over the first S-1
// samples; rgb = sum tau radiance[:S-1], depth = sum tau / (sum tau + 1e-10) d, acc = sum tau.  fp64
// prefix products / sums rounded per element, as in the render kernel (volsdf_composite).
__device__ __forceinline__ float vs_sigma_t(float v, float alpha, float beta) {
  const float e = fmul(0.5f, expf(fdiv(-fabsf(v), beta)));
  return fmul(alpha, v >= 0.0f ? e : fsub(1.0f, e));
}
__device__ __forceinline__ float vs_sdf_bg(const float* sdf, const float* pts, int64_t i, int use_bg, float r_bg,
                                           bool& masked) {
  float v = sdf[i];
  masked = false;
  if (use_bg) {
    const float x = pts[i * 3], y = pts[i * 3 + 1], z = pts[i * 3 + 2];
    const float dbg = fsub(r_bg, __fsqrt_rn(fadd(fadd(fmul(x, x), fmul(y, y)), fmul(z, z))));
    if (dbg < v) {
      v = dbg;
      masked = true;
    }
  }
  return v;
}
// With the NeRF++ background (volsdf.py:455-469) the N background samples follow the S inner ones:
// sigma_bg [R,N] (the background net's raw sigma), radiance_bg [R,N,3], d_bg [R,N]; M = S + N samples
// are integrated (p, tau over M-1, sigma over M).  N = 0: the inner samples only.
struct VsBg {
  const float* sig;
  const float* rad;
  const float* d;
  int N;
};
__global__ void volsdf_composite_fwd_kernel(const float* __restrict__ sdf, const float* __restrict__ pts,
                                            const float* __restrict__ beta_dev, const float* __restrict__ rad,
                                            const float* __restrict__ d_all, int64_t R, int S, int use_bg, float r_bg,
                                            int white_bkgd, VsBg bg, float* __restrict__ rgb,
                                            float* __restrict__ depth, float* __restrict__ acc,
                                            float* __restrict__ tau_out, float* __restrict__ p_out,
                                            float* __restrict__ sigma_out, float* __restrict__ sdf_out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const float beta = *beta_dev, alpha = fdiv(1.0f, beta);
  const int M = S + bg.N, M1 = M - 1;
  auto dv = [&](int i) { return i < S ? d_all[r * S + i] : bg.d[r * bg.N + i - S]; };
  auto rv = [&](int i) { return i < S ? rad + (r * S + i) * 3 : bg.rad + (r * bg.N + i - S) * 3; };
  double T = 1.0, a_acc = 0.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
  bool m;
  float sg = vs_sigma_t(vs_sdf_bg(sdf, pts, r * S, use_bg, r_bg, m), alpha, beta);
  for (int i = 0; i < M; ++i) {
    float si;
    if (i < S) {
      const int64_t q = r * S + i;
      const float v = vs_sdf_bg(sdf, pts, q, use_bg, r_bg, m);
      si = vs_sigma_t(v, alpha, beta);
      if (sdf_out) sdf_out[q] = v;
    } else {
      si = bg.sig[r * bg.N + i - S];
    }
    if (sigma_out) sigma_out[r * M + i] = si;
    if (i == 0) continue;
    // sample i-1's interval
    const float p = expf(-fmaxf(fmul(sg, fsub(dv(i), dv(i - 1))), 0.0f));
    const float tau = fmul(fadd(fsub(1.0f, p), 1e-10f), (float)T);
    T *= (double)p;
    const int64_t k = r * M1 + i - 1;
    const float* rr = rv(i - 1);
    c0 += (double)fmul(tau, rr[0]);
    c1 += (double)fmul(tau, rr[1]);
    c2 += (double)fmul(tau, rr[2]);
    a_acc += (double)tau;
    tau_out[k] = tau;
    if (p_out) p_out[k] = p;
    sg = si;
  }
  const float accf = (float)a_acc;
  const float den = fadd(accf, 1e-10f);
  double dep = 0.0;
  for (int i = 0; i < M1; ++i) dep += (double)fmul(fdiv(tau_out[r * M1 + i], den), dv(i));
  float o0 = (float)c0, o1 = (float)c1, o2 = (float)c2;
  if (white_bkgd) {
    const float bg_ = fsub(1.0f, accf);
    o0 = fadd(o0, bg_); o1 = fadd(o1, bg_); o2 = fadd(o2, bg_);
  }
  rgb[r * 3 + 0] = o0;
  rgb[r * 3 + 1] = o1;
  rgb[r * 3 + 2] = o2;
  depth[r] = (float)dep;
  acc[r] = accf;
}

// backward of the above: grads of rgb [R,3], depth [R], acc [R], tau [R,M-1] and the background-applied
// sdf [R,S] (all optional) -> d sdf (network values) [R,S], d radiance [R,S,3] (rows past the first M-1
// samples are 0: volsdf.py:495 uses radiances[..., :-1, :]), d beta per ray [R] (the host sums; both the
// alpha = 1/beta and the psi(beta) paths), and with the NeRF++ background d sigma_bg [R,N] and
// d radiance_bg [R,N,3].  tau_i = u_i P_i with u_i = 1 - p_i + 1e-10 and P_i = prod_{j<i} p_j, so
// pbar_i = P_i (G_i - taubar_i) with G_i = sum_{k>i} taubar_k u_k prod_{i<j<k} p_j (no division by p).
__global__ void volsdf_composite_bwd_kernel(const float* __restrict__ sdf, const float* __restrict__ pts,
                                            const float* __restrict__ beta_dev, const float* __restrict__ rad,
                                            const float* __restrict__ d_all, int64_t R, int S, int use_bg, float r_bg,
                                            int white_bkgd, VsBg bg, const float* __restrict__ g_rgb,
                                            const float* __restrict__ g_depth, const float* __restrict__ g_acc,
                                            const float* __restrict__ g_tau, const float* __restrict__ g_sdf,
                                            float* __restrict__ work, float* __restrict__ d_sdf,
                                            float* __restrict__ d_rad, float* __restrict__ d_beta,
                                            float* __restrict__ d_sig_bg, float* __restrict__ d_rad_bg) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  const float beta = *beta_dev, alpha = fdiv(1.0f, beta);
  const int M = S + bg.N, M1 = M - 1;
  auto dv = [&](int i) { return i < S ? d_all[r * S + i] : bg.d[r * bg.N + i - S]; };
  auto rv = [&](int i) { return i < S ? rad + (r * S + i) * 3 : bg.rad + (r * bg.N + i - S) * 3; };
  auto drv = [&](int i) { return i < S ? d_rad + (r * S + i) * 3 : d_rad_bg + (r * bg.N + i - S) * 3; };
  // work rows: v (bg-applied sdf) [M], sigma [M], p [M], P [M], tau [M]
  float* v = work + r * (5 * M);
  float* sg = v + M;
  float* p = sg + M;
  float* P = p + M;
  float* tau = P + M;
  double T = 1.0, a_acc = 0.0, wd = 0.0;
  for (int i = 0; i < M; ++i) {
    bool m;
    if (i < S) {
      v[i] = vs_sdf_bg(sdf, pts, r * S + i, use_bg, r_bg, m);
      sg[i] = vs_sigma_t(v[i], alpha, beta);
    } else {
      v[i] = 0.0f;
      sg[i] = bg.sig[r * bg.N + i - S];
    }
  }
  for (int i = 0; i < M1; ++i) {
    p[i] = expf(-fmaxf(fmul(sg[i], fsub(dv(i + 1), dv(i))), 0.0f));
    P[i] = (float)T;
    tau[i] = fmul(fadd(fsub(1.0f, p[i]), 1e-10f), P[i]);
    T *= (double)p[i];
    a_acc += (double)tau[i];
  }
  const float accf = (float)a_acc;
  const double A = (double)fadd(accf, 1e-10f);
  for (int i = 0; i < M1; ++i) wd += (double)tau[i] * (double)dv(i);
  const float gr0 = g_rgb ? g_rgb[r * 3 + 0] : 0.f, gr1 = g_rgb ? g_rgb[r * 3 + 1] : 0.f,
              gr2 = g_rgb ? g_rgb[r * 3 + 2] : 0.f;
  const double gd = g_depth ? (double)g_depth[r] : 0.0;
  const double ga = (g_acc ? (double)g_acc[r] : 0.0) - (white_bkgd ? (double)gr0 + gr1 + gr2 : 0.0);
  double G = 0.0, bbar = 0.0;
  const double ib2 = 1.0 / ((double)beta * beta);
  for (int i = M - 1; i >= 0; --i) {
    double vbar = 0.0, sbar = 0.0;
    float* dr = drv(i);
    if (i < M1) {
      const float* rr = rv(i);
      double tb = (double)gr0 * rr[0] + (double)gr1 * rr[1] + (double)gr2 * rr[2] + ga;
      tb += gd * ((double)dv(i) / A - wd / (A * A));
      if (g_tau) tb += (double)g_tau[r * M1 + i];
      dr[0] = fmul(tau[i], gr0);
      dr[1] = fmul(tau[i], gr1);
      dr[2] = fmul(tau[i], gr2);
      const double u = (double)fadd(fsub(1.0f, p[i]), 1e-10f);
      const double pbar = (double)P[i] * (G - tb);
      G = tb * u + (double)p[i] * G;
      const float delta = fsub(dv(i + 1), dv(i));
      if (fmul(sg[i], delta) > 0.0f) sbar = -pbar * (double)p[i] * (double)delta;
      if (i < S && sbar != 0.0) {
        // sigma = alpha psi(v, beta), psi = e or 1 - e, e = 0.5 exp(-|v| / beta)
        const double e = (double)fmul(0.5f, expf(fdiv(-fabsf(v[i]), beta)));
        const double sgn = v[i] > 0.0f ? 1.0 : (v[i] < 0.0f ? -1.0 : 0.0);
        const double psi = v[i] >= 0.0f ? e : 1.0 - e;
        const double br = v[i] >= 0.0f ? 1.0 : -1.0;  // d psi / d e
        vbar = sbar * (double)alpha * br * e * (-sgn / (double)beta);
        bbar += sbar * (psi * (-ib2) + (double)alpha * br * e * fabs((double)v[i]) * ib2);
      }
    } else {
      dr[0] = 0.0f;
      dr[1] = 0.0f;
      dr[2] = 0.0f;
    }
    if (i < S) {
      const int64_t q = r * S + i;
      if (g_sdf) vbar += (double)g_sdf[q];
      bool m;
      (void)vs_sdf_bg(sdf, pts, q, use_bg, r_bg, m);
      d_sdf[q] = m ? 0.0f : (float)vbar;
    } else {
      d_sig_bg[r * bg.N + i - S] = (float)sbar;
    }
  }
  d_beta[r] = (float)bbar;
}

// ---- NeRF++ background in the training step (neus.py:303-343) ------------------------------------
// inputs of the background MLP at the R x M depths d_out (= cat([d_mid, d_vals_out])): p = o + d dir,
// x4 = [p / |p|, 1 / |p|] embedded with 10 log-sampled frequencies (Embedder(input_dim=4)), the view
// direction embedded with 4; inside[k] = |p_k| <= r_obj for the S-1 mid-points (k < n_mid)
__device__ __forceinline__ float emb4_f(int f, const float (&x)[4]) {
  if (f < 4) return x[f];
  const int fp = f - 4, band = fp >> 3, m = fp & 7;
  const float v = fmul(x[m & 3], (float)(1 << band));
  return m < 4 ? sinf(v) : cosf(v);
}
__global__ void nerf_train_input_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                        const float* __restrict__ d_out, int64_t R, int M, int n_mid, float r_obj,
                                        float* __restrict__ x_emb, float* __restrict__ v_emb,
                                        uint8_t* __restrict__ inside) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * M) return;
  const int64_t r = i / M;
  const int k = (int)(i - r * M);
  const float d = d_out[i];
  const float px = fadd(ro[r * 3 + 0], fmul(rd[r * 3 + 0], d)), py = fadd(ro[r * 3 + 1], fmul(rd[r * 3 + 1], d)),
              pz = fadd(ro[r * 3 + 2], fmul(rd[r * 3 + 2], d));
  const float rr = norm3_ref(px, py, pz);
  const float x4[4] = {fdiv(px, rr), fdiv(py, rr), fdiv(pz, rr), fdiv(1.0f, rr)};
  for (int f = 0; f < 84; ++f) x_emb[i * 84 + f] = emb4_f(f, x4);
  const float vs[3] = {rd[r * 3], rd[r * 3 + 1], rd[r * 3 + 2]};
  for (int f = 0; f < 27; ++f) v_emb[i * 27 + f] = emb_f(f, vs, 4);
  if (k < n_mid) inside[r * n_mid + k] = rr <= r_obj ? 1 : 0;
}

// inputs of VolSDF's NeRF++ background net (volsdf.py:456-467): p = o + d_bg dir at the radius rs of
// each sample, x4 = [p / rs, 1 / rs] embedded with 10 frequencies (Embedder(input_dim=4)), the view
// direction with 4
__global__ void volsdf_nerf_input_kernel(const float* __restrict__ ro, const float* __restrict__ rd,
                                         const float* __restrict__ d_bg, const float* __restrict__ rs, int64_t R,
                                         int N, float* __restrict__ x_emb, float* __restrict__ v_emb) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= R * N) return;
  const int64_t r = i / N;
  const float d = d_bg[i], rr = rs[i];
  const float px = fadd(ro[r * 3 + 0], fmul(rd[r * 3 + 0], d)), py = fadd(ro[r * 3 + 1], fmul(rd[r * 3 + 1], d)),
              pz = fadd(ro[r * 3 + 2], fmul(rd[r * 3 + 2], d));
  const float x4[4] = {fdiv(px, rr), fdiv(py, rr), fdiv(pz, rr), fdiv(1.0f, rr)};
  for (int f = 0; f < 84; ++f) x_emb[i * 84 + f] = emb4_f(f, x4);
  const float vs[3] = {rd[r * 3], rd[r * 3 + 1], rd[r * 3 + 2]};
  for (int f = 0; f < 27; ++f) v_emb[i * 27 + f] = emb_f(f, vs, 4);
}

// F.softplus (beta 1, threshold 20) and its derivative (softplus_backward)
__device__ __forceinline__ float sp1(float x) { return x > 20.0f ? x : log1pf(expf(x)); }
__device__ __forceinline__ double sp1_grad(float x) { return x > 20.0f ? 1.0 : 1.0 / (1.0 + exp(-(double)x)); }

// composite with the background merged (neus.py:325-352): sample k < S-1 takes the SDF alpha and the
// radiance net's colour where inside[k], else the background's; k >= S-1 are background samples.
// alpha_out = 1 - exp(-softplus(sigma) dist), dist = d_{k+1} - d_k (1e10 for the last).
// One ray per 64-lane wave, as neus_composite_fwd_kernel (r05; one thread per ray gave a 512-ray
// training batch 8 waves for the chip: 0.35 ms fwd + 0.52 ms bwd per step): the per-sample CDFs,
// alphas (softplus, exp) and colour staging across the lanes, the prefix product and sums on lane 0
// in the per-ray order.  LDS floats: S + 6 M.
__global__ __launch_bounds__(64) void neus_composite_bg_fwd_kernel(
    const float* __restrict__ sdf, const float* __restrict__ s_dev, const float* __restrict__ rad,
    const float* __restrict__ sig_o, const float* __restrict__ rad_o, const float* __restrict__ d_out,
    const uint8_t* __restrict__ inside, int64_t R, int S, int M, int white_bkgd, float* __restrict__ rgb,
    float* __restrict__ depth, float* __restrict__ acc, float* __restrict__ w_out, float* __restrict__ alpha_out,
    float* __restrict__ cdf_out) {
  extern __shared__ float lds[];
  const int64_t r = blockIdx.x;
  const int l = threadIdx.x, S1 = S - 1;
  const float s = *s_dev;
  const float* sd = sdf + r * S;
  const float* dk = d_out + r * M;
  float* c = lds;            // [S] cdf
  float* la = c + S;         // [M] alpha
  float* lw = la + M;        // [M] weights
  float* lcol = lw + M;      // [3 M] colour
  float* ld = lcol + 3 * M;  // [M] depths
  for (int i = l; i < S; i += 64) {
    const float v = sigmoidf_ref(fmul(sd[i], s));
    c[i] = v;
    if (cdf_out) cdf_out[r * S + i] = v;
  }
  __syncthreads();
  for (int k = l; k < M; k += 64) {
    const float d0 = dk[k];
    const float* col = rad_o + (r * M + k) * 3;
    float al;
    if (k < S1 && inside[r * S1 + k]) {
      al = fmaxf(fdiv(fsub(c[k], c[k + 1]), fadd(c[k], 1e-10f)), 0.0f);
      col = rad + (r * S1 + k) * 3;
    } else {
      const float dist = k + 1 < M ? fsub(dk[k + 1], d0) : 1e10f;
      al = fsub(1.0f, expf(fmul(-sp1(sig_o[r * M + k]), dist)));
    }
    la[k] = al;
    lcol[3 * k + 0] = col[0];
    lcol[3 * k + 1] = col[1];
    lcol[3 * k + 2] = col[2];
    ld[k] = d0;
    if (alpha_out) alpha_out[r * M + k] = al;
  }
  __syncthreads();
  if (l == 0) {
    double T = 1.0, a_acc = 0.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
    for (int k = 0; k < M; ++k) {
      const float al = la[k];
      const float w = fmul(al, (float)T);
      T *= (double)fadd(fsub(1.0f, al), 1e-10f);
      c0 += (double)fmul(w, lcol[3 * k + 0]);
      c1 += (double)fmul(w, lcol[3 * k + 1]);
      c2 += (double)fmul(w, lcol[3 * k + 2]);
      a_acc += (double)w;
      lw[k] = w;
    }
    const float accf = (float)a_acc;
    const float den = fadd(accf, 1e-10f);
    double dep = 0.0;
    for (int k = 0; k < M; ++k) dep += (double)fmul(fdiv(lw[k], den), ld[k]);
    float o0 = (float)c0, o1 = (float)c1, o2 = (float)c2;
    if (white_bkgd) {
      const float bg = fsub(1.0f, accf);
      o0 = fadd(o0, bg); o1 = fadd(o1, bg); o2 = fadd(o2, bg);
    }
    rgb[r * 3 + 0] = o0;
    rgb[r * 3 + 1] = o1;
    rgb[r * 3 + 2] = o2;
    depth[r] = (float)dep;
    acc[r] = accf;
  }
  __syncthreads();
  for (int k = l; k < M; k += 64) w_out[r * M + k] = lw[k];
}

// backward of the above -> d sdf [R,S], d radiance [R,S-1,3], d sigma_out [R,M], d radiance_out
// [R,M,3], d s per ray [R].  One ray per wave: the elementwise parts (alphas, weight adjoints, the
// colour gradients, d sigma from the stored alpha adjoints) across the lanes, the prefix product and
// the reverse suffix walk on lane 0.  LDS: 8 (M + 2) + 4 (3 S + 5 M) bytes.
__global__ __launch_bounds__(64) void neus_composite_bg_bwd_kernel(
    const float* __restrict__ sdf, const float* __restrict__ s_dev, const float* __restrict__ rad,
    const float* __restrict__ sig_o, const float* __restrict__ rad_o, const float* __restrict__ d_out,
    const uint8_t* __restrict__ inside, int64_t R, int S, int M, int white_bkgd, const float* __restrict__ g_rgb,
    const float* __restrict__ g_depth, const float* __restrict__ g_acc, const float* __restrict__ g_w,
    float* __restrict__ d_sdf, float* __restrict__ d_rad, float* __restrict__ d_sig, float* __restrict__ d_rad_o,
    float* __restrict__ d_s) {
  extern __shared__ double ldsd[];
  const int64_t r = blockIdx.x;
  const int l = threadIdx.x, S1 = S - 1;
  const float s = *s_dev;
  const float* sd = sdf + r * S;
  const float* dk = d_out + r * M;
  double* lab = ldsd;              // [M] alpha adjoints
  double* ldb = lab + M;           // A, wd
  float* c = (float*)(ldb + 2);    // [S] cdf
  float* ls = c + S;               // [S] sdf
  float* lo = ls + S;              // [S] d sdf
  float* al = lo + S;              // [M] alpha
  float* Tt = al + M;              // [M] T
  float* w = Tt + M;               // [M] weights
  float* wb = w + M;               // [M] weight adjoints
  float* ld = wb + M;              // [M] depths
  auto is_in = [&](int k) { return k < S1 && inside[r * S1 + k] != 0; };
  for (int i = l; i < S; i += 64) {
    const float v = sd[i];
    ls[i] = v;
    c[i] = sigmoidf_ref(fmul(v, s));
  }
  __syncthreads();
  for (int k = l; k < M; k += 64) {
    const float d0 = dk[k];
    float a;
    if (is_in(k)) {
      a = fmaxf(fdiv(fsub(c[k], c[k + 1]), fadd(c[k], 1e-10f)), 0.0f);
    } else {
      const float dist = k + 1 < M ? fsub(dk[k + 1], d0) : 1e10f;
      a = fsub(1.0f, expf(fmul(-sp1(sig_o[r * M + k]), dist)));
    }
    al[k] = a;
    ld[k] = d0;
  }
  __syncthreads();
  if (l == 0) {
    double T = 1.0, a_acc = 0.0, wd = 0.0;
    for (int k = 0; k < M; ++k) {
      const float a = al[k];
      Tt[k] = (float)T;
      w[k] = fmul(a, (float)T);
      T *= (double)fadd(fsub(1.0f, a), 1e-10f);
      a_acc += (double)w[k];
    }
    const float accf = (float)a_acc;
    ldb[0] = (double)fadd(accf, 1e-10f);
    for (int k = 0; k < M; ++k) wd += (double)w[k] * (double)ld[k];
    ldb[1] = wd;
  }
  __syncthreads();
  const double A = ldb[0], wd = ldb[1];
  const float gr0 = g_rgb ? g_rgb[r * 3 + 0] : 0.f, gr1 = g_rgb ? g_rgb[r * 3 + 1] : 0.f,
              gr2 = g_rgb ? g_rgb[r * 3 + 2] : 0.f;
  const double gd = g_depth ? (double)g_depth[r] : 0.0;
  const double ga = (g_acc ? (double)g_acc[r] : 0.0) - (white_bkgd ? (double)gr0 + gr1 + gr2 : 0.0);
  for (int k = l; k < M; k += 64) {
    const bool in = is_in(k);
    const float* col = in ? rad + (r * S1 + k) * 3 : rad_o + (r * M + k) * 3;
    double v = (double)gr0 * col[0] + (double)gr1 * col[1] + (double)gr2 * col[2] + ga;
    v += gd * ((double)ld[k] / A - wd / (A * A));
    if (g_w) v += (double)g_w[r * M + k];
    wb[k] = (float)v;
    float* dro = d_rad_o + (r * M + k) * 3;
    dro[0] = in ? 0.f : fmul(w[k], gr0);
    dro[1] = in ? 0.f : fmul(w[k], gr1);
    dro[2] = in ? 0.f : fmul(w[k], gr2);
    if (k < S1) {
      float* dri = d_rad + (r * S1 + k) * 3;
      dri[0] = in ? fmul(w[k], gr0) : 0.f;
      dri[1] = in ? fmul(w[k], gr1) : 0.f;
      dri[2] = in ? fmul(w[k], gr2) : 0.f;
    }
  }
  __syncthreads();
  if (l == 0) {
    double suffix = 0.0, sbar = 0.0;
    float cbar_next = 0.0f;  // gradient reaching c_{k+1} from alpha_{k+1}'s c_i term
    for (int k = M - 1; k >= 0; --k) {
      const double u = (double)fadd(fsub(1.0f, al[k]), 1e-10f);
      const double abar = (double)wb[k] * Tt[k] - suffix / u;
      suffix += (double)wb[k] * al[k] * Tt[k];
      lab[k] = abar;
      if (k < S1) {
        double ci_bar = 0.0, cn_bar = 0.0;
        if (is_in(k)) {
          const float num = fsub(c[k], c[k + 1]), den = fadd(c[k], 1e-10f);
          if (fdiv(num, den) >= 0.0f) {
            ci_bar = abar / den - abar * num / ((double)den * den);
            cn_bar = -abar / den;
          }
        }
        const double cb_next = cn_bar + (double)cbar_next;
        const float cc = c[k + 1];
        const double sg = cb_next * cc * (1.0 - cc);
        lo[k + 1] = (float)(sg * s);
        sbar += sg * ls[k + 1];
        cbar_next = (float)ci_bar;
      }
    }
    const float cc = c[0];
    const double sg = (double)cbar_next * cc * (1.0 - cc);
    lo[0] = (float)(sg * s);
    sbar += sg * ls[0];
    d_s[r] = (float)sbar;
  }
  __syncthreads();
  for (int k = l; k < M; k += 64) {
    if (is_in(k)) {
      d_sig[r * M + k] = 0.f;
    } else {
      // d alpha_out / d sigma = exp(-softplus(sigma) dist) dist softplus'(sigma)
      const float dist = k + 1 < M ? fsub(ld[k + 1], ld[k]) : 1e10f;
      const float x = sig_o[r * M + k];
      const double e = exp(-(double)sp1(x) * (double)dist);
      d_sig[r * M + k] = (float)(lab[k] * e * (double)dist * sp1_grad(x));
    }
  }
  for (int i = l; i < S; i += 64) d_sdf[r * S + i] = lo[i];
}

// ---- UNISURF compositing with a graph (unisurf.py:219-236, get_opacity_from_surface :53-62) ------------
// One thread per ray, P samples.  alpha_i = odds / (1 + odds), odds = exp(-logit_i); T_i = prod_{j<i}
// (1 - alpha_j + 1e-10) (the cumprod of the shifted transparency); w_i = alpha_i T_i; rgb = sum w c,
// acc = sum w, depth = sum w / (acc + 1e-10) d.  Same arithmetic as the render kernel (uni_composite):
// fp64 prefix product and sums, rounded per element.
__device__ __forceinline__ float uni_alpha(float lg) {
  const float odds = expf(-lg);
  return fdiv(odds, fadd(1.0f, odds));
}
__global__ void unisurf_composite_fwd_kernel(const float* __restrict__ logits, const float* __restrict__ rad,
                                             const float* __restrict__ d_all, int64_t R, int P, int white_bkgd,
                                             float* __restrict__ rgb, float* __restrict__ depth,
                                             float* __restrict__ acc, float* __restrict__ w_out,
                                             float* __restrict__ alpha_out) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  double T = 1.0, a_acc = 0.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
  for (int i = 0; i < P; ++i) {
    const int64_t q = r * P + i;
    const float al = uni_alpha(logits[q]);
    const float w = fmul(al, (float)T);
    T *= (double)fadd(fsub(1.0f, al), 1e-10f);
    c0 += (double)fmul(w, rad[q * 3 + 0]);
    c1 += (double)fmul(w, rad[q * 3 + 1]);
    c2 += (double)fmul(w, rad[q * 3 + 2]);
    a_acc += (double)w;
    w_out[q] = w;
    if (alpha_out) alpha_out[q] = al;
  }
  const float accf = (float)a_acc;
  const float den = fadd(accf, 1e-10f);
  double dep = 0.0;
  for (int i = 0; i < P; ++i) dep += (double)fmul(fdiv(w_out[r * P + i], den), d_all[r * P + i]);
  float o0 = (float)c0, o1 = (float)c1, o2 = (float)c2;
  if (white_bkgd) {
    const float bg = fsub(1.0f, accf);
    o0 = fadd(o0, bg); o1 = fadd(o1, bg); o2 = fadd(o2, bg);
  }
  rgb[r * 3 + 0] = o0;
  rgb[r * 3 + 1] = o1;
  rgb[r * 3 + 2] = o2;
  depth[r] = (float)dep;
  acc[r] = accf;
}

// backward: G_i = dL/dw_i (rgb, acc, depth and direct weight gradients); w_i = alpha_i T_i with
// T_i = T_k u_k prod_{k<j<i} u_j (u = 1 - alpha + 1e-10), so
//   dL/dalpha_k = T_k (G_k - S_k),  S_k = sum_{i>k} G_i alpha_i prod_{k<j<i} u_j
// (suffix recursion S_k = G_{k+1} alpha_{k+1} + u_{k+1} S_{k+1}: no division by u), and
// dalpha/dlogit = -alpha (1 - alpha).
__global__ void unisurf_composite_bwd_kernel(const float* __restrict__ logits, const float* __restrict__ rad,
                                             const float* __restrict__ d_all, int64_t R, int P, int white_bkgd,
                                             const float* __restrict__ g_rgb, const float* __restrict__ g_depth,
                                             const float* __restrict__ g_acc, const float* __restrict__ g_w,
                                             float* __restrict__ work, float* __restrict__ d_logits,
                                             float* __restrict__ d_rad) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= R) return;
  float* al = work + r * (3 * (int64_t)P);  // alpha, T, w
  float* Tt = al + P;
  float* w = Tt + P;
  double T = 1.0, a_acc = 0.0, wd = 0.0;
  for (int i = 0; i < P; ++i) {
    const int64_t q = r * P + i;
    const float a = uni_alpha(logits[q]);
    al[i] = a;
    Tt[i] = (float)T;
    w[i] = fmul(a, (float)T);
    T *= (double)fadd(fsub(1.0f, a), 1e-10f);
    a_acc += (double)w[i];
    wd += (double)w[i] * (double)d_all[q];
  }
  const double A = (double)fadd((float)a_acc, 1e-10f);
  const float gr0 = g_rgb ? g_rgb[r * 3 + 0] : 0.f, gr1 = g_rgb ? g_rgb[r * 3 + 1] : 0.f,
              gr2 = g_rgb ? g_rgb[r * 3 + 2] : 0.f;
  const double gd = g_depth ? (double)g_depth[r] : 0.0;
  const double ga = (g_acc ? (double)g_acc[r] : 0.0) - (white_bkgd ? (double)gr0 + gr1 + gr2 : 0.0);
  double S = 0.0;  // S_k for the current k (walking backwards)
  for (int k = P - 1; k >= 0; --k) {
    const int64_t q = r * P + k;
    double G = (double)gr0 * rad[q * 3 + 0] + (double)gr1 * rad[q * 3 + 1] + (double)gr2 * rad[q * 3 + 2] + ga;
    G += gd * ((double)d_all[q] / A - wd / (A * A));
    if (g_w) G += (double)g_w[q];
    const double abar = (double)Tt[k] * (G - S);
    const double a = al[k];
    d_logits[q] = (float)(-abar * a * (1.0 - a));
    d_rad[q * 3 + 0] = fmul(w[k], gr0);
    d_rad[q * 3 + 1] = fmul(w[k], gr1);
    d_rad[q * 3 + 2] = fmul(w[k], gr2);
    S = G * a + (double)fadd(fsub(1.0f, al[k]), 1e-10f) * S;  // S_{k-1}
  }
}

}  // namespace
}  // namespace nr

using namespace nr;

#define NR_LAUNCH_CHECK() NR_HIP_CHECK(hipGetLastError())

extern "C" {

int nr_embed(const float* x, int64_t P, int nfreq, float* out, void* stream) {
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  return nr_embed_padded(x, P, nfreq, out, nf, stream);
}

int nr_embed_padded(const float* x, int64_t P, int nfreq, float* out, int ldo, void* stream) {
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  NR_REQUIRE(x && out && P >= 0 && nfreq <= 10 && ldo >= nf, NR_ERR_ARG, "nr_embed: bad argument");
  if (P == 0) return NR_OK;
  hipLaunchKernelGGL(embed_kernel, emb_grid(P), dim3(256), 0, (hipStream_t)stream, x,
                     P, nfreq, out, ldo);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_embed_jvp(const float* x, const float* v, int64_t P, int nfreq, float* out, void* stream) {
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  return nr_embed_jvp_padded(x, v, P, nfreq, out, nf, stream);
}

int nr_embed_jvp_padded(const float* x, const float* v, int64_t P, int nfreq, float* out, int ldo, void* stream) {
  const int nf = nfreq < 0 ? 3 : 3 + 6 * nfreq;
  NR_REQUIRE(x && v && out && P >= 0 && nfreq <= 10 && ldo >= nf, NR_ERR_ARG, "nr_embed_jvp: bad argument");
  if (P == 0) return NR_OK;
  hipLaunchKernelGGL(embed_jvp_kernel, emb_grid(P), dim3(256), 0,
                     (hipStream_t)stream, x, v, P, nfreq, out, ldo);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_embed_vjp(const float* x, const float* e0, int ld0, const float* e1, int ld1, float s1, int64_t P, int nfreq,
                 float* out, void* stream) {
  NR_REQUIRE(x && e0 && out && P >= 0 && nfreq <= 10, NR_ERR_ARG, "nr_embed_vjp: bad argument");
  if (P == 0) return NR_OK;
  hipLaunchKernelGGL(embed_vjp_kernel, emb_grid(P), dim3(256), 0,
                     (hipStream_t)stream, x, e0, ld0, e1, ld1, s1, P, nfreq, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_softplus100(const float* z, int64_t n, float* h, float* s, void* stream) {
  NR_REQUIRE(z && h && s && n >= 0, NR_ERR_ARG, "nr_softplus100: bad argument");
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(softplus100_kernel, grid1(n), dim3(kBlk), 0, (hipStream_t)stream, z, n, h, s);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_scale_cols(const float* a, int64_t P, int lda, int col0, int ncols, const float* s, float scale, float* out,
                  void* stream) {
  NR_REQUIRE(a && out && P >= 0 && col0 >= 0 && ncols >= 0 && col0 + ncols <= lda, NR_ERR_ARG,
             "nr_scale_cols: bad argument");
  if (P == 0 || ncols == 0) return NR_OK;
  hipLaunchKernelGGL(scale_cols_kernel, grid1(P * ncols), dim3(kBlk), 0, (hipStream_t)stream, a, P, lda, col0, ncols,
                     s, scale, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_softplus_adjoint(const float* hbar, int ldh, const float* s, const float* g, const float* zdot, int64_t P,
                        int n, float* zbar, void* stream) {
  NR_REQUIRE(hbar && s && zbar && (!g == !zdot) && P >= 0 && n >= 0 && ldh >= n, NR_ERR_ARG,
             "nr_softplus_adjoint: bad argument");
  if (P == 0 || n == 0) return NR_OK;
  hipLaunchKernelGGL(softplus_adjoint_kernel, grid1(P * n), dim3(kBlk), 0, (hipStream_t)stream, hbar, ldh, s, g, zdot,
                     P, n, zbar);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

size_t nr_colsum_workspace_bytes(int n) { return (size_t)kColBlocks * (size_t)(n > 0 ? n : 1) * sizeof(float); }

int nr_colsum(const float* a, int64_t P, int n, float* out, void* workspace, size_t workspace_bytes, void* stream) {
  NR_REQUIRE(a && out && P >= 0 && n >= 1, NR_ERR_ARG, "nr_colsum: bad argument");
  NR_REQUIRE(workspace && workspace_bytes >= nr_colsum_workspace_bytes(n), NR_ERR_WORKSPACE,
             "nr_colsum: workspace too small");
  float* part = (float*)workspace;
  hipLaunchKernelGGL(colsum_partial_kernel, dim3(kColBlocks), dim3(256), 0, (hipStream_t)stream, a, P, n, part);
  NR_LAUNCH_CHECK();
  hipLaunchKernelGGL(colsum_final_kernel, dim3((n + 63) / 64), dim3(1024), 0, (hipStream_t)stream, part, n, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_sine30(const float* z, int64_t n, float* h, float* s, void* stream) {
  NR_REQUIRE(z && h && s && n >= 0, NR_ERR_ARG, "nr_sine30: bad argument");
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(sine30_kernel, grid1(n), dim3(kBlk), 0, (hipStream_t)stream, z, n, h, s);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_sine_adjoint(const float* hbar, int ldh, const float* s, const float* h, const float* g, const float* zdot,
                    int64_t P, int n, float* zbar, void* stream) {
  NR_REQUIRE(hbar && s && h && zbar && P >= 0 && n >= 1 && ldh >= n && (!g || zdot), NR_ERR_ARG,
             "nr_sine_adjoint: bad argument");
  if (P == 0) return NR_OK;
  hipLaunchKernelGGL(sine_adjoint_kernel, grid1(P * n), dim3(kBlk), 0, (hipStream_t)stream, hbar, ldh, s, h, g, zdot,
                     P, n, zbar);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_mul(const float* a, const float* b, int64_t n, float* out, void* stream) {
  NR_REQUIRE(a && b && out && n >= 0, NR_ERR_ARG, "nr_mul: bad argument");
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(mul_kernel, grid1(n), dim3(kBlk), 0, (hipStream_t)stream, a, b, n, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_activation(float* y, float* g, int64_t n, int mode, void* stream) {
  NR_REQUIRE(y && n >= 0 && mode >= 0 && mode <= 3 && (mode % 2 == 0 || g), NR_ERR_ARG, "nr_activation: bad argument");
  if (n == 0) return NR_OK;
  hipLaunchKernelGGL(act_kernel, grid1(n), dim3(kBlk), 0, (hipStream_t)stream, y, g, n, mode);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

static int wn_launch(const NrWnLayer* layers, int n, void* stream, bool bwd) {
  NR_REQUIRE(layers && n >= 1 && n <= NR_WN_MAX, NR_ERR_ARG, "nr_weight_norm: 1..NR_WN_MAX layers");
  WnBatch b{};
  b.n = n;
  b.row0[0] = 0;
  for (int i = 0; i < n; ++i) {
    const NrWnLayer& L = layers[i];
    NR_REQUIRE(L.v && L.g && L.norm && L.rows > 0 && L.cols > 0, NR_ERR_ARG, "nr_weight_norm: bad layer");
    NR_REQUIRE(bwd ? (L.grad_v && L.grad_g) : (L.w != nullptr), NR_ERR_ARG, "nr_weight_norm: null output");
    b.l[i] = L;
    b.row0[i + 1] = b.row0[i] + L.rows;
  }
  const unsigned blocks = (unsigned)((b.row0[n] + 3) / 4);
  if (bwd) hipLaunchKernelGGL(weight_norm_bwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, b);
  else hipLaunchKernelGGL(weight_norm_fwd_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, b);
  NR_LAUNCH_CHECK();
  return NR_OK;
}
int nr_weight_norm_fwd(const NrWnLayer* layers, int n, void* stream) { return wn_launch(layers, n, stream, false); }
int nr_weight_norm_bwd(const NrWnLayer* layers, int n, void* stream) { return wn_launch(layers, n, stream, true); }

int nr_adam_step(const NrAdamTensor* tensors, int n, int64_t step, double lr, double beta1, double beta2, double eps,
                 double weight_decay, void* stream) {
  NR_REQUIRE(tensors && n >= 1 && n <= NR_ADAM_MAX && step >= 1, NR_ERR_ARG, "nr_adam_step: 1..NR_ADAM_MAX tensors, step >= 1");
  NR_REQUIRE(beta1 >= 0.0 && beta1 < 1.0 && beta2 >= 0.0 && beta2 < 1.0 && eps >= 0.0 && lr >= 0.0,
             NR_ERR_ARG, "nr_adam_step: bad hyper-parameter");
  AdamBatch b{};
  b.n = n;
  b.chunk0[0] = 0;
  for (int i = 0; i < n; ++i) {
    const NrAdamTensor& T = tensors[i];
    NR_REQUIRE(T.param && T.grad && T.exp_avg && T.exp_avg_sq && T.n > 0, NR_ERR_ARG, "nr_adam_step: bad tensor");
    const int64_t nc = (T.n + kAdamChunk - 1) / kAdamChunk;
    NR_REQUIRE(b.chunk0[i] + nc < (int64_t)1 << 30, NR_ERR_ARG, "nr_adam_step: too many elements");
    b.t[i] = T;
    b.chunk0[i + 1] = b.chunk0[i] + (int)nc;
  }
  // torch's fused Adam: step_size = lr / (1 - beta1^step), denom = sqrt(v) / sqrt(1 - beta2^step) + eps
  b.beta1 = (float)beta1;
  b.beta2 = (float)beta2;
  b.omb1 = (float)(1.0 - beta1);
  b.omb2 = (float)(1.0 - beta2);
  b.eps = (float)eps;
  b.wd = (float)weight_decay;
  b.step_size = (float)(lr / (1.0 - std::pow(beta1, (double)step)));
  b.bc2_sqrt = (float)std::sqrt(1.0 - std::pow(beta2, (double)step));
  hipLaunchKernelGGL(adam_kernel, dim3((unsigned)b.chunk0[n]), dim3(256), 0, (hipStream_t)stream, b);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_radiance_input(const float* x, const float* v, const float* nrm, const float* feat, int64_t P, int nfreq_view,
                      int use_view_dirs, int wfeat, float* out, void* stream) {
  // wfeat = 0: the small inputs only (the training GEMM reads the feature from its own tensor)
  NR_REQUIRE(x && (!use_view_dirs || (v && nrm)) && (feat || wfeat == 0) && out && P >= 0 && nfreq_view <= 10 &&
                 wfeat >= 0,
             NR_ERR_ARG, "nr_radiance_input: bad argument");
  const int ld = use_view_dirs ? 6 + (nfreq_view < 0 ? 3 : 3 + 6 * nfreq_view) + wfeat : 3 + wfeat;
  if (P == 0) return NR_OK;
  hipLaunchKernelGGL(radiance_input_kernel, grid1(P * ld), dim3(kBlk), 0, (hipStream_t)stream, x, v, nrm, feat, P,
                     nfreq_view, use_view_dirs ? 1 : 0, wfeat, out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_neus_points(const float* rays_o, const float* rays_d, const float* d_all, int64_t R, int S, float* pts,
                   float* mids, float* dmid, void* stream) {
  NR_REQUIRE(rays_o && rays_d && d_all && pts && mids && dmid && R >= 0 && S >= 2, NR_ERR_ARG,
             "nr_neus_points: bad argument");
  if (R == 0) return NR_OK;
  hipLaunchKernelGGL(neus_points_kernel, grid1(R * S), dim3(kBlk), 0, (hipStream_t)stream, rays_o, rays_d, d_all, R, S,
                     pts, mids, dmid);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_neus_composite_fwd(const float* sdf, const float* s_dev, const float* rad, const float* dmid, int64_t R, int S,
                          int white_bkgd, float* rgb, float* depth, float* acc, float* weights, float* alpha,
                          float* cdf, void* stream) {
  NR_REQUIRE(sdf && s_dev && rad && dmid && rgb && depth && acc && weights && R >= 0 && S >= 2, NR_ERR_ARG,
             "nr_neus_composite_fwd: bad argument");
  if (R == 0) return NR_OK;
  NR_REQUIRE((size_t)2 * S * sizeof(float) <= 65536, NR_ERR_UNSUPPORTED, "nr_neus_composite_fwd: S too large");
  hipLaunchKernelGGL(neus_composite_fwd_kernel, dim3((unsigned)R), dim3(64), 2 * S * sizeof(float), (hipStream_t)stream,
                     sdf, s_dev, rad, dmid, R, S, white_bkgd, rgb, depth, acc, weights, alpha, cdf);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

size_t nr_neus_composite_bwd_workspace_bytes(int64_t R, int S) { return (size_t)R * 5 * S * sizeof(float); }

int nr_neus_composite_bwd(const float* sdf, const float* s_dev, const float* rad, const float* dmid, int64_t R, int S,
                          int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc,
                          const float* g_weights, float* d_sdf, float* d_rad, float* d_s, void* workspace,
                          size_t workspace_bytes, void* stream) {
  NR_REQUIRE(sdf && s_dev && rad && dmid && d_sdf && d_rad && d_s && R >= 0 && S >= 2, NR_ERR_ARG,
             "nr_neus_composite_bwd: bad argument");
  if (R == 0) return NR_OK;
  NR_REQUIRE(workspace && workspace_bytes >= nr_neus_composite_bwd_workspace_bytes(R, S), NR_ERR_WORKSPACE,
             "nr_neus_composite_bwd: workspace too small");
  const size_t lds = (size_t)S * sizeof(double) + (size_t)5 * S * sizeof(float);
  NR_REQUIRE(lds <= 65536, NR_ERR_UNSUPPORTED, "nr_neus_composite_bwd: S too large");
  hipLaunchKernelGGL(neus_composite_bwd_kernel, dim3((unsigned)R), dim3(64), lds,
                     (hipStream_t)stream, sdf, s_dev, rad, dmid, R, S, white_bkgd, g_rgb, g_depth, g_acc, g_weights,
                     d_sdf, d_rad, d_s);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_nerf_train_input(const float* rays_o, const float* rays_d, const float* d_out, int64_t R, int M, int n_mid,
                        float r_obj, float* x_emb, float* v_emb, uint8_t* inside, void* stream) {
  NR_REQUIRE(rays_o && rays_d && d_out && x_emb && v_emb && inside && R >= 0 && M >= 1 && n_mid >= 0 && n_mid <= M,
             NR_ERR_ARG, "nr_nerf_train_input: bad argument");
  if (R == 0) return NR_OK;
  hipLaunchKernelGGL(nerf_train_input_kernel, grid1(R * M), dim3(kBlk), 0, (hipStream_t)stream, rays_o, rays_d, d_out,
                     R, M, n_mid, r_obj, x_emb, v_emb, inside);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_neus_composite_bg_fwd(const float* sdf, const float* s_dev, const float* rad, const float* sigma_out,
                             const float* rad_out, const float* d_out, const uint8_t* inside, int64_t R, int S, int M,
                             int white_bkgd, float* rgb, float* depth, float* acc, float* weights, float* alpha,
                             float* cdf, void* stream) {
  NR_REQUIRE(sdf && s_dev && rad && sigma_out && rad_out && d_out && inside && rgb && depth && acc && weights &&
                 R >= 0 && S >= 2 && M >= S - 1,
             NR_ERR_ARG, "nr_neus_composite_bg_fwd: bad argument");
  if (R == 0) return NR_OK;
  const size_t lds = (size_t)(S + 6 * M) * sizeof(float);
  NR_REQUIRE(lds <= 65536, NR_ERR_UNSUPPORTED, "nr_neus_composite_bg_fwd: S + M too large");
  hipLaunchKernelGGL(neus_composite_bg_fwd_kernel, dim3((unsigned)R), dim3(64), lds, (hipStream_t)stream, sdf, s_dev,
                     rad, sigma_out, rad_out, d_out, inside, R, S, M, white_bkgd, rgb, depth, acc, weights, alpha, cdf);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

size_t nr_neus_composite_bg_bwd_workspace_bytes(int64_t R, int S, int M) {
  return (size_t)(R > 0 ? R : 1) * (size_t)(2 * S + 4 * M) * sizeof(float);
}

int nr_neus_composite_bg_bwd(const float* sdf, const float* s_dev, const float* rad, const float* sigma_out,
                             const float* rad_out, const float* d_out, const uint8_t* inside, int64_t R, int S, int M,
                             int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc,
                             const float* g_weights, float* d_sdf, float* d_rad, float* d_sigma_out,
                             float* d_rad_out, float* d_s, void* workspace, size_t workspace_bytes, void* stream) {
  NR_REQUIRE(sdf && s_dev && rad && sigma_out && rad_out && d_out && inside && d_sdf && d_rad && d_sigma_out &&
                 d_rad_out && d_s && R >= 0 && S >= 2 && M >= S - 1,
             NR_ERR_ARG, "nr_neus_composite_bg_bwd: bad argument");
  if (R == 0) return NR_OK;
  NR_REQUIRE(workspace && workspace_bytes >= nr_neus_composite_bg_bwd_workspace_bytes(R, S, M), NR_ERR_WORKSPACE,
             "nr_neus_composite_bg_bwd: workspace too small");
  const size_t lds = (size_t)(M + 2) * sizeof(double) + (size_t)(3 * S + 5 * M) * sizeof(float);
  NR_REQUIRE(lds <= 65536, NR_ERR_UNSUPPORTED, "nr_neus_composite_bg_bwd: S + M too large");
  hipLaunchKernelGGL(neus_composite_bg_bwd_kernel, dim3((unsigned)R), dim3(64), lds, (hipStream_t)stream, sdf, s_dev,
                     rad, sigma_out, rad_out, d_out, inside, R, S, M, white_bkgd, g_rgb, g_depth, g_acc, g_weights,
                     d_sdf, d_rad, d_sigma_out, d_rad_out, d_s);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_unisurf_composite_fwd(const float* logits, const float* rad, const float* d_all, int64_t R, int P,
                             int white_bkgd, float* rgb, float* depth, float* acc, float* weights, float* alpha,
                             void* stream) {
  NR_REQUIRE(logits && rad && d_all && rgb && depth && acc && weights && R >= 0 && P >= 1, NR_ERR_ARG,
             "nr_unisurf_composite_fwd: bad argument");
  if (R == 0) return NR_OK;
  hipLaunchKernelGGL(unisurf_composite_fwd_kernel, dim3((unsigned)((R + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     logits, rad, d_all, R, P, white_bkgd, rgb, depth, acc, weights, alpha);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

size_t nr_unisurf_composite_bwd_workspace_bytes(int64_t R, int P) {
  return (size_t)(R > 0 ? R : 1) * 3 * (size_t)P * sizeof(float);
}

int nr_unisurf_composite_bwd(const float* logits, const float* rad, const float* d_all, int64_t R, int P,
                             int white_bkgd, const float* g_rgb, const float* g_depth, const float* g_acc,
                             const float* g_weights, float* d_logits, float* d_rad, void* workspace,
                             size_t workspace_bytes, void* stream) {
  NR_REQUIRE(logits && rad && d_all && d_logits && d_rad && R >= 0 && P >= 1, NR_ERR_ARG,
             "nr_unisurf_composite_bwd: bad argument");
  if (R == 0) return NR_OK;
  NR_REQUIRE(workspace && workspace_bytes >= nr_unisurf_composite_bwd_workspace_bytes(R, P), NR_ERR_WORKSPACE,
             "nr_unisurf_composite_bwd: workspace too small");
  hipLaunchKernelGGL(unisurf_composite_bwd_kernel, dim3((unsigned)((R + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     logits, rad, d_all, R, P, white_bkgd, g_rgb, g_depth, g_acc, g_weights, (float*)workspace,
                     d_logits, d_rad);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_volsdf_composite_bg_fwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                               const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd,
                               const float* sigma_bg, const float* rad_bg, const float* d_bg, int N, float* rgb,
                               float* depth, float* acc, float* tau, float* p_i, float* sigma, float* sdf_out,
                               void* stream) {
  NR_REQUIRE(sdf && pts && beta_dev && rad && d_all && rgb && depth && acc && tau && R >= 0 && S >= 2 && N >= 0 &&
                 (N == 0 || (sigma_bg && rad_bg && d_bg)),
             NR_ERR_ARG, "nr_volsdf_composite_fwd: bad argument");
  if (R == 0) return NR_OK;
  hipLaunchKernelGGL(volsdf_composite_fwd_kernel, dim3((unsigned)((R + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     sdf, pts, beta_dev, rad, d_all, R, S, use_bg, r_bg, white_bkgd, VsBg{sigma_bg, rad_bg, d_bg, N},
                     rgb, depth, acc, tau, p_i, sigma, sdf_out);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_volsdf_composite_fwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                            const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd, float* rgb,
                            float* depth, float* acc, float* tau, float* p_i, float* sigma, float* sdf_out,
                            void* stream) {
  return nr_volsdf_composite_bg_fwd(sdf, pts, beta_dev, rad, d_all, R, S, use_bg, r_bg, white_bkgd, nullptr, nullptr,
                                    nullptr, 0, rgb, depth, acc, tau, p_i, sigma, sdf_out, stream);
}

size_t nr_volsdf_composite_bg_bwd_workspace_bytes(int64_t R, int S, int N) {
  return (size_t)(R > 0 ? R : 1) * 5 * (size_t)(S + N) * sizeof(float);
}

size_t nr_volsdf_composite_bwd_workspace_bytes(int64_t R, int S) {
  return nr_volsdf_composite_bg_bwd_workspace_bytes(R, S, 0);
}

int nr_volsdf_composite_bg_bwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                               const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd,
                               const float* sigma_bg, const float* rad_bg, const float* d_bg, int N,
                               const float* g_rgb, const float* g_depth, const float* g_acc, const float* g_tau,
                               const float* g_sdf, float* d_sdf, float* d_rad, float* d_beta, float* d_sigma_bg,
                               float* d_rad_bg, void* workspace, size_t workspace_bytes, void* stream) {
  NR_REQUIRE(sdf && pts && beta_dev && rad && d_all && d_sdf && d_rad && d_beta && R >= 0 && S >= 2 && N >= 0 &&
                 (N == 0 || (sigma_bg && rad_bg && d_bg && d_sigma_bg && d_rad_bg)),
             NR_ERR_ARG, "nr_volsdf_composite_bwd: bad argument");
  if (R == 0) return NR_OK;
  NR_REQUIRE(workspace && workspace_bytes >= nr_volsdf_composite_bg_bwd_workspace_bytes(R, S, N), NR_ERR_WORKSPACE,
             "nr_volsdf_composite_bwd: workspace too small");
  hipLaunchKernelGGL(volsdf_composite_bwd_kernel, dim3((unsigned)((R + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     sdf, pts, beta_dev, rad, d_all, R, S, use_bg, r_bg, white_bkgd, VsBg{sigma_bg, rad_bg, d_bg, N},
                     g_rgb, g_depth, g_acc, g_tau, g_sdf, (float*)workspace, d_sdf, d_rad, d_beta, d_sigma_bg,
                     d_rad_bg);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

int nr_volsdf_composite_bwd(const float* sdf, const float* pts, const float* beta_dev, const float* rad,
                            const float* d_all, int64_t R, int S, int use_bg, float r_bg, int white_bkgd,
                            const float* g_rgb, const float* g_depth, const float* g_acc, const float* g_tau,
                            const float* g_sdf, float* d_sdf, float* d_rad, float* d_beta, void* workspace,
                            size_t workspace_bytes, void* stream) {
  return nr_volsdf_composite_bg_bwd(sdf, pts, beta_dev, rad, d_all, R, S, use_bg, r_bg, white_bkgd, nullptr, nullptr,
                                    nullptr, 0, g_rgb, g_depth, g_acc, g_tau, g_sdf, d_sdf, d_rad, d_beta, nullptr,
                                    nullptr, workspace, workspace_bytes, stream);
}

int nr_volsdf_nerf_input(const float* rays_o, const float* rays_d, const float* d_bg, const float* rs, int64_t R,
                         int N, float* x_emb, float* v_emb, void* stream) {
  NR_REQUIRE(rays_o && rays_d && d_bg && rs && x_emb && v_emb && R >= 0 && N >= 1, NR_ERR_ARG,
             "nr_volsdf_nerf_input: bad argument");
  if (R == 0) return NR_OK;
  hipLaunchKernelGGL(volsdf_nerf_input_kernel, grid1(R * N), dim3(kBlk), 0, (hipStream_t)stream, rays_o, rays_d, d_bg,
                     rs, R, N, x_emb, v_emb);
  NR_LAUNCH_CHECK();
  return NR_OK;
}

}  // extern "C"
