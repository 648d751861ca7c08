// neurecon_amd — shared device/host helpers for the gfx950 (CDNA4) render kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/neurecon_hip.h"

// NR_EXP_* switches skip work inside the kernels (timing experiments, results are garbage): only
// tools/build_variants.py may set them, and it also defines NR_VARIANT_BUILD
#if !defined(NR_VARIANT_BUILD) &&                                                                  \
    (defined(NR_EXP_NO_DMA) || defined(NR_EXP_NO_ESTORE) || defined(NR_EXP_NO_ELOAD) ||             \
     defined(NR_EXP_NO_SOFTPLUS) || defined(NR_EXP_NO_SPLIT) || defined(NR_EXP_NO_BARRIER) ||       \
     defined(NR_EXP_UNROLL) || defined(NR_EXP_NO_PINGPONG) || defined(NR_EXP_NO_EPI) ||             \
     defined(NR_EXP_NO_MFMA) || defined(NR_EXP_NO_TRANS) || defined(NR_EXP_NO_EPISPLIT) ||   \
     defined(NR_EXP_SHARED_W) || defined(NR_EXP_NO_AREAD) || defined(NR_EXP_STAMPS))
#error "NR_EXP_* experiment switches are for tools/build_variants.py builds only"
#endif

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

namespace nr {

// ---------------------------------------------------------------------------------------------
// error plumbing (C-ABI returns int status; text via nr_last_error)
// ---------------------------------------------------------------------------------------------
void set_error(const std::string& msg);

#define NR_HIP_CHECK(expr)                                                              \
  do {                                                                                  \
    hipError_t _e = (expr);                                                             \
    if (_e != hipSuccess) {                                                             \
      ::nr::set_error(std::string(#expr) + ": " + hipGetErrorString(_e));               \
      return NR_ERR_HIP;                                                                \
    }                                                                                   \
  } while (0)

#define NR_REQUIRE(cond, code, msg)                                                     \
  do {                                                                                  \
    if (!(cond)) {                                                                      \
      ::nr::set_error(msg);                                                             \
      return code;                                                                      \
    }                                                                                   \
  } while (0)

// opt-in kernel timing (nr_profile.hip): brackets a launch with events on its stream
bool prof_on();
class ProfScope {
 public:
  // dev_units: optional device-side unit count (a compacted launch); the record's units become
  // min(units, *dev_units * mult), read when the statistics are
  ProfScope(const char* name, double units, hipStream_t st, const int* dev_units = nullptr, int mult = 1);
  ~ProfScope();

 private:
  hipStream_t st_;
  bool on_;
  size_t idx_ = 0;
};

// ---------------------------------------------------------------------------------------------
// Exact-rounding fp32 arithmetic.  The reference runs eager fp32 PyTorch ops, i.e. every
// mul/add is rounded separately; hipcc would otherwise contract a*b+c into one FMA.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fdiv(float a, float b) { return __fdiv_rn(a, b); }

// ATen's CPU float sum of one contiguous row (cascade_sum -> vectorized_inner_sum, or row_sum for
// rows shorter than a vector), reproduced operation for operation so that normalisers feeding a
// discrete decision (sample_pdf's `denom < eps`, searchsorted) round exactly like the reference.
// Vector width 8 and the 4-way ILP / 4-level cascade were verified against torch.sum (2.10, x86).
template <class Load>
__device__ float aten_row_sum(int n, Load ld) {
  constexpr int V = 8;
  if (n < V) {
    float p[4] = {0.f, 0.f, 0.f, 0.f};
    const int si = n / 4;
    for (int i = 0; i < si; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] = __fadd_rn(p[k], ld(4 * i + k));
    for (int t = si * 4; t < n; ++t) p[0] = __fadd_rn(p[0], ld(t));
    return __fadd_rn(__fadd_rn(__fadd_rn(p[0], p[1]), p[2]), p[3]);
  }
  const int vec_size = n / V, size_ilp = vec_size / 4;
  float acc[4][4][V];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < V; ++l) acc[j][k][l] = 0.f;
  int cl2 = 1;
  if (size_ilp > 2) { cl2 = 0; while ((1 << cl2) < size_ilp) ++cl2; }
  const int lp = (cl2 / 4) > 4 ? (cl2 / 4) : 4;
  const int step = 1 << lp, mask = step - 1;
  int i = 0;
  while (i + step <= size_ilp) {
    for (int j = 0; j < step; ++j, ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < V; ++l) acc[0][k][l] = __fadd_rn(acc[0][k][l], ld((4 * i + k) * V + l));
#pragma unroll
    for (int j = 1; j < 4; ++j) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int l = 0; l < V; ++l) {
          acc[j][k][l] = __fadd_rn(acc[j][k][l], acc[j - 1][k][l]);
          acc[j - 1][k][l] = 0.f;
        }
      if ((i & (mask << (j * lp))) != 0) break;
    }
  }
  for (; i < size_ilp; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < V; ++l) acc[0][k][l] = __fadd_rn(acc[0][k][l], ld((4 * i + k) * V + l));
#pragma unroll
  for (int j = 1; j < 4; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int l = 0; l < V; ++l) acc[0][k][l] = __fadd_rn(acc[0][k][l], acc[j][k][l]);
  for (int t = size_ilp * 4; t < vec_size; ++t)
#pragma unroll
    for (int l = 0; l < V; ++l) acc[0][0][l] = __fadd_rn(acc[0][0][l], ld(t * V + l));
#pragma unroll
  for (int k = 1; k < 4; ++k)
#pragma unroll
    for (int l = 0; l < V; ++l) acc[0][0][l] = __fadd_rn(acc[0][0][l], acc[0][k][l]);
  float fa = 0.f;
  for (int t = vec_size * V; t < n; ++t) fa = __fadd_rn(fa, ld(t));
#pragma unroll
  for (int l = 0; l < V; ++l) fa = __fadd_rn(fa, acc[0][0][l]);
  return fa;
}

// inverse-CDF sample for one u (rend_util.py:284-290)
__device__ __forceinline__ float invert_one(float u, float c0, float c1, float b0, float b1) {
  float denom = fsub(c1, c0);
  if (denom < 1e-5f) denom = 1.0f;
  const float t = fdiv(fsub(u, c0), denom);
  return fadd(b0, fmul(t, fsub(b1, b0)));
}

// torch CPU x.norm(dim=-1) of a 3-vector (and F.normalize's denominator): the reduction loop
// accumulates with fused multiply-adds, sqrt(fma(z, z, fma(y, y, x*x))) -- verified bit-exact vs
// torch.norm on the host (tests/test_sum_order.py)
__device__ __forceinline__ float norm3_ref(float x, float y, float z) {
  return sqrtf(__fmaf_rn(z, z, __fmaf_rn(y, y, fmul(x, x))));
}

// torch.sigmoid(x) = 1 / (1 + exp(-x))
__device__ __forceinline__ float sigmoidf_ref(float x) { return fdiv(1.0f, fadd(1.0f, expf(-x))); }

// torch.linspace(0, 1, n)[i] (float): symmetric two-sided formula used by ATen's linspace kernel
__host__ __device__ inline float linspace01(int i, int n) {
  if (n == 1) return 0.0f;
  const float step = 1.0f / (float)(n - 1);
  const int halfway = n / 2;
  return i < halfway ? 0.0f + step * (float)i : 1.0f - step * (float)(n - 1 - i);
}

}  // namespace nr
