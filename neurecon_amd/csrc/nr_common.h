// neurecon_amd — shared device/host helpers for the gfx950 (CDNA4) render kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string>

#include "../../include/neurecon_hip.h"

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

// ---------------------------------------------------------------------------------------------
// Exact-rounding fp32 arithmetic.  The reference runs eager fp32 PyTorch ops, i.e. every
// mul/add is rounded separately; hipcc would otherwise contract a*b+c into one FMA.
// ---------------------------------------------------------------------------------------------
__device__ __forceinline__ float fmul(float a, float b) { return __fmul_rn(a, b); }
__device__ __forceinline__ float fadd(float a, float b) { return __fadd_rn(a, b); }
__device__ __forceinline__ float fsub(float a, float b) { return __fsub_rn(a, b); }
__device__ __forceinline__ float fdiv(float a, float b) { return __fdiv_rn(a, b); }

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
