// neurecon_amd — layer products of the fp32 / SIREN nets' training step (models/base.py:118-129
// nn.Linear / DenseLayer forward, :243-282 and its autograd; base.py:84-115 SirenLayer): C = A op(B)
// (+ bias), the products torch.addmm / mm ran on hipBLASLt through r05.
//
// * ACC64 (the default): exact fp32 products accumulated in fp64 on v_mfma_f64_16x16x4_f64 (an fp32 x
//   fp32 product is exact in fp64; the sum of <= 300 of them carries ~1e-16 relative error), rounded to
//   fp32 once, the bias added last.  Why (tools/train_error_probe.py, profiles/r06/train_error_probe.txt):
//   the fp32 mode's excess gradient error against float64 on the SDF net's layers 0 and 4 comes from the
//   fp32 rounding of these layer products -- with them in float64 the 512-ray step's worst error falls
//   from 8.5e-5 to 3.6e-5 of the tensor scale, inside the CPU fp32 oracle's own envelope (4.8e-5), while
//   float64 weight gradients change nothing; every GPU fp32 product tried (hipBLASLt, and the fp32
//   fmaf chain below) lands at 7.3-8.5e-5;
// * !ACC64: exact fp32 products on v_mfma_f32_16x16x4_f32 accumulated in k order (an fmaf chain per
//   element, the association of a CPU sgemm's register accumulation) -- kept for the A/B;
// * 128 x 64 output tile per 256-thread workgroup (4 waves of 32 rows x 64 columns: 2 x 4 MFMA tiles),
//   K in blocks of 32 staged through a double-buffered fp32 LDS image, the next block's global loads in
//   flight during the current block's MFMAs;
// * LDS images [row][k] with a 34-float row stride: a fragment read (lanes 0-15: rows 0-15 of k-slot 0,
//   lanes 16-31 of k-slot 1, ...) hits 2 r + k -> 32 distinct banks per half-wave;
// * any M, N, K and row strides (edges zero-filled on load, masked on store); op(B) = Bᵀ for B [N, K]
//   (trans_b: A Wᵀ, nn.Linear) or B [K, N].
#include "nr_common.h"
#include <type_traits>

namespace nr {
namespace g32 {

constexpr int TM = 128, TN = 64, TK = 32, LS = TK + 2;  // LS: LDS row stride (floats)
constexpr int NT = 256;

struct Args {
  const float* A;
  int64_t lda;
  const float* B;
  int64_t ldb;
  int trans_b;
  const float* bias;
  float* C;
  int64_t ldc;
  int64_t M;
  int N, K;
};

typedef double f64x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f32x4 mfma(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f64x4 mfma(double a, double b, f64x4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

template <bool ACC64>
__global__ __launch_bounds__(NT) void gemm32_kernel(Args a) {
  using T = typename std::conditional<ACC64, double, float>::type;
  using V4 = typename std::conditional<ACC64, f64x4, f32x4>::type;
  __shared__ float As[2][TM * LS];
  __shared__ float Bs[2][TN * LS];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int64_t m0 = (int64_t)blockIdx.y * TM;
  const int n0 = blockIdx.x * TN;
  float ra[16], rb[8];
  // A tile: element e = t + 256 j -> row e >> 5, k e & 31 (32 consecutive threads read one row's 128 B)
  auto load = [&](int k0) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int e = t + NT * j, r = e >> 5, kk = e & 31;
      const int64_t m = m0 + r;
      const int k = k0 + kk;
      ra[j] = (m < a.M && k < a.K) ? a.A[m * a.lda + k] : 0.0f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = t + NT * j;
      // Bᵀ: W rows along the threads' k; B [K, N]: consecutive threads along n (both coalesced)
      const int r = a.trans_b ? (e >> 5) : (e & 63), kk = a.trans_b ? (e & 31) : (e >> 6);
      const int n = n0 + r, k = k0 + kk;
      rb[j] = (n < a.N && k < a.K) ? (a.trans_b ? a.B[(int64_t)n * a.ldb + k] : a.B[(int64_t)k * a.ldb + n]) : 0.0f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int e = t + NT * j;
      As[buf][(e >> 5) * LS + (e & 31)] = ra[j];
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = t + NT * j;
      const int r = a.trans_b ? (e >> 5) : (e & 63), kk = a.trans_b ? (e & 31) : (e >> 6);
      Bs[buf][r * LS + kk] = rb[j];
    }
  };
  V4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = V4{0, 0, 0, 0};
  const int nkb = (a.K + TK - 1) / TK;
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int kb = 0; kb < nkb; ++kb) {
    const int buf = kb & 1;
    if (kb + 1 < nkb) load((kb + 1) * TK);  // in flight during this block's MFMAs
    const float* as = As[buf] + (32 * w + fr) * LS + fk;
    const float* bs = Bs[buf] + fr * LS + fk;
#pragma unroll
    for (int ks = 0; ks < TK / 4; ++ks) {
      const T a0 = (T)as[4 * ks], a1 = (T)as[16 * LS + 4 * ks];
      T b[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) b[j] = (T)bs[16 * j * LS + 4 * ks];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[0][j] = mfma(a0, b[j], acc[0][j]);
        acc[1][j] = mfma(a1, b[j], acc[1][j]);
      }
    }
    if (kb + 1 < nkb) {
      store(buf ^ 1);  // the other image: no wave reads it before the barrier below
      __syncthreads();
    }
  }
  // acc[i][j] register r: column 16 j + (lane & 15), row 32 w + 16 i + 4 (lane >> 4) + r (f32 MFMA) or
  // 32 w + 16 i + (lane >> 4) + 4 r (f64 MFMA: its own C/D map, cdna_hip_programming.md §3)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int n = n0 + 16 * j + fr;
    if (n >= a.N) continue;
    const float bn = a.bias ? a.bias[n] : 0.0f;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t m = m0 + 32 * w + 16 * i + (ACC64 ? fk + 4 * r : 4 * fk + r);
        const float v = (float)acc[i][j][r];  // one rounding of the fp64 sum
        if (m < a.M) a.C[m * a.ldc + n] = a.bias ? fadd(v, bn) : v;
      }
  }
}

}  // namespace g32
}  // namespace nr

extern "C" int nr_gemm32(const float* A, int64_t lda, const float* B, int64_t ldb, int trans_b, const float* bias,
                         float* C, int64_t ldc, int64_t M, int N, int K, int acc32, void* stream) {
  using namespace nr;
  NR_REQUIRE(A && B && C && M >= 0 && N >= 0 && K >= 0, NR_ERR_ARG, "nr_gemm32: null argument or negative size");
  NR_REQUIRE(lda >= K && ldc >= N && ldb >= (trans_b ? K : N), NR_ERR_ARG, "nr_gemm32: leading dimension too small");
  NR_REQUIRE(K > 0, NR_ERR_ARG, "nr_gemm32: K must be positive");
  NR_REQUIRE((M + g32::TM - 1) / g32::TM <= 65535, NR_ERR_ARG, "nr_gemm32: M above 65535 row tiles (split the rows)");
  if (M == 0 || N == 0) return NR_OK;
  g32::Args a{A, lda, B, ldb, trans_b, bias, C, ldc, M, N, K};
  ProfScope prof("gemm32", (double)M * N * K, (hipStream_t)stream);
  // the N tiles of one row tile are consecutive blocks: they run together and share the A tile's reads
  const dim3 grid((N + g32::TN - 1) / g32::TN, (unsigned)((M + g32::TM - 1) / g32::TM));
  if (acc32) hipLaunchKernelGGL(g32::gemm32_kernel<false>, grid, dim3(g32::NT), 0, (hipStream_t)stream, a);
  else hipLaunchKernelGGL(g32::gemm32_kernel<true>, grid, dim3(g32::NT), 0, (hipStream_t)stream, a);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}
