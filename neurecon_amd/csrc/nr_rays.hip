// neurecon_amd — pixel -> ray generation (utils/rend_util.py:95-164, `get_rays` + `lift`).
#include "nr_common.h"

namespace nr {

// one thread per (camera b, ray n).  Pixel coords are integer indices (torch.linspace(0, W-1, W)
// is exact): i = column, j = row; no +0.5 centre offset (rend_util.py:126-128).
__global__ void get_rays_kernel(const float* __restrict__ c2w, const float* __restrict__ K, int B, int H, int W,
                                const int64_t* __restrict__ sel, int64_t N, float* __restrict__ ro,
                                float* __restrict__ rd) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * N) return;
  const int b = (int)(t / N);
  const int64_t n = t - (int64_t)b * N;
  const int64_t pix = sel ? sel[t] : n;
  const float x = (float)(pix % W), y = (float)(pix / W);
  const float* k = K + b * 16;
  const float fx = k[0], fy = k[5], cx = k[2], cy = k[6], sk = k[1];
  // lift (rend_util.py:105-106), z = 1
  const float xl = fdiv(fsub(fadd(fsub(x, cx), fdiv(fmul(cy, sk), fy)), fdiv(fmul(sk, y), fy)), fx);
  const float yl = fdiv(fsub(y, cy), fy);
  const float* m = c2w + b * 16;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float w = fadd(fadd(fadd(fmul(m[c * 4 + 0], xl), fmul(m[c * 4 + 1], yl)), m[c * 4 + 2]), m[c * 4 + 3]);
    ro[t * 3 + c] = m[c * 4 + 3];
    rd[t * 3 + c] = fsub(w, m[c * 4 + 3]);
  }
}

}  // namespace nr

extern "C" int nr_get_rays(const float* c2w, const float* K, int B, int H, int W, const int64_t* select_inds,
                           int64_t N, float* rays_o, float* rays_d, void* stream) {
  NR_REQUIRE(c2w && K && rays_o && rays_d && B >= 0 && H > 0 && W > 0, NR_ERR_ARG, "nr_get_rays: bad argument");
  const int64_t total = (int64_t)B * N;
  if (total <= 0) return NR_OK;
  hipLaunchKernelGGL(nr::get_rays_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     c2w, K, B, H, W, select_inds, N, rays_o, rays_d);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

namespace nr {
// training ray batch targets (neus.py:432, :449): out[b, n, :] = src[b, idx[b, n], :] for rows of
// row_bytes bytes (rgb: 12, mask: 1 or 4), one thread per output byte-word
__global__ void gather_rows_kernel(const uint8_t* __restrict__ src, int64_t HW, int64_t row_bytes,
                                   const int64_t* __restrict__ idx, int64_t N, int64_t total, uint8_t* __restrict__ out) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= total) return;
  const int64_t row = t / row_bytes, k = t - row * row_bytes;
  const int64_t b = row / N;
  out[t] = src[(b * HW + idx[row]) * row_bytes + k];
}
}  // namespace nr

extern "C" int nr_gather_rows(const void* src, int64_t B, int64_t HW, int64_t row_bytes, const int64_t* idx,
                              int64_t N, void* out, void* stream) {
  NR_REQUIRE(src && idx && out && B >= 0 && HW > 0 && row_bytes > 0 && N >= 0, NR_ERR_ARG,
             "nr_gather_rows: bad argument");
  const int64_t total = B * N * row_bytes;
  if (total <= 0) return NR_OK;
  hipLaunchKernelGGL(nr::gather_rows_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                     (const uint8_t*)src, HW, row_bytes, idx, N, total, (uint8_t*)out);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}
