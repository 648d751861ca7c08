// Probe: lane layout of global_load_lds_dwordx3 in LDS (lane * 12 B or lane * 16 B?) and the
// saddr form of global_store_dwordx3.  Prints PASS/FAIL lines.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
__global__ void k(const uint32_t* src, uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[1024];
  const int lane = threadIdx.x;
  for (int i = lane; i < 1024; i += 64) lds[i] = 0xdeadbeefu;
  __syncthreads();
  const uint32_t voff = lane * 12;
  const uint32_t m0 = (uint32_t)(uintptr_t)((__attribute__((address_space(3))) uint32_t*)lds) + 64;
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx3 %0, %1\n\ts_waitcnt vmcnt(0)"
               : : "v"(voff), "s"(src), "s"(m0) : "memory", "m0");
  __syncthreads();
  for (int i = lane; i < 1024; i += 64) out[i] = lds[i];
  // store: lane writes 3 dwords at out2 + lane * 12 bytes (saddr form)
  uint32_t* out2 = out + 1024;
  const uint32_t a0 = 1000 + 3 * lane, a1 = a0 + 1, a2 = a0 + 2;
  typedef uint32_t u3 __attribute__((ext_vector_type(3)));
  u3 d = {a0, a1, a2};
  asm volatile("global_store_dwordx3 %0, %1, %2\n\ts_nop 1\n\ts_waitcnt vmcnt(0)" : : "v"(voff), "v"(d), "s"(out2) : "memory");
}
int main() {
  uint32_t *src, *out;
  hipMalloc(&src, 4096 * 4); hipMalloc(&out, 4096 * 4);
  uint32_t h[4096];
  for (int i = 0; i < 4096; ++i) h[i] = i;
  hipMemcpy(src, h, sizeof(h), hipMemcpyHostToDevice);
  hipMemset(out, 0, 4096 * 4);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, src, out);
  hipError_t e = hipDeviceSynchronize();
  hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost);
  printf("sync: %s\n", hipGetErrorString(e));
  // expected with 12-B lane stride: lds[16 + 3*lane + j] = src[3*lane + j] for j < 3 (m0 offset 64 B = 16 dwords)
  int ok12 = 1, ok16 = 1;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 3; ++j) {
      if (h[16 + 3 * l + j] != (uint32_t)(3 * l + j)) ok12 = 0;
      if (h[16 + 4 * l + j] != (uint32_t)(3 * l + j)) ok16 = 0;
    }
  printf("ldsdma_x3 lane stride 12 B: %s; 16 B: %s\n", ok12 ? "PASS" : "FAIL", ok16 ? "PASS" : "FAIL");
  printf("lds[16..24] = %u %u %u %u %u %u %u %u\n", h[16], h[17], h[18], h[19], h[20], h[21], h[22], h[23]);
  int oks = 1;
  for (int l = 0; l < 64; ++l)
    for (int j = 0; j < 3; ++j)
      if (h[1024 + 3 * l + j] != (uint32_t)(1000 + 3 * l + j)) oks = 0;
  printf("store_dwordx3 saddr lane*12: %s\n", oks ? "PASS" : "FAIL");
  return 0;
}
