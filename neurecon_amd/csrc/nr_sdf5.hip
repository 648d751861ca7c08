// neurecon_amd — SDF MLP forward (ImplicitSurface.forward, models/base.py:243-263) on
// v_mfma_f32_32x32x16_f16: one wave per SIMD, 32 points per wave, 128 points per workgroup tile.
//
// The f16x3 design of sdf4_kernel (nr_mlp.hip, DESIGN.md §2.1: weights streamed HBM/L2 -> LDS by
// LDS-DMA, per-point power-of-two operand scales fixed before each op from pack-time bounds, the
// accumulator of op l is the B operand of op l+1, the previous chunk's epilogue staged beside the
// current chunk's MFMAs), on the 32x32x16 MFMA instead of 16x16x32:
//  * one A-fragment read (ds_read_b128, 1 KB per wave) serves 32 points instead of 16, so a chunk's
//    32 weight rows x K cost 2 reads per 16 k (hi, lo) per 32 points;
//  * an MFMA holds the SIMD's issue for 8 of its 32 cycles (MI355X_MICROARCH.md, cycle constants), so
//    24 cycles of every MFMA gap are left for the epilogue VALU, fragment reads and DMA pieces
//    (16x16x32: 8 of 16) -- 1.5x the issue room per MAC;
//  * one wave per SIMD (512 registers): both 32-point operands (hi + lo f16, up to 18 k-steps x 8
//    registers each) stay resident.
// Layouts:
//  * lane l: point r = l & 31 of the wave's 32, half h = l >> 5;
//  * B operand, k-step s (16 input features), element j of lane (r, h): feature
//    16 s + 8 (j >> 2) + 4 h + (j & 3) of point r;
//  * accumulator of an output chunk c (32 rows): register i of lane (r, h) holds row
//    32 c + (i & 3) + 8 (i >> 2) + 4 h, so registers 0..7 are k-step 2c and 8..15 k-step 2c+1 of the
//    next op's B operand, element j = i (mod 8) -- no permutation at all;
//  * packed A (pack_word's l32 layout): chunk c = [k-step s][hi, lo][lane][8 halves], lane (r, h)
//    element j = W[row 32 c + r][feature 16 s + 8 (j >> 2) + 4 h + (j & 3)]; the same bytes per chunk
//    as the 16x16x32 pack (2 KB per input block + the 1 KB bias slot).
#include "nr_common.h"
#include "nr_mlp.h"
#include <type_traits>

namespace nr {
namespace s5 {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kW = 4;           // waves per workgroup: one per SIMD
constexpr int kT = 64 * kW;     // 256 threads
constexpr int kTilePts = 32 * kW;  // 128 points per tile
constexpr int kRing = 4;        // weight-ring slots: three chunks in flight
constexpr float kT2 = 144.26944f;      // ~100 log2(e) (nr_mlp.hip kT: kT2 * kC2 = 1 within 2e-10)
constexpr float kC2 = 0.0069314749f;   // ~ln2 / 100
constexpr float kSpSlack = 0.0070f;    // softplus(z) <= max(z, 0) + ln2/100

__host__ __device__ constexpr int cbytes(int KB) { return (2 * KB + 1) * 1024; }

__device__ __forceinline__ f32x16 mfma32(f16x8 a, f16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}

template <class T>
__device__ __forceinline__ T* uniform_ptr(T* p) {
  const uint64_t v = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v), hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (T*)(uintptr_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t lds_u32(const void* p) {
  return (uint32_t)(uintptr_t)((__attribute__((address_space(3))) const char*)p);
}
// s_waitcnt vmcnt(n) for a runtime n (immediate operand)
__device__ __forceinline__ void wait_vmcnt(int n) {
  switch (n) {
    case 0: asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); break;
    case 1: asm volatile("s_waitcnt vmcnt(1)" ::: "memory"); break;
    case 2: asm volatile("s_waitcnt vmcnt(2)" ::: "memory"); break;
    case 3: asm volatile("s_waitcnt vmcnt(3)" ::: "memory"); break;
    case 4: asm volatile("s_waitcnt vmcnt(4)" ::: "memory"); break;
    case 5: asm volatile("s_waitcnt vmcnt(5)" ::: "memory"); break;
    case 6: asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); break;
    case 7: asm volatile("s_waitcnt vmcnt(7)" ::: "memory"); break;
    case 8: asm volatile("s_waitcnt vmcnt(8)" ::: "memory"); break;
    case 9: asm volatile("s_waitcnt vmcnt(9)" ::: "memory"); break;
    case 10: asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); break;
    case 11: asm volatile("s_waitcnt vmcnt(11)" ::: "memory"); break;
    case 12: asm volatile("s_waitcnt vmcnt(12)" ::: "memory"); break;
    case 13: asm volatile("s_waitcnt vmcnt(13)" ::: "memory"); break;
    case 14: asm volatile("s_waitcnt vmcnt(14)" ::: "memory"); break;
    case 15: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
    case 16: asm volatile("s_waitcnt vmcnt(16)" ::: "memory"); break;
    case 17: asm volatile("s_waitcnt vmcnt(17)" ::: "memory"); break;
    case 18: asm volatile("s_waitcnt vmcnt(18)" ::: "memory"); break;
    case 19: asm volatile("s_waitcnt vmcnt(19)" ::: "memory"); break;
    case 20: asm volatile("s_waitcnt vmcnt(20)" ::: "memory"); break;
    case 21: asm volatile("s_waitcnt vmcnt(21)" ::: "memory"); break;
    default: asm volatile("s_waitcnt vmcnt(22)" ::: "memory"); break;  // callers stay <= 22
  }
}

// one 1 KB LDS-DMA piece (64 lanes x 16 B), wave-uniform global base + per-lane offset; inline asm so
// that the compiler neither waits for it before ds_reads nor drains it at barriers (nr_mlp.hip glds16m)
__device__ __forceinline__ void dma_piece(const char* sbase, uint32_t voff, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, %1"
               :
               : "v"(voff), "s"(sbase), "s"(lds_addr)
               : "memory", "m0");
}

// Weight ring: kRing chunk slots; chunk c + 3 is issued during chunk c into the slot chunk c - 1 left.
// Every wave is a loader: a chunk's NB 1 KB pieces are dealt as runs of NPW = ceil(NB / 4) per wave
// (the last run shifted back to end at the chunk's end: overlapping pieces write identical bytes), and a
// wave issues its run piece by piece inside the chunk's k-step regions (beside the MFMAs), not as a
// burst at the chunk start: with one wave per SIMD nothing else would issue MFMAs meanwhile.
// V: experiment bits (nr_sdf5_enable(1 + V)): 1 fragments two k-steps ahead; timing only (results
// invalid): 2 no epilogue, 4 no weight DMA, 8 no chunk barrier
template <int CBMAX, int V>
struct Ring {
  static constexpr int kV = V;
  char* lds;
  int cur;   // slot of the chunk being computed
  int prev;  // pieces this wave issued in the previous chunk iteration
  __device__ __forceinline__ static int wave() { return __builtin_amdgcn_readfirstlane(threadIdx.x >> 6); }
  template <int BYTES>
  __device__ __forceinline__ static constexpr int npw() { return (BYTES / 1024 + kW - 1) / kW; }
  __device__ __forceinline__ int ahead_slot() const { return cur == 0 ? kRing - 1 : cur - 1; }
  template <int BYTES>
  __device__ __forceinline__ void piece(const char* gsrc, int slot, int j) const {
    constexpr int NB = BYTES / 1024, NPW = npw<BYTES>();
    const int first = __builtin_amdgcn_readfirstlane(min(wave() * NPW, NB - NPW)) + j;
    dma_piece(uniform_ptr(gsrc) + first * 1024, (threadIdx.x & 63) * 16u,
              __builtin_amdgcn_readfirstlane(lds_u32(lds) + (uint32_t)(slot * CBMAX) + (uint32_t)(first * 1024)));
  }
  template <int BYTES>
  __device__ __forceinline__ void all(const char* gsrc, int slot) const {
#pragma unroll
    for (int j = 0; j < npw<BYTES>(); ++j) piece<BYTES>(gsrc, slot, j);
  }
  template <int B0>
  __device__ __forceinline__ void start(const char* g) {
    cur = 0;
    all<B0>(g, 0);
    all<B0>(g + B0, 1);
    all<B0>(g + 2 * B0, 2);
    prev = npw<B0>();
    wait_vmcnt(2 * npw<B0>());
    __syncthreads();
  }
  __device__ __forceinline__ const float4* buf() const {
    uint32_t off = cur * CBMAX;
    asm volatile("" : "+s"(off));
    return (const float4*)(lds + off);
  }
  // n: pieces issued in this iteration; chunk c + 1 went out two iterations ago
  __device__ __forceinline__ void flip(int n) {
    wait_vmcnt(n + prev);
    prev = n;
    if constexpr (!(V & 8)) __syncthreads();
    cur = cur == kRing - 1 ? 0 : cur + 1;
  }
};

// hi = f16(v sc), lo = f16(v sc - hi) for 8 values, packed pairs by v_fma_mix (nr_mlp.hip split8a)
__device__ __forceinline__ void split8(const float (&v)[8], float sc, f16x8& h, f16x8& l) {
  uint32_t hw[4], lw[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    uint32_t hh;
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, 0" : "=v"(hh) : "v"(v[2 * i]), "v"(sc));
    asm volatile("v_fma_mixhi_f16 %0, %1, %2, 0" : "+v"(hh) : "v"(v[2 * i + 1]), "v"(sc));
    uint32_t lo;
    asm volatile("v_fma_mixlo_f16 %0, %1, %2, -%3 op_sel_hi:[0,0,1]" : "=v"(lo) : "v"(v[2 * i]), "v"(sc), "v"(hh));
    asm volatile("v_fma_mixhi_f16 %0, %1, %2, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
                 : "+v"(lo)
                 : "v"(v[2 * i + 1]), "v"(sc), "v"(hh));
    hw[i] = hh;
    lw[i] = lo;
  }
  h = __builtin_bit_cast(f16x8, make_uint4(hw[0], hw[1], hw[2], hw[3]));
  l = __builtin_bit_cast(f16x8, make_uint4(lw[0], lw[1], lw[2], lw[3]));
}
// ... parked in AGPRs: B operands are read only by MFMAs, which take AGPR sources directly, and the
// 256 VGPRs stay free for the epilogue (both operands of an op pair need 272 registers)
__device__ __forceinline__ void split8a(const float (&v)[8], float sc, f16x8& h, f16x8& l) {
  split8(v, sc, h, l);
  asm volatile("" : "+a"(h), "+a"(l));
}
// power-of-two scale putting a bound M at < 2^14 (1 for M = 0, inf or NaN)
__device__ __forceinline__ float bound_scale(float M) {
  if (!(M > 0.0f) || __builtin_isinf(M)) return 1.0f;
  return __builtin_ldexpf(1.0f, 14 - __builtin_amdgcn_frexp_expf(M));
}
// max / sum over the two halves of a point (lanes l, l ^ 32)
__device__ __forceinline__ float max_halves(float m) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(m), __float_as_uint(m), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
// v(lane r) + v(lane r + 32) in every lane of the pair (v_permlane32_swap of v with itself returns
// the low half's values in r[0] and the high half's in r[1], in all 64 lanes)
__device__ __forceinline__ float sum_halves(float v) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// positional encoding (models/base.py:14-81), as nr_mlp.hip's embed_feature
__device__ __noinline__ float embed_feature5(int f, float x0, float x1, float x2, int nfreq) {
  if (f < 3) return f == 0 ? x0 : (f == 1 ? x1 : x2);
  const int fp = f - 3;
  if (fp >= 6 * nfreq) return 0.0f;
  const int band = fp / 6, m = fp - band * 6, c = m % 3;
  const float xc = c == 0 ? x0 : (c == 1 ? x1 : x2);
  const float v = fmul(xc, (float)(1 << band));
  return m < 3 ? sinf(v) : cosf(v);
}

// compile-time loop: f(std::integral_constant<int, I>{}) for I = 0 .. N-1
template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

__device__ __forceinline__ f16x8 frag(const float4* __restrict__ A, int i, int lane) {
  return __builtin_bit_cast(f16x8, A[i * 64 + lane]);
}

// One chunk's products: acc += A[32 rows x 16 KB] · B, three f16 products per k-step (lo·hi, hi·lo,
// hi·hi, the small terms first), fragments read one k-step ahead; stage(s) is VALU work (the previous
// chunk's epilogue, DMA pieces) placed in k-step s's scheduling region beside its MFMAs.
template <int KB, bool PF2, int NB, class Stage>
__device__ __forceinline__ void mma5(const float4* __restrict__ A, const f16x8 (&bh)[NB], const f16x8 (&bl)[NB],
                                     f32x16& acc, int lane, Stage&& stage) {
  static_assert(KB <= NB, "operand k-steps");
  constexpr int D = PF2 ? 2 : 1;  // k-steps of fragment prefetch
  f16x8 fh[D + 1], fl[D + 1];
#pragma unroll
  for (int d = 0; d < D; ++d)
    if (d < KB) {
      fh[d] = frag(A, 2 * d, lane);
      fl[d] = frag(A, 2 * d + 1, lane);
    }
#pragma unroll
  for (int s = 0; s < KB; ++s) {
    const f16x8 h = fh[s % (D + 1)], l = fl[s % (D + 1)];
    if (s + D < KB) {
      fh[(s + D) % (D + 1)] = frag(A, 2 * (s + D), lane);
      fl[(s + D) % (D + 1)] = frag(A, 2 * (s + D) + 1, lane);
    }
    stage(s);
    acc = mfma32(l, bh[s], acc);
    acc = mfma32(h, bl[s], acc);
    acc = mfma32(h, bh[s], acc);
    if (s + D < KB) __builtin_amdgcn_sched_group_barrier(0x100, 2, 0);
    __builtin_amdgcn_sched_group_barrier(0x008, 3, 0);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// a finished chunk: raw accumulators, the scale and bias that turn them into pre-activations, and the
// op's per-row vector (F7: the sdf row W8[0, :]) -- read from the chunk's LDS slot before its flip
struct Z5 {
  f32x16 acc;
  float4 b[4];    // rows 8q + 4h .. +3 of the chunk, q = register group
  float4 aux[4];
  float inv;
};

// One GEMM op (NBO / 2 chunks of 32 rows, fully unrolled): chunk c's epilogue runs in chunk c+1's
// iteration, its 8 stages spread over the k-steps; the DMA pieces of chunk c + 3 (this op's or the next
// op's) go out one per k-step region from region 1 on.
template <int KB, int NBO, int NXT_CB, bool AUX, bool TS, int NB, class R, class Epi>
__device__ __forceinline__ void op5(R& ring, const char* __restrict__ op, const char* nxt, const f16x8 (&bh)[NB],
                                    const f16x8 (&bl)[NB], float xinv, Epi&& epi, int lane) {
  constexpr int CB = cbytes(KB);
  constexpr int NCH = NBO / 2;
  constexpr int LA = kRing - 1;
  static_assert(NCH >= 2, "ops of >= 2 chunks");
  const int h = lane >> 5;
  Z5 zq;
  static_for<0, NCH>([&](auto ci) {
    constexpr int c = decltype(ci)::value;
    const char* opc = op;
    const char* nxc = nxt;
    asm volatile("" : "+s"(opc), "+s"(nxc));
    // this iteration's DMA: chunk c + LA of this op, or of the next op (with no next op, harmless bytes
    // of this op into the free slot: the piece count, and with it every wait, stays a constant)
    constexpr bool OWN = c + LA < NCH;
    constexpr int DB = OWN ? CB : NXT_CB;
    const char* dsrc = OWN ? opc + (c + LA) * CB : (nxc ? nxc + (c + LA - NCH) * NXT_CB : opc);
    constexpr int npend = R::template npw<DB>();
    const int slot = ring.ahead_slot();
    const float4* A = ring.buf();
    f32x16 acc = {};
    mma5<KB, (R::kV & 1) != 0>(A, bh, bl, acc, lane, [&](int s) {
      if constexpr (!(R::kV & 4)) {
#pragma unroll
        for (int j = 0; j < npend; ++j)
          if (1 + j * (KB - 1) / npend == s) ring.template piece<DB>(dsrc, slot, j);
      }
      if constexpr (R::kV & 2) {
        if (s == 0) asm volatile("" : : "a"(zq.acc));
      } else if constexpr (c > 0) {
        constexpr int NST = std::decay_t<Epi>::kStages;
#pragma unroll
        for (int e = 0; e < NST; ++e)
          if (e * KB / NST == s) epi(c - 1, zq, e);
      }
    });
    zq.acc = acc;
    float wi = A[2 * KB * 64 + 8].x;
    if constexpr (TS) wi *= kT2;
    zq.inv = xinv * wi;
#pragma unroll
    for (int q = 0; q < 4; ++q) zq.b[q] = A[2 * KB * 64 + (TS ? 24 : 0) + 2 * q + h];
    if constexpr (AUX) {
#pragma unroll
      for (int q = 0; q < 4; ++q) zq.aux[q] = A[2 * KB * 64 + 16 + 2 * q + h];
    }
    ring.flip(npend);
  });
  if constexpr (R::kV & 2) {
    asm volatile("" : : "a"(zq.acc));
  } else {
#pragma unroll
    for (int e = 0; e < std::decay_t<Epi>::kStages; ++e) epi(NCH - 1, zq, e);
  }
}

__device__ __forceinline__ float f4(const float4& v, int r) { return r == 0 ? v.x : (r == 1 ? v.y : (r == 2 ? v.z : v.w)); }

// forward softplus op (TS: the accumulators give t = 100 log2(e) z), nr_mlp.hip FwdEpi4's arithmetic:
//   L = log2(1 + 2^min(t, 126)),  y = max(L, t) ln2/100;
// the 16 outputs of chunk c become k-steps 2c, 2c+1 of the next operand (split at the scale sc fixed
// before the op); the running max tracks max(L, t).  LAST (F7): instead of the split, the sdf row's
// running dot product sdf_part += y * W8[0, row].
template <int NO, bool LAST>
struct FwdEpi5 {
  f16x8 (&oh)[NO];
  f16x8 (&ol)[NO];
  float sc;     // operand scale of the outputs (the split multiplies max(L, t) by sc ln2/100)
  float& mrun;
  float& sdf_part;
  float t[16], e[16], m[16];
  // kStages stages of roughly equal issue cost (~48-64 cycles: 16 plain VALU or 8 transcendentals),
  // two halves of 8 values each, spread over the chunk's k-step regions by op5
  static constexpr int kStages = 11;
  __device__ __forceinline__ void operator()(int c, const Z5& z, int st) {
    if (st <= 1) {  // A: pre-activations t (100 log2(e) z) and the exp2 argument, half st
      const int i0 = 8 * st;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int i = i0 + k;
        t[i] = __builtin_fmaf(z.acc[i], z.inv, f4(z.b[i >> 2], i & 3));
        e[i] = fminf(t[i], 126.0f);
      }
    } else if (st <= 3) {  // B: 2^t
      const int i0 = 8 * (st - 2);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[i0 + k] = __builtin_amdgcn_exp2f(e[i0 + k]);
    } else if (st == 4) {  // C: 1 + 2^t
#pragma unroll
      for (int i = 0; i < 16; ++i) e[i] = e[i] + 1.0f;
    } else if (st <= 6) {  // D: L = log2(1 + 2^t)
      const int i0 = 8 * (st - 5);
#pragma unroll
      for (int k = 0; k < 8; ++k) e[i0 + k] = __builtin_amdgcn_logf(e[i0 + k]);
    } else if (st <= 8) {  // E: max(L, t) and the running max (softplus ops) / nothing (F7)
      const int i0 = 8 * (st - 7);
#pragma unroll
      for (int k = 0; k < 8; ++k) m[i0 + k] = fmaxf(e[i0 + k], t[i0 + k]);
      if constexpr (!LAST) {
        float r = mrun;
#pragma unroll
        for (int k = 0; k < 8; k += 2) r = __builtin_fmaxf(r, __builtin_fmaxf(m[i0 + k], m[i0 + k + 1]));
        mrun = r;
      }
    } else {  // F: k-step 2c + half of the next operand / the sdf row's dot product (F7)
      const int i0 = 8 * (st - 9);
      if constexpr (LAST) {
        float sp = sdf_part;
#pragma unroll
        for (int k = 0; k < 8; ++k) sp = __builtin_fmaf(m[i0 + k] * kC2, f4(z.aux[(i0 + k) >> 2], k & 3), sp);
        sdf_part = sp;
      } else {
        const float v[8] = {m[i0], m[i0 + 1], m[i0 + 2], m[i0 + 3], m[i0 + 4], m[i0 + 5], m[i0 + 6], m[i0 + 7]};
        split8a(v, sc * kC2, oh[2 * c + (st - 9)], ol[2 * c + (st - 9)]);
      }
    }
  }
};

struct Sdf5Args {
  const char* packed;  // the l32 copy of the ops (SdfLayout::l32_off)
  SdfLayout L;
  const float* pts;
  int64_t P;
  float* sdf;
  int nfreq;
  const int* P_dev;
  int P_mult;
};

// SDF forward (sdf only), persistent over 128-point tiles
template <int V>
__global__ __attribute__((amdgpu_flat_work_group_size(kT, kT), amdgpu_waves_per_eu(1, 1)))
void sdf5_fwd_kernel(Sdf5Args a) {
  constexpr int C4 = cbytes(4), C16 = cbytes(16), C18 = cbytes(18);
  __shared__ __attribute__((aligned(16))) char smem[kRing * C18];
  Ring<C18, V> ring{smem, 0, 0};
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int r = lane & 31, h = lane >> 5;
  const char* W = a.packed;
  auto OP = [&](int i) {
    const char* w = W;
    asm volatile("" : "+s"(w));
    return w + sdf_op_off(i);
  };
  const float b8 = *(const float*)(a.packed - a.L.l32_off + a.L.misc_off);
  ring.template start<C4>(OP(F0));
  const int64_t Pn = a.P_dev ? min(a.P, (int64_t)(*a.P_dev) * a.P_mult) : a.P;
  for (int64_t base = (int64_t)blockIdx.x * kTilePts; base < Pn; base += (int64_t)gridDim.x * kTilePts) {
    const bool has_next = base + (int64_t)gridDim.x * kTilePts < Pn;
    const int64_t p = base + wave * 32 + r;
    const bool valid = p < Pn;
    const int64_t pq = valid ? p : Pn - 1;
    const float x0 = a.pts[pq * 3 + 0], x1 = a.pts[pq * 3 + 1], x2 = a.pts[pq * 3 + 2];
    f16x8 Uh[18], Ul[18], Vh[16], Vl[16];
    // embedding, k-steps 0..3 (features 0..63, 39 valid), element j of k-step s: 16 s + 8 (j >> 2) + 4 h + (j & 3)
    float E[32];
    float mE = 0.0f;
#pragma unroll
    for (int i = 0; i < 32; ++i) {
      const int s = i >> 3, j = i & 7;
      E[i] = embed_feature5(16 * s + 8 * (j >> 2) + 4 * h + (j & 3), x0, x1, x2, a.nfreq);
      mE = fmaxf(mE, fabsf(E[i]));
    }
    mE = max_halves(mE);
    {
      const float sE = bound_scale(mE);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float v[8] = {E[8 * s], E[8 * s + 1], E[8 * s + 2], E[8 * s + 3],
                            E[8 * s + 4], E[8 * s + 5], E[8 * s + 6], E[8 * s + 7]};
        split8a(v, sE, Uh[s], Ul[s]);
      }
    }
    float xinv = 1.0f / bound_scale(mE), m_in = mE, mrun = 0.0f, sdf_part = 0.0f;
    auto next_scale = [&](int kb, float floor_max) {
      const float4 v = ring.buf()[2 * kb * 64 + 8];
      return bound_scale(fmaxf(fmaf(v.y, m_in, v.z) + kSpSlack, floor_max));
    };
    auto finish = [&](float sc) {
      m_in = max_halves(mrun) * kC2;
      mrun = 0.0f;
      xinv = 1.0f / sc;
    };
    // ---- forward (base.py:243-257) ----
    {
      const float sc = next_scale(4, 0.0f);
      op5<4, 16, C16, false, true>(ring, OP(F0), OP(F1), Uh, Ul, xinv, FwdEpi5<16, false>{Vh, Vl, sc, mrun, sdf_part}, lane);
      finish(sc);
    }
    {
      const float sc = next_scale(16, 0.0f);
      op5<16, 16, C16, false, true>(ring, OP(F1), OP(F2), Vh, Vl, xinv, FwdEpi5<18, false>{Uh, Ul, sc, mrun, sdf_part}, lane);
      finish(sc);
    }
    {
      const float sc = next_scale(16, 0.0f);
      op5<16, 16, C16, false, true>(ring, OP(F2), OP(F3), Uh, Ul, xinv, FwdEpi5<16, false>{Vh, Vl, sc, mrun, sdf_part}, lane);
      finish(sc);
    }
    {
      // F3's outputs (h3: 217 rows in 14 blocks -> k-steps 0..13) and the embedding (k-steps 14..17)
      // form F4's operand: one scale
      const float sc = next_scale(16, mE);
      op5<16, 14, C18, false, true>(ring, OP(F3), OP(F4), Vh, Vl, xinv, FwdEpi5<18, false>{Uh, Ul, sc, mrun, sdf_part}, lane);
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const float v[8] = {E[8 * s], E[8 * s + 1], E[8 * s + 2], E[8 * s + 3],
                            E[8 * s + 4], E[8 * s + 5], E[8 * s + 6], E[8 * s + 7]};
        split8(v, sc, Uh[14 + s], Ul[14 + s]);
      }
      mrun = fmaxf(mrun, mE * (1.0f / kC2));  // mrun is in max(L, t) units here
      finish(sc);
    }
    {
      const float sc = next_scale(18, 0.0f);
      op5<18, 16, C16, false, true>(ring, OP(F4), OP(F5), Uh, Ul, xinv, FwdEpi5<16, false>{Vh, Vl, sc, mrun, sdf_part}, lane);
      finish(sc);
    }
    {
      const float sc = next_scale(16, 0.0f);
      op5<16, 16, C16, false, true>(ring, OP(F5), OP(F6), Vh, Vl, xinv, FwdEpi5<18, false>{Uh, Ul, sc, mrun, sdf_part}, lane);
      finish(sc);
    }
    {
      const float sc = next_scale(16, 0.0f);
      op5<16, 16, C16, false, true>(ring, OP(F6), OP(F7), Uh, Ul, xinv, FwdEpi5<16, false>{Vh, Vl, sc, mrun, sdf_part}, lane);
      finish(sc);
    }
    // F7: softplus and the sdf row (aux = W8[0, :]) as a running dot product
    op5<16, 16, C4, true, true>(ring, OP(F7), has_next ? OP(F0) : nullptr, Vh, Vl, xinv,
                                FwdEpi5<18, true>{Uh, Ul, 1.0f, mrun, sdf_part}, lane);
    const float sdf = sum_halves(sdf_part) + b8;
    if (valid && h == 0) a.sdf[p] = sdf;
  }
  wait_vmcnt(0);
}

}  // namespace s5

int launch_sdf5_fwd(const SdfLayout& L, const void* packed, const float* pts, int64_t P, float* sdf, int nfreq,
                    hipStream_t stream, const int* P_dev, int P_mult) {
  if (P <= 0) return NR_OK;
  NR_REQUIRE(L.prec == NR_PREC_F16X3 && !L.siren && L.l32_off, NR_ERR_UNSUPPORTED, "sdf5: f16x3 softplus nets only");
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t need = (P + s5::kTilePts - 1) / s5::kTilePts;
  const int grid = (int)(need < cus ? need : cus);
  s5::Sdf5Args a{(const char*)packed + L.l32_off, L, pts, P, sdf, nfreq, P_dev, P_mult};
  ProfScope prof("sdf_fwd", (double)P, stream, P_dev, P_mult);
  switch (g_sdf5) {
    case 2: hipLaunchKernelGGL(s5::sdf5_fwd_kernel<1>, dim3(grid), dim3(s5::kT), 0, stream, a); break;
    case 3: hipLaunchKernelGGL(s5::sdf5_fwd_kernel<2>, dim3(grid), dim3(s5::kT), 0, stream, a); break;
    case 4: hipLaunchKernelGGL(s5::sdf5_fwd_kernel<4>, dim3(grid), dim3(s5::kT), 0, stream, a); break;
    case 5: hipLaunchKernelGGL(s5::sdf5_fwd_kernel<8>, dim3(grid), dim3(s5::kT), 0, stream, a); break;
    case 6: hipLaunchKernelGGL(s5::sdf5_fwd_kernel<14>, dim3(grid), dim3(s5::kT), 0, stream, a); break;
    default: hipLaunchKernelGGL(s5::sdf5_fwd_kernel<0>, dim3(grid), dim3(s5::kT), 0, stream, a); break;
  }
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

}  // namespace nr

extern "C" int nr_sdf5_enable(int on) {
  const int was = nr::g_sdf5;
  if (on > 0 && !nr::g_sdf5_pack) {
    nr::set_error("nr_sdf5_enable: start the process with NR_SDF5 set (the packs then carry the 32x32x16 layout)");
    return -1;
  }
  nr::g_sdf5 = on < 0 ? 0 : on;  // 1: the kernel; 2..6: experiment variants (tools/sdf5_ab.py)
  return was;
}
