// neurecon_amd — fused SDF / radiance MLP kernels for gfx950 (MI355X, CDNA4).
//
// Replaces ImplicitSurface.forward / forward_with_nablas (models/base.py:243-282) and
// RadianceNet.forward (models/base.py:372-391) of SuwoongHeo/neurecon.
//
// Design:
//  * Transposed GEMM formulation: activations are held as Xᵀ [features x points]; one wave owns a
//    tile of 16 points, a workgroup of 8 waves owns 128 points.  With v_mfma_f32_16x16x4_f32 the
//    accumulator of layer l (rows = output features, cols = points) is *directly* the B operand of
//    layer l+1: register r of 16-feature block b in lane-group g holds feature 16b+4g+r, which is
//    the k-index g of k-step (b,r).  No LDS round trip or shuffle between layers; the weight
//    packing (host side) applies the matching k permutation.
//  * Weights are streamed through LDS in chunks of 2 output blocks (32 output features x K) by
//    global_load_lds (LDS-DMA), double buffered, shared by the 8 waves.
//  * Softplus(beta=100) keeps exp(100 z) per element; the reverse pass (nablas) reloads it from a
//    per-wave scratch slab and applies torch's softplus_backward formula g*e/(e+1).
//  * Everything per point (embedding, nabla chain rule through sin/cos, sdf row dot product,
//    sigmoid head) is VALU work in the same kernel.
#include "nr_common.h"
#include "nr_mlp.h"

namespace nr {

using lds_ptr = __attribute__((address_space(3))) void*;

// ---------------------------------------------------------------------------------------------
// LDS weight stream: 2 buffers of kMaxChunkBytes, filled by LDS-DMA (global_load_lds, 16 B/lane)
// ---------------------------------------------------------------------------------------------
struct WStream {
  char* lds;
  int cur;
  __device__ __forceinline__ void issue(const char* gsrc, int bytes) {
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    char* dst = lds + (cur ^ 1) * kMaxChunkBytes;
    for (int off = wave * 1024; off < bytes; off += kThreads * 16) {
      __builtin_amdgcn_global_load_lds((const void*)(gsrc + off + lane * 16), (lds_ptr)(dst + off), 16, 0, 0);
    }
  }
  __device__ __forceinline__ const float4* buf() const { return (const float4*)(lds + cur * kMaxChunkBytes); }
  __device__ __forceinline__ void flip() {
    __syncthreads();  // drains the LDS-DMA (vmcnt) and orders it for every wave
    cur ^= 1;
  }
};

__device__ __forceinline__ f32x4 mfma4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 tof(float4 v) { return f32x4{v.x, v.y, v.z, v.w}; }
__device__ __forceinline__ float4 fromf(f32x4 v) { return make_float4(v[0], v[1], v[2], v[3]); }

// One chunk = 2 output blocks.  A layout in LDS: [obl(2)][b(KB)][lane(64)] float4 (r = .x.y.z.w)
// Software-pipelined one input block deep: the A fragments of block b+1 are read from LDS while
// block b's 8 MFMAs issue; sched_barrier stops hipcc from hoisting every LDS read of the chunk
// (which would cost ~128 VGPRs and force spills at 2 waves/SIMD).
template <int KBX, int KBE>
__device__ __forceinline__ void mma_chunk(const float4* __restrict__ A, const float4 (&X)[16], const float4 (&E)[4],
                                          f32x4& acc0, f32x4& acc1, int lane) {
  constexpr int KB = KBX + KBE;
  float4 n0 = A[lane], n1 = A[KB * 64 + lane];
#pragma unroll
  for (int b = 0; b < KB; ++b) {
    const float4 a0 = n0, a1 = n1;
    if (b + 1 < KB) {
      n0 = A[(b + 1) * 64 + lane];
      n1 = A[(KB + b + 1) * 64 + lane];
    }
    const float4 x = b < KBX ? X[b < KBX ? b : 0] : E[b < KBX ? 0 : b - KBX];
    acc0 = mfma4(a0.x, x.x, acc0);
    acc1 = mfma4(a1.x, x.x, acc1);
    acc0 = mfma4(a0.y, x.y, acc0);
    acc1 = mfma4(a1.y, x.y, acc1);
    acc0 = mfma4(a0.z, x.z, acc0);
    acc1 = mfma4(a1.z, x.z, acc1);
    acc0 = mfma4(a0.w, x.w, acc0);
    acc1 = mfma4(a1.w, x.w, acc1);
    __builtin_amdgcn_sched_barrier(0);
  }
}

// rotate-in a pair of output blocks: after N/2 pushes Y[0..N-1] holds the outputs in order
template <int N>
__device__ __forceinline__ void push2(float4 (&Y)[16], float4 a, float4 b) {
#pragma unroll
  for (int i = 0; i + 2 < N; ++i) Y[i] = Y[i + 2];
  Y[N - 2] = a;
  Y[N - 1] = b;
}
// same over the concatenation [Y[0..N1-1], Z[0..N2-1]]
template <int N1, int N2>
__device__ __forceinline__ void push2cat(float4 (&Y)[16], float4 (&Z)[4], float4 a, float4 b) {
  constexpr int N = N1 + N2;
#pragma unroll
  for (int i = 0; i + 2 < N; ++i) {
    const float4 v = (i + 2 < N1) ? Y[i + 2] : Z[i + 2 - N1];
    if (i < N1) Y[i] = v; else Z[i - N1] = v;
  }
  if (N - 2 < N1) Y[N - 2] = a; else Z[N - 2 - N1] = a;
  if (N - 1 < N1) Y[N - 1] = b; else Z[N - 1 - N1] = b;
}

// ---------------------------------------------------------------------------------------------
// activations (torch CPU semantics, models/base.py:202, :361-363)
// ---------------------------------------------------------------------------------------------
// Softplus(beta=100, threshold=20): y = (100 z > 20) ? z : log1p(exp(100 z)) / 100.
// e = exp(100 z) is kept for the backward (softplus_backward: g * e / (e + 1)); +inf marks the
// linear branch (gradient passes through unchanged).
__device__ __forceinline__ void softplus_fwd(float z, float& y, float& e) {
  const float t = fmul(z, 100.0f);
  const float ex = expf(t);
  const bool lin = t > 20.0f;
  y = lin ? z : fdiv(log1pf(ex), 100.0f);
  e = lin ? __builtin_inff() : ex;
}
__device__ __forceinline__ float softplus_bwd(float g, float e) {
  return __builtin_isinf(e) ? g : fdiv(fmul(g, e), fadd(e, 1.0f));
}

enum { ACT_NONE = 0, ACT_SOFTPLUS = 1, ACT_RELU = 2 };

// chunk = [A: 2*KB KB][bias slot: 32 floats (2 output blocks), padded to 1 KB]
__host__ __device__ constexpr int chunk_bytes(int KB) { return (2 * KB + 1) * 1024; }

// Forward GEMM layer: Y[0..NBO) = act(W · [X[0..KBX) ; E[0..KBE)] + bias).
// `op` chunks are consumed from the stream; `nxt/nxt_bytes` is the chunk that follows this op.
template <int KBX, int KBE, int NBO, int ACT>
__device__ __forceinline__ void gemm_fwd(WStream& ws, const char* __restrict__ op, const char* nxt, int nxt_bytes,
                                         const float4 (&X)[16], const float4 (&E)[4], float4 (&Y)[16],
                                         float4* __restrict__ e_out, float* __restrict__ feat_out, bool feat_ok,
                                         int lane) {
  constexpr int KB = KBX + KBE;
  constexpr int CB = chunk_bytes(KB);
  const int g = lane >> 4;
#pragma unroll 1
  for (int c = 0; c < NBO / 2; ++c) {
    if (c + 1 < NBO / 2) ws.issue(op + (c + 1) * CB, CB);
    else if (nxt) ws.issue(nxt, nxt_bytes);
    const float4* A = ws.buf();
    f32x4 acc0 = tof(A[2 * KB * 64 + g]);
    f32x4 acc1 = tof(A[2 * KB * 64 + 4 + g]);
    mma_chunk<KBX, KBE>(A, X, E, acc0, acc1, lane);
    float4 y0, y1;
    if constexpr (ACT == ACT_SOFTPLUS) {
      float4 e0, e1;
      softplus_fwd(acc0[0], y0.x, e0.x); softplus_fwd(acc0[1], y0.y, e0.y);
      softplus_fwd(acc0[2], y0.z, e0.z); softplus_fwd(acc0[3], y0.w, e0.w);
      softplus_fwd(acc1[0], y1.x, e1.x); softplus_fwd(acc1[1], y1.y, e1.y);
      softplus_fwd(acc1[2], y1.z, e1.z); softplus_fwd(acc1[3], y1.w, e1.w);
      if (e_out) {
        e_out[(2 * c) * 64 + lane] = e0;
        e_out[(2 * c + 1) * 64 + lane] = e1;
      }
    } else if constexpr (ACT == ACT_RELU) {
      y0 = make_float4(fmaxf(acc0[0], 0.f), fmaxf(acc0[1], 0.f), fmaxf(acc0[2], 0.f), fmaxf(acc0[3], 0.f));
      y1 = make_float4(fmaxf(acc1[0], 0.f), fmaxf(acc1[1], 0.f), fmaxf(acc1[2], 0.f), fmaxf(acc1[3], 0.f));
    } else {
      y0 = fromf(acc0);
      y1 = fromf(acc1);
    }
    if (feat_out && feat_ok) {  // row-major [P][256] feature rows of this chunk
      *(float4*)(feat_out + (2 * c) * 16 + g * 4) = y0;
      *(float4*)(feat_out + (2 * c + 1) * 16 + g * 4) = y1;
    }
    push2<NBO>(Y, y0, y1);
    ws.flip();
  }
}

// Backward GEMM layer: out = Wᵀ · G (no bias).  The first NBO1 output blocks are scaled by
// softplus'(z) of the previous layer (e_prev) and rotated into Y; the remaining NBO2 blocks are
// gradients w.r.t. the positional encoding and are handed to `emb(block, value)` as produced.
template <int KBG, int NBO1, int NBO2, class EmbFn>
__device__ __forceinline__ void gemm_bwd(WStream& ws, const char* __restrict__ op, const char* nxt, int nxt_bytes,
                                         const float4 (&G)[16], float4 (&Y)[16], const float4* __restrict__ e_prev,
                                         int lane, EmbFn&& emb) {
  constexpr int NBO = NBO1 + NBO2;
  static_assert(NBO1 % 2 == 0 && NBO2 % 2 == 0, "output segments must be chunk aligned");
  constexpr int CB = chunk_bytes(KBG);
  const float4 dummy[4] = {};
#pragma unroll 1
  for (int c = 0; c < NBO / 2; ++c) {
    if (c + 1 < NBO / 2) ws.issue(op + (c + 1) * CB, CB);
    else if (nxt) ws.issue(nxt, nxt_bytes);
    const bool main = 2 * c < NBO1;
    float4 e0 = make_float4(0, 0, 0, 0), e1 = e0;
    if (main && e_prev) {
      e0 = e_prev[(2 * c) * 64 + lane];
      e1 = e_prev[(2 * c + 1) * 64 + lane];
    }
    f32x4 acc0 = {0, 0, 0, 0}, acc1 = {0, 0, 0, 0};
    mma_chunk<KBG, 0>(ws.buf(), G, dummy, acc0, acc1, lane);
    float4 y0 = fromf(acc0), y1 = fromf(acc1);
    if (main) {
      if (e_prev) {
        y0 = make_float4(softplus_bwd(y0.x, e0.x), softplus_bwd(y0.y, e0.y), softplus_bwd(y0.z, e0.z),
                         softplus_bwd(y0.w, e0.w));
        y1 = make_float4(softplus_bwd(y1.x, e1.x), softplus_bwd(y1.y, e1.y), softplus_bwd(y1.z, e1.z),
                         softplus_bwd(y1.w, e1.w));
      }
      if constexpr (NBO1 > 0) push2<NBO1>(Y, y0, y1);
    } else {
      emb(2 * c - NBO1, y0);
      emb(2 * c + 1 - NBO1, y1);
    }
    ws.flip();
  }
}

// ---------------------------------------------------------------------------------------------
// positional encoding (models/base.py:14-81): feature f of [x, sin(x), cos(x), sin(2x), ...]
// ---------------------------------------------------------------------------------------------
// noinline: the accurate sinf/cosf expansions are large; one call per feature keeps code and
// register pressure of the (once per tile) encoding small
__device__ __noinline__ float embed_feature(int f, float x0, float x1, float x2, int nfreq) {
  if (f < 3) return f == 0 ? x0 : (f == 1 ? x1 : x2);
  const int fp = f - 3;
  if (fp >= 6 * nfreq) return 0.0f;
  const int band = fp / 6, m = fp - band * 6, c = m % 3;
  const float xc = c == 0 ? x0 : (c == 1 ? x1 : x2);
  const float v = fmul(xc, (float)(1 << band));
  return m < 3 ? sinf(v) : cosf(v);
}
// d/dx of the embedding, applied to the gradient gf of feature f (autograd: Sin/CosBackward
// then MulBackward by freq), accumulated into n[c]
__device__ __noinline__ void embed_backward(int f, float gf, float x0, float x1, float x2, int nfreq, float& n0,
                                            float& n1, float& n2) {
  float contrib;
  int c;
  if (f < 3) {
    contrib = gf;
    c = f;
  } else {
    const int fp = f - 3;
    if (fp >= 6 * nfreq) return;
    const int band = fp / 6, m = fp - band * 6;
    c = m % 3;
    const float freq = (float)(1 << band);
    const float xc = c == 0 ? x0 : (c == 1 ? x1 : x2);
    const float v = fmul(xc, freq);
    contrib = m < 3 ? fmul(fmul(gf, cosf(v)), freq) : fmul(fmul(gf, -sinf(v)), freq);
  }
  if (c == 0) n0 = fadd(n0, contrib);
  else if (c == 1) n1 = fadd(n1, contrib);
  else n2 = fadd(n2, contrib);
}

__device__ __forceinline__ float wave_sum4(float v) {  // sum over the 4 lane-groups of a point
  v += __shfl_xor(v, 16);
  v += __shfl_xor(v, 32);
  return v;
}

// =============================================================================================
// SDF kernel
// =============================================================================================
struct SdfKArgs {
  const char* packed;
  SdfLayout L;
  const float* pts;
  int64_t P;
  float* sdf;
  float* nabla;
  float* feature;
  float4* scratch;  // [grid*8 waves][8 layers][16 blocks][64 lanes] float4
  int nfreq;
};

template <bool NABLA>
__global__ __launch_bounds__(kThreads) void sdf_kernel(SdfKArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kMaxChunkBytes];
  WStream ws{smem, 1};
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const SdfLayout& L = a.L;
  const char* W = a.packed;
  auto OP = [&](int i) { return W + L.op_off[i]; };
  auto OPB = [&](int i) { return (int)L.op_bytes[i]; };
  const float* w8 = (const float*)(W + L.w8row0_off);
  const float b8 = *(const float*)(W + L.misc_off);
  float4* escr = a.scratch + (size_t)(blockIdx.x * kWaves + wave) * (8 * 16 * 64);
  const bool want_feat = a.feature != nullptr;

  // first chunk of the stream
  ws.issue(OP(F0), OPB(F0));
  ws.flip();

  for (int64_t base = (int64_t)blockIdx.x * kPointsPerWG; base < a.P; base += (int64_t)gridDim.x * kPointsPerWG) {
    const bool has_next = base + (int64_t)gridDim.x * kPointsPerWG < a.P;
    const int64_t p = base + wave * kTile + j;
    const bool valid = p < a.P;
    const int64_t pc = valid ? p : a.P - 1;
    const float x0 = a.pts[pc * 3 + 0], x1 = a.pts[pc * 3 + 1], x2 = a.pts[pc * 3 + 2];

    float4 E[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = 16 * b + 4 * g;
      E[b] = make_float4(embed_feature(f + 0, x0, x1, x2, a.nfreq), embed_feature(f + 1, x0, x1, x2, a.nfreq),
                         embed_feature(f + 2, x0, x1, x2, a.nfreq), embed_feature(f + 3, x0, x1, x2, a.nfreq));
    }
    float4 X[16], Y[16];
    float4* e_l[8];
#pragma unroll
    for (int l = 0; l < 8; ++l) e_l[l] = NABLA ? escr + l * 16 * 64 : nullptr;

    // ---- forward (base.py:243-257) -----------------------------------------------------------
    gemm_fwd<0, 4, 16, ACT_SOFTPLUS>(ws, OP(F0), OP(F1), OPB(F1), X, E, Y, e_l[0], nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_SOFTPLUS>(ws, OP(F1), OP(F2), OPB(F2), Y, E, X, e_l[1], nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_SOFTPLUS>(ws, OP(F2), OP(F3), OPB(F3), X, E, Y, e_l[2], nullptr, false, lane);
    gemm_fwd<16, 0, 14, ACT_SOFTPLUS>(ws, OP(F3), OP(F4), OPB(F4), Y, E, X, e_l[3], nullptr, false, lane);
    gemm_fwd<14, 4, 16, ACT_SOFTPLUS>(ws, OP(F4), OP(F5), OPB(F5), X, E, Y, e_l[4], nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_SOFTPLUS>(ws, OP(F5), OP(F6), OPB(F6), Y, E, X, e_l[5], nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_SOFTPLUS>(ws, OP(F6), OP(F7), OPB(F7), X, E, Y, e_l[6], nullptr, false, lane);
    {
      const char* n = want_feat ? OP(F8) : (NABLA ? OP(B7) : (has_next ? OP(F0) : nullptr));
      const int nb = want_feat ? OPB(F8) : (NABLA ? OPB(B7) : OPB(F0));
      gemm_fwd<16, 0, 16, ACT_SOFTPLUS>(ws, OP(F7), n, nb, Y, E, X, e_l[7], nullptr, false, lane);
    }
    // ---- last layer, row 0 = sdf (VALU dot product) ---------------------------------------------
    float part = 0.0f;
#pragma unroll
    for (int b = 0; b < 16; ++b) {
      const float4 w = *(const float4*)(w8 + 16 * b + 4 * g);
      part = fmaf(X[b].x, w.x, part);
      part = fmaf(X[b].y, w.y, part);
      part = fmaf(X[b].z, w.z, part);
      part = fmaf(X[b].w, w.w, part);
    }
    const float sdf = wave_sum4(part) + b8;
    if (valid && g == 0) a.sdf[p] = sdf;
    // ---- geometry feature rows 1..256 -------------------------------------------------------------
    if (want_feat) {
      const char* n = NABLA ? OP(B7) : (has_next ? OP(F0) : nullptr);
      const int nb = NABLA ? OPB(B7) : OPB(F0);
      gemm_fwd<16, 0, 16, ACT_NONE>(ws, OP(F8), n, nb, X, E, Y, nullptr, a.feature + pc * 256, valid,
                                    lane);
    }
    if constexpr (NABLA) {
      // ---- reverse pass (autograd.grad of sdf w.r.t. x, base.py:265-282) ---------------------------
      // d sdf / d h7 = W8[0,:], scaled by softplus'(z7); h7 (X) is dead now and holds the gradient
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const float4 w = *(const float4*)(w8 + 16 * b + 4 * g);
        const float4 e = e_l[7][b * 64 + lane];
        X[b] = make_float4(softplus_bwd(w.x, e.x), softplus_bwd(w.y, e.y), softplus_bwd(w.z, e.z),
                           softplus_bwd(w.w, e.w));
      }
      // gradients w.r.t. the positional encoding (skip layer + first layer) are parked in the
      // (already consumed) layer-7 slab and folded into the nabla after the GEMM chain
      float4* park = e_l[7];
      auto emb_skip = [&](int eb, float4 gv) { park[eb * 64 + lane] = gv; };
      auto emb_first = [&](int eb, float4 gv) { park[(4 + eb) * 64 + lane] = gv; };
      auto noemb = [](int, float4) {};
      gemm_bwd<16, 16, 0>(ws, OP(B7), OP(B6), OPB(B6), X, Y, e_l[6], lane, noemb);
      gemm_bwd<16, 16, 0>(ws, OP(B6), OP(B5), OPB(B5), Y, X, e_l[5], lane, noemb);
      gemm_bwd<16, 16, 0>(ws, OP(B5), OP(B4), OPB(B4), X, Y, e_l[4], lane, noemb);
      // skip layer: rows 0..216 -> h3 (scaled by softplus'(z3)), rows 217..255 -> embedding
      gemm_bwd<16, 14, 4>(ws, OP(B4), OP(B3), OPB(B3), Y, X, e_l[3], lane, emb_skip);
      gemm_bwd<14, 16, 0>(ws, OP(B3), OP(B2), OPB(B2), X, Y, e_l[2], lane, noemb);
      gemm_bwd<16, 16, 0>(ws, OP(B2), OP(B1), OPB(B1), Y, X, e_l[1], lane, noemb);
      gemm_bwd<16, 16, 0>(ws, OP(B1), OP(B0), OPB(B0), X, Y, e_l[0], lane, noemb);
      gemm_bwd<16, 0, 4>(ws, OP(B0), has_next ? OP(F0) : nullptr, OPB(F0), Y, X, nullptr, lane, emb_first);
      // chain rule through the positional encoding (autograd sums both uses of embed(x))
      float n0 = 0.f, n1 = 0.f, n2 = 0.f;
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const float4 u = park[b * 64 + lane], v = park[(4 + b) * 64 + lane];
        const int f = 16 * b + 4 * g;
        embed_backward(f + 0, fadd(v.x, u.x), x0, x1, x2, a.nfreq, n0, n1, n2);
        embed_backward(f + 1, fadd(v.y, u.y), x0, x1, x2, a.nfreq, n0, n1, n2);
        embed_backward(f + 2, fadd(v.z, u.z), x0, x1, x2, a.nfreq, n0, n1, n2);
        embed_backward(f + 3, fadd(v.w, u.w), x0, x1, x2, a.nfreq, n0, n1, n2);
      }
      n0 = wave_sum4(n0);
      n1 = wave_sum4(n1);
      n2 = wave_sum4(n2);
      if (valid && g == 0) {
        a.nabla[p * 3 + 0] = n0;
        a.nabla[p * 3 + 1] = n1;
        a.nabla[p * 3 + 2] = n2;
      }
    }
  }
}

// =============================================================================================
// Radiance kernel (RadianceNet): cat([x, embed_view(v), normals, feature]) -> 4x ReLU(256) -> 3
// =============================================================================================
struct RadKArgs {
  const char* packed;
  RadLayout L;
  const float* x;
  const float* vdir;
  int64_t vdiv;
  int64_t vmod;
  const float* normals;
  const float* feature;
  int64_t P;
  float* rgb;
  int nfreq_view;  // <0: identity
};

// small input features [x(3), view-embedding(3+6F or 3), normals(3)] in block layout
__device__ __forceinline__ float rad_small_feature(int f, const float (&x)[3], const float (&v)[3],
                                                   const float (&n)[3], int nfreq_view) {
  if (f < 3) return x[f];
  f -= 3;
  const int nv = nfreq_view < 0 ? 3 : 3 + 6 * nfreq_view;
  if (f < nv) return embed_feature(f, v[0], v[1], v[2], nfreq_view < 0 ? 0 : nfreq_view);
  f -= nv;
  if (f < 3) return n[f];
  return 0.0f;
}

template <int KBS>
__global__ __launch_bounds__(kThreads) void radiance_kernel(RadKArgs a) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kMaxChunkBytes];
  WStream ws{smem, 1};
  const int lane = threadIdx.x & 63, wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int j = lane & 15, g = lane >> 4;
  const RadLayout& L = a.L;
  const char* W = a.packed;
  auto OP = [&](int i) { return W + L.op_off[i]; };
  auto OPB = [&](int i) { return (int)L.op_bytes[i]; };
  const float* head = (const float*)(W + L.head_off);  // [3][256] weights then [3] bias

  ws.issue(OP(0), OPB(0));
  ws.flip();
  for (int64_t base = (int64_t)blockIdx.x * kPointsPerWG; base < a.P; base += (int64_t)gridDim.x * kPointsPerWG) {
    const bool has_next = base + (int64_t)gridDim.x * kPointsPerWG < a.P;
    const int64_t p = base + wave * kTile + j;
    const bool valid = p < a.P;
    const int64_t pc = valid ? p : a.P - 1;
    float xs[3], vs[3], ns[3];
    const int64_t pv = (pc / a.vdiv) % a.vmod;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      xs[c] = a.x[pc * 3 + c];
      vs[c] = a.vdir[pv * 3 + c];
      ns[c] = a.normals[pc * 3 + c];
    }
    float4 S[4];
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int f = 16 * b + 4 * g;
      S[b] = b < KBS ? make_float4(rad_small_feature(f, xs, vs, ns, a.nfreq_view),
                                   rad_small_feature(f + 1, xs, vs, ns, a.nfreq_view),
                                   rad_small_feature(f + 2, xs, vs, ns, a.nfreq_view),
                                   rad_small_feature(f + 3, xs, vs, ns, a.nfreq_view))
                     : make_float4(0, 0, 0, 0);
    }
    float4 X[16], Y[16];
#pragma unroll
    for (int b = 0; b < 16; ++b) X[b] = *(const float4*)(a.feature + pc * 256 + 16 * b + 4 * g);

    gemm_fwd<16, KBS, 16, ACT_RELU>(ws, OP(0), OP(1), OPB(1), X, S, Y, nullptr, nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_RELU>(ws, OP(1), OP(2), OPB(2), Y, S, X, nullptr, nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_RELU>(ws, OP(2), OP(3), OPB(3), X, S, Y, nullptr, nullptr, false, lane);
    gemm_fwd<16, 0, 16, ACT_RELU>(ws, OP(3), has_next ? OP(0) : nullptr, OPB(0), Y, S, X, nullptr,
                                  nullptr, false, lane);
    // head: Linear(256 -> 3) + sigmoid  (VALU dot products)
    float r[3];
#pragma unroll
    for (int o = 0; o < 3; ++o) {
      float part = 0.f;
#pragma unroll
      for (int b = 0; b < 16; ++b) {
        const float4 w = *(const float4*)(head + o * 256 + 16 * b + 4 * g);
        part = fmaf(X[b].x, w.x, part);
        part = fmaf(X[b].y, w.y, part);
        part = fmaf(X[b].z, w.z, part);
        part = fmaf(X[b].w, w.w, part);
      }
      r[o] = sigmoidf_ref(wave_sum4(part) + head[3 * 256 + o]);
    }
    if (valid && g == 0) {
      a.rgb[p * 3 + 0] = r[0];
      a.rgb[p * 3 + 1] = r[1];
      a.rgb[p * 3 + 2] = r[2];
    }
  }
}

// =============================================================================================
// weight packing (device): effective W [rows][ld] -> chunk layout of one GEMM op
// =============================================================================================
__global__ void pack_op_kernel(PackOp op, float* __restrict__ dst, int64_t n) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  const int KB = op.in[0].nblk + op.in[1].nblk;
  const int per_chunk = (2 * KB + 1) * 256;  // floats
  const int c = (int)(e / per_chunk);
  const int w = (int)(e - (int64_t)c * per_chunk);
  float v = 0.0f;
  if (w >= 2 * KB * 256) {  // bias slot: 2 blocks x 16 rows, then padding
    const int idx = w - 2 * KB * 256;
    if (idx < 32 && op.bias) {
      int ob_loc = 2 * c + idx / 16;
      for (int s = 0; s < 2; ++s) {
        if (ob_loc < op.out[s].nblk) {
          const int rl = 16 * ob_loc + (idx & 15);
          if (rl < op.out[s].nvalid) v = op.bias[op.out[s].off + rl];
          break;
        }
        ob_loc -= op.out[s].nblk;
      }
    }
    dst[e] = v;
    return;
  }
  const int r = w & 3;
  const int lane = (w >> 2) & 63;
  const int t = w >> 8;
  const int b = t % KB;
  const int obl = t / KB;
  const int ob = 2 * c + obl;
  const int i = lane & 15, gg = lane >> 4;
  int row = -1;
  {
    int ob_loc = ob;
    for (int s = 0; s < 2; ++s) {
      if (ob_loc < op.out[s].nblk) {
        const int rl = 16 * ob_loc + i;
        if (rl < op.out[s].nvalid) row = op.out[s].off + rl;
        break;
      }
      ob_loc -= op.out[s].nblk;
    }
  }
  int col = -1;
  {
    int b_loc = b;
    for (int s = 0; s < 2; ++s) {
      if (b_loc < op.in[s].nblk) {
        const int cl = 16 * b_loc + 4 * gg + r;
        if (cl < op.in[s].nvalid) col = op.in[s].off + cl;
        break;
      }
      b_loc -= op.in[s].nblk;
    }
  }
  if (row >= 0 && col >= 0) v = (op.transpose ? op.W[(int64_t)col * op.ld + row] : op.W[(int64_t)row * op.ld + col]) * op.scale;
  dst[e] = v;
}

__global__ void pack_vec_kernel(const float* __restrict__ src, int off, int nvalid, int n, float* __restrict__ dst) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= n) return;
  dst[e] = e < nvalid ? src[off + e] : 0.0f;
}

// ---------------------------------------------------------------------------------------------
// host side
// ---------------------------------------------------------------------------------------------
int launch_pack_op(const PackOp& op, char* dst, hipStream_t stream) {
  const int KB = op.in[0].nblk + op.in[1].nblk;
  const int NBO = op.out[0].nblk + op.out[1].nblk;
  const int64_t n = (int64_t)(NBO / 2) * (2 * KB + 1) * 256;
  hipLaunchKernelGGL(pack_op_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, stream, op, (float*)dst, n);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

int launch_pack_vec(const float* src, int off, int nvalid, int n, char* dst, hipStream_t stream) {
  hipLaunchKernelGGL(pack_vec_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, src, off, nvalid, n, (float*)dst);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

static int grid_for(int64_t P) {
  int dev = 0, cus = 256;
  if (hipGetDevice(&dev) == hipSuccess) hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  const int64_t need = (P + kPointsPerWG - 1) / kPointsPerWG;
  return (int)(need < cus ? (need > 0 ? need : 1) : cus);
}

int launch_sdf(const SdfLayout& L, const void* packed, const float* pts, int64_t P, float* sdf, float* nabla,
               float* feature, int nfreq, void* ws, size_t ws_bytes, hipStream_t stream) {
  if (P <= 0) return NR_OK;
  const int grid = grid_for(P);
  SdfKArgs a{(const char*)packed, L, pts, P, sdf, nabla, feature, (float4*)ws, nfreq};
  ProfScope prof(nabla ? (feature ? "sdf_nabla_feat" : "sdf_nabla") : (feature ? "sdf_feat" : "sdf_fwd"), (double)P,
                 stream);
  if (nabla) {
    const size_t need = (size_t)grid * kScratchPerWG;
    NR_REQUIRE(ws && ws_bytes >= need, NR_ERR_WORKSPACE, "sdf nabla workspace too small");
    hipLaunchKernelGGL(sdf_kernel<true>, dim3(grid), dim3(kThreads), 0, stream, a);
  } else {
    hipLaunchKernelGGL(sdf_kernel<false>, dim3(grid), dim3(kThreads), 0, stream, a);
  }
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

int launch_radiance(const RadLayout& L, const void* packed, const float* x, const float* vdir, int64_t vdiv,
                    int64_t vmod, const float* normals, const float* feature, int64_t P, float* rgb, int nfreq_view,
                    hipStream_t stream) {
  if (P <= 0) return NR_OK;
  const int grid = grid_for(P);
  RadKArgs a{(const char*)packed, L, x, vdir, vdiv, vmod, normals, feature, P, rgb, nfreq_view};
  ProfScope prof("radiance", (double)P, stream);
  switch (L.kbs) {
    case 2: hipLaunchKernelGGL(radiance_kernel<2>, dim3(grid), dim3(kThreads), 0, stream, a); break;
    case 4: hipLaunchKernelGGL(radiance_kernel<4>, dim3(grid), dim3(kThreads), 0, stream, a); break;
    default: set_error("radiance: unsupported small-input block count"); return NR_ERR_UNSUPPORTED;
  }
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

}  // namespace nr
