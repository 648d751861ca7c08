// neurecon_amd -- weight gradients of the training step on MFMA (gfx950): C = scale * sum_q A_q^T B_q.
//
// The training step's layer weight gradients (models/base.py:118-129 DenseLayer under the double
// backward of base.py:265-282 and train.py:205) are products of two tall activation matrices over the
// sample points: dW_l = zbar_l^T hin_l (+ delta_l^T hdot_in_l for the tangent sweep), A [P, m] and
// B [P, n] row-major fp32 with P ~ 65 k and m, n <= 289.  The contraction runs over the ROW index of
// both operands, so each is transposed on its way through LDS:
//
//  * grid = S row slices x (m tiles of 256) x (n tiles of 128); a workgroup (8 waves) accumulates its
//    256 x 128 output tile over its slice, 32 rows (one MFMA k-step) at a time, and writes a partial;
//    wgrad_reduce sums the S partials in slice order (deterministic) into C.  The n tiles of one slice
//    run on one XCD back to back (blockIdx -> XCD is round robin), so their shared A rows come from L2.
//  * k-step: every wave loads 32 A columns of the 32 rows (4 x 16 B per lane) and 16 B columns
//    (2 x 16 B) through buffer resources rebased per k-step (rows past P read as zero; loop-invariant
//    lane offsets; operands row-major or 16 x 16 blocked, NrWgrad.blocked), three k-steps in flight in
//    registers, every load issued unconditionally (no branch around a load).
//  * per column quad (4 columns x 32 rows) a running power-of-two scale: the quad's max (DPP row
//    rotations + permlane16/32 swaps) only lowers the exponent, with 16x headroom, when it would reach
//    2^14; v * scale split into f16 hi + lo (22 significant bits), both planes written row-major into
//    LDS (row strides 544 / 288 B: the 8 rows a 32-lane half reads land 8 banks apart);
//    double-buffered stages, one barrier per k-step.
//  * MFMA operands come back with ds_read_b64_tr_b16 (4 rows x 16 columns, delivered column-major):
//    lane group G of a 16x16x32 operand takes rows {4G..4G+3} and {16+4G..16+4G+3}, the same rows for
//    A and B, so each k-slot pairs the same point.  Per 16x16 tile and k-step Al Bh + Ah Bl + Ah Bh
//    accumulate in place (a lane's 4 output rows are one A quad and its column one B quad); a k-step that
//    lowered an exponent rescales the affected tiles by 2^(e_new - e_old) first, and 2^-(eA + eB) is
//    applied once at the end.
//  * optional: column sums of A_0 (the bias gradient) and B_0^T v for a [P] vector v (the sdf row of
//    the output layer, dW8[0, :]) accumulated in fp32 from the loaded values, reduced in fixed order.
//  * NrWgrad.fp32 (the fp32-precision nets' training step): the same loaders, slices and reduction with
//    exact fp32 products on v_mfma_f32_16x16x4_f32.  The k-step's rows are stored into LDS as fp32 (the
//    A / B row images take the bytes of the hi + lo planes: 272 / 144 floats per row, 16 banks apart
//    per row, so a fragment's 2 x 16 consecutive floats per 32 lanes read conflict-free) and each
//    16 x 16 tile accumulates 8 k-substeps of 4 rows in order: A[i][k] = a[p0 + k][m0 + i] is lane
//    (k, i)'s ds_read_b32, B[k][j] likewise.  Each slice sums its rows in order, the slices are summed
//    in fixed order: a deterministic fp32 reduction in place of hipBLASLt's split-K products.
#include <algorithm>
#include <cstdlib>
#include "nr_common.h"

namespace nr {

constexpr int kWgThreads = 512;   // 8 waves: wave w owns output rows [32 w, 32 w + 32) of the m tile
constexpr int kWgM = 256, kWgN = 128, kWgK = 32;
#ifndef NR_WG_PP_BIT
#define NR_WG_PP_BIT 0
#endif
// waves w with (w & bit) run the split before the MFMAs; 0 = none (measured r04: splitting the phases
// between the two waves of a SIMD, bit 4, took 114 us per two-pair call against 104-107 without)
constexpr int kPingPongBit = NR_WG_PP_BIT;
constexpr int kAStride = 272;     // halfs per A row in LDS (544 B: 8 rows of a half-wave read land 8 banks apart)
constexpr int kBStride = 144;     // halfs per B row (288 B, the same property)
constexpr int kAPlane = kWgK * kAStride;
constexpr int kBPlane = kWgK * kBStride;
constexpr int kStage = 2 * kAPlane + 2 * kBPlane;  // halfs: A hi, A lo, B hi, B lo

struct WgKArgs {
  const float* a[2];
  int64_t lda[2];
  const float* b[2];
  int64_t ldb[2];
  int npairs;
  int64_t P;
  int m, n;
  int nmt, nnt, S;
  int64_t KP;        // 32-row steps per pair: ceil(P / 32)
  float* part;       // [S][nnt * 128][nmt * 256]
  float* part_cs;    // [S][nmt * 256] column sums of A_0 (nullptr: none)
  const float* avec; // [P] at avec[p * ldv] (nullptr: none)
  int64_t ldv;
  float* part_vec;   // [S][nnt * 128]
  int blocked;       // NR_WG_BLK_* bits
};

typedef short v4s __attribute__((ext_vector_type(4)));
using lds_v4s = __attribute__((address_space(3))) v4s;

__device__ __forceinline__ v4s tr16(const _Float16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)((__attribute__((address_space(3))) _Float16*)p));
}

__device__ __forceinline__ f16x8 frag(const _Float16* plane, int stride, int col, int lane) {
  // rows {4G + q} and {16 + 4G + q} of the 16-column block starting at `col` (T10 addressing: lane
  // 4q + p' of its 16-lane group supplies row q's columns 4p' .. 4p' + 3)
  const int G = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const v4s lo = tr16(plane + (4 * G + q) * stride + col + 4 * p);
  const v4s hi = tr16(plane + (16 + 4 * G + q) * stride + col + 4 * p);
  const short s[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  f16x8 r;
#pragma unroll
  for (int e = 0; e < 8; ++e) r[e] = __builtin_bit_cast(_Float16, s[e]);
  return r;
}

// max over lanes l ^ 8, l ^ 16, l ^ 32 (and l ^ 4 with FOUR), all VALU: DPP row rotations within each
// 16-lane row (by 4 and 8: the set {l, l +- 4, l + 8}; by 8: {l, l ^ 8}), then permlane16 / permlane32
// swaps (a wave-wide max of the pair (v, swapped v) is the max over l and l ^ 16, resp. l ^ 32)
template <bool FOUR>
__device__ __forceinline__ float quad_max(float v) {
  if constexpr (FOUR)
    v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false)));
  v = fmaxf(v, __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false)));
  const auto r16 = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(r16[0]), __uint_as_float(r16[1]));
  const auto r32 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(r32[0]), __uint_as_float(r32[1]));
}

// power-of-two exponent e with M * 2^e < 2^14, at most kExpCap (also for M = 0 / inf / NaN): a quad of
// tiny values (|v| < 2^-86, e.g. adjoints of points the loss does not see) would otherwise get an
// infinite scale 2^e (and 0 * inf = NaN); capped, such values flush to zero in f16 -- contributions
// below 2^-86 of the operand scale
constexpr int kExpCap = 100;
constexpr int kHeadroom = 4;
__device__ __forceinline__ int split_exp(float M) {
  if (!(M > 0.0f) || __builtin_isinf(M)) return kExpCap;
  return min(14 - __builtin_amdgcn_frexp_expf(M), kExpCap);
}

// v * 2^e -> (hi, lo) f16 pairs, 4 values: 8 B each plane
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ void split4(float4 v, float sc, uint2& h, uint2& l) {
  const float x[4] = {v.x * sc, v.y * sc, v.z * sc, v.w * sc};
  _Float16 hh[4], ll[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    hh[e] = (_Float16)x[e];
    ll[e] = (_Float16)(x[e] - (float)hh[e]);
  }
  h = make_uint2(__builtin_bit_cast(uint32_t, h2{hh[0], hh[1]}), __builtin_bit_cast(uint32_t, h2{hh[2], hh[3]}));
  l = make_uint2(__builtin_bit_cast(uint32_t, h2{ll[0], ll[1]}), __builtin_bit_cast(uint32_t, h2{ll[2], ll[3]}));
}

// Operand loads go through buffer resources rebased at each k-step's first row and sized to the rows
// left before P: an offset past the size reads as zero, so rows past P need no test; a lane whose
// columns lie past the operand's width (or an idle wave) uses an out-of-range offset.  The per-lane
// offsets are loop invariant, so a k-step's loads cost no vector ALU and no branch (a divergent branch
// around a load makes the compiler wait for every load in flight, which defeats the prefetch).  Each
// operand spans < 2^31 bytes (checked on the host).
constexpr uint32_t kOob = 0x80000000u;
constexpr int kRsrcFlags = 0x00020000;  // gfx9 buffer resource word 3 (32-bit dword format)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const float* p, int64_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc((void*)p, (short)0, (int)bytes, kRsrcFlags);
}
typedef int i32x4 __attribute__((ext_vector_type(4)));

// byte offset of (row, col) in a row-major or 16 x 16 blocked operand (include/neurecon_hip.h NR_BLK_*;
// rows relative to a 16-aligned k-step start), or kOob when the lane is off / col >= ncol
__device__ __forceinline__ uint32_t lane_off(int row, int col, int64_t ld, int ncol, bool on, bool blk) {
  if (!(on && col < ncol)) return kOob;
  if (blk)
    return ((((uint32_t)row >> 4) * (uint32_t)(ld >> 4) + ((uint32_t)col >> 4)) * 256u + ((uint32_t)row & 15u) * 16u +
            ((uint32_t)col & 15u)) * 4u;
  return (uint32_t)(row * ld + col) * 4u;
}

// 4 consecutive columns at byte offset o (kOob: zeros).  VEC: ncol % 4 == 0 and 16-byte aligned rows
// (one dwordx4); otherwise four dwords, each tested against ncol (c = the first column)
template <bool VEC>
__device__ __forceinline__ float4 ld4(__amdgpu_buffer_rsrc_t rs, uint32_t o, int c, int ncol) {
  if constexpr (VEC) {
    const i32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, o, 0, 0);
    return make_float4(__int_as_float(v[0]), __int_as_float(v[1]), __int_as_float(v[2]), __int_as_float(v[3]));
  } else {
    float v[4];
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, o != kOob && c + e < ncol ? o + 4u * e : kOob, 0, 0));
    return make_float4(v[0], v[1], v[2], v[3]);
  }
}

__device__ __forceinline__ float4 add4(float4 a, float4 b) { return make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ float4 fma4(float s, float4 b, float4 c) {
  return make_float4(fmaf(s, b.x, c.x), fmaf(s, b.y, c.y), fmaf(s, b.z, c.z), fmaf(s, b.w, c.w));
}
__device__ __forceinline__ float4 shfl_xor4(float4 v, int o) {
  return make_float4(__shfl_xor(v.x, o), __shfl_xor(v.y, o), __shfl_xor(v.z, o), __shfl_xor(v.w, o));
}
__device__ __forceinline__ float amax4(float4 v) {
  return fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w)));
}

// one k-step's operands in registers: A rows (lane >> 3) + 8 j, B rows (lane >> 2) + 16 j
struct WgRegs {
  float4 va[4], vb[2];
  float vv[2];
  int q;
};

// VEC: the B_0^T v row is wanted (a.avec set).  A template parameter, not a runtime test: its loads and
// accumulators (10 VGPRs) pushed the common launches to the 256-VGPR limit, where the compiler's
// temporaries land on in-flight load destinations (each such hazard is a vmcnt wait on the prefetch)
// SAME: both pairs have one geometry (leading dims, blocked bits; every call of the training step), so
// one set of lane offsets serves both and a k-step's loads need no per-lane select (whose VGPR
// temporaries at the loop head aliased registers the prologue's loads were still filling: a vmcnt(0)
// drain once per unrolled iteration)
template <bool VA, bool VB, bool F32 = false, bool VEC = false, bool SAME = false>
__global__ __launch_bounds__(kWgThreads) void wgrad_kernel(WgKArgs a) {
  __shared__ __attribute__((aligned(16))) _Float16 lds[2 * kStage];
  // per stage: the rescale ratios 2^(e_new - e_old) of the 64 A column quads, then the 32 B quads, and
  // one byte per wave: "a B quad this wave loads lowered its exponent"; [2]: the final 2^-e
  __shared__ float s_rat[3][64 + 32];
  __shared__ __attribute__((aligned(8))) unsigned char s_chg[2][8];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int NT = a.nmt * a.nnt;
  // block -> (slice, m tile, n tile): with S % 8 == 0 the tiles of one slice share an XCD
  int slice, t;
  if (a.S % 8 == 0) {
    const int xcd = blockIdx.x & 7, seq = blockIdx.x >> 3;
    slice = (seq / NT) * 8 + xcd;
    t = seq % NT;
  } else {
    slice = blockIdx.x / NT;
    t = blockIdx.x % NT;
  }
  if (slice >= a.S) return;
  const int mt = t / a.nnt, nt = t % a.nnt;
  const int m0 = mt * kWgM, n0 = nt * kWgN;
  const int mloc = min(kWgM, a.m - m0);
  const bool wvalid = 32 * w < mloc;                   // wave-uniform: this wave has output rows
  // k-step indices are 32-bit (the host caps P): a 64-bit compare has no scalar form on gfx9, so the
  // compiler copies an operand into a VGPR -- at this kernel's register budget one an in-flight prefetch
  // load writes, and the hazard wait (vmcnt(2) at the loop head) drained the 3-deep prefetch every k-step
  const int KP = (int)a.KP, KS = a.npairs * KP;
  const int k0 = (int)((int64_t)KS * slice / a.S), k1 = (int)((int64_t)KS * (slice + 1) / a.S);

  f32x4 acc[2][8];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float4 cs = make_float4(0.f, 0.f, 0.f, 0.f), vs = make_float4(0.f, 0.f, 0.f, 0.f);
  const bool want_cs = a.part_cs && nt == 0, want_vec = VEC && mt == 0;

  // loader geometry: A lane -> column quad (lane & 7) of the wave's 32 columns, rows (lane >> 3) + 8 j;
  // B lane -> column quad (lane & 3) of the wave's 16 columns, rows (lane >> 2) + 16 j
  const int ac = 32 * w + 4 * (lane & 7), ar = lane >> 3;
  const int bc = 16 * w + 4 * (lane & 3), br = lane >> 2;
  // loop-invariant lane offsets within a k-step's rows, per pair (the pairs may differ in leading dims)
  constexpr int NQ = SAME ? 1 : 2;
  uint32_t oa[NQ][4], ob[NQ][2], ov[2];
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int qq = q < a.npairs ? q : 0;
    const bool blka = (a.blocked & (NR_WG_BLK_A0 << qq)) != 0, blkb = (a.blocked & (NR_WG_BLK_B0 << qq)) != 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) oa[q][j] = lane_off(ar + 8 * j, m0 + ac, a.lda[qq], a.m, wvalid, blka);
#pragma unroll
    for (int j = 0; j < 2; ++j) ob[q][j] = lane_off(br + 16 * j, n0 + bc, a.ldb[qq], a.n, true, blkb);
  }
#pragma unroll
  for (int j = 0; j < 2; ++j) ov[j] = VEC && want_vec ? (uint32_t)((br + 16 * j) * a.ldv) * 4u : kOob;
  // live = false (past the slice's last k-step): zero-sized resources, the loads return zeros and touch
  // no memory.  Issued unconditionally, so the compiler counts the loads in flight exactly (a
  // conditional prefetch makes it wait for all of them)
  auto load = [&](int ks, WgRegs& R, bool live) __attribute__((always_inline)) {
#ifdef NR_WG_EXP_NO_LOAD
    const float x = (float)(ks & 7) + 0.5f;
    for (int j = 0; j < 4; ++j) R.va[j] = make_float4(x, x, x, x);
    for (int j = 0; j < 2; ++j) { R.vb[j] = make_float4(x, x, x, x); R.vv[j] = x; }
    R.q = 0;
    return;
#endif
    ks = live ? ks : 0;
    const int q = ks >= KP;
    const int64_t r0 = (int64_t)(ks - (q ? KP : 0)) * kWgK;
    const int64_t lda = q ? a.lda[1] : a.lda[0], ldb = q ? a.ldb[1] : a.ldb[0];
    const int64_t rows = live ? a.P - r0 : 0;
    const __amdgpu_buffer_rsrc_t ra = rsrc((q ? a.a[1] : a.a[0]) + r0 * lda, rows * lda * 4);
    const __amdgpu_buffer_rsrc_t rb = rsrc((q ? a.b[1] : a.b[0]) + r0 * ldb, rows * ldb * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) R.va[j] = ld4<VA>(ra, SAME ? oa[0][j] : q ? oa[NQ - 1][j] : oa[0][j], m0 + ac, a.m);
#pragma unroll
    for (int j = 0; j < 2; ++j) R.vb[j] = ld4<VB>(rb, SAME ? ob[0][j] : q ? ob[NQ - 1][j] : ob[0][j], n0 + bc, a.n);
    if constexpr (VEC) {
      const __amdgpu_buffer_rsrc_t rv = rsrc(a.avec + r0 * a.ldv, q == 0 ? rows * a.ldv * 4 : 0);
#pragma unroll
      for (int j = 0; j < 2; ++j) R.vv[j] = __int_as_float(__builtin_amdgcn_raw_buffer_load_b32(rv, ov[j], 0, 0));
    }
    R.q = q;
  };
  [[maybe_unused]] float sink = 0.0f;  // timing experiments only (NR_WG_EXP_NO_STORE keeps the loads alive)
  // Running per-quad exponents: a quad keeps one scale over the slice (e only decreases), so MFMAs
  // accumulate straight into acc.  A k-step whose quad max M would reach 2^14 at the current scale
  // lowers it to put M at 2^(14 - kHeadroom) (16x headroom: later maxima rarely force another change),
  // and the accumulated tiles of that quad are multiplied by 2^(e_new - e_old); the final 2^-(eA + eB)
  // is applied once.  A value below the running scale keeps its absolute precision: |error| < 2^-35 of
  // the quad's running max (the f16 subnormal quantum at a 2^10 scale).
  int ea_cur = kExpCap, eb_cur = kExpCap;
  bool cha[2] = {false, false};
  auto store = [&](int stg, const WgRegs& R) __attribute__((always_inline)) {
#ifdef NR_WG_EXP_NO_STORE
    sink += R.va[0].x + R.va[1].y + R.va[2].z + R.va[3].w + R.vb[0].x + R.vb[1].w + R.vv[0] + R.vv[1];
    return;
#endif
    _Float16* S0 = lds + stg * kStage;
    if (want_cs && R.q == 0) cs = add4(cs, add4(add4(R.va[0], R.va[1]), add4(R.va[2], R.va[3])));
    if constexpr (VEC)
      if (want_vec && R.q == 0) vs = fma4(R.vv[1], R.vb[1], fma4(R.vv[0], R.vb[0], vs));
    if constexpr (F32) {  // fp32 row images: A [32][kAStride floats], B [32][kBStride floats] (no split)
      float* A32 = (float*)S0;
      float* B32 = (float*)(S0 + 2 * kAPlane);
#pragma unroll
      for (int j = 0; j < 4; ++j) *(float4*)(A32 + (ar + 8 * j) * kAStride + ac) = R.va[j];
#pragma unroll
      for (int j = 0; j < 2; ++j) *(float4*)(B32 + (br + 16 * j) * kBStride + bc) = R.vb[j];
      return;
    }
    // per column quad: the max over its 32 rows (this lane's 4 rows x 8 lanes) -> power-of-two scale
    const float ma = quad_max<false>(fmaxf(fmaxf(amax4(R.va[0]), amax4(R.va[1])), fmaxf(amax4(R.va[2]), amax4(R.va[3]))));
    const int ta = split_exp(ma);
    const int ea = ta < ea_cur ? ta - kHeadroom : ea_cur;
    const float sa = __builtin_ldexpf(1.0f, ea);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint2 h, l;
      split4(R.va[j], sa, h, l);
      const int o = (ar + 8 * j) * kAStride + ac;
      *(uint2*)(S0 + o) = h;
      *(uint2*)(S0 + kAPlane + o) = l;
    }
    if (lane < 8) s_rat[stg][ac >> 2] = __builtin_ldexpf(1.0f, ea - ea_cur);
    cha[stg] = __builtin_amdgcn_ballot_w64(ea != ea_cur) != 0;  // this wave's A quads = its output rows
    ea_cur = ea;
    const float mb = quad_max<true>(fmaxf(amax4(R.vb[0]), amax4(R.vb[1])));
    const int tb = split_exp(mb);
    const int eb = tb < eb_cur ? tb - kHeadroom : eb_cur;
    const float sb = __builtin_ldexpf(1.0f, eb);
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      uint2 h, l;
      split4(R.vb[j], sb, h, l);
      const int o = (br + 16 * j) * kBStride + bc;
      *(uint2*)(S0 + 2 * kAPlane + o) = h;
      *(uint2*)(S0 + 2 * kAPlane + kBPlane + o) = l;
    }
    if (lane < 4) s_rat[stg][64 + (bc >> 2)] = __builtin_ldexpf(1.0f, eb - eb_cur);
    const bool chb = __builtin_amdgcn_ballot_w64(eb != eb_cur) != 0;
    if (lane == 0) s_chg[stg][w] = chb ? 1 : 0;
    eb_cur = eb;
  };
  const int G = lane >> 4, col = lane & 15;
  // multiply each output tile by its A quad's and its B quad's factor in table s_rat[tab]
  auto rescale = [&](int tab) __attribute__((always_inline)) {
    const float fa0 = s_rat[tab][8 * w + G], fa1 = s_rat[tab][8 * w + 4 + G];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float fb = s_rat[tab][64 + 4 * j + (col >> 2)];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        acc[0][j][r] = acc[0][j][r] * fa0 * fb;
        acc[1][j][r] = acc[1][j][r] * fa1 * fb;
      }
    }
  };
  auto compute = [&](int stg) __attribute__((always_inline)) {
    if (!wvalid) return;
#ifdef NR_WG_EXP_NO_MFMA
    return;
#endif
    if constexpr (F32) {
      const float* A32 = (const float*)(lds + stg * kStage);
      const float* B32 = (const float*)(lds + stg * kStage + 2 * kAPlane);
#pragma unroll
      for (int s = 0; s < kWgK / 4; ++s) {
        const int r = 4 * s + G;
        float av[2], bv[8];
#pragma unroll
        for (int i = 0; i < 2; ++i) av[i] = A32[r * kAStride + 32 * w + 16 * i + col];
#pragma unroll
        for (int j = 0; j < 8; ++j) bv[j] = B32[r * kBStride + 16 * j + col];
#pragma unroll
        for (int j = 0; j < 8; ++j)
#pragma unroll
          for (int i = 0; i < 2; ++i) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[i], bv[j], acc[i][j], 0, 0, 0);
      }
      return;
    }
    uint64_t chb;
    __builtin_memcpy(&chb, s_chg[stg], 8);
    if (cha[stg] || chb != 0) rescale(stg);  // wave-uniform
    const _Float16* S0 = lds + stg * kStage;
    f16x8 ah[2], al[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      ah[i] = frag(S0, kAStride, 32 * w + 16 * i, lane);
      al[i] = frag(S0 + kAPlane, kAStride, 32 * w + 16 * i, lane);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const f16x8 bh = frag(S0 + 2 * kAPlane, kBStride, 16 * j, lane);
      const f16x8 bl = frag(S0 + 2 * kAPlane + kBPlane, kBStride, 16 * j, lane);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(al[i], bh, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bl, acc[i][j], 0, 0, 0);
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ah[i], bh, acc[i][j], 0, 0, 0);
      }
    }
  };

  // three k-steps of loads in flight: while k-step ks runs its MFMAs from LDS stage ks & 1, register set
  // (ks + 1) % 3 holds k-step ks + 1 (split into the other stage after the MFMAs) and the two other sets
  // k-steps ks + 2 and ks + 3 (the set k-step ks came from is refilled first).  Unrolled by 6 = lcm(2, 3).
  // Loads past the slice's end are dead (zeros, no memory); stores past it fill a stage nobody reads.
  WgRegs R0, R1, R2;
  load(k0, R0, k0 < k1);
  load(k0 + 1, R1, k0 + 1 < k1);
  load(k0 + 2, R2, k0 + 2 < k1);
  store(0, R0);
  __syncthreads();
  int ks = k0;
  // Within a barrier interval the MFMAs read stage stg and the split writes stage stg ^ 1, so their
  // order is free (the kPingPongBit experiment: the two waves of a SIMD in different phases).
  const bool split_first = (w & kPingPongBit) != 0;
  auto step = [&](int stg, WgRegs& refill, WgRegs& next) __attribute__((always_inline)) {
    load(ks + 3, refill, ks + 3 < k1);
    if (split_first) {
      store(stg ^ 1, next);
      compute(stg);
    } else {
      compute(stg);
      store(stg ^ 1, next);
    }
    __syncthreads();
    return ++ks < k1;
  };
  while (ks < k1) {
    if (!step(0, R0, R1)) break;
    if (!step(1, R1, R2)) break;
    if (!step(0, R2, R0)) break;
    if (!step(1, R0, R1)) break;
    if (!step(0, R1, R2)) break;
    if (!step(1, R2, R0)) break;
  }
  // the final exponents -> 2^-e per quad, applied once (two factors: 2^-(eA + eB) can underflow)
  if constexpr (!F32) {
    if (lane < 8) s_rat[2][ac >> 2] = __builtin_ldexpf(1.0f, -ea_cur);
    if (lane < 4) s_rat[2][64 + (bc >> 2)] = __builtin_ldexpf(1.0f, -eb_cur);
    __syncthreads();
#ifndef NR_WG_EXP_NO_MFMA
    if (wvalid) rescale(2);
#endif
  }

  // partial tile: lane (G, col) register r holds row 4G + r of each 16 x 16 tile -> part[s][n][m]
  const int64_t ldp = (int64_t)a.nmt * kWgM;
  float* P0 = a.part + (int64_t)slice * (a.nnt * kWgN) * ldp;
  {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int64_t nn = n0 + 16 * j + col, mm = m0 + 32 * w + 16 * i + 4 * G;
#ifdef NR_WG_EXP_NO_STORE
        acc[i][j][0] += sink;
#endif
        *(float4*)(P0 + nn * ldp + mm) = wvalid ? make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3])
                                                : make_float4(0.f, 0.f, 0.f, 0.f);
      }
  }
  if (want_cs) {  // lanes with equal (lane & 7) hold the same columns: fixed-order butterfly
    cs = add4(cs, shfl_xor4(cs, 8));
    cs = add4(cs, shfl_xor4(cs, 16));
    cs = add4(cs, shfl_xor4(cs, 32));
    if (lane < 8) *(float4*)(a.part_cs + (int64_t)slice * ldp + m0 + ac) = cs;
  }
  if (VEC && want_vec) {
    vs = add4(vs, shfl_xor4(vs, 4));
    vs = add4(vs, shfl_xor4(vs, 8));
    vs = add4(vs, shfl_xor4(vs, 16));
    vs = add4(vs, shfl_xor4(vs, 32));
    if (lane < 4) *(float4*)(a.part_vec + (int64_t)slice * (a.nnt * kWgN) + n0 + bc) = vs;
  }
}

// C[i, j] = scale * sum_s part[s][j][i] (i < m, j < n), deterministic: a block takes 32 float4 groups of
// (j, 4 consecutive i); its 8 thread groups sum the slices s = g, g + 8, g + 16, ... in order, then the
// 8 group sums are added in group order.  The last blocks do the same for the column sums of A_0 and
// the vector row (one float per thread instead of a float4).
constexpr int kRedGroups = 8;
struct WgRedArgs {
  const float* part;
  int S, m, n;
  int64_t ldp, ldn;
  float scale;
  float* c;
  int64_t ldc;
  int nb_c, nb_cs;          // blocks for C, then for the column sums; the rest for the vector row
  const float* part_cs;
  float* cs;
  const float* part_vec;
  float* vec;
  float vscale;
};

__global__ __launch_bounds__(256) void wgrad_reduce(WgRedArgs r) {
  __shared__ float4 acc[kRedGroups][32];
  const int t = threadIdx.x & 31, g = threadIdx.x >> 5;
  const int b = blockIdx.x;
  if (b < r.nb_c) {
    const int64_t q = (int64_t)b * 32 + t;  // float4 group: j = q / (ldp / 4), i = 4 (q % (ldp / 4))
    const int64_t qpr = r.ldp / 4, nq = (int64_t)r.n * qpr;
    float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
    if (q < nq) {
      const float4* p = (const float4*)r.part + q;
      const int64_t stride = r.ldn * qpr;  // one slice, in float4
#pragma unroll 4
      for (int k = g; k < r.S; k += kRedGroups) s = add4(s, p[(int64_t)k * stride]);
    }
    acc[g][t] = s;
    __syncthreads();
    if (g == 0 && q < nq) {
      float4 v = acc[0][t];
#pragma unroll
      for (int k = 1; k < kRedGroups; ++k) v = add4(v, acc[k][t]);
      const int64_t j = q / qpr, i = 4 * (q % qpr);
      const float e4[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int e = 0; e < 4; ++e)
        if (i + e < r.m) r.c[(i + e) * r.ldc + j] = e4[e] * r.scale;
    }
    return;
  }
  // a column sum (index < m, slices ldp apart) or a vector-row entry (index < n, slices ldn apart)
  const bool is_cs = b < r.nb_c + r.nb_cs;
  const int64_t idx = (int64_t)(b - (is_cs ? r.nb_c : r.nb_c + r.nb_cs)) * 32 + t;
  const int len = is_cs ? r.m : r.n;
  const int64_t ld = is_cs ? r.ldp : r.ldn;
  const float* p = is_cs ? r.part_cs : r.part_vec;
  float s = 0.0f;
  if (idx < len) {
#pragma unroll 4
    for (int k = g; k < r.S; k += kRedGroups) s += p[(int64_t)k * ld + idx];
  }
  acc[g][t].x = s;
  __syncthreads();
  if (g == 0 && idx < len) {
    float v = acc[0][t].x;
#pragma unroll
    for (int k = 1; k < kRedGroups; ++k) v += acc[k][t].x;
    if (is_cs) r.cs[idx] = v;
    else r.vec[idx] = v * r.vscale;
  }
}

template <bool VA, bool VB, bool F32>
static void wg_launch(bool vec, bool same, dim3 grid, hipStream_t st, const WgKArgs& k) {
  if (vec && same) hipLaunchKernelGGL((wgrad_kernel<VA, VB, F32, true, true>), grid, dim3(kWgThreads), 0, st, k);
  else if (vec) hipLaunchKernelGGL((wgrad_kernel<VA, VB, F32, true, false>), grid, dim3(kWgThreads), 0, st, k);
  else if (same) hipLaunchKernelGGL((wgrad_kernel<VA, VB, F32, false, true>), grid, dim3(kWgThreads), 0, st, k);
  else hipLaunchKernelGGL((wgrad_kernel<VA, VB, F32, false, false>), grid, dim3(kWgThreads), 0, st, k);
}

struct WgPlan {
  int nmt, nnt, S;
  int64_t KP;
  size_t part_bytes, cs_bytes, vec_bytes;
};

static WgPlan wgrad_plan(int64_t P, int m, int n, int npairs) {
  WgPlan p{};
  p.nmt = (m + kWgM - 1) / kWgM;
  p.nnt = (n + kWgN - 1) / kWgN;
  p.KP = (P + kWgK - 1) / kWgK;
  const int64_t KS = std::max<int64_t>(1, npairs * p.KP);
  // about one workgroup per CU (256), in whole groups of 8 slices (the XCD mapping), >= 1 k-step each
  int S = (int)std::max<int64_t>(1, 256 / (p.nmt * p.nnt));
  S = S >= 8 ? S / 8 * 8 : S;
  if (S > KS) S = (int)KS;
  p.S = std::max(S, 1);
  p.part_bytes = (size_t)p.S * p.nnt * kWgN * p.nmt * kWgM * 4;
  p.cs_bytes = (size_t)p.S * p.nmt * kWgM * 4;
  p.vec_bytes = (size_t)p.S * p.nnt * kWgN * 4;
  return p;
}

}  // namespace nr

using namespace nr;

extern "C" {

size_t nr_wgrad_workspace_bytes(int64_t P, int m, int n, int npairs) {
  const WgPlan p = wgrad_plan(P, m, n, npairs);
  return p.part_bytes + p.cs_bytes + p.vec_bytes + 768;
}

int nr_wgrad(const NrWgrad* w, void* stream) {
  NR_REQUIRE(w, NR_ERR_ARG, "nr_wgrad: null args");
  NR_REQUIRE(w->npairs == 1 || w->npairs == 2, NR_ERR_ARG, "nr_wgrad: npairs must be 1 or 2");
  NR_REQUIRE(w->m > 0 && w->n > 0 && w->P >= 0, NR_ERR_ARG, "nr_wgrad: bad shape");
  NR_REQUIRE(w->c && w->ldc >= w->n, NR_ERR_ARG, "nr_wgrad: null output or ldc < n");
  for (int q = 0; q < w->npairs; ++q)
    NR_REQUIRE(w->a[q] && w->b[q] && w->lda[q] >= w->m && w->ldb[q] >= w->n, NR_ERR_ARG,
               "nr_wgrad: null operand or leading dimension below its column count");
  NR_REQUIRE(!w->vec || w->avec, NR_ERR_ARG, "nr_wgrad: vec output without avec");
  {  // operands are read through buffer resources with 32-bit byte offsets
    const int64_t lim = (int64_t)1 << 31;
    bool fits = !w->avec || w->P * std::max<int64_t>(w->ldv, 1) * 4 < lim;
    for (int q = 0; q < w->npairs; ++q) fits = fits && w->P * w->lda[q] * 4 < lim && w->P * w->ldb[q] * 4 < lim;
    NR_REQUIRE(fits, NR_ERR_ARG, "nr_wgrad: an operand spans 2 GiB or more (split the rows over calls)");
  }
  if (w->blocked) {  // 16 x 16 blocked operands: whole blocks of rows and columns
    bool ok = w->P % 16 == 0 && (w->blocked & ~0xf) == 0;
    for (int q = 0; q < w->npairs; ++q) {
      if (w->blocked & (NR_WG_BLK_A0 << q)) ok = ok && w->lda[q] % 16 == 0;
      if (w->blocked & (NR_WG_BLK_B0 << q)) ok = ok && w->ldb[q] % 16 == 0;
    }
    NR_REQUIRE(ok, NR_ERR_ARG, "nr_wgrad: a blocked operand needs P and its leading dimension multiples of 16");
  }
  WgPlan p = wgrad_plan(w->P, w->m, w->n, w->npairs);
#ifdef NR_WG_EXP_SLICES_ENV  // measurement builds only (tools/wgrad_bench.py): fewer slices
  if (const char* e = getenv("NR_WGRAD_SLICES")) {
    const int s = atoi(e);
    if (s > 0 && s < p.S) p.S = s;
  }
#endif
  NR_REQUIRE(w->workspace && w->workspace_bytes >= p.part_bytes + p.cs_bytes + p.vec_bytes, NR_ERR_WORKSPACE,
             "nr_wgrad: workspace too small (nr_wgrad_workspace_bytes)");
  hipStream_t st = (hipStream_t)stream;
  char* ws = (char*)w->workspace;
  WgKArgs k{};
  bool va = true, vb = true;
  for (int q = 0; q < w->npairs; ++q) {
    k.a[q] = w->a[q]; k.lda[q] = w->lda[q];
    k.b[q] = w->b[q]; k.ldb[q] = w->ldb[q];
    va = va && w->m % 4 == 0 && w->lda[q] % 4 == 0 && ((uintptr_t)w->a[q] & 15) == 0;
    vb = vb && w->n % 4 == 0 && w->ldb[q] % 4 == 0 && ((uintptr_t)w->b[q] & 15) == 0;
  }
  k.npairs = w->npairs; k.P = w->P; k.m = w->m; k.n = w->n;
  k.nmt = p.nmt; k.nnt = p.nnt; k.S = p.S; k.KP = p.KP;
  k.part = (float*)ws;
  k.part_cs = w->colsum ? (float*)(ws + p.part_bytes) : nullptr;
  k.avec = w->vec ? w->avec : nullptr;
  k.ldv = w->ldv > 0 ? w->ldv : 1;
  k.part_vec = w->vec ? (float*)(ws + p.part_bytes + p.cs_bytes) : nullptr;
  k.blocked = w->blocked;
  {
    // units: the operands' bytes (the HBM-bound roofline's algorithmic traffic)
    ProfScope prof("wgrad", (double)w->npairs * w->P * (w->m + w->n) * 4.0, st);
    const dim3 grid((unsigned)(p.S * p.nmt * p.nnt));
    // S % 8 == 0 needs the grid padded to whole XCD rounds of the mapping (it already is: S * NT)
    const bool vec = k.avec != nullptr;
    // one lane-offset geometry for both pairs (a single pair trivially)
    const int bits0 = w->blocked & (NR_WG_BLK_A0 | NR_WG_BLK_B0), bits1 = (w->blocked >> 1) & (NR_WG_BLK_A0 | NR_WG_BLK_B0);
    const bool same = w->npairs == 1 || (w->lda[0] == w->lda[1] && w->ldb[0] == w->ldb[1] && bits0 == bits1);
    if (w->fp32) {
      if (va && vb) wg_launch<true, true, true>(vec, same, grid, st, k);
      else if (va) wg_launch<true, false, true>(vec, same, grid, st, k);
      else if (vb) wg_launch<false, true, true>(vec, same, grid, st, k);
      else wg_launch<false, false, true>(vec, same, grid, st, k);
    } else {
      if (va && vb) wg_launch<true, true, false>(vec, same, grid, st, k);
      else if (va) wg_launch<true, false, false>(vec, same, grid, st, k);
      else if (vb) wg_launch<false, true, false>(vec, same, grid, st, k);
      else wg_launch<false, false, false>(vec, same, grid, st, k);
    }
    NR_HIP_CHECK(hipGetLastError());
  }
  const int64_t ldp = (int64_t)p.nmt * kWgM, ldn = (int64_t)p.nnt * kWgN;
  WgRedArgs r{};
  r.part = k.part; r.S = p.S; r.m = w->m; r.n = w->n; r.ldp = ldp; r.ldn = ldn;
  r.scale = w->scale; r.c = w->c; r.ldc = w->ldc;
  r.nb_c = (int)((w->n * (ldp / 4) + 31) / 32);
  r.nb_cs = w->colsum ? (w->m + 31) / 32 : 0;
  const int nb_vec = w->vec ? (w->n + 31) / 32 : 0;
  r.part_cs = k.part_cs; r.cs = w->colsum; r.part_vec = k.part_vec; r.vec = w->vec; r.vscale = w->vec_scale;
  hipLaunchKernelGGL(wgrad_reduce, dim3((unsigned)(r.nb_c + r.nb_cs + nb_vec)), dim3(256), 0, st, r);
  NR_HIP_CHECK(hipGetLastError());
  return NR_OK;
}

}  // extern "C"
