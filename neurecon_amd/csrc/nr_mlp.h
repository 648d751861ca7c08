// neurecon_amd — MLP kernel constants, packed-weight layouts and launchers (internal header).
#pragma once
#include "nr_common.h"

namespace nr {

constexpr int kWaves = 8;                       // waves per workgroup (2 per SIMD)
constexpr int kThreads = 64 * kWaves;           // 512
constexpr int kTile = 16;                       // points per wave (MFMA N dimension)
constexpr int kPointsPerWG = kTile * kWaves;    // 128
constexpr int kMaxChunkBytes = 48 * 1024;       // LDS chunk: 2 output blocks x <=24 input blocks x 1 KB
constexpr size_t kScratchPerWG = (size_t)kWaves * 8 * 16 * 64 * 16;  // exp(100z) slabs, 1 MiB
// sdf4_kernel reverse-pass slabs of one 16-point column: layers 0..6 hold 24-bit codes of
// 2^-L = 1 - softplus'(z) (per chunk [block 2][column][lane] x 12 B: 8 chunks x 1536 B = 12 KB per
// layer), layer 7 holds d sdf / d z7 (and, during the forward, the parked embedding) in fp32
// ([block 16][column][lane] x 16 B); 100 KB instead of 8 x 16 KB of fp32 slabs
// NR_SLAB32: each code as the fp32 F = 2^23 + round(c 2^23) (bits 0x4B000000 | code), 16 B per 4 codes:
// the forward forms it with one fma and the reverse pass softplus' = 2 - F 2^-23 with one more, instead
// of packing / unpacking 24-bit fields (128 KB per column)
#ifdef NR_SLAB32
constexpr int kSlabVB = 16;                             // slab bytes per lane and 4 codes
#else
constexpr int kSlabVB = 12;
#endif
constexpr int kSlab24Chunk = 2 * 64 * kSlabVB;          // one chunk of one column: 1536 B (2 KB with NR_SLAB32)
constexpr int kSlab24Layer = 8 * kSlab24Chunk;          // 12 KB (16 KB)
constexpr int kSlabColBytes = 7 * kSlab24Layer + 16 * 64 * 16;  // 100 KB (128 KB) per column (deferred tile)

// SDF GEMM ops in stream order (forward F*, feature F8, backward B*)
enum SdfOp { F0, F1, F2, F3, F4, F5, F6, F7, F8, B7, B6, B5, B4, B3, B2, B1, B0, kSdfOps };

// (input blocks, output blocks) of each SDF GEMM op, stream order F0..F8, B7..B0; ops are packed
// back to back in this order, chunk = 2 output blocks x KB input blocks + a 1 KB bias slot
constexpr int kSdfKB[kSdfOps] = {4, 16, 16, 16, 18, 16, 16, 16, 16, 16, 16, 16, 16, 14, 16, 16, 16};
constexpr int kSdfNBO[kSdfOps] = {16, 16, 16, 14, 16, 16, 16, 16, 16, 16, 16, 16, 18, 16, 16, 16, 4};
__host__ __device__ constexpr uint32_t sdf_op_off(int i) {
  uint32_t off = 0;
  for (int k = 0; k < i; ++k) off += (uint32_t)(kSdfNBO[k] / 2) * (2 * kSdfKB[k] + 1) * 1024;
  return off;
}

// SIREN SDF net (base.py:84-115, D=5, no skip, identity embedding): forward S0..S4, feature SF,
// backward SB4..SB0; S0 reads the 3 coordinates from a 4-block (64-feature, zero-padded) input and
// SB0 writes their gradient into 4 blocks, as the softplus net's F0 / B0 do
enum SirenOp { S0, S1, S2, S3, S4, SF, SB4, SB3, SB2, SB1, SB0, kSirenOps };
constexpr int kSirenKB[kSirenOps] = {4, 16, 16, 16, 16, 16, 16, 16, 16, 16, 16};
constexpr int kSirenNBO[kSirenOps] = {16, 16, 16, 16, 16, 16, 16, 16, 16, 16, 4};
static_assert(kSirenOps <= kSdfOps, "SIREN ops share SdfLayout's offset table");

struct SdfLayout {
  uint32_t op_off[kSdfOps];
  uint32_t op_bytes[kSdfOps];  // bytes of one chunk of the op
  uint32_t scale_off;          // [kSdfOps] max |W| per op (f16x3 weight scaling)
  uint32_t bound_off;          // [kSdfOps][2] max row L1 norm, max |bias| per op (f16x3 operand scales)
  uint32_t w8row0_off;         // sdf row of the last layer [256]
  uint32_t misc_off;           // [0] = sdf bias
  uint32_t l32_off;            // f16x3 softplus nets: the ops again in the 32x32x16 layout (nr_sdf5.hip),
                               // at l32_off + op_off[i]; 0: none
  uint32_t total;
  int prec;
  int siren;                   // op_off / op_bytes indexed by SirenOp
};

struct RadLayout {
  uint32_t op_off[5];
  uint32_t op_bytes[5];
  uint32_t head_off;  // [3][256] weights, then [3] bias
  uint32_t scale_off; // [4] max |W| per op
  uint32_t bound_off; // [5][2] max row L1 norm, max |bias| per op (rad4_kernel's operand scales)
  uint32_t total;
  int prec;
  int kbs;            // small-input blocks (even)
  int n_small;        // 3 + view-embedding + 3, or 3 without view dirs
  int view;           // use_view_dirs: view embedding and normals in the input
  int D;              // hidden layers (4 or 5)
  int siren;          // sine hidden layers
};

// NeRF++ background MLP (models/base.py:395-453): 8 x (Linear+ReLU) with the input re-injected
// after layer 4, sigma head, feature Linear, view branch Linear(256+27 -> 128)+ReLU, rgb head.
// f16x3 (nerf4_kernel): NF carries alpha_linear as output blocks 16-17 (row 0 = sigma), 9 chunks.
enum NerfOp { N0, N1, N2, N3, N4, N5, N6, N7, NF, NV, kNerfOps };

struct NerfLayout {
  uint32_t op_off[kNerfOps];
  uint32_t op_bytes[kNerfOps];
  uint32_t scale_off;  // [kNerfOps] max |W| per op
  uint32_t bound_off;  // [kNerfOps][2] max row L1 norm, max |bias| per op (nerf4_kernel's operand scales)
  uint32_t alpha_off;  // [256] weights, [256] = bias
  uint32_t rgb_off;    // [3][128] weights, then [3] bias
  uint32_t total;
  int prec;
};

// NeRF++ training pack (nr_nerf_train_pack, fp32 or f16x3): the transposed ops of the backward data gradients,
// chained by nerf_train32_bwd_kernel: views (Wv[:, :256]^T: 128 -> 256), feature (Wf^T), then W7^T ..
// W1^T (W5^T restricted to its h columns 84..339); Wr [3][128] and Wa [256] for the VALU heads
enum NerfBwdOp { NBV, NBF, NB7, NB6, NB5, NB4, NB3, NB2, NB1, kNerfBwdOps };

struct NerfBwdLayout {
  uint32_t op_off[kNerfBwdOps];
  uint32_t op_bytes[kNerfBwdOps];
  uint32_t scale_off;  // [kNerfBwdOps] max |W| per op (written by the pack scan)
  uint32_t wr_off;     // [3][128] rgb_linear weights
  uint32_t wa_off;     // [256] alpha_linear weights
  uint32_t total;
};

struct PackSeg {
  int nblk;    // 16-feature blocks
  int off;     // first source index
  int nvalid;  // valid source indices (rest zero-padded)
};

struct PackOp {
  const float* W;
  const float* bias;  // per output row (same row mapping as W), or null
  int64_t wn;         // elements of W (for the max-|W| scan)
  int ld;
  int transpose;  // 1: value = W[in][out] (Wᵀ)
  PackSeg out[2];
  PackSeg in[2];
  float scale;
  int prec;            // NR_PREC_*
  float* wmax;         // device word receiving max |W * scale| (f16x3 scaling)
  const float* aux;    // optional per-output-row vector written to bias-slot floats 64..95 of each chunk
  float* bound;        // optional [2]: max over output rows of sum |W * scale|, max |bias|
  const float* W2;     // optional second matrix [rows][ld2] (not transposed) for the rows of out[1]
  const float* bias2;  //   ... and its bias
  int64_t wn2;
  int ld2;
  int l32;             // f16x3: the 32x32x16 A layout of nr_sdf5.hip instead of the 16x16x32 one
};

int launch_pack_op(const PackOp& op, char* dst, hipStream_t stream);
// the ops of one pack call, batched (three launches per 20 ops)
int launch_pack_ops(const PackOp* ops, char* const* dst, int nops, hipStream_t stream);
int launch_pack_vec(const float* src, int off, int nvalid, int n, char* dst, hipStream_t stream);
int launch_sdf(const SdfLayout& L, const void* packed, const float* pts, int64_t P, float* sdf, float* nabla,
               float* feature, int nfreq, void* ws, size_t ws_bytes, hipStream_t stream,
               const int* P_dev = nullptr, int P_mult = 0);  // P_dev: device count, P_eff = min(P, *P_dev * P_mult)
// SDF forward (sdf only) on the 32x32x16 kernel (nr_sdf5.hip): needs L.l32_off
int launch_sdf5_fwd(const SdfLayout& L, const void* packed, const float* pts, int64_t P, float* sdf, int nfreq,
                    hipStream_t stream, const int* P_dev, int P_mult);
extern int g_sdf5;             // route launch_sdf's forward-only f16x3 launches to it (nr_sdf5_enable)
extern const int g_sdf5_pack;  // $NR_SDF5 (a nonzero integer) at load: the layout carries the 32x32x16 copy
// deferred sample nablas (sdf4_kernel STAGE 1 / 2): stage 1 = sdf + slabs per 16-point tile into
// `slabs` (P/16 x kSlabColBytes); stage 2 = nablas of the tiles tiles[0 .. *n_tiles) from their slabs;
// stage 4 = nablas of the points tiles[0 .. *n_tiles) (neus_point_list's layout: 16-aligned segments of
// slots within one 1024-slot range, padded with -1)
int launch_sdf_deferred(const SdfLayout& L, const void* packed, const float* pts, int64_t P, float* sdf, float* nabla,
                        int nfreq, float4* slabs, const int* tiles, const int* n_tiles, int stage, hipStream_t stream);
int launch_nerf(const NerfLayout& L, const void* packed, const float* x4, const float* vdir, int64_t vdiv,
                int64_t vmod, int64_t P, float* sigma, float* rgb, hipStream_t stream,
                const int* P_dev = nullptr);  // P_dev: device count, P_eff = min(P, *P_dev)
int launch_radiance(const RadLayout& L, const void* packed, const float* x, const float* vdir, int64_t vdiv,
                    int64_t vmod, const float* normals, const float* feature, int64_t P, float* rgb, int nfreq_view,
                    hipStream_t stream, const int* P_dev = nullptr);  // P_dev: device count, P_eff = min(P, *P_dev)

// training forward of a ReLU D=4 radiance net on its fp32 pack: h[0..3] [P][256], rgb [P][3]
int launch_radiance_train32(const RadLayout& L, const void* packed, const float* feat, const float* small,
                            int64_t ld_small, int n_small, int64_t P, float* const* h, float* rgb, hipStream_t stream);
// NeRF++ training forward on the fp32 render pack (xe [P][84], ve [P][27] -> h[0..7] [P][256], feat
// [P][256], hv [P][128], sigma [P], rgb [P][3]) and the data gradients on the training pack
int launch_nerf_train32_fwd(const NerfLayout& L, const void* packed, const float* xe, const float* ve, int64_t P,
                            float* const* h, float* feat, float* hv, float* sigma, float* rgb, hipStream_t stream);
int launch_nerf_train32_bwd(const NerfBwdLayout& B, const void* packed, const float* rgb, const float* hv,
                            const float* const* h, const float* g_rgb, const float* g_sigma, int64_t P, float* g3,
                            float* ghv, float* g_feat, float* const* gz, hipStream_t stream,
                            bool f16x3 = false);
SdfLayout sdf_layout(const NrSdfDesc& d);
RadLayout rad_layout(const NrRadDesc& d);
int check_sdf_desc(const NrSdfDesc* d);
int check_rad_desc(const NrRadDesc* d);

}  // namespace nr
