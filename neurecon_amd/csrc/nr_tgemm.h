// neurecon_amd -- training layer GEMM arguments (internal header; nr_mlp.hip's tgemm_kernel)
#pragma once
#include <cstdint>
#include "nr_common.h"

namespace nr {

struct TGemmArgs {
  const char* op;        // packed op (render weight-stream format, f16x3)
  int64_t P;             // points (rows)
  const float* x1;       // input blocks [0, KB - KB2): x1[p * ld1 + col], n1 valid columns (rest zero)
  int64_t ld1;
  int n1;
  const float* x2;       // input blocks [KB - KB2, KB): x2[p * ld2 + col], n2 valid columns
  int64_t ld2;
  int n2;
  int use_bias;          // add the op's bias (bias slot floats 0..31)
  int mode;              // TgMode
  float yscale;          // TG_NONE / TG_MUL / TG_SPADJ: z * yscale first
  float* y;              // output blocks [0, NBO - NB2): y[p * ldy + 16 B + ...]
  int64_t ldy;
  float* yb;             // output blocks [NBO - NB2, NBO) (null: not stored)
  int64_t ldyb;
  float* y2;             // TG_SOFTPLUS: softplus';  TG_MUL: a * y   (blocks of y)
  int64_t ldy2;
  float* y3;             // TG_SOFTPLUS: softplus' * the op's per-row vector (blocks of y)
  int64_t ldy3;
  const float* a;        // TG_MUL factor, TG_SPADJ softplus', TG_RELUMASK activation (blocks of y)
  int64_t lda;
  const float* g;        // TG_SPADJ g (null: 0, or the op's per-row vector with g_row)
  int64_t ldg;
  const float* zd;       // TG_SPADJ zdot
  int64_t ldzd;
  int g_row;
  float* dot;            // TG_SOFTPLUS: per point h . (per-row vector) + dot_bias
  float dot_bias;
  const float* head;     // TG_RELU: radiance head [3][256] (device), rgb = sigmoid(y . head + head_bias)
  const float* head_bias;
  float* head_out;       // [P][3]
};

int launch_tgemm(const TGemmArgs& a, int KB, int KB2, int NBO, int NB2, hipStream_t stream);

}  // namespace nr
