// neurecon_amd -- training layer GEMM (internal header; nr_mlp.hip's tgemm_kernel, C-ABI
// NrTrainGemm in include/neurecon_hip.h)
#pragma once
#include <cstdint>
#include "nr_common.h"

namespace nr {

using TGemmArgs = NrTrainGemm;

int launch_tgemm(const TGemmArgs& a, int KB, int KB2, int NBO, int NB2, hipStream_t stream);

}  // namespace nr
