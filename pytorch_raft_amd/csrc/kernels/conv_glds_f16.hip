// fp16-operand instantiations of the LDS-DMA conv kernel (conv_glds.h): the update block under
// fp16 autocast (`core/raft.py:99,110,127` with --mixed_precision) runs the same tiles and
// epilogues as bf16 on v_mfma_f32_32x32x16_f16.
#include "conv_glds.h"

bool launch_conv_glds_f16(const ConvFwdArgs& a, int epi, int idx, hipStream_t stream) {
  using namespace conv_detail;
  switch (epi_kind(epi)) {
    case EPI_BF16: return launch_glds_epi<EPI_BF16 | EPI_F16>(a, idx, stream);
    case EPI_RELU_BF16: return launch_glds_epi<EPI_RELU_BF16 | EPI_F16>(a, idx, stream);
    case EPI_F32: return launch_glds_epi<EPI_F32 | EPI_F16>(a, idx, stream);
    case EPI_GRU_ZR: return launch_glds_epi<EPI_GRU_ZR | EPI_F16>(a, idx, stream);
    case EPI_GRU_Q: return launch_glds_epi<EPI_GRU_Q | EPI_F16>(a, idx, stream);
    case EPI_DGRAD: return launch_glds_epi<EPI_DGRAD | EPI_F16>(a, idx, stream);
    case EPI_DGRAD_GATE: return launch_glds_epi<EPI_DGRAD_GATE | EPI_F16>(a, idx, stream);
    case EPI_F32_NCHW: return launch_glds_epi<EPI_F32_NCHW | EPI_F16>(a, idx, stream);
    default: return false;
  }
}
