// bf16-operand instantiations of the LDS-DMA conv kernel (conv_glds.h)
#include "conv_glds.h"

// config index -> LDS-DMA kernel launch (indices as in conv_igemm.hip's kCfgs table)
bool launch_conv_glds(const ConvFwdArgs& a, int epi, int idx, hipStream_t stream) {
  using namespace conv_detail;
  if (epi_f16(epi)) return launch_conv_glds_f16(a, epi, idx, stream);
  if (epi_spl(epi)) return launch_conv_glds_spl(a, epi, idx, stream);
  switch (epi) {
    case EPI_BF16: return launch_glds_epi<EPI_BF16>(a, idx, stream);
    case EPI_RELU_BF16: return launch_glds_epi<EPI_RELU_BF16>(a, idx, stream);
    case EPI_F32: return launch_glds_epi<EPI_F32>(a, idx, stream);
    case EPI_ACC_F32: return launch_glds_epi<EPI_ACC_F32>(a, idx, stream);
    case EPI_GRU_ZR: return launch_glds_epi<EPI_GRU_ZR>(a, idx, stream);
    case EPI_GRU_Q: return launch_glds_epi<EPI_GRU_Q>(a, idx, stream);
    case EPI_DGRAD: return launch_glds_epi<EPI_DGRAD>(a, idx, stream);
    case EPI_DGRAD_GATE: return launch_glds_epi<EPI_DGRAD_GATE>(a, idx, stream);
    case EPI_F32_NCHW: return launch_glds_epi<EPI_F32_NCHW>(a, idx, stream);
    default: return false;
  }
}
