// split-fp32 instantiations of the LDS-DMA conv kernel (conv_glds.h): the update block of the
// fp32 schedule (`train_standard.sh`, no --mixed_precision) runs the bf16 tiles on K thirds
// [hi | lo | hi] x [w_hi | w_hi | w_lo] (ConvFwdArgs.spl), its epilogues reading and writing
// activations as bf16 hi / lo pairs (EPI_SPL).
#include "conv_glds.h"

bool launch_conv_glds_spl(const ConvFwdArgs& a, int epi, int idx, hipStream_t stream) {
  using namespace conv_detail;
  switch (epi_kind(epi)) {
    case EPI_BF16: return launch_glds_epi<EPI_BF16 | EPI_SPL>(a, idx, stream);
    case EPI_RELU_BF16: return launch_glds_epi<EPI_RELU_BF16 | EPI_SPL>(a, idx, stream);
    case EPI_F32: return launch_glds_epi<EPI_F32 | EPI_SPL>(a, idx, stream);
    case EPI_F32_NCHW: return launch_glds_epi<EPI_F32_NCHW | EPI_SPL>(a, idx, stream);
    case EPI_GRU_ZR: return launch_glds_epi<EPI_GRU_ZR | EPI_SPL>(a, idx, stream);
    case EPI_GRU_Q: return launch_glds_epi<EPI_GRU_Q | EPI_SPL>(a, idx, stream);
    case EPI_DGRAD: return launch_glds_epi<EPI_DGRAD | EPI_SPL>(a, idx, stream);
    case EPI_DGRAD_GATE: return launch_glds_epi<EPI_DGRAD_GATE | EPI_SPL>(a, idx, stream);
    default: return false;
  }
}
