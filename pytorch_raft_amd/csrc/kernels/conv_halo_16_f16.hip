// Instantiations of the halo-tile conv kernel (conv_halo.h) whose A image takes 16 LDS-DMA
// pieces per thread and chunk, fp16 operands; one translation unit per (image size, operand type)
// so they compile in parallel.
#include "conv_halo.h"

namespace conv_detail {
RAFT_HALO_TU(16, EPI_F16)
}  // namespace conv_detail
