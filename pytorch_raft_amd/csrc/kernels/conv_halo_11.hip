// Instantiations of the halo-tile conv kernel (conv_halo.h) whose A image takes 11 LDS-DMA
// pieces per thread and chunk, bf16 operands; one translation unit per (image size, operand type)
// so they compile in parallel.
#include "conv_halo.h"

namespace conv_detail {
RAFT_HALO_TU(11, 0)
}  // namespace conv_detail
