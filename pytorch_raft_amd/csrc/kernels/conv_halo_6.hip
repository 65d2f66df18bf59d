// Instantiations of the halo-tile conv kernel (conv_halo.h) whose A image takes 6 LDS-DMA
// pieces per thread and chunk, bf16 operands; one translation unit per (image size, operand type)
// so they compile in parallel.
#include "conv_halo.h"

namespace conv_detail {
RAFT_HALO_TU(6, 0)
}  // namespace conv_detail

// image size -> the smallest instantiation that holds it (none beyond 16 pieces: 2 x 64 KiB)
bool launch_conv_halo(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm, hipStream_t stream) {
  using namespace conv_detail;
  if (a.cin_small || a.cin_pad % BK != 0 || a.nseg < 1 || a.nseg > 3) return false;
  const int bm = 32 * tm * wvm;
  const int npa = halo_pieces(halo_rows(bm, a.W, a.KH, a.KW, a.PH, a.PW));
  const int ty = epi_f16(epi) ? EPI_F16 : (epi_spl(epi) ? EPI_SPL : 0);
#define RAFT_HALO_PICK(N)                                                           \
  return ty == EPI_F16 ? launch_conv_halo_npa<N, EPI_F16>(a, epi, tm, tn, wvm, stream) \
         : ty == EPI_SPL ? launch_conv_halo_npa<N, EPI_SPL>(a, epi, tm, tn, wvm, stream) \
                         : launch_conv_halo_npa<N, 0>(a, epi, tm, tn, wvm, stream);
  if (npa <= 6) RAFT_HALO_PICK(6)
  if (npa <= 11) RAFT_HALO_PICK(11)
  if (npa <= 16) RAFT_HALO_PICK(16)
#undef RAFT_HALO_PICK
  return false;
}
