// Instantiations of the halo-tile conv kernel (conv_halo.h) whose A image takes 6 LDS-DMA pieces
// per thread and chunk; one translation unit per image size so they compile in parallel.
#include "conv_halo.h"

namespace conv_detail {

template <int EPI, int TM, int TN, int WVM>
static void launch_halo_one_6(const ConvFwdArgs& a, hipStream_t stream) {
  constexpr int BM = 32 * TM * WVM, BN = 32 * TN * (4 / WVM);
  const int P = a.B * a.H * a.W;
  dim3 grid(conv_grid_1d(raft_cdiv(P, BM), raft_cdiv(a.cout, BN)));
  hipLaunchKernelGGL((conv_fwd_halo_kernel<TM, TN, WVM, EPI, 6>), grid, dim3(NT), 0, stream, a);
}

template <int EPI>
static bool halo_cfg_6(const ConvFwdArgs& a, int tm, int tn, int wvm, hipStream_t s) {
  if (tm == 5 && tn == 1 && wvm == 1) { launch_halo_one_6<EPI, 5, 1, 1>(a, s); return true; }
  if (tm == 5 && tn == 2 && wvm == 1) { launch_halo_one_6<EPI, 5, 2, 1>(a, s); return true; }
  if (tm == 4 && tn == 2 && wvm == 1) { launch_halo_one_6<EPI, 4, 2, 1>(a, s); return true; }
  if (tm == 2 && tn == 2 && wvm == 2) { launch_halo_one_6<EPI, 2, 2, 2>(a, s); return true; }
  return false;
}

template <>
bool launch_conv_halo_npa<6>(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm, hipStream_t s) {
  switch (epi) {
    case EPI_BF16: return halo_cfg_6<EPI_BF16>(a, tm, tn, wvm, s);
    case EPI_RELU_BF16: return halo_cfg_6<EPI_RELU_BF16>(a, tm, tn, wvm, s);
    case EPI_F32: return halo_cfg_6<EPI_F32>(a, tm, tn, wvm, s);
    case EPI_GRU_ZR: return halo_cfg_6<EPI_GRU_ZR>(a, tm, tn, wvm, s);
    case EPI_GRU_Q: return halo_cfg_6<EPI_GRU_Q>(a, tm, tn, wvm, s);
    case EPI_DGRAD: return halo_cfg_6<EPI_DGRAD>(a, tm, tn, wvm, s);
    case EPI_DGRAD_GATE: return halo_cfg_6<EPI_DGRAD_GATE>(a, tm, tn, wvm, s);
    default: return false;
  }
}

}  // namespace conv_detail

// image size -> the smallest instantiation that holds it (none beyond 16 pieces: 2 x 64 KiB)
bool launch_conv_halo(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm, hipStream_t stream) {
  using namespace conv_detail;
  if (a.cin_small || a.cin_pad % BK != 0 || a.nseg < 1 || a.nseg > 3) return false;
  const int bm = 32 * tm * wvm;
  const int npa = halo_pieces(halo_rows(bm, a.W, a.KH, a.KW, a.PH, a.PW));
  if (npa <= 6) return launch_conv_halo_npa<6>(a, epi, tm, tn, wvm, stream);
  if (npa <= 11) return launch_conv_halo_npa<11>(a, epi, tm, tn, wvm, stream);
  if (npa <= 16) return launch_conv_halo_npa<16>(a, epi, tm, tn, wvm, stream);
  return false;
}
