// Instantiations + launcher of the pipelined v3 conv kernel (conv_v3.h); its own translation unit
// so the (tile x epilogue) instantiations compile in parallel with the other conv kernels.
#include "conv_v3.h"

namespace conv_detail {

template <int EPI, int TM, int TN, int OCC>
void launch_one_v3(const ConvFwdArgs& a, hipStream_t stream) {
  using T = V3Tile<TM, TN>;
  const int P = a.B * a.H * a.W;
  dim3 grid(conv_grid_1d(raft_cdiv(P, T::BM), raft_cdiv(a.cout, T::BN)));
  hipLaunchKernelGGL((conv_fwd_v3_kernel<TM, TN, EPI, OCC>), grid, dim3(NT), 0, stream, a,
                     (unsigned long long*)nullptr);
}

template <int EPI>
bool launch_v3_epi(const ConvFwdArgs& a, int tm, int tn, hipStream_t stream) {
  if (tm == 5 && tn == 1) { launch_one_v3<EPI, 5, 1, 2>(a, stream); return true; }
  if (tm == 3 && tn == 1) { launch_one_v3<EPI, 3, 1, 2>(a, stream); return true; }
  // the wide tiles' GRU-gate epilogues spill (scratch): not offered there
  if constexpr (EPI != EPI_GRU_ZR && EPI != EPI_DGRAD_GATE) {
    if (tm == 5 && tn == 2) { launch_one_v3<EPI, 5, 2, 1>(a, stream); return true; }
  }
  if constexpr (EPI != EPI_DGRAD_GATE) {
    if (tm == 3 && tn == 2) { launch_one_v3<EPI, 3, 2, 2>(a, stream); return true; }
  }
  return false;
}

}  // namespace conv_detail

bool launch_conv_v3(const ConvFwdArgs& a, int epi, int tm, int tn, hipStream_t stream) {
  using namespace conv_detail;
  // the kernel advances the A position by whole 64-channel chunks: every segment a multiple of 64
  for (int q = 0; q < a.nseg; ++q)
    if (a.seg[q].cnt % BK) return false;
  if (a.KH * a.KW > 32) return false;  // per-piece tap masks are 32 bits
  switch (epi) {
    case EPI_BF16: return launch_v3_epi<EPI_BF16>(a, tm, tn, stream);
    case EPI_RELU_BF16: return launch_v3_epi<EPI_RELU_BF16>(a, tm, tn, stream);
    case EPI_F32: return launch_v3_epi<EPI_F32>(a, tm, tn, stream);
    case EPI_ACC_F32: return launch_v3_epi<EPI_ACC_F32>(a, tm, tn, stream);
    case EPI_GRU_ZR: return launch_v3_epi<EPI_GRU_ZR>(a, tm, tn, stream);
    case EPI_GRU_Q: return launch_v3_epi<EPI_GRU_Q>(a, tm, tn, stream);
    case EPI_DGRAD: return launch_v3_epi<EPI_DGRAD>(a, tm, tn, stream);
    case EPI_DGRAD_GATE: return launch_v3_epi<EPI_DGRAD_GATE>(a, tm, tn, stream);
    case EPI_F32_NCHW: return launch_v3_epi<EPI_F32_NCHW>(a, tm, tn, stream);
    default: return false;
  }
}
