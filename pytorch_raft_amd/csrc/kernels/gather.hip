// Multi-source gather + cast: the per-step weight packing of the fused update block and of the
// encoders' 16-bit channels_last weights (ops/update_hip.py:_Packed, ops/encoder.py:_CastWeightsCL).
//
// out[i] = cast(src[k][off]) with (k, off) = idx[i] >> 26, idx[i] & (2^26 - 1); k == 63 is the
// zero padding slot.  The parameters are read where they live (no torch.cat of all of them into
// one flat buffer first), and the cast happens on the store, so packing every kernel-layout
// weight of a step is ONE launch instead of cat + int64 gather + cast.  The source set
// (~25-60 small fp32 parameters, a few MB) stays in L2; the int32 index stream and the 2-byte
// stores are the HBM traffic.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include "launchers.h"

namespace {

template <int OT>
__device__ __forceinline__ void store1(void* out, int64_t i, float v) {
  if constexpr (OT == 0) {
    static_cast<__hip_bfloat16*>(out)[i] = __float2bfloat16(v);
  } else if constexpr (OT == 1) {
    static_cast<__half*>(out)[i] = __float2half(v);
  } else {
    static_cast<float*>(out)[i] = v;
  }
}

template <int IT>
__device__ __forceinline__ float load1(const void* p, int off) {
  if constexpr (IT == 0) {
    return __bfloat162float(static_cast<const __hip_bfloat16*>(p)[off]);
  } else if constexpr (IT == 1) {
    return __half2float(static_cast<const __half*>(p)[off]);
  } else {
    return static_cast<const float*>(p)[off];
  }
}

template <int IT, int OT>
__global__ __launch_bounds__(256) void gather_cast_kernel(GatherSrcs s, const int32_t* __restrict__ idx,
                                                          void* __restrict__ out, int64_t n) {
  // 4 elements per thread per round, all index loads issued before the dependent value loads
  const int64_t stride = (int64_t)gridDim.x * blockDim.x * 4;
  for (int64_t i0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4; i0 < n; i0 += stride) {
    int32_t e[4];
    if (i0 + 3 < n) {
      const int4 q = *reinterpret_cast<const int4*>(idx + i0);
      e[0] = q.x; e[1] = q.y; e[2] = q.z; e[3] = q.w;
    } else {
#pragma unroll
      for (int u = 0; u < 4; ++u) e[u] = i0 + u < n ? idx[i0 + u] : (RAFT_GATHER_ZERO << 26);
    }
    float v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int k = (int)((uint32_t)e[u] >> 26);
      const int off = e[u] & ((1 << 26) - 1);
      v[u] = k == RAFT_GATHER_ZERO ? 0.f : load1<IT>(s.p[k], off);
      // split-fp32 weight packs: the residual of the bf16 rounding (bf16(v - bf16(v)) stored)
      if (k >= s.lo_from && k != RAFT_GATHER_ZERO) v[u] -= __bfloat162float(__float2bfloat16(v[u]));
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (i0 + u < n) store1<OT>(out, i0 + u, v[u]);
  }
}

}  // namespace

bool launch_gather_cast(const GatherSrcs& s, const int32_t* idx, void* out, int64_t n, int it, int ot,
                        hipStream_t stream) {
  if (n <= 0) return true;
  if (s.n < 1 || s.n > RAFT_GATHER_MAX || it < 0 || it > 2 || ot < 0 || ot > 2) return false;
  const int64_t want = (n + 1023) / 1024;
  const unsigned blocks = (unsigned)std::min<int64_t>(want, 256 * 16);
  // the per-step packings: fp32 parameters -> bf16 / fp16 / fp32 kernel layouts, and the
  // encoders' bf16 / fp16 / fp32 weight gradients -> fp32 parameter layout
#define RAFT_GATHER_LAUNCH(I, O)                                                                   \
  if (it == I && ot == O) {                                                                        \
    hipLaunchKernelGGL((gather_cast_kernel<I, O>), dim3(blocks), dim3(256), 0, stream, s, idx, out, n); \
    return true;                                                                                   \
  }
  RAFT_GATHER_LAUNCH(2, 0)
  RAFT_GATHER_LAUNCH(2, 1)
  RAFT_GATHER_LAUNCH(2, 2)
  RAFT_GATHER_LAUNCH(0, 2)
  RAFT_GATHER_LAUNCH(1, 2)
#undef RAFT_GATHER_LAUNCH
  return false;
}
