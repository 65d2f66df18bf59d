// Encoder input preparation in one pass (`core/raft.py:94-95` + `core/extractor.py:176-179`):
// the two (B,3,H,W) fp32 frames in 0..255 -> 2 * (x / 255) - 1 -> the feature encoder's batch
// [frame1 ; frame2] as ONE channels_last tensor (2B,H,W,3) in the encoders' compute dtype.  The
// context encoder reads its first half (frame1) in place.  Replaces per step: the two normalising
// chains (3 elementwise kernels each), the batch cat, the dtype cast and the channels_last copy.
//
// Numerics: the same three fp32 roundings as the eager ops -- ATen divides by a scalar as a
// multiply by its (double-computed, float-rounded) reciprocal, then 2 * t (exact), then t - 1 --
// and one rounding to the compute dtype: bitwise the eager path's conv input.
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <hip/hip_fp16.h>

#include "launchers.h"

namespace {

template <int OT>
__device__ __forceinline__ void put(void* out, int64_t i, float v) {
  if constexpr (OT == 0) {
    static_cast<__hip_bfloat16*>(out)[i] = __float2bfloat16(v);
  } else if constexpr (OT == 1) {
    static_cast<__half*>(out)[i] = __float2half(v);
  } else {
    static_cast<float*>(out)[i] = v;
  }
}

template <int OT>
__global__ __launch_bounds__(256) void image_prep_kernel(const float* __restrict__ a,
                                                         const float* __restrict__ b, void* __restrict__ out,
                                                         int B, int64_t HW, float inv255) {
  const int64_t total = 2 * (int64_t)B * HW;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < total;
       p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = p / HW, s = p - n * HW;
    const float* src = n < B ? a + n * 3 * HW : b + (n - B) * 3 * HW;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      float t = src[c * HW + s] * inv255;
      t = 2.0f * t;
      t = t - 1.0f;
      put<OT>(out, p * 3 + c, t);
    }
  }
}

}  // namespace

bool launch_image_prep(const float* a, const float* b, void* out, int B, int64_t HW, int ot,
                       hipStream_t stream) {
  if (B < 1 || HW < 1 || ot < 0 || ot > 2) return false;
  const int64_t total = 2 * (int64_t)B * HW;
  const unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 256 * 32);
  const float inv255 = 1.0f / 255.0f;   // ATen's reciprocal of the float scalar
  if (ot == 0)
    hipLaunchKernelGGL(image_prep_kernel<0>, dim3(blocks), dim3(256), 0, stream, a, b, out, B, HW, inv255);
  else if (ot == 1)
    hipLaunchKernelGGL(image_prep_kernel<1>, dim3(blocks), dim3(256), 0, stream, a, b, out, B, HW, inv255);
  else
    hipLaunchKernelGGL(image_prep_kernel<2>, dim3(blocks), dim3(256), 0, stream, a, b, out, B, HW, inv255);
  return true;
}
