// Multi-tensor AdamW with the global-norm gradient clip folded in (the training step's update:
// reference `train.py:158-181` -- clip_grad_norm_(1.0), AdamW(lr, wd, eps), OneCycle lr).
//
// torch's fused AdamW spent 4 multi-tensor launches x ~72 us on RAFT's 5.3 M parameters in ~150
// tensors (a few thousand elements per workgroup, most of the GPU idle) plus two launches for the
// foreach clip.  Here every tensor is cut into CH-element chunks, one workgroup per chunk over
// all tensors at once (~1.4 K workgroups), in three launches:
//   1. sum of squares of the gradients per chunk (fixed-order block reduction, no atomics);
//   2. one workgroup: total norm in fixed chunk order -> clip coefficient min(1, max/(norm+1e-6));
//   3. the AdamW update with the clipped gradient (torch's non-amsgrad AdamW arithmetic:
//      p *= 1 - lr wd;  m = lerp(m, g, 1-b1);  v = b2 v + (1-b2) g^2;
//      p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)).
// Tensor pointers come in a small device table (the gradients are new allocations every step);
// a workgroup finds its tensor by binary search over the cumulative chunk counts.
#include "common.h"
#include "launchers.h"

namespace {

constexpr int ADAM_CH = 4096;  // elements per chunk (workgroup)
constexpr int ADAM_NT = 256;

struct AdamTab {
  const AdamTensor* t;  // [T]
  const int* cum;       // [T + 1] cumulative chunk counts
  int T;
};

__device__ __forceinline__ int find_tensor(const int* __restrict__ cum, int T, int c) {
  int lo = 0, hi = T - 1;  // largest i with cum[i] <= c
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (cum[mid] <= c) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = v;
  __syncthreads();
  float s = 0.f;
  if (threadIdx.x == 0)
    for (int w = 0; w < ADAM_NT / 64; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(ADAM_NT) void adam_sumsq_kernel(AdamTab tab, float* __restrict__ part) {
  __shared__ float red[ADAM_NT / 64];
  const int c = blockIdx.x;
  const int ti = find_tensor(tab.cum, tab.T, c);
  const AdamTensor t = tab.t[ti];
  const int64_t s0 = (int64_t)(c - tab.cum[ti]) * ADAM_CH;
  const int64_t n = min((int64_t)ADAM_CH, t.numel - s0);
  const float* g = t.g + s0;
  float acc = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += ADAM_NT) acc += g[e] * g[e];
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) part[c] = s;
}

// coef[0] = clip coefficient, coef[1] = total norm
__global__ __launch_bounds__(ADAM_NT) void adam_clip_kernel(const float* __restrict__ part, int nchunks,
                                                            float max_norm, float* __restrict__ coef) {
  __shared__ float red[ADAM_NT];
  float s = 0.f;
  for (int c = threadIdx.x; c < nchunks; c += ADAM_NT) s += part[c];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int i = 0; i < ADAM_NT; ++i) tot += red[i];
    const float norm = sqrtf(tot);
    coef[0] = fminf(1.f, max_norm / (norm + 1e-6f));
    coef[1] = norm;
  }
}

__global__ __launch_bounds__(ADAM_NT) void adam_update_kernel(AdamTab tab, const float* __restrict__ lr_dev,
                                                              float lr_host, float b1, float b2, float omb1,
                                                              float omb2, float eps,
                                                              float wd, float bc1, float bc2_sqrt,
                                                              const float* __restrict__ coef) {
  const int c = blockIdx.x;
  const int ti = find_tensor(tab.cum, tab.T, c);
  const AdamTensor t = tab.t[ti];
  const int64_t s0 = (int64_t)(c - tab.cum[ti]) * ADAM_CH;
  const int64_t n = min((int64_t)ADAM_CH, t.numel - s0);
  const float lr = lr_dev != nullptr ? lr_dev[0] : lr_host;
  const float k = coef != nullptr ? coef[0] : 1.f;
  const float decay = 1.f - lr * wd, step = lr / bc1;
  float* p = t.p + s0;
  const float* g = t.g + s0;
  float* m = t.m + s0;
  float* v = t.v + s0;
  for (int64_t e = threadIdx.x; e < n; e += ADAM_NT) {
    const float gg = g[e] * k;
    const float mm = m[e] + omb1 * (gg - m[e]);  // lerp(m, g, 1 - b1)
    const float vv = b2 * v[e] + omb2 * gg * gg;
    m[e] = mm;
    v[e] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    p[e] = p[e] * decay - step * mm / denom;
  }
}

}  // namespace

int adam_chunk_elems() { return ADAM_CH; }

void launch_adamw_multi(const AdamTensor* tab, const int* cum, int T, int nchunks, const float* lr_dev,
                        float lr_host, double b1, double b2, float eps, float wd, float bc1, float bc2,
                        float max_norm, float* part, float* coef, hipStream_t stream) {
  // 1 - beta in double, like torch (1 - 0.999 from a float-rounded beta is 1.3e-5 off)
  AdamTab at{tab, cum, T};
  if (max_norm > 0.f) {
    hipLaunchKernelGGL(adam_sumsq_kernel, dim3((unsigned)nchunks), dim3(ADAM_NT), 0, stream, at, part);
    hipLaunchKernelGGL(adam_clip_kernel, dim3(1), dim3(ADAM_NT), 0, stream, part, nchunks, max_norm, coef);
  }
  hipLaunchKernelGGL(adam_update_kernel, dim3((unsigned)nchunks), dim3(ADAM_NT), 0, stream, at, lr_dev,
                     lr_host, (float)b1, (float)b2, (float)(1.0 - b1), (float)(1.0 - b2), eps, wd, bc1,
                     sqrtf(bc2), max_norm > 0.f ? coef : nullptr);
}
