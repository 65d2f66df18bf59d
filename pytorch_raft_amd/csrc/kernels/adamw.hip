// Multi-tensor AdamW with the global-norm gradient clip and the fp16 GradScaler's unscale /
// overflow skip folded in (the training step's update: reference `train.py:158-181` --
// scaler.unscale_, clip_grad_norm_(1.0), scaler.step(AdamW(lr, wd, eps)), OneCycle lr).
//
// torch's fused AdamW spent 4 multi-tensor launches x ~72 us on RAFT's 5.3 M parameters in ~150
// tensors (a few thousand elements per workgroup, most of the GPU idle) plus two launches for the
// foreach clip.  Here every tensor of every parameter group is cut into CH-element chunks, one
// workgroup per chunk over all tensors at once (~1.4 K workgroups), in three launches:
//   1. sum of squares of the gradients per chunk (fixed-order block reduction, no atomics);
//   2. one workgroup: total norm over ALL groups in fixed chunk order, unscaled by the
//      GradScaler's 1/S -> clip coefficient min(1, max/(norm+1e-6)) / S, found_inf = the norm is
//      not finite (an inf / nan anywhere makes the sum of squares non-finite); on a finite step
//      every tensor's device step counter advances (a skipped step leaves the moments, the
//      parameters and the step counts untouched, as torch's GradScaler.step does);
//   3. the AdamW update with the clipped gradient (torch's non-amsgrad AdamW arithmetic:
//      p *= 1 - lr wd;  m = lerp(m, g, 1-b1);  v = b2 v + (1-b2) g^2;
//      p -= (lr / bc1) m / (sqrt(v) / sqrt(bc2) + eps)), bias corrections from the tensor's own
//      step count, hyper-parameters from its group; optionally the clipped, unscaled gradient is
//      written back to .grad (what clip_grad_norm_ / unscale_ leave there).
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

// sum of squares of the UNSCALED gradients (g / S): the fp16 scale (up to 2^24) squared would
// overflow fp32 on gradients that torch's per-element unscale_ check passes
__global__ __launch_bounds__(ADAM_NT) void adam_sumsq_kernel(AdamTab tab, const float* __restrict__ inv_scale,
                                                             float* __restrict__ part) {
  __shared__ float red[ADAM_NT / 64];
  const int c = blockIdx.x;
  const int ti = find_tensor(tab.cum, tab.T, c);
  const AdamTensor t = tab.t[ti];
  const int64_t s0 = (int64_t)(c - tab.cum[ti]) * ADAM_CH;
  const int64_t n = min((int64_t)ADAM_CH, t.numel - s0);
  const float* g = t.g + s0;
  const float is = inv_scale != nullptr ? inv_scale[0] : 1.f;
  float acc = 0.f;
  for (int64_t e = threadIdx.x; e < n; e += ADAM_NT) {
    const float u = g[e] * is;
    acc += u * u;
  }
  const float s = block_sum(acc, red);
  if (threadIdx.x == 0) part[c] = s;
}

// coef[0] = gradient multiplier (clip coefficient / S), coef[1] = total (unscaled) norm,
// coef[2] = found_inf (1: skip the step); the tensors' step counters advance on a finite step
__global__ __launch_bounds__(ADAM_NT) void adam_clip_kernel(AdamTab tab, const float* __restrict__ part,
                                                            int nchunks, float max_norm,
                                                            const float* __restrict__ inv_scale,
                                                            float* __restrict__ coef,
                                                            float* __restrict__ found_inf) {
  __shared__ float red[ADAM_NT];
  __shared__ int fin;
  float s = 0.f;
  if (part != nullptr)
    for (int c = threadIdx.x; c < nchunks; c += ADAM_NT) s += part[c];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float tot = 0.f;
    for (int i = 0; i < ADAM_NT; ++i) tot += red[i];
    const float is = inv_scale != nullptr ? inv_scale[0] : 1.f;
    const float norm = sqrtf(tot);  // partials are of unscaled gradients
    const bool finite = isfinite(norm);
    const float k = max_norm > 0.f ? fminf(1.f, max_norm / (norm + 1e-6f)) : 1.f;
    coef[0] = k * is;
    coef[1] = norm;
    coef[2] = finite ? 0.f : 1.f;
    if (found_inf != nullptr) found_inf[0] = finite ? 0.f : 1.f;
    fin = finite ? 1 : 0;
  }
  __syncthreads();
  if (fin)
    for (int i = threadIdx.x; i < tab.T; i += ADAM_NT) tab.t[i].step[0] += 1.f;
}

__global__ __launch_bounds__(ADAM_NT) void adam_update_kernel(AdamTab tab, const AdamGroup* __restrict__ grp,
                                                              const float* __restrict__ coef,
                                                              int write_grad) {
  if (coef[2] != 0.f) return;   // overflow: the whole step is skipped
  const int c = blockIdx.x;
  const int ti = find_tensor(tab.cum, tab.T, c);
  const AdamTensor t = tab.t[ti];
  const AdamGroup gp = grp[t.group];
  const int64_t s0 = (int64_t)(c - tab.cum[ti]) * ADAM_CH;
  const int64_t n = min((int64_t)ADAM_CH, t.numel - s0);
  const float lr = gp.lr_dev != nullptr ? gp.lr_dev[0] : gp.lr;
  const float k = coef[0];
  // bias corrections of this tensor's own step count (already advanced by the clip kernel); in
  // double like torch's host-side 1 - beta ** step
  const double st = (double)t.step[0];
  const float bc1 = (float)(1.0 - pow((double)gp.b1, st));
  const float bc2_sqrt = sqrtf((float)(1.0 - pow((double)gp.b2, st)));
  const float decay = 1.f - lr * gp.wd, step = lr / bc1;
  const float b2 = gp.b2, omb1 = gp.omb1, omb2 = gp.omb2, eps = gp.eps;
  float* p = t.p + s0;
  float* g = t.g + s0;
  float* m = t.m + s0;
  float* v = t.v + s0;
  for (int64_t e = threadIdx.x; e < n; e += ADAM_NT) {
    const float gg = g[e] * k;
    if (write_grad) g[e] = gg;
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

void launch_adamw_multi(const AdamTensor* tab, const int* cum, int T, int nchunks, const AdamGroup* groups,
                        float max_norm, const float* inv_scale, int need_norm, int write_grad,
                        float* part, float* coef, float* found_inf, hipStream_t stream) {
  AdamTab at{tab, cum, T};
  if (need_norm)
    hipLaunchKernelGGL(adam_sumsq_kernel, dim3((unsigned)nchunks), dim3(ADAM_NT), 0, stream, at, inv_scale, part);
  hipLaunchKernelGGL(adam_clip_kernel, dim3(1), dim3(ADAM_NT), 0, stream, at, need_norm ? part : nullptr,
                     nchunks, max_norm, inv_scale, coef, found_inf);
  hipLaunchKernelGGL(adam_update_kernel, dim3((unsigned)nchunks), dim3(ADAM_NT), 0, stream, at, groups,
                     coef, write_grad);
}
