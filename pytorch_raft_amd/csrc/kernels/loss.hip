// Fused RAFT sequence loss + EPE metrics (forward) and its gradient (backward).
//
// Reference `sequence_loss` (`train.py:47-72`): per prediction i, gamma^(n-i-1) * mean(valid*|p_i-gt|)
// over (B,2,H,W), valid = (valid >= 0.5) & (|gt| < max_flow); metrics epe/1px/3px/5px over the valid
// pixels of the last prediction.  The reference launches ~5 kernels per prediction plus a boolean
// index and four `.item()` host syncs per step.  Here: one pass over all n predictions writes
// per-block partials, a one-block pass reduces them deterministically (fixed order, fp64) to
// [loss, epe_mean, 1px, 3px, 5px, n_valid] on the device -- no host sync anywhere.
#include "common.h"
#include "launchers.h"

namespace {

constexpr int LOSS_BLOCKS = 1024;
constexpr int NSTAT = 6;  // wloss, epe_sum, cnt, c1, c3, c5

__global__ __launch_bounds__(256) void seq_loss_partial_kernel(PredPtrs preds, int n,
                                                               const float* __restrict__ gt,
                                                               const float* __restrict__ valid,
                                                               float gamma, float max_flow, int B,
                                                               int64_t HW, float* __restrict__ partial) {
  float st[NSTAT] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int64_t total = (int64_t)B * HW;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / HW, p = t % HW;
    const int64_t o0 = b * 2 * HW + p, o1 = o0 + HW;
    const float gx = gt[o0], gy = gt[o1];
    const float mag = sqrtf(gx * gx + gy * gy);
    const bool v = (valid[t] >= 0.5f) && (mag < max_flow);
    if (!v) continue;
    // predictions four at a time, their 8 loads issued before the sums (the same accumulation
    // order as one at a time: newest first, w = gamma^(n-1-i))
    float w = 1.f, wl = 0.f;
    for (int i0 = n - 1; i0 >= 0; i0 -= 4) {
      float px[4], py[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int i = i0 - u >= 0 ? i0 - u : 0;   // past the oldest: a valid (unused) read
        px[u] = preds.p[i][o0];
        py[u] = preds.p[i][o1];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (i0 - u >= 0) {
          wl += w * (fabsf(px[u] - gx) + fabsf(py[u] - gy));
          w *= gamma;
        }
      }
    }
    const float* P = preds.p[n - 1];
    const float dx = P[o0] - gx, dy = P[o1] - gy;
    const float epe = sqrtf(dx * dx + dy * dy);
    st[0] += wl;
    st[1] += epe;
    st[2] += 1.f;
    st[3] += epe < 1.f ? 1.f : 0.f;
    st[4] += epe < 3.f ? 1.f : 0.f;
    st[5] += epe < 5.f ? 1.f : 0.f;
  }
  __shared__ float red[4][NSTAT];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < NSTAT; ++k) {
    float s = wave_sum(st[k]);
    if (lane == 0) red[wv][k] = s;
  }
  __syncthreads();
  if (threadIdx.x < NSTAT) {
    const int k = threadIdx.x;
    partial[blockIdx.x * NSTAT + k] = ((red[0][k] + red[1][k]) + red[2][k]) + red[3][k];
  }
}

__global__ __launch_bounds__(256) void seq_loss_final_kernel(const float* __restrict__ partial,
                                                             int nblocks, double numel,
                                                             float* __restrict__ out) {
  __shared__ double red[256][NSTAT];
  double st[NSTAT] = {0, 0, 0, 0, 0, 0};
  for (int i = threadIdx.x; i < nblocks; i += 256)
    for (int k = 0; k < NSTAT; ++k) st[k] += (double)partial[i * NSTAT + k];
  for (int k = 0; k < NSTAT; ++k) red[threadIdx.x][k] = st[k];
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s)
      for (int k = 0; k < NSTAT; ++k) red[threadIdx.x][k] += red[threadIdx.x + s][k];
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double cnt = red[0][2];
    out[0] = (float)(red[0][0] / numel);
    out[1] = (float)(red[0][1] / cnt);  // NaN when nothing is valid, like the reference
    out[2] = (float)(red[0][3] / cnt);
    out[3] = (float)(red[0][4] / cnt);
    out[4] = (float)(red[0][5] / cnt);
    out[5] = (float)cnt;
  }
}

__global__ __launch_bounds__(256) void seq_loss_bwd_kernel(PredPtrs preds, PredPtrsMut grads, int n,
                                                           const float* __restrict__ gt,
                                                           const float* __restrict__ valid,
                                                           const float* __restrict__ dloss,
                                                           float gamma, float max_flow, int B,
                                                           int64_t HW, float inv_numel) {
  const int64_t total = (int64_t)B * HW;
  const float g = dloss[0] * inv_numel;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = t / HW, p = t % HW;
    const int64_t o0 = b * 2 * HW + p, o1 = o0 + HW;
    const float gx = gt[o0], gy = gt[o1];
    const float mag = sqrtf(gx * gx + gy * gy);
    const bool v = (valid[t] >= 0.5f) && (mag < max_flow);
    float w = v ? g : 0.f;
    for (int i = n - 1; i >= 0; --i) {
      const float* P = preds.p[i];
      const float d0 = P[o0] - gx, d1 = P[o1] - gy;
      // d|x|/dx = sign(x), 0 at 0 (matches torch.abs backward)
      grads.p[i][o0] = w * (float)((d0 > 0.f) - (d0 < 0.f));
      grads.p[i][o1] = w * (float)((d1 > 0.f) - (d1 < 0.f));
      w *= gamma;
    }
  }
}

}  // namespace

int seq_loss_partial_count() { return LOSS_BLOCKS * NSTAT; }

void launch_seq_loss_fwd(const PredPtrs& preds, int n, const float* gt, const float* valid,
                         float gamma, float max_flow, int B, int64_t HW, float* partial, float* out,
                         hipStream_t stream) {
  int64_t total = (int64_t)B * HW;
  int blocks = (int)std::min<int64_t>(LOSS_BLOCKS, (total + 255) / 256);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(seq_loss_partial_kernel, dim3(blocks), dim3(256), 0, stream, preds, n, gt,
                     valid, gamma, max_flow, B, HW, partial);
  hipLaunchKernelGGL(seq_loss_final_kernel, dim3(1), dim3(256), 0, stream, partial, blocks,
                     (double)B * 2.0 * (double)HW, out);
}

void launch_seq_loss_bwd(const PredPtrs& preds, const PredPtrsMut& grads, int n, const float* gt,
                         const float* valid, const float* dloss, float gamma, float max_flow, int B,
                         int64_t HW, hipStream_t stream) {
  int64_t total = (int64_t)B * HW;
  int blocks = (int)std::min<int64_t>(4096, (total + 255) / 256);
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(seq_loss_bwd_kernel, dim3(blocks), dim3(256), 0, stream, preds, grads, n, gt,
                     valid, dloss, gamma, max_flow, B, HW, (float)(1.0 / ((double)B * 2.0 * HW)));
}
