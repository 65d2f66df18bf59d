// Flow-driven bilinear backward warping (forward + backward), zero padding.
//
// Used by the warping applications (reference `warp()` in demo_warp*.py: grid + flow -> normalise ->
// F.grid_sample) and usable as a differentiable photometric-warp op.  One thread per output pixel
// loops over channels; the sample position is  s = (p + flow(p)) * scale + shift  per axis, which
// covers both conventions:
//   exact      scale = 1,           shift = 0      (sample exactly at p + flow)
//   reference  scale = W / (W - 1), shift = -0.5   (normalised with (W-1) but sampled with
//                                                  align_corners=False, as `demo_warp.py:45-49`)
// Backward: d(img) by float atomics (many-to-one), d(flow) from the bilinear weight derivatives.
#include "common.h"
#include "launchers.h"

namespace {

__global__ __launch_bounds__(256) void warp_fwd_kernel(const float* __restrict__ img,
                                                       const float* __restrict__ flow,
                                                       float* __restrict__ out, int B, int C, int H,
                                                       int W, float sx, float bx, float sy, float by) {
  const int64_t HW = (int64_t)H * W;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * HW) return;
  const int x = (int)(t % W), y = (int)((t / W) % H);
  const int64_t b = t / HW;
  const float fx = flow[(b * 2) * HW + (int64_t)y * W + x];
  const float fy = flow[(b * 2 + 1) * HW + (int64_t)y * W + x];
  const float px = (x + fx) * sx + bx, py = (y + fy) * sy + by;
  const float x0f = floorf(px), y0f = floorf(py);
  const float ax = px - x0f, ay = py - y0f;
  const int x0 = (int)fminf(fmaxf(x0f, -2.f), (float)W + 1), y0 = (int)fminf(fmaxf(y0f, -2.f), (float)H + 1);
  const bool vx0 = x0 >= 0 && x0 < W, vx1 = x0 + 1 >= 0 && x0 + 1 < W;
  const bool vy0 = y0 >= 0 && y0 < H, vy1 = y0 + 1 >= 0 && y0 + 1 < H;
  for (int c = 0; c < C; ++c) {
    const float* I = img + (b * C + c) * HW;
    float v = 0.f;
    if (vy0 && vx0) v += (1.f - ax) * (1.f - ay) * I[(int64_t)y0 * W + x0];
    if (vy0 && vx1) v += ax * (1.f - ay) * I[(int64_t)y0 * W + x0 + 1];
    if (vy1 && vx0) v += (1.f - ax) * ay * I[(int64_t)(y0 + 1) * W + x0];
    if (vy1 && vx1) v += ax * ay * I[(int64_t)(y0 + 1) * W + x0 + 1];
    out[(b * C + c) * HW + (int64_t)y * W + x] = v;
  }
}

__global__ __launch_bounds__(256) void warp_bwd_kernel(const float* __restrict__ img,
                                                       const float* __restrict__ flow,
                                                       const float* __restrict__ dout,
                                                       float* __restrict__ dimg,
                                                       float* __restrict__ dflow, int B, int C, int H,
                                                       int W, float sx, float bx, float sy, float by) {
  const int64_t HW = (int64_t)H * W;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * HW) return;
  const int x = (int)(t % W), y = (int)((t / W) % H);
  const int64_t b = t / HW;
  const float fx = flow[(b * 2) * HW + (int64_t)y * W + x];
  const float fy = flow[(b * 2 + 1) * HW + (int64_t)y * W + x];
  const float px = (x + fx) * sx + bx, py = (y + fy) * sy + by;
  const float x0f = floorf(px), y0f = floorf(py);
  const float ax = px - x0f, ay = py - y0f;
  const int x0 = (int)fminf(fmaxf(x0f, -2.f), (float)W + 1), y0 = (int)fminf(fmaxf(y0f, -2.f), (float)H + 1);
  const bool vx0 = x0 >= 0 && x0 < W, vx1 = x0 + 1 >= 0 && x0 + 1 < W;
  const bool vy0 = y0 >= 0 && y0 < H, vy1 = y0 + 1 >= 0 && y0 + 1 < H;
  float gx = 0.f, gy = 0.f;
  for (int c = 0; c < C; ++c) {
    const float* I = img + (b * C + c) * HW;
    float* dI = dimg + (b * C + c) * HW;
    const float g = dout[(b * C + c) * HW + (int64_t)y * W + x];
    const float v00 = (vy0 && vx0) ? I[(int64_t)y0 * W + x0] : 0.f;
    const float v01 = (vy0 && vx1) ? I[(int64_t)y0 * W + x0 + 1] : 0.f;
    const float v10 = (vy1 && vx0) ? I[(int64_t)(y0 + 1) * W + x0] : 0.f;
    const float v11 = (vy1 && vx1) ? I[(int64_t)(y0 + 1) * W + x0 + 1] : 0.f;
    gx += g * ((1.f - ay) * (v01 - v00) + ay * (v11 - v10));
    gy += g * ((1.f - ax) * (v10 - v00) + ax * (v11 - v01));
    if (vy0 && vx0) atomicAdd(&dI[(int64_t)y0 * W + x0], (1.f - ax) * (1.f - ay) * g);
    if (vy0 && vx1) atomicAdd(&dI[(int64_t)y0 * W + x0 + 1], ax * (1.f - ay) * g);
    if (vy1 && vx0) atomicAdd(&dI[(int64_t)(y0 + 1) * W + x0], (1.f - ax) * ay * g);
    if (vy1 && vx1) atomicAdd(&dI[(int64_t)(y0 + 1) * W + x0 + 1], ax * ay * g);
  }
  dflow[(b * 2) * HW + (int64_t)y * W + x] = gx * sx;
  dflow[(b * 2 + 1) * HW + (int64_t)y * W + x] = gy * sy;
}

}  // namespace

void launch_warp_fwd(const float* img, const float* flow, float* out, int B, int C, int H, int W,
                     float sx, float bx, float sy, float by, hipStream_t stream) {
  const int64_t total = (int64_t)B * H * W;
  hipLaunchKernelGGL(warp_fwd_kernel, dim3(raft_cdiv(total, 256)), dim3(256), 0, stream, img, flow,
                     out, B, C, H, W, sx, bx, sy, by);
}

void launch_warp_bwd(const float* img, const float* flow, const float* dout, float* dimg,
                     float* dflow, int B, int C, int H, int W, float sx, float bx, float sy,
                     float by, hipStream_t stream) {
  const int64_t total = (int64_t)B * H * W;
  hipLaunchKernelGGL(warp_bwd_kernel, dim3(raft_cdiv(total, 256)), dim3(256), 0, stream, img, flow,
                     dout, dimg, dflow, B, C, H, W, sx, bx, sy, by);
}
