// Convex 8x upsampling of a 1/8-resolution flow field (forward + backward), and upflow8.
//
// Reference `RAFT.upsample_flow` (`core/raft.py:72-83`) is view -> softmax over the 9 neighbours ->
// F.unfold(8*flow, 3x3, pad 1) -> weighted sum -> 6-D permute -> reshape: five ATen kernels and two
// full-resolution temporaries per call.  Here one kernel reads the 576-channel mask once and writes
// the full-resolution flow; the backward is one kernel for d(mask) plus a tiny gather for d(flow).
//
// Mask channel m = k*64 + a*8 + b  (k = ky*3 + kx neighbour, (a, b) = sub-pixel row/col);
// output pixel (8y + a, 8x + b); neighbour (ky, kx) of cell (y, x) is (y+ky-1, x+kx-1), zero outside.
//
// Work split: a 256-thread workgroup owns 64 consecutive cells of one row (lane = cell, so every mask
// read is a coalesced 256-B row) and 4 groups of 16 sub-pixels.
#include "common.h"
#include "launchers.h"

namespace {

template <typename TM>
__global__ __launch_bounds__(256) void convex_up_fwd_kernel(const float* __restrict__ flow,
                                                            const TM* __restrict__ mask, int64_t mbs,
                                                            int64_t mcs, int64_t mps,
                                                            float* __restrict__ out, int H, int W) {
  const int xi = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int x = blockIdx.x * 64 + xi, y = blockIdx.y, b = blockIdx.z;
  if (x >= W) return;
  const int64_t HW = (int64_t)H * W;
  const float* F = flow + (int64_t)b * 2 * HW;
  float nf[9][2];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    nf[k][0] = ok ? 8.f * F[(int64_t)yy * W + xx] : 0.f;
    nf[k][1] = ok ? 8.f * F[HW + (int64_t)yy * W + xx] : 0.f;
  }
  const TM* M = mask + (int64_t)b * mbs + ((int64_t)y * W + x) * mps;
  float* O = out + (int64_t)b * 2 * 64 * HW;
  const int W8 = 8 * W;
  for (int s = g * 16; s < g * 16 + 16; ++s) {
    float m[9];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      m[k] = Ld<TM>::get(M, (int64_t)(k * 64 + s) * mcs);
      mx = fmaxf(mx, m[k]);
    }
    float den = 0.f, o0 = 0.f, o1 = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float e = __expf(m[k] - mx);
      den += e;
      o0 += e * nf[k][0];
      o1 += e * nf[k][1];
    }
    const float inv = 1.f / den;
    const int64_t oy = 8 * y + (s >> 3), ox = 8 * x + (s & 7);
    O[oy * W8 + ox] = o0 * inv;
    O[64 * HW + oy * W8 + ox] = o1 * inv;
  }
}

// d(mask) directly; per-cell neighbour weights Wk[k][c] = sum_s p_k(s) * dout_c(s) go to `wbuf`
// (B, 18, H, W) and are gathered into d(flow) by convex_up_bwd_flow_kernel.
template <typename TM>
__global__ __launch_bounds__(256) void convex_up_bwd_kernel(const float* __restrict__ flow,
                                                            const TM* __restrict__ mask,
                                                            int64_t mbs, int64_t mcs, int64_t mps,
                                                            const float* __restrict__ dout,
                                                            TM* __restrict__ dmask,
                                                            float* __restrict__ wbuf, int H, int W) {
  __shared__ float red[4][18][64];
  const int xi = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int x = blockIdx.x * 64 + xi, y = blockIdx.y, b = blockIdx.z;
  const bool active = x < W;
  const int64_t HW = (int64_t)H * W;
  float acc[9][2];
#pragma unroll
  for (int k = 0; k < 9; ++k) acc[k][0] = acc[k][1] = 0.f;
  if (active) {
    const float* F = flow + (int64_t)b * 2 * HW;
    float nf[9][2];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      nf[k][0] = ok ? 8.f * F[(int64_t)yy * W + xx] : 0.f;
      nf[k][1] = ok ? 8.f * F[HW + (int64_t)yy * W + xx] : 0.f;
    }
    const int64_t cell = (int64_t)y * W + x;
    const TM* M = mask + (int64_t)b * mbs + cell * mps;
    TM* DM = dmask + (int64_t)b * mbs + cell * mps;
    const float* DO = dout + (int64_t)b * 2 * 64 * HW;
    const int W8 = 8 * W;
    for (int s = g * 16; s < g * 16 + 16; ++s) {
      float m[9];
      float mx = -INFINITY;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        m[k] = Ld<TM>::get(M, (int64_t)(k * 64 + s) * mcs);
        mx = fmaxf(mx, m[k]);
      }
      float den = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        m[k] = __expf(m[k] - mx);
        den += m[k];
      }
      const float inv = 1.f / den;
      const int64_t oy = 8 * y + (s >> 3), ox = 8 * x + (s & 7);
      const float d0 = DO[oy * W8 + ox], d1 = DO[64 * HW + oy * W8 + ox];
      float gk[9], dot = 0.f;
#pragma unroll
      for (int k = 0; k < 9; ++k) {
        m[k] *= inv;  // p_k
        gk[k] = d0 * nf[k][0] + d1 * nf[k][1];
        dot += m[k] * gk[k];
        acc[k][0] += m[k] * d0;
        acc[k][1] += m[k] * d1;
      }
#pragma unroll
      for (int k = 0; k < 9; ++k)
        St<TM>::put(DM, (int64_t)(k * 64 + s) * mcs, m[k] * (gk[k] - dot));
    }
  }
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    red[g][2 * k][xi] = acc[k][0];
    red[g][2 * k + 1][xi] = acc[k][1];
  }
  __syncthreads();
  // 18 x 64 partial sums reduced over the 4 groups; 256 threads cover 4.5 rounds
  for (int e = threadIdx.x; e < 18 * 64; e += 256) {
    const int c = e >> 6, xx = e & 63;
    const int gx = blockIdx.x * 64 + xx;
    if (gx < W) {
      const float v = red[0][c][xx] + red[1][c][xx] + red[2][c][xx] + red[3][c][xx];
      wbuf[((int64_t)b * 18 + c) * HW + (int64_t)y * W + gx] = v;
    }
  }
}

__global__ __launch_bounds__(256) void convex_up_bwd_flow_kernel(const float* __restrict__ wbuf,
                                                                 float* __restrict__ dflow, int B,
                                                                 int H, int W) {
  const int64_t HW = (int64_t)H * W;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * HW) return;
  const int x = (int)(t % W), y = (int)((t / W) % H);
  const int64_t b = t / HW;
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    // the cell whose neighbour k is (y, x)
    const int cy = y - (k / 3 - 1), cx = x - (k % 3 - 1);
    if (cy >= 0 && cy < H && cx >= 0 && cx < W) {
      const int64_t o = (int64_t)cy * W + cx;
      s0 += wbuf[(b * 18 + 2 * k) * HW + o];
      s1 += wbuf[(b * 18 + 2 * k + 1) * HW + o];
    }
  }
  dflow[(b * 2) * HW + (int64_t)y * W + x] = 8.f * s0;
  dflow[(b * 2 + 1) * HW + (int64_t)y * W + x] = 8.f * s1;
}

// ---- NHWC bf16 mask (B,H,W,576) as written by the fused update block: one wave per cell,
// lane = sub-pixel s, so the 9 mask reads per lane are 9 coalesced 128-B rows.
__device__ __forceinline__ void cell_flows(const float* F, int64_t HW, int y, int x, int H, int W,
                                           float (&nf)[9][2]) {
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const int yy = y + k / 3 - 1, xx = x + k % 3 - 1;
    const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
    nf[k][0] = ok ? 8.f * F[(int64_t)yy * W + xx] : 0.f;
    nf[k][1] = ok ? 8.f * F[HW + (int64_t)yy * W + xx] : 0.f;
  }
}

// 4 consecutive mask channels of a NHWC row: bf16 (8-B access) or fp32 (16-B access; the fp32
// model's mask head writes NHWC fp32)
__device__ __forceinline__ void mask_ld4(const uint16_t* p, float (&v)[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = __uint_as_float(u.x << 16);
  v[1] = __uint_as_float(u.x & 0xffff0000u);
  v[2] = __uint_as_float(u.y << 16);
  v[3] = __uint_as_float(u.y & 0xffff0000u);
}
__device__ __forceinline__ void mask_ld4(const float* p, float (&v)[4]) {
  const float4 u = *reinterpret_cast<const float4*>(p);
  v[0] = u.x; v[1] = u.y; v[2] = u.z; v[3] = u.w;
}
__device__ __forceinline__ void mask_st4(uint16_t* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) =
      make_uint2((uint32_t)raft_f32_to_bf16(v[0]) | ((uint32_t)raft_f32_to_bf16(v[1]) << 16),
                 (uint32_t)raft_f32_to_bf16(v[2]) | ((uint32_t)raft_f32_to_bf16(v[3]) << 16));
}
__device__ __forceinline__ void mask_st4(float* p, const float (&v)[4]) {
  *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
}
// fp16 mask (fp16 autocast)
__device__ __forceinline__ void mask_ld4(const _Float16* p, float (&v)[4]) {
  const uint2 u = *reinterpret_cast<const uint2*>(p);
  v[0] = raft_h2f<true>((uint16_t)(u.x & 0xffffu));
  v[1] = raft_h2f<true>((uint16_t)(u.x >> 16));
  v[2] = raft_h2f<true>((uint16_t)(u.y & 0xffffu));
  v[3] = raft_h2f<true>((uint16_t)(u.y >> 16));
}
__device__ __forceinline__ void mask_st4(_Float16* p, const float (&v)[4]) {
  *reinterpret_cast<uint2*>(p) =
      make_uint2((uint32_t)raft_f2h<true>(v[0]) | ((uint32_t)raft_f2h<true>(v[1]) << 16),
                 (uint32_t)raft_f2h<true>(v[2]) | ((uint32_t)raft_f2h<true>(v[3]) << 16));
}

// 16 lanes per cell, 4 consecutive sub-pixels per lane (4 cells per wave): 8-B (bf16) / 16-B
// (fp32) mask reads, 16-B output stores
template <typename TM>
__global__ __launch_bounds__(256) void convex_up_nhwc_fwd_kernel(const float* __restrict__ flow,
                                                                 const TM* __restrict__ mask,
                                                                 float* __restrict__ out, int B,
                                                                 int H, int W) {
  const int q = threadIdx.x & 15;
  const int64_t cell = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t HW = (int64_t)H * W;
  if (cell >= (int64_t)B * HW) return;
  const int64_t b = cell / HW;
  const int yx = (int)(cell - b * HW), y = yx / W, x = yx % W;
  float nf[9][2];
  cell_flows(flow + b * 2 * HW, HW, y, x, H, W, nf);
  const TM* M = mask + cell * 576 + 4 * q;
  float m[9][4], mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    mask_ld4(M + k * 64, m[k]);
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = fmaxf(mx[j], m[k][j]);
  }
  float o0[4], o1[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float den = 0.f, a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float e = __expf(m[k][j] - mx[j]);
      den += e;
      a0 += e * nf[k][0];
      a1 += e * nf[k][1];
    }
    const float inv = 1.f / den;
    o0[j] = a0 * inv;
    o1[j] = a1 * inv;
  }
  const int64_t W8 = 8 * (int64_t)W;
  const int64_t o = (int64_t)(8 * y + (q >> 1)) * W8 + 8 * x + (q & 1) * 4;
  float* O = out + b * 2 * 64 * HW;
  *reinterpret_cast<float4*>(O + o) = make_float4(o0[0], o0[1], o0[2], o0[3]);
  *reinterpret_cast<float4*>(O + 64 * HW + o) = make_float4(o1[0], o1[1], o1[2], o1[3]);
}

// 16 lanes per cell, 4 consecutive sub-pixels per lane (4 cells per wave): the mask / dmask rows
// move as 8-B pieces, dout as 16-B pieces, and the 18 neighbour-weight sums are reduced over the
// lane's 4 sub-pixels in registers first, leaving 4 shuffle steps per sum (was 6 over 64 lanes).
template <typename TM>
__global__ __launch_bounds__(256) void convex_up_nhwc_bwd_kernel(const float* __restrict__ flow,
                                                                 const TM* __restrict__ mask,
                                                                 const float* __restrict__ dout,
                                                                 TM* __restrict__ dmask,
                                                                 float* __restrict__ wbuf, int B,
                                                                 int H, int W) {
  const int q = threadIdx.x & 15;
  const int64_t cell = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int64_t HW = (int64_t)H * W;
  if (cell >= (int64_t)B * HW) return;  // a 16-lane group exits together (cell is group-uniform)
  const int64_t b = cell / HW;
  const int yx = (int)(cell - b * HW), y = yx / W, x = yx % W;
  float nf[9][2];
  cell_flows(flow + b * 2 * HW, HW, y, x, H, W, nf);
  const TM* M = mask + cell * 576 + 4 * q;
  float p[9][4], mx[4] = {-INFINITY, -INFINITY, -INFINITY, -INFINITY};
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    mask_ld4(M + k * 64, p[k]);
#pragma unroll
    for (int j = 0; j < 4; ++j) mx[j] = fmaxf(mx[j], p[k][j]);
  }
  float den[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 9; ++k)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      p[k][j] = __expf(p[k][j] - mx[j]);
      den[j] += p[k][j];
    }
  const int64_t W8 = 8 * (int64_t)W;
  const int64_t o = (int64_t)(8 * y + (q >> 1)) * W8 + 8 * x + (q & 1) * 4;
  const float* DO = dout + b * 2 * 64 * HW;
  const float4 da = *reinterpret_cast<const float4*>(DO + o);
  const float4 db = *reinterpret_cast<const float4*>(DO + 64 * HW + o);
  const float d0[4] = {da.x, da.y, da.z, da.w}, d1[4] = {db.x, db.y, db.z, db.w};
  float g[9][4], dot[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const float inv = 1.f / den[j];
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      p[k][j] *= inv;
      g[k][j] = d0[j] * nf[k][0] + d1[j] * nf[k][1];
      dot[j] += p[k][j] * g[k][j];
    }
  }
  TM* DM = dmask + cell * 576 + 4 * q;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float dm[4] = {p[k][0] * (g[k][0] - dot[0]), p[k][1] * (g[k][1] - dot[1]),
                         p[k][2] * (g[k][2] - dot[2]), p[k][3] * (g[k][3] - dot[3])};
    mask_st4(DM + k * 64, dm);
  }
  // neighbour weights W[k][c] = sum_s p_k d_c: the lane's 4 sub-pixels, then its 16-lane group
  // (a DPP row) by four DPP butterfly adds -- every lane ends with the sum; 72 ds_bpermute
  // shuffles per lane before -- and lane q of the cell stores sums q and 16 + q
  float wq = 0.f, wq2 = 0.f;
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    const float w0 = raft_row16_sum((p[k][0] * d0[0] + p[k][1] * d0[1]) + (p[k][2] * d0[2] + p[k][3] * d0[3]));
    const float w1 = raft_row16_sum((p[k][0] * d1[0] + p[k][1] * d1[1]) + (p[k][2] * d1[2] + p[k][3] * d1[3]));
    wq = q == 2 * k ? w0 : (q == 2 * k + 1 ? w1 : wq);
    if (k == 8) wq2 = q == 0 ? w0 : w1;
  }
  wbuf[(b * 18 + q) * HW + yx] = wq;
  if (q < 2) wbuf[(b * 18 + 16 + q) * HW + yx] = wq2;
}

}  // namespace

bool launch_convex_up_nhwc_fwd(const float* flow, const void* mask, int mask_is_bf16, float* out,
                               int B, int H, int W, hipStream_t stream) {
  const int64_t cells = (int64_t)B * H * W;
  if (mask_is_bf16 == 2)   // mask kind: 0 fp32, 1 bf16, 2 fp16
    hipLaunchKernelGGL(convex_up_nhwc_fwd_kernel<_Float16>, dim3(raft_cdiv(cells, 16)), dim3(256), 0,
                       stream, flow, static_cast<const _Float16*>(mask), out, B, H, W);
  else if (mask_is_bf16)
    hipLaunchKernelGGL(convex_up_nhwc_fwd_kernel<uint16_t>, dim3(raft_cdiv(cells, 16)), dim3(256), 0,
                       stream, flow, static_cast<const uint16_t*>(mask), out, B, H, W);
  else
    hipLaunchKernelGGL(convex_up_nhwc_fwd_kernel<float>, dim3(raft_cdiv(cells, 16)), dim3(256), 0,
                       stream, flow, static_cast<const float*>(mask), out, B, H, W);
  return true;
}

bool launch_convex_up_nhwc_bwd(const float* flow, const void* mask, int mask_is_bf16,
                               const float* dout, void* dmask, float* wbuf, float* dflow, int B,
                               int H, int W, hipStream_t stream) {
  const int64_t cells = (int64_t)B * H * W;
  if (mask_is_bf16 == 2)
    hipLaunchKernelGGL(convex_up_nhwc_bwd_kernel<_Float16>, dim3(raft_cdiv(cells, 16)), dim3(256), 0,
                       stream, flow, static_cast<const _Float16*>(mask), dout,
                       static_cast<_Float16*>(dmask), wbuf, B, H, W);
  else if (mask_is_bf16)
    hipLaunchKernelGGL(convex_up_nhwc_bwd_kernel<uint16_t>, dim3(raft_cdiv(cells, 16)), dim3(256), 0,
                       stream, flow, static_cast<const uint16_t*>(mask), dout,
                       static_cast<uint16_t*>(dmask), wbuf, B, H, W);
  else
    hipLaunchKernelGGL(convex_up_nhwc_bwd_kernel<float>, dim3(raft_cdiv(cells, 16)), dim3(256), 0,
                       stream, flow, static_cast<const float*>(mask), dout, static_cast<float*>(dmask),
                       wbuf, B, H, W);
  hipLaunchKernelGGL(convex_up_bwd_flow_kernel, dim3(raft_cdiv(cells, 256)), dim3(256), 0, stream,
                     wbuf, dflow, B, H, W);
  return true;
}

bool launch_convex_up_fwd(const float* flow, const void* mask, int mask_is_bf16, int64_t mbs,
                          int64_t mcs, int64_t mps, float* out, int B, int H, int W,
                          hipStream_t stream) {
  dim3 grid(raft_cdiv(W, 64), H, B);
  if (mask_is_bf16)
    hipLaunchKernelGGL(convex_up_fwd_kernel<uint16_t>, grid, dim3(256), 0, stream, flow,
                       (const uint16_t*)mask, mbs, mcs, mps, out, H, W);
  else
    hipLaunchKernelGGL(convex_up_fwd_kernel<float>, grid, dim3(256), 0, stream, flow,
                       (const float*)mask, mbs, mcs, mps, out, H, W);
  return true;
}

bool launch_convex_up_bwd(const float* flow, const void* mask, int mask_is_bf16, int64_t mbs,
                          int64_t mcs, int64_t mps, const float* dout, void* dmask, float* wbuf,
                          float* dflow, int B, int H, int W, hipStream_t stream) {
  dim3 grid(raft_cdiv(W, 64), H, B);
  if (mask_is_bf16)
    hipLaunchKernelGGL(convex_up_bwd_kernel<uint16_t>, grid, dim3(256), 0, stream, flow,
                       (const uint16_t*)mask, mbs, mcs, mps, dout, (uint16_t*)dmask, wbuf, H, W);
  else
    hipLaunchKernelGGL(convex_up_bwd_kernel<float>, grid, dim3(256), 0, stream, flow,
                       (const float*)mask, mbs, mcs, mps, dout, (float*)dmask, wbuf, H, W);
  const int64_t total = (int64_t)B * H * W;
  hipLaunchKernelGGL(convex_up_bwd_flow_kernel, dim3(raft_cdiv(total, 256)), dim3(256), 0, stream,
                     wbuf, dflow, B, H, W);
  return true;
}
