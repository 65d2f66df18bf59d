// flow_head.conv2 of the full update block: 3x3 conv, 256 -> 2 channels (`core/update.py:6-14`),
// forward, input gradient (fused with the head ReLU backward) and weight/bias gradient.
//
// With only two output channels this conv is not a GEMM worth MFMA tiles: through the implicit-GEMM
// kernel the N=2 output pads to a 32-wide tile and the launch is latency-bound (~28 us fwd, ~40 us
// dgrad per iteration at the chairs shape, and the padded batched wgrad ~0.4 ms per step).  Here
// each direction is one bandwidth-shaped VALU kernel over NHWC bf16 activations:
//
//   fwd    thread = (pixel, 8-channel group): 9 coalesced 16-B loads, 72 v_dot2_f32_bf16 against
//          bf16-pair weights staged once per block in LDS, 32-lane shuffle reduction, fp32 NCHW
//          delta (+bias)
//   dgrad  thread = (pixel, 8-channel group): the two output-gradient channels of each tap form a
//          bf16 pair, dot2 against (W0[c], W1[c]) pairs from LDS, ReLU gate from fm, one 16-B
//          bf16 store                                                          (adjoint, zero pad)
//   wgrad  thread = (output row, 8-channel group), a 3x4 window of 16-B input vectors slides along
//          x in blocks of 2 pixels (6 loads in flight per block), 144 fp32 accumulators, LDS
//          combine over the 8 row lanes, one partial row per workgroup (summed by the caller);
//          all GRU iterations of a step in one launch.
//
// Weights: the module's fp32 (2, 256, 3, 3) tensor; weight gradient in the packed layout of the
// fused block, dw[o][tap * 256 + c] (tap = ky * 3 + kx).
#include "common.h"
#include "launchers.h"

#include <cstdlib>

namespace {

constexpr int FH_C = 256;

// 16-bit operand helpers: bf16 (F16 = false) or fp16 (fp16 autocast: v_dot2_f32_f16)
template <bool F16>
__device__ __forceinline__ void bf16x8_to_f32(const uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = raft_h2f<F16>((uint16_t)(w[i] & 0xffffu));
    f[2 * i + 1] = raft_h2f<F16>((uint16_t)(w[i] >> 16));
  }
}

typedef __bf16 __attribute__((ext_vector_type(2))) bf16x2_t;
typedef _Float16 __attribute__((ext_vector_type(2))) f16x2_t;

template <bool F16>
__device__ __forceinline__ uint32_t pack_bf2(float lo, float hi) {
  return (uint32_t)raft_f2h<F16>(lo) | ((uint32_t)raft_f2h<F16>(hi) << 16);
}
template <bool F16>
__device__ __forceinline__ float dot2(uint32_t a, uint32_t b, float c) {
  if constexpr (F16)
    return __builtin_amdgcn_fdot2(__builtin_bit_cast(f16x2_t, a), __builtin_bit_cast(f16x2_t, b), c, false);
  else
    return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2_t, a), __builtin_bit_cast(bf16x2_t, b),
                                           c, false);
}

// out[b,o,y,x] = bias[o] + sum_{t,c} in[b, y+ky-1, x+kx-1, c] * W[o][c][t]
// thread = (NPIX pixels, 8-channel group = 4 bf16 pairs); block 256 = 8 x NPIX pixels.  No loop:
// every load (weights once, then all pixels' taps) is issued before the first use, so the launch
// costs one memory round trip; NPIX > 1 divides the weight-table re-reads.  wf: bf16 pairs
// [t][o][c/2] from the packing gather; products by v_dot2_f32_bf16; 32-lane shuffle reduction.
template <int NPIX, bool F16>
__global__ __launch_bounds__(256) void fh2_fwd_kernel(const uint16_t* __restrict__ in, int cs,
                                                      const uint32_t* __restrict__ wf,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ out, int B, int H,
                                                      int W, const float* __restrict__ coords,
                                                      float* __restrict__ cnew,
                                                      float* __restrict__ fnew) {
  const int g = threadIdx.x & 31;
  const int64_t hw = (int64_t)H * W, P = (int64_t)B * hw;
  uint4 w0[9], w1[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {
    w0[t] = *reinterpret_cast<const uint4*>(wf + (t * 2 + 0) * 128 + g * 4);
    w1[t] = *reinterpret_cast<const uint4*>(wf + (t * 2 + 1) * 128 + g * 4);
  }
  uint4 v[NPIX][9];
#pragma unroll
  for (int k = 0; k < NPIX; ++k) {
    const int64_t p = ((int64_t)blockIdx.x * NPIX + k) * 8 + (threadIdx.x >> 5);
    const int64_t pc = min(p, P - 1);
    const int b = (int)(pc / hw);
    const int yx = (int)(pc - (int64_t)b * hw);
    const int y = yx / W, x = yx - y * W;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int yy = y + t / 3 - 1, xx = x + t % 3 - 1;
      const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
      v[k][t] = ok ? *reinterpret_cast<const uint4*>(in + ((int64_t)(b * H + yy) * W + xx) * cs + g * 8)
                   : make_uint4(0, 0, 0, 0);
    }
  }
#pragma unroll
  for (int k = 0; k < NPIX; ++k) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      a0 = dot2<F16>(v[k][t].x, w0[t].x, a0);
      a1 = dot2<F16>(v[k][t].x, w1[t].x, a1);
      a2 = dot2<F16>(v[k][t].y, w0[t].y, a2);
      a3 = dot2<F16>(v[k][t].y, w1[t].y, a3);
      a0 = dot2<F16>(v[k][t].z, w0[t].z, a0);
      a1 = dot2<F16>(v[k][t].z, w1[t].z, a1);
      a2 = dot2<F16>(v[k][t].w, w0[t].w, a2);
      a3 = dot2<F16>(v[k][t].w, w1[t].w, a3);
    }
    float s0 = a0 + a2, s1 = a1 + a3;
#pragma unroll
    for (int m = 16; m > 0; m >>= 1) {
      s0 += __shfl_xor(s0, m, 32);
      s1 += __shfl_xor(s1, m, 32);
    }
    const int64_t p = ((int64_t)blockIdx.x * NPIX + k) * 8 + (threadIdx.x >> 5);
    if (g == 0 && p < P) {
      const int64_t b = p / hw, yx = p - b * hw;
      const float d0 = s0 + bias[0], d1 = s1 + bias[1];
      out[b * 2 * hw + yx] = d0;
      out[b * 2 * hw + hw + yx] = d1;
      if (coords) {
        // coords1 + delta and (coords1 + delta) - coords0 of `core/raft.py:134-135`, with
        // coords0 = (x, y) the pixel grid: the same two fp32 roundings as the eager ops
        const int y = (int)(yx / W), x = (int)(yx - (int64_t)y * W);
        const float c0 = coords[b * 2 * hw + yx] + d0, c1 = coords[b * 2 * hw + hw + yx] + d1;
        cnew[b * 2 * hw + yx] = c0;
        cnew[b * 2 * hw + hw + yx] = c1;
        fnew[b * 2 * hw + yx] = c0 - (float)x;
        fnew[b * 2 * hw + hw + yx] = c1 - (float)y;
      }
    }
  }
}

// dx[b,y,x,c] = [fm > 0] * sum_{ky,kx,o} gout[b,o,y-ky+1,x-kx+1] * W[o][c][ky][kx]
// Per channel the two output channels form one 16-bit pair: s[c] += dot2((g0, g1), (W0[c], W1[c])),
// wd: pairs [t][c] from the packing gather.  A workgroup owns a 4 x 16 pixel tile; the tile's
// 6 x 18 halo of the two fp32 output-gradient planes is staged once in LDS as 16-bit pairs, so a
// tap is one broadcast LDS read instead of two scattered global loads per lane (a per-pixel
// gather version was ~4x slower than its bytes: 72 gathers per thread).
// thread = 8-channel group (tid & 31) x 8 of the tile's pixels.
constexpr int DTH = 4, DTW = 16;
template <bool F16>
__global__ __launch_bounds__(256) void fh2_dgrad_tile_kernel(const float* __restrict__ gout,
                                                             const uint32_t* __restrict__ wd,
                                                             const uint16_t* __restrict__ fm, int fs,
                                                             uint16_t* __restrict__ dx, int ds, int B,
                                                             int H, int W, int tiles_y, int tiles_x) {
  constexpr int HH = DTH + 2, HW_ = DTW + 2;
  __shared__ uint32_t gp[HH * HW_];
  const int g = threadIdx.x & 31;
  int t = blockIdx.x;
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int b = t / tiles_y;
  const int y0 = ty * DTH, x0 = tx * DTW;
  const int64_t hw = (int64_t)H * W;
  const float* g0 = gout + (int64_t)b * 2 * hw;
  for (int e = threadIdx.x; e < HH * HW_; e += 256) {
    const int yy = y0 - 1 + e / HW_, xx = x0 - 1 + e % HW_;
    uint32_t v = 0u;
    if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
      const int64_t o = (int64_t)yy * W + xx;
      v = pack_bf2<F16>(g0[o], g0[hw + o]);
    }
    gp[e] = v;
  }
  uint4 wa[9], wb[9];
#pragma unroll
  for (int k = 0; k < 9; ++k) {
    wa[k] = *reinterpret_cast<const uint4*>(wd + k * FH_C + g * 8);
    wb[k] = *reinterpret_cast<const uint4*>(wd + k * FH_C + g * 8 + 4);
  }
  constexpr int NP = DTH * DTW / 8;  // pixels per thread
  uint4 m[NP];
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int p = (threadIdx.x >> 5) + 8 * k;
    const int yy = y0 + p / DTW, xx = x0 + p % DTW;
    m[k] = (yy < H && xx < W)
               ? *reinterpret_cast<const uint4*>(fm + (((int64_t)b * H + yy) * W + xx) * fs + g * 8)
               : make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < NP; ++k) {
    const int p = (threadIdx.x >> 5) + 8 * k;
    const int py = p / DTW, px = p % DTW;
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = 0.f;
#pragma unroll
    for (int tap = 0; tap < 9; ++tap) {
      // tap (ky, kx) of the adjoint: gout at (y - ky + 1, x - kx + 1) = halo (py + 2 - ky, px + 2 - kx)
      const uint32_t gv = gp[(py + 2 - tap / 3) * HW_ + px + 2 - tap % 3];
      const uint32_t wv[8] = {wa[tap].x, wa[tap].y, wa[tap].z, wa[tap].w,
                              wb[tap].x, wb[tap].y, wb[tap].z, wb[tap].w};
#pragma unroll
      for (int i = 0; i < 8; ++i) s[i] = dot2<F16>(gv, wv[i], s[i]);
    }
    const uint32_t mw[4] = {m[k].x, m[k].y, m[k].z, m[k].w};
    uint32_t ov[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const bool lo = (mw[q] & 0x8000u) == 0 && (mw[q] & 0x7fffu) != 0;
      const bool hi = (mw[q] & 0x80000000u) == 0 && (mw[q] & 0x7fff0000u) != 0;
      const uint32_t a = lo ? raft_f2h<F16>(s[2 * q]) : 0u;
      const uint32_t c = hi ? raft_f2h<F16>(s[2 * q + 1]) : 0u;
      ov[q] = a | (c << 16);
    }
    const int yy = y0 + py, xx = x0 + px;
    if (yy < H && xx < W)
      *reinterpret_cast<uint4*>(dx + (((int64_t)b * H + yy) * W + xx) * ds + g * 8) =
          make_uint4(ov[0], ov[1], ov[2], ov[3]);
  }
}

// dw[o][t*256 + c] += sum_items sum_p gout[p][o] * in[p + off_t][c];  db[o] += sum gout[p][o]
// block 256 = 8 row lanes x 32 channel groups; a unit = (item, image, 8-row block)
template <bool F16>
__global__ __launch_bounds__(256) void fh2_wgrad_kernel(Fh2Items it, int cs, int B, int H, int W,
                                                        float* __restrict__ part) {
  __shared__ float red[8 * 32 * 73];  // 72 accumulators (+1 pad) per thread, one half at a time
  const int g = threadIdx.x & 31, rl = threadIdx.x >> 5;
  const int yblocks = (H + 7) / 8;
  const int units = it.n * B * yblocks;
  float acc[2][9][8];
#pragma unroll
  for (int o = 0; o < 2; ++o)
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[o][t][i] = 0.f;
  float bs0 = 0.f, bs1 = 0.f;
  const int64_t hw = (int64_t)H * W;
  for (int u = blockIdx.x; u < units; u += gridDim.x) {
    const int item = u / (B * yblocks);
    const int rem = u - item * B * yblocks;
    const int b = rem / yblocks, y = (rem - b * yblocks) * 8 + rl;
    if (y >= H) continue;
    const uint16_t* in = it.in[item] + (int64_t)b * hw * cs + g * 8;
    const float* go = it.gout[item] + (int64_t)b * 2 * hw + (int64_t)y * W;
    // window columns (xb-1 .. xb+XB) of rows (y-1, y, y+1) for a block of XB output pixels: the
    // 3*XB loads of a block's new columns are issued together (one round trip per XB pixels)
    constexpr int XB = 2;
    uint4 win[3][XB + 2];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      win[r][0] = make_uint4(0, 0, 0, 0);  // column -1: zero padding
      const int yy = y + r - 1;
      win[r][1] = (yy >= 0 && yy < H) ? *reinterpret_cast<const uint4*>(in + ((int64_t)yy * W) * cs)
                                      : make_uint4(0, 0, 0, 0);
    }
    for (int xb = 0; xb < W; xb += XB) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int yy = y + r - 1;
#pragma unroll
        for (int j = 0; j < XB; ++j) {
          const int xx = xb + 1 + j;
          win[r][2 + j] = (yy >= 0 && yy < H && xx < W)
                              ? *reinterpret_cast<const uint4*>(in + ((int64_t)yy * W + xx) * cs)
                              : make_uint4(0, 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < XB; ++j) {
        const int x = xb + j;
        const bool ok = x < W;
        const float d0 = ok ? go[x] : 0.f, d1 = ok ? go[hw + x] : 0.f;
        bs0 += d0;
        bs1 += d1;
#pragma unroll
        for (int r = 0; r < 3; ++r)
#pragma unroll
          for (int k = 0; k < 3; ++k) {
            float f[8];
            bf16x8_to_f32<F16>(win[r][j + k], f);
#pragma unroll
            for (int i = 0; i < 8; ++i) {
              acc[0][r * 3 + k][i] = fmaf(d0, f[i], acc[0][r * 3 + k][i]);
              acc[1][r * 3 + k][i] = fmaf(d1, f[i], acc[1][r * 3 + k][i]);
            }
          }
      }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        win[r][0] = win[r][XB];
        win[r][1] = win[r][XB + 1];
      }
    }
  }
  // combine the 8 row lanes (fixed order), one output channel o per round; each block writes its
  // own partial row (summed over blocks by the caller: deterministic, no same-address atomics)
  float* prow = part + (int64_t)blockIdx.x * (2 * 9 * FH_C + 2);
#pragma unroll
  for (int o = 0; o < 2; ++o) {
    float* mine = red + (rl * 32 + g) * 73;
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int i = 0; i < 8; ++i) mine[t * 8 + i] = acc[o][t][i];
    __syncthreads();
    // 2304 (t, c) sums of this o over 256 threads: 9 each
    for (int e = threadIdx.x; e < 9 * FH_C; e += 256) {
      const int t = e / FH_C, c = e - t * FH_C;
      const int gg = c >> 3, i = c & 7;
      float s = 0.f;
#pragma unroll
      for (int l = 0; l < 8; ++l) s += red[(l * 32 + gg) * 73 + t * 8 + i];
      prow[o * 9 * FH_C + e] = s;
    }
    __syncthreads();
  }
  // bias sums: every (row lane, group 0) thread holds one row's; combine the 8 in LDS
  if (g == 0) {
    red[rl * 2] = bs0;
    red[rl * 2 + 1] = bs1;
  }
  __syncthreads();
  if (threadIdx.x < 2) {
    float s = 0.f;
#pragma unroll
    for (int l = 0; l < 8; ++l) s += red[l * 2 + threadIdx.x];
    prow[2 * 9 * FH_C + threadIdx.x] = s;
  }
}

}  // namespace

bool launch_fh2_fwd(const uint16_t* in, int cs, const uint32_t* wf, const float* bias, float* out,
                    int B, int H, int W, int f16, hipStream_t stream, const float* coords,
                    float* cnew, float* fnew) {
  if (cs % 8 != 0 || cs < FH_C) return false;
  const int64_t P = (int64_t)B * H * W;
  if (f16)
    hipLaunchKernelGGL((fh2_fwd_kernel<2, true>), dim3(raft_cdiv(P, 16)), dim3(256), 0, stream, in, cs, wf,
                       bias, out, B, H, W, coords, cnew, fnew);
  else
    hipLaunchKernelGGL((fh2_fwd_kernel<2, false>), dim3(raft_cdiv(P, 16)), dim3(256), 0, stream, in, cs, wf,
                       bias, out, B, H, W, coords, cnew, fnew);
  return true;
}

bool launch_fh2_dgrad(const float* gout, const uint32_t* wd, const uint16_t* fm, int fs, uint16_t* dx,
                      int ds, int B, int H, int W, int f16, hipStream_t stream) {
  if (fs % 8 != 0 || ds % 8 != 0 || fs < FH_C || ds < FH_C) return false;
  const int ty = (H + DTH - 1) / DTH, tx = (W + DTW - 1) / DTW;
  if (f16)
    hipLaunchKernelGGL(fh2_dgrad_tile_kernel<true>, dim3((unsigned)(B * ty * tx)), dim3(256), 0, stream,
                       gout, wd, fm, fs, dx, ds, B, H, W, ty, tx);
  else
    hipLaunchKernelGGL(fh2_dgrad_tile_kernel<false>, dim3((unsigned)(B * ty * tx)), dim3(256), 0, stream,
                       gout, wd, fm, fs, dx, ds, B, H, W, ty, tx);
  return true;
}

int fh2_wgrad_units(int n, int B, int H) { return n * B * ((H + 7) / 8); }

bool launch_fh2_wgrad(const Fh2Items& it, int cs, int B, int H, int W, float* part, int blocks,
                      int f16, hipStream_t stream) {
  if (it.n < 1 || it.n > RAFT_FH2_MAX_ITEMS || cs % 8 != 0 || cs < FH_C || blocks < 1) return false;
  if (f16)
    hipLaunchKernelGGL(fh2_wgrad_kernel<true>, dim3(blocks), dim3(256), 0, stream, it, cs, B, H, W, part);
  else
    hipLaunchKernelGGL(fh2_wgrad_kernel<false>, dim3(blocks), dim3(256), 0, stream, it, cs, B, H, W, part);
  return true;
}
