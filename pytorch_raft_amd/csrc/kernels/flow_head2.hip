// flow_head.conv2 of the full update block: 3x3 conv, 256 -> 2 channels (`core/update.py:6-14`),
// forward, input gradient (fused with the head ReLU backward) and weight/bias gradient.
//
// With only two output channels this conv is not a GEMM worth MFMA tiles: through the implicit-GEMM
// kernel the N=2 output pads to a 32-wide tile and the launch is latency-bound (~28 us fwd, ~40 us
// dgrad per iteration at the chairs shape, and the padded batched wgrad ~0.4 ms per step).  Here
// each direction is one bandwidth-shaped VALU kernel over NHWC bf16 activations:
//
//   fwd    thread = (pixel, 64-channel quarter), 9 taps x 8 16-B loads, weights broadcast from LDS,
//          4-way LDS combine, fp32 NCHW delta (+bias)                                    (wave64)
//   dgrad  thread = (pixel, 8-channel group), its 144 weights held in VGPRs for the whole launch,
//          18 broadcast loads of the fp32 NCHW output gradient per pixel, ReLU gate from fm,
//          one 16-B bf16 store                                                 (adjoint, zero pad)
//   wgrad  thread = (output row, 8-channel group), a 3x3 window of 16-B input vectors slides along
//          x (3 new loads per pixel), 144 fp32 accumulators, LDS combine over the 8 row lanes,
//          one fp32 atomic per (weight, workgroup); all GRU iterations of a step in one launch.
//
// Weights: the module's fp32 (2, 256, 3, 3) tensor; weight gradient in the packed layout of the
// fused block, dw[o][tap * 256 + c] (tap = ky * 3 + kx).
#include "common.h"
#include "launchers.h"

namespace {

constexpr int FH_C = 256;

__device__ __forceinline__ void bf16x8_to_f32(const uint4 v, float (&f)[8]) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    f[2 * i] = __uint_as_float(w[i] << 16);
    f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
  }
}

// grid (ceil(W/64), H, B), block 256: lane = pixel, wave = channel quarter
__global__ __launch_bounds__(256) void fh2_fwd_kernel(const uint16_t* __restrict__ in, int cs,
                                                      const float* __restrict__ w,
                                                      const float* __restrict__ bias,
                                                      float* __restrict__ out, int H, int W) {
  __shared__ float2 wl[9 * FH_C];
  __shared__ float2 red[4][64];
  const int tid = threadIdx.x;
  for (int i = tid; i < 9 * FH_C; i += 256) {
    const int t = i / FH_C, c = i - t * FH_C;
    wl[i] = make_float2(w[c * 9 + t], w[(FH_C + c) * 9 + t]);
  }
  __syncthreads();
  const int px = tid & 63, q = tid >> 6;
  const int b = blockIdx.z, y = blockIdx.y, x = blockIdx.x * 64 + px;
  float a0 = 0.f, a1 = 0.f;
  if (x < W) {
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = y + ky - 1;
      if (yy < 0 || yy >= H) continue;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = x + kx - 1;
        if (xx < 0 || xx >= W) continue;
        const uint16_t* p = in + ((int64_t)(b * H + yy) * W + xx) * cs + q * 64;
        const float2* wt = wl + (ky * 3 + kx) * FH_C + q * 64;
        uint4 v[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const uint4*>(p + j * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          float f[8];
          bf16x8_to_f32(v[j], f);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            const float2 ww = wt[j * 8 + i];
            a0 = fmaf(f[i], ww.x, a0);
            a1 = fmaf(f[i], ww.y, a1);
          }
        }
      }
    }
  }
  red[q][px] = make_float2(a0, a1);
  __syncthreads();
  if (q == 0 && x < W) {
    const float2 r0 = red[0][px], r1 = red[1][px], r2 = red[2][px], r3 = red[3][px];
    const int64_t hw = (int64_t)H * W, o = (int64_t)y * W + x;
    out[(int64_t)b * 2 * hw + o] = ((r0.x + r1.x) + (r2.x + r3.x)) + bias[0];
    out[(int64_t)b * 2 * hw + hw + o] = ((r0.y + r1.y) + (r2.y + r3.y)) + bias[1];
  }
}

// dx[b,y,x,c] = [fm > 0] * sum_{ky,kx,o} gout[b,o,y-ky+1,x-kx+1] * W[o][c][ky][kx]
// block 256 = 8 pixel lanes x 32 channel groups; grid-stride over pixels
__global__ __launch_bounds__(256) void fh2_dgrad_kernel(const float* __restrict__ gout,
                                                        const float* __restrict__ w,
                                                        const uint16_t* __restrict__ fm, int fs,
                                                        uint16_t* __restrict__ dx, int ds, int B,
                                                        int H, int W) {
  const int g = threadIdx.x & 31, pl = threadIdx.x >> 5;
  float wr[9][2][8];
#pragma unroll
  for (int t = 0; t < 9; ++t)
#pragma unroll
    for (int o = 0; o < 2; ++o)
#pragma unroll
      for (int i = 0; i < 8; ++i) wr[t][o][i] = w[(o * FH_C + g * 8 + i) * 9 + t];
  const int64_t hw = (int64_t)H * W, P = (int64_t)B * hw;
  for (int64_t p = (int64_t)blockIdx.x * 8 + pl; p < P; p += (int64_t)gridDim.x * 8) {
    const int b = (int)(p / hw);
    const int yx = (int)(p - (int64_t)b * hw);
    const int y = yx / W, x = yx - y * W;
    const float* g0 = gout + (int64_t)b * 2 * hw;
    float s[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) s[i] = 0.f;
#pragma unroll
    for (int ky = 0; ky < 3; ++ky) {
      const int yy = y - ky + 1;
#pragma unroll
      for (int kx = 0; kx < 3; ++kx) {
        const int xx = x - kx + 1;
        const bool ok = yy >= 0 && yy < H && xx >= 0 && xx < W;
        const int64_t o = ok ? (int64_t)yy * W + xx : 0;
        const float d0 = ok ? g0[o] : 0.f, d1 = ok ? g0[hw + o] : 0.f;
#pragma unroll
        for (int i = 0; i < 8; ++i)
          s[i] = fmaf(d0, wr[ky * 3 + kx][0][i], fmaf(d1, wr[ky * 3 + kx][1][i], s[i]));
      }
    }
    const uint4 m = *reinterpret_cast<const uint4*>(fm + p * fs + g * 8);
    const uint32_t mw[4] = {m.x, m.y, m.z, m.w};
    uint32_t ov[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const bool lo = (mw[k] & 0x8000u) == 0 && (mw[k] & 0x7fffu) != 0;
      const bool hi = (mw[k] & 0x80000000u) == 0 && (mw[k] & 0x7fff0000u) != 0;
      const uint32_t a = lo ? raft_f32_to_bf16(s[2 * k]) : 0u;
      const uint32_t c = hi ? raft_f32_to_bf16(s[2 * k + 1]) : 0u;
      ov[k] = a | (c << 16);
    }
    *reinterpret_cast<uint4*>(dx + p * ds + g * 8) = make_uint4(ov[0], ov[1], ov[2], ov[3]);
  }
}

// dw[o][t*256 + c] += sum_items sum_p gout[p][o] * in[p + off_t][c];  db[o] += sum gout[p][o]
// block 256 = 8 row lanes x 32 channel groups; a unit = (item, image, 8-row block)
__global__ __launch_bounds__(256) void fh2_wgrad_kernel(Fh2Items it, int cs, int B, int H, int W,
                                                        float* __restrict__ dw,
                                                        float* __restrict__ db) {
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
    // window columns (x-1, x, x+1) of rows (y-1, y, y+1); column -1 is zero padding
    uint4 win[3][3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      win[r][0] = make_uint4(0, 0, 0, 0);
      const int yy = y + r - 1;
      win[r][1] = (yy >= 0 && yy < H) ? *reinterpret_cast<const uint4*>(in + ((int64_t)yy * W) * cs)
                                      : make_uint4(0, 0, 0, 0);
    }
    for (int x = 0; x < W; ++x) {
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int yy = y + r - 1;
        win[r][2] = (yy >= 0 && yy < H && x + 1 < W)
                        ? *reinterpret_cast<const uint4*>(in + ((int64_t)yy * W + x + 1) * cs)
                        : make_uint4(0, 0, 0, 0);
      }
      const float d0 = go[x], d1 = go[hw + x];
      bs0 += d0;
      bs1 += d1;
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          float f[8];
          bf16x8_to_f32(win[r][k], f);
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            acc[0][r * 3 + k][i] = fmaf(d0, f[i], acc[0][r * 3 + k][i]);
            acc[1][r * 3 + k][i] = fmaf(d1, f[i], acc[1][r * 3 + k][i]);
          }
        }
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        win[r][0] = win[r][1];
        win[r][1] = win[r][2];
      }
    }
  }
  // combine the 8 row lanes (fixed order), one output channel o per round
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
      atomicAdd(dw + (int64_t)o * 9 * FH_C + e, s);
    }
    __syncthreads();
  }
  if (db != nullptr && g == 0) {
    atomicAdd(db, bs0);
    atomicAdd(db + 1, bs1);
  }
}

}  // namespace

bool launch_fh2_fwd(const uint16_t* in, int cs, const float* w, const float* bias, float* out, int B,
                    int H, int W, hipStream_t stream) {
  if (cs % 8 != 0 || cs < FH_C) return false;
  dim3 grid(raft_cdiv(W, 64), H, B);
  hipLaunchKernelGGL(fh2_fwd_kernel, grid, dim3(256), 0, stream, in, cs, w, bias, out, H, W);
  return true;
}

bool launch_fh2_dgrad(const float* gout, const float* w, const uint16_t* fm, int fs, uint16_t* dx,
                      int ds, int B, int H, int W, hipStream_t stream) {
  if (fs % 8 != 0 || ds % 8 != 0 || fs < FH_C || ds < FH_C) return false;
  const int64_t P = (int64_t)B * H * W;
  // ~4 pixels per pixel lane: weights are loaded once per thread, so keep blocks few but >= 2/CU
  const int64_t blocks = std::max<int64_t>(512, std::min<int64_t>((P + 31) / 32, 2048));
  hipLaunchKernelGGL(fh2_dgrad_kernel, dim3((unsigned)blocks), dim3(256), 0, stream, gout, w, fm, fs,
                     dx, ds, B, H, W);
  return true;
}

bool launch_fh2_wgrad(const Fh2Items& it, int cs, int B, int H, int W, float* dw, float* db,
                      hipStream_t stream) {
  if (it.n < 1 || it.n > RAFT_FH2_MAX_ITEMS || cs % 8 != 0 || cs < FH_C) return false;
  const int units = it.n * B * ((H + 7) / 8);
  // ~2 workgroups per CU: each adds its 4608 partial sums with one fp32 atomic apiece
  const int blocks = std::min(units, 512);
  hipLaunchKernelGGL(fh2_wgrad_kernel, dim3(blocks), dim3(256), 0, stream, it, cs, B, H, W, dw, db);
  return true;
}
