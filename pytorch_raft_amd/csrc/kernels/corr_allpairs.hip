// All-pairs correlation pyramid on MI355X (gfx950).
//
// Replaces the reference's `torch.matmul(fmap1^T, fmap2) / sqrt(C)` + 3x `F.avg_pool2d(2,2)`
// (`core/corr.py:19-27,52-60`) with ONE kernel: an fp32-in / fp32-accumulate MFMA GEMM
// (v_mfma_f32_32x32x2_f32 -- exact f32, the reference runs the correlation in fp32 outside autocast)
// whose epilogue writes level 0 and the three average-pooled levels straight from LDS.
//
// Tiling: a workgroup (4 waves, 2x2 of 32x32 MFMA tiles) owns 64 query pixels i x an 8x8 spatial
// block of target pixels j.  Because the j-block is 8-aligned on the fmap2 grid, every pooled cell of
// levels 1..3 (2x2, 4x4, 8x8 L0 footprints, floor semantics for odd sizes) lies inside one block, so
// the pyramid never round-trips through HBM.  K = C is staged through LDS 32 channels at a time with
// the next chunk's global loads issued before the current chunk's MFMAs (register-staged pipeline).
//
// Backward pieces (`corr_pyr_grad_reduce`): the lookup backward accumulates into a persistent
// pyramid-gradient buffer across all GRU iterations (see corr_lookup.hip); one pass then folds the
// coarse levels back onto level 0 (avg-pool adjoint) and applies 1/sqrt(C).
#include "common.h"
#include "launchers.h"

#include <type_traits>

namespace {

constexpr int BI = 64;   // query pixels per workgroup
constexpr int TJ = 8;    // target block is TJ x TJ on the fmap2 grid
constexpr int BJ = TJ * TJ;
constexpr int KC = 32;   // channels per LDS stage
constexpr int NT = 256;  // threads

__device__ __forceinline__ void pyr_st(float* p, float v) { *p = v; }
__device__ __forceinline__ void pyr_st(uint16_t* p, float v) { *p = raft_f32_to_bf16(v); }

struct Pyr4 {
  float* lvl[4];
  int h[4];
  int w[4];
};

__global__ __launch_bounds__(NT) void corr_build_kernel(const float* __restrict__ f1,
                                                        const float* __restrict__ f2, Pyr4 out,
                                                        int C, int H, int W, int levels,
                                                        float sqrt_c, int tiles_x, int tiles_j) {
  __shared__ float As[KC][BI];
  __shared__ float Bs[KC][BJ];
  __shared__ float Cs[BI][BJ + 1];
  __shared__ float P1[BI][16];
  __shared__ float P2[BI][4];

  const int N = H * W;
  const int b = blockIdx.y;
  const int tile = blockIdx.x;
  const int jt = tile % tiles_j;
  const int it = tile / tiles_j;
  const int i0 = it * BI;
  const int y0 = (jt / tiles_x) * TJ;
  const int x0 = (jt % tiles_x) * TJ;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wr = wave >> 1, wc = wave & 1;

  const float* A = f1 + (int64_t)b * C * N;
  const float* Bm = f2 + (int64_t)b * C * N;

  // each thread stages 8 A and 8 B elements per chunk
  float ra[8], rb[8];
  auto load_chunk = [&](int k0) {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      int e = tid + NT * m;
      int k = e >> 6, jj = e & 63;
      int kk = k0 + k;
      int i = i0 + jj;
      ra[m] = (kk < C && i < N) ? A[(int64_t)kk * N + i] : 0.f;
      int y = y0 + (jj >> 3), x = x0 + (jj & 7);
      rb[m] = (kk < C && y < H && x < W) ? Bm[(int64_t)kk * N + y * W + x] : 0.f;
    }
  };
  auto store_chunk = [&]() {
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      int e = tid + NT * m;
      As[e >> 6][e & 63] = ra[m];
      Bs[e >> 6][e & 63] = rb[m];
    }
  };

  f32x16 acc;
#pragma unroll
  for (int r = 0; r < 16; ++r) acc[r] = 0.f;

  load_chunk(0);
  for (int k0 = 0; k0 < C; k0 += KC) {
    store_chunk();
    __syncthreads();
    if (k0 + KC < C) load_chunk(k0 + KC);  // in flight while the MFMAs below run
#pragma unroll
    for (int kk = 0; kk < KC / 2; ++kk) {
      float a = As[2 * kk + (lane >> 5)][wr * 32 + (lane & 31)];
      float bb = Bs[2 * kk + (lane >> 5)][wc * 32 + (lane & 31)];
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bb, acc, 0, 0, 0);
    }
    __syncthreads();
  }

  // accumulator -> LDS (C/D map: col = lane&31, row = (r&3) + 8*(r>>2) + 4*(lane>>5))
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    int row = wr * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    int col = wc * 32 + (lane & 31);
    Cs[row][col] = acc[r] / sqrt_c;
  }
  __syncthreads();

  // level 0
  {
    float* L0 = out.lvl[0];
    for (int e = tid; e < BI * BJ; e += NT) {
      int ii = e >> 6, jj = e & 63;
      int i = i0 + ii, y = y0 + (jj >> 3), x = x0 + (jj & 7);
      if (i < N && y < H && x < W) L0[(((int64_t)b * N + i) * H + y) * W + x] = Cs[ii][jj];
    }
  }
  if (levels > 1) {
    float* L1 = out.lvl[1];
    const int h1 = out.h[1], w1 = out.w[1];
    for (int e = tid; e < BI * 16; e += NT) {
      int ii = e >> 4, c = e & 15;
      int cy = c >> 2, cx = c & 3;
      const float* row0 = &Cs[ii][(2 * cy) * TJ + 2 * cx];
      const float* row1 = row0 + TJ;
      float v = (((row0[0] + row0[1]) + row1[0]) + row1[1]) * 0.25f;
      P1[ii][c] = v;
      int i = i0 + ii, Y = (y0 >> 1) + cy, X = (x0 >> 1) + cx;
      if (i < N && Y < h1 && X < w1) L1[(((int64_t)b * N + i) * h1 + Y) * w1 + X] = v;
    }
  }
  __syncthreads();
  if (levels > 2) {
    float* L2 = out.lvl[2];
    const int h2 = out.h[2], w2 = out.w[2];
    for (int e = tid; e < BI * 4; e += NT) {
      int ii = e >> 2, c = e & 3;
      int cy = c >> 1, cx = c & 1;
      const float* row0 = &P1[ii][(2 * cy) * 4 + 2 * cx];
      const float* row1 = row0 + 4;
      float v = (((row0[0] + row0[1]) + row1[0]) + row1[1]) * 0.25f;
      P2[ii][c] = v;
      int i = i0 + ii, Y = (y0 >> 2) + cy, X = (x0 >> 2) + cx;
      if (i < N && Y < h2 && X < w2) pyr_st(&L2[(((int64_t)b * N + i) * h2 + Y) * w2 + X], v);
    }
  }
  __syncthreads();
  if (levels > 3) {
    float* L3 = out.lvl[3];
    const int h3 = out.h[3], w3 = out.w[3];
    for (int ii = tid; ii < BI; ii += NT) {
      float v = (((P2[ii][0] + P2[ii][1]) + P2[ii][2]) + P2[ii][3]) * 0.25f;
      int i = i0 + ii, Y = y0 >> 3, X = x0 >> 3;
      if (i < N && Y < h3 && X < w3) pyr_st(&L3[(((int64_t)b * N + i) * h3 + Y) * w3 + X], v);
    }
  }
}

// ------------------------------------------------------------------ bf16 NHWC variant
// Mixed precision: the fmaps are the encoders' bf16 outputs, so a bf16 MFMA with fp32 accumulation
// (v_mfma_f32_32x32x16_bf16, 16x the f32-MFMA rate) forms exactly the products the reference's fp32
// matmul forms from them; only the summation order differs.  Both operands are channel-contiguous
// (NHWC), which is exactly the MFMA fragment layout (8 consecutive K values per lane): fragments go
// global -> registers as 16-B loads (L2-resident fmaps), no LDS staging.
//
// Tile: 64 query pixels i x one 8-row x 64-column band of target pixels j.  Wave w owns target rows
// y0+2w, y0+2w+1 (2 i-tiles x 4 j-tiles of 32x32).  The band is 8-row / 64-column aligned, so:
//   level 0 -> stored from the accumulators (32 lanes = 32 consecutive x: 128-B row segments);
//   level 1 -> the wave's own two rows summed in registers + the neighbour lane (x pair);
//   levels 2, 3 -> from a 32 KB LDS image of level 1.
// Floor pooling for odd sizes holds: a level-l cell is written only if it is inside the level-l map,
// and every such cell's footprint is inside level 0 (h_l = floor(h_{l-1} / 2)).
constexpr int BB_I = 64, BB_Y = 8, BB_X = 64;

// pyramid element type: fp32, or bf16 for the NHWC lookup of the fused update block (half the
// bytes of the ~0.5 GB volume the per-iteration window gathers read at chairs / B = 12)
template <typename T>
struct PyrO {
  T* lvl[4];
  int h[4];
  int w[4];
};

template <typename OutT>
__global__ __launch_bounds__(256, 2) void corr_build_bf16_kernel(const uint16_t* __restrict__ f1,
                                                                 const uint16_t* __restrict__ f2,
                                                                 PyrO<OutT> out, int C, int H, int W,
                                                                 int levels, float scale,
                                                                 int tiles_i, int bands_y,
                                                                 int tiles_x) {
  __shared__ float P1[BB_I][4][32 + 1];
  __shared__ float P2[BB_I][2][16 + 1];

  const int N = H * W;
  const int b = blockIdx.y;
  int t = blockIdx.x;
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int by = t % bands_y;
  const int ti0 = t / bands_y;
  const int i0 = ti0 * BB_I, y0 = by * BB_Y, x0 = tx * BB_X;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int l32 = lane & 31, kh = (lane >> 5) * 8;

  // fragment row pointers (element offsets); out-of-range rows read a valid row, masked to zero
  const uint16_t* arow[2];
  bool aok[2];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    const int i = i0 + 32 * a + l32;
    aok[a] = i < N;
    arow[a] = f1 + ((int64_t)b * N + (aok[a] ? i : 0)) * C + kh;
  }
  const uint16_t* brow[4];
  bool bok[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int y = y0 + 2 * wave + (j >> 1), x = x0 + 32 * (j & 1) + l32;
    bok[j] = y < H && x < W;
    brow[j] = f2 + ((int64_t)b * N + (bok[j] ? y * W + x : 0)) * C + kh;
  }

  f32x16 acc[2][4];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[a][j][r] = 0.f;

  const bf16x8 zero = {0, 0, 0, 0, 0, 0, 0, 0};
  bf16x8 fa[2][2], fb[2][4];
  auto load = [&](int k, int s) {
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      fa[s][a] = *reinterpret_cast<const bf16x8*>(arow[a] + k);
      if (!aok[a]) fa[s][a] = zero;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      fb[s][j] = *reinterpret_cast<const bf16x8*>(brow[j] + k);
      if (!bok[j]) fb[s][j] = zero;
    }
  };
  load(0, 0);
  const int ksteps = C / 16;
  for (int kk = 0; kk < ksteps; kk += 2) {
    if (kk + 1 < ksteps) load((kk + 1) * 16, 1);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[0][a], fb[0][j], acc[a][j], 0, 0, 0);
    if (kk + 1 >= ksteps) break;
    if (kk + 2 < ksteps) load((kk + 2) * 16, 0);
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        acc[a][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[1][a], fb[1][j], acc[a][j], 0, 0, 0);
  }

  // ---- level 0 straight from the accumulators; level 1 from the wave's row pair
  OutT* L0 = out.lvl[0];
  const int h1 = out.h[1], w1 = out.w[1];
  OutT* L1 = out.lvl[1];
#pragma unroll
  for (int a = 0; a < 2; ++a) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int il = 32 * a + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int i = i0 + il;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int y = y0 + 2 * wave + (j >> 1), x = x0 + 32 * (j & 1) + l32;
        if (i < N && y < H && x < W) pyr_st(&L0[(((int64_t)b * N + i) * H + y) * W + x], acc[a][j][r] * scale);
      }
      if (levels > 1) {
#pragma unroll
        for (int xh = 0; xh < 2; ++xh) {
          const float top = acc[a][xh][r] * scale, bot = acc[a][2 + xh][r] * scale;
          // ((y,x) + (y,x+1)) + ((y+1,x) + (y+1,x+1)), as avg_pool2d sums a 2x2 window
          const float rt = top + __shfl_xor(top, 1, 64);
          const float rb = bot + __shfl_xor(bot, 1, 64);
          const float v = (rt + rb) * 0.25f;
          if (!(l32 & 1)) {
            const int Xl = 16 * xh + (l32 >> 1);
            const int Y = (y0 >> 1) + wave, X = (x0 >> 1) + Xl;
            P1[il][wave][Xl] = v;
            if (i < N && Y < h1 && X < w1) pyr_st(&L1[(((int64_t)b * N + i) * h1 + Y) * w1 + X], v);
          }
        }
      }
    }
  }
  if (levels <= 2) return;  // uniform
  __syncthreads();
  {
    OutT* L2 = out.lvl[2];
    const int h2 = out.h[2], w2 = out.w[2];
    for (int e = threadIdx.x; e < BB_I * 2 * 16; e += 256) {
      const int il = e >> 5, c = e & 31;
      const int Yl = c >> 4, Xl = c & 15;
      const float* r0 = &P1[il][2 * Yl][2 * Xl];
      const float* r1 = &P1[il][2 * Yl + 1][2 * Xl];
      const float v = ((r0[0] + r0[1]) + (r1[0] + r1[1])) * 0.25f;
      P2[il][Yl][Xl] = v;
      const int i = i0 + il, Y = (y0 >> 2) + Yl, X = (x0 >> 2) + Xl;
      if (i < N && Y < h2 && X < w2) pyr_st(&L2[(((int64_t)b * N + i) * h2 + Y) * w2 + X], v);
    }
  }
  __syncthreads();
  if (levels > 3) {
    OutT* L3 = out.lvl[3];
    const int h3 = out.h[3], w3 = out.w[3];
    for (int e = threadIdx.x; e < BB_I * 8; e += 256) {
      const int il = e >> 3, Xl = e & 7;
      const float v = ((P2[il][0][2 * Xl] + P2[il][0][2 * Xl + 1]) +
                       (P2[il][1][2 * Xl] + P2[il][1][2 * Xl + 1])) * 0.25f;
      const int i = i0 + il, Y = y0 >> 3, X = (x0 >> 3) + Xl;
      if (i < N && Y < h3 && X < w3) pyr_st(&L3[(((int64_t)b * N + i) * h3 + Y) * w3 + X], v);
    }
  }
}

// dL0 = (G0 + 1/4 up(G1) + 1/16 up(G2) + 1/64 up(G3)) / sqrt(C)   (avg-pool adjoint chain)
__global__ __launch_bounds__(256) void corr_pyr_grad_reduce_kernel(Pyr4 g, float* __restrict__ out,
                                                                   int64_t planes, int levels,
                                                                   float inv_sqrt_c) {
  const int H = g.h[0], W = g.w[0];
  const int64_t total = planes * H * W;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
       t += (int64_t)gridDim.x * blockDim.x) {
    int x = (int)(t % W);
    int y = (int)((t / W) % H);
    int64_t p = t / ((int64_t)H * W);
    float v = g.lvl[0][t];
    float s = 0.25f;
    for (int l = 1; l < levels; ++l) {
      int yl = y >> l, xl = x >> l;
      if (yl < g.h[l] && xl < g.w[l]) v += s * g.lvl[l][(p * g.h[l] + yl) * g.w[l] + xl];
      s *= 0.25f;
    }
    out[t] = v * inv_sqrt_c;
  }
}

}  // namespace

void launch_corr_build(const float* f1, const float* f2, float* const* lvl, const int* hs,
                       const int* ws, int B, int C, int H, int W, int levels, hipStream_t stream) {
  Pyr4 p;
  for (int l = 0; l < 4; ++l) {
    p.lvl[l] = l < levels ? lvl[l] : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
  }
  const int N = H * W;
  const int tiles_x = (int)raft_cdiv(W, TJ), tiles_y = (int)raft_cdiv(H, TJ);
  const int tiles_j = tiles_x * tiles_y;
  const int tiles_i = (int)raft_cdiv(N, BI);
  dim3 grid(tiles_i * tiles_j, B);
  hipLaunchKernelGGL(corr_build_kernel, grid, dim3(NT), 0, stream, f1, f2, p, C, H, W, levels,
                     sqrtf((float)C), tiles_x, tiles_j);
}

void launch_corr_build_bf16(const uint16_t* f1, const uint16_t* f2, void* const* lvl, const int* hs,
                            const int* ws, int B, int C, int H, int W, int levels, bool pyr_bf16,
                            hipStream_t stream) {
  const int N = H * W;
  const int tiles_i = (int)raft_cdiv(N, BB_I), bands_y = (int)raft_cdiv(H, BB_Y);
  const int tiles_x = (int)raft_cdiv(W, BB_X);
  dim3 grid(tiles_i * bands_y * tiles_x, B);
  auto go = [&](auto* tag) {
    using T = std::remove_pointer_t<decltype(tag)>;
    PyrO<T> p;
    for (int l = 0; l < 4; ++l) {
      p.lvl[l] = l < levels ? static_cast<T*>(lvl[l]) : nullptr;
      p.h[l] = l < levels ? hs[l] : 0;
      p.w[l] = l < levels ? ws[l] : 0;
    }
    hipLaunchKernelGGL(corr_build_bf16_kernel<T>, grid, dim3(256), 0, stream, f1, f2, p, C, H, W,
                       levels, 1.0f / sqrtf((float)C), tiles_i, bands_y, tiles_x);
  };
  if (pyr_bf16) go((uint16_t*)nullptr);
  else go((float*)nullptr);
}

void launch_corr_pyr_grad_reduce(float* const* glvl, const int* hs, const int* ws, int64_t planes,
                                 int levels, float inv_sqrt_c, float* out, hipStream_t stream) {
  Pyr4 p;
  for (int l = 0; l < 4; ++l) {
    p.lvl[l] = l < levels ? glvl[l] : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
  }
  int64_t total = planes * hs[0] * ws[0];
  unsigned blocks = (unsigned)std::min<int64_t>((total + 255) / 256, 256 * 16);
  hipLaunchKernelGGL(corr_pyr_grad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, p, out,
                     planes, levels, inv_sqrt_c);
}
