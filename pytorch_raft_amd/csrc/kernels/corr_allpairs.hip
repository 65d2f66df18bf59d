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

namespace {

constexpr int BI = 64;   // query pixels per workgroup
constexpr int TJ = 8;    // target block is TJ x TJ on the fmap2 grid
constexpr int BJ = TJ * TJ;
constexpr int KC = 32;   // channels per LDS stage
constexpr int NT = 256;  // threads

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
      if (i < N && Y < h2 && X < w2) L2[(((int64_t)b * N + i) * h2 + Y) * w2 + X] = v;
    }
  }
  __syncthreads();
  if (levels > 3) {
    float* L3 = out.lvl[3];
    const int h3 = out.h[3], w3 = out.w[3];
    for (int ii = tid; ii < BI; ii += NT) {
      float v = (((P2[ii][0] + P2[ii][1]) + P2[ii][2]) + P2[ii][3]) * 0.25f;
      int i = i0 + ii, Y = y0 >> 3, X = x0 >> 3;
      if (i < N && Y < h3 && X < w3) L3[(((int64_t)b * N + i) * h3 + Y) * w3 + X] = v;
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
