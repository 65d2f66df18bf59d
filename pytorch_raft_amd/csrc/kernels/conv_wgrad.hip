// Weight gradient of the NHWC implicit-GEMM convolution (bf16 MFMA, fp32 accumulation).
//
//   dW[co][tap][ci] = sum_p  G[p][co] * X[p + off(tap)][ci]        (G = dL/d(pre-activation))
//
// GEMM view: M = Cout, N = packed K (tap x CinPad, the same layout as the forward's packed weights),
// reduction over pixels p.  Both operands are stored pixel-major ([p][channel], channels
// contiguous), i.e. the reduction index is the OUTER one, so the MFMA fragments (8 consecutive
// reduction elements per lane) are gathered with the gfx950 transposing LDS read
// ds_read_b64_tr_b16 (`__builtin_amdgcn_ds_read_tr16_b64_v4bf16`): a 16-lane group reads a
// 4-row x 16-column block and lane i receives column i -- two reads give the 8-deep K fragment of
// v_mfma_f32_32x32x16_bf16 with no register shuffles.  The pixel dimension is split across
// workgroups (split-K); each workgroup's 128x128 fp32 partial tile is added with 128-B-segment
// float atomics (the shape MI355X's memory-side atomic units run at full rate).
//
// Pipeline: 64 pixels per step, two register sets (loads of the next two steps in flight during
// the current step's MFMAs), two LDS buffers, one barrier per step.
// Bias gradient: the column sums of G are accumulated from the LDS tiles by the workgroups of the
// first K-tile column (no extra pass over G); col_sum_kernel remains for callers without wgrad.
#include "common.h"
#include "launchers.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;
constexpr int NT = 256;
constexpr int BKP = 64;  // pixels per pipeline step

template <int BM, int BN, bool SMALLC>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_kernel(ConvWgradArgs a, float* __restrict__ db) {
  // 4 waves as 2 x 2, each owns (BM/2) x (BN/2)
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int GCH = BKP * BM / 8;  // 16-B chunks per stage
  constexpr int XCH = BKP * BN / 8;
  constexpr int G_PER = (GCH + NT - 1) / NT;
  constexpr int X_PER = (XCH + NT - 1) / NT;
  // rows padded by 16 bf16 (32 B): the 4 rows of a ds_read_b64_tr_b16 16-lane group land on
  // disjoint bank ranges
  constexpr int GS = BM + 16, XS = BN + 16;
  __shared__ __attribute__((aligned(16))) uint16_t Gs[2][BKP * GS];
  __shared__ __attribute__((aligned(16))) uint16_t Xs[2][BKP * XS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  const int ntile_n = (a.kpad + BN - 1) / BN;
  const int tm = blockIdx.x / ntile_n, tn = blockIdx.x % ntile_n;
  const int m0 = tm * BM, k0 = tn * BN;
  const int p_begin = blockIdx.y * a.pix_per_split;
  const int p_end = min(P, p_begin + a.pix_per_split);
  const int ktot_small = a.KH * a.KW * a.cin_small;

  auto load = [&](int pbase, uint4 (&rg)[G_PER], uint4 (&rx)[X_PER]) {
#pragma unroll
    for (int j = 0; j < G_PER; ++j) {
      const int e = tid + j * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < GCH) {
        const int row = e / (BM / 8), ch = e % (BM / 8);
        const int p = pbase + row, n = m0 + ch * 8;
        if (p < p_end) {
          const uint16_t* src = a.g + (int64_t)p * a.g_stride + n;
          if (n + 8 <= a.cout) {
            v = *reinterpret_cast<const uint4*>(src);
          } else if (n < a.cout) {
            uint16_t t[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) t[q] = (n + q < a.cout) ? src[q] : 0;
            v = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
          }
        }
      }
      rg[j] = v;
    }
#pragma unroll
    for (int j = 0; j < X_PER; ++j) {
      const int e = tid + j * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < XCH) {
        const int row = e / (BN / 8), ch = e % (BN / 8);
        const int p = pbase + row;
        const int kc = k0 + ch * 8;
        if (p < p_end && kc < a.kpad) {
          const int b = p / HW;
          const int rr = p - b * HW;
          const int y = rr / a.W, x = rr - (rr / a.W) * a.W;
          if constexpr (!SMALLC) {
            const int tap = kc / a.cin_pad, c = kc - tap * a.cin_pad;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            const int yy = y + kh - a.PH, xx = x + kw - a.PW;
            if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
              int s = 0, sbase = 0;
#pragma unroll
              for (int q = 0; q < 2; ++q)
                if (s + 1 < a.nseg && c >= sbase + a.seg[s].cnt) { sbase += a.seg[s].cnt; ++s; }
              const Seg sg = a.seg[s];
              v = *reinterpret_cast<const uint4*>(sg.ptr + ((int64_t)(b * a.H + yy) * a.W + xx) * sg.stride + (c - sbase));
            }
          } else {
            uint16_t t[8];
#pragma unroll
            for (int q = 0; q < 8; ++q) {
              const int k = kc + q;
              uint16_t val = 0;
              if (k < ktot_small) {
                const int tap = k / a.cin_small, c = k - tap * a.cin_small;
                const int kh = tap / a.KW, kw = tap - kh * a.KW;
                const int yy = y + kh - a.PH, xx = x + kw - a.PW;
                if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
                  val = a.seg[0].ptr[((int64_t)(b * a.H + yy) * a.W + xx) * a.seg[0].stride + c];
              }
              t[q] = val;
            }
            v = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
          }
        }
      }
      rx[j] = v;
    }
  };
  auto store = [&](int buf, const uint4 (&rg)[G_PER], const uint4 (&rx)[X_PER]) {
#pragma unroll
    for (int j = 0; j < G_PER; ++j) {
      const int e = tid + j * NT;
      const int row = e / (BM / 8), ch = e % (BM / 8);
      if (e < GCH) *reinterpret_cast<uint4*>(&Gs[buf][row * GS + ch * 8]) = rg[j];
    }
#pragma unroll
    for (int j = 0; j < X_PER; ++j) {
      const int e = tid + j * NT;
      const int row = e / (BN / 8), ch = e % (BN / 8);
      if (e < XCH) *reinterpret_cast<uint4*>(&Xs[buf][row * XS + ch * 8]) = rx[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const int gi = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  // bias gradient (column sums of G) rides along in the first K-tile column of workgroups
  const bool do_bias = db != nullptr && tn == 0;
  float bsum = 0.f;
  auto compute = [&](int cur) {
#pragma unroll
    for (int s = 0; s < BKP / 16; ++s) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * WM + i * 32 + (gi & 1) * 16 + 4 * pp;
        const int row = s * 16 + (gi >> 1) * 8 + q;
        bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(&Gs[cur][row * GS + col]));
        bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(&Gs[cur][(row + 4) * GS + col]));
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 32 + (gi & 1) * 16 + 4 * pp;
        const int row = s * 16 + (gi >> 1) * 8 + q;
        bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(&Xs[cur][row * XS + col]));
        bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16(
            (lds_bf16x4_t*)(&Xs[cur][(row + 4) * XS + col]));
        bfr[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (do_bias) {
      // NT / BM threads per column, each a contiguous run of rows
      constexpr int TPC = NT / BM, RPT = BKP / TPC;
      const int c = tid % BM, r0 = (tid / BM) * RPT;
#pragma unroll
      for (int r = 0; r < RPT; ++r) bsum += raft_bf16_to_f32(Gs[cur][(r0 + r) * GS + c]);
    }
  };

  const int steps = (p_end - p_begin + BKP - 1) / BKP;
  uint4 rg0[G_PER], rx0[X_PER], rg1[G_PER], rx1[X_PER];
  if (steps > 0) {
    load(p_begin, rg0, rx0);
    if (steps > 1) load(p_begin + BKP, rg1, rx1);
    store(0, rg0, rx0);
  }
  __syncthreads();
  for (int t = 0; t < steps; t += 2) {
    if (t + 2 < steps) load(p_begin + (t + 2) * BKP, rg0, rx0);
    compute(0);
    if (t + 1 < steps) store(1, rg1, rx1);
    __syncthreads();
    if (t + 1 >= steps) break;
    if (t + 3 < steps) load(p_begin + (t + 3) * BKP, rg1, rx1);
    compute(1);
    if (t + 2 < steps) store(0, rg0, rx0);
    __syncthreads();
  }
  if (steps == 0) return;
  if (do_bias) {
    const int c = m0 + tid % BM;
    if (c < a.cout) atomicAdd(db + c, bsum);
  }

#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int kc = k0 + wn * WN + j * 32 + (lane & 31);
      if (kc >= a.kpad) continue;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (n < a.cout) atomicAdd(a.dw + (int64_t)n * a.kpad + kc, acc[i][j][r]);
      }
    }
}

// db[n] = sum_p G[p][n]: each block sums a pixel range for 64 channels, then one atomic per channel
__global__ __launch_bounds__(256) void col_sum_kernel(const uint16_t* __restrict__ g, int stride,
                                                      int cout, int P, int pix_per_block,
                                                      float* __restrict__ db) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rowg = threadIdx.x >> 6;
  const int p0 = blockIdx.y * pix_per_block;
  const int p1 = min(P, p0 + pix_per_block);
  float s = 0.f;
  if (c < cout)
    for (int p = p0 + rowg; p < p1; p += 4) s += raft_bf16_to_f32(g[(int64_t)p * stride + c]);
  red[rowg][threadIdx.x & 63] = s;
  __syncthreads();
  if (threadIdx.x < 64 && c < cout)
    atomicAdd(db + c, (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]));
}

}  // namespace

bool launch_conv_wgrad(const ConvWgradArgs& a, int bm, bool smallc, float* db,
                       hipStream_t stream) {
  const int P = a.B * a.H * a.W;
  const int splits = (P + a.pix_per_split - 1) / a.pix_per_split;
  constexpr int BN = 128;
  const int tiles_n = (a.kpad + BN - 1) / BN;
  if (bm == 128) {
    dim3 grid(raft_cdiv(a.cout, 128) * tiles_n, splits);
    if (smallc) hipLaunchKernelGGL((conv_wgrad_kernel<128, BN, true>), grid, dim3(NT), 0, stream, a, db);
    else hipLaunchKernelGGL((conv_wgrad_kernel<128, BN, false>), grid, dim3(NT), 0, stream, a, db);
  } else {
    dim3 grid(raft_cdiv(a.cout, 64) * tiles_n, splits);
    if (smallc) hipLaunchKernelGGL((conv_wgrad_kernel<64, BN, true>), grid, dim3(NT), 0, stream, a, db);
    else hipLaunchKernelGGL((conv_wgrad_kernel<64, BN, false>), grid, dim3(NT), 0, stream, a, db);
  }
  return true;
}

void launch_col_sum(const uint16_t* g, int stride, int cout, int P, float* db, hipStream_t stream) {
  // 64 pixels per block (16 per thread row): ~P/64 x cout/64 blocks keep every CU busy; the
  // reduction is latency-bound, not bandwidth-bound, at 1024 pixels per block (measured 60 us)
  const int ppb = 64;
  dim3 grid(raft_cdiv(cout, 64), raft_cdiv(P, ppb));
  hipLaunchKernelGGL(col_sum_kernel, grid, dim3(256), 0, stream, g, stride, cout, P, ppb, db);
}
