// Feature-map gradients of the all-pairs correlation on MFMA (bf16 operands, fp32 accumulation).
//
// Reference: `core/corr.py:52-60` computes corr = F1^T F2 / sqrt(C) with torch.matmul; autograd's
// backward is two batched GEMMs over the dense correlation gradient dC (B, N, N):
//     dF1 = dC F2        (B, N, C)        dF2 = dC^T F1        (B, N, C)
// at chairs / batch 12 two 50-GFLOP GEMMs per step (M = N = 2852 query / target pixels, K = 2852,
// N_out = C = 256).  Here they are two launches of one LDS-DMA pipelined MFMA kernel:
//
//  * MODE 0 (dF1): both operands k-contiguous -- A = dC rows (i, k = j), B = F2^T rows (c, k = j),
//    the transposed feature map written once by corr_transpose_pad_kernel (NCHW, rows padded to
//    the fold's row pitch with zeros).  Fragment reads as in the conv kernels: 128-B LDS rows with
//    the 16-B chunk XOR swizzle (row >> 1) & 7, applied on the DMA source side.
//  * MODE 1 (dF2): both operands k-major -- A = dC rows (k = i, m = j), B = F1 rows (k = i, c) --
//    read through ds_read_b64_tr_b16 transposed fragment reads (256-B LDS rows, chunk swizzle
//    4 (row & 3)), the conv weight-gradient kernels' layout (conv_wgrad.hip).
//
// dC comes from the correlation fold (corr_window.hip) with its rows padded to a multiple of 64
// columns (zeros), so every A row is 16-B aligned and MODE 0's K runs whole 64-wide steps.
// fp32 correlation (the fp16 / fp32 schedules: the reference runs the correlation in fp32 outside
// autocast): dC and the fp32 feature maps are carried as bf16 pairs x = hi + lo, and each GEMM is
// ONE launch over three K passes -- dC_hi F_hi + dC_lo F_hi + dC_hi F_lo, fp32 accumulation, fp32
// output (~2^-16 relative; the dropped lo*lo term is ~2^-18) -- the split-bf16 scheme of the conv
// kernels, at 3x the bf16 MFMA work instead of the 1/8-rate fp32 MFMA.
// Workgroup = 4 waves in 2 x 2, tile 128 x 128, 64-deep K steps double-buffered through LDS
// (64 KB), XCD-aware tile order (the two C tiles of one row block share an L2).  The bf16 outputs
// are the NHWC (B, N, C) gradients the channels_last encoder outputs take.
#include <algorithm>

#include "common.h"
#include "launchers.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t OOB = 0x80000000u;
constexpr int NT = 256, BM = 128, BN = 128, BK = 64;
constexpr int WM = 64, WN = 64, TM = 2, TN = 2;

__device__ __forceinline__ rsrc_t mk_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

// MODE 0 layout: [128 rows][8 x 16-B chunks], chunk c of row r at slot r * 8 + (c ^ ((r >> 1) & 7))
__device__ __forceinline__ int swz128(int row, int chunk) { return row * 8 + (chunk ^ ((row >> 1) & 7)); }
// MODE 1 layout: [64 rows][16 x 16-B chunks], chunk c of row r at slot c ^ 4 (r & 3)
__device__ __forceinline__ int swz256(int row) { return 4 * (row & 3); }

// K passes of one launch: pass p multiplies A operand a[p] by B operand b[p] (bf16: one pass;
// split fp32: the three products above)
struct GemmOps {
  const uint16_t* a[3];
  const uint16_t* b[3];
};

template <int MODE, int NPROD, bool OUT32>
__global__ __launch_bounds__(NT, 2) void corr_bwd_gemm_kernel(GemmOps ops, int lda, int ldb,
                                                              void* __restrict__ out, int B, int N,
                                                              int C, int K, int64_t a_bstride,
                                                              int64_t b_bstride) {
  constexpr int STAGE = (BM + BN) * BK * 2;  // bytes: 32 KB
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int mt_n = (N + BM - 1) / BM, nt_n = C / BN;
  const int tiles = B * mt_n * nt_n;
  // XCD-aware order: consecutive logical tiles (the C tiles of a row block, then the next row
  // block of the same image) run on one XCD
  const int L = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
  if (L >= tiles) return;
  const int b = L / (mt_n * nt_n);
  const int rem = L - b * mt_n * nt_n;
  const int mt = rem / nt_n, nt = rem - mt * nt_n;
  const int m0 = mt * BM, n0 = nt * BN;

  // descriptors sized to the image's operand (rows past the end read zeros), one per pass
  rsrc_t a_rs[NPROD], b_rs[NPROD];
#pragma unroll
  for (int p = 0; p < NPROD; ++p) {
    a_rs[p] = mk_rsrc(ops.a[p] + (int64_t)b * a_bstride, (uint32_t)(a_bstride * 2));
    b_rs[p] = mk_rsrc(ops.b[p] + (int64_t)b * b_bstride, (uint32_t)(b_bstride * 2));
  }
  const uint32_t lds0 = raft_lds_addr(smem);
  const uint32_t wave_off = __builtin_amdgcn_readfirstlane(wave * 64 * 16);

  // per-thread DMA pieces of one stage: 4 of A, 4 of B (16 B each)
  uint32_t a_off[4], b_off[4];
  uint32_t a_kstep, b_kstep;  // byte advance per K step
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = tid + j * NT;
    if constexpr (MODE == 0) {
      // rows m / n, logical k chunk lc of the 64-deep step
      const int row = e >> 3, lc = (e & 7) ^ ((row >> 1) & 7);
      const int m = m0 + row, n = n0 + row;
      a_off[j] = m < N ? (uint32_t)(((int64_t)m * lda + lc * 8) * 2) : OOB;
      b_off[j] = n < C ? (uint32_t)(((int64_t)n * ldb + lc * 8) * 2) : OOB;
    } else {
      // rows k (64 per step), logical column chunk lc of the 128-wide tile
      const int row = e >> 4, lc = (e & 15) ^ swz256(row);
      a_off[j] = (uint32_t)(((int64_t)row * lda + m0 + lc * 8) * 2);
      b_off[j] = (uint32_t)(((int64_t)row * ldb + n0 + lc * 8) * 2);
    }
  }
  if constexpr (MODE == 0) {
    a_kstep = BK * 2;
    b_kstep = BK * 2;
  } else {
    a_kstep = (uint32_t)(BK * lda * 2);
    b_kstep = (uint32_t)(BK * ldb * 2);
  }
  const int ksteps = (K + BK - 1) / BK;
  const int steps = NPROD * ksteps;

  auto issue = [&](int t2, int buf) {
    const int p = t2 / ksteps, t = t2 - p * ksteps;   // pass, K step of the pass (uniform)
    rsrc_t ar = a_rs[0], br = b_rs[0];
    if constexpr (NPROD > 1) {
      if (p == 1) { ar = a_rs[1]; br = b_rs[1]; }
      else if (p == 2) { ar = a_rs[NPROD - 1]; br = b_rs[NPROD - 1]; }
    }
    const uint32_t base = lds0 + (uint32_t)(buf * STAGE) + wave_off;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      uint32_t ao = a_off[j] == OOB ? OOB : a_off[j] + (uint32_t)t * a_kstep;
      uint32_t bo = b_off[j] == OOB ? OOB : b_off[j] + (uint32_t)t * b_kstep;
      if constexpr (MODE == 1) {
        // K tail: rows k >= K read zeros
        const int k = t * BK + ((tid + j * NT) >> 4);
        if (k >= K) { ao = OOB; bo = OOB; }
      }
      raft_dma16(ar, base + j * NT * 16, ao);
      raft_dma16(br, base + (BM * BK * 2) + j * NT * 16, bo);
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  auto compute = [&](int buf) {
    const uint8_t* As = smem + buf * STAGE;
    const uint8_t* Bs = As + BM * BK * 2;
    if constexpr (MODE == 0) {
      const uint4* A4 = reinterpret_cast<const uint4*>(As);
      const uint4* B4 = reinterpret_cast<const uint4*>(Bs);
      bf16x8_t af[BK / 16][TM], bfr[BK / 16][TN];
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
          af[kk][i] = __builtin_bit_cast(bf16x8_t, A4[swz128(wm * WM + i * 32 + (lane & 31), kk * 2 + (lane >> 5))]);
#pragma unroll
        for (int j = 0; j < TN; ++j)
          bfr[kk][j] = __builtin_bit_cast(bf16x8_t, B4[swz128(wn * WN + j * 32 + (lane & 31), kk * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk][i], bfr[kk][j], acc[i][j], 0, 0, 0);
    } else {
      const int gi = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
      auto rd_tr = [](const uint8_t* base, int row, int col) {
        const int off = row * 256 + (((col >> 3) ^ swz256(row)) << 4) + (col & 7) * 2;
        return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(base + off));
      };
#pragma unroll
      for (int s = 0; s < BK / 16; ++s) {
        bf16x8_t af[TM], bfr[TN];
        const int row = s * 16 + (gi >> 1) * 8 + q;
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int col = wm * WM + i * 32 + (gi & 1) * 16 + 4 * pp;
          const auto lo = rd_tr(As, row, col), hi = rd_tr(As, row + 4, col);
          af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * WN + j * 32 + (gi & 1) * 16 + 4 * pp;
          const auto lo = rd_tr(Bs, row, col), hi = rd_tr(Bs, row + 4, col);
          bfr[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
  };

  // double-buffered: step t+1's DMAs in flight during step t's MFMAs
  issue(0, 0);
  for (int t = 0; t < steps; ++t) {
    if (t + 1 < steps) {
      issue(t + 1, (t + 1) & 1);
      raft_wait_vmcnt<8>();   // this thread's 8 pieces of step t have landed
    } else {
      raft_wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();   // every wave's pieces of step t are in LDS
    compute(t & 1);
    __builtin_amdgcn_s_barrier();   // step t's buffer is free for step t + 2
  }

  // bf16 (or fp32) store of the (m, c) tile: out[b][m][c]
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= N) continue;
        const int64_t o = ((int64_t)b * N + m) * C + n;
        if constexpr (OUT32) static_cast<float*>(out)[o] = acc[i][j][r];
        else static_cast<uint16_t*>(out)[o] = raft_f32_to_bf16(acc[i][j][r]);
      }
    }
}

// fp32 F (B, C, N) -> the split pair [hi | lo] as two (B, C, ldt) bf16 planes (hi plane, then lo
// plane at + B C ldt), columns N..ldt-1 zero: MODE 0's B operand (F2^T rows, k = j contiguous)
__global__ __launch_bounds__(256) void corr_split_pad_kernel(const float* __restrict__ F,
                                                             uint16_t* __restrict__ out, int64_t rows,
                                                             int N, int ldt) {
  const int64_t per_row = ldt / 4;   // 4 columns per thread
  const int64_t tot = rows * per_row;
  uint16_t* lo_plane = out + rows * ldt;
  for (int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x; e < tot; e += (int64_t)gridDim.x * 256) {
    const int64_t r = e / per_row;
    const int c0 = (int)(e - r * per_row) * 4;
    uint16_t h[4], l[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v = c0 + u < N ? F[r * N + c0 + u] : 0.f;
      h[u] = raft_f32_to_bf16(v);
      l[u] = raft_f32_to_bf16(v - raft_bf16_to_f32(h[u]));
    }
    *reinterpret_cast<uint2*>(out + r * ldt + c0) = make_uint2(h[0] | ((uint32_t)h[1] << 16), h[2] | ((uint32_t)h[3] << 16));
    *reinterpret_cast<uint2*>(lo_plane + r * ldt + c0) = make_uint2(l[0] | ((uint32_t)l[1] << 16), l[2] | ((uint32_t)l[3] << 16));
  }
}

// fp32 F (B, C, N) -> split pair planes (B, N, C) bf16 (hi, then lo at + B N C): MODE 1's B
// operand (F1 rows k = i, channel-contiguous).  64 pixels x 64 channels per workgroup through LDS.
__global__ __launch_bounds__(256) void corr_split_transpose_kernel(const float* __restrict__ F,
                                                                   uint16_t* __restrict__ out, int B,
                                                                   int N, int C) {
  __shared__ float tile[64][64 + 1];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  const float* Fb = F + (int64_t)b * C * N;
  // load: 64 channel rows x 64 pixels (coalesced along N)
  for (int e = tid; e < 64 * 64; e += 256) {
    const int c = e >> 6, p = e & 63;
    tile[c][p] = (p0 + p < N && c0 + c < C) ? Fb[(int64_t)(c0 + c) * N + p0 + p] : 0.f;
  }
  __syncthreads();
  uint16_t* hi = out + (int64_t)b * N * C;
  uint16_t* lo = hi + (int64_t)B * N * C;
  // store: 64 pixel rows x 8 chunks of 8 channels (16-B stores along C)
  for (int e = tid; e < 64 * 8; e += 256) {
    const int p = e >> 3, ch = e & 7;
    if (p0 + p >= N) continue;
    uint32_t hw[4], lw[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float v0 = tile[ch * 8 + 2 * u][p], v1 = tile[ch * 8 + 2 * u + 1][p];
      const uint16_t h0 = raft_f32_to_bf16(v0), h1 = raft_f32_to_bf16(v1);
      hw[u] = h0 | ((uint32_t)h1 << 16);
      lw[u] = raft_f32_to_bf16(v0 - raft_bf16_to_f32(h0)) |
              ((uint32_t)raft_f32_to_bf16(v1 - raft_bf16_to_f32(h1)) << 16);
    }
    const int64_t o = (int64_t)(p0 + p) * C + c0 + ch * 8;
    *reinterpret_cast<uint4*>(hi + o) = make_uint4(hw[0], hw[1], hw[2], hw[3]);
    *reinterpret_cast<uint4*>(lo + o) = make_uint4(lw[0], lw[1], lw[2], lw[3]);
  }
}

// F (B, N, C) bf16 -> Ft (B, C, ldt) bf16, columns N..ldt-1 zero: 64 pixels x 64 channels per
// workgroup through an LDS tile (16-B reads along C, 16-B writes along N)
__global__ __launch_bounds__(256) void corr_transpose_pad_kernel(const uint16_t* __restrict__ F,
                                                                 uint16_t* __restrict__ Ft, int N, int C,
                                                                 int ldt) {
  __shared__ uint16_t tile[64][64 + 8];
  const int b = blockIdx.z;
  const int p0 = blockIdx.x * 64, c0 = blockIdx.y * 64;
  const int tid = threadIdx.x;
  const uint16_t* Fb = F + (int64_t)b * N * C;
  // load: 64 rows (pixels) x 8 chunks of 8 channels
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = tid + k * 256;
    const int r = e >> 3, ch = e & 7;
    const int p = p0 + r;
    uint4 v = make_uint4(0u, 0u, 0u, 0u);
    if (p < N) v = *reinterpret_cast<const uint4*>(Fb + (int64_t)p * C + c0 + ch * 8);
    const uint16_t* s = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
    for (int u = 0; u < 8; ++u) tile[ch * 8 + u][r] = s[u];
  }
  __syncthreads();
  uint16_t* Tb = Ft + (int64_t)b * C * ldt;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int e = tid + k * 256;
    const int c = e >> 3, ch = e & 7;
    const int p = p0 + ch * 8;
    if (p >= ldt) continue;
    uint4 v;
    uint16_t* d = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
    for (int u = 0; u < 8; ++u) d[u] = (p + u < N) ? tile[c][ch * 8 + u] : (uint16_t)0;
    *reinterpret_cast<uint4*>(Tb + (int64_t)(c0 + c) * ldt + p) = v;
  }
}

template <int MODE, int NPROD, bool OUT32>
void launch_gemm(const GemmOps& ops, int lda, int ldb, void* out, int B, int N, int C, int K,
                 int64_t as, int64_t bs, hipStream_t stream) {
  const int tiles = B * ((N + BM - 1) / BM) * (C / BN);
  dim3 grid((unsigned)((tiles + 7) / 8 * 8));
  hipLaunchKernelGGL((corr_bwd_gemm_kernel<MODE, NPROD, OUT32>), grid, dim3(NT), 0, stream, ops, lda, ldb,
                     out, B, N, C, K, as, bs);
}

}  // namespace

bool launch_corr_bwd_fmaps(const uint16_t* dc, int ldc, const uint16_t* f1, const uint16_t* f2,
                           uint16_t* f2t, uint16_t* g1, uint16_t* g2, int B, int N, int C,
                           hipStream_t stream) {
  if (C % BN != 0 || ldc % BK != 0 || ldc < N) return false;
  if ((int64_t)N * ldc * 2 >= (int64_t(1) << 31) || (int64_t)C * ldc * 2 >= (int64_t(1) << 31))
    return false;   // per-image operands must fit one buffer descriptor
  dim3 tg((unsigned)((ldc + 63) / 64), (unsigned)(C / 64), (unsigned)B);
  hipLaunchKernelGGL(corr_transpose_pad_kernel, tg, dim3(256), 0, stream, f2, f2t, N, C, ldc);
  // dF1 = dC F2:  rows of dC (k = j) against rows of F2^T (k = j), K = the padded pitch
  launch_gemm<0, 1, false>(GemmOps{{dc}, {f2t}}, ldc, ldc, g1, B, N, C, ldc, (int64_t)N * ldc,
                           (int64_t)C * ldc, stream);
  // dF2 = dC^T F1:  k = i rows of dC (columns j) and of F1 (columns c), K = N
  launch_gemm<1, 1, false>(GemmOps{{dc}, {f1}}, ldc, C, g2, B, N, C, N, (int64_t)N * ldc,
                           (int64_t)N * C, stream);
  return true;
}

// fp32 correlation: dc2 = split dC planes [hi | lo] (2, B, N, ldc) bf16 from the fold; f1 / f2
// fp32 (B, C, N) (NCHW fmaps); scratch: f2s (2, B, C, ldc), f1s (2, B, N, C) bf16; g1 / g2 fp32
// (B, N, C)
bool launch_corr_bwd_fmaps_split(const uint16_t* dc2, int ldc, const float* f1, const float* f2,
                                 uint16_t* f2s, uint16_t* f1s, float* g1, float* g2, int B, int N, int C,
                                 hipStream_t stream) {
  if (C % BN != 0 || C % 64 != 0 || ldc % BK != 0 || ldc < N) return false;
  if ((int64_t)N * ldc * 2 >= (int64_t(1) << 31) || (int64_t)C * ldc * 2 >= (int64_t(1) << 31))
    return false;
  const int64_t rows = (int64_t)B * C;
  const int64_t work = rows * (ldc / 4);
  hipLaunchKernelGGL(corr_split_pad_kernel, dim3((unsigned)std::min<int64_t>((work + 255) / 256, 8192)),
                     dim3(256), 0, stream, f2, f2s, rows, N, ldc);
  dim3 tg((unsigned)((N + 63) / 64), (unsigned)(C / 64), (unsigned)B);
  hipLaunchKernelGGL(corr_split_transpose_kernel, tg, dim3(256), 0, stream, f1, f1s, B, N, C);
  const uint16_t* dlo = dc2 + (int64_t)B * N * ldc;
  const uint16_t* f2lo = f2s + (int64_t)B * C * ldc;
  const uint16_t* f1lo = f1s + (int64_t)B * N * C;
  // passes: dC_hi F_hi + dC_lo F_hi + dC_hi F_lo
  launch_gemm<0, 3, true>(GemmOps{{dc2, dlo, dc2}, {f2s, f2s, f2lo}}, ldc, ldc, g1, B, N, C, ldc,
                          (int64_t)N * ldc, (int64_t)C * ldc, stream);
  launch_gemm<1, 3, true>(GemmOps{{dc2, dlo, dc2}, {f1s, f1s, f1lo}}, ldc, C, g2, B, N, C, N,
                          (int64_t)N * ldc, (int64_t)N * C, stream);
  return true;
}
