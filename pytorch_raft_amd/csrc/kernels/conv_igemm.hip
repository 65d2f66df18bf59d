// Implicit-GEMM 2-D convolution for the RAFT update block on MI355X (bf16 MFMA, NHWC).
//
// The update block (`core/update.py:79-136`) is 73 % of RAFT's FLOPs: 1x1 / 3x3 / 7x7 / 1x5 / 5x1
// stride-1 "same" convolutions on (B, H/8, W/8) maps, run 12-32 times per pair.  The reference
// runs them as NCHW cuDNN convs with torch.cat / sigmoid / tanh / mul / add glue around them; on
// ROCm that becomes MIOpen CK kernels bracketed by NCHW<->NHWC transposes.  Here:
//
//   GEMM view  M = pixels (B*H*W), N = Cout, K = KH*KW*Cin;  A = input patch rows gathered on the
//              fly from NHWC bf16 activations (no im2col buffer), B = weights pre-packed per step
//              as [Npad][KH*KW][CinPad] bf16 (k contiguous).
//   Tiling     workgroup = 4 waves (256 threads), tile BM x BN (128|64 x 128|64, 128x32),
//              BK = 64 (one filter tap x 64 channels), v_mfma_f32_32x32x16_bf16 with fp32
//              accumulators; A/B staged global -> registers -> LDS: two register sets keep the
//              loads of the next TWO K-steps in flight during the current step's MFMAs, two LDS
//              buffers, one barrier per step; LDS rows are 128 B and XOR-swizzled on the 16-B
//              chunk index so ds_read_b128 fragment reads are bank-conflict free.
//   Inputs     "virtual concat": up to 3 NHWC channel segments from different buffers form the
//              input channels (e.g. [h | x] for the GRU), so no torch.cat copies exist.
//   Epilogues  fused per element: bias, scale, ReLU, bf16/fp32 store into a channel slice of a
//              wider NHWC buffer, the GRU z/r gates (z = s(.), r*h) and the GRU state update
//              (q = tanh(.), h' = h + z (q - h)), and fp32 accumulate (for dgrad).
//   Small Cin  (convf1: Cin = 2, 7x7) packs K = KH*KW*Cin densely (98 -> 128) and gathers
//              scalars instead of wasting 94 % of the MFMA on zero channels.
//
// dgrad reuses this kernel with flipped / transposed packed weights (stride-1 same padding is
// self-adjoint up to the flip); wgrad lives in conv_wgrad.hip.
#include "common.h"
#include "launchers.h"

#include <cmath>

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int BK = 64;   // K per pipeline step: one filter tap x 64 channels (128-B LDS rows)
constexpr int NT = 256;

// 16-B chunk `chunk` (0..7) of LDS row `row` (128 B): XOR swizzle on the row's low 3 bits so the 8
// lanes of a ds_read_b128 phase (8 consecutive rows, same logical chunk) hit 8 distinct bank groups
__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ (row & 7)); }

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + __expf(-v)); }
__device__ __forceinline__ float tanhf_(float v) {
  const float e = __expf(-2.f * fabsf(v));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, v);
}

// Pipeline (per 64-deep K step, one barrier):  global loads for step t+2 are issued into one of
// two register sets before the MFMAs of step t (two steps = ~1000+ MFMA cycles of latency cover),
// the other set (step t+1, loaded one step earlier) is written to the idle LDS buffer after them.
template <int BM, int BN, int WM, int WN, int EPI, bool SMALLC>
__global__ __launch_bounds__(NT, 2) void conv_fwd_kernel(ConvFwdArgs a) {
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * WAVES_N == 4, "4 waves per workgroup");
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_CHUNKS = BM * 8;  // 16-B chunks per A stage
  constexpr int B_CHUNKS = BN * 8;
  constexpr int A_PER = A_CHUNKS / NT;
  constexpr int B_PER = (B_CHUNKS + NT - 1) / NT;

  __shared__ __attribute__((aligned(16))) uint4 As[2][A_CHUNKS];
  __shared__ __attribute__((aligned(16))) uint4 Bs[2][B_CHUNKS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  // per-thread A rows (fixed over the K loop): chunk e -> row e>>3, 16-B column e&7
  int a_b[A_PER], a_y[A_PER], a_x[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * NT;
    const int m = m0 + (e >> 3);
    a_ok[j] = m < P;
    const int mm = a_ok[j] ? m : 0;
    a_b[j] = mm / HW;
    const int r = mm - a_b[j] * HW;
    a_y[j] = r / a.W;
    a_x[j] = r - a_y[j] * a.W;
  }

  const int nchunk = SMALLC ? 0 : a.cin_pad / BK;
  const int steps = SMALLC ? a.kpad / BK : a.KH * a.KW * nchunk;

  auto load = [&](int t, uint4 (&ra)[A_PER], uint4 (&rb)[B_PER]) {
    if constexpr (!SMALLC) {
      const int tap = t / nchunk, ch = t - tap * nchunk;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
      const int c0 = ch * BK;
      int s = 0, sbase = 0;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (s + 1 < a.nseg && c0 >= sbase + a.seg[s].cnt) { sbase += a.seg[s].cnt; ++s; }
      const Seg sg = a.seg[s];
#pragma unroll
      for (int j = 0; j < A_PER; ++j) {
        const int e = tid + j * NT;
        const int yy = a_y[j] + kh - a.PH, xx = a_x[j] + kw - a.PW;
        uint4 v = make_uint4(0, 0, 0, 0);
        if (a_ok[j] && yy >= 0 && yy < a.H && xx >= 0 && xx < a.W) {
          const uint16_t* p = sg.ptr + ((int64_t)(a_b[j] * a.H + yy) * a.W + xx) * sg.stride +
                              (c0 - sbase) + (e & 7) * 8;
          v = *reinterpret_cast<const uint4*>(p);
        }
        ra[j] = v;
      }
    } else {
      // dense K = tap * cs + c ; each thread gathers 8 consecutive k of one row per chunk
      const Seg sg = a.seg[0];
      const int cs = a.cin_small;
      const int ktot = a.KH * a.KW * cs;
#pragma unroll
      for (int j = 0; j < A_PER; ++j) {
        const int e = tid + j * NT;
        uint16_t vals[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int k = t * BK + (e & 7) * 8 + q;
          uint16_t v = 0;
          if (a_ok[j] && k < ktot) {
            const int tap = k / cs, c = k - tap * cs;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            const int yy = a_y[j] + kh - a.PH, xx = a_x[j] + kw - a.PW;
            if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
              v = sg.ptr[((int64_t)(a_b[j] * a.H + yy) * a.W + xx) * sg.stride + c];
          }
          vals[q] = v;
        }
        ra[j] = make_uint4(vals[0] | (vals[1] << 16), vals[2] | (vals[3] << 16),
                           vals[4] | (vals[5] << 16), vals[6] | (vals[7] << 16));
      }
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int e = tid + j * NT;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (e < B_CHUNKS) {
        const int n = n0 + (e >> 3);
        v = *reinterpret_cast<const uint4*>(a.wpk + (int64_t)n * a.kpad + t * BK + (e & 7) * 8);
      }
      rb[j] = v;
    }
  };
  auto store = [&](int buf, const uint4 (&ra)[A_PER], const uint4 (&rb)[B_PER]) {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int e = tid + j * NT;
      As[buf][swz(e >> 3, e & 7)] = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int e = tid + j * NT;
      if (e < B_CHUNKS) Bs[buf][swz(e >> 3, e & 7)] = rb[j];
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
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + (lane & 31);
        af[i] = __builtin_bit_cast(bf16x8_t, As[buf][swz(row, kk * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + (lane & 31);
        bfr[j] = __builtin_bit_cast(bf16x8_t, Bs[buf][swz(row, kk * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  uint4 ra0[A_PER], rb0[B_PER], ra1[A_PER], rb1[B_PER];
  load(0, ra0, rb0);
  if (steps > 1) load(1, ra1, rb1);
  store(0, ra0, rb0);
  __syncthreads();
  for (int t = 0; t < steps; t += 2) {
    // even step: LDS[0] = step t, regs1 = step t+1 (in flight), regs0 free
    if (t + 2 < steps) load(t + 2, ra0, rb0);
    compute(0);
    if (t + 1 < steps) store(1, ra1, rb1);
    __syncthreads();
    if (t + 1 >= steps) break;
    // odd step: LDS[1] = step t+1, regs0 = step t+2 (in flight), regs1 free
    if (t + 3 < steps) load(t + 3, ra1, rb1);
    compute(1);
    if (t + 2 < steps) store(0, ra0, rb0);
    __syncthreads();
  }

  // ---------------------------------------------------------------- fused epilogue
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wn * WN + j * 32 + (lane & 31);
      if (n >= a.cout) continue;
      const float bias = a.bias ? a.bias[n] : 0.f;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m >= P) continue;
        const float v = (acc[i][j][r] + bias) * a.scale;
        if constexpr (EPI == EPI_BF16) {
          ((uint16_t*)a.out0)[(int64_t)m * a.out0_stride + n] = raft_f32_to_bf16(v);
        } else if constexpr (EPI == EPI_RELU_BF16) {
          ((uint16_t*)a.out0)[(int64_t)m * a.out0_stride + n] = raft_f32_to_bf16(fmaxf(v, 0.f));
        } else if constexpr (EPI == EPI_F32) {
          ((float*)a.out0)[(int64_t)m * a.out0_stride + n] = v;
        } else if constexpr (EPI == EPI_ACC_F32) {
          ((float*)a.out0)[(int64_t)m * a.out0_stride + n] += v;
        } else if constexpr (EPI == EPI_GRU_ZR) {
          const float g = sigmoidf_(v);
          if (n < a.split) {
            ((uint16_t*)a.out0)[(int64_t)m * a.out0_stride + n] = raft_f32_to_bf16(g);  // z
          } else {
            const int c = n - a.split;
            const float h = raft_bf16_to_f32(a.aux0[(int64_t)m * a.aux0_stride + c]);
            ((uint16_t*)a.out1)[(int64_t)m * a.out1_stride + c] = raft_f32_to_bf16(g * h);  // r*h
            ((uint16_t*)a.out2)[(int64_t)m * a.out2_stride + c] = raft_f32_to_bf16(g);      // r
          }
        } else if constexpr (EPI == EPI_DGRAD) {
          // output channel n -> one of up to 3 fp32 gradient buffers (store or accumulate)
          int s = 0, base = 0;
#pragma unroll
          for (int q = 0; q < 2; ++q)
            if (s + 1 < a.noseg && n >= base + a.oseg[s].cnt) { base += a.oseg[s].cnt; ++s; }
          const OSeg o = a.oseg[s];
          const int c = n - base;
          if (o.ptr != nullptr && c < o.real) {
            float* dst = o.ptr + (int64_t)m * o.stride + c;
            if (o.acc) *dst += v; else *dst = v;
          }
        } else if constexpr (EPI == EPI_F32_NCHW) {
          const int b = m / HW, yx = m - b * HW;
          ((float*)a.out0)[((int64_t)b * a.cout + n) * HW + yx] = v;
        } else if constexpr (EPI == EPI_GRU_Q) {
          const float q = tanhf_(v);
          const float h = raft_bf16_to_f32(a.aux0[(int64_t)m * a.aux0_stride + n]);
          const float z = raft_bf16_to_f32(a.aux1[(int64_t)m * a.aux1_stride + n]);
          ((uint16_t*)a.out0)[(int64_t)m * a.out0_stride + n] = raft_f32_to_bf16(h + z * (q - h));
          ((uint16_t*)a.out1)[(int64_t)m * a.out1_stride + n] = raft_f32_to_bf16(q);
        }
      }
    }
}

// Tile choice: M = B*H*W is ~34k pixels at chairs (267 x 128 rows), so 128-row tiles leave the
// 256 CUs with ~1.05 "rounds" of work for N <= 256 -- BM = 64 doubles the tile count and cuts the
// tail; 128-row tiles keep the better LDS reuse when there are already many tiles.
int pick_bm(int P, int cout, int bn) {
  const int nt = (cout + bn - 1) / bn;
  const int t128 = ((P + 127) / 128) * nt;
  const int t64 = ((P + 63) / 64) * nt;
  const double slots128 = 256.0 * 2, slots64 = 256.0 * 3;
  // rounds x per-tile time (a 64-row tile costs ~0.55 of a 128-row one: lower fragment reuse)
  const double c128 = std::ceil(t128 / slots128) * 1.0;
  const double c64 = std::ceil(t64 / slots64) * 0.55;
  return c64 < c128 ? 64 : 128;
}

template <int EPI, bool SMALLC>
void launch_cfg(const ConvFwdArgs& a, int bn, hipStream_t stream) {
  const int P = a.B * a.H * a.W;
  const int bm = pick_bm(P, a.cout, bn);
  if (bn == 128) {
    if (bm == 128) {
      dim3 grid(raft_cdiv(P, 128), raft_cdiv(a.cout, 128));
      hipLaunchKernelGGL((conv_fwd_kernel<128, 128, 64, 64, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
    } else {
      dim3 grid(raft_cdiv(P, 64), raft_cdiv(a.cout, 128));
      hipLaunchKernelGGL((conv_fwd_kernel<64, 128, 32, 64, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
    }
  } else if (bn == 64) {
    if (bm == 128) {
      dim3 grid(raft_cdiv(P, 128), raft_cdiv(a.cout, 64));
      hipLaunchKernelGGL((conv_fwd_kernel<128, 64, 64, 32, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
    } else {
      dim3 grid(raft_cdiv(P, 64), raft_cdiv(a.cout, 64));
      hipLaunchKernelGGL((conv_fwd_kernel<64, 64, 32, 32, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
    }
  } else {
    dim3 grid(raft_cdiv(P, 128), raft_cdiv(a.cout, 32));
    hipLaunchKernelGGL((conv_fwd_kernel<128, 32, 32, 32, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
  }
}

template <int EPI>
void launch_epi(const ConvFwdArgs& a, int bn, bool smallc, hipStream_t stream) {
  if (smallc) launch_cfg<EPI, true>(a, bn, stream);
  else launch_cfg<EPI, false>(a, bn, stream);
}

}  // namespace

bool launch_conv_fwd(const ConvFwdArgs& a, int epi, int bn, bool smallc, hipStream_t stream) {
  switch (epi) {
    case EPI_BF16: launch_epi<EPI_BF16>(a, bn, smallc, stream); return true;
    case EPI_RELU_BF16: launch_epi<EPI_RELU_BF16>(a, bn, smallc, stream); return true;
    case EPI_F32: launch_epi<EPI_F32>(a, bn, smallc, stream); return true;
    case EPI_ACC_F32: launch_epi<EPI_ACC_F32>(a, bn, smallc, stream); return true;
    case EPI_GRU_ZR: launch_epi<EPI_GRU_ZR>(a, bn, false, stream); return true;
    case EPI_GRU_Q: launch_epi<EPI_GRU_Q>(a, bn, false, stream); return true;
    case EPI_DGRAD: launch_epi<EPI_DGRAD>(a, bn, smallc, stream); return true;
    case EPI_F32_NCHW: launch_epi<EPI_F32_NCHW>(a, bn, smallc, stream); return true;
    default: return false;
  }
}
