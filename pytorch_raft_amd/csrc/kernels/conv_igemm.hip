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
//   Tiling     workgroup = 4 waves (256 threads), tile BM x BN (128x128 / 128x64 / 128x32),
//              BK = 32 (one filter tap x 32 channels), v_mfma_f32_32x32x16_bf16 with fp32
//              accumulators; A/B staged global -> registers -> LDS with a 2-deep LDS ring (the next
//              K-step's global loads are in flight during the current step's MFMAs); LDS rows are
//              64 B and XOR-swizzled on the 16-B chunk index so ds_read_b128 fragment reads are
//              bank-conflict free.
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

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int BK = 32;
constexpr int NT = 256;

__device__ __forceinline__ int swz(int row, int chunk) {  // 16-B chunk index within a 64-B row
  return row * 4 + (chunk ^ ((row >> 2) & 3));
}

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + __expf(-v)); }
__device__ __forceinline__ float tanhf_(float v) {
  const float e = __expf(-2.f * fabsf(v));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, v);
}

template <int BM, int BN, int WM, int WN, int EPI, bool SMALLC>
__global__ __launch_bounds__(NT) void conv_fwd_kernel(ConvFwdArgs a) {
  constexpr int WAVES_N = BN / WN;
  static_assert((BM / WM) * WAVES_N == 4, "4 waves per workgroup");
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int A_CHUNKS = BM * 4;  // 16-B chunks per A stage
  constexpr int B_CHUNKS = BN * 4;
  constexpr int A_PER = (A_CHUNKS + NT - 1) / NT;
  constexpr int B_PER = (B_CHUNKS + NT - 1) / NT;

  __shared__ __attribute__((aligned(16))) uint4 As[2][A_CHUNKS];
  __shared__ __attribute__((aligned(16))) uint4 Bs[2][B_CHUNKS];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

  // per-thread A rows (fixed over the K loop)
  int a_b[A_PER], a_y[A_PER], a_x[A_PER];
  bool a_ok[A_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * NT;
    const int m = m0 + (e >> 2);
    a_ok[j] = (e < A_CHUNKS) && (m < P);
    const int mm = a_ok[j] ? m : 0;
    a_b[j] = mm / HW;
    const int r = mm - a_b[j] * HW;
    a_y[j] = r / a.W;
    a_x[j] = r - a_y[j] * a.W;
  }

  const int nchunk = SMALLC ? 0 : a.cin_pad / BK;
  const int steps = SMALLC ? a.kpad / BK : a.KH * a.KW * nchunk;

  uint4 ra[A_PER], rb[B_PER];
  auto load = [&](int t) {
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
                              (c0 - sbase) + (e & 3) * 8;
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
          const int k = t * BK + (e & 3) * 8 + q;
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
        const int n = n0 + (e >> 2);
        v = *reinterpret_cast<const uint4*>(a.wpk + (int64_t)n * a.kpad + t * BK + (e & 3) * 8);
      }
      rb[j] = v;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int e = tid + j * NT;
      if (e < A_CHUNKS) As[buf][swz(e >> 2, e & 3)] = ra[j];
    }
#pragma unroll
    for (int j = 0; j < B_PER; ++j) {
      const int e = tid + j * NT;
      if (e < B_CHUNKS) Bs[buf][swz(e >> 2, e & 3)] = rb[j];
    }
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  load(0);
  store(0);
  __syncthreads();
  for (int t = 0; t < steps; ++t) {
    const int cur = t & 1;
    if (t + 1 < steps) load(t + 1);
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      bf16x8_t af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + (lane & 31);
        af[i] = __builtin_bit_cast(bf16x8_t, As[cur][swz(row, s * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + (lane & 31);
        bfr[j] = __builtin_bit_cast(bf16x8_t, Bs[cur][swz(row, s * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (t + 1 < steps) store(cur ^ 1);
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

template <int EPI, bool SMALLC>
void launch_cfg(const ConvFwdArgs& a, int bn, hipStream_t stream) {
  const int P = a.B * a.H * a.W;
  if (bn == 128) {
    dim3 grid(raft_cdiv(P, 128), raft_cdiv(a.cout, 128));
    hipLaunchKernelGGL((conv_fwd_kernel<128, 128, 64, 64, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
  } else if (bn == 64) {
    dim3 grid(raft_cdiv(P, 128), raft_cdiv(a.cout, 64));
    hipLaunchKernelGGL((conv_fwd_kernel<128, 64, 64, 32, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
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
