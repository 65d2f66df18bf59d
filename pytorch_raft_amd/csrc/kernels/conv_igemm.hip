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
#include "conv_common.h"

#include <type_traits>
#include "conv_halo.h"

#include <cmath>
#include <cstdlib>
#include <map>
#include <mutex>
#include <tuple>

namespace {
using namespace conv_detail;
// Pipeline (per 64-deep K step, one barrier):  global loads for step t+2 are issued into one of
// two register sets before the MFMAs of step t (two steps = ~1000+ MFMA cycles of latency cover),
// the other set (step t+1, loaded one step earlier) is written to the idle LDS buffer after them.
// Wave tile (32*TM) x (32*TN); WVM x (4/WVM) waves -> block tile BM x BN.  Larger wave tiles
// cut LDS traffic per MFMA ((TM+TN)/(TM*TN) fragment reads per MFMA): at 2x2 the four SIMDs
// already need the LDS's full 128 B/clk, so the big-M configs (4x2, 5x2) exist for that reason.


template <int TM, int TN, int WVM, int EPI, bool SMALLC>
__global__ __launch_bounds__(NT, (ConvTile<TM, TN, WVM>::OCC)) void conv_fwd_kernel(ConvFwdArgs a) {
  using T = ConvTile<TM, TN, WVM>;
  constexpr int BM = T::BM, BN = T::BN, WM = 32 * TM, WN = 32 * TN;
  constexpr int WAVES_N = T::WVN;
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
  int mt, nt;
  if (!conv_tile_coords(raft_cdiv(P, BM), raft_cdiv(a.cout, BN), mt, nt)) return;
  const int m0 = mt * BM, n0 = nt * BN;

  // per-thread A rows (fixed over the K loop): chunk e -> row e>>3, 16-B column e&7;
  // (pixel index, y, x) with y = -2^20 marking rows past P
  int a_pix[A_PER], a_y[A_PER], a_x[A_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * NT;
    const int m = m0 + (e >> 3);
    const int mm = m < P ? m : 0;
    const int r = mm % HW;
    a_pix[j] = mm;
    a_y[j] = m < P ? r / a.W : -(1 << 20);
    a_x[j] = r % a.W;
  }

  const int nchunk = SMALLC ? 0 : tile_nchunk(a, n0, BN);
  const int ntap = a.KH * a.KW;
  const int steps = SMALLC ? a.kpad / BK : ntap * nchunk;   // channel-chunk-major (conv_glds.hip)
  // buffer descriptors: out-of-range offsets (padding taps, rows past P, weight rows past cout)
  // read as zeros with no branch and no register pre-zeroing
  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = make_rsrc(a.seg[qq].ptr, (uint32_t)P * a.seg[qq].stride * 2u);
  }
  const rsrc_t w_rs = make_rsrc(a.wpk, (uint32_t)a.cout * a.kpad * 2u);

  auto load = [&](int t, uint4 (&ra)[A_PER], uint4 (&rb)[B_PER]) {
    if constexpr (!SMALLC) {
      const int ch = t / ntap, tap = t - ch * ntap;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
      const int c0 = ch * BK;
      int s = 0, sbase = 0;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (s + 1 < a.nseg && c0 >= sbase + a.seg[s].cnt) { sbase += a.seg[s].cnt; ++s; }
      const rsrc_t rs = s == 0 ? seg_rs[0] : (s == 1 ? seg_rs[1] : seg_rs[2]);
      const int stride = a.seg[s].stride;
      const int dy = kh - a.PH, dx = kw - a.PW;
      const int dpix = dy * a.W + dx;
      const int coff = c0 - sbase;
      const int creal = a.seg[s].real;
#pragma unroll
      for (int j = 0; j < A_PER; ++j) {
        const int e = tid + j * NT;
        const int yy = a_y[j] + dy, xx = a_x[j] + dx;
        const bool ok = (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W &&
                        coff + (e & 7) * 8 < creal;
        const uint32_t off = (uint32_t)(((a_pix[j] + dpix) * stride + coff + (e & 7) * 8) * 2);
        ra[j] = buf_load16(rs, ok ? off : OOB);
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
          if (a_y[j] >= 0 && k < ktot) {
            const int tap = k / cs, c = k - tap * cs;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            const int yy = a_y[j] + kh - a.PH, xx = a_x[j] + kw - a.PW;
            if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
              v = sg.ptr[(int64_t)(a_pix[j] + (kh - a.PH) * a.W + (kw - a.PW)) * sg.stride + c];
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
      const int n = n0 + (e >> 3);
      // rows past cout read as zeros (range-checked descriptor); the packed tensor may end there
      int kcol = t * BK;
      if constexpr (!SMALLC) {
        const int ch = t / ntap, tap = t - ch * ntap;
        kcol = tap * a.cin_pad + ch * BK;
      }
      const uint32_t off = (uint32_t)(((int64_t)n * a.kpad + kcol + (e & 7) * 8) * 2);
      rb[j] = buf_load16(w_rs, e < B_CHUNKS ? off : OOB);
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
          acc[i][j] = mfma16<epi_f16(EPI)>(af[i], bfr[j], acc[i][j]);
    }
  };

  if constexpr (TM * TN >= 8) {
    // big wave tiles: one register set (the step's 32+ MFMAs per wave cover one load latency)
    uint4 ra[A_PER], rb[B_PER];
    const int last = steps - 1;
    load(0, ra, rb);
    store(0, ra, rb);
    __syncthreads();
    for (int t = 0; t < steps; ++t) {
      const int cur = t & 1;
      load(min(t + 1, last), ra, rb);
      compute(cur);
      store(cur ^ 1, ra, rb);
      __syncthreads();
    }
  } else {
    // loads / stores are unconditional (the last steps re-load the final K step): no branch
    // around a memory op, so hipcc's counted waits keep the newer register set in flight
    uint4 ra0[A_PER], rb0[B_PER], ra1[A_PER], rb1[B_PER];
    const int last = steps - 1;
    load(0, ra0, rb0);
    load(min(1, last), ra1, rb1);
    store(0, ra0, rb0);
    __syncthreads();
    for (int t = 0; t < steps; t += 2) {
      // even step: LDS[0] = step t, regs1 = step t+1 (in flight), regs0 free
      load(min(t + 2, last), ra0, rb0);
      compute(0);
      store(1, ra1, rb1);
      __syncthreads();
      if (t + 1 >= steps) break;
      // odd step: LDS[1] = step t+1, regs0 = step t+2 (in flight), regs1 free
      load(min(t + 3, last), ra1, rb1);
      compute(1);
      store(0, ra0, rb0);
      __syncthreads();
    }
  }

  conv_epilogue<TM, TN, WM, WN, EPI>(a, acc, m0, n0, wm, wn, lane, P, HW);
}

// ------------------------------------------------------------------ tile configurations
struct CfgDesc {
  int tm, tn, wvm, bm, bn;
  bool small_ok;
  int glds;  // 0: register-staged kernel; n: LDS-DMA kernel with n pipeline stages; HALO
};
constexpr int HALO = 9;
// (keep in sync with the dispatch switch below)
constexpr CfgDesc kCfgs[] = {
    {2, 2, 2, 128, 128, true, false},  {1, 2, 2, 64, 128, true, false},
    {2, 1, 2, 128, 64, false, false},  {1, 1, 2, 64, 64, false, false},
    {1, 1, 4, 128, 32, true, false},   {4, 2, 2, 256, 128, false, false},
    {5, 2, 1, 160, 256, false, false}, {5, 1, 1, 160, 128, false, false},
    {4, 2, 1, 128, 256, false, false}, {3, 2, 1, 96, 256, false, false},
    // LDS-DMA variants (last field: pipeline stages)
    {2, 2, 2, 128, 128, false, 2},  {1, 2, 2, 64, 128, false, 2},
    {2, 1, 2, 128, 64, false, 2},   {4, 2, 2, 256, 128, false, 2},
    {4, 2, 1, 128, 256, false, 2},  {3, 2, 1, 96, 256, false, 2},
    {5, 1, 1, 160, 128, false, 2},  {1, 1, 2, 64, 64, false, 2},
    {2, 2, 2, 128, 128, false, 4},  {1, 2, 2, 64, 128, false, 3},
    {5, 1, 1, 160, 128, false, 4},  {2, 1, 2, 128, 64, false, 4},
    {1, 1, 2, 64, 64, false, 4},    {4, 2, 1, 128, 256, false, 3},
    {3, 1, 1, 96, 128, false, 4},   {3, 1, 1, 96, 128, false, 2},
    // one-round tiles for M = 34,224 (chairs, B = 12): 214 / 238 / 179 workgroups
    {5, 2, 1, 160, 256, false, 2},  {5, 2, 1, 160, 256, false, 3},
    {9, 1, 1, 288, 128, false, 2},  {3, 3, 2, 192, 192, false, 2},
    // halo-tile kernel (conv_halo.h; glds = HALO): A image per channel chunk, B straight to VGPRs
    {5, 1, 1, 160, 128, false, HALO}, {5, 2, 1, 160, 256, false, HALO},
    {4, 2, 1, 128, 256, false, HALO}, {2, 2, 2, 128, 128, false, HALO},
};
constexpr int kNumCfgs = sizeof(kCfgs) / sizeof(kCfgs[0]);

template <int EPI, bool SMALLC, int TM, int TN, int WVM>
void launch_one(const ConvFwdArgs& a, hipStream_t stream) {
  using T = ConvTile<TM, TN, WVM>;
  const int P = a.B * a.H * a.W;
  dim3 grid(conv_grid_1d(raft_cdiv(P, T::BM), raft_cdiv(a.cout, T::BN)));
  hipLaunchKernelGGL((conv_fwd_kernel<TM, TN, WVM, EPI, SMALLC>), grid, dim3(NT), 0, stream, a);
}


template <int EPI, bool SMALLC>
bool launch_cfg_idx(const ConvFwdArgs& a, int idx, hipStream_t stream) {
  if constexpr (epi_f16(EPI)) {
    // fp16 operands: LDS-DMA and halo kernels only
    if (SMALLC || idx < 0 || idx >= kNumCfgs || !kCfgs[idx].glds) return false;
    if (kCfgs[idx].glds == HALO)
      return launch_conv_halo(a, EPI, kCfgs[idx].tm, kCfgs[idx].tn, kCfgs[idx].wvm, stream);
    return launch_conv_glds(a, EPI, idx, stream);
  } else if constexpr (SMALLC) {
    switch (idx) {
      case 0: launch_one<EPI, true, 2, 2, 2>(a, stream); return true;
      case 1: launch_one<EPI, true, 1, 2, 2>(a, stream); return true;
      case 4: launch_one<EPI, true, 1, 1, 4>(a, stream); return true;
      default: return false;
    }
  } else {
    switch (idx) {
      case 0: launch_one<EPI, false, 2, 2, 2>(a, stream); return true;
      case 1: launch_one<EPI, false, 1, 2, 2>(a, stream); return true;
      case 2: launch_one<EPI, false, 2, 1, 2>(a, stream); return true;
      case 3: launch_one<EPI, false, 1, 1, 2>(a, stream); return true;
      case 4: launch_one<EPI, false, 1, 1, 4>(a, stream); return true;
      case 5: launch_one<EPI, false, 4, 2, 2>(a, stream); return true;
      case 6:  // the GRU epilogues spill at this tile (160 fp32 accumulators + gate math)
        if constexpr (EPI == EPI_GRU_ZR || EPI == EPI_GRU_Q) return false;
        else { launch_one<EPI, false, 5, 2, 1>(a, stream); return true; }
      case 7: launch_one<EPI, false, 5, 1, 1>(a, stream); return true;
      case 8: launch_one<EPI, false, 4, 2, 1>(a, stream); return true;
      case 9: launch_one<EPI, false, 3, 2, 1>(a, stream); return true;
      default:
        if (idx >= 0 && idx < kNumCfgs && kCfgs[idx].glds == HALO)
          return launch_conv_halo(a, EPI, kCfgs[idx].tm, kCfgs[idx].tn, kCfgs[idx].wvm, stream);
        if (idx >= 0 && idx < kNumCfgs && kCfgs[idx].glds) return launch_conv_glds(a, EPI, idx, stream);
        return false;
    }
  }
}

bool launch_epi_idx(const ConvFwdArgs& a, int epi, int idx, bool smallc, hipStream_t stream) {
#define RAFT_EPI_CASE(E) \
  case E: return smallc ? launch_cfg_idx<E, true>(a, idx, stream) : launch_cfg_idx<E, false>(a, idx, stream);
  switch (epi) {
    RAFT_EPI_CASE(EPI_BF16)
    RAFT_EPI_CASE(EPI_RELU_BF16)
    RAFT_EPI_CASE(EPI_F32)
    RAFT_EPI_CASE(EPI_ACC_F32)
    RAFT_EPI_CASE(EPI_DGRAD)
    case EPI_DGRAD_GATE: return !smallc && launch_cfg_idx<EPI_DGRAD_GATE, false>(a, idx, stream);
    RAFT_EPI_CASE(EPI_F32_NCHW)
    case EPI_GRU_ZR: return !smallc && launch_cfg_idx<EPI_GRU_ZR, false>(a, idx, stream);
    case EPI_GRU_Q: return !smallc && launch_cfg_idx<EPI_GRU_Q, false>(a, idx, stream);
    case EPI_BF16 | EPI_F16: return launch_cfg_idx<EPI_BF16 | EPI_F16, false>(a, idx, stream);
    case EPI_RELU_BF16 | EPI_F16: return launch_cfg_idx<EPI_RELU_BF16 | EPI_F16, false>(a, idx, stream);
    case EPI_F32 | EPI_F16: return launch_cfg_idx<EPI_F32 | EPI_F16, false>(a, idx, stream);
    case EPI_GRU_ZR | EPI_F16: return launch_cfg_idx<EPI_GRU_ZR | EPI_F16, false>(a, idx, stream);
    case EPI_GRU_Q | EPI_F16: return launch_cfg_idx<EPI_GRU_Q | EPI_F16, false>(a, idx, stream);
    case EPI_DGRAD | EPI_F16: return launch_cfg_idx<EPI_DGRAD | EPI_F16, false>(a, idx, stream);
    case EPI_DGRAD_GATE | EPI_F16: return launch_cfg_idx<EPI_DGRAD_GATE | EPI_F16, false>(a, idx, stream);
    case EPI_F32_NCHW | EPI_F16: return launch_cfg_idx<EPI_F32_NCHW | EPI_F16, false>(a, idx, stream);
    default:
      // split fp32 (ConvFwdArgs.spl): LDS-DMA / halo configs only (cfg_allowed), dispatched by
      // conv_glds.hip / conv_halo_6.hip on the full epilogue id
      if (epi_spl(epi) && !epi_f16(epi) && !smallc && idx >= 0 && idx < kNumCfgs && kCfgs[idx].glds) {
        if (kCfgs[idx].glds == HALO)
          return launch_conv_halo(a, epi, kCfgs[idx].tm, kCfgs[idx].tn, kCfgs[idx].wvm, stream);
        return launch_conv_glds(a, epi, idx, stream);
      }
      return false;
  }
#undef RAFT_EPI_CASE
}

bool halo_disabled() {
  static const bool off = [] {
    const char* e = getenv("RAFT_CONV_HALO");
    return e && e[0] == '0';
  }();
  return off;
}

bool glds_disabled() {
  static const bool off = [] {
    const char* e = getenv("RAFT_CONV_GLDS");
    return e && e[0] == '0';
  }();
  return off;
}

bool cfg_allowed(int idx, int cout, bool smallc, int epi) {
  const CfgDesc& c = kCfgs[idx];
  // fp16 / split fp32: LDS-DMA / halo kernels only
  if ((epi_f16(epi) || epi_spl(epi)) && (smallc || !c.glds)) return false;
  if (smallc && !c.small_ok) return false;
  if (c.glds && glds_disabled()) return false;
  if (c.glds == HALO && halo_disabled()) return false;
  if (idx == 6 && (epi_kind(epi) == EPI_GRU_ZR || epi_kind(epi) == EPI_GRU_Q)) return false;
  const int npad = (cout + 31) / 32 * 32;
  return c.bn <= 2 * npad || c.bn <= 32;  // no config more than half empty in N
}

// Analytic fallback (stream capture / autotune disabled): rounds of workgroups x tile cost,
// with the 2x2-wave tiles' LDS-bandwidth penalty.
int heuristic_cfg(int P, int cout, bool smallc, int epi) {
  const bool f16 = epi_f16(epi) || epi_spl(epi);  // fp16 / split: the 2-stage LDS-DMA configs
  double best = 1e30;
  int bi = f16 ? 17 : 0;
  for (int i = 0; i < kNumCfgs; ++i) {
    if (!cfg_allowed(i, cout, smallc, epi) || (f16 ? kCfgs[i].glds != 2 : kCfgs[i].glds != 0)) continue;
    const CfgDesc& c = kCfgs[i];
    const int tiles = raft_cdiv(P, c.bm) * raft_cdiv(cout, c.bn);
    const int occ = (2 * (c.bm + c.bn) * 128 <= 65536 && c.tm * c.tn <= 4) ? 2 : 1;
    const double rounds = std::ceil(tiles / (256.0 * occ));
    const double ratio = double(c.tm + c.tn) / double(c.tm * c.tn);  // LDS KB per MFMA
    const double eff = std::min(1.0, 0.8 / ratio);
    const double cost = rounds * c.bm * c.bn / (eff * occ);
    if (cost < best) { best = cost; bi = i; }
  }
  return bi;
}

struct TuneKey {
  int P, H, W, KH, KW, cin, cout, small, f32out, creal;
  bool operator<(const TuneKey& o) const {
    return std::tie(P, H, W, KH, KW, cin, cout, small, f32out, creal) <
           std::tie(o.P, o.H, o.W, o.KH, o.KW, o.cin, o.cout, o.small, o.f32out, o.creal);
  }
};
std::map<TuneKey, int> g_tuned;
std::mutex g_tune_mu;
float* g_scratch = nullptr;
size_t g_scratch_bytes = 0;
void* g_scratch2 = nullptr;   // redirected outputs of input-gradient convs under autotune
size_t g_scratch2_bytes = 0;

bool tune_real_dgrad() {
  static const bool on = [] {
    const char* e = getenv("RAFT_TUNE_REAL_DGRAD");  // 0: time dgrads on the fp32 scratch store
    return !(e && e[0] == '0');
  }();
  return on;
}

// byte range [lo, hi) of a per-pixel NHWC buffer (P rows of `stride` elements of `esz` bytes)
struct Range { uintptr_t lo, hi; };
inline Range nhwc_range(const void* p, int P, int stride, int esz) {
  const uintptr_t lo = (uintptr_t)p;
  return Range{lo, p ? lo + (uintptr_t)P * (uintptr_t)stride * (uintptr_t)esz : lo};
}
inline bool ranges_meet(Range x, Range y) { return x.lo < x.hi && y.lo < y.hi && x.lo < y.hi && y.lo < x.hi; }

bool outputs_overlap_inputs(const ConvFwdArgs& a, int epi_any) {
  const int epi = epi_kind(epi_any);
  const int P = a.B * a.H * a.W;
  const bool f32 = epi == EPI_F32 || epi == EPI_F32_NCHW;
  Range outs[3] = {nhwc_range(a.out0, P, epi == EPI_F32_NCHW ? a.cout : a.out0_stride, f32 ? 4 : 2),
                   nhwc_range(a.out1, P, a.out1_stride, 2), nhwc_range(a.out2, P, a.out2_stride, 2)};
  const int nout = epi == EPI_GRU_ZR ? 3 : (epi == EPI_GRU_Q ? 2 : 1);
  Range ins[6];
  int nin = 0;
  for (int q = 0; q < a.nseg && q < 3; ++q) ins[nin++] = nhwc_range(a.seg[q].ptr, P, a.seg[q].stride, 2);
  if (epi == EPI_GRU_ZR || epi == EPI_GRU_Q) {
    ins[nin++] = nhwc_range(a.aux0, P, a.aux0_stride, 2);
    if (epi == EPI_GRU_Q) ins[nin++] = nhwc_range(a.aux1, P, a.aux1_stride, 2);
    if (a.bmap) ins[nin++] = nhwc_range(a.bmap, P, a.bmap_stride, a.bmap_bf16 ? 2 : 4);
  }
  for (int o = 0; o < nout; ++o)
    for (int i = 0; i < nin; ++i)
      if (ranges_meet(outs[o], ins[i])) return true;
  return false;
}

// Time every allowed config on the real operands (output into a private scratch buffer
// through the fp32 epilogue) and cache the fastest.  Runs only outside stream capture.
int autotune(const ConvFwdArgs& a, int epi, bool smallc, hipStream_t stream) {
  const int P = a.B * a.H * a.W;
  const size_t need = (size_t)P * ((a.cout + 255) / 256 * 256) * sizeof(float);
  if (need > g_scratch_bytes) {
    if (g_scratch) (void)hipFree(g_scratch);
    if (hipMalloc(&g_scratch, need) != hipSuccess) { g_scratch = nullptr; g_scratch_bytes = 0; return -1; }
    g_scratch_bytes = need;
  }
  ConvFwdArgs t = a;
  t.out0 = g_scratch;
  t.out0_stride = (a.cout + 255) / 256 * 256;
  t.noseg = 0;
  // input-gradient convs: timed with their REAL epilogue (the fused GRU gate backward moves as
  // many bytes as its GEMM), every written / read-modify-written pointer redirected into scratch
  const int ek = epi_kind(epi);
  const bool dgrad_real = (ek == EPI_DGRAD || ek == EPI_DGRAD_GATE) && tune_real_dgrad();
  ConvFwdArgs td = a;
  if (dgrad_real) {
    size_t tot = 0;
    auto sz = [&](const void* p, int stride, int esz) {
      return p ? ((size_t)P * stride * esz + 255) / 256 * 256 : (size_t)0;
    };
    for (int o = 0; o < a.noseg; ++o) {
      const OSeg& q = a.oseg[o];
      tot += sz(q.ptr, q.stride, 4) + sz(q.ob, q.ob_stride, 2) + sz(q.gb, q.gb_stride, 2) +
             sz(q.gz, q.gz_stride, 2) + sz(q.gf1, q.gf_stride, 4);
    }
    if (tot > g_scratch2_bytes) {
      if (g_scratch2) (void)hipFree(g_scratch2);
      if (hipMalloc(&g_scratch2, tot) != hipSuccess) { g_scratch2 = nullptr; g_scratch2_bytes = 0; tot = 0; }
      else g_scratch2_bytes = tot;
    }
    if (g_scratch2 != nullptr && tot > 0) {
      char* cur = static_cast<char*>(g_scratch2);
      auto take = [&](auto* p, int stride, int esz) {
        using T = std::remove_pointer_t<std::remove_reference_t<decltype(p)>>;
        if (!p) return p;
        T* r = reinterpret_cast<T*>(cur);
        cur += sz(p, stride, esz);
        return r;
      };
      for (int o = 0; o < a.noseg; ++o) {
        OSeg& q = td.oseg[o];
        q.ptr = take(q.ptr, q.stride, 4);
        q.ob = take(q.ob, q.ob_stride, 2);
        q.gb = take(q.gb, q.gb_stride, 2);
        q.gz = take(q.gz, q.gz_stride, 2);
        q.gf1 = take(q.gf1, q.gf_stride, 4);
      }
    }
  }
  // store-only epilogues are timed as they will run (the GRU gate epilogues cost registers and
  // bytes the fp32 scratch epilogue does not): their outputs are rewritten by the real launch
  // that follows; accumulating epilogues (ACC_F32, DGRAD) are timed on the fp32 scratch
  bool real_epi = ek == EPI_BF16 || ek == EPI_RELU_BF16 || ek == EPI_GRU_ZR ||
                  ek == EPI_GRU_Q || ek == EPI_F32 || ek == EPI_F32_NCHW;
  // ... but only while no output overlaps an operand the launches read (an in-place GRU state
  // update, say): repeated candidate launches would then read their own outputs
  if (real_epi && outputs_overlap_inputs(a, epi)) real_epi = false;
  const bool dgr = dgrad_real && g_scratch2 != nullptr;
  const ConvFwdArgs& ta = dgr ? td : (real_epi ? a : t);
  const int te = (real_epi || dgr) ? epi : (EPI_F32 | (epi & (EPI_F16 | EPI_SPL)));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  int best = -1;
  float best_ms = 1e30f;
  static const int trials = [] {
    const char* e = getenv("RAFT_CONV_TUNE_TRIALS");  // more trials when building tune_db/
    const int n = e ? atoi(e) : 3;
    return n < 1 ? 1 : (n > 50 ? 50 : n);
  }();
  for (int i = 0; i < kNumCfgs; ++i) {
    if (!cfg_allowed(i, a.cout, smallc, epi)) continue;
    if (!launch_epi_idx(ta, te, i, smallc, stream)) continue;  // warm (code load, caches)
    // min over 3 trials of 2 launches: one noisy trial (clock ramp, a co-running stream) must
    // not flip the choice -- run-to-run step time varied by ~0.8 ms with single-trial timing
    float ms = 1e30f;
    for (int trial = 0; trial < trials; ++trial) {
      (void)hipEventRecord(e0, stream);
      for (int r = 0; r < 2; ++r) launch_epi_idx(ta, te, i, smallc, stream);
      (void)hipEventRecord(e1, stream);
      (void)hipEventSynchronize(e1);
      float tms = 0.f;
      (void)hipEventElapsedTime(&tms, e0, e1);
      ms = fminf(ms, tms);
    }
    if (ms < best_ms) { best_ms = ms; best = i; }
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return best;
}

int g_forced_cfg = -1;
int g_autotune_override = -1;  // -1: RAFT_CONV_AUTOTUNE decides; 0 / 1: off / on (data parallel)
int g_autotune_runs = 0;

int choose_cfg(const ConvFwdArgs& a, int epi, bool smallc, hipStream_t stream) {
  if (g_forced_cfg >= 0) return g_forced_cfg;
  static const int forced = [] {
    const char* e = getenv("RAFT_CONV_CFG");
    return e ? atoi(e) : -1;
  }();
  static const bool tune = [] {
    const char* e = getenv("RAFT_CONV_AUTOTUNE");
    return !(e && e[0] == '0');
  }();
  const int P = a.B * a.H * a.W;
  if (forced >= 0 && forced < kNumCfgs && cfg_allowed(forced, a.cout, smallc, epi)) return forced;
  const int ek = epi_kind(epi);
  const bool f32out = ek == EPI_F32 || ek == EPI_ACC_F32 || ek == EPI_DGRAD ||
                      ek == EPI_F32_NCHW;
  // the gated input-gradient convs tune apart from the plain ones of the same geometry (their
  // epilogue is timed for real); fp16 operands tune apart from bf16 (LDS-DMA / halo only)
  const int eclass = (ek == EPI_DGRAD_GATE ? 3
                      : (f32out ? 1 : ((ek == EPI_GRU_ZR || ek == EPI_GRU_Q) ? 2 : 0))) +
                     (epi_f16(epi) ? 4 : 0) + (epi_spl(epi) ? 8 : 0);
  int creal = 0;
  for (int q = 0; q < a.nseg && q < 3; ++q) creal += a.seg[q].real;
  const TuneKey key{P, a.H, a.W, a.KH, a.KW, smallc ? a.cin_small : a.cin_pad, a.cout, (int)smallc,
                    eclass, creal};
  std::lock_guard<std::mutex> lk(g_tune_mu);
  auto it = g_tuned.find(key);
  if (it != g_tuned.end()) return it->second;
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  (void)hipStreamIsCapturing(stream, &cs);
  int idx = -1;
  const bool tune_now = g_autotune_override >= 0 ? g_autotune_override == 1 : tune;
  if (tune_now && cs == hipStreamCaptureStatusNone) {
    idx = autotune(a, epi, smallc, stream);
    ++g_autotune_runs;
  }
  if (idx < 0) idx = heuristic_cfg(P, a.cout, smallc, epi);
  if (cs == hipStreamCaptureStatusNone) g_tuned[key] = idx;
  return idx;
}

}  // namespace

bool launch_conv_fwd(const ConvFwdArgs& a, int epi, int bn, bool smallc, hipStream_t stream) {
  (void)bn;  // tile shape is chosen per geometry (autotuned once, cached)
  const int idx = choose_cfg(a, epi, smallc, stream);
  if (launch_epi_idx(a, epi, idx, smallc, stream)) return true;
  // a cached pick is shared by the epilogues of one class (TuneKey.f32out); should it not offer
  // this epilogue, the analytic register-staged choice (every epilogue instantiated) runs instead
  return launch_epi_idx(a, epi, heuristic_cfg(a.B * a.H * a.W, a.cout, smallc, epi), smallc, stream);
}

void conv_set_forced_cfg(int idx) { g_forced_cfg = idx < kNumCfgs ? idx : -1; }

void conv_set_autotune(int mode) { g_autotune_override = mode < 0 ? -1 : (mode ? 1 : 0); }

int conv_autotune_runs() { return g_autotune_runs; }

int conv_import_tuned(const int* rows, int n) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  int done = 0;
  for (int i = 0; i < n; ++i) {
    const int* r = rows + 13 * i;
    if (r[9] < 0 || r[9] >= kNumCfgs) continue;  // a table from another build: keep our choice
    // the row names its config by index AND tile shape: a renumbered config table since the row
    // was written leaves the key to the autotuner instead of launching the wrong tile
    if (kCfgs[r[9]].bm != r[10] || kCfgs[r[9]].bn != r[11]) continue;
    const int ec = r[8];  // TuneKey.f32out: the epilogue class of choose_cfg
    const int epi = ((ec & 3) == 2 ? EPI_GRU_ZR : EPI_BF16) | ((ec & 4) ? EPI_F16 : 0) | ((ec & 8) ? EPI_SPL : 0);
    if (!cfg_allowed(r[9], r[6], r[7] != 0, epi)) continue;
    g_tuned[TuneKey{r[0], r[1], r[2], r[3], r[4], r[5], r[6], r[7], r[8], r[12]}] = r[9];
    ++done;
  }
  return done;
}

int conv_tuned_table(int* out, int max_rows) {
  std::lock_guard<std::mutex> lk(g_tune_mu);
  int n = 0;
  for (const auto& kv : g_tuned) {
    if (n >= max_rows) break;
    const TuneKey& k = kv.first;
    const CfgDesc& c = kCfgs[kv.second];
    const int row[13] = {k.P, k.H, k.W, k.KH, k.KW, k.cin, k.cout, k.small, k.f32out, kv.second,
                         c.bm, c.bn, k.creal};
    for (int i = 0; i < 13; ++i) out[n * 13 + i] = row[i];
    ++n;
  }
  return n;
}
