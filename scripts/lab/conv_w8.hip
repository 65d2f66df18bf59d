// LAB (not built into the library): measured and dropped in round 3 -- ties the 4-wave LDS-DMA
// kernel on every update-block layer (profiles/r3/w8/sweep_*.txt) and is neutral in the step.
// Kept as a record of the experiment; to rebuild it, copy it back into csrc/kernels and restore
// its config-table rows.
// Two-waves-per-SIMD implicit-GEMM conv kernel (see conv_igemm.hip for the GEMM view, epilogues and
// the tile-config dispatch).
//
// Why: on the one-wave-per-SIMD LDS-DMA kernel (conv_glds.hip) every K step is serial within the
// SIMD -- barrier, issue the next stage's LDS-DMA pieces (~60-100 cycles each, 9 per wave per step
// on the 160x128 tile), then the step's 20 MFMAs -- and the stamped lab kernel spent ~1.9k cycles
// per step against a 640-cycle MFMA floor (profiles/r3/conv_lab_dma_stamps.txt).  Here a
// workgroup is 8 waves (512 threads) all along N: each SIMD holds two waves, so one wave's DMA
// issue and barrier wait run beside the partner's MFMAs.  The workgroup tile is 32*TM pixels x
// 256 output channels: every A row is DMA'd once for all 256 outputs (the 128-wide tiles fetched
// the A tile twice per M row), the per-step bytes per FLOP drop by 1/3, and at TM = 5 the chairs
// geometry (M = 34,224) is one round of 214 workgroups.
//
// Same LDS image (128-B rows, XOR swizzle on the source side), same descriptors and same fused
// epilogues as the LDS-DMA kernel; one barrier per K step with NS pipeline stages.
#include "conv_common.h"

namespace conv_detail {

template <int TM, int NWN, int NS, bool BREG = false>
struct W8Tile {
  static constexpr int NTW = 64 * NWN;            // threads
  static constexpr int BM = 32 * TM, BN = 32 * NWN;
  static constexpr int A_CHUNKS = BM * 8, B_CHUNKS = BN * 8;   // 16-B slots per stage
  static constexpr int A_PER = (A_CHUNKS + NTW - 1) / NTW;     // pieces per thread (last may be partial)
  static constexpr int B_PER = BREG ? 0 : B_CHUNKS / NTW;      // BREG: B fragments go to VGPRs
  static constexpr int STAGE = A_CHUNKS + (BREG ? 0 : B_CHUNKS);
  static constexpr int LDS = NS * STAGE * 16;
  static_assert(B_CHUNKS % NTW == 0, "whole B pieces");
  static_assert(A_CHUNKS % 64 == 0, "A pieces are whole wave instructions");
  static_assert(LDS <= 160 * 1024, "LDS");
};

// pieces of the wave's stage (A pieces past the tile are skipped wave-uniformly)
template <int CNT>
__device__ __forceinline__ void w8_wait(int n) {
  // vmcnt(n) with n in {CNT, CNT - 1, ...}: a switch over the few per-wave values
  if constexpr (CNT <= 0) {
    raft_wait_vmcnt<0>();
  } else {
    if (n >= CNT) raft_wait_vmcnt<(CNT < 63 ? CNT : 63)>();
    else w8_wait<CNT - 1>(n);
  }
}

template <int TM, int NWN, int EPI, int NS, bool BREG>
__global__ __launch_bounds__(64 * NWN, 1) void conv_fwd_w8_kernel(ConvFwdArgs a) {
  using T = W8Tile<TM, NWN, NS, BREG>;
  constexpr int NTW = T::NTW, BM = T::BM, BN = T::BN, WM = 32 * TM, WN = 32;
  constexpr int A_PER = T::A_PER, B_PER = T::B_PER, A_CHUNKS = T::A_CHUNKS, STAGE = T::STAGE;
  static_assert(NS >= 2 && NS <= 3, "2..3 pipeline stages");

  __shared__ __attribute__((aligned(16))) uint4 smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  int mt, nt;
  if (!conv_tile_coords(raft_cdiv(P, BM), raft_cdiv(a.cout, BN), mt, nt)) return;
  const int m0 = mt * BM, n0 = nt * BN;

  // A pieces this wave issues (wave-uniform): piece j covers slots [j*NTW + wave*64, +64)
  int a_cnt = 0;
#pragma unroll
  for (int j = 0; j < A_PER; ++j) a_cnt += (j * NTW + wave * 64 < A_CHUNKS) ? 1 : 0;
  const int lps = a_cnt + B_PER;  // pieces per stage issued by this wave

  int a_pix[A_PER], a_y[A_PER], a_x[A_PER], a_lc[A_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * NTW;
    const int row = e >> 3;
    const int m = m0 + row;
    const bool in = e < A_CHUNKS && m < P;
    const int mm = in ? m : 0;
    const int r = mm % HW;
    a_pix[j] = mm;
    a_y[j] = in ? r / a.W : -(1 << 20);
    a_x[j] = r % a.W;
    a_lc[j] = ((e & 7) ^ ((row >> 1) & 7)) * 8;
  }
  uint32_t b_off[B_PER > 0 ? B_PER : 1];
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int e = tid + j * NTW;
    const int row = e >> 3;
    const int n = n0 + row;
    const int lc = (e & 7) ^ ((row >> 1) & 7);
    b_off[j] = n < a.cout ? (uint32_t)(((int64_t)n * a.kpad + lc * 8) * 2) : OOB;
  }
  // BREG: this lane's B fragment row (output channel) and k offset inside a 16-deep slice
  const int bn_reg = n0 + wn * 32 + (lane & 31);
  const uint32_t b_reg_off = bn_reg < a.cout ? (uint32_t)(((int64_t)bn_reg * a.kpad + (lane >> 5) * 8) * 2) : OOB;

  // K loop channel-chunk-major, taps inner (shifted reads of one 64-channel slice hit L2)
  const int nchunk = a.cin_pad / BK;
  const int ntap = a.KH * a.KW;
  const int steps = ntap * nchunk;
  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = make_rsrc(a.seg[qq].ptr, a.nullmem ? 0u : (uint32_t)P * a.seg[qq].stride * 2u);
  }
  const rsrc_t w_rs = make_rsrc(a.wpk, a.nullmem ? 0u : (uint32_t)a.cout * a.kpad * 2u);
  // B fragments of step t -> registers (4 k-slices of 16)
  auto load_b = [&](int t, bf16x8_t (&bq)[BK / 16]) {
    const int ch = t / ntap, tap = t - ch * ntap;
    const uint32_t kb = (uint32_t)((tap * a.cin_pad + ch * BK) * 2);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
      bq[kk] = __builtin_bit_cast(bf16x8_t, buf_load16(w_rs, b_reg_off == OOB ? OOB : b_reg_off + kb + kk * 32));
  };
  const uint32_t lds0 = raft_lds_addr(smem) + __builtin_amdgcn_readfirstlane(wave * 64 * 16);

  auto issue = [&](int t, int buf) {
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
    const uint32_t base = lds0 + (uint32_t)(buf * STAGE * 16);
    const uint32_t kb = (uint32_t)((tap * a.cin_pad + c0) * 2);
    // B first: every wave has the same B count, so the counted waits below see the same order
#pragma unroll
    for (int j = 0; j < B_PER; ++j)
      raft_dma16(w_rs, base + (A_CHUNKS + j * NTW) * 16, b_off[j] == OOB ? OOB : b_off[j] + kb);
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      if (j * NTW + wave * 64 < A_CHUNKS) {  // wave-uniform
        const int yy = a_y[j] + dy, xx = a_x[j] + dx;
        const bool ok = (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
        const uint32_t off = (uint32_t)(((a_pix[j] + dpix) * stride + coff + a_lc[j]) * 2);
        raft_dma16(rs, base + j * NTW * 16, ok ? off : OOB);
      }
    }
  };

  f32x16 acc[TM][1];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][0][r] = 0.f;

  // the wave's output columns lie past cout (Cout 192 on a 256-wide tile): no MFMAs, loads only
  const bool live = n0 + wn * WN < a.cout;

  auto compute = [&](int buf, const bf16x8_t (&breg)[BK / 16]) {
    const uint4* As = smem + buf * STAGE;
    const uint4* Bs = As + A_CHUNKS;
    bf16x8_t af[BK / 16][TM], bfr[BK / 16];
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int brow = wn * WN + (lane & 31);
      if constexpr (BREG) bfr[kk] = breg[kk];
      else bfr[kk] = __builtin_bit_cast(bf16x8_t, Bs[swz(brow, kk * 2 + (lane >> 5))]);
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = i * 32 + (lane & 31);
        af[kk][i] = __builtin_bit_cast(bf16x8_t, As[swz(row, kk * 2 + (lane >> 5))]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
        acc[i][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[kk][i], bfr[kk], acc[i][0], 0, 0, 0);
    __builtin_amdgcn_sched_group_barrier(0x100, (BK / 16) * (TM + (BREG ? 0 : 1)), 0);
    __builtin_amdgcn_sched_group_barrier(0x008, (BK / 16) * TM, 0);
  };

  bf16x8_t bq0[BK / 16], bq1[BK / 16];
#pragma unroll
  for (int kk = 0; kk < BK / 16; ++kk) bq0[kk] = bq1[kk] = zero_frag8();
  if constexpr (BREG) load_b(0, bq0);
#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < steps) issue(s, s);
  int cur = 0;
  // one K step: wait for its operands, barrier, issue the stages / B fragments ahead, MFMAs
  auto step = [&](int t, const bf16x8_t (&bc)[BK / 16], bf16x8_t (&bn)[BK / 16]) {
    const int newer = min(NS - 2, steps - 1 - t);
    if (NS >= 3 && newer >= 1) w8_wait<(NS >= 3 ? A_PER + B_PER + (BREG ? BK / 16 : 0) : 0)>(lps + (BREG ? BK / 16 : 0));
    else raft_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < steps) {
      int nb = cur + NS - 1;
      nb = nb >= NS ? nb - NS : nb;
      issue(t + NS - 1, nb);
    }
    if constexpr (BREG) {
      if (t + 1 < steps) load_b(t + 1, bn);
    }
    if (live) compute(cur, bc);
    cur = cur + 1 == NS ? 0 : cur + 1;
  };
  for (int t = 0; t < steps; t += 2) {
    step(t, bq0, bq1);
    if (t + 1 < steps) step(t + 1, bq1, bq0);
  }

  conv_epilogue<TM, 1, WM, WN, EPI>(a, acc, m0, n0, 0, wn, lane, P, HW);
}

template <int EPI, int TM, int NWN, int NS, bool BREG = false>
void launch_one_w8(const ConvFwdArgs& a, hipStream_t stream) {
  using T = W8Tile<TM, NWN, NS, BREG>;
  const int P = a.B * a.H * a.W;
  dim3 grid(conv_grid_1d(raft_cdiv(P, T::BM), raft_cdiv(a.cout, T::BN)));
  hipLaunchKernelGGL((conv_fwd_w8_kernel<TM, NWN, EPI, NS, BREG>), grid, dim3(T::NTW), 0, stream, a);
}

template <int EPI>
bool launch_w8_epi(const ConvFwdArgs& a, int tm, int ns, hipStream_t stream) {
  if (tm == 5 && ns == 2) { launch_one_w8<EPI, 5, 8, 2>(a, stream); return true; }
  if (tm == 5 && ns == 3) { launch_one_w8<EPI, 5, 8, 3>(a, stream); return true; }
  return false;
}

}  // namespace conv_detail

// 8-wave tile (32*tm pixels x 256 channels, `ns` stages); false if the geometry is not offered
bool launch_conv_w8(const ConvFwdArgs& a, int epi, int tm, int ns, hipStream_t stream) {
  using namespace conv_detail;
  if (a.cin_small || a.cin_pad % BK != 0) return false;
  for (int q = 0; q < a.nseg; ++q)
    if (a.seg[q].cnt % BK) return false;  // the K loop advances whole 64-channel chunks per segment
  switch (epi) {
    case EPI_BF16: return launch_w8_epi<EPI_BF16>(a, tm, ns, stream);
    case EPI_RELU_BF16: return launch_w8_epi<EPI_RELU_BF16>(a, tm, ns, stream);
    case EPI_F32: return launch_w8_epi<EPI_F32>(a, tm, ns, stream);
    case EPI_ACC_F32: return launch_w8_epi<EPI_ACC_F32>(a, tm, ns, stream);
    case EPI_GRU_ZR: return launch_w8_epi<EPI_GRU_ZR>(a, tm, ns, stream);
    case EPI_GRU_Q: return launch_w8_epi<EPI_GRU_Q>(a, tm, ns, stream);
    case EPI_DGRAD: return launch_w8_epi<EPI_DGRAD>(a, tm, ns, stream);
    case EPI_DGRAD_GATE: return launch_w8_epi<EPI_DGRAD_GATE>(a, tm, ns, stream);
    case EPI_F32_NCHW: return launch_w8_epi<EPI_F32_NCHW>(a, tm, ns, stream);
    default: return false;
  }
}
