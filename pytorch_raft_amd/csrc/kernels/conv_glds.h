// LDS-DMA pipelined implicit-GEMM conv kernel (see conv_igemm.hip for the GEMM view, epilogues
// and the tile-config dispatch).  Instantiated by conv_glds.hip (bf16 operands) and
// conv_glds_f16.hip (fp16 operands) -- separate translation units, so the instantiations (tile
// shapes x pipeline depths x epilogues x operand types) compile in parallel.
#pragma once
#include "conv_common.h"

#ifndef RAFT_CONV_UPFRONT
#define RAFT_CONV_UPFRONT 1
#endif

namespace conv_detail {

// ------------------------------------------------------------------ LDS-DMA variant
// Same tiling / epilogues, but the A (input patch) and B (weight) tiles go global -> LDS with
// buffer_load_dwordx4 ... lds: no staging VGPRs and no ds_write pass (on the register-staged
// kernel the 13-cycle ds_write_b128 transfers cost as much LDS time as the fragment reads).
// The DMA image is lane-linear (wave-uniform M0 base + 16 B x lane), so the XOR swizzle is
// applied on the SOURCE side: the lane that lands in physical 16-B slot `pc` of row `row` loads
// logical chunk pc ^ ((row >> 1) & 7); fragment reads use the same swz() as the register kernel.
// Out-of-range taps / rows read as zeros through the range-checked descriptor (the DMA writes
// the zeros).
// NS-stage pipeline, ONE barrier per K step:  wait (counted vmcnt) for this wave's step-t DMAs
// with the newer stages still in flight -> barrier (all waves' step-t data landed AND all waves
// finished computing step t-1) -> issue step t+NS-1 into the buffer step t-1 used -> MFMAs on t.
template <int TM, int TN, int WVM, int NS>
struct GldsTile {
  static constexpr int BM = 32 * TM * WVM, BN = 32 * TN * (4 / WVM);
  static constexpr int STAGE_BYTES = (BM + BN) * 128;
  static constexpr int LDS = NS * STAGE_BYTES;
  static constexpr int OCC = (LDS <= 80 * 1024 && TM * TN <= 4) ? 2 : 1;
};

template <int TM, int TN, int WVM, int EPI, int NS>
__global__ __launch_bounds__(NT, (GldsTile<TM, TN, WVM, NS>::OCC)) void conv_fwd_glds_kernel(ConvFwdArgs a) {
  using T = ConvTile<TM, TN, WVM>;
  constexpr int BM = T::BM, BN = T::BN, WM = 32 * TM, WN = 32 * TN;
  constexpr int WAVES_N = T::WVN;
  constexpr int A_CHUNKS = BM * 8, B_CHUNKS = BN * 8;
  static_assert(A_CHUNKS % NT == 0 && B_CHUNKS % NT == 0, "whole wave instructions per stage");
  static_assert(NS >= 2 && NS <= 4, "2..4 pipeline stages");
  constexpr int A_PER = A_CHUNKS / NT, B_PER = B_CHUNKS / NT;
  constexpr int STAGE = A_CHUNKS + B_CHUNKS;  // 16-B slots per pipeline stage
  constexpr int LPS = A_PER + B_PER;          // DMA instructions per thread per step
  constexpr bool UPFRONT = RAFT_CONV_UPFRONT && TM * TN >= 4;

  __shared__ __attribute__((aligned(16))) uint4 smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WAVES_N, wn = wave % WAVES_N;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  int mt, nt;
  if (!conv_tile_coords(raft_cdiv(P, BM), raft_cdiv(a.cout, BN), mt, nt)) return;
  const int m0 = mt * BM, n0 = nt * BN;

  int a_pix[A_PER], a_y[A_PER], a_x[A_PER], a_lc[A_PER];
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e >> 3;
    const int m = m0 + row;
    const int mm = m < P ? m : 0;
    const int r = mm % HW;
    a_pix[j] = mm;
    a_y[j] = m < P ? r / a.W : -(1 << 20);
    a_x[j] = r % a.W;
    a_lc[j] = ((e & 7) ^ ((row >> 1) & 7)) * 8;  // logical channel offset this lane fetches
  }
  uint32_t b_off[B_PER];
#pragma unroll
  for (int j = 0; j < B_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e >> 3;
    const int n = n0 + row;
    const int lc = (e & 7) ^ ((row >> 1) & 7);
    b_off[j] = n < a.cout ? (uint32_t)(((int64_t)n * a.kpad + lc * 8) * 2) : OOB;
  }

  // K loop channel-chunk-major, taps inner: the KH*KW shifted reads of one 64-channel slice of
  // the A rows follow each other while those rows are still in L2 (tap-major order re-fetched
  // the whole tile per tap: ~10x the input's bytes went to MALL / HBM on the 1x5 / 5x1 convs)
  const int nchunk = tile_nchunk(a, n0, BN);
  const int ntap = a.KH * a.KW;
  const int steps = ntap * nchunk;
  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = make_rsrc(a.seg[qq].ptr, (uint32_t)P * a.seg[qq].stride * 2u);
  }
  const rsrc_t w_rs = make_rsrc(a.wpk, (uint32_t)a.cout * a.kpad * 2u);
  const uint32_t lds0 = raft_lds_addr(smem) + __builtin_amdgcn_readfirstlane(wave * 64 * 16);

  auto issue = [&](int t, int buf) {
    const int ch = t / ntap, tap = t - ch * ntap;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    int c0 = ch * BK, lo = 0;
    if constexpr (epi_spl(EPI)) {  // split-fp32 K thirds [hi | lo | hi]
      const int third = a.cin_pad / 3, part = c0 / third;
      c0 -= part * third;
      lo = part == 1;
    }
    int s = 0, sbase = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (s + 1 < a.nseg && c0 >= sbase + a.seg[s].cnt) { sbase += a.seg[s].cnt; ++s; }
    const rsrc_t rs = s == 0 ? seg_rs[0] : (s == 1 ? seg_rs[1] : seg_rs[2]);
    const int stride = a.seg[s].stride;
    const int dy = kh - a.PH, dx = kw - a.PW;
    const int dpix = dy * a.W + dx;
    const int coff = c0 - sbase;
    const int cshift = lo ? stride / 2 : 0;
    const int creal = a.seg[s].real;
    const uint32_t base = lds0 + (uint32_t)(buf * STAGE * 16);
#pragma unroll
    for (int j = 0; j < A_PER; ++j) {
      const int yy = a_y[j] + dy, xx = a_x[j] + dx;
      const bool ok = (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W &&
                      coff + a_lc[j] < creal;
      const uint32_t off = (uint32_t)(((a_pix[j] + dpix) * stride + coff + cshift + a_lc[j]) * 2);
      raft_dma16(rs, base + j * NT * 16, ok ? off : OOB);
    }
    const uint32_t kb = (uint32_t)((tap * a.cin_pad + ch * BK) * 2);  // packed K: unsplit index
#pragma unroll
    for (int j = 0; j < B_PER; ++j)
      raft_dma16(w_rs, base + (A_CHUNKS + j * NT) * 16, b_off[j] == OOB ? OOB : b_off[j] + kb);
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  // All fragments of the step are read up front (4 k-slices x (TM + TN) ds_reads) and the group
  // barriers pin that order: the MFMAs of slice kk wait (counted lgkmcnt) only for their own
  // reads while the later slices' reads are in flight.  Left to itself hipcc sank every read to
  // just before its first MFMA with lgkmcnt(1) waits, exposing the LDS latency ~10x per step at
  // one wave per SIMD (profiles/r2: 29% MFMA busy on the 5x2 tile).
  auto compute_upfront = [&](int buf) {
    const uint4* As = smem + buf * STAGE;
    const uint4* Bs = As + A_CHUNKS;
    bf16x8_t af[BK / 16][TM], bfr[BK / 16][TN];
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + (lane & 31);
        bfr[kk][j] = __builtin_bit_cast(bf16x8_t, Bs[swz(row, kk * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + (lane & 31);
        af[kk][i] = __builtin_bit_cast(bf16x8_t, As[swz(row, kk * 2 + (lane >> 5))]);
      }
    }
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16<epi_f16(EPI)>(af[kk][i], bfr[kk][j], acc[i][j]);
    __builtin_amdgcn_sched_group_barrier(0x100, (BK / 16) * (TM + TN), 0);
    __builtin_amdgcn_sched_group_barrier(0x008, (BK / 16) * TM * TN, 0);
  };

  // fragments of k-slice kk+1 are read from LDS before the MFMAs of slice kk (two register sets),
  // so each ds_read has a whole slice of MFMAs to land instead of one or two
  auto compute = [&](int buf) {
    const uint4* As = smem + buf * STAGE;
    const uint4* Bs = As + A_CHUNKS;
    bf16x8_t af[2][TM], bfr[2][TN];
    auto rd = [&](int kk, int set) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wm * WM + i * 32 + (lane & 31);
        af[set][i] = __builtin_bit_cast(bf16x8_t, As[swz(row, kk * 2 + (lane >> 5))]);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wn * WN + j * 32 + (lane & 31);
        bfr[set][j] = __builtin_bit_cast(bf16x8_t, Bs[swz(row, kk * 2 + (lane >> 5))]);
      }
    };
    rd(0, 0);
#pragma unroll
    for (int kk = 0; kk < BK / 16; ++kk) {
      const int cur = kk & 1;
      if (kk + 1 < BK / 16) rd(kk + 1, cur ^ 1);
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16<epi_f16(EPI)>(af[cur][i], bfr[cur][j], acc[i][j]);
    }
  };

#pragma unroll
  for (int s = 0; s < NS - 1; ++s)
    if (s < steps) issue(s, s);
  int cur = 0;  // buffer of step t
  for (int t = 0; t < steps; ++t) {
    // stages issued after step t that may stay in flight: min(NS - 2, steps - 1 - t)
    const int newer = min(NS - 2, steps - 1 - t);
    if (NS >= 4 && newer >= 2) raft_wait_vmcnt<(NS >= 4 ? 2 : 0) * LPS>();
    else if (NS >= 3 && newer >= 1) raft_wait_vmcnt<(NS >= 3 ? 1 : 0) * LPS>();
    else raft_wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    if (t + NS - 1 < steps) {
      int nb = cur + NS - 1;
      nb = nb >= NS ? nb - NS : nb;
      issue(t + NS - 1, nb);
    }
    if constexpr (UPFRONT) compute_upfront(cur);
    else compute(cur);
    cur = cur + 1 == NS ? 0 : cur + 1;
  }

  conv_epilogue<TM, TN, WM, WN, EPI>(a, acc, m0, n0, wm, wn, lane, P, HW);
}


template <int EPI, int TM, int TN, int WVM, int NS>
void launch_one_glds(const ConvFwdArgs& a, hipStream_t stream) {
  using T = ConvTile<TM, TN, WVM>;
  const int P = a.B * a.H * a.W;
  dim3 grid(conv_grid_1d(raft_cdiv(P, T::BM), raft_cdiv(a.cout, T::BN)));
  hipLaunchKernelGGL((conv_fwd_glds_kernel<TM, TN, WVM, EPI, NS>), grid, dim3(NT), 0, stream, a);
}

template <int EPI>
bool launch_glds_epi(const ConvFwdArgs& a, int idx, hipStream_t stream) {
  switch (idx) {
      case 10: launch_one_glds<EPI, 2, 2, 2, 2>(a, stream); return true;
      case 11: launch_one_glds<EPI, 1, 2, 2, 2>(a, stream); return true;
      case 12: launch_one_glds<EPI, 2, 1, 2, 2>(a, stream); return true;
      case 13: launch_one_glds<EPI, 4, 2, 2, 2>(a, stream); return true;
      case 14: launch_one_glds<EPI, 4, 2, 1, 2>(a, stream); return true;
      case 15: launch_one_glds<EPI, 3, 2, 1, 2>(a, stream); return true;
      case 16: launch_one_glds<EPI, 5, 1, 1, 2>(a, stream); return true;
      case 17: launch_one_glds<EPI, 1, 1, 2, 2>(a, stream); return true;
      case 18: launch_one_glds<EPI, 2, 2, 2, 4>(a, stream); return true;
      case 19: launch_one_glds<EPI, 1, 2, 2, 3>(a, stream); return true;
      case 20: launch_one_glds<EPI, 5, 1, 1, 4>(a, stream); return true;
      case 21: launch_one_glds<EPI, 2, 1, 2, 4>(a, stream); return true;
      case 22: launch_one_glds<EPI, 1, 1, 2, 4>(a, stream); return true;
      case 23: launch_one_glds<EPI, 4, 2, 1, 3>(a, stream); return true;
      case 24: launch_one_glds<EPI, 3, 1, 1, 4>(a, stream); return true;
      case 25: launch_one_glds<EPI, 3, 1, 1, 2>(a, stream); return true;
      case 26: launch_one_glds<EPI, 5, 2, 1, 2>(a, stream); return true;
      case 27: launch_one_glds<EPI, 5, 2, 1, 3>(a, stream); return true;
      case 28: launch_one_glds<EPI, 9, 1, 1, 2>(a, stream); return true;
      case 29: launch_one_glds<EPI, 3, 3, 2, 2>(a, stream); return true;
    default: return false;
  }
}

}  // namespace conv_detail

// fp16-operand epilogues (EPI_F16 set): conv_glds_f16.hip; split-fp32 (EPI_SPL): conv_glds_spl.hip
bool launch_conv_glds_f16(const ConvFwdArgs& a, int epi, int idx, hipStream_t stream);
bool launch_conv_glds_spl(const ConvFwdArgs& a, int epi, int idx, hipStream_t stream);
