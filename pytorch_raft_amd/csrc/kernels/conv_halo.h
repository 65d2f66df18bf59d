// Halo-tile implicit-GEMM conv kernel (forward and input-gradient convs of the update block).
//
// Why: the LDS-DMA kernel (conv_glds.hip) re-fetches its BM-row A tile for EVERY filter tap and
// stages the weight tile through LDS although, with the waves split over N, no other wave reads
// it.  Its K step therefore issues (BM + BN) / 32 LDS-DMA pieces per wave for 20 MFMAs -- at
// ~60-185 issue cycles a piece (MI355X_MICROARCH.md, LDS-DMA piece issue cost) about as many
// cycles as the MFMAs themselves, which is where its 20-25 % MFMA utilisation went (loads that
// return zeros ran no faster: profiles/r2/nullmem_*.log).
//
// Here, per 64-channel chunk, the A rows of ALL taps -- the tile's BM pixels plus the halo the
// taps reach (PH*W + PW pixels before, (KH-1-PH)*W + (KW-1-PW) after) -- land in LDS ONCE
// (NPA pieces per thread for the chunk, issued one chunk ahead), and every tap reads its shifted
// rows from that image: a 3x3 conv issues 11 A pieces per chunk instead of 45, a 1x5 6 instead
// of 25.  LDS rows are 144 B (128 B of channels + 16 B pad) so a fragment read of 16 rows is
// bank-conflict free at ANY row shift (row r starts at dword 36 r mod 64 = 4 (9 r mod 16)); the
// lane-linear LDS-DMA image simply skips the pad slot (every 9th 16-B slot loads nothing).  Rows
// whose shifted neighbour leaves the image (x + dx or y + dy outside, or past the batch) read a
// zero row instead.  B fragments (32 output channels x 16 K per lane group) are loaded straight
// into VGPRs one K step ahead: no LDS round trip for an operand no other wave shares.
//
// Software pipeline (one wave per SIMD, so the wave itself must overlap its latencies): the
// fragment reads of step t+1 sit in the gaps of step t's MFMAs, B(t+1) is loaded during step t,
// and the next chunk's image is DMA'd one chunk ahead; the only barrier is at a chunk switch.
// Waits are counted by hand (every vector-memory op of the main loop is inline asm the compiler
// does not track): before the MFMAs of step t, B(t) must have landed while B(t+1) -- and the A
// pieces of a chunk switch right after step t-1 -- may stay in flight: vmcnt(4 TN [+ NPA]).  At
// a switch the new chunk's image is older than B(t) (for 1x1 convs, where every step switches,
// it is not: vmcnt(4 TN)).  Chunks past the last issue dummy (out-of-range) LDS-DMA pieces so the
// counts hold; B loads stop at the last step (a dead asm register load would still land).
#pragma once
#include "conv_common.h"

namespace conv_detail {

typedef unsigned int u32x4_t __attribute__((ext_vector_type(4)));

constexpr int HALO_ROWB = 144;  // LDS bytes per A row (128 data + 16 pad)

// halo rows a tile of BM pixels needs for a KH x KW conv on W-wide rows
__host__ __device__ inline int halo_rows(int BM, int W, int KH, int KW, int PH, int PW) {
  return BM + PH * W + PW + (KH - 1 - PH) * W + (KW - 1 - PW);
}
// LDS-DMA pieces per thread (256 threads x 16 B, 9 slots per row) covering `rows` rows
__host__ __device__ inline int halo_pieces(int rows) { return (rows * 9 + NT - 1) / NT; }

// B fragment load (16 B per lane) into VGPRs, not tracked by the compiler's waitcnt insertion
template <int IMM>
__device__ __forceinline__ void halo_bload(u32x4_t& dst, rsrc_t r, uint32_t voff, uint32_t soff) {
  asm volatile("buffer_load_dwordx4 %0, %1, %2, %3 offen offset:%4"
               : "=v"(dst)
               : "v"(voff), "s"(r), "s"(soff), "n"(IMM)
               : "memory");
}

template <int TM, int TN, int WVM, int EPI, int NPA>
__global__ __launch_bounds__(NT, 1) void conv_fwd_halo_kernel(ConvFwdArgs a) {
  constexpr int WVN = 4 / WVM;
  constexpr int BM = 32 * TM * WVM, BN = 32 * TN * WVN, WM = 32 * TM, WN = 32 * TN;
  constexpr int ABUF = NPA * NT * 16;  // bytes of one A halo image (whole DMA pieces)
  constexpr int LB = 4 * TN;           // B fragment loads per wave per K step
  static_assert(LB + NPA <= 63, "vmcnt range");

  __shared__ __attribute__((aligned(16))) uint4 smem[(2 * ABUF + HALO_ROWB) / 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WVN, wn = wave % WVN;
  const int H = a.H, W = a.W;
  const int HW = H * W;
  const int P = a.B * HW;
  int mt, nt;
  if (!conv_tile_coords(raft_cdiv(P, BM), raft_cdiv(a.cout, BN), mt, nt)) return;
  const int m0 = mt * BM, n0 = nt * BN;
  const int HL = a.PH * W + a.PW;  // halo rows before the tile

  const uint32_t lds0 = raft_lds_addr(smem);
  const uint32_t zrow = 2 * ABUF;  // byte offset of the zero row
  if (tid < HALO_ROWB / 16) smem[zrow / 16 + tid] = make_uint4(0u, 0u, 0u, 0u);

  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = make_rsrc(a.seg[qq].ptr, (uint32_t)P * a.seg[qq].stride * 2u);
  }
  const int nchunk = tile_nchunk(a, n0, BN);
  const int ntap = a.KH * a.KW;
  const int steps = ntap * nchunk;
  const uint32_t wave_off = __builtin_amdgcn_readfirstlane(wave * 64 * 16);
  // chunk c's halo image into buffer c & 1 (c >= nchunk: dummy pieces, nothing is read)
  auto issue_a = [&](int c) {
    const bool real = c < nchunk;
    int c0 = (real ? c : 0) * BK, lo = 0;
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
    const int coff = c0 - sbase;
    const int cshift = lo ? stride / 2 : 0;
    const int creal = a.seg[s].real;
    const uint32_t base = lds0 + (uint32_t)((c & 1) * ABUF) + wave_off;
    // thread slot g = j * NT + tid of the image -> (row g / 9, 16-B slot g % 9; slot 8 = pad)
#pragma unroll
    for (int j = 0; j < NPA; ++j) {
      const int g = j * NT + tid;
      const int row = g / 9, slot = g - row * 9;
      const int q = m0 - HL + row;
      const bool ok = real && slot < 8 && q >= 0 && q < P && coff + slot * 8 < creal;
      raft_dma16(rs, base + j * NT * 16, ok ? (uint32_t)((q * stride + coff + cshift + slot * 8) * 2) : OOB);
    }
  };

  // ---- B fragments straight to VGPRs: lane -> output channel row (lane & 31), k half (lane >> 5)
  const rsrc_t w_rs = make_rsrc(a.wpk, (uint32_t)a.cout * a.kpad * 2u);
  uint32_t b_voff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wn * WN + j * 32 + (lane & 31);
    b_voff[j] = n < a.cout ? (uint32_t)(((int64_t)n * a.kpad + 8 * (lane >> 5)) * 2) : OOB;
  }
  // K offset of step (chunk ch, tap) = tap * cin_pad + ch * 64; `real` false: dummy (zero) loads
  auto issue_b = [&](bool real, int ch, int tap, u32x4_t (&dst)[4][TN]) {
    const uint32_t kb = real ? (uint32_t)((tap * a.cin_pad + ch * BK) * 2) : 0u;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const uint32_t v = real ? b_voff[j] : OOB;
      halo_bload<0>(dst[0][j], w_rs, v, kb);
      halo_bload<32>(dst[1][j], w_rs, v, kb);
      halo_bload<64>(dst[2][j], w_rs, v, kb);
      halo_bload<96>(dst[3][j], w_rs, v, kb);
    }
  };

  // ---- per-lane A rows (pixel coordinates) of the wave's TM fragments
  int r_y[TM], r_x[TM];
  uint32_t r_base[TM];
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int rloc = wm * WM + i * 32 + (lane & 31);
    const int m = m0 + rloc;
    const int mm = m < P ? m : 0;
    const int r = mm % HW;
    r_y[i] = m < P ? r / W : -(1 << 20);
    r_x[i] = r % W;
    r_base[i] = (uint32_t)(rloc + HL) * HALO_ROWB + (uint32_t)(lane >> 5) * 16u;
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  const char* smem_b = reinterpret_cast<const char*>(smem);
  // A fragments of the step at (chunk ch, tap offset dy, dx) from the chunk's halo image
  auto read_frags = [&](int ch, int dy, int dx, bf16x8_t (&af)[4][TM]) {
    const uint32_t shift = (uint32_t)((ch & 1) * ABUF + (dy * W + dx) * HALO_ROWB);
    uint32_t addr[TM];
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const bool ok = (unsigned)(r_y[i] + dy) < (unsigned)H && (unsigned)(r_x[i] + dx) < (unsigned)W;
      addr[i] = ok ? r_base[i] + shift : zrow + (uint32_t)(lane >> 5) * 16u;
    }
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
        af[kk][i] = *reinterpret_cast<const bf16x8_t*>(smem_b + addr[i] + kk * 32);
  };
  auto fence_b = [&](u32x4_t (&bf)[4][TN]) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int j = 0; j < TN; ++j) asm volatile("" : "+v"(bf[kk][j]));
  };
  // MFMAs of one step with the NEXT step's fragment reads interleaved (TN MFMAs per read)
  // (after the last step the reads go to a valid, unused image position: one basic block, so the
  // group barriers can interleave them)
  auto mfma_step = [&](const bf16x8_t (&af)[4][TM], const u32x4_t (&bf)[4][TN], int ch, int dy,
                       int dx, bf16x8_t (&afn)[4][TM]) {
#pragma unroll
    for (int kk = 0; kk < 4; ++kk)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = mfma16<epi_f16(EPI)>(af[kk][i], __builtin_bit_cast(bf16x8_t, bf[kk][j]),
                                           acc[i][j]);
    read_frags(ch, dy, dx, afn);
#pragma unroll
    for (int u = 0; u < 4 * TM; ++u) {
      __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
    }
  };

  // position (chunk, tap, kh, kw) of the step whose fragments / B are prefetched next
  int nch = 0, ntp = 0, nkh = 0, nkw = 0;
  auto advance = [&]() {
    if (++nkw == a.KW) { nkw = 0; ++nkh; }
    if (++ntp == ntap) { ntp = 0; nkh = 0; nkw = 0; ++nch; }
  };
  bf16x8_t afr[2][4][TM];
  u32x4_t breg[2][4][TN];

  // prologue: A(0), B(0); A(0) landed (B(0) younger) -> zero row + image visible -> A(1); frags(0)
  issue_a(0);
  issue_b(true, 0, 0, breg[0]);
  raft_wait_vmcnt<LB>();
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the zero row is written
  __builtin_amdgcn_s_barrier();
  issue_a(1);
  read_frags(0, nkh - a.PH, nkw - a.PW, afr[0]);
  advance();  // -> step 1
  // step t (register sets p = t & 1):  B(t+1) issued; B(t) waited for (younger: B(t+1) and the A
  // pieces of a chunk switch right after step t-1); at the chunk's last step the next chunk's
  // image is waited for (1x1 convs: it is younger than B(t)) + barrier, then the image after it
  // goes into the buffer this chunk used; MFMAs(t) with frags(t+1) reads in their gaps
  auto step = [&](int t, bf16x8_t (&af)[4][TM], bf16x8_t (&afn)[4][TM], u32x4_t (&bc)[4][TN],
                  u32x4_t (&bn)[4][TN], bool prev_switch) {
    const bool more = t + 1 < steps;
    // no load past the last step: an asm load whose registers are dead would still write them
    // when its data returns, after the compiler may have handed them to another value
    if (more) issue_b(true, nch, ntp, bn);
    if (more) {
      if (prev_switch) raft_wait_vmcnt<LB + NPA>();
      else raft_wait_vmcnt<LB>();
    } else {
      if (prev_switch) raft_wait_vmcnt<NPA>();
      else raft_wait_vmcnt<0>();
    }
    fence_b(bc);
    const bool sw = more && ntp == 0;  // step t+1 opens chunk nch
    if (sw) {
      if (ntap == 1) raft_wait_vmcnt<LB>();
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): frags(t) are in registers
      __builtin_amdgcn_s_barrier();
      issue_a(nch + 1);                    // into buffer (nch + 1) & 1 = the chunk just finished
    }
    mfma_step(af, bc, nch, nkh - a.PH, nkw - a.PW, afn);
    advance();
    return sw;
  };
  bool psw = true;  // A(1) was issued after B(0)
  for (int t = 0; t < steps; t += 2) {
    psw = step(t, afr[0], afr[1], breg[0], breg[1], psw);
    if (t + 1 < steps) psw = step(t + 1, afr[1], afr[0], breg[1], breg[0], psw);
  }
  raft_wait_vmcnt<0>();  // no LDS-DMA may still target LDS when the workgroup retires

  conv_epilogue<TM, TN, WM, WN, EPI>(a, acc, m0, n0, wm, wn, lane, P, HW);
}

template <int EPI, int TM, int TN, int WVM, int NPA>
void launch_halo_one(const ConvFwdArgs& a, hipStream_t stream) {
  constexpr int BM = 32 * TM * WVM, BN = 32 * TN * (4 / WVM);
  const int P = a.B * a.H * a.W;
  dim3 grid(conv_grid_1d(raft_cdiv(P, BM), raft_cdiv(a.cout, BN)));
  hipLaunchKernelGGL((conv_fwd_halo_kernel<TM, TN, WVM, EPI, NPA>), grid, dim3(NT), 0, stream, a);
}

template <int EPI, int NPA>
bool halo_cfg(const ConvFwdArgs& a, int tm, int tn, int wvm, hipStream_t s) {
  if (tm == 5 && tn == 1 && wvm == 1) { launch_halo_one<EPI, 5, 1, 1, NPA>(a, s); return true; }
  if (tm == 5 && tn == 2 && wvm == 1) { launch_halo_one<EPI, 5, 2, 1, NPA>(a, s); return true; }
  if (tm == 4 && tn == 2 && wvm == 1) { launch_halo_one<EPI, 4, 2, 1, NPA>(a, s); return true; }
  if (tm == 2 && tn == 2 && wvm == 2) { launch_halo_one<EPI, 2, 2, 2, NPA>(a, s); return true; }
  return false;
}

// the epilogues the halo kernel serves, for one operand type (TY = 0 bf16, EPI_F16 fp16,
// EPI_SPL split fp32)
template <int NPA, int TY>
bool halo_switch(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm, hipStream_t s) {
  switch (epi_kind(epi)) {
    case EPI_BF16: return halo_cfg<EPI_BF16 | TY, NPA>(a, tm, tn, wvm, s);
    case EPI_RELU_BF16: return halo_cfg<EPI_RELU_BF16 | TY, NPA>(a, tm, tn, wvm, s);
    case EPI_F32: return halo_cfg<EPI_F32 | TY, NPA>(a, tm, tn, wvm, s);
    case EPI_GRU_ZR: return halo_cfg<EPI_GRU_ZR | TY, NPA>(a, tm, tn, wvm, s);
    case EPI_GRU_Q: return halo_cfg<EPI_GRU_Q | TY, NPA>(a, tm, tn, wvm, s);
    case EPI_DGRAD: return halo_cfg<EPI_DGRAD | TY, NPA>(a, tm, tn, wvm, s);
    case EPI_DGRAD_GATE: return halo_cfg<EPI_DGRAD_GATE | TY, NPA>(a, tm, tn, wvm, s);
    default: return false;
  }
}

// one translation unit per (image size, operand type TY): conv_halo_<NPA>[_f16|_spl].hip
template <int NPA, int TY>
bool launch_conv_halo_npa(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm, hipStream_t stream);
#define RAFT_HALO_DECL(N)                                                                       \
  template <> bool launch_conv_halo_npa<N, 0>(const ConvFwdArgs&, int, int, int, int, hipStream_t); \
  template <> bool launch_conv_halo_npa<N, EPI_F16>(const ConvFwdArgs&, int, int, int, int, hipStream_t); \
  template <> bool launch_conv_halo_npa<N, EPI_SPL>(const ConvFwdArgs&, int, int, int, int, hipStream_t);
RAFT_HALO_DECL(6)
RAFT_HALO_DECL(11)
RAFT_HALO_DECL(16)
#undef RAFT_HALO_DECL
#define RAFT_HALO_TU(N, TY)                                                                     \
  template <>                                                                                   \
  bool launch_conv_halo_npa<N, TY>(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm,     \
                                   hipStream_t s) {                                             \
    return halo_switch<N, TY>(a, epi, tm, tn, wvm, s);                                          \
  }

}  // namespace conv_detail

// halo kernel of config (tm, tn, wvm) if its geometry fits (LDS image, epilogue); false otherwise
bool launch_conv_halo(const ConvFwdArgs& a, int epi, int tm, int tn, int wvm, hipStream_t stream);
