// Pipelined implicit-GEMM conv kernel, v3 (forward and input-gradient convs of the update block).
//
// Why a third main loop: s_memtime stamps per K step (scripts/lab/conv_lab.hip, diagnostic
// build) show where the LDS-DMA kernels lose their time: ONE `buffer_load_dwordx4 ... lds`
// piece holds the issuing wave for ~170 cycles (5 pieces: 750-900 cycles of a 64-deep K step
// whose 20 MFMAs take 640), and the LDS-DMA kernel also ran a tap/chunk division, a kernarg
// s_load with an lgkmcnt(0) wait and ~10 VALU of address math per piece between the barrier and
// its first MFMA -- with one wave per SIMD nothing hid any of it (~2,100 cycles per step).
//
// Here a step's MFMAs start right after the barrier and the rest of the pipeline runs in their
// gaps:
//  * A (the pixel tile, shared by the 4 waves) is register-staged: global -> VGPR two steps ahead
//    (buffer loads, cheap to issue), VGPR -> LDS (ds_write_b128, ~13 cycles) one step ahead, into
//    a 3-slot ring.  Per piece the address is one v_mad_u32_u24 on a precomputed pixel index and
//    the tap validity one bit test of a per-piece mask computed once; the tap / chunk / segment
//    position advances incrementally in SGPRs (no division, no kernarg load in the loop).
//  * B (weights) is not shared (the waves split N): each wave loads its fragments straight into
//    VGPRs one step ahead, K offset in the scalar soffset, k-slice in the immediate: no VALU.
//  * The fragment reads of step t+1 are interleaved with the MFMAs of step t.
//  * ONE barrier per step.  Top of step t: this wave's ds_writes of A(t+1) done (lgkmcnt) and
//    B(t) landed (vmcnt) -> barrier: A(t+1) visible to every wave AND every wave is past step t-1,
//    whose frag reads of slot (t+2) % 3 (= A(t-1)) were consumed by its MFMAs, so A(t+2) may be
//    written there during step t.
//  * <= 256 VGPR+AGPR per lane and <= 80 KB LDS (launch bounds OCC = 2): two workgroups per CU
//    (two waves per SIMD) overlap each other's prologue / epilogue / barrier waits with MFMAs.
// The global loads are inline asm the compiler does not count (explicit waits); the loop is
// straight-line over two steps (steps padded to an even count: a padded step reads zero A and
// zero B and adds exact zeros) so the asm-loaded register sets keep fixed registers (no copy of
// a not-yet-landed value), and an empty asm "+v" pins each use behind its wait.
#pragma once
#include "conv_common.h"

namespace conv_detail {

typedef unsigned int v3_u32x4 __attribute__((ext_vector_type(4)));

// 16 B per lane into VGPRs through a compiler-visible buffer load: the compiler places the vmcnt
// wait before the first use (B: the step's first MFMA; A: its ds_write one step later) and
// handles every register hazard.  (Inline-asm loads with hand-counted waits produced wrong
// tiles whenever two workgroups shared a CU: a load could overwrite registers a queued MFMA /
// ds_write had not read yet.)
template <int IMM>
__device__ __forceinline__ void v3_load16(v3_u32x4& dst, rsrc_t r, uint32_t voff, uint32_t soff) {
  dst = __builtin_bit_cast(v3_u32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff + IMM, soff, 0));
}

template <int TM, int TN>
struct V3Tile {
  static constexpr int BM = 32 * TM, BN = 128 * TN, WN = 32 * TN;
  static constexpr int STAGE = BM * 128;     // bytes of one A ring slot
  static constexpr int LDS = 3 * STAGE;
  static constexpr int A_PER = TM;           // 16-B A pieces per thread per step (BM * 8 / 256)
  static constexpr int LB = 4 * TN;          // B fragment loads per wave per step
};

// STAMP: diagnostic build only -- s_memtime per phase of every step of wave 0 into stamp[]
// (nothing in the kernel reads it back).
// EXP (timing experiments only, results are wrong): bit 0 -- no A global loads, bit 1 -- no B
// global loads (the staging / fragment registers keep stale values).
template <int TM, int TN, int EPI, int OCC, bool STAMP = false, int EXP = 0>
__global__ __launch_bounds__(NT, OCC) void conv_fwd_v3_kernel(ConvFwdArgs a, unsigned long long* stamp) {
  using T = V3Tile<TM, TN>;
  constexpr int BM = T::BM, BN = T::BN, WN = T::WN;
  constexpr int A_PER = T::A_PER, LB = T::LB;
  static_assert(A_PER + LB <= 60, "vmcnt range");

  __shared__ __attribute__((aligned(16))) uint4 smem[T::LDS / 16];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int H = a.H, W = a.W;
  const int HW = H * W;
  const int P = a.B * HW;
  int mt, nt;
  if (!conv_tile_coords(raft_cdiv(P, BM), raft_cdiv(a.cout, BN), mt, nt)) return;
  const int m0 = mt * BM, n0 = nt * BN;
  // every kernel argument the loop needs, read once (kernarg reads inside the loop made the
  // compiler keep a scratch copy of the whole argument block)
  const int KH = a.KH, KW = a.KW, PH = a.PH, PW = a.PW, cin_pad = a.cin_pad;
  const int ntap = KH * KW;
  const int nchunk = cin_pad / BK;
  const int steps = ntap * nchunk;
  const int steps2 = (steps + 1) & ~1;

  // ---- segments (<= 3): separate scalars, static kernarg indices (an array selected by a
  // runtime index, or a dynamic a.seg[i], ends up in scratch)
  const int nseg = a.nseg;
  const Seg sg0 = a.seg[0], sg1 = a.seg[1], sg2 = a.seg[2];
  const rsrc_t rs0 = make_rsrc(sg0.ptr, (uint32_t)P * sg0.stride * 2u);
  const rsrc_t rs1 = nseg > 1 ? make_rsrc(sg1.ptr, (uint32_t)P * sg1.stride * 2u) : rs0;
  const rsrc_t rs2 = nseg > 2 ? make_rsrc(sg2.ptr, (uint32_t)P * sg2.stride * 2u) : rs0;
  const int st0 = sg0.stride * 2;
  const int st1 = nseg > 1 ? sg1.stride * 2 : st0;
  const int st2 = nseg > 2 ? sg2.stride * 2 : st0;
  const int cnt0 = sg0.cnt;
  const int cnt1 = nseg > 1 ? sg1.cnt : (1 << 30);
  const int cnt2 = nseg > 2 ? sg2.cnt : (1 << 30);

  // ---- A pieces: thread slot e = j * 256 + tid -> tile row e >> 3, physical 16-B slot e & 7,
  // logical channel chunk (e & 7) ^ ((row >> 1) & 7) (the fragment reads' swizzle)
  int a_pix[A_PER];         // pixel index (m, clamped)
  uint32_t a_lc2[A_PER];    // byte offset of the logical chunk inside a 128-B row
  uint32_t a_tmask[A_PER];  // bit tap: the tap's shifted pixel is inside the image (taps <= 32)
#pragma unroll
  for (int j = 0; j < A_PER; ++j) {
    const int e = j * NT + tid;
    const int row = e >> 3;
    const int m = m0 + row;
    const bool in = m < P;
    const int mm = in ? m : 0;
    const int r = mm % HW;
    const int y = r / W, x = r - (r / W) * W;
    a_pix[j] = mm;
    a_lc2[j] = (uint32_t)(((e & 7) ^ ((row >> 1) & 7)) * 16);
    uint32_t msk = 0;
    int tp = 0;
    for (int kh = 0; kh < KH; ++kh) {
      const bool yok = (unsigned)(y + kh - PH) < (unsigned)H;
      for (int kw = 0; kw < KW; ++kw, ++tp)
        if (in && yok && (unsigned)(x + kw - PW) < (unsigned)W && tp < 32) msk |= 1u << tp;
    }
    a_tmask[j] = msk;
  }
  char* smem_b = reinterpret_cast<char*>(smem);
  const uint32_t a_wr = (uint32_t)tid * 16u;  // this thread's ds_write offset (+ j * 4096)

  // ---- B fragments: lane -> output channel row (lane & 31), k half (lane >> 5)
  const rsrc_t w_rs = make_rsrc(a.wpk, (uint32_t)a.cout * a.kpad * 2u);
  uint32_t b_voff[TN];
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int n = n0 + wave * WN + j * 32 + (lane & 31);
    b_voff[j] = n < a.cout ? (uint32_t)(((int64_t)n * a.kpad + 8 * (lane >> 5)) * 2) : OOB;
  }

  // ---- fragment read offsets inside a ring slot: row i*32 + (lane & 31), chunk 2 kk +
  // (lane >> 5), swizzle key ((lane & 31) >> 1) & 7 (the same for every i)
  uint32_t f_off[4];
  {
    const int r = lane & 31, h = lane >> 5, key = (r >> 1) & 7;
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) f_off[kk] = (uint32_t)(r * 128 + (((2 * kk + h) ^ key) * 16));
  }

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  bf16x8_t af[2][TM];     // A fragments, one k-slice ahead (two slices live)
  v3_u32x4 bq[2][4][TN] = {};
  v3_u32x4 ast[2][A_PER];  // A staging, two steps ahead (set = step & 1)

  unsigned long long* st_row = nullptr;
  if constexpr (STAMP) {
    if (tid == 0) st_row = stamp + (size_t)blockIdx.x * 256;
  }
  // Macros, not lambdas, below: the optimizer left lambda closures over these locals as stack
  // objects (the pipeline state then lived in scratch and the loop went divergent).
#define V3_STAMP(k)                                                                             \
  if constexpr (STAMP) {                                                                       \
    if (tid == 0) st_row[(k)] = __builtin_amdgcn_s_memtime();                                  \
  }
  // A position (step, tap, kh, kw, channel, segment) of the next A global load, advanced
  // incrementally (chunk-major, taps inner)
  int p_t = 0, p_tap = 0, p_kh = 0, p_kw = 0, p_c0 = 0, p_s = 0, p_sbase = 0;
#define V3_A_LOAD(set)                                                                          \
  {                                                                                            \
    const bool real_ = p_t < steps;                                                            \
    const rsrc_t rs_ = p_s == 0 ? rs0 : (p_s == 1 ? rs1 : rs2);                                \
    const int st_ = p_s == 0 ? st0 : (p_s == 1 ? st1 : st2);                                   \
    const int dpix_ = (p_kh - PH) * W + (p_kw - PW);                                           \
    const uint32_t cadd_ = (uint32_t)((p_c0 - p_sbase) * 2);                                   \
    _Pragma("unroll") for (int j = 0; j < A_PER; ++j) {                                        \
      const bool ok_ = real_ && ((a_tmask[j] >> p_tap) & 1u);                                  \
      const uint32_t off_ = __umul24((uint32_t)(a_pix[j] + dpix_), (uint32_t)st_) + cadd_ + a_lc2[j]; \
      if constexpr (!(EXP & 1)) v3_load16<0>(ast[set][j], rs_, ok_ ? off_ : OOB, 0u);          \
      else ast[set][j] = v3_u32x4{off_, 0u, 0u, (uint32_t)ok_};                               \
    }                                                                                          \
    ++p_t;                                                                                     \
    if (++p_kw == KW) { p_kw = 0; ++p_kh; }                                                    \
    if (++p_tap == ntap) {                                                                     \
      p_tap = 0; p_kh = 0; p_kw = 0; p_c0 += BK;                                               \
      const int cnt_ = p_s == 0 ? cnt0 : (p_s == 1 ? cnt1 : cnt2);                             \
      if (p_s < 2 && p_c0 >= p_sbase + cnt_) { p_sbase += cnt_; ++p_s; }                       \
    }                                                                                          \
  }
#define V3_A_WRITE(slot, set)                                                                   \
  {                                                                                            \
    char* dst_ = smem_b + (slot) * T::STAGE + a_wr;                                            \
    _Pragma("unroll") for (int j = 0; j < A_PER; ++j)                                          \
      *reinterpret_cast<v3_u32x4*>(dst_ + j * NT * 16) = ast[set][j];                          \
  }
  // B position of the next B load (one step ahead of the MFMAs)
  int b_t = 0, b_tap = 0, b_c0 = 0;
#define V3_B_LOAD(set)                                                                          \
  {                                                                                            \
    const bool real_ = b_t < steps;                                                            \
    const uint32_t kb_ = real_ ? (uint32_t)((b_tap * cin_pad + b_c0) * 2) : 0u;                \
    if constexpr (!(EXP & 2)) _Pragma("unroll") for (int j = 0; j < TN; ++j) {                 \
      const uint32_t v_ = real_ ? b_voff[j] : OOB;                                             \
      v3_load16<0>(bq[set][0][j], w_rs, v_, kb_);                                              \
      v3_load16<32>(bq[set][1][j], w_rs, v_, kb_);                                             \
      v3_load16<64>(bq[set][2][j], w_rs, v_, kb_);                                             \
      v3_load16<96>(bq[set][3][j], w_rs, v_, kb_);                                             \
    }                                                                                          \
    ++b_t;                                                                                     \
    if (++b_tap == ntap) { b_tap = 0; b_c0 += BK; }                                            \
  }

  // ---- prologue: A(0) -> slot 0, A(1) -> slot 1 (through the staging registers), B(0), A(2)
  // and A(3) loads in flight; slice 0 of frags(0)
  V3_STAMP(0)
  V3_A_LOAD(0)
  V3_A_WRITE(0, 0)
  V3_A_LOAD(1)
  V3_B_LOAD(0)
  V3_A_WRITE(1, 1)
  V3_A_LOAD(0)  // A(2): written during step 0
  V3_A_LOAD(1)  // A(3): written during step 1
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this wave's slot writes done
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
#pragma unroll
  for (int i = 0; i < TM; ++i)
    af[0][i] = *reinterpret_cast<const bf16x8_t*>(smem_b + f_off[0] + i * 4096);
  V3_STAMP(1)

  // step t (ph = t & 1, a literal): B(t+1) -> set ph^1; MFMAs of A(t) x B(t), k-slice kk on frag
  // set kk & 1 while slice kk+1 (kk = 3: slice 0 of A(t+1), slot (t+1) % 3) is read into the
  // other; after the first k-slice A(t+2) (loaded into staging set ph during step t-2) is written
  // into slot (t+2) % 3 and A(t+4) is loaded into that set.  The compiler places every vmcnt
  // wait (all loads are builtins).  Slot (t+2) % 3 held A(t-1), whose last frag reads (step t-1,
  // slice 2) were consumed before this step's barrier.
#define V3_SLICE(kk, ph)                                                                        \
  {                                                                                            \
    _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                           \
      _Pragma("unroll") for (int j = 0; j < TN; ++j) acc[i][j] =                               \
          __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[(kk) & 1][i],                             \
                                                  __builtin_bit_cast(bf16x8_t, bq[ph][kk][j]), \
                                                  acc[i][j], 0, 0, 0);                         \
      af[((kk) + 1) & 1][i] = *reinterpret_cast<const bf16x8_t*>(                              \
          smem_b + ((kk) == 3 ? sb1_ + f_off[0] : sb0_ + f_off[((kk) + 1) & 3]) + i * 4096);   \
    }                                                                                          \
    _Pragma("unroll") for (int i = 0; i < TM; ++i) {                                           \
      __builtin_amdgcn_sched_group_barrier(0x008, TN, 0);                                      \
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                                       \
    }                                                                                          \
  }
#define V3_STEP(ph)                                                                             \
  {                                                                                            \
    __builtin_amdgcn_s_waitcnt(0xC07F); /* lgkmcnt(0): this wave's ds_writes of A(t+1) done */ \
    __builtin_amdgcn_s_barrier();                                                              \
    asm volatile("" ::: "memory");                                                             \
    if (STAMP && t < 60) { V3_STAMP(4 + 4 * t) }                                               \
    V3_B_LOAD((ph) ^ 1)                                                                        \
    const uint32_t sb0_ = (uint32_t)((t % 3) * T::STAGE);                                      \
    const uint32_t sb1_ = (uint32_t)(((t + 1) % 3) * T::STAGE);                                \
    V3_SLICE(0, ph)                                                                            \
    if (STAMP && t < 60) { V3_STAMP(5 + 4 * t) }                                               \
    V3_A_WRITE((t + 2) % 3, ph)                                                                \
    V3_A_LOAD(ph)                                                                              \
    if (STAMP && t < 60) { V3_STAMP(6 + 4 * t) }                                               \
    V3_SLICE(1, ph)                                                                            \
    V3_SLICE(2, ph)                                                                            \
    V3_SLICE(3, ph)                                                                            \
    ++t;                                                                                       \
  }
  for (int t = 0; t < steps2;) {
    V3_STEP(0)
    V3_STEP(1)
  }
#undef V3_STEP
#undef V3_SLICE
#undef V3_B_LOAD
#undef V3_A_WRITE
#undef V3_A_LOAD
  V3_STAMP(2)

  conv_epilogue<TM, TN, BM, WN, EPI>(a, acc, m0, n0, 0, wave, lane, P, HW);
  if constexpr (STAMP) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    V3_STAMP(3)
  }
#undef V3_STAMP
}

}  // namespace conv_detail
