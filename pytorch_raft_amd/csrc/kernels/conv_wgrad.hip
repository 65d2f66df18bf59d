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
  typedef __amdgpu_buffer_rsrc_t rsrc_t;
  constexpr uint32_t OOB = 0x80000000u;  // past every num_records: the buffer load returns zeros
  auto mk = [](const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  auto ld16 = [](rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  };
  const rsrc_t g_rs = mk(a.g, (uint32_t)P * a.g_stride * 2u);
  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = mk(a.seg[qq].ptr, (uint32_t)P * a.seg[qq].stride * 2u);
  }

  // G chunks: fixed column n per thread, row (pixel) advances by BKP per step
  int g_row[G_PER];
  bool g_ok[G_PER];
#pragma unroll
  for (int j = 0; j < G_PER; ++j) {
    const int e = tid + j * NT;
    g_row[j] = e / (BM / 8);
    g_ok[j] = e < GCH && m0 + (e % (BM / 8)) * 8 < a.cout;
  }
  // X chunks: the packed-K column (tap, channel, segment) is fixed per thread -> decoded once;
  // the pixel (p, y, x) of each chunk is advanced incrementally by BKP per step
  int x_dpix[X_PER], x_dy[X_PER], x_dx[X_PER], x_coff[X_PER], x_seg[X_PER], x_stride[X_PER];
  int x_p[X_PER], x_y[X_PER], x_x[X_PER];
  bool x_ok[X_PER];
#pragma unroll
  for (int j = 0; j < X_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e / (BN / 8), ch = e % (BN / 8);
    const int kc = k0 + ch * 8;
    x_ok[j] = e < XCH && kc < a.kpad;
    int dy = 0, dx = 0, coff = 0, sidx = 0;
    if (!SMALLC) {
      const int tap = kc / a.cin_pad, c = kc - tap * a.cin_pad;
      const int kh = tap / a.KW, kw = tap - kh * a.KW;
      dy = kh - a.PH;
      dx = kw - a.PW;
      int sbase = 0;
#pragma unroll
      for (int q = 0; q < 2; ++q)
        if (sidx + 1 < a.nseg && c >= sbase + a.seg[sidx].cnt) { sbase += a.seg[sidx].cnt; ++sidx; }
      coff = c - sbase;
    }
    x_dy[j] = dy;
    x_dx[j] = dx;
    x_dpix[j] = dy * a.W + dx;
    x_coff[j] = coff;
    x_seg[j] = sidx;
    x_stride[j] = a.seg[sidx].stride;
    const int p = p_begin + row;
    const int pp = p < P ? p : 0;
    const int r = pp % HW;
    x_p[j] = p;
    x_y[j] = r / a.W;
    x_x[j] = r - (r / a.W) * a.W;
  }
  auto advance = [&]() {  // every chunk's pixel += BKP
#pragma unroll
    for (int j = 0; j < X_PER; ++j) {
      x_p[j] += BKP;
      int xx = x_x[j] + BKP, yy = x_y[j];
      while (xx >= a.W) { xx -= a.W; yy = (yy + 1 == a.H) ? 0 : yy + 1; }
      x_x[j] = xx;
      x_y[j] = yy;
    }
  };

  auto load = [&](int pbase, uint4 (&rg)[G_PER], uint4 (&rx)[X_PER]) {
#pragma unroll
    for (int j = 0; j < G_PER; ++j) {
      const int e = tid + j * NT;
      const int p = pbase + g_row[j];
      const uint32_t off = (uint32_t)(((int64_t)p * a.g_stride + m0 + (e % (BM / 8)) * 8) * 2);
      rg[j] = ld16(g_rs, (g_ok[j] && p < p_end) ? off : OOB);
    }
#pragma unroll
    for (int j = 0; j < X_PER; ++j) {
      const int p = x_p[j];
      if constexpr (!SMALLC) {
        const int yy = x_y[j] + x_dy[j], xx = x_x[j] + x_dx[j];
        const bool ok = x_ok[j] && p < p_end && (unsigned)yy < (unsigned)a.H &&
                        (unsigned)xx < (unsigned)a.W;
        const uint32_t off = (uint32_t)(((p + x_dpix[j]) * x_stride[j] + x_coff[j]) * 2);
        const rsrc_t rs = x_seg[j] == 0 ? seg_rs[0] : (x_seg[j] == 1 ? seg_rs[1] : seg_rs[2]);
        rx[j] = ld16(rs, ok ? off : OOB);
      } else {
        const int e = tid + j * NT;
        const int kc = k0 + (e % (BN / 8)) * 8;
        uint16_t t[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const int k = kc + q;
          uint16_t val = 0;
          if (x_ok[j] && p < p_end && k < ktot_small) {
            const int tap = k / a.cin_small, c = k - tap * a.cin_small;
            const int kh = tap / a.KW, kw = tap - kh * a.KW;
            const int yy = x_y[j] + kh - a.PH, xx = x_x[j] + kw - a.PW;
            if (yy >= 0 && yy < a.H && xx >= 0 && xx < a.W)
              val = a.seg[0].ptr[(int64_t)(p + (kh - a.PH) * a.W + (kw - a.PW)) * a.seg[0].stride + c];
          }
          t[q] = val;
        }
        rx[j] = make_uint4(t[0] | (t[1] << 16), t[2] | (t[3] << 16), t[4] | (t[5] << 16), t[6] | (t[7] << 16));
      }
    }
    advance();
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

  // loads past p_end read zeros (range check), so the pipeline runs unconditionally: no branch
  // around a memory op, and hipcc keeps the newer register set in flight across each store
  const int steps = (p_end - p_begin + BKP - 1) / BKP;
  if (steps <= 0) return;
  uint4 rg0[G_PER], rx0[X_PER], rg1[G_PER], rx1[X_PER];
  load(p_begin, rg0, rx0);
  load(p_begin + BKP, rg1, rx1);
  store(0, rg0, rx0);
  __syncthreads();
  for (int t = 0; t < steps; t += 2) {
    load(p_begin + (t + 2) * BKP, rg0, rx0);
    compute(0);
    store(1, rg1, rx1);
    __syncthreads();
    if (t + 1 >= steps) break;
    load(p_begin + (t + 3) * BKP, rg1, rx1);
    compute(1);
    store(0, rg0, rx0);
    __syncthreads();
  }
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

// ------------------------------------------------------------------ multi-item LDS-DMA kernel
// dW = sum over ITEMS (the GRU iterations of one training step: the weights are shared, so the
// per-iteration weight gradients are summed) and pixels of G^T X.  Batching every iteration into
// one launch makes the reduction 12x longer per output tile, so the split-K partials that leave
// the chip as float atomics shrink 12x (they ran at the ~1.3 TB/s memory-side atomic rate).
// Operands go global -> LDS by buffer_load ... lds (no staging VGPRs / ds_write pass).  LDS image:
// [64 pixel rows][RB bytes] per operand, 16-B chunks XOR-swizzled per row on the SOURCE side so
// the transposing ds_read_b64_tr_b16 fragment reads (16-lane group = 4 rows x 32 B) hit 16
// distinct bank groups:  RB = 256: chunk ^= 4*(row & 3);  RB = 128: chunk ^= 4*((row >> 1) & 1).
template <int RB>
__device__ __forceinline__ int wg_swz(int row) {
  return RB == 256 ? 4 * (row & 3) : 4 * ((row >> 1) & 1);
}

template <int BM>
__global__ __launch_bounds__(NT, 2) void conv_wgrad_multi_kernel(ConvWgradArgs a, WgradItems it,
                                                                 float* __restrict__ db) {
  constexpr int BN = 128;
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 32, TN = WN / 32;
  constexpr int RBG = BM * 2, RBX = BN * 2;          // LDS row bytes
  constexpr int CPRG = BM / 8, CPRX = BN / 8;        // 16-B chunks per row
  constexpr int GCH = BKP * CPRG, XCH = BKP * CPRX;  // chunks per stage
  static_assert(GCH % NT == 0 && XCH % NT == 0, "whole wave instructions");
  constexpr int G_PER = GCH / NT, X_PER = XCH / NT;
  constexpr int LPS = G_PER + X_PER;
  constexpr int STAGE = (GCH + XCH) * 16;  // bytes
  typedef __amdgpu_buffer_rsrc_t rsrc_t;
  constexpr uint32_t OOB = 0x80000000u;
  __shared__ __attribute__((aligned(16))) uint8_t smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  const int ntile_n = (a.kpad + BN - 1) / BN;
  const int tm = blockIdx.x / ntile_n, tn = blockIdx.x % ntile_n;
  const int m0 = tm * BM, k0 = tn * BN;
  const int item = blockIdx.y / a.splits_per_item;
  const int p_begin = (blockIdx.y - item * a.splits_per_item) * a.pix_per_split;
  const int p_end = min(P, p_begin + a.pix_per_split);
  const int steps = (p_end - p_begin + BKP - 1) / BKP;
  if (steps <= 0) return;  // uniform

  auto mk = [](const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
  };
  const rsrc_t g_rs = mk(it.g[item], (uint32_t)P * a.g_stride * 2u);
  rsrc_t seg_rs[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int qq = q < a.nseg ? q : 0;
    seg_rs[q] = mk(it.seg[item][qq], (uint32_t)P * a.seg[qq].stride * 2u);
  }

  // G chunks: row r (pixel p_begin + r + 64 t), logical channel chunk lc (fixed per lane)
  int g_row[G_PER];
  uint32_t g_col[G_PER];  // byte offset of the chunk within a G row, or OOB
#pragma unroll
  for (int j = 0; j < G_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e / CPRG, lc = (e % CPRG) ^ wg_swz<RBG>(row);
    g_row[j] = row;
    g_col[j] = m0 + lc * 8 < a.cout ? (uint32_t)(m0 + lc * 8) * 2u : OOB;
  }
  // X chunks: packed-K column decoded once, pixel walked incrementally
  int x_dpix[X_PER], x_dy[X_PER], x_dx[X_PER], x_coff[X_PER], x_seg[X_PER];
  int x_p[X_PER], x_y[X_PER], x_x[X_PER];
  bool x_ok[X_PER];
#pragma unroll
  for (int j = 0; j < X_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e / CPRX, lc = (e % CPRX) ^ wg_swz<RBX>(row);
    const int kc = k0 + lc * 8;
    x_ok[j] = kc < a.kpad;
    const int tap = kc / a.cin_pad, c = kc - tap * a.cin_pad;
    const int kh = tap / a.KW, kw = tap - kh * a.KW;
    x_dy[j] = kh - a.PH;
    x_dx[j] = kw - a.PW;
    x_dpix[j] = x_dy[j] * a.W + x_dx[j];
    int sidx = 0, sbase = 0;
#pragma unroll
    for (int q = 0; q < 2; ++q)
      if (sidx + 1 < a.nseg && c >= sbase + a.seg[sidx].cnt) { sbase += a.seg[sidx].cnt; ++sidx; }
    x_coff[j] = c - sbase;
    x_seg[j] = sidx;
    const int p = p_begin + row;
    const int pp = p < P ? p : 0;
    const int r = pp % HW;
    x_p[j] = p;
    x_y[j] = r / a.W;
    x_x[j] = r - (r / a.W) * a.W;
  }

  const uint32_t lds0 = raft_lds_addr(smem);
  const uint32_t wave_off = __builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int t, int buf) {
    const uint32_t base = lds0 + buf * STAGE + wave_off;
    const int pb = p_begin + t * BKP;
#pragma unroll
    for (int j = 0; j < G_PER; ++j) {
      const int p = pb + g_row[j];
      const uint32_t off = (p < p_end && g_col[j] != OOB) ? (uint32_t)p * a.g_stride * 2u + g_col[j] : OOB;
      raft_dma16(g_rs, base + j * NT * 16, off);
    }
#pragma unroll
    for (int j = 0; j < X_PER; ++j) {
      const int p = x_p[j];
      const int yy = x_y[j] + x_dy[j], xx = x_x[j] + x_dx[j];
      const bool ok = x_ok[j] && p < p_end && (unsigned)yy < (unsigned)a.H && (unsigned)xx < (unsigned)a.W;
      // segment widths are multiples of the 128-wide K tile (host check): the segment is
      // wave-uniform, so the descriptor select stays scalar (a per-lane descriptor would make
      // hipcc wrap every DMA in a readfirstlane waterfall loop)
      const int s = __builtin_amdgcn_readfirstlane(x_seg[j]);
      const uint32_t off = (uint32_t)(((p + x_dpix[j]) * a.seg[s].stride + x_coff[j]) * 2);
      const rsrc_t rs = s == 0 ? seg_rs[0] : (s == 1 ? seg_rs[1] : seg_rs[2]);
      raft_dma16(rs, base + (GCH + j * NT) * 16, ok ? off : OOB);
      // advance this chunk's pixel by BKP -- branch-free (a divergent wrap loop here made hipcc
      // drain vmcnt(0) before it, i.e. wait for the DMAs just issued): q = (x + BKP) / W by a
      // magic multiply (exact for (x + BKP) * W < 2^32), at most one image wrap (host: HW >= 128)
      x_p[j] += BKP;
      const uint32_t xn = (uint32_t)(x_x[j] + BKP);
      const uint32_t qw = __umulhi(xn, a.w_magic);
      int yn = x_y[j] + (int)qw;
      yn = yn >= a.H ? yn - a.H : yn;
      x_x[j] = (int)(xn - qw * (uint32_t)a.W);
      x_y[j] = yn;
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
  const bool do_bias = db != nullptr && tn == 0;
  // bias: thread sums 4 adjacent channels over 64 / (NT / (BM / 4)) rows per step
  constexpr int BT = BM / 4;            // threads per row of the bias sweep
  constexpr int BROWS = BKP / (NT / BT);
  const int bcol = (tid % BT) * 4, brow0 = (tid / BT) * BROWS;
  float bsum[4] = {0.f, 0.f, 0.f, 0.f};

  auto rd_tr = [](const uint8_t* base, int rb_row_bytes, int swz, int row, int col) {
    const int off = row * rb_row_bytes + (((col >> 3) ^ swz) << 4) + (col & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(base + off));
  };
  auto compute = [&](int buf) {
    const uint8_t* Gs = smem + buf * STAGE;
    const uint8_t* Xs = Gs + GCH * 16;
#pragma unroll
    for (int s = 0; s < BKP / 16; ++s) {
      bf16x8_t af[TM], bfr[TN];
      const int row = s * 16 + (gi >> 1) * 8 + q;
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int col = wm * WM + i * 32 + (gi & 1) * 16 + 4 * pp;
        bf16x4_t lo = rd_tr(Gs, RBG, wg_swz<RBG>(row), row, col);
        bf16x4_t hi = rd_tr(Gs, RBG, wg_swz<RBG>(row + 4), row + 4, col);
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int col = wn * WN + j * 32 + (gi & 1) * 16 + 4 * pp;
        bf16x4_t lo = rd_tr(Xs, RBX, wg_swz<RBX>(row), row, col);
        bf16x4_t hi = rd_tr(Xs, RBX, wg_swz<RBX>(row + 4), row + 4, col);
        bfr[j] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (do_bias) {
#pragma unroll
      for (int r = 0; r < BROWS; ++r) {
        const int row = brow0 + r;
        const int off = row * RBG + (((bcol >> 3) ^ wg_swz<RBG>(row)) << 4) + (bcol & 7) * 2;
        const uint2 v = *reinterpret_cast<const uint2*>(Gs + off);
        bsum[0] += __uint_as_float(v.x << 16);
        bsum[1] += __uint_as_float(v.x & 0xffff0000u);
        bsum[2] += __uint_as_float(v.y << 16);
        bsum[3] += __uint_as_float(v.y & 0xffff0000u);
      }
    }
  };

  issue(0, 0);
  for (int t = 0; t < steps; ++t) {
    if (t + 1 < steps) {
      issue(t + 1, (t + 1) & 1);
      raft_wait_vmcnt<LPS>();
    } else {
      raft_wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    compute(t & 1);
    __builtin_amdgcn_s_barrier();
  }

  if (do_bias) {
#pragma unroll
    for (int c = 0; c < 4; ++c)
      if (m0 + bcol + c < a.cout) atomicAdd(db + m0 + bcol + c, bsum[c]);
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

bool launch_conv_wgrad_multi(const ConvWgradArgs& a, const WgradItems& it, int bm, float* db,
                             hipStream_t stream) {
  constexpr int BN = 128;
  const int tiles_n = (a.kpad + BN - 1) / BN;
  dim3 grid(raft_cdiv(a.cout, bm) * tiles_n, it.n * a.splits_per_item);
  if (bm == 128) hipLaunchKernelGGL((conv_wgrad_multi_kernel<128>), grid, dim3(NT), 0, stream, a, it, db);
  else if (bm == 64) hipLaunchKernelGGL((conv_wgrad_multi_kernel<64>), grid, dim3(NT), 0, stream, a, it, db);
  else return false;
  return true;
}

void launch_col_sum(const uint16_t* g, int stride, int cout, int P, float* db, hipStream_t stream) {
  // 64 pixels per block (16 per thread row): ~P/64 x cout/64 blocks keep every CU busy; the
  // reduction is latency-bound, not bandwidth-bound, at 1024 pixels per block (measured 60 us)
  const int ppb = 64;
  dim3 grid(raft_cdiv(cout, 64), raft_cdiv(P, ppb));
  hipLaunchKernelGGL(col_sum_kernel, grid, dim3(256), 0, stream, g, stride, cout, P, ppb, db);
}
