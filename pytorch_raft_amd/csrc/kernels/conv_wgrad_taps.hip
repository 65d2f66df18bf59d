// Tap-fused weight gradient of the NHWC implicit-GEMM convolutions (bf16 MFMA, fp32 accumulation).
//
//   dW[co][t][ci] = sum_items sum_p  G[p][co] * X[p + off(t)][ci]      db[co] = sum G[p][co]
//
// conv_wgrad_multi_kernel (conv_wgrad.hip) tiles the packed K = taps x Cin in 128-wide tiles, so a
// pixel's gradient row G[p] is re-read once per K tile (15x for the 1x5 GRU convs) and its input
// row X[p] once per tap and Cout tile (10x): ~26 GB of L2->CU traffic per training step
// (profiles/r2/pmc_step_s2.txt).  Here a workgroup owns (128 Cout) x (64 Cin) x ALL taps and walks
// 8x8-pixel chunks: per chunk the G tile (64 px x 128 co) and the X halo tile
// ((8+KH-1) x (8+KW-1) px x 64 ci) go global -> LDS once (LDS-DMA, double buffered) and every tap
// is a shifted view of the halo:  T x 2 MFMA 32x32x16 per 16-pixel k-step per wave, the G fragment
// read once per k-step for all taps.
//
// MFMA operands via ds_read_b64_tr_b16 (pixel-major LDS rows -> 8 consecutive pixels per lane):
// A = G^T (rows co), B = X (cols ci); a 16-lane group reads 4 pixel rows x 16 columns, rows of the
// B operand are halo rows of the tap-shifted pixels (4 consecutive pixels never cross a tile row,
// so they are 4 consecutive halo rows: the same conflict-free swizzle as the dense kernel).
//
// Split-K over the chunks (items x images x 8x8 tiles): every workgroup stores its partial tile
// with plain 128-B row stores into a workspace (no same-address float atomics: 64 partial tiles
// per output would pile up ~100 MB of memory-side atomics per launch); conv_wgrad_reduce_kernel
// then adds the partials (fixed order: deterministic) into dW / db.
#include "common.h"
#include "launchers.h"

#include <cstdlib>

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr int BC = 64;            // Cin per workgroup
constexpr int TP = 8;             // pixel tile edge (8 x 8 = 64 pixels per chunk)
constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ rsrc_t mk_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

// LDS images: G rows 256 B (128 co) or 128 B (64 co), X rows 128 B (64 ci); XOR swizzle of the
// 16-B chunk index by row
__device__ __forceinline__ int swz_g(int row) { return 4 * (row & 3); }
__device__ __forceinline__ int swz_x(int row) { return 4 * ((row >> 1) & 1); }
template <int ROWB>
__device__ __forceinline__ int swz_rows(int row) { return ROWB == 256 ? swz_g(row) : swz_x(row); }

// Workgroup = BMT Cout (64 or 128) x 64 Cin x all taps.  TG tap groups x (BMT / 64) x 2 waves;
// wave (tg, wm, wn) owns taps [tg*TPG, +TPG) of Cout [wm*64, +64) x Cin [wn*32, +32).  TG = 2
// for 3x3 at BMT = 128 keeps 2 x 5 accumulator tiles per wave (2 waves per SIMD instead of 1
// wave holding all 18: the second wave hides the first one's LDS / barrier waits); BMT = 64
// (Cout <= 64: the encoders' 64-channel layers, the motion encoder's f2) uses TG = 3.
template <int KH, int KW, int TG, int BMT>
struct TapGeo {
  static constexpr int WMW = BMT / 64;                // waves along Cout
  static constexpr int NT = 64 * WMW * 2 * TG;
  static constexpr int GRB = BMT * 2;                 // G row bytes
  static constexpr int G_CPR = BMT / 8;               // 16-B chunks per G row
  static constexpr int T = KH * KW;
  static constexpr int TPG = (T + TG - 1) / TG;      // taps per group
  static constexpr int HWD = TP + KW - 1;            // halo width
  static constexpr int HALO = (TP + KH - 1) * HWD;   // halo rows (pixels)
  static constexpr int G_CH = 64 * G_CPR;            // 16-B chunks of the G tile
  static constexpr int X_CH = HALO * (BC / 8);
  static constexpr int G_PER = (G_CH + NT - 1) / NT;  // DMA instructions per thread
  static constexpr int X_PER = (X_CH + NT - 1) / NT;
  static constexpr int G_BYTES = G_PER * NT * 16;    // lane-linear DMA images (rounded up)
  static constexpr int X_BYTES = X_PER * NT * 16;    // lane-linear DMA image (rounded up)
  static constexpr int STAGE = G_BYTES + X_BYTES;
};

// NS: LDS pipeline stages.  The 128-Cout 3x3 kernel runs one workgroup per CU (its accumulators
// fill the register file), so a chunk's DMA has to land behind the MFMAs of NS - 1 earlier chunks:
// with two stages the ~1300-cycle chunk of MFMAs did not cover the global -> LDS latency (39% MFMA
// busy, profiles/r2/pmc_step_final.txt).  The other kernels keep two stages and two or three
// resident workgroups per CU instead.
template <int KH, int KW, int TG, int BMT, int NS, bool F16>
__global__ __launch_bounds__((TapGeo<KH, KW, TG, BMT>::NT), 1) void conv_wgrad_taps_kernel(
    ConvWgradArgs a, WgradItems it, WgradTapArgs ta) {
  using Geo = TapGeo<KH, KW, TG, BMT>;
  constexpr int NT = Geo::NT, GRB = Geo::GRB, G_CPR = Geo::G_CPR, WMW = Geo::WMW;
  constexpr int T = Geo::T, TPG = Geo::TPG, HWD = Geo::HWD, HALO = Geo::HALO;
  constexpr int G_PER = Geo::G_PER, X_PER = Geo::X_PER, LPS = G_PER + X_PER;
  static_assert(NS >= 2 && NS <= 4, "2..4 pipeline stages");
  static_assert(NS * Geo::STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) uint8_t smem[NS * Geo::STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int HW = a.H * a.W;
  const int P = a.B * HW;
  // XCD-aware block order: the dispatcher deals consecutive workgroups round-robin over the 8
  // XCDs, so logical block L = (lin % 8) * (grid / 8) + lin / 8 puts the n_co x n_ci workgroups of
  // one chunk range (which read the same G and X tiles) on the SAME XCD, sharing its L2
  const int pairs = ta.n_co * ta.n_ci;
  const int L = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
  if (L >= pairs * ta.splits) return;            // grid padded to a multiple of 8
  const int pair = L % pairs;
  const int ci_chunk = pair % ta.n_ci;
  const int m0 = (pair / ta.n_ci) * BMT;
  const int ci_cnt = ta.ci_cnt[ci_chunk];         // valid channels of this chunk (64 or 32)
  const int sidx = ta.ci_seg[ci_chunk];           // input segment of this Cin chunk (uniform)
  const int coff = ta.ci_off[ci_chunk];           // channel offset inside that segment
  const int kbase = ta.ci_k[ci_chunk];            // first packed-K column of this chunk (tap 0)
  const int split = L / pairs;
  const int c_begin = split * ta.chunks_per_split;
  const int c_end = min(ta.total_chunks, c_begin + ta.chunks_per_split);
  const int nsteps = c_end - c_begin;
  const bool do_bias = ta.db_part != nullptr && ci_chunk == 0;
  const int stride = a.seg[sidx].stride;

  // DMA slots: G chunk e = tid + j*NT -> (pixel row e / G_CPR, physical 16-B chunk e % G_CPR);
  // slots past the tile (rounding of the lane-linear image) load nothing
  int g_row[G_PER];
  uint32_t g_col[G_PER];
#pragma unroll
  for (int j = 0; j < G_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e / G_CPR, lc = (e % G_CPR) ^ swz_rows<GRB>(row);
    g_row[j] = row < 64 ? row : 0;
    g_col[j] = (row < 64 && m0 + lc * 8 < a.cout) ? (uint32_t)(m0 + lc * 8) * 2u : OOB;
  }
  int x_hy[X_PER], x_hx[X_PER];
  uint32_t x_col[X_PER];
#pragma unroll
  for (int j = 0; j < X_PER; ++j) {
    const int e = tid + j * NT;
    const int row = e >> 3, lc = (e & 7) ^ swz_x(row);
    x_hy[j] = row < HALO ? row / HWD : -(1 << 20);
    x_hx[j] = row < HALO ? row % HWD : 0;
    x_col[j] = (uint32_t)(coff + lc * 8) * 2u;
  }

  const uint32_t lds0 = raft_lds_addr(smem);
  const uint32_t wave_off = __builtin_amdgcn_readfirstlane(wave * 64 * 16);
  auto issue = [&](int c, int buf) {
    // chunk c -> (item, image, tile y, tile x): all wave-uniform
    const int item = c / ta.chunks_per_item;
    int r = c - item * ta.chunks_per_item;
    const int b = r / ta.tiles_per_img;
    r -= b * ta.tiles_per_img;
    const int ty = r / ta.tiles_x, tx = r - ty * ta.tiles_x;
    const int y0 = ty * TP, x0 = tx * TP;
    const rsrc_t g_rs = mk_rsrc(it.g[item], (uint32_t)P * a.g_stride * 2u);
    const rsrc_t x_rs = mk_rsrc(it.seg[item][sidx], (uint32_t)P * stride * 2u);
    const uint32_t base = lds0 + buf * Geo::STAGE + wave_off;
#pragma unroll
    for (int j = 0; j < G_PER; ++j) {
      const int py = y0 + (g_row[j] >> 3), px = x0 + (g_row[j] & 7);
      const bool ok = py < a.H && px < a.W && g_col[j] != OOB;
      const uint32_t off = (uint32_t)((b * HW + py * a.W + px) * a.g_stride) * 2u + g_col[j];
      raft_dma16(g_rs, base + j * NT * 16, ok ? off : OOB);
    }
#pragma unroll
    for (int j = 0; j < X_PER; ++j) {
      const int py = y0 - a.PH + x_hy[j], px = x0 - a.PW + x_hx[j];
      const bool ok = (unsigned)py < (unsigned)a.H && (unsigned)px < (unsigned)a.W;
      const uint32_t off = (uint32_t)((b * HW + py * a.W + px) * stride) * 2u + x_col[j];
      raft_dma16(x_rs, base + Geo::G_BYTES + j * NT * 16, ok ? off : OOB);
    }
  };

  // wave (tg, wm, wn): per 16-pixel k-step 2 G fragments (shared by the group's taps) + TPG X
  // fragments for 2 TPG MFMAs
  const int tg = __builtin_amdgcn_readfirstlane(wave / (2 * WMW));
  const int wm = (wave >> 1) % WMW, wn = wave & 1;
  const int t0 = tg * TPG;
  f32x16 acc[TPG][2];
#pragma unroll
  for (int t = 0; t < TPG; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[t][i][r] = 0.f;
  // bias: lane l of a wn == 0 wave sums G[co = l % 32][its 8 pixels] straight from the A fragments
  const bool bias_wave = do_bias && wn == 0 && tg == 0;
  float bsum[2] = {0.f, 0.f};

  const int gi = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  auto rd_tr = [](const uint8_t* base, int row_bytes, int swz, int row, int col) {
    const int off = row * row_bytes + (((col >> 3) ^ swz) << 4) + (col & 7) * 2;
    return __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(base + off));
  };
  const int a_col = wm * 64 + (gi & 1) * 16 + 4 * pp;   // Cout column of this lane's A reads (+32 i)
  const int b_col = wn * 32 + (gi & 1) * 16 + 4 * pp;   // Cin column of its B reads

  // split-fp32 items (binding): only the leading db_items items' G columns enter the bias sum
  // (chunks are item-major: a chunk index bound, no division)
  const int db_end = ta.db_items > 0 ? ta.db_items * ta.chunks_per_item : 0x7fffffff;
  auto compute = [&](int buf, int cidx) {
    const bool bias_now = bias_wave && cidx < db_end;
    const uint8_t* Gs = smem + buf * Geo::STAGE;
    const uint8_t* Xs = Gs + Geo::G_BYTES;
#pragma unroll
    for (int s = 0; s < 4; ++s) {              // 4 k-steps of 16 pixels (2 tile rows)
      const int k = s * 16 + (gi >> 1) * 8 + q;   // this lane's first pixel (second: k + 4)
      bf16x8_t af[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bf16x4_t lo = rd_tr(Gs, GRB, swz_rows<GRB>(k), k, a_col + 32 * i);
        const bf16x4_t hi = rd_tr(Gs, GRB, swz_rows<GRB>(k + 4), k + 4, a_col + 32 * i);
        af[i] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
      if (bias_now) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int e = 0; e < 8; ++e)
            bsum[i] += F16 ? (float)__builtin_bit_cast(raft_v8f16, af[i])[e] : (float)af[i][e];
      }
      const int ky0 = k >> 3, kx0 = k & 7;     // k and k + 4 share the tile row
#pragma unroll
      for (int tt = 0; tt < TPG; ++tt) {
        const int t = t0 + tt;
        if (TPG * TG != T && t >= T) break;    // last group of an uneven split
        const int dy = t / KW, dx = t - dy * KW;
        const int h0 = (ky0 + dy) * HWD + kx0 + dx;
        const int h1 = h0 + 4;
        const bf16x4_t lo = rd_tr(Xs, 128, swz_x(h0), h0, b_col);
        const bf16x4_t hi = rd_tr(Xs, 128, swz_x(h1), h1, b_col);
        const bf16x8_t bfr = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[tt][i] = raft_mfma32<F16>(af[i], bfr, acc[tt][i]);
      }
    }
  };

  if constexpr (NS == 2) {
    if (nsteps > 0) {
      issue(c_begin, 0);
      for (int t = 0; t < nsteps; ++t) {
        if (t + 1 < nsteps) {
          issue(c_begin + t + 1, (t + 1) & 1);
          raft_wait_vmcnt<LPS>();
        } else {
          raft_wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        compute(t & 1, c_begin + t);
        __builtin_amdgcn_s_barrier();
      }
    }
  } else {
    // NS-stage ring, ONE barrier per chunk: wait (counted vmcnt) for this wave's chunk-t DMAs with
    // the newer stages still in flight -> barrier (every wave's chunk-t data landed AND every wave
    // finished computing chunk t-1) -> issue chunk t+NS-1 into the buffer chunk t-1 used -> MFMAs
#pragma unroll
    for (int q = 0; q < NS - 1; ++q)
      if (q < nsteps) issue(c_begin + q, q);
    int cur = 0;
    for (int t = 0; t < nsteps; ++t) {
      const int newer = min(NS - 2, nsteps - 1 - t);
      if (NS >= 4 && newer >= 2) raft_wait_vmcnt<(NS >= 4 ? 2 : 0) * LPS>();
      else if (newer >= 1) raft_wait_vmcnt<LPS>();
      else raft_wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
      if (t + NS - 1 < nsteps) {
        int nb = cur + NS - 1;
        nb = nb >= NS ? nb - NS : nb;
        issue(c_begin + t + NS - 1, nb);
      }
      compute(cur, c_begin + t);
      cur = cur + 1 == NS ? 0 : cur + 1;
    }
  }

  // partial tile -> workspace [split][cout][kpad]: 32 lanes = 32 consecutive Cin = 128-B rows.
  // A 32-channel tail chunk (Cin = 96) stores only its wn = 0 half: the packed K has no padding
  // there, so the other half's columns belong to the next tap.
  float* part = ta.w_part + (int64_t)split * a.cout * a.kpad;
  const bool ci_ok = wn * 32 < ci_cnt;
#pragma unroll
  for (int tt = 0; tt < TPG; ++tt)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int t = t0 + tt;
      if (TPG * TG != T && t >= T) break;
      if (!ci_ok) break;
      const int kc = t * a.cin_pad + kbase + wn * 32 + (lane & 31);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = m0 + wm * 64 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (n < a.cout) part[(int64_t)n * a.kpad + kc] = acc[tt][i][r];
      }
    }
  if (bias_wave) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float v = bsum[i] + __shfl_xor(bsum[i], 32);   // lanes l, l + 32: the two k halves
      const int co = m0 + wm * 64 + i * 32 + lane;
      if (lane < 32 && co < a.cout) ta.db_part[(int64_t)split * a.cout + co] = v;
    }
  }
}

// dw[i] += sum_s part[s][i]: 16 float4 columns x 16 split groups per workgroup (split group g
// sums splits g, g + 16, ... with 4 loads in flight), then a fixed-order LDS combine over the
// groups: deterministic, and ~splits/16 dependent load rounds instead of splits
// dw_bf16 != null: store bf16(sum) (fp16 when dw_f16) there instead (no fp32 read-modify-write; the encoders'
// bf16 weight gradients, packed (co, tap, ci) = the channels_last weight layout)
__global__ __launch_bounds__(256) void conv_wgrad_reduce_kernel(const float* __restrict__ part,
                                                                int splits, int64_t n,
                                                                float* __restrict__ dw,
                                                                const float* __restrict__ bpart,
                                                                int cout, float* __restrict__ db,
                                                                uint16_t* __restrict__ dw_bf16,
                                                                int dw_f16) {
  __shared__ float4 red[16][17];
  const int col = threadIdx.x & 15, grp = threadIdx.x >> 4;
  const int64_t n4 = n / 4;
  const int64_t nbw = (n4 + 15) / 16;
  if (blockIdx.x >= nbw) {                   // bias columns: same scheme, scalar
    float* rs = reinterpret_cast<float*>(red);
    const int c = (int)(blockIdx.x - nbw) * 16 + col;
    float t = 0.f;
    if (c < cout)
      for (int k = grp; k < splits; k += 16) t += bpart[(int64_t)k * cout + c];
    rs[grp * 16 + col] = t;
    __syncthreads();
    if (grp == 0 && c < cout) {
      float u = db[c];
      for (int g = 0; g < 16; ++g) u += rs[g * 16 + col];
      db[c] = u;
    }
    return;
  }
  const int64_t v = (int64_t)blockIdx.x * 16 + col;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (v < n4) {
    const float4* p = reinterpret_cast<const float4*>(part) + v;
    int k = grp;
    for (; k + 48 < splits; k += 64) {
      const float4 a0 = p[(int64_t)k * n4], a1 = p[(int64_t)(k + 16) * n4];
      const float4 a2 = p[(int64_t)(k + 32) * n4], a3 = p[(int64_t)(k + 48) * n4];
      s.x += (a0.x + a1.x) + (a2.x + a3.x); s.y += (a0.y + a1.y) + (a2.y + a3.y);
      s.z += (a0.z + a1.z) + (a2.z + a3.z); s.w += (a0.w + a1.w) + (a2.w + a3.w);
    }
    for (; k < splits; k += 16) {
      const float4 a0 = p[(int64_t)k * n4];
      s.x += a0.x; s.y += a0.y; s.z += a0.z; s.w += a0.w;
    }
  }
  red[grp][col] = s;
  __syncthreads();
  if (grp == 0 && v < n4) {
    float4 t = dw_bf16 ? make_float4(0.f, 0.f, 0.f, 0.f) : reinterpret_cast<const float4*>(dw)[v];
#pragma unroll
    for (int g = 0; g < 16; ++g) {
      const float4 r = red[g][col];
      t.x += r.x; t.y += r.y; t.z += r.z; t.w += r.w;
    }
    if (dw_bf16 && dw_f16) {
      const uint32_t lo = (uint32_t)raft_f2h<true>(t.x) | ((uint32_t)raft_f2h<true>(t.y) << 16);
      const uint32_t hi = (uint32_t)raft_f2h<true>(t.z) | ((uint32_t)raft_f2h<true>(t.w) << 16);
      reinterpret_cast<uint2*>(dw_bf16)[v] = make_uint2(lo, hi);
    } else if (dw_bf16) {
      const uint32_t lo = (uint32_t)raft_f32_to_bf16(t.x) | ((uint32_t)raft_f32_to_bf16(t.y) << 16);
      const uint32_t hi = (uint32_t)raft_f32_to_bf16(t.z) | ((uint32_t)raft_f32_to_bf16(t.w) << 16);
      reinterpret_cast<uint2*>(dw_bf16)[v] = make_uint2(lo, hi);
    } else {
      reinterpret_cast<float4*>(dw)[v] = t;
    }
  }
}

template <int KH, int KW, int TG, int BMT, int NS>
void launch_taps(const ConvWgradArgs& a, const WgradItems& it, const WgradTapArgs& ta,
                 hipStream_t stream) {
  dim3 grid((ta.n_co * ta.n_ci * ta.splits + 7) / 8 * 8);
  if (a.f16)
    hipLaunchKernelGGL((conv_wgrad_taps_kernel<KH, KW, TG, BMT, NS, true>), grid,
                       dim3(TapGeo<KH, KW, TG, BMT>::NT), 0, stream, a, it, ta);
  else
    hipLaunchKernelGGL((conv_wgrad_taps_kernel<KH, KW, TG, BMT, NS, false>), grid,
                       dim3(TapGeo<KH, KW, TG, BMT>::NT), 0, stream, a, it, ta);
}

int taps_stages_3x3() {
  static const int ns = [] {
    const char* e = getenv("RAFT_WGRAD_STAGES");  // A/B: 2 = the round-3 pipeline
    const int v = e ? atoi(e) : 4;
    return v == 2 || v == 3 ? v : 4;
  }();
  return ns;
}

}  // namespace

bool launch_conv_wgrad_taps(const ConvWgradArgs& a, const WgradItems& it, const WgradTapArgs& ta,
                            float* db, hipStream_t stream) {
  const int ns = taps_stages_3x3();
  if (ta.bm == 64) {
    // two resident workgroups per CU (6 waves, 60 KB each) cover each other's DMA latency
    if (a.KH == 3 && a.KW == 3) launch_taps<3, 3, 3, 64, 2>(a, it, ta, stream);
    else return false;
  } else if (a.KH == 1 && a.KW == 1) launch_taps<1, 1, 1, 128, 2>(a, it, ta, stream);
  else if (a.KH == 1 && a.KW == 5) launch_taps<1, 5, 1, 128, 2>(a, it, ta, stream);
  else if (a.KH == 5 && a.KW == 1) launch_taps<5, 1, 1, 128, 2>(a, it, ta, stream);
  else if (a.KH == 3 && a.KW == 3) {
    if (ns == 4) launch_taps<3, 3, 2, 128, 4>(a, it, ta, stream);
    else if (ns == 3) launch_taps<3, 3, 2, 128, 3>(a, it, ta, stream);
    else launch_taps<3, 3, 2, 128, 2>(a, it, ta, stream);
  } else {
    return false;
  }
  const int64_t n = (int64_t)a.cout * a.kpad;
  const bool bias = ta.db_part != nullptr && db != nullptr;
  const unsigned blocks = (unsigned)((n / 4 + 15) / 16 + (bias ? (a.cout + 15) / 16 : 0));
  hipLaunchKernelGGL(conv_wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, stream, ta.w_part,
                     ta.splits, n, a.dw, bias ? ta.db_part : nullptr, a.cout, db, ta.dw_bf16, ta.dw_f16);
  return true;
}

int conv_wgrad_taps_max_ci_chunks() { return RAFT_WG_MAX_CI_CHUNKS; }
