// On-the-fly ("alternate") correlation lookup on MFMA, forward + backward, O(HW * r^2) memory.
//
// Capability parity with `alt_cuda_corr` (`alt_cuda_corr/correlation_kernel.cu:18-119` forward,
// `:122-256` backward) and `AlternateCorrBlock` (`core/corr.py:63-91`), re-designed for CDNA4:
//
// * A workgroup owns an 8x8 tile of query pixels (64 = two 32-row MFMA blocks).  Per pyramid level
//   it takes the bounding box of the tile's (2r+2)^2 integer windows, clipped to the map (flow is
//   locally smooth, so at chairs this is ~18x18 positions at level 0 and shrinks with the level),
//   and computes the dense tile GEMM S = F1_tile (64 x C) * F2_box^T (C x U) with
//   v_mfma_f32_32x32x16_bf16 (fp32 accumulation).  fmap2 rows are streamed through LDS in chunks
//   of 64 positions (register prefetch of the next chunk overlaps the MFMAs); the fmap1 fragments
//   stay in registers for all levels.  Each accumulator element is dropped into the owning pixel's
//   private (2r+2)^2 window in LDS, from which the (2r+1)^2 bilinear taps are blended.  The
//   reference does the same dots one 32-channel slice at a time on scalar FMAs.
// * Backward per level: the bilinear adjoint gives each pixel's window gradient dW (LDS); per chunk
//   dS (64 px x 64 pos, bf16) is scattered from dW, then two MFMA GEMMs run with transposed LDS
//   fragments (ds_read_b64_tr_b16):  dF1_tile += dS * F2_chunk (kept in registers across chunks and
//   levels, one plain store per tile) and dF2_chunk = dS^T * F1_tile (fp32 atomics, 128-B
//   segments, into a per-level gradient buffer that persists across GRU iterations).
// * Pixels whose window misses the map entirely do not widen the box; every coordinate is clamped
//   and bounds-checked (the reference backward reads coords out of range when H % 4 or W % 8 != 0,
//   and relies on 32-thread lock-step for its LDS hand-offs).
// * Output is written channels-last (B, H, W, S) at channel l*(2r+1)^2 + tap, x-offset-major tap
//   order (`core/corr.py:37-43`); the channels [L*(2r+1)^2, S) are zero-filled so the bf16 variant
//   feeds the fused update block's first 1x1 conv directly.
#include "common.h"
#include "launchers.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;

constexpr int TPX = 8;     // query tile width
constexpr int TP = 64;     // query pixels per tile (8 x 8)
constexpr int NCH = 64;    // fmap2 positions per LDS chunk
constexpr int NT = 256;

struct OtfLvls {
  const uint16_t* f2[4];
  float* g2[4];
  int h[4];
  int w[4];
  // deterministic dF2 (backward): a tile's box gradient goes to its private slab rows
  // slab[l][tile][cap[l]][C] and its box to boxes[tile][l] (bw = 0: not slabbed -- an empty box,
  // or one past the capacity, whose rows went out as float atomics instead); the reduce kernel
  // then sums the overlapping tiles' rows per fmap2 position in tile order
  float* slab[4];
  int cap[4];
  int* boxes;
  // 1: the dS operand is the bf16 RESIDUAL of the window gradient, v - bf16(v) (the fp32-accurate
  // backward: passes (dS_hi, F_hi) + (dS_lo, F_hi) + (dS_hi, F_lo) accumulate into the gradients)
  int dslo;
};

__device__ __forceinline__ float clampc(float v) { return fminf(fmaxf(v, -1.0e6f), 1.0e6f); }

__device__ __forceinline__ int wave_min_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = min(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ int wave_max_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware work decode: the dispatcher deals consecutive workgroups round-robin over the 8 XCDs,
// so workgroup ids are mapped to give each XCD a contiguous range of ceil(n_items / 8) query
// tiles (the same images and neighbouring tiles, whose fmap2 boxes overlap, meet in one XCD's L2)
// for every group (pyramid level / backward half), groups in order inside each XCD.  The grid is
// 8 * ceil(n_items / 8) * n_groups; false for the padding workgroups.
__device__ __forceinline__ bool xcd_item(int n_items, int n_groups, int& group, int& item) {
  const int per = (n_items + 7) / 8;
  const int x = (int)(blockIdx.x & 7), k = (int)(blockIdx.x >> 3);
  group = k / per;
  item = x * per + (k - group * per);
  return group < n_groups && item < n_items;
}
inline unsigned xcd_grid(int n_items, int n_groups) { return 8u * (unsigned)((n_items + 7) / 8) * (unsigned)n_groups; }

struct Geo {
  int x0[TP], y0[TP];
  float ax[TP], ay[TP];
  int box[4];  // bx0, by0, bw, bh
};

// wave 0, lane = tile pixel: window origin / fractions at level l and the tile's clipped box
template <int R>
__device__ __forceinline__ void tile_geometry(Geo& g, int lane, bool act, float x, float y, int l,
                                              int hl, int wl) {
  constexpr int E = 2 * R + 2;
  const float inv = 1.f / (float)(1 << l);
  const float cx = clampc(x * inv), cy = clampc(y * inv);
  const float fx = floorf(cx), fy = floorf(cy);
  const int x0 = (int)fx - R, y0 = (int)fy - R;
  const bool hit = act && x0 <= wl - 1 && x0 + E - 1 >= 0 && y0 <= hl - 1 && y0 + E - 1 >= 0;
  g.x0[lane] = act ? x0 : -(1 << 28);
  g.y0[lane] = act ? y0 : -(1 << 28);
  g.ax[lane] = cx - fx;
  g.ay[lane] = cy - fy;
  const int mnx = wave_min_i(hit ? x0 : 0x7fffffff);
  const int mxx = wave_max_i(hit ? x0 + E - 1 : -0x7fffffff);
  const int mny = wave_min_i(hit ? y0 : 0x7fffffff);
  const int mxy = wave_max_i(hit ? y0 + E - 1 : -0x7fffffff);
  if (lane == 0) {
    const int bx0 = max(mnx, 0), bx1 = min(mxx, wl - 1);
    const int by0 = max(mny, 0), by1 = min(mxy, hl - 1);
    const bool ok = bx1 >= bx0 && by1 >= by0;
    g.box[0] = bx0;
    g.box[1] = by0;
    g.box[2] = ok ? bx1 - bx0 + 1 : 0;
    g.box[3] = ok ? by1 - by0 + 1 : 0;
  }
}

__device__ __forceinline__ bf16x8_t ld_frag(const uint16_t* p) {
  return __builtin_bit_cast(bf16x8_t, *reinterpret_cast<const uint4*>(p));
}
__device__ __forceinline__ bf16x8_t zero_frag() {
  return __builtin_bit_cast(bf16x8_t, make_uint4(0, 0, 0, 0));
}
// 8-deep K fragment of a [k][col] LDS matrix (row stride S elements) for columns base..base+31
__device__ __forceinline__ bf16x8_t tr_frag(const uint16_t* X, int S, int kbase, int base,
                                            int lane) {
  const int gi = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int col = base + (gi & 1) * 16 + 4 * pp;
  const int row = kbase + (gi >> 1) * 8 + q;
  bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(X + row * S + col));
  bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(X + (row + 4) * S + col));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// chunk of NCH fmap2 positions of the box -> registers (zero rows past U)
template <int C>
struct ChunkLoader {
  static constexpr int LPR = C / 8;             // 16-B units per position row
  static constexpr int PER = NCH * LPR / NT;    // units per thread
  uint4 r[PER];
  __device__ __forceinline__ void load(const uint16_t* F2, int wl, int bx0, int by0, int bw, int U,
                                       int c, int tid) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = tid + j * NT;
      const int n = e / LPR, q = e % LPR;
      const int pos = c * NCH + n;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (pos < U) {
        const int iy = by0 + pos / bw, ix = bx0 + pos % bw;
        v = *reinterpret_cast<const uint4*>(F2 + ((int64_t)iy * wl + ix) * C + q * 8);
      }
      r[j] = v;
    }
  }
  __device__ __forceinline__ void store(uint16_t* Bs, int RS, int tid) {
#pragma unroll
    for (int j = 0; j < PER; ++j) {
      const int e = tid + j * NT;
      const int n = e / LPR, q = e % LPR;
      *reinterpret_cast<uint4*>(Bs + n * RS + q * 8) = r[j];
    }
  }
};

// SPLIT: fp32-accurate mode, operands carried as bf16 hi + lo parts (x ~= hi + lo) and
// S = hi*hi + hi*lo + lo*hi on three MFMAs (~2^-16 relative error instead of bf16's 2^-9).
template <int R, int C, typename TO, bool SPLIT>
__global__ __launch_bounds__(NT, SPLIT ? 1 : 2) void corr_otf_fwd_kernel(
    const uint16_t* __restrict__ f1, const uint16_t* __restrict__ f1lo, OtfLvls lv, OtfLvls lo,
    const float* __restrict__ coords, TO* __restrict__ out, int ostride, int B, int H, int W, int levels, int tiles_x, int tiles_y,
    float isc) {
  constexpr int D = 2 * R + 1, E = D + 1, NP = E * E, DD = D * D;
  constexpr int KS = C / 16;
  constexpr int RS = C + 16;  // padded LDS row (bf16)
  constexpr int NB = SPLIT ? 2 : 1;
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NB * NCH * RS];
  __shared__ float win[TP * NP];
  __shared__ Geo geo;

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int mb = wave & 1, nh = wave >> 1;
  // one workgroup per (pyramid level, query tile), level-major within each XCD's tile range: the
  // heavy level-0 boxes are dispatched first and the light coarse levels fill the tail (one launch
  // is ~4.5 rounds of the chip instead of ~1.1 with a last round 1/8 full); levels write disjoint
  // output channels
  const int ntile = B * tiles_x * tiles_y;
  int lev, t;
  if (!xcd_item(ntile, levels, lev, t)) return;
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int b = t / tiles_y;
  const int HW = H * W;

  // fmap1 fragments of this wave's 32 pixels, all K, kept for every level
  bf16x8_t af[KS], afl[SPLIT ? KS : 1];
  {
    const int p = mb * 32 + (lane & 31);
    const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
    const bool act = py < H && px < W;
    const int64_t off = ((int64_t)b * HW + (act ? py * W + px : 0)) * C + 8 * (lane >> 5);
#pragma unroll
    for (int s = 0; s < KS; ++s) af[s] = act ? ld_frag(f1 + off + 16 * s) : zero_frag();
    if constexpr (SPLIT) {
#pragma unroll
      for (int s = 0; s < KS; ++s) afl[s] = act ? ld_frag(f1lo + off + 16 * s) : zero_frag();
    }
  }
  // wave 0 owns the per-pixel coordinates
  float cxv = 0.f, cyv = 0.f;
  bool cact = false;
  if (wave == 0) {
    const int py = ty * TPX + lane / TPX, px = tx * TPX + lane % TPX;
    cact = py < H && px < W;
    if (cact) {
      cxv = coords[((int64_t)b * 2) * HW + py * W + px];
      cyv = coords[((int64_t)b * 2 + 1) * HW + py * W + px];
    }
  }

  ChunkLoader<C> ld, ldl;
  {
    const int l = lev;
    const int hl = lv.h[l], wl = lv.w[l];
    if (wave == 0) tile_geometry<R>(geo, lane, cact, cxv, cyv, l, hl, wl);
    for (int e = tid; e < TP * NP; e += NT) win[e] = 0.f;
    __syncthreads();
    const int bx0 = geo.box[0], by0 = geo.box[1], bw = geo.box[2], bh = geo.box[3];
    const int U = bw * bh;
    const int nchunk = (U + NCH - 1) / NCH;
    const int64_t boff = (int64_t)b * hl * wl * C;
    const uint16_t* F2 = lv.f2[l] + boff;
    const uint16_t* F2l = SPLIT ? lo.f2[l] + boff : nullptr;
    if (nchunk > 0) {
      ld.load(F2, wl, bx0, by0, bw, U, 0, tid);
      if constexpr (SPLIT) ldl.load(F2l, wl, bx0, by0, bw, U, 0, tid);
    }
    for (int c = 0; c < nchunk; ++c) {
      ld.store(Bs, RS, tid);
      if constexpr (SPLIT) ldl.store(Bs + NCH * RS, RS, tid);
      __syncthreads();
      if (c + 1 < nchunk) {
        ld.load(F2, wl, bx0, by0, bw, U, c + 1, tid);
        if constexpr (SPLIT) ldl.load(F2l, wl, bx0, by0, bw, U, c + 1, tid);
      }
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      const int nb = nh * 32 + (lane & 31);
#pragma unroll
      for (int s = 0; s < KS; ++s) {
        const bf16x8_t bf = ld_frag(Bs + nb * RS + 16 * s + 8 * (lane >> 5));
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bf, acc, 0, 0, 0);
        if constexpr (SPLIT) {
          const bf16x8_t bl = ld_frag(Bs + (NCH + nb) * RS + 16 * s + 8 * (lane >> 5));
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af[s], bl, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afl[s], bf, acc, 0, 0, 0);
        }
      }
      const int pos = c * NCH + nb;
      if (pos < U) {
        const int iy = by0 + pos / bw, ix = bx0 + pos % bw;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int p = mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          const int rx = ix - geo.x0[p], ry = iy - geo.y0[p];
          if ((unsigned)rx < (unsigned)E && (unsigned)ry < (unsigned)E)
            win[p * NP + ry * E + rx] = acc[r] * isc;
        }
      }
      __syncthreads();
    }
    // bilinear taps from the windows (x-offset-major tap order)
    for (int e = tid; e < TP * DD; e += NT) {
      const int p = e / DD, tt = e % DD;
      const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
      if (py >= H || px >= W) continue;
      const int ix = tt / D, iy = tt % D;
      const float* w0 = &win[p * NP + iy * E + ix];
      const float ax = geo.ax[p], ay = geo.ay[p];
      const float v = (1.f - ay) * ((1.f - ax) * w0[0] + ax * w0[1]) +
                      ay * ((1.f - ax) * w0[E] + ax * w0[E + 1]);
      St<TO>::put(out, ((int64_t)b * HW + py * W + px) * ostride + l * DD + tt, v);
    }
    __syncthreads();
  }
  const int pad = ostride - levels * DD;
  if (pad > 0 && lev == levels - 1) {
    for (int e = tid; e < TP * pad; e += NT) {
      const int p = e / pad, cc = e % pad;
      const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
      if (py < H && px < W)
        St<TO>::put(out, ((int64_t)b * HW + py * W + px) * ostride + levels * DD + cc, 0.f);
    }
  }
}

// Window origins of the multi-iteration backward, packed (x0 & 0xffff) | (y0 << 16): a window
// that hits the map has -E < x0 < w_l, -E < y0 < h_l (the launcher bounds the maps below 2^15)
constexpr int WMISS = -32768;
__device__ __forceinline__ int pack_xy(int x0, int y0) { return (int)(((unsigned)x0 & 0xffffu) | ((unsigned)y0 << 16)); }
__device__ __forceinline__ int unpack_x(int v) { return (int)(short)(v & 0xffff); }
__device__ __forceinline__ int unpack_y(int v) { return v >> 16; }

// wave 0, lane = tile pixel: window origins (packed) and bilinear fractions of every iteration in
// `wl` at level l + the union box.  The pixel's coordinates of all iterations were loaded into
// registers once per tile (cx/cy, NIT entries, the first wl.n valid): no global load here.
template <int R, int NIT>
__device__ __forceinline__ void tile_geometry_multi(int (*gxy)[TP], float (*fx)[TP], float (*fy)[TP],
                                                    int* box, const float* cxr, const float* cyr,
                                                    int n, int lane, bool act, int l, int hl,
                                                    int w_l) {
  constexpr int E = 2 * R + 2;
  const float inv = 1.f / (float)(1 << l);
  int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    if (it >= n) break;
    int x0 = WMISS, y0 = WMISS;
    float ax = 0.f, ay = 0.f;
    if (act) {
      const float cx = clampc(cxr[it] * inv);
      const float cy = clampc(cyr[it] * inv);
      ax = cx - floorf(cx);
      ay = cy - floorf(cy);
      x0 = (int)floorf(cx) - R;
      y0 = (int)floorf(cy) - R;
      if (x0 <= w_l - 1 && x0 + E - 1 >= 0 && y0 <= hl - 1 && y0 + E - 1 >= 0) {
        mnx = min(mnx, x0);
        mxx = max(mxx, x0 + E - 1);
        mny = min(mny, y0);
        mxy = max(mxy, y0 + E - 1);
      } else {
        x0 = y0 = WMISS;  // misses the map: contributes nothing
      }
    }
    gxy[it][lane] = pack_xy(x0, y0);
    fx[it][lane] = ax;
    fy[it][lane] = ay;
  }
  mnx = wave_min_i(mnx);
  mxx = wave_max_i(mxx);
  mny = wave_min_i(mny);
  mxy = wave_max_i(mxy);
  if (lane == 0) {
    const int bx0 = max(mnx, 0), bx1 = min(mxx, w_l - 1);
    const int by0 = max(mny, 0), by1 = min(mxy, hl - 1);
    const bool ok = bx1 >= bx0 && by1 >= by0;
    box[0] = bx0;
    box[1] = by0;
    box[2] = ok ? bx1 - bx0 + 1 : 0;
    box[3] = ok ? by1 - by0 + 1 : 0;
  }
}

// Window-gradient cell (rx, ry) in [0, 2r+2)^2 of one lookup: the bilinear adjoint of its
// (2r+1)^2 bf16 tap gradients T (x-offset-major, tap ix*D + iy; ax, ay = the lookup centre's
// fractions), in the expression order of corr_window_grad_kernel.
template <int R>
__device__ __forceinline__ float win_cell(const uint16_t* T, int rx, int ry, float ax, float ay) {
  constexpr int D = 2 * R + 1;
  float acc = 0.f;
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int iy = ry - k;
    if (iy < 0 || iy >= D) continue;
    const float wy = k == 0 ? (1.f - ay) : ay;
    float s = 0.f;
    if (rx < D) s += (1.f - ax) * raft_bf16_to_f32(T[rx * D + iy]);
    if (rx > 0) s += ax * raft_bf16_to_f32(T[(rx - 1) * D + iy]);
    acc += wy * s;
  }
  return acc;
}

// MULTI = false: one lookup's gradient, dout (B,H,W,dstride) -> bilinear adjoint in LDS.
// MULTI = true : every iteration of the step at once, straight from the iterations' bf16 tap
//                gradients (WinList dout / coords), so the fmap2 box GEMMs and the dF2 atomics
//                run once per step over the union box instead of once per iteration.
template <int R, int C, typename TD, bool MULTI>
__global__ __launch_bounds__(NT, 1) void corr_otf_bwd_kernel(
    const uint16_t* __restrict__ f1, OtfLvls lv, const float* __restrict__ coords,
    const TD* __restrict__ dout, int dstride, WinList wl, float* __restrict__ df1,
    float* __restrict__ df1b, int B, int H, int W, int levels, int tiles_x, int tiles_y, float isc) {
  constexpr int D = 2 * R + 1, E = D + 1, NP = E * E, DD = D * D;
  constexpr int RS = C + 16;       // [row][channel] bf16 rows (fmap1 tile, fmap2 chunk)
  constexpr int SS = NCH + 16;     // dS [pixel][position] bf16 rows
  constexpr int WC = C / 4;        // channels per wave
  constexpr int TN = WC / 32;      // 32-column MFMA blocks per wave
  constexpr int NIT = MULTI ? RAFT_MAX_WIN : 1;
  __shared__ __attribute__((aligned(16))) uint16_t F1s[TP * RS];
  __shared__ __attribute__((aligned(16))) uint16_t Bs[NCH * RS];
  __shared__ __attribute__((aligned(16))) uint16_t dS[TP * SS];
  __shared__ float dwin[MULTI ? 1 : TP * NP];
  __shared__ int gx[1][TP], gy[1][TP];   // !MULTI: the lookup's window origins
  // MULTI: every iteration's packed window origins and bilinear fractions at the current level
  __shared__ int gxy[NIT][TP];
  __shared__ float pax[NIT][TP], pay[NIT][TP];
  struct GeoBox { int box[4]; };
  __shared__ std::conditional_t<MULTI, GeoBox, Geo> geo;
  // MULTI: per pixel, the sum over the iterations of its window gradients on a UG x UG grid at
  // the union of its windows (the windows of one pixel move only a few positions over a step),
  // so building a dS chunk element is one LDS read instead of a global read per iteration
  constexpr int UG = 15, UGG = UG * UG;
  __shared__ float ugrid[MULTI ? TP * UGG : 1];
  __shared__ int uxy[MULTI ? 2 * TP + 1 : 1];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  // df1b != nullptr (MULTI, levels >= 2): two workgroups per query tile -- the first ntile
  // blocks take levels 1..levels-1 (three union grids: the heavier half, dispatched first) and
  // store their dF1 part to df1b; the next ntile take level 0 and add theirs to df1.  The
  // launcher then adds df1b to df1 (fixed order).  At one workgroup per CU (160 KB LDS) the
  // 2x tiles fill the chip's rounds instead of leaving a 1/4-full last one.
  const int ntile = B * tiles_x * tiles_y;
  int half, t;
  if (!xcd_item(ntile, df1b != nullptr ? 2 : 1, half, t)) return;   // no barrier before this
  int lbeg = 0, lend = levels;
  bool part = false;
  if (df1b != nullptr) {
    part = half == 0;
    if (part) lbeg = 1;
    else lend = 1;
  }
  const int tile = t;
  const int tx = t % tiles_x;
  t /= tiles_x;
  const int ty = t % tiles_y;
  const int b = t / tiles_y;
  const int HW = H * W;

  // fmap1 tile -> LDS [pixel][channel]
  for (int e = tid; e < TP * (C / 8); e += NT) {
    const int p = e / (C / 8), q = e % (C / 8);
    const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
    uint4 v = make_uint4(0, 0, 0, 0);
    if (py < H && px < W)
      v = *reinterpret_cast<const uint4*>(f1 + ((int64_t)b * HW + py * W + px) * C + q * 8);
    *reinterpret_cast<uint4*>(F1s + p * RS + q * 8) = v;
  }
  float cxv = 0.f, cyv = 0.f;
  bool cact = false;
  int64_t cidx = 0;
  if (wave == 0) {
    const int py = ty * TPX + lane / TPX, px = tx * TPX + lane % TPX;
    cact = py < H && px < W;
    cidx = (int64_t)b * 2 * HW + (cact ? py * W + px : 0);
    if (cact && !MULTI) {
      cxv = coords[cidx];
      cyv = coords[cidx + HW];
    }
  }
  // MULTI: wave 0's pixel coordinates of every iteration, all loads in flight at once (the
  // per-level geometry then reads registers, not a chain of dependent global loads)
  float cxr[NIT], cyr[NIT];
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    cxr[it] = 0.f;
    cyr[it] = 0.f;
    if (MULTI && wave == 0 && cact && it < wl.n) {
      cxr[it] = wl.coords[it][cidx];
      cyr[it] = wl.coords[it][cidx + HW];
    }
  }

  f32x16 g1[2][TN];  // dF1: 64 pixels x this wave's WC channels
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) g1[i][j][r] = 0.f;

  ChunkLoader<C> ld;
  for (int l = lbeg; l < lend; ++l) {
    const int hl = lv.h[l], wl_ = lv.w[l];
    if (wave == 0) {
      if constexpr (MULTI) {
        tile_geometry_multi<R, NIT>(gxy, pax, pay, geo.box, cxr, cyr, wl.n, lane, cact, l, hl, wl_);
      } else {
        tile_geometry<R>(geo, lane, cact, cxv, cyv, l, hl, wl_);
        gx[0][lane] = geo.x0[lane];
        gy[0][lane] = geo.y0[lane];
      }
    }
    __syncthreads();
    if constexpr (!MULTI) {
      // adjoint of the bilinear blend: window position (qx, qy) collects from up to 4 taps
      for (int e = tid; e < TP * NP; e += NT) {
        const int p = e / NP, qq = e % NP;
        const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
        float g = 0.f;
        if (py < H && px < W) {
          const int qx = qq % E, qy = qq / E;
          const float ax = geo.ax[p], ay = geo.ay[p];
          const TD* dO = dout + ((int64_t)b * HW + py * W + px) * dstride + l * DD;
#pragma unroll
          for (int dyi = 0; dyi < 2; ++dyi)
#pragma unroll
            for (int dxi = 0; dxi < 2; ++dxi) {
              const int ix = qx - dxi, iy = qy - dyi;
              if (ix >= 0 && ix < D && iy >= 0 && iy < D)
                g += (dxi ? ax : 1.f - ax) * (dyi ? ay : 1.f - ay) * Ld<TD>::get(dO, ix * D + iy);
            }
        }
        dwin[e] = g * isc;
      }
      __syncthreads();
    }
    bool ufits = false;
    if constexpr (MULTI) {
      // union origin of each pixel's windows; the fast path needs every pixel's union <= UG^2
      if (wave == 0) {
        int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
        for (int it = 0; it < wl.n; ++it) {
          const int v = gxy[it][lane];
          const int x0 = unpack_x(v), y0 = unpack_y(v);
          if (x0 != WMISS) {
            mnx = min(mnx, x0);
            mxx = max(mxx, x0);
            mny = min(mny, y0);
            mxy = max(mxy, y0);
          }
        }
        const bool none = mnx > mxx;
        const bool fit = none || (mxx - mnx + E <= UG && mxy - mny + E <= UG);
        uxy[lane] = none ? -(1 << 28) : mnx;
        uxy[TP + lane] = none ? -(1 << 28) : mny;
        const bool all = __builtin_amdgcn_read_exec() == __ballot(fit);
        if (lane == 0) uxy[2 * TP] = all ? 1 : 0;
      }
      __syncthreads();
      ufits = uxy[2 * TP] != 0;
      if (ufits) {
        // Per iteration (fixed order), each window cell of each pixel adds the bilinear adjoint of
        // up to 4 of its bf16 tap gradients into the pixel's union grid: within one iteration the
        // cells of a pixel's window are distinct grid cells (one writer each), and a barrier
        // separates the iterations -- deterministic, no atomics.  The 64 pixels' level-l taps of
        // iteration it+1 (16-B pieces of the 8-aligned span around l*D*D) are loaded into
        // registers before iteration it's cells are added and written to LDS after them (the
        // fmap2 chunk buffer, free here; two slots), so the loads' latency hides behind the adds:
        // the window gradients never go through global memory.
        constexpr int TROW = ((DD + 7 + 7) / 8) * 8;  // staged taps per pixel (8-aligned span)
        constexpr int SPT = (TP * (TROW / 8) + NT - 1) / NT;  // 16-B pieces per thread
        // two slots (stage it+1 during it) where the chunk buffer holds them (C = 256), else one
        constexpr int NSLOT = 2 * TP * TROW <= NCH * RS ? 2 : 1;
        static_assert(TP * TROW <= NCH * RS, "a tap slot fits the chunk buffer");
        const int t0 = (l * DD) & ~7, tpieces = ((l * DD + DD + 7) & ~7) / 8 - t0 / 8;
        uint4 sv[SPT];
        auto issue = [&](int it) {
#pragma unroll
          for (int j = 0; j < SPT; ++j) {
            const int e = tid + j * NT;
            const int p = e / tpieces, q = e - p * tpieces;
            const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
            uint4 v = make_uint4(0, 0, 0, 0);
            if (e < TP * tpieces && py < H && px < W)
              v = *reinterpret_cast<const uint4*>(wl.dout[it] + ((int64_t)b * HW + py * W + px) * wl.cbuf + t0 + q * 8);
            sv[j] = v;
          }
        };
        auto commit = [&](int it) {
          uint16_t* Ts = Bs + (it % NSLOT) * TP * TROW;
#pragma unroll
          for (int j = 0; j < SPT; ++j) {
            const int e = tid + j * NT;
            const int p = e / tpieces, q = e - p * tpieces;
            if (e < TP * tpieces) *reinterpret_cast<uint4*>(Ts + p * TROW + q * 8) = sv[j];
          }
        };
        for (int e = tid; e < TP * UGG; e += NT) ugrid[e] = 0.f;
        if (NSLOT == 2 && wl.n > 0) {
          issue(0);
          commit(0);
        }
        for (int it = 0; it < wl.n; ++it) {
          __syncthreads();  // iteration it-1's adds done; 2 slots: it committed
          if (NSLOT == 1) {
            issue(it);
            commit(it);
            __syncthreads();
          } else if (it + 1 < wl.n) {
            issue(it + 1);
          }
          const uint16_t* Ts = Bs + (it % NSLOT) * TP * TROW + (l * DD - t0);
          // fixed trip count, unrolled: several cells' LDS reads in flight per wave (one wave
          // per SIMD here, so a cell-at-a-time loop waits out every LDS latency)
          static_assert(TP * NP % NT == 0, "whole cells per thread");
#pragma unroll 4
          for (int k = 0; k < TP * NP / NT; ++k) {
            const int e = tid + k * NT;
            const int p = e / NP, qq = e - p * NP;
            const int v = gxy[it][p];
            const int x0 = unpack_x(v);
            if (x0 != WMISS) {  // WMISS: this iteration's window misses the map
              const int ry = qq / E, rx = qq - ry * E;
              const int cy = unpack_y(v) - uxy[TP + p] + ry, cxg = x0 - uxy[p] + rx;
              ugrid[p * UGG + cy * UG + cxg] += win_cell<R>(Ts + p * TROW, rx, ry, pax[it][p], pay[it][p]);
            }
          }
          // 2 slots: slot (it+1) % 2 was last read by iteration it-1's adds (before the barrier)
          if (NSLOT == 2 && it + 1 < wl.n) commit(it + 1);
        }
        __syncthreads();
      }
    }
    const int bx0 = geo.box[0], by0 = geo.box[1], bw = geo.box[2], bh = geo.box[3];
    const int U = bw * bh;
    const int nchunk = (U + NCH - 1) / NCH;
    const uint16_t* F2 = lv.f2[l] + (int64_t)b * hl * wl_ * C;
    float* G2 = lv.g2[l] + (int64_t)b * hl * wl_ * C;
    const bool slabbed = lv.slab[l] != nullptr && U > 0 && U <= lv.cap[l];
    float* S2 = slabbed ? lv.slab[l] + (int64_t)tile * lv.cap[l] * C : nullptr;
    if (lv.boxes != nullptr && tid == 0) {
      int* bx = lv.boxes + ((int64_t)tile * 4 + l) * 4;
      bx[0] = bx0;
      bx[1] = by0;
      bx[2] = slabbed ? bw : 0;
      bx[3] = slabbed ? bh : 0;
    }
    if (nchunk > 0) ld.load(F2, wl_, bx0, by0, bw, U, 0, tid);
    for (int c = 0; c < nchunk; ++c) {
      ld.store(Bs, RS, tid);
      // dS chunk (64 px x 64 positions)
      static_assert(TP * NCH % NT == 0, "whole dS elements per thread");
#pragma unroll 4
      for (int k = 0; k < TP * NCH / NT; ++k) {
        const int e = tid + k * NT;
        const int p = e / NCH, n = e % NCH;
        const int pos = c * NCH + n;
        float v = 0.f;
        if (pos < U) {
          const int iy = by0 + pos / bw, ix = bx0 + pos % bw;
          if constexpr (MULTI) {
            if (ufits) {
              const int rx = ix - uxy[p], ry = iy - uxy[TP + p];
              if ((unsigned)rx < (unsigned)UG && (unsigned)ry < (unsigned)UG)
                v = ugrid[p * UGG + ry * UG + rx];
            } else {  // a pixel's windows spread wider than the grid: from the global taps
              const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
              const int64_t pix = (int64_t)b * HW + py * W + px;
              for (int it = 0; it < wl.n; ++it) {  // fixed order -> deterministic
                const int g = gxy[it][p];  // WMISS: rx out of range
                const int rx = ix - unpack_x(g), ry = iy - unpack_y(g);
                if ((unsigned)rx < (unsigned)E && (unsigned)ry < (unsigned)E)
                  v += win_cell<R>(wl.dout[it] + pix * wl.cbuf + l * DD, rx, ry, pax[it][p], pay[it][p]);
              }
            }
            v *= isc;
          } else {
            const int rx = ix - gx[0][p], ry = iy - gy[0][p];
            if ((unsigned)rx < (unsigned)E && (unsigned)ry < (unsigned)E)
              v = dwin[p * NP + ry * E + rx];
          }
        }
        if (lv.dslo) v -= raft_bf16_to_f32(raft_f32_to_bf16(v));
        dS[p * SS + n] = raft_f32_to_bf16(v);
      }
      __syncthreads();
      if (c + 1 < nchunk) ld.load(F2, wl_, bx0, by0, bw, U, c + 1, tid);

      // dF1 (64 px x WC) += dS (64 px x 64 pos) * F2 chunk (64 pos x WC)
#pragma unroll
      for (int ks = 0; ks < NCH / 16; ++ks) {
        bf16x8_t a[2], bb[TN];
#pragma unroll
        for (int i = 0; i < 2; ++i)
          a[i] = ld_frag(dS + (i * 32 + (lane & 31)) * SS + 16 * ks + 8 * (lane >> 5));
#pragma unroll
        for (int j = 0; j < TN; ++j) bb[j] = tr_frag(Bs, RS, 16 * ks, wave * WC + j * 32, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            g1[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], bb[j], g1[i][j], 0, 0, 0);
      }
      // dF2 chunk (64 pos x WC) = dS^T (64 pos x 64 px) * F1 tile (64 px x WC)
      f32x16 g2[2][TN];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int r = 0; r < 16; ++r) g2[i][j][r] = 0.f;
#pragma unroll
      for (int ks = 0; ks < TP / 16; ++ks) {
        bf16x8_t a[2], bb[TN];
#pragma unroll
        for (int i = 0; i < 2; ++i) a[i] = tr_frag(dS, SS, 16 * ks, i * 32, lane);
#pragma unroll
        for (int j = 0; j < TN; ++j) bb[j] = tr_frag(F1s, RS, 16 * ks, wave * WC + j * 32, lane);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j)
            g2[i][j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[i], bb[j], g2[i][j], 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int pos = c * NCH + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
          if (pos >= U) continue;
          if (slabbed) {  // plain 128-B row stores into this tile's slab rows
            float* dst = S2 + (int64_t)pos * C + wave * WC + (lane & 31);
#pragma unroll
            for (int j = 0; j < TN; ++j) dst[j * 32] = g2[i][j][r];
          } else {
            const int iy = by0 + pos / bw, ix = bx0 + pos % bw;
            float* dst = G2 + ((int64_t)iy * wl_ + ix) * C + wave * WC + (lane & 31);
#pragma unroll
            for (int j = 0; j < TN; ++j) atomicAdd(dst + j * 32, g2[i][j][r]);
          }
        }
      __syncthreads();
    }
    __syncthreads();  // every wave has read this level's box before wave 0 rewrites it
  }
  // dF1: the tile owns its pixels (launches on one stream are ordered) -> plain read-modify-write
  // (the coarse-level part: a plain store into its own buffer)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int p = i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      const int py = ty * TPX + p / TPX, px = tx * TPX + p % TPX;
      if (py >= H || px >= W) continue;
      const int64_t o = ((int64_t)b * HW + py * W + px) * C + wave * WC + (lane & 31);
      if (part) {
#pragma unroll
        for (int j = 0; j < TN; ++j) df1b[o + j * 32] = g1[i][j][r];
      } else {
#pragma unroll
        for (int j = 0; j < TN; ++j) df1[o + j * 32] += g1[i][j][r];
      }
    }
}

// df1 += df1b (the coarse levels' dF1 part of the split multi-iteration backward)
__global__ __launch_bounds__(256) void add_f32_kernel(float* __restrict__ a, const float* __restrict__ b,
                                                      int64_t n4) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 x = reinterpret_cast<float4*>(a)[i];
    const float4 y = reinterpret_cast<const float4*>(b)[i];
    x.x += y.x; x.y += y.y; x.z += y.z; x.w += y.w;
    reinterpret_cast<float4*>(a)[i] = x;
  }
}

OtfLvls make_lvls(const uint16_t* const* f2, float* const* g2, const int* hs, const int* ws,
                  int levels) {
  OtfLvls p;
  for (int l = 0; l < 4; ++l) {
    p.f2[l] = l < levels ? f2[l] : nullptr;
    p.g2[l] = (g2 && l < levels) ? g2[l] : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
    p.slab[l] = nullptr;
    p.cap[l] = 0;
  }
  p.boxes = nullptr;
  p.dslo = 0;
  return p;
}

// dF2 of one level, deterministic: workgroup = an 8 x 8 block of fmap2 positions x 64 channels;
// thread = 4 positions x 4 channels (float4).  The query tiles of the same image are visited in
// tile order; a tile whose slabbed box covers a position contributes that slab row.  The sum is
// added to the level gradient (which may already hold atomically-added unslabbed boxes).
template <int C>
__global__ __launch_bounds__(256) void corr_otf_df2_reduce_kernel(const float* __restrict__ slab, int cap,
                                                                  const int* __restrict__ boxes, int l,
                                                                  int tiles_img, int hl, int wl,
                                                                  float* __restrict__ g2) {
  const int ptx = (wl + 7) / 8, pty = (hl + 7) / 8;
  int t = blockIdx.x;
  const int bx = t % ptx;
  t /= ptx;
  const int by = t % pty;
  const int b = t / pty;
  const int c0 = blockIdx.y * 64 + (threadIdx.x & 15) * 4;
  const int pr = threadIdx.x >> 4;
  float4 acc[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) acc[k] = make_float4(0.f, 0.f, 0.f, 0.f);
  const int y0 = by * 8, x0 = bx * 8;
  for (int q = 0; q < tiles_img; ++q) {
    const int64_t T = (int64_t)b * tiles_img + q;
    const int4 box = *reinterpret_cast<const int4*>(boxes + (T * 4 + l) * 4);
    const int bw = box.z, bh = box.w;
    if (bw == 0) continue;  // uniform
    if (box.x > x0 + 7 || box.x + bw <= x0 || box.y > y0 + 7 || box.y + bh <= y0) continue;
    const float* S = slab + T * cap * C + c0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int p = pr + 16 * k;
      const int py = y0 + (p >> 3), px = x0 + (p & 7);
      const int ry = py - box.y, rx = px - box.x;
      if ((unsigned)ry < (unsigned)bh && (unsigned)rx < (unsigned)bw) {
        const float4 v = *reinterpret_cast<const float4*>(S + (int64_t)(ry * bw + rx) * C);
        acc[k].x += v.x; acc[k].y += v.y; acc[k].z += v.z; acc[k].w += v.w;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int p = pr + 16 * k;
    const int py = y0 + (p >> 3), px = x0 + (p & 7);
    if (py >= hl || px >= wl) continue;
    float4* dst = reinterpret_cast<float4*>(g2 + (((int64_t)b * hl + py) * wl + px) * C + c0);
    float4 o = *dst;
    o.x += acc[k].x; o.y += acc[k].y; o.z += acc[k].z; o.w += acc[k].w;
    *dst = o;
  }
}

}  // namespace

#define OTF_CASES(LAUNCH)                                        \
  do {                                                           \
    if (radius == 4 && C == 256) { LAUNCH(4, 256); return true; } \
    if (radius == 3 && C == 128) { LAUNCH(3, 128); return true; } \
    if (radius == 4 && C == 128) { LAUNCH(4, 128); return true; } \
    if (radius == 3 && C == 256) { LAUNCH(3, 256); return true; } \
    return false;                                                \
  } while (0)

bool launch_corr_otf_fwd(const uint16_t* f1, const uint16_t* const* f2lvl, const uint16_t* f1lo,
                         const uint16_t* const* f2lo, const int* hs, const int* ws, int levels,
                         const float* coords, void* out, int out_bf16, int ostride, int B, int C,
                         int H, int W, int radius, hipStream_t stream) {
  const OtfLvls p = make_lvls(f2lvl, nullptr, hs, ws, levels);
  const OtfLvls q = make_lvls(f2lo ? f2lo : f2lvl, nullptr, hs, ws, levels);
  const bool split = f1lo != nullptr && f2lo != nullptr;
  const int tx = (W + TPX - 1) / TPX, ty = (H + TPX - 1) / TPX;
  if (levels < 1 || levels > 4) return false;
  const dim3 grid(xcd_grid(B * tx * ty, levels));
  const float isc = 1.f / sqrtf((float)C);
#define FWD(RR, CC, TO, SP)                                                                     \
  hipLaunchKernelGGL((corr_otf_fwd_kernel<RR, CC, TO, SP>), grid, dim3(NT), 0, stream, f1, f1lo, \
                     p, q, coords, (TO*)out, ostride, B, H, W, levels, tx, ty, isc)
#define FWD_BF16(RR, CC) FWD(RR, CC, uint16_t, false)
#define FWD_F32(RR, CC) FWD(RR, CC, float, false)
#define FWD_BF16_SPLIT(RR, CC) FWD(RR, CC, uint16_t, true)
#define FWD_F16_SPLIT(RR, CC) FWD(RR, CC, Fp16Bits, true)
#define FWD_F32_SPLIT(RR, CC) FWD(RR, CC, float, true)
  // out_bf16: 0 fp32, 1 bf16, 2 fp16 (the fp32-accurate split forward under fp16 autocast)
  if (split) {
    if (out_bf16 == 2) OTF_CASES(FWD_F16_SPLIT);
    if (out_bf16) OTF_CASES(FWD_BF16_SPLIT);
    OTF_CASES(FWD_F32_SPLIT);
  }
  if (out_bf16 == 2) return false;
  if (out_bf16) OTF_CASES(FWD_BF16);
  OTF_CASES(FWD_F32);
#undef FWD
}

void launch_df2_reduce(float* const* slab, const int* cap, const int* boxes, int levels,
                       const int* hs, const int* ws, int tiles_img, int B, int C, float* const* df2lvl,
                       hipStream_t stream);

bool launch_corr_otf_bwd(const uint16_t* f1, const uint16_t* const* f2lvl, const int* hs,
                         const int* ws, int levels, const float* coords, const void* dout,
                         int dout_bf16, int dstride, float* df1, float* const* df2lvl, int B,
                         int C, int H, int W, int radius, float* const* slab, const int* cap,
                         int* boxes, int dslo, hipStream_t stream) {
  if (!((radius == 4 || radius == 3) && (C == 128 || C == 256))) return false;
  OtfLvls p = make_lvls(f2lvl, df2lvl, hs, ws, levels);
  p.dslo = dslo;
  if (slab != nullptr) {
    for (int l = 0; l < levels; ++l) {
      p.slab[l] = slab[l];
      p.cap[l] = cap[l];
    }
    p.boxes = boxes;
  }
  const int tx = (W + TPX - 1) / TPX, ty = (H + TPX - 1) / TPX;
  const dim3 grid(xcd_grid(B * tx * ty, 1));
  const float isc = 1.f / sqrtf((float)C);
  WinList none;
  none.n = 0;
#define BWD(RR, CC, TD)                                                                        \
  hipLaunchKernelGGL((corr_otf_bwd_kernel<RR, CC, TD, false>), grid, dim3(NT), 0, stream, f1, p, \
                     coords, (const TD*)dout, dstride, none, df1, nullptr, B, H, W, levels, tx, ty, isc)
#define BWD_BF16(RR, CC) BWD(RR, CC, uint16_t)
#define BWD_F32(RR, CC) BWD(RR, CC, float)
  if (dout_bf16) {
    if (radius == 4 && C == 256) BWD_BF16(4, 256);
    else if (radius == 3 && C == 128) BWD_BF16(3, 128);
    else if (radius == 4 && C == 128) BWD_BF16(4, 128);
    else BWD_BF16(3, 256);
  } else {
    if (radius == 4 && C == 256) BWD_F32(4, 256);
    else if (radius == 3 && C == 128) BWD_F32(3, 128);
    else if (radius == 4 && C == 128) BWD_F32(4, 128);
    else BWD_F32(3, 256);
  }
#undef BWD
  if (slab != nullptr) launch_df2_reduce(slab, cap, boxes, levels, hs, ws, tx * ty, B, C, df2lvl, stream);
  return true;
}

void launch_df2_reduce(float* const* slab, const int* cap, const int* boxes, int levels,
                       const int* hs, const int* ws, int tiles_img, int B, int C, float* const* df2lvl,
                       hipStream_t stream) {
  for (int l = 0; l < levels; ++l) {
    const dim3 rg((unsigned)(B * ((hs[l] + 7) / 8) * ((ws[l] + 7) / 8)), (unsigned)(C / 64));
    if (C == 256)
      hipLaunchKernelGGL(corr_otf_df2_reduce_kernel<256>, rg, dim3(256), 0, stream, slab[l], cap[l],
                         boxes, l, tiles_img, hs[l], ws[l], df2lvl[l]);
    else
      hipLaunchKernelGGL(corr_otf_df2_reduce_kernel<128>, rg, dim3(256), 0, stream, slab[l], cap[l],
                         boxes, l, tiles_img, hs[l], ws[l], df2lvl[l]);
  }
}

int otf_tiles(int B, int H, int W) { return B * ((W + TPX - 1) / TPX) * ((H + TPX - 1) / TPX); }

bool launch_corr_otf_window_bwd(const uint16_t* f1, const uint16_t* const* f2lvl, const int* hs,
                                const int* ws, int levels, const WinList& wl, float* df1,
                                float* const* df2lvl, int B, int C, int H, int W, int radius,
                                float* const* slab, const int* cap, int* boxes, float* df1b,
                                hipStream_t stream) {
  if (wl.n < 1 || wl.n > RAFT_MAX_WIN) return false;
  if (!((radius == 4 || radius == 3) && (C == 128 || C == 256))) return false;
  for (int l = 0; l < levels; ++l)
    if (hs[l] >= 32000 || ws[l] >= 32000) return false;  // 16-bit packed window origins
  OtfLvls p = make_lvls(f2lvl, df2lvl, hs, ws, levels);
  if (slab != nullptr) {
    for (int l = 0; l < levels; ++l) {
      p.slab[l] = slab[l];
      p.cap[l] = cap[l];
    }
    p.boxes = boxes;
  }
  const int tx = (W + TPX - 1) / TPX, ty = (H + TPX - 1) / TPX;
  if (levels < 2) df1b = nullptr;
  const dim3 grid(xcd_grid(B * tx * ty, df1b != nullptr ? 2 : 1));
  const float isc = 1.f / sqrtf((float)C);
#define BWDW(RR, CC)                                                                           \
  hipLaunchKernelGGL((corr_otf_bwd_kernel<RR, CC, float, true>), grid, dim3(NT), 0, stream, f1, \
                     p, nullptr, (const float*)nullptr, 0, wl, df1, df1b, B, H, W, levels, tx, ty, isc)
  if (radius == 4 && C == 256) BWDW(4, 256);
  else if (radius == 3 && C == 128) BWDW(3, 128);
  else if (radius == 4 && C == 128) BWDW(4, 128);
  else BWDW(3, 256);
#undef BWDW
  if (df1b != nullptr) {
    const int64_t n4 = (int64_t)B * H * W * C / 4;
    const unsigned blocks = (unsigned)std::min<int64_t>((n4 + 255) / 256, 256 * 16);
    hipLaunchKernelGGL(add_f32_kernel, dim3(blocks), dim3(256), 0, stream, df1, df1b, n4);
  }
  if (slab != nullptr) launch_df2_reduce(slab, cap, boxes, levels, hs, ws, tx * ty, B, C, df2lvl, stream);
  return true;
}
