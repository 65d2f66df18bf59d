// NHWC correlation lookup for the fused update block + window-compact backward.
//
// Forward (corr_lookup_rows_kernel): a workgroup owns 4 consecutive query pixels; every window
// row of every (pixel, level) is fetched as whole aligned 16-B pieces into LDS, the (2r+1)^2
// bilinear taps are interpolated into an LDS tile, and the tile is written out as whole pixel
// rows of the 16-bit (B,H,W,Cbuf) buffer the first 1x1 conv reads, zero padding included (no
// separate memset, no scattered 2-byte stores).  bf16 or fp32 pyramids; bf16, fp16 or split-fp32
// taps.
//
// Backward, two phases instead of a dense read-modify-write of the whole pyramid gradient:
//  1. per iteration (corr_window_grad_kernel): the adjoint of one pixel's bilinear window is a
//     (2r+2)^2 integer-position patch per level; it is written COMPACTLY, [b][i][level][row][col]
//     fp32 -- fully coalesced, ~55 MB per iteration at chairs/B=12 instead of RMW traffic spread
//     over a 500 MB buffer.
//  2. once per step (corr_window_reduce_kernel): a workgroup per query pixel accumulates every
//     iteration's patches into per-level planes held in LDS (iterations in a fixed order ->
//     deterministic), applies the avg-pool adjoint (level l cell -> its 2^l x 2^l level-0 block,
//     weight 4^-l) and 1/sqrt(C), and streams the level-0 gradient row of dcorr (B, N, N) out once.
//     That matrix feeds the two backward GEMMs (dF1 = F2 dC^T, dF2 = F1 dC).
#include "common.h"
#include "launchers.h"

#include <algorithm>
#include <cstdlib>

namespace {

struct PyrC4 {
  const float* lvl[4];
  int h[4];
  int w[4];
};

__device__ __forceinline__ float clampc(float v) { return fminf(fmaxf(v, -1.0e7f), 1.0e7f); }

constexpr int TP = 64;  // pixels per workgroup of the window-gradient kernel

// Row-vector lookup (the launcher's kernel for every pyramid / tap type): the window of a
// (pixel, level) is 2r+2 rows of 2r+2 consecutive cells of the pixel's correlation plane.  Phase 1
// fetches every window row as whole ALIGNED 16-B pieces (bf16 cells: 2, or 3 when the row
// straddles a third piece; fp32 cells: 3 or 4) -- a few vector loads per row instead of 2r+2
// scalar gathers, all of a thread's rows in flight at once -- and parks them raw in LDS; phase 2
// reads the row cells at the row's start offset inside its pieces (LDS indexing is free), masks
// cells outside the plane and interpolates the (2r+1)^2 taps into the pixel-row tile; phase 3
// streams the tile out as 16-B pixel-row pieces.
//   PF32: fp32 pyramid (the fp16 / fp32 schedules: the reference's fp32 correlation), else bf16
//   OT:   output taps 0 bf16, 1 fp16, 2 split fp32 (bf16 hi at channel c, bf16(v - hi) at
//         cbuf + c of a 2 cbuf-wide row: the fp32 schedule's fused update block)
// pixels per workgroup: the TPVK template parameter (16: 42 KB LDS, three workgroups per CU; 8: 21 KB)

// one aligned 16-B piece; a piece that runs past the range end (the last rows of the range's
// last plane) is read as four range-checked dwords: a 16-B load that is only partly in range
// returns zeros for all of it, in-range bytes included
__device__ __forceinline__ uint4 piece16(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t lim) {
  if (off == 0x80000000u || off + 16u <= lim)
    return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
  return make_uint4(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0),
                    __builtin_amdgcn_raw_buffer_load_b32(r, off + 4u, 0, 0),
                    __builtin_amdgcn_raw_buffer_load_b32(r, off + 8u, 0, 0),
                    __builtin_amdgcn_raw_buffer_load_b32(r, off + 12u, 0, 0));
}

template <int R, int TPVK, bool PF32 = false, int OT = 0>
__global__ __launch_bounds__(256) void corr_lookup_rows_kernel(PyrC4 pyr, const float* __restrict__ coords,
                                                               uint16_t* __restrict__ out, int cbuf,
                                                               int B, int H, int W, int levels) {
  constexpr int D = 2 * R + 1, E = D + 1;
  constexpr int ROWT = (4 * D * D + 7) / 8 * 8;
  constexpr uint32_t OOB = 0x80000000u;
  constexpr int ES = PF32 ? 4 : 2;         // bytes per pyramid cell
  constexpr int EPP = 16 / ES;             // cells per 16-B piece
  constexpr int NPC = (EPP - 1 + E + EPP - 1) / EPP;  // pieces a row can touch
  constexpr int NH = OT == 2 ? 2 : 1;      // halves of an output row
  __shared__ __attribute__((aligned(16))) uint4 rows[TPVK * 4 * E * NPC];
  __shared__ float cxy[TPVK * 4 * 2];
  __shared__ __attribute__((aligned(16))) uint16_t tile[NH * TPVK * ROWT];
  const int N = H * W;
  const int tiles = (N + TPVK - 1) / TPVK;
  const int b = blockIdx.x / tiles;
  const int i0 = (blockIdx.x % tiles) * TPVK;
  const int tid = threadIdx.x;
  const int npx = min(TPVK, N - i0);
  if (tid < TPVK * 4) {
    const int px = tid >> 2, l = tid & 3;
    const int i = min(i0 + px, N - 1);
    const float inv = 1.0f / (float)(1 << l);
    cxy[tid * 2] = clampc(coords[((int64_t)b * 2) * N + i] * inv);
    cxy[tid * 2 + 1] = clampc(coords[((int64_t)b * 2 + 1) * N + i] * inv);
  }
  // per level: a 16-B aligned base at or below this workgroup's first plane; `dl` = cells
  // between that base and the first plane (0..EPP-1)
  __amdgpu_buffer_rsrc_t rs[4];
  int dl[4];
  uint32_t nbytes[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    const int ll = l < levels ? l : 0;
    const int64_t plane = (int64_t)pyr.h[ll] * pyr.w[ll];
    const int64_t first = ((int64_t)b * N + i0) * plane;  // cell index of the first plane
    const int64_t abase = first & ~(int64_t)(EPP - 1);
    dl[l] = (int)(first - abase);
    const char* base = reinterpret_cast<const char*>(pyr.lvl[ll]) + abase * ES;
    // rounded up to whole dwords: a dword read only partly inside num_records returns zero, so
    // an odd bf16 cell count would lose the last plane's last cell (the allocation is padded,
    // the extra bytes are masked cells)
    const uint32_t bytes = (uint32_t)(((dl[l] + (int64_t)npx * plane) * ES + 3) & ~(int64_t)3);
    nbytes[l] = bytes;
    rs[l] = __builtin_amdgcn_make_buffer_rsrc(const_cast<char*>(base), (short)0, (int)bytes, 0x00020000);
  }
  __syncthreads();
  // ---- phase 1: every window row's aligned 16-B pieces -> LDS (all loads before any store).
  // Items are level-major in 64-aligned per-level ranges, so every wave reads ONE level: the
  // buffer resource stays wave-uniform (a lane-varying descriptor costs a waterfall loop)
  constexpr int IPL = (TPVK * E + 63) / 64 * 64;  // items per level (padded)
  constexpr int ITEMS = 4 * IPL;
  constexpr int PER = (ITEMS + 255) / 256;
  uint4 v[PER][NPC];
  int slot[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    const int e = tid + k * 256;
    const int l = __builtin_amdgcn_readfirstlane(e / IPL), rem = e - l * IPL;
    const int px = rem / E, r = rem - px * E;
    slot[k] = rem < TPVK * E && l < 4 ? (px * 4 + l) * E + r : -1;
    uint32_t o[NPC];
#pragma unroll
    for (int u = 0; u < NPC; ++u) o[u] = OOB;
    const int lq = l < levels ? l : 0;
    if (rem < TPVK * E && px < npx && l < levels) {
      const int hl = pyr.h[l], wl = pyr.w[l];
      const float cx = cxy[(px * 4 + l) * 2], cy = cxy[(px * 4 + l) * 2 + 1];
      const int xs = (int)floorf(cx) - R, gy = (int)floorf(cy) - R + r;
      if ((unsigned)gy < (unsigned)hl) {
        const int er = dl[l] + px * hl * wl + gy * wl + xs;  // cell offset of the row start
        // floor division: er < 0 only before the first plane (those cells are masked)
        const int q0 = er >= 0 ? er / EPP : -((-er + EPP - 1) / EPP);
        const int lead = er - q0 * EPP;
#pragma unroll
        for (int u = 0; u < NPC; ++u)
          o[u] = (q0 + u >= 0 && (u < 2 || lead + E > u * EPP)) ? (uint32_t)(q0 + u) * 16u : OOB;
      }
    }
    const __amdgpu_buffer_rsrc_t r0 = lq == 0 ? rs[0] : (lq == 1 ? rs[1] : (lq == 2 ? rs[2] : rs[3]));
    const uint32_t lim = nbytes[lq];
#pragma unroll
    for (int u = 0; u < NPC; ++u) v[k][u] = piece16(r0, o[u], lim);
  }
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    if (slot[k] >= 0) {
#pragma unroll
      for (int u = 0; u < NPC; ++u) rows[slot[k] * NPC + u] = v[k][u];
    }
  }
  __syncthreads();
  // ---- phase 2: (pixel, level, window row iy) -> the 2r+1 taps of that row
  const int items2 = TPVK * levels * D;
  for (int it = tid; it < items2; it += 256) {
    const int px = it / (levels * D), rem = it - px * (levels * D), l = rem / D, iy = rem - l * D;
    const int hl = pyr.h[l], wl = pyr.w[l];
    const float cx = cxy[(px * 4 + l) * 2], cy = cxy[(px * 4 + l) * 2 + 1];
    const float fx = floorf(cx), fy = floorf(cy);
    const float ax = cx - fx, ay = cy - fy;
    const int xs = (int)fx - R, ys = (int)fy - R;
    float hr[2][D];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int r = iy + k, gy = ys + r;
      const bool rowok = (unsigned)gy < (unsigned)hl;
      const int er = dl[l] + px * hl * wl + gy * wl + xs;
      const int lead = ((er % EPP) + EPP) % EPP;
      const char* src = reinterpret_cast<const char*>(rows + ((px * 4 + l) * E + r) * NPC) + lead * ES;
      float c[E];
#pragma unroll
      for (int xx = 0; xx < E; ++xx) {
        const int gx = xs + xx;
        float cv;
        if constexpr (PF32) cv = reinterpret_cast<const float*>(src)[xx];
        else cv = raft_bf16_to_f32(reinterpret_cast<const uint16_t*>(src)[xx]);
        c[xx] = (rowok && (unsigned)gx < (unsigned)wl) ? cv : 0.f;
      }
#pragma unroll
      for (int ix = 0; ix < D; ++ix) hr[k][ix] = (1.f - ax) * c[ix] + ax * c[ix + 1];
    }
    uint16_t* T = tile + px * ROWT + l * D * D;
#pragma unroll
    for (int ix = 0; ix < D; ++ix) {
      const float tv = (1.f - ay) * hr[0][ix] + ay * hr[1][ix];
      const uint16_t h = raft_f2h<OT == 1>(tv);
      T[ix * D + iy] = h;
      if constexpr (OT == 2) T[TPVK * ROWT + ix * D + iy] = raft_f32_to_bf16(tv - raft_bf16_to_f32(h));
    }
  }
  __syncthreads();
  // ---- phase 3: whole 16-B pieces of the (B,H,W,NH cbuf) rows, zero padding included
  const int ctot = levels * D * D;
  const int chunks = cbuf / 8;
  for (int e = tid; e < NH * npx * chunks; e += 256) {
    const int hf = e / (npx * chunks), e2 = e - hf * (npx * chunks);
    const int px = e2 / chunks, ch = e2 - px * chunks;
    const uint16_t* tl = tile + hf * (TPVK * ROWT);
    uint4 o;
    if (ch * 8 + 8 <= ctot) {
      o = *reinterpret_cast<const uint4*>(tl + px * ROWT + ch * 8);
    } else {
      uint16_t q8[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int c = ch * 8 + q;
        q8[q] = c < ctot ? tl[px * ROWT + c] : (uint16_t)0;
      }
      o = make_uint4(q8[0] | ((uint32_t)q8[1] << 16), q8[2] | ((uint32_t)q8[3] << 16),
                     q8[4] | ((uint32_t)q8[5] << 16), q8[6] | ((uint32_t)q8[7] << 16));
    }
    *reinterpret_cast<uint4*>(out + ((int64_t)b * N + i0 + px) * (NH * cbuf) + hf * cbuf + ch * 8) = o;
  }
}

// dout: (B,H,W,cbuf) bf16 (channels [0, L*D*D) used); wg: (B, N, L, E, E) fp32
template <int R>
__global__ __launch_bounds__(256) void corr_window_grad_kernel(const float* __restrict__ coords,
                                                               const uint16_t* __restrict__ dout,
                                                               int cbuf, float* __restrict__ wg,
                                                               int B, int H, int W, int levels) {
  constexpr int D = 2 * R + 1, E = D + 1;
  constexpr int ROW = (4 * D * D + 7) / 8 * 8;
  __shared__ __attribute__((aligned(16))) uint16_t tile[TP * ROW];
  const int N = H * W;
  const int tiles = (N + TP - 1) / TP;
  const int b = blockIdx.x / tiles;
  const int i0 = (blockIdx.x % tiles) * TP;
  const int ctot = levels * D * D;
  // stage the 64 pixels' incoming tap gradients (coalesced rows)
  const int chunks = (ctot + 7) / 8;
  for (int e = threadIdx.x; e < TP * chunks; e += 256) {
    const int px = e / chunks, ch = e % chunks;
    const int i = i0 + px;
    if (i >= N) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(dout + ((int64_t)b * N + i) * cbuf + ch * 8);
    *reinterpret_cast<uint4*>(tile + px * ROW + ch * 8) = v;
  }
  __syncthreads();
  const int items = TP * levels * E;
  for (int it = threadIdx.x; it < items; it += 256) {
    const int yy = it % E;
    const int rest = it / E;
    const int l = rest % levels, px = rest / levels;
    const int i = i0 + px;
    if (i >= N) continue;
    const float inv = 1.0f / (float)(1 << l);
    const float cx = clampc(coords[((int64_t)b * 2) * N + i] * inv);
    const float cy = clampc(coords[((int64_t)b * 2 + 1) * N + i] * inv);
    const float ax = cx - floorf(cx), ay = cy - floorf(cy);
    const uint16_t* T = tile + px * ROW + l * D * D;
    float acc[E];
#pragma unroll
    for (int xx = 0; xx < E; ++xx) acc[xx] = 0.f;
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int iy = yy - k;
      if (iy < 0 || iy >= D) continue;
      const float wy = k == 0 ? (1.f - ay) : ay;
      float d[D];
#pragma unroll
      for (int ix = 0; ix < D; ++ix) d[ix] = raft_bf16_to_f32(T[ix * D + iy]);
#pragma unroll
      for (int xx = 0; xx < E; ++xx) {
        float s = 0.f;
        if (xx < D) s += (1.f - ax) * d[xx];
        if (xx > 0) s += ax * d[xx - 1];
        acc[xx] += wy * s;
      }
    }
    float* dst = wg + ((((int64_t)b * N + i) * levels + l) * E + yy) * E;
#pragma unroll
    for (int xx = 0; xx < E; ++xx) dst[xx] = acc[xx];
  }
}

template <int R>
__global__ __launch_bounds__(256) void corr_window_reduce_kernel(WinList wl_, int levels, int B, int H,
                                                                 int W, float inv_sqrt_c,
                                                                 void* __restrict__ out, int out_bf16) {
  constexpr int D = 2 * R + 1, E = D + 1;
  extern __shared__ float planes[];
  const int N = H * W;
  const int b = blockIdx.x / N, i = blockIdx.x % N;
  int hs[4], ws[4], off[4];
  int tot = 0;
  {
    int h = H, w = W;
    for (int l = 0; l < 4; ++l) {
      hs[l] = h; ws[l] = w; off[l] = tot;
      if (l < levels) tot += h * w;
      h >>= 1; w >>= 1;
    }
  }
  for (int e = threadIdx.x; e < tot; e += 256) planes[e] = 0.f;
  // iterations are folded in a fixed order (deterministic), KC at a time: all of a chunk's
  // coordinate and patch loads are issued before its first LDS add, so a workgroup waits for
  // one memory round trip per chunk instead of one per iteration
  constexpr int KC = 6;
  constexpr int CPT = (4 * E * E + 255) / 256;  // window cells per thread (all levels)
  const int cells = levels * E * E;
  for (int k0 = 0; k0 < wl_.n; k0 += KC) {
    float gv[KC][CPT];
    int pos[KC][CPT];
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const int k = k0 + kk;
      const bool kok = k < wl_.n;
      const float* C = wl_.coords[kok ? k : 0];
      const float* G = wl_.wg[kok ? k : 0] + ((int64_t)b * N + i) * levels * E * E;
      const float x = C[((int64_t)b * 2) * N + i], y = C[((int64_t)b * 2 + 1) * N + i];
#pragma unroll
      for (int q = 0; q < CPT; ++q) {
        const int e = threadIdx.x + q * 256;
        pos[kk][q] = -1;
        gv[kk][q] = 0.f;
        if (kok && e < cells) {
          const int l = e / (E * E), yy = (e / E) % E, xx = e % E;
          const float inv = 1.0f / (float)(1 << l);
          const int xs = (int)floorf(clampc(x * inv)) - R, ys = (int)floorf(clampc(y * inv)) - R;
          const int gy = ys + yy, gx = xs + xx;
          if (gy >= 0 && gy < hs[l] && gx >= 0 && gx < ws[l]) {
            pos[kk][q] = off[l] + gy * ws[l] + gx;
            gv[kk][q] = G[e];
          }
        }
      }
    }
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      __syncthreads();  // previous adds (and the zero fill) visible; one writer per cell per round
#pragma unroll
      for (int q = 0; q < CPT; ++q)
        if (pos[kk][q] >= 0) planes[pos[kk][q]] += gv[kk][q];
    }
  }
  __syncthreads();
  float* O = (float*)out + ((int64_t)b * N + i) * N;
  uint16_t* Ob = (uint16_t*)out + ((int64_t)b * N + i) * N;
  for (int e = threadIdx.x; e < N; e += 256) {
    const int y = e / W, x = e % W;
    float v = planes[e];
    float s = 0.25f;
    for (int l = 1; l < levels; ++l) {
      const int yl = y >> l, xl = x >> l;
      if (yl < hs[l] && xl < ws[l]) v += s * planes[off[l] + yl * ws[l] + xl];
      s *= 0.25f;
    }
    if (out_bf16) Ob[e] = raft_f32_to_bf16(v * inv_sqrt_c);
    else O[e] = v * inv_sqrt_c;
  }
}

// Fold straight from the lookup's tap gradients (no per-iteration compact window pass): the
// workgroup of query pixel (b, i) stages, KC iterations at a time, the pixel's bf16 tap-gradient
// rows (levels*(2r+1)^2 taps of the (B,H,W,cbuf) lookup-output gradient; 16-B loads, all issued
// before use) in LDS, then every thread forms its window cells' bilinear adjoint (the same
// arithmetic as corr_window_grad_kernel) and adds it into the level planes -- iterations in a
// fixed order, one writer per cell per round (deterministic; bitwise the two-pass result).  Reads
// ~0.77 KB per pixel-iteration instead of writing and re-reading a 1.6 KB fp32 window.
template <int R, bool TF16 = false>
__global__ __launch_bounds__(256) void corr_tap_reduce_kernel(TapList tl, int levels, int B, int H,
                                                              int W, float inv_sqrt_c,
                                                              void* __restrict__ out, int out_bf16,
                                                              const int* __restrict__ list) {
  constexpr int D = 2 * R + 1, E = D + 1;
  constexpr int KC = 6;
  constexpr int CPT = (4 * E * E + 255) / 256;
  extern __shared__ float planes[];
  const int N = H * W;
  // list != nullptr: the pixels the box kernel could not take (list[0] = count, then the pixel
  // indices), grid-strided; otherwise one pixel per workgroup
  const int nitems = list != nullptr ? list[0] : B * N;
  for (int w = blockIdx.x; w < nitems; w += (list != nullptr ? gridDim.x : nitems)) {
  const int q = list != nullptr ? list[1 + w] : w;
  const int b = q / N, i = q % N;
  int hs[4], ws[4], off[4];
  int tot = 0;
  {
    int h = H, w = W;
    for (int l = 0; l < 4; ++l) {
      hs[l] = h; ws[l] = w; off[l] = tot;
      if (l < levels) tot += h * w;
      h >>= 1; w >>= 1;
    }
  }
  const int ctot = levels * D * D;
  const int chunks = (ctot + 7) / 8;                    // 16-B pieces of one tap row
  const int trow = chunks * 8;                          // bf16 per staged row
  uint16_t* taps = reinterpret_cast<uint16_t*>(planes + ((tot + 3) & ~3));
  for (int e = threadIdx.x; e < tot; e += 256) planes[e] = 0.f;
  const int cells = levels * E * E;
  // this thread's window cells: (level, row, column) decoded once, not per iteration
  int cl[CPT], cyy[CPT], cxx[CPT];
  float cinv[CPT];
#pragma unroll
  for (int q = 0; q < CPT; ++q) {
    const int e = threadIdx.x + q * 256;
    cl[q] = e < cells ? e / (E * E) : -1;
    cyy[q] = (e / E) % E;
    cxx[q] = e % E;
    cinv[q] = cl[q] >= 0 ? 1.0f / (float)(1 << cl[q]) : 0.f;
  }
  for (int k0 = 0; k0 < tl.n; k0 += KC) {
    const int kn = min(KC, tl.n - k0);
    // one 16-B piece per thread: (kk, ch)
    uint4 piece = make_uint4(0, 0, 0, 0);
    const int kk_ld = threadIdx.x / chunks, ch = threadIdx.x % chunks;
    const bool ld = kk_ld < kn;
    if (ld)
      piece = *reinterpret_cast<const uint4*>(tl.dout[k0 + kk_ld] + ((int64_t)b * N + i) * tl.cbuf + ch * 8);
    float cx[KC], cy[KC];
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      const float* C = tl.coords[k0 + (kk < kn ? kk : 0)];
      cx[kk] = C[((int64_t)b * 2) * N + i];
      cy[kk] = C[((int64_t)b * 2 + 1) * N + i];
    }
    __syncthreads();  // previous chunk's tap reads and plane adds done
    if (ld) *reinterpret_cast<uint4*>(taps + kk_ld * trow + ch * 8) = piece;
#pragma unroll
    for (int kk = 0; kk < KC; ++kk) {
      __syncthreads();  // staged taps + previous round's adds visible
      if (kk >= kn) continue;
      const uint16_t* T0 = taps + kk * trow;
#pragma unroll
      for (int q = 0; q < CPT; ++q) {
        const int l = cl[q];
        if (l < 0) continue;
        const int yy = cyy[q], xx = cxx[q];
        const float fxc = clampc(cx[kk] * cinv[q]), fyc = clampc(cy[kk] * cinv[q]);
        const float flx = floorf(fxc), fly = floorf(fyc);
        const int gy = (int)fly - R + yy, gx = (int)flx - R + xx;
        if (gy < 0 || gy >= hs[l] || gx < 0 || gx >= ws[l]) continue;
        const float ax = fxc - flx, ay = fyc - fly;
        const uint16_t* T = T0 + l * D * D;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < 2; ++k) {
          const int iy = yy - k;
          if (iy < 0 || iy >= D) continue;
          const float wy = k == 0 ? (1.f - ay) : ay;
          float sx = 0.f;
          if (xx < D) sx += (1.f - ax) * raft_h2f<TF16>(T[xx * D + iy]);
          if (xx > 0) sx += ax * raft_h2f<TF16>(T[(xx - 1) * D + iy]);
          acc += wy * sx;
        }
        planes[off[l] + gy * ws[l] + gx] += acc;
      }
    }
  }
  __syncthreads();
  // level-0 gradient row with the avg-pool adjoint of the coarser levels; two columns per thread
  // (4-B stores of bf16 pairs when the row is 4-B aligned, i.e. N even)
  const int ldo = tl.ldo;
  const int64_t row = ((int64_t)b * N + i) * ldo;
  const float inv_w = 1.0f / (float)W;
  auto cell = [&](int e) {
    const int y = (int)(((float)e + 0.5f) * inv_w), x = e - y * W;  // exact for e < 2^22
    float v = planes[e];
    float sc = 0.25f;
    for (int l = 1; l < levels; ++l) {
      const int yl = y >> l, xl = x >> l;
      if (yl < hs[l] && xl < ws[l]) v += sc * planes[off[l] + yl * ws[l] + xl];
      sc *= 0.25f;
    }
    return v * inv_sqrt_c;
  };
  if (out_bf16 == 2) {
    // split fp32: bf16 hi plane at out, lo plane at out + B N ldo
    uint16_t* Oh = (uint16_t*)out + row;
    uint16_t* Ol = (uint16_t*)out + (int64_t)B * N * ldo + row;
    for (int e = threadIdx.x; e < ldo; e += 256) {
      const float v = e < N ? cell(e) : 0.f;
      const uint16_t h = raft_f32_to_bf16(v);
      Oh[e] = h;
      Ol[e] = raft_f32_to_bf16(v - raft_bf16_to_f32(h));
    }
  } else if (out_bf16 && (N & 1) == 0) {
    uint32_t* Ob = reinterpret_cast<uint32_t*>((uint16_t*)out + row);
    for (int e2 = threadIdx.x; e2 < ldo / 2; e2 += 256)
      Ob[e2] = 2 * e2 < N ? (uint32_t)raft_f32_to_bf16(cell(2 * e2)) |
                                ((uint32_t)raft_f32_to_bf16(cell(2 * e2 + 1)) << 16)
                          : 0u;
  } else if (out_bf16) {
    uint16_t* Ob = (uint16_t*)out + row;
    for (int e = threadIdx.x; e < ldo; e += 256) Ob[e] = e < N ? raft_f32_to_bf16(cell(e)) : (uint16_t)0;
  } else {
    float* O = (float*)out + row;
    for (int e = threadIdx.x; e < ldo; e += 256) O[e] = e < N ? cell(e) : 0.f;
  }
  __syncthreads();  // the next listed pixel reuses the planes
  }
}

// Union-box fold (the launcher's default, W even): one WAVE per query pixel whose level planes
// are held only over the union box of its windows across the step's iterations (<= 24 x 24 cells
// per level: 5.4 KB per wave at chairs instead of the full 15 KB planes, ~5 waves per SIMD), so
// the zero fill and the LDS footprint shrink and the write-out reads the boxes.
//  * fold: lane = (level, window column rx) in 16-lane rows; a lane takes its tap column from the
//    staged tap row (5 dword reads), the column to its left from lane - 1 (DPP row shift), and
//    adds its 2r+2 window cells (x- then y-interpolated, the same bilinear adjoint as the other
//    folds) down the column: ~2.5 LDS operations per cell instead of 6.
//  * iterations in order, one writer per cell and iteration, waves never share planes: no
//    barrier, deterministic.
//  * a pixel whose windows spread past a 24 x 24 box at some level is appended to `list` and
//    folded afterwards by corr_tap_reduce_kernel (list mode).
constexpr int BOXC = 24;   // box side cap (cells)
struct BoxGeo {
  int cap[4];    // floats reserved per level box
  int off[4];
  int wave_floats;
};

BoxGeo box_geo(int H, int W, int levels, int radius) {
  BoxGeo g{};
  int h = H, w = W, tot = 0;
  for (int l = 0; l < 4; ++l) {
    const int c = l < levels ? (std::min(BOXC * BOXC, h * w) + 3) & ~3 : 0;
    g.cap[l] = c;
    g.off[l] = tot;
    tot += c;
    h >>= 1;
    w >>= 1;
  }
  const int D = 2 * radius + 1;
  const int trow = (levels * D * D + 7) / 8 * 8;
  g.wave_floats = tot + 2 * trow / 2;
  return g;
}

// OM: dC output 0 bf16, 1 fp32, 2 split bf16 planes (hi at out, lo at out + B N ldo)
template <int R, bool TF16 = false, int OM = 0>
__global__ __launch_bounds__(256) void corr_tap_fold_box_kernel(TapList tl, BoxGeo bg, int levels, int B,
                                                                int H, int W, float inv_sqrt_c,
                                                                void* __restrict__ out, int* __restrict__ list) {
  constexpr int D = 2 * R + 1, E = D + 1;
  extern __shared__ float lds_all[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int N = H * W;
  const int q = blockIdx.x * (blockDim.x >> 6) + wv;
  if (q >= B * N) return;  // no workgroup barrier below
  const int b = q / N, i = q - b * N;
  float* box = lds_all + wv * bg.wave_floats;
  const int ctot = levels * D * D;
  const int chunks = (ctot + 7) / 8;
  const int trow = chunks * 8;
  uint16_t* taps = reinterpret_cast<uint16_t*>(box + (bg.wave_floats - trow));  // [2][trow]
  const int n = tl.n;
  const int64_t prow = ((int64_t)b * N + i) * tl.cbuf;
  // iteration k's coordinates in lane k (k < n <= 32)
  float cxv = 0.f, cyv = 0.f;
  if (lane < n) {
    const float* C = tl.coords[lane];
    cxv = C[(int64_t)b * 2 * N + i];
    cyv = C[(int64_t)b * 2 * N + N + i];
  }
  // tap rows of the next BPF iterations in flight (registers) while one is folded
  constexpr int BPF = 4;
  uint4 piece[BPF];
#pragma unroll
  for (int j = 0; j < BPF; ++j)
    piece[j] = (lane < chunks && j < n) ? *reinterpret_cast<const uint4*>(tl.dout[j] + prow + lane * 8)
                                        : make_uint4(0, 0, 0, 0);
  // this lane's level / column and its level's plane
  const int ll = lane >> 4, rx = lane & 15;
  const bool lact = ll < levels;
  const int hl = H >> ll, wl = W >> ll;
  const float inv = 1.0f / (float)(1 << ll);
  // union box of the level's windows (every lane of the level computes the same box)
  int mnx = 0x7fffffff, mxx = -0x7fffffff, mny = 0x7fffffff, mxy = -0x7fffffff;
  for (int k = 0; k < n; ++k) {
    const float cx = clampc(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cxv), k)) * inv);
    const float cy = clampc(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cyv), k)) * inv);
    const int x0 = (int)floorf(cx) - R, y0 = (int)floorf(cy) - R;
    if (x0 <= wl - 1 && x0 + E - 1 >= 0 && y0 <= hl - 1 && y0 + E - 1 >= 0) {
      mnx = min(mnx, x0);
      mxx = max(mxx, x0 + E - 1);
      mny = min(mny, y0);
      mxy = max(mxy, y0 + E - 1);
    }
  }
  int bx0 = max(mnx, 0), by0 = max(mny, 0);
  const int bx1 = min(mxx, wl - 1), by1 = min(mxy, hl - 1);
  if (ll == 0) bx0 &= ~1;  // level 0: even origin and width -> 8-B pair reads in the write-out
  int bw = bx1 >= bx0 ? bx1 - bx0 + 1 : 0, bh = by1 >= by0 ? by1 - by0 + 1 : 0;
  if (ll == 0) bw = (bw + 1) & ~1;
  if (bw == 0 || bh == 0) bw = bh = 0;
  const bool over = lact && (bw > BOXC || bh > BOXC);
  if (__builtin_amdgcn_read_exec() & __ballot(over)) {
    if (lane == 0) {
      const int slot = atomicAdd(list, 1);
      list[1 + slot] = q;
    }
    return;
  }
  // level boxes' geometry from their lanes (uniform); zero only the boxes' cells
  int gbx[4], gby[4], gbw[4], gbh[4];
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    gbx[l] = __builtin_amdgcn_readlane(bx0, l * 16);
    gby[l] = __builtin_amdgcn_readlane(by0, l * 16);
    gbw[l] = __builtin_amdgcn_readlane(bw, l * 16);
    gbh[l] = __builtin_amdgcn_readlane(bh, l * 16);
  }
#pragma unroll
  for (int l = 0; l < 4; ++l) {
    if (l >= levels) break;
    const int n4 = (gbw[l] * gbh[l] + 3) >> 2;  // <= cap / 4 (caps are multiples of 4)
    uint4* z = reinterpret_cast<uint4*>(box + bg.off[l]);
    for (int e = lane; e < n4; e += 64) z[e] = make_uint4(0, 0, 0, 0);
  }
  float* mybox = box + (ll == 0 ? bg.off[0] : ll == 1 ? bg.off[1] : ll == 2 ? bg.off[2] : bg.off[3]);
  const bool colact = lact && rx < E;
  for (int k0 = 0; k0 < n; k0 += BPF) {
#pragma unroll
  for (int j = 0; j < BPF; ++j) {
    const int k = k0 + j;
    if (k >= n) break;
    uint16_t* T0 = taps + (k & 1) * trow;
    if (lane < chunks) reinterpret_cast<uint4*>(T0)[lane] = piece[j];
    if (k + BPF < n && lane < chunks)
      piece[j] = *reinterpret_cast<const uint4*>(tl.dout[k + BPF] + prow + lane * 8);
    __builtin_amdgcn_wave_barrier();
    const float cx = clampc(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cxv), k)) * inv);
    const float cy = clampc(__builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, cyv), k)) * inv);
    const float flx = floorf(cx), fly = floorf(cy);
    const float ax = cx - flx, ay = cy - fly;
    const int gx = (int)flx - R + rx, gy0 = (int)fly - R;
    // tap column rx (zero past the last tap column) -> fp32, 9 values
    float tc[D];
    {
      const int start = (lact ? ll : 0) * D * D + min(rx, D - 1) * D;
      const uint32_t* Tw = reinterpret_cast<const uint32_t*>(T0) + (start >> 1);
      uint32_t wd[(D + 2) / 2];
#pragma unroll
      for (int u = 0; u < (D + 2) / 2; ++u) wd[u] = Tw[u];
      const int sh = start & 1;
#pragma unroll
      for (int t = 0; t < D; ++t) {
        const int idx = t + sh;
        const uint32_t h16 = (wd[idx >> 1] >> ((idx & 1) * 16)) & 0xffffu;
        tc[t] = (rx < D) ? raft_h2f<TF16>((uint16_t)h16) : 0.f;
      }
    }
    // the column to the left (lane - 1 of the same 16-lane row; zero for rx = 0)
    float tl_[D];
#pragma unroll
    for (int t = 0; t < D; ++t)
      tl_[t] = __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, tc[t]),
                                                                      0x111, 0xf, 0xf, false));
    if (colact && gx >= bx0 && gx < bx0 + bw) {
      float hx[D];
#pragma unroll
      for (int t = 0; t < D; ++t) {
        float sx = 0.f;
        if (rx < D) sx += (1.f - ax) * tc[t];
        if (rx > 0) sx += ax * tl_[t];
        hx[t] = sx;
      }
      float* colp = mybox + (gx - bx0);
#pragma unroll
      for (int ry = 0; ry < E; ++ry) {
        const int gy = gy0 + ry;
        if (gy < by0 || gy >= by0 + bh) continue;
        float acc = 0.f;
        if (ry < D) acc += (1.f - ay) * hx[ry];
        if (ry > 0) acc += ay * hx[ry - 1];
        colp[(gy - by0) * bw] += acc;
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  }
  // dC row: bf16 pairs (mixed precision: the bf16 GEMMs' operand) or fp32 pairs (fp16 / fp32
  // schedules: the reference's fp32 correlation gradient)
  const int64_t row = ((int64_t)b * N + i) * tl.ldo;
  uint32_t* Ob = reinterpret_cast<uint32_t*>(static_cast<uint16_t*>(out) + row);
  uint32_t* Ol = reinterpret_cast<uint32_t*>(static_cast<uint16_t*>(out) + (int64_t)B * N * tl.ldo + row);
  float2* Of = reinterpret_cast<float2*>(static_cast<float*>(out) + row);
  const float inv_w = 1.0f / (float)W;
  for (int e2 = N / 2 + lane; e2 < tl.ldo / 2; e2 += 64) {
    if constexpr (OM == 1) Of[e2] = make_float2(0.f, 0.f);
    else Ob[e2] = 0u;
    if constexpr (OM == 2) Ol[e2] = 0u;
  }
  for (int e2 = lane; e2 < N / 2; e2 += 64) {
    const int e = 2 * e2;
    const int y = (int)(((float)e + 0.5f) * inv_w), x = e - y * W;
    float v0 = 0.f, v1 = 0.f;
    {
      const int yy = y - gby[0], xx = x - gbx[0];
      if ((unsigned)yy < (unsigned)gbh[0] && (unsigned)xx < (unsigned)gbw[0]) {
        const float2 p = *reinterpret_cast<const float2*>(box + bg.off[0] + yy * gbw[0] + xx);
        v0 = p.x;
        v1 = p.y;
      }
    }
    float sc = 0.25f;
#pragma unroll
    for (int l = 1; l < 4; ++l) {
      if (l < levels) {
        const int yy = (y >> l) - gby[l], xx = (x >> l) - gbx[l];
        if ((unsigned)yy < (unsigned)gbh[l] && (unsigned)xx < (unsigned)gbw[l]) {
          const float c = sc * box[bg.off[l] + yy * gbw[l] + xx];
          v0 += c;
          v1 += c;
        }
      }
      sc *= 0.25f;
    }
    if constexpr (OM == 1) {
      Of[e2] = make_float2(v0 * inv_sqrt_c, v1 * inv_sqrt_c);
    } else {
      const float s0 = v0 * inv_sqrt_c, s1 = v1 * inv_sqrt_c;
      const uint16_t h0 = raft_f32_to_bf16(s0), h1 = raft_f32_to_bf16(s1);
      Ob[e2] = (uint32_t)h0 | ((uint32_t)h1 << 16);
      if constexpr (OM == 2)
        Ol[e2] = (uint32_t)raft_f32_to_bf16(s0 - raft_bf16_to_f32(h0)) |
                 ((uint32_t)raft_f32_to_bf16(s1 - raft_bf16_to_f32(h1)) << 16);
    }
  }
}

}  // namespace

bool launch_corr_lookup_tile(const void* const* lvl, const int* hs, const int* ws, int levels,
                             const float* coords, uint16_t* out, int cbuf, int B, int H, int W,
                             int radius, bool pyr_bf16, int out_f16, hipStream_t stream) {
  PyrC4 p;
  for (int l = 0; l < 4; ++l) {
    p.lvl[l] = l < levels ? static_cast<const float*>(lvl[l]) : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
  }
  if (radius != 4 && radius != 3) return false;
  if (pyr_bf16 && out_f16 != 0) return false;  // a bf16 pyramid feeds bf16 taps only
  const int N = H * W;
  if (pyr_bf16) {
    // pixels per workgroup (RAFT_LOOKUP_TPV): 4 (default, 10.5 KB LDS) -- 27.7 / 28.8 / 34.7 us
    // per call for 4 / 8 / 16 at chairs (profiles/r4/lookup_tpv.txt): more workgroups in flight
    // per CU keep more window-row loads outstanding
    static const int tpv = [] {
      const char* e = getenv("RAFT_LOOKUP_TPV");
      const int v = e ? atoi(e) : 4;
      return v == 8 || v == 16 ? v : 4;
    }();
    dim3 grid((unsigned)(B * ((N + tpv - 1) / tpv)));
#define RAFT_ROWS(RR, TT) \
  hipLaunchKernelGGL((corr_lookup_rows_kernel<RR, TT>), grid, dim3(256), 0, stream, p, coords, out, cbuf, B, H, W, levels)
    if (tpv == 4) { if (radius == 4) RAFT_ROWS(4, 4); else RAFT_ROWS(3, 4); }
    else if (tpv == 8) { if (radius == 4) RAFT_ROWS(4, 8); else RAFT_ROWS(3, 8); }
    else { if (radius == 4) RAFT_ROWS(4, 16); else RAFT_ROWS(3, 16); }
#undef RAFT_ROWS
    return true;
  }
  // fp32 pyramid (the reference's fp32 correlation: fp16 autocast and the fp32 schedule): bf16,
  // fp16 (out_f16 = 1) or split-fp32 (out_f16 = 2) taps, 4 pixels per workgroup
  dim3 grid((unsigned)(B * ((N + 3) / 4)));
#define RAFT_ROWS32(RR, OT) \
  hipLaunchKernelGGL((corr_lookup_rows_kernel<RR, 4, true, OT>), grid, dim3(256), 0, stream, p, coords, out, cbuf, B, H, W, levels)
  if (radius == 4) {
    if (out_f16 == 1) RAFT_ROWS32(4, 1); else if (out_f16 == 2) RAFT_ROWS32(4, 2); else RAFT_ROWS32(4, 0);
  } else {
    if (out_f16 == 1) RAFT_ROWS32(3, 1); else if (out_f16 == 2) RAFT_ROWS32(3, 2); else RAFT_ROWS32(3, 0);
  }
#undef RAFT_ROWS32
  return true;
}

bool launch_corr_window_grad(const float* coords, const uint16_t* dout, int cbuf, float* wg, int B,
                             int H, int W, int levels, int radius, hipStream_t stream) {
  const int N = H * W;
  dim3 grid((unsigned)(B * ((N + TP - 1) / TP)));
  if (radius == 4) hipLaunchKernelGGL(corr_window_grad_kernel<4>, grid, dim3(256), 0, stream, coords, dout, cbuf, wg, B, H, W, levels);
  else if (radius == 3) hipLaunchKernelGGL(corr_window_grad_kernel<3>, grid, dim3(256), 0, stream, coords, dout, cbuf, wg, B, H, W, levels);
  else return false;
  return true;
}

int corr_window_reduce_lds_bytes(int H, int W, int levels) {
  int tot = 0, h = H, w = W;
  for (int l = 0; l < levels; ++l) { tot += h * w; h >>= 1; w >>= 1; }
  return tot * 4;
}

bool launch_corr_window_reduce(const WinList& wl, int levels, int B, int H, int W, int radius,
                               float inv_sqrt_c, void* out, int out_bf16, hipStream_t stream) {
  const int lds = corr_window_reduce_lds_bytes(H, W, levels);
  dim3 grid((unsigned)(B * H * W));
  if (radius == 4) hipLaunchKernelGGL(corr_window_reduce_kernel<4>, grid, dim3(256), lds, stream, wl, levels, B, H, W, inv_sqrt_c, out, out_bf16);
  else if (radius == 3) hipLaunchKernelGGL(corr_window_reduce_kernel<3>, grid, dim3(256), lds, stream, wl, levels, B, H, W, inv_sqrt_c, out, out_bf16);
  else return false;
  return true;
}

int corr_tap_reduce_lds_bytes(int H, int W, int levels, int radius) {
  int tot = 0, h = H, w = W;
  for (int l = 0; l < levels; ++l) { tot += h * w; h >>= 1; w >>= 1; }
  const int D = 2 * radius + 1;
  const int trow = (levels * D * D + 7) / 8 * 8;
  return ((tot + 3) & ~3) * 4 + 6 * trow * 2;
}

bool launch_corr_tap_reduce(const TapList& tl, int levels, int B, int H, int W, int radius,
                            float inv_sqrt_c, void* out, int out_bf16, int* list, hipStream_t stream) {
  const int D = 2 * radius + 1;
  if ((levels * D * D + 7) / 8 * 6 > 256) return false;  // one 16-B piece per thread per chunk
  if (radius != 3 && radius != 4) return false;
  const int64_t P = (int64_t)B * H * W;
  const int lds = corr_tap_reduce_lds_bytes(H, W, levels, radius);
  if ((W & 1) == 0 && list != nullptr && tl.n <= 32 && (levels * D * D + 7) / 8 <= 64) {
    // union-box fold for every tap type (bf16, fp16, split-fp32 rows) and dC type (bf16 pairs
    // for the mixed-precision GEMMs, fp32 for the fp16 / fp32 schedules' fp32 correlation)
    const BoxGeo bg = box_geo(H, W, levels, radius);
    const int wpb = 4;
    (void)hipMemsetAsync(list, 0, sizeof(int), stream);
    dim3 grid((unsigned)((P + wpb - 1) / wpb));
    const size_t sh = (size_t)wpb * bg.wave_floats * 4;
#define RAFT_BOX(RR, TF, OM)                                                                         \
  hipLaunchKernelGGL((corr_tap_fold_box_kernel<RR, TF, OM>), grid, dim3(64 * wpb), sh, stream, tl, bg, \
                     levels, B, H, W, inv_sqrt_c, out, list)
#define RAFT_BOX_OM(RR, TF) \
  do { if (out_bf16 == 2) RAFT_BOX(RR, TF, 2); else if (out_bf16) RAFT_BOX(RR, TF, 0); else RAFT_BOX(RR, TF, 1); } while (0)
    if (radius == 4) {
      if (tl.tf16) RAFT_BOX_OM(4, true); else RAFT_BOX_OM(4, false);
    } else {
      if (tl.tf16) RAFT_BOX_OM(3, true); else RAFT_BOX_OM(3, false);
    }
#undef RAFT_BOX_OM
#undef RAFT_BOX
    // the pixels whose windows spread past the box cap (usually none): grid-strided over the list
    dim3 g2((unsigned)std::min<int64_t>(P, 1024));
    if (tl.tf16) {
      if (radius == 4) hipLaunchKernelGGL((corr_tap_reduce_kernel<4, true>), g2, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)list);
      else hipLaunchKernelGGL((corr_tap_reduce_kernel<3, true>), g2, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)list);
    } else {
      if (radius == 4) hipLaunchKernelGGL(corr_tap_reduce_kernel<4>, g2, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)list);
      else hipLaunchKernelGGL(corr_tap_reduce_kernel<3>, g2, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)list);
    }
    return true;
  }
  if (tl.tf16) {
    // fp16 tap gradients, other fold modes: the workgroup-per-pixel fold
    dim3 grid((unsigned)P);
    if (radius == 4) hipLaunchKernelGGL((corr_tap_reduce_kernel<4, true>), grid, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)nullptr);
    else hipLaunchKernelGGL((corr_tap_reduce_kernel<3, true>), grid, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)nullptr);
    return true;
  }
  dim3 grid((unsigned)P);
  if (radius == 4) hipLaunchKernelGGL(corr_tap_reduce_kernel<4>, grid, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)nullptr);
  else hipLaunchKernelGGL(corr_tap_reduce_kernel<3>, grid, dim3(256), lds, stream, tl, levels, B, H, W, inv_sqrt_c, out, out_bf16, (const int*)nullptr);
  return true;
}
