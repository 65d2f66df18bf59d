// Stride-1 3x3 conv for the encoders' 64 -> 64-channel layers (`core/extractor.py:22-23`, layer1 of
// both encoders at 1/2 resolution: 184 x 248 for chairs, 12-24 images) -- forward and input
// gradient (the same conv on the flipped / transposed weight), NHWC bf16, fp32 accumulation.
//
// Why a kernel of its own: at Cin = 64 the implicit GEMM has K = 9 x 64 = 576, i.e. 9 K steps, and
// the general kernels (conv_glds.hip) re-fetch their A tile for every tap through LDS-DMA: 6 DMA
// pieces per thread per 8 MFMAs per wave, ~110 us per call at ~20 % MFMA use (profiles/r3).
// Here a workgroup is persistent and
//   * keeps the whole weight matrix in LDS (64 x 576 bf16, rows padded to 1168 B: conflict-free
//     fragment reads), loaded once;
//   * works on 2-D tiles of 8 x 16 output pixels: the tile's 10 x 18 input halo (all 64 channels,
//     144-B padded pixels, 2816-B padded rows: bank-conflict-free fragment reads) is loaded ONCE
//     and every tap reads its shifted rows from it -- 1.4x the tile's bytes instead of 9x;
//   * stages the halo through registers three tiles ahead (buffer loads, zeros outside the image,
//     no branches) while a tile's 72 MFMAs per wave run, the K loop reading the next tap's
//     fragments ahead of the current tap's MFMAs;
//   * writes the output tile through LDS as 16-B rows (per-lane 2-B stores of the MFMA layout
//     were store-issue bound: ~115 us per call either way, profiles/r3/c2_kernel_summary.txt);
//   * optionally (part != null: the output feeds a training-statistics norm) reduces the tile's
//     rounded outputs into per-channel statistics of the norm that follows -- count, mean and
//     sum of squared deviations, one [4][64] row per tile (encoder_norm.hip's tiled finalize) --
//     so the norm skips its statistics pass over the output.
// 4 waves as 2 (pixels) x 2 (channels): a wave owns 64 pixels (4 tile rows) x 32 channels.
#include "common.h"
#include "launchers.h"

#include <cstdlib>
#include <cstring>

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t mk_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

constexpr int TH = 8, TW = 16;                 // output tile
constexpr int HH = TH + 2, HWD = TW + 2;       // halo tile
constexpr int HROWS = HH * HWD;                // 180 halo pixels
constexpr int AROW = 144;                      // LDS bytes per halo pixel (128 + 16 pad)
constexpr int BROW = 1168;                     // LDS bytes per weight row (1152 + 16 pad)
constexpr int KTOT = 9 * 64;
constexpr int NTH = 256;
constexpr uint32_t OOB = 0x80000000u;          // buffer offset past any descriptor's range
constexpr int APIECES = HROWS * 8;             // 16-B pieces of a halo tile
constexpr int APER = (APIECES + NTH - 1) / NTH;  // 6 per thread
// halo rows of 18 pixels padded to 2816 B = 704 dwords, a multiple of the 64 banks: a fragment
// read (ds_read_b128, 16-lane groups spanning two tile rows) then covers all 64 banks once.  With
// unpadded 2592-B rows (648 dwords = 8 mod 64) every A-fragment read was 2-way conflicted and the
// LDS array, at 4 waves x (8 A x 8 + 4 B x 4) cycles per tap, outran the tap's 8 MFMAs (256).
constexpr int AROWB = 2816;
constexpr int ABUF = 11 * AROWB;               // 10 halo rows + the spare pieces, 30,976 B
constexpr int BBUF = 64 * BROW;                // 74,752 B
constexpr int OROW = 144;                      // LDS bytes per staged output pixel (128 + 16 pad)
constexpr int OBUF = TH * TW * OROW;           // 18,432 B
constexpr int SBUF = 3 * 2 * 64 * 4;           // tile-statistics halves (count, mean, M2), 1,536 B

// LDS offset of halo pixel hp (row-major over the 10 x 18 halo; hp >= 180: spare row 10)
__device__ __forceinline__ int hoff(int hp) { return (hp / HWD) * AROWB + (hp % HWD) * AROW; }

// The K loop reads the next tap's 12 fragments (4 weight + 8 halo, ds_read_b128) before the
// current tap's 8 MFMAs, fenced by scheduling barriers.  Left to itself the compiler issued each
// MFMA pair's reads just before it and waited on them (lgkmcnt(0..2) ahead of every second MFMA),
// exposing the LDS latency at one wave per SIMD.
// NSET = 3 register sets of halo loads in flight (tiles ahead).  One workgroup per CU moves a
// tile's 24.6 KB halo per ~3.7 us, so at HBM latency under load the loads in flight, not the
// MFMAs, set the pace: 3 sets keep ~74 KB per CU outstanding instead of ~49 KB with 2.
constexpr int NSET = 3;
template <bool F16 = false>
__global__ __launch_bounds__(NTH, 1) void conv_enc64_kernel(const uint16_t* __restrict__ x,
                                                            const uint16_t* __restrict__ wpk,
                                                            uint16_t* __restrict__ out, int B,
                                                            int H, int W, int tiles_y,
                                                            int tiles_x, float* __restrict__ part) {
  __shared__ __attribute__((aligned(16))) char smem[2 * ABUF + BBUF + OBUF + SBUF];
  char* As = smem;                 // 2 halo buffers
  char* Bs = smem + 2 * ABUF;      // weights
  char* Os = Bs + BBUF;            // output tile staging (bf16 [pixel][channel])
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave >> 1, wn = wave & 1;
  const int ntiles = B * tiles_y * tiles_x;

  // weights [n][tap * 64 + c] -> padded LDS rows (once per workgroup)
  for (int e = tid; e < 64 * (KTOT / 8); e += NTH) {
    const int n = e / (KTOT / 8), q = e - n * (KTOT / 8);
    *reinterpret_cast<uint4*>(Bs + n * BROW + q * 16) =
        *reinterpret_cast<const uint4*>(wpk + (int64_t)n * KTOT + q * 8);
  }

  // halo piece e = tid + j * NTH of tile t -> registers (zeros outside the image)
  auto load_a = [&](int t, uint4 (&areg)[APER]) {
    const int b = t / (tiles_y * tiles_x), r = t - b * tiles_y * tiles_x;
    const int y0 = (r / tiles_x) * TH - 1, x0 = (r % tiles_x) * TW - 1;
    // branch-free: per-image buffer descriptor, out-of-image pieces (and tiles past the end:
    // zero-sized descriptor) read as zeros -- no control flow, so the wait before this register
    // set's LDS store counts only its own loads, not the next tile's
    const rsrc_t rs = mk_rsrc(x + (int64_t)b * H * W * 64, t < ntiles ? (uint32_t)H * W * 128 : 0u);
#pragma unroll
    for (int j = 0; j < APER; ++j) {
      const int e = tid + j * NTH;
      const int hp = e >> 3, q = e & 7;
      const int yy = y0 + hp / HWD, xx = x0 + hp % HWD;
      const bool in = e < APIECES && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const uint32_t off = in ? (uint32_t)((yy * W + xx) * 128 + q * 16) : OOB;
      areg[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
  auto store_a = [&](int buf, const uint4 (&areg)[APER]) {
#pragma unroll
    for (int j = 0; j < APER; ++j) {
      const int e = tid + j * NTH;
      // pieces past the halo land in the buffer's spare rows (no branch)
      *reinterpret_cast<uint4*>(As + buf * ABUF + hoff(e >> 3) + (e & 7) * 16) = areg[j];
    }
  };

  // this lane's A rows: fragment i covers tile rows wm*4 + 2i + (lane&31)/16, column lane & 15
  int hbase[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int tr = wm * 4 + 2 * i + ((lane & 31) >> 4), tc = lane & 15;
    hbase[i] = tr * AROWB + tc * AROW + (lane >> 5) * 16;
  }
  const int bbase = (wn * 32 + (lane & 31)) * BROW + (lane >> 5) * 16;

  // three tiles of halo loads in flight per thread: register sets R0 / R1 / R2 rotate; the loop
  // is unrolled by three so all stay static
  uint4 R0[APER], R1[APER], R2[APER];
  const int G = gridDim.x;
  load_a(blockIdx.x, R0);
  load_a(blockIdx.x + G, R1);
  load_a(blockIdx.x + 2 * G, R2);
  auto tile = [&](int t, int buf, uint4 (&R)[APER]) {
    store_a(buf, R);
    __syncthreads();  // halo (and, first time, weights) visible; the other buffer is free
    load_a(t + NSET * G, R);  // NSET tiles ahead, in flight during this tile and the next ones

    f32x16 acc[2];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
    const char* Ab = As + buf * ABUF;
    auto frags = [&](int tap, bf16x8_t (&af)[4][2], bf16x8_t (&bfr)[4]) {
      const int shift = (tap / 3) * AROWB + (tap % 3) * AROW;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bfr[kk] = *reinterpret_cast<const bf16x8_t*>(Bs + bbase + (tap * 64 + kk * 16) * 2);
#pragma unroll
        for (int i = 0; i < 2; ++i)
          af[kk][i] = *reinterpret_cast<const bf16x8_t*>(Ab + hbase[i] + shift + kk * 32);
      }
    };
    auto mma = [&](const bf16x8_t (&af)[4][2], const bf16x8_t (&bfr)[4]) {
#pragma unroll
      for (int kk = 0; kk < 4; ++kk)
#pragma unroll
        for (int i = 0; i < 2; ++i)
          acc[i] = raft_mfma32<F16>(af[kk][i], bfr[kk], acc[i]);
    };
    {
      bf16x8_t af[2][4][2], bfr[2][4];
      frags(0, af[0], bfr[0]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) frags(tap + 1, af[(tap + 1) & 1], bfr[(tap + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
        mma(af[tap & 1], bfr[tap & 1]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }

    const int b = t / (tiles_y * tiles_x), r = t - b * tiles_y * tiles_x;
    const int ty0 = (r / tiles_x) * TH, tx0 = (r % tiles_x) * TW;
    // epilogue: the accumulators go to an LDS [pixel][channel] bf16 tile, then out as 16-B rows
    // of 8 channels (4 stores per thread instead of 32 scattered 2-B stores per lane, whose issue
    // set the tile time); pixels past the image edge dropped
    const int n = wn * 32 + (lane & 31);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int p = wm * 64 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
        *reinterpret_cast<uint16_t*>(Os + p * OROW + n * 2) = raft_f2h<F16>(acc[i][rr]);
      }
    float* red = reinterpret_cast<float*>(Os + OBUF);
    if (part != nullptr) {
      // norm statistics from the registers: this lane's 32 rounded values of channel n (two
      // passes: mean, then squared deviations), merged with lane + 32's (Chan) and staged per
      // pixel half wm; the two halves are merged after the staging barrier -- no extra barrier,
      // no LDS re-read of the tile
      float v[2][16];
      float cnt = 0.f, sum = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int p = wm * 64 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
          const bool ok = ty0 + p / TW < H && tx0 + p % TW < W;
          v[i][rr] = ok ? raft_h2f<F16>(raft_f2h<F16>(acc[i][rr])) : 0.f;
          cnt += ok ? 1.f : 0.f;
          sum += v[i][rr];
        }
      const float mu = cnt > 0.f ? sum / cnt : 0.f;
      float m2 = 0.f;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int rr = 0; rr < 16; ++rr) {
          const int p = wm * 64 + i * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
          const bool ok = ty0 + p / TW < H && tx0 + p % TW < W;
          const float d = v[i][rr] - mu;
          m2 += ok ? d * d : 0.f;
        }
      const float cb = __shfl_xor(cnt, 32, 64), mb = __shfl_xor(mu, 32, 64), qb = __shfl_xor(m2, 32, 64);
      const float nn = cnt + cb;
      const float dl = mb - mu;
      if (lane < 32) {
        red[wm * 64 + n] = nn;
        red[128 + wm * 64 + n] = nn > 0.f ? mu + dl * (cb / nn) : 0.f;
        red[256 + wm * 64 + n] = m2 + qb + (nn > 0.f ? dl * dl * cnt * cb / nn : 0.f);
      }
    }
    __syncthreads();  // staged tile (and statistics halves) complete; the next tile's stores come
                      // after its own barrier
    const rsrc_t ro = mk_rsrc(out + (int64_t)b * H * W * 64, (uint32_t)H * W * 128);
#pragma unroll
    for (int j = 0; j < TH * TW * 8 / NTH; ++j) {
      const int e = tid + j * NTH;
      const int p = e >> 3, q = e & 7;
      const int yy = ty0 + p / TW, xx = tx0 + p % TW;
      const uint4 v = *reinterpret_cast<const uint4*>(Os + p * OROW + q * 16);
      // pixels past the image edge: out-of-range offset, the store is dropped (no branch)
      const uint32_t off = yy < H && xx < W ? (uint32_t)((yy * W + xx) * 128 + q * 16) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                             ro, off, 0, 0);
    }
    if (part != nullptr && tid < 64) {
      // the tile's row for the tiled norm finalize: sum (x - K) = 0 with K = the tile mean,
      // sum (x - K)^2 = M2, K, count (halves merged in a fixed order: deterministic)
      const float na = red[tid], nb = red[64 + tid];
      const float ma = red[128 + tid], mb = red[192 + tid];
      const float nn = na + nb, dl = mb - ma;
      float* dst = part + (int64_t)t * 256;
      dst[tid] = 0.f;
      dst[64 + tid] = red[256 + tid] + red[320 + tid] + (nn > 0.f ? dl * dl * na * nb / nn : 0.f);
      dst[128 + tid] = nn > 0.f ? ma + dl * (nb / nn) : 0.f;
      dst[192 + tid] = nn;
    }
  };
  // three register sets, two LDS buffers: the buffer index alternates at run time
  int k = 0;
  for (int t = blockIdx.x; t < ntiles; t += 3 * G, k += 3) {
    tile(t, k & 1, R0);
    if (t + G < ntiles) tile(t + G, (k + 1) & 1, R1);
    if (t + 2 * G < ntiles) tile(t + 2 * G, k & 1, R2);
  }
}

// ---- channel-half variant: two workgroups per CU.
// The kernel above holds ~152 KB of LDS, so one workgroup (one wave per SIMD) owns a CU and its
// phases -- halo store, barrier, K loop, output staging, barrier, stores -- never overlap: 27 %
// MFMA-busy at 2.4 TB/s (profiles/r6/final/pmc.txt).  Here a workgroup computes one 32-channel
// half of a tile: the half's 32 weight rows (37 KB), ONE halo buffer (the staging barrier already
// orders the next tile's halo store after every wave's K loop) and a 32-channel output stage fit
// in ~77 KB, so two workgroups share a CU and one's MFMAs run beside the other's barriers and
// epilogue.  4 waves x 32 pixels (two tile rows) x 32 channels, 36 MFMAs per wave per tile.
// Work items (tile, half): i = 16a + 8h + r -> tile 8a + r, half h.  The grid is a multiple of 16,
// so a workgroup keeps one half for its whole life (weights loaded once) and the two halves of a
// tile go to workgroups b and b + 8 -- the same XCD under round-robin dispatch, where the second
// read of the halo hits L2.
constexpr int HBBUF = 32 * BROW;               // 37,376 B
constexpr int HOROW = 80;                      // staged pixel: 32 channels (64 B) + 16 pad
constexpr int HOBUF = TH * TW * HOROW;         // 10,240 B
template <bool F16 = false>
__global__ __launch_bounds__(NTH, 2) void conv_enc64h_kernel(const uint16_t* __restrict__ x,
                                                             const uint16_t* __restrict__ wpk,
                                                             uint16_t* __restrict__ out, int B,
                                                             int H, int W, int tiles_y,
                                                             int tiles_x, int nitems) {
  __shared__ __attribute__((aligned(16))) char smem[ABUF + HBBUF + HOBUF];
  char* As = smem;                 // halo
  char* Bs = smem + ABUF;          // the half's weights
  char* Os = Bs + HBBUF;           // output staging (bf16 [pixel][32 channels])
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ntiles = B * tiles_y * tiles_x;
  const int G = gridDim.x;
  const int h = (blockIdx.x >> 3) & 1;

  for (int e = tid; e < 32 * (KTOT / 8); e += NTH) {
    const int n = e / (KTOT / 8), q = e - n * (KTOT / 8);
    *reinterpret_cast<uint4*>(Bs + n * BROW + q * 16) =
        *reinterpret_cast<const uint4*>(wpk + (int64_t)(h * 32 + n) * KTOT + q * 8);
  }
  auto tile_of = [](int i) { return (i >> 4) * 8 + (i & 7); };
  auto load_a = [&](int i, uint4 (&areg)[APER]) {
    const int t = tile_of(i);
    const bool live = i < nitems && t < ntiles;
    const int tt = live ? t : 0;
    const int b = tt / (tiles_y * tiles_x), r = tt - b * tiles_y * tiles_x;
    const int y0 = (r / tiles_x) * TH - 1, x0 = (r % tiles_x) * TW - 1;
    const rsrc_t rs = mk_rsrc(x + (int64_t)b * H * W * 64, live ? (uint32_t)H * W * 128 : 0u);
#pragma unroll
    for (int j = 0; j < APER; ++j) {
      const int e = tid + j * NTH;
      const int hp = e >> 3, q = e & 7;
      const int yy = y0 + hp / HWD, xx = x0 + hp % HWD;
      const bool in = e < APIECES && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const uint32_t off = in ? (uint32_t)((yy * W + xx) * 128 + q * 16) : OOB;
      areg[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
  auto store_a = [&](const uint4 (&areg)[APER]) {
#pragma unroll
    for (int j = 0; j < APER; ++j) {
      const int e = tid + j * NTH;
      *reinterpret_cast<uint4*>(As + hoff(e >> 3) + (e & 7) * 16) = areg[j];
    }
  };
  const int hbase = (2 * wave + ((lane & 31) >> 4)) * AROWB + (lane & 15) * AROW + (lane >> 5) * 16;
  const int bbase = (lane & 31) * BROW + (lane >> 5) * 16;

  uint4 R0[APER], R1[APER], R2[APER];
  load_a(blockIdx.x, R0);
  load_a(blockIdx.x + G, R1);
  load_a(blockIdx.x + 2 * G, R2);
  auto tile = [&](int i, uint4 (&R)[APER]) {
    store_a(R);
    __syncthreads();  // halo (and, first time, weights) visible
    load_a(i + NSET * G, R);
    f32x16 acc;
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] = 0.f;
    auto frags = [&](int tap, bf16x8_t (&af)[4], bf16x8_t (&bfr)[4]) {
      const int shift = (tap / 3) * AROWB + (tap % 3) * AROW;
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        bfr[kk] = *reinterpret_cast<const bf16x8_t*>(Bs + bbase + (tap * 64 + kk * 16) * 2);
        af[kk] = *reinterpret_cast<const bf16x8_t*>(As + hbase + shift + kk * 32);
      }
    };
    {
      bf16x8_t af[2][4], bfr[2][4];
      frags(0, af[0], bfr[0]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) frags(tap + 1, af[(tap + 1) & 1], bfr[(tap + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) acc = raft_mfma32<F16>(af[tap & 1][kk], bfr[tap & 1][kk], acc);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
    const int t = tile_of(i);
    const bool live = t < ntiles;   // i < nitems here
    const int tt = live ? t : 0;
    const int b = tt / (tiles_y * tiles_x), r = tt - b * tiles_y * tiles_x;
    const int ty0 = (r / tiles_x) * TH, tx0 = (r % tiles_x) * TW;
    const int n = lane & 31;
#pragma unroll
    for (int rr = 0; rr < 16; ++rr) {
      const int p = wave * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
      *reinterpret_cast<uint16_t*>(Os + p * HOROW + n * 2) = raft_f2h<F16>(acc[rr]);
    }
    __syncthreads();  // staged tile complete; the next tile's staging comes after its own barrier
    const rsrc_t ro = mk_rsrc(out + (int64_t)b * H * W * 64, live ? (uint32_t)H * W * 128 : 0u);
#pragma unroll
    for (int j = 0; j < TH * TW * 4 / NTH; ++j) {
      const int e = tid + j * NTH;
      const int p = e >> 2, q = e & 3;
      const int yy = ty0 + p / TW, xx = tx0 + p % TW;
      const uint4 v = *reinterpret_cast<const uint4*>(Os + p * HOROW + q * 16);
      const uint32_t off = yy < H && xx < W ? (uint32_t)((yy * W + xx) * 128 + h * 64 + q * 16) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                             ro, off, 0, 0);
    }
  };
  for (int i = blockIdx.x; i < nitems; i += 3 * G) {
    tile(i, R0);
    if (i + G < nitems) tile(i + G, R1);
    if (i + 2 * G < nitems) tile(i + 2 * G, R2);
  }
}

// ---- producer / MFMA wave split (the per-phase stamps of the kernel above: the K loop is 44 % of
// a wave's time, the halo loads, LDS stores, output staging, stores and barriers the rest, and
// those phases never overlap the wave's own MFMAs).  8 waves: waves 0-3 run only the K loop and
// the output staging of a 32-channel tile half (as above), waves 4-7 only move data -- the next
// item's halo registers -> LDS, the item after that global -> registers, the previous item's
// staged output LDS -> global.  Two halo buffers and two output stages in LDS (119,808 B, one
// workgroup per CU), ONE barrier per item: in phase k the MFMA waves work on item k while the
// producers store item k + 1's halo and drain item k - 1's output.
constexpr int NTH2 = 512;                      // 4 MFMA waves + 4 producer waves
constexpr int NPT = NTH2 - 256;                // producer threads
constexpr int APERP = (APIECES + NPT - 1) / NPT;  // 6 halo pieces per producer thread
template <bool F16 = false>
__global__ __launch_bounds__(NTH2, 1) void conv_enc64p_kernel(const uint16_t* __restrict__ x,
                                                              const uint16_t* __restrict__ wpk,
                                                              uint16_t* __restrict__ out, int B,
                                                              int H, int W, int tiles_y,
                                                              int tiles_x, int nitems) {
  __shared__ __attribute__((aligned(16))) char smem[HBBUF + 2 * ABUF + 2 * HOBUF];
  char* Bs = smem;                         // the half's weights
  char* As = smem + HBBUF;                 // 2 halo buffers
  char* Os = As + 2 * ABUF;                // 2 output stages
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bool producer = wave >= 4;
  const int ptid = tid - 256;              // producer thread index (valid when producer)
  const int ntiles = B * tiles_y * tiles_x;
  const int G = gridDim.x;
  const int h = (blockIdx.x >> 3) & 1;
  const int K = (nitems - (int)blockIdx.x + G - 1) / G;   // items of this workgroup (>= 1)

  for (int e = tid; e < 32 * (KTOT / 8); e += NTH2) {
    const int n = e / (KTOT / 8), q = e - n * (KTOT / 8);
    *reinterpret_cast<uint4*>(Bs + n * BROW + q * 16) =
        *reinterpret_cast<const uint4*>(wpk + (int64_t)(h * 32 + n) * KTOT + q * 8);
  }
  auto tile_of = [](int i) { return (i >> 4) * 8 + (i & 7); };
  auto item = [&](int k) { return (int)blockIdx.x + k * G; };
  auto load_a = [&](int i, uint4 (&areg)[APERP]) {
    const int t = tile_of(i);
    const bool live = i < nitems && t < ntiles;
    const int tt = live ? t : 0;
    const int b = tt / (tiles_y * tiles_x), r = tt - b * tiles_y * tiles_x;
    const int y0 = (r / tiles_x) * TH - 1, x0 = (r % tiles_x) * TW - 1;
    const rsrc_t rs = mk_rsrc(x + (int64_t)b * H * W * 64, live ? (uint32_t)H * W * 128 : 0u);
#pragma unroll
    for (int j = 0; j < APERP; ++j) {
      const int e = ptid + j * NPT;
      const int hp = e >> 3, q = e & 7;
      const int yy = y0 + hp / HWD, xx = x0 + hp % HWD;
      const bool in = e < APIECES && (unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W;
      const uint32_t off = in ? (uint32_t)((yy * W + xx) * 128 + q * 16) : OOB;
      areg[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
  auto store_a = [&](char* dst, const uint4 (&areg)[APERP]) {
#pragma unroll
    for (int j = 0; j < APERP; ++j) {
      const int e = ptid + j * NPT;   // pieces past the halo land in the spare row (no branch)
      *reinterpret_cast<uint4*>(dst + hoff(e >> 3) + (e & 7) * 16) = areg[j];
    }
  };
  auto drain = [&](int i, const char* src) {   // staged output of item i -> global
    const int t = tile_of(i);
    const bool live = t < ntiles;
    const int tt = live ? t : 0;
    const int b = tt / (tiles_y * tiles_x), r = tt - b * tiles_y * tiles_x;
    const int ty0 = (r / tiles_x) * TH, tx0 = (r % tiles_x) * TW;
    const rsrc_t ro = mk_rsrc(out + (int64_t)b * H * W * 64, live ? (uint32_t)H * W * 128 : 0u);
#pragma unroll
    for (int j = 0; j < TH * TW * 4 / NPT; ++j) {
      const int e = ptid + j * NPT;
      const int p = e >> 2, q = e & 3;
      const int yy = ty0 + p / TW, xx = tx0 + p % TW;
      const uint4 v = *reinterpret_cast<const uint4*>(src + p * HOROW + q * 16);
      const uint32_t off = yy < H && xx < W ? (uint32_t)((yy * W + xx) * 128 + h * 64 + q * 16) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                             ro, off, 0, 0);
    }
  };

  uint4 R[APERP];
  if (producer) {
    load_a(item(0), R);
    store_a(As, R);
    load_a(item(1), R);   // item >= nitems: zero-size descriptor, zeros
  }
  __syncthreads();        // weights and item 0's halo visible

  const int hbase = (2 * (wave & 3) + ((lane & 31) >> 4)) * AROWB + (lane & 15) * AROW + (lane >> 5) * 16;
  const int bbase = (lane & 31) * BROW + (lane >> 5) * 16;
  // producers first at issue arbitration, so their loads go out while the MFMA waves run: fnet
  // 113.4 / 113.5 vs 116.9 / 118.3 us per call (MFMA waves first: 112.9 / 118.5;
  // profiles/r6/enc64h/pipe_prio_ab.log)
  if (producer) __builtin_amdgcn_s_setprio(1);
  for (int k = 0; k < K; ++k) {
    if (!producer) {
      const char* Ab = As + (k & 1) * ABUF;
      f32x16 acc;
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = 0.f;
      auto frags = [&](int tap, bf16x8_t (&af)[4], bf16x8_t (&bfr)[4]) {
        const int shift = (tap / 3) * AROWB + (tap % 3) * AROW;
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) {
          bfr[kk] = *reinterpret_cast<const bf16x8_t*>(Bs + bbase + (tap * 64 + kk * 16) * 2);
          af[kk] = *reinterpret_cast<const bf16x8_t*>(Ab + hbase + shift + kk * 32);
        }
      };
      bf16x8_t af[2][4], bfr[2][4];
      frags(0, af[0], bfr[0]);
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        if (tap + 1 < 9) frags(tap + 1, af[(tap + 1) & 1], bfr[(tap + 1) & 1]);
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int kk = 0; kk < 4; ++kk) acc = raft_mfma32<F16>(af[tap & 1][kk], bfr[tap & 1][kk], acc);
        __builtin_amdgcn_sched_barrier(0);
      }
      char* Ob = Os + (k & 1) * HOBUF;
      const int n = lane & 31;
#pragma unroll
      for (int rr = 0; rr < 16; ++rr) {
        const int p = (wave & 3) * 32 + (rr & 3) + 8 * (rr >> 2) + 4 * (lane >> 5);
        *reinterpret_cast<uint16_t*>(Ob + p * HOROW + n * 2) = raft_f2h<F16>(acc[rr]);
      }
    } else {
      if (k + 1 < K) store_a(As + ((k + 1) & 1) * ABUF, R);
      if (k + 2 < K) load_a(item(k + 2), R);
      if (k >= 1) drain(item(k - 1), Os + ((k - 1) & 1) * HOBUF);
    }
    __syncthreads();  // item k's output staged, item k + 1's halo stored
  }
  if (producer) drain(item(K - 1), Os + ((K - 1) & 1) * HOBUF);
}

}  // namespace

// persistent grids: the channel-half kernel (default, plain launches) runs 2 x CUs workgroups of
// ~77 KB of LDS, the statistics kernel one workgroup per CU (~153 KB), capped by the work items.
// Channel-half vs one-per-CU at chairs: fnet 127.3 -> 119.6 us, cnet 66.5 -> 58.5 us per call,
// bitwise-equal outputs (profiles/r6/enc64h/)
bool launch_conv_enc64(const uint16_t* x, const uint16_t* wpk, uint16_t* out, int B, int H, int W,
                       int grid_cap, int f16, hipStream_t stream, float* part) {
  const int ty = (H + TH - 1) / TH, tx = (W + TW - 1) / TW;
  const int ntiles = B * ty * tx;
  if (ntiles <= 0) return true;
  // RAFT_ENC64_KERNEL (A/B of the plain conv; the tile statistics, part != null, are only in the
  // one-workgroup-per-CU kernel): pipe (producer / MFMA waves, default) | half | wg1
  static const int kind = [] {
    const char* e = std::getenv("RAFT_ENC64_KERNEL");
    if (e && std::strcmp(e, "half") == 0) return 1;
    if (e && std::strcmp(e, "wg1") == 0) return 2;
    return 0;
  }();
  if (kind == 0 && part == nullptr) {
    const int nitems = (ntiles + 7) / 8 * 16;
    int g = grid_cap < nitems ? grid_cap : nitems;
    g = g / 16 * 16;
    if (f16)
      hipLaunchKernelGGL((conv_enc64p_kernel<true>), dim3(g), dim3(NTH2), 0, stream, x, wpk, out, B, H, W,
                         ty, tx, nitems);
    else
      hipLaunchKernelGGL((conv_enc64p_kernel<false>), dim3(g), dim3(NTH2), 0, stream, x, wpk, out, B, H, W,
                         ty, tx, nitems);
    return true;
  }
  if (kind == 1 && part == nullptr) {
    const int nitems = (ntiles + 7) / 8 * 16;
    int g = 2 * grid_cap < nitems ? 2 * grid_cap : nitems;
    g = g / 16 * 16;
    if (f16)
      hipLaunchKernelGGL((conv_enc64h_kernel<true>), dim3(g), dim3(NTH), 0, stream, x, wpk, out, B, H, W,
                         ty, tx, nitems);
    else
      hipLaunchKernelGGL((conv_enc64h_kernel<false>), dim3(g), dim3(NTH), 0, stream, x, wpk, out, B, H, W,
                         ty, tx, nitems);
    return true;
  }
  const int grid = ntiles < grid_cap ? ntiles : grid_cap;
  if (f16)   // fp16 operands (fp16 autocast)
    hipLaunchKernelGGL((conv_enc64_kernel<true>), dim3(grid), dim3(NTH), 0, stream, x, wpk, out, B,
                       H, W, ty, tx, part);
  else
    hipLaunchKernelGGL((conv_enc64_kernel<false>), dim3(grid), dim3(NTH), 0, stream, x, wpk, out, B, H,
                       W, ty, tx, part);
  return true;
}
