// Encoder stem conv on MFMA (`core/extractor.py:129,165`: conv1 = 7x7, stride 2, pad 3, 3 -> 64
// channels; 32 for SmallEncoder) -- forward and weight gradient, NHWC 16-bit operands (bf16, or
// fp16 under fp16 autocast), fp32 accumulation.  The input gradient is never needed on the
// training path (the conv reads the images).
//
// MIOpen ran this conv as an implicit GEMM over 3-channel K slices (igemm_fwd_gtcx35 bt256x64x8,
// ~100 us per call at chairs) and its weight gradient as igemm_wrw ... gkgs (~134 us per call plus
// a zero fill of the output).  Here the GEMM K runs over (ky, kx * 3 + c): for one filter row ky
// the 21 products of an output pixel read 21 CONTIGUOUS 16-bit values of one input row -- the
// 7 taps x 3 channels of the NHWC pixels 2x-3 .. 2x+3 -- so an 8-deep MFMA K fragment is one
// 16-byte span of the tile's input region staged in LDS (4 dword reads at 4-byte alignment).
// Each filter row is padded to 32 K slots (K = 7 x 32 = 224, 14 MFMA K steps): the weights are
// zero in slots 21..31, whose products read neighbouring finite values of the region.
//
//   forward: persistent workgroups holding the packed weight fragments in registers; 8 x 16 output
//            tiles whose 21 x 37 x 3 input region is staged once per tile (loaded a tile ahead
//            into registers, zeros outside the image through out-of-range buffer offsets);
//            output through LDS as 16-byte rows.
//   weight gradient: the same tiles, dW[n][k] += G^T A with the tile's 128 pixels as the MFMA K
//            (one tile row = one K step of 16): G fragments by transposing LDS reads
//            (ds_read_b64_tr_b16), A fragments gathered from the region; fp32 per-workgroup
//            partials summed in a fixed order by stem_wgrad_reduce_kernel (no atomics), which also
//            writes the (C, 7, 7, 3)-ordered 16-bit weight gradient.
#include "common.h"
#include "launchers.h"

namespace {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4_t __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) bf16x4_t lds_bf16x4_t;
typedef __amdgpu_buffer_rsrc_t rsrc_t;

__device__ __forceinline__ rsrc_t mk_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}

constexpr int TH = 8, TW = 16, TP = TH * TW;        // output tile: 128 pixels
constexpr int RH = 2 * TH + 5, RW = 2 * TW + 5;     // input region: 21 x 37 pixels
constexpr int RVALS = RW * 3;                        // 111 16-bit values per region row
constexpr int RROW = 112;                            // staged row (4-byte aligned rows)
constexpr int RBUF = RH * RROW + 32;                 // + slack: K spans run <= 10 past a row
constexpr int RELEMS = RH * RVALS;                   // 2331 staged values per tile
constexpr int NTH = 256;
constexpr int RPER = (RELEMS + NTH - 1) / NTH;       // 10 per thread
constexpr int KP = 224, KSTEPS = KP / 16;            // padded K, 16-deep steps
constexpr uint32_t OOB = 0x80000000u;

struct TileGeo {
  int b, oy0, ox0;
};
__device__ __forceinline__ TileGeo tile_geo(int t, int ty, int tx) {
  TileGeo g;
  g.b = t / (ty * tx);
  const int r = t - g.b * ty * tx;
  g.oy0 = (r / tx) * TH;
  g.ox0 = (r % tx) * TW;
  return g;
}

// the tile's input region -> registers (RPER 16-bit values per thread; zeros outside the image)
__device__ __forceinline__ void load_region(const uint16_t* __restrict__ x, int H, int W, int t,
                                            int ntiles, int ty, int tx, int tid, uint16_t (&rv)[RPER]) {
  const TileGeo g = tile_geo(t < ntiles ? t : 0, ty, tx);
  const rsrc_t rs = mk_rsrc(x + (int64_t)g.b * H * W * 3, t < ntiles ? (uint32_t)H * W * 6 : 0u);
  const int iy0 = 2 * g.oy0 - 3, ix0 = 2 * g.ox0 - 3;
#pragma unroll
  for (int j = 0; j < RPER; ++j) {
    const int e = tid + j * NTH;
    const int row = e / RVALS, col = e - row * RVALS;
    const int iy = iy0 + row, ix = ix0 + col / 3;
    const bool in = e < RELEMS && (unsigned)iy < (unsigned)H && (unsigned)ix < (unsigned)W;
    const uint32_t off = in ? (uint32_t)(((iy * W + ix) * 3 + col % 3) * 2) : OOB;
    rv[j] = __builtin_amdgcn_raw_buffer_load_b16(rs, off, 0, 0);
  }
}
__device__ __forceinline__ void store_region(uint16_t* R, int tid, const uint16_t (&rv)[RPER]) {
#pragma unroll
  for (int j = 0; j < RPER; ++j) {
    const int e = tid + j * NTH;
    const int row = e / RVALS, col = e - row * RVALS;
    if (e < RELEMS) R[row * RROW + col] = rv[j];
  }
}

// 8 contiguous 16-bit values at a 4-byte aligned LDS address as one MFMA fragment
__device__ __forceinline__ bf16x8_t ld_span8(const uint16_t* p) {
  const uint32_t* q = reinterpret_cast<const uint32_t*>(p);
  return __builtin_bit_cast(bf16x8_t, make_uint4(q[0], q[1], q[2], q[3]));
}

// NB = output channels / 32 (2: BasicEncoder, 1: SmallEncoder)
template <int NB, bool F16>
__global__ __launch_bounds__(NTH, 2) void stem_conv_fwd_kernel(const uint16_t* __restrict__ x,
                                                               const uint16_t* __restrict__ w,
                                                               uint16_t* __restrict__ out, int B,
                                                               int H, int W, int Ho, int Wo) {
  constexpr int C = NB * 32;
  constexpr int OROW = C * 2 + 16;   // staged output row bytes (padded)
  __shared__ __attribute__((aligned(16))) uint16_t R[2][RBUF];
  __shared__ __attribute__((aligned(16))) char Os[TP * OROW];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ty = (Ho + TH - 1) / TH, tx = (Wo + TW - 1) / TW;
  const int ntiles = B * ty * tx;

  // region buffers: the row tails and the slack are never staged and must read as zeros
  for (int e = tid; e < 2 * RBUF; e += NTH) (&R[0][0])[e] = 0;
  __syncthreads();   // zeros in place before any region store
  // this lane's weight fragments, all K steps: w is the (C, 7, 7, 3) weight, i.e. per output
  // channel 7 rows of 21 values (ky, kx * 3 + c); slot 21..31 of each padded row is zero
  bf16x8_t wf[KSTEPS][NB];
#pragma unroll
  for (int s = 0; s < KSTEPS; ++s)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb) {
      const int n = nb * 32 + (lane & 31);
      const int k0 = 16 * s + 8 * (lane >> 5);
      const int ky = k0 >> 5, j0 = k0 & 31;
      uint16_t v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = j0 + i < 21 ? w[n * 147 + ky * 21 + j0 + i] : (uint16_t)0;
      wf[s][nb] = __builtin_bit_cast(bf16x8_t, make_uint4(v[0] | ((uint32_t)v[1] << 16), v[2] | ((uint32_t)v[3] << 16),
                                                          v[4] | ((uint32_t)v[5] << 16), v[6] | ((uint32_t)v[7] << 16)));
    }
  // this lane's A rows: pixel p = wave * 32 + (lane & 31) of the tile (2 tile rows per wave), K
  // half (lane >> 5); step s reads region row 2 py + s / 2 at column 6 px + 16 (s & 1) + 8 half
  const int p = wave * 32 + (lane & 31);
  const int abase = 2 * (p / TW) * RROW + 6 * (p % TW) + 8 * (lane >> 5);

  uint16_t rv[RPER];
  load_region(x, H, W, blockIdx.x, ntiles, ty, tx, tid, rv);
  int buf = 0;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x, buf ^= 1) {
    store_region(R[buf], tid, rv);
    __syncthreads();   // region visible; the previous tile's output staging fully read
    load_region(x, H, W, t + gridDim.x, ntiles, ty, tx, tid, rv);   // next tile, in flight
    f32x16 acc[NB];
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[nb][r] = 0.f;
    const uint16_t* Rb = R[buf] + abase;
#pragma unroll
    for (int s = 0; s < KSTEPS; ++s) {
      const bf16x8_t af = ld_span8(Rb + (s >> 1) * RROW + 16 * (s & 1));
#pragma unroll
      for (int nb = 0; nb < NB; ++nb) acc[nb] = raft_mfma32<F16>(af, wf[s][nb], acc[nb]);
    }
    // output tile through LDS, then 16-byte rows (pixels past the map dropped)
#pragma unroll
    for (int nb = 0; nb < NB; ++nb)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int pp = wave * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        *reinterpret_cast<uint16_t*>(Os + pp * OROW + (nb * 32 + (lane & 31)) * 2) = raft_f2h<F16>(acc[nb][r]);
      }
    __syncthreads();
    const TileGeo g = tile_geo(t, ty, tx);
    const rsrc_t ro = mk_rsrc(out + (int64_t)g.b * Ho * Wo * C, (uint32_t)Ho * Wo * C * 2);
    constexpr int CH = C / 8;   // 16-byte chunks per pixel
#pragma unroll
    for (int j = 0; j < TP * CH / NTH; ++j) {
      const int e = tid + j * NTH;
      const int pp = e / CH, q = e % CH;
      const int oy = g.oy0 + pp / TW, ox = g.ox0 + pp % TW;
      const uint4 v = *reinterpret_cast<const uint4*>(Os + pp * OROW + q * 16);
      const uint32_t off = oy < Ho && ox < Wo ? (uint32_t)(((oy * Wo + ox) * C + q * 8) * 2) : OOB;
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, v),
                                             ro, off, 0, 0);
    }
  }
}

// 8-deep K fragment of a [k][col] LDS matrix (row stride S elements), columns base..base+31
__device__ __forceinline__ bf16x8_t tr_frag8(const uint16_t* X, int S, int kbase, int base, int lane) {
  const int gi = lane >> 4, li = lane & 15, q = li >> 2, pp = li & 3;
  const int col = base + (gi & 1) * 16 + 4 * pp;
  const int row = kbase + (gi >> 1) * 8 + q;
  bf16x4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(X + row * S + col));
  bf16x4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4_t*)(X + (row + 4) * S + col));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// dW partials: part[blockIdx.x][C][224] = sum over this workgroup's tiles of G^T A
template <int NB, bool F16>
__global__ __launch_bounds__(NTH, 3) void stem_conv_wgrad_kernel(const uint16_t* __restrict__ x,
                                                                 const uint16_t* __restrict__ gy,
                                                                 float* __restrict__ part, int B,
                                                                 int H, int W, int Ho, int Wo) {
  constexpr int C = NB * 32;
  constexpr int GS = C + 16;                 // G tile rows (16-bit elements, padded)
  constexpr int NBLK = NB * 7;               // 32 x 32 output blocks: (channel block, ky)
  constexpr int MAXB = (NBLK + 3) / 4;       // per wave
  constexpr int GCH = TP * C / 8;            // 16-byte chunks of a G tile
  constexpr int GPER = GCH / NTH;
  __shared__ __attribute__((aligned(16))) uint16_t R[2][RBUF];
  __shared__ __attribute__((aligned(16))) uint16_t Gs[2][TP * GS];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int ty = (Ho + TH - 1) / TH, tx = (Wo + TW - 1) / TW;
  const int ntiles = B * ty * tx;
  for (int e = tid; e < 2 * RBUF; e += NTH) (&R[0][0])[e] = 0;
  __syncthreads();   // zeros in place before any region store

  auto load_g = [&](int t, uint4 (&gv)[GPER]) {
    const TileGeo g = tile_geo(t < ntiles ? t : 0, ty, tx);
    const rsrc_t rs = mk_rsrc(gy + (int64_t)g.b * Ho * Wo * C, t < ntiles ? (uint32_t)Ho * Wo * C * 2 : 0u);
#pragma unroll
    for (int j = 0; j < GPER; ++j) {
      const int e = tid + j * NTH;
      const int pp = e / (C / 8), q = e % (C / 8);
      const int oy = g.oy0 + pp / TW, ox = g.ox0 + pp % TW;
      const uint32_t off = oy < Ho && ox < Wo ? (uint32_t)(((oy * Wo + ox) * C + q * 8) * 2) : OOB;
      gv[j] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  };
  auto store_g = [&](uint16_t* G, const uint4 (&gv)[GPER]) {
#pragma unroll
    for (int j = 0; j < GPER; ++j) {
      const int e = tid + j * NTH;
      const int pp = e / (C / 8), q = e % (C / 8);
      *reinterpret_cast<uint4*>(G + pp * GS + q * 8) = gv[j];
    }
  };

  f32x16 acc[MAXB];
#pragma unroll
  for (int i = 0; i < MAXB; ++i)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  // this wave's blocks: wave, wave + 4, ...; block = (channel block mb, filter row ky)
  const int col = lane & 31;   // the block column: region value (ky, kx * 3 + c) slot col

  uint16_t rv[RPER];
  uint4 gv[GPER];
  load_region(x, H, W, blockIdx.x, ntiles, ty, tx, tid, rv);
  load_g(blockIdx.x, gv);
  int buf = 0;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x, buf ^= 1) {
    store_region(R[buf], tid, rv);
    store_g(Gs[buf], gv);
    __syncthreads();   // both tiles visible; the other buffers were last read before this barrier
    load_region(x, H, W, t + gridDim.x, ntiles, ty, tx, tid, rv);
    load_g(t + gridDim.x, gv);
    const uint16_t* Rb = R[buf];
    const uint16_t* Gb = Gs[buf];
    // K step s = tile row s (16 pixels); this lane's 8 pixels px = 8 (lane >> 5) + i
#pragma unroll
    for (int s = 0; s < TH; ++s) {
      bf16x8_t gfr[NB];
#pragma unroll
      for (int mb = 0; mb < NB; ++mb) gfr[mb] = tr_frag8(Gb, GS, 16 * s, mb * 32, lane);
#pragma unroll
      for (int i = 0; i < MAXB; ++i) {
        const int blk = wave + 4 * i;
        if (blk < NBLK) {
          const int mb = blk / 7, ky = blk - mb * 7;
          // region row 2 s + ky, columns 6 px + col for the lane's 8 pixels (stride 6 values)
          const uint16_t* rp = Rb + (2 * s + ky) * RROW + 48 * (lane >> 5) + col;
          uint16_t v[8];
#pragma unroll
          for (int q = 0; q < 8; ++q) v[q] = rp[6 * q];
          const bf16x8_t af = __builtin_bit_cast(bf16x8_t, make_uint4(v[0] | ((uint32_t)v[1] << 16), v[2] | ((uint32_t)v[3] << 16),
                                                                      v[4] | ((uint32_t)v[5] << 16), v[6] | ((uint32_t)v[7] << 16)));
          acc[i] = raft_mfma32<F16>(mb == 0 ? gfr[0] : gfr[NB - 1], af, acc[i]);
        }
      }
    }
  }
  // partial rows: D[n][k] with n = mb * 32 + (r & 3) + 8 (r >> 2) + 4 (lane >> 5), k = ky * 32 + col
  float* P = part + (int64_t)blockIdx.x * C * KP;
#pragma unroll
  for (int i = 0; i < MAXB; ++i) {
    const int blk = wave + 4 * i;
    if (blk < NBLK) {
      const int mb = blk / 7, ky = blk - mb * 7;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int n = mb * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        P[n * KP + ky * 32 + col] = acc[i][r];
      }
    }
  }
}

// dw[n][ky][kx][c] (16-bit, the (C, 7, 7, 3) order of a channels_last (C, 3, 7, 7) weight) = sum
// over the nparts workgroup partials, fixed order: block = 16 elements x 16 lanes, lane L sums
// partials L, L + 16, ..., then the 16 lane sums in order (588 blocks for C = 64: every CU
// streams partial rows; 4 lanes per element and 64 elements per block left the reduce waiting
// on one strided load chain per element on 37 CUs: 41 us per call)
template <bool F16>
__global__ __launch_bounds__(256) void stem_wgrad_reduce_kernel(const float* __restrict__ part, int nparts,
                                                                int C, uint16_t* __restrict__ dw) {
  constexpr int LANES = 16, EPB = 16;
  __shared__ float red[LANES][EPB];
  const int el = threadIdx.x & (EPB - 1), l = threadIdx.x / EPB;
  const int e = blockIdx.x * EPB + el;
  const int total = C * 147;
  float s = 0.f;
  if (e < total) {
    const int n = e / 147, k = e - n * 147, ky = k / 21, j = k - ky * 21;
    const int src = n * KP + ky * 32 + j;
    for (int q = l; q < nparts; q += LANES) s += part[(int64_t)q * C * KP + src];
  }
  red[l][el] = s;
  __syncthreads();
  if (l == 0 && e < total) {
    float v = 0.f;
#pragma unroll
    for (int q = 0; q < LANES; ++q) v += red[q][el];
    dw[e] = raft_f2h<F16>(v);
  }
}

}  // namespace

int stem_conv_tiles(int B, int Ho, int Wo) {
  return B * ((Ho + TH - 1) / TH) * ((Wo + TW - 1) / TW);
}

bool launch_stem_conv_fwd(const uint16_t* x, const uint16_t* w, uint16_t* out, int B, int H, int W,
                          int Ho, int Wo, int C, int grid, int f16, hipStream_t stream) {
  if (grid <= 0) return true;
#define STEM_FWD(NB, F)                                                                          \
  hipLaunchKernelGGL((stem_conv_fwd_kernel<NB, F>), dim3(grid), dim3(NTH), 0, stream, x, w, out, B, H, \
                     W, Ho, Wo)
  if (C == 64) { if (f16) STEM_FWD(2, true); else STEM_FWD(2, false); }
  else if (C == 32) { if (f16) STEM_FWD(1, true); else STEM_FWD(1, false); }
  else return false;
#undef STEM_FWD
  return true;
}

bool launch_stem_conv_wgrad(const uint16_t* x, const uint16_t* gy, float* part, uint16_t* dw, int B,
                            int H, int W, int Ho, int Wo, int C, int grid, int f16, hipStream_t stream) {
  if (grid <= 0) return false;
#define STEM_WG(NB, F)                                                                                \
  hipLaunchKernelGGL((stem_conv_wgrad_kernel<NB, F>), dim3(grid), dim3(NTH), 0, stream, x, gy, part, B, H, \
                     W, Ho, Wo)
  if (C == 64) { if (f16) STEM_WG(2, true); else STEM_WG(2, false); }
  else if (C == 32) { if (f16) STEM_WG(1, true); else STEM_WG(1, false); }
  else return false;
#undef STEM_WG
  const dim3 rg((unsigned)((C * 147 + 15) / 16));
  if (f16) hipLaunchKernelGGL((stem_wgrad_reduce_kernel<true>), rg, dim3(256), 0, stream, part, grid, C, dw);
  else hipLaunchKernelGGL((stem_wgrad_reduce_kernel<false>), rg, dim3(256), 0, stream, part, grid, C, dw);
  return true;
}
