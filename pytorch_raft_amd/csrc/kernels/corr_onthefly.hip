// On-the-fly ("alternate") correlation lookup, forward + backward, O(HW * r^2) memory.
//
// Capability parity with `alt_cuda_corr` (`alt_cuda_corr/correlation_kernel.cu:18-119` forward,
// `:122-256` backward) and `AlternateCorrBlock` (`core/corr.py:63-91`), re-designed for wave64:
//
// * one wave per query pixel; its fmap1 row (C channels) lives in registers, C/64 channels per lane,
//   so every fmap2 row read is one coalesced 512 B / 1 KiB wave access (the reference stages
//   32-channel slices through LDS from a 32-thread block, i.e. half a wave on CDNA);
// * the (2r+2)^2 integer-position dot products are finished with a 64-way reduce-scatter across the
//   lanes (63 shuffles per 64 positions instead of 6 per position), after which lane p owns
//   position p and the (2r+1)^2 bilinear taps are blended from LDS;
// * output is written channels-last (B, H, W, L*(2r+1)^2) so each pixel's taps are contiguous; the
//   Python side returns it as an NCHW-shaped channels_last tensor;
// * explicit bounds on every coordinate (the reference backward reads coords out of range when
//   H % 4 or W % 8 != 0) and no reliance on lock-step execution for LDS hand-offs;
// * the backward is wired into autograd (the reference's is unreachable): d(fmap1) per wave in
//   registers, d(fmap2 level) via float atomics into a buffer that persists across iterations.
#include "common.h"
#include "launchers.h"

namespace {

struct F2Lvls {
  const float* lvl[4];
  int h[4];
  int w[4];
};
struct G2Lvls {
  float* lvl[4];
  int h[4];
  int w[4];
};

__device__ __forceinline__ float clampc(float v) { return fminf(fmaxf(v, -1.0e7f), 1.0e7f); }

// v[0..63] per lane -> lane L returns sum over lanes of v[L]
__device__ __forceinline__ float reduce_scatter64(float (&v)[64], int lane) {
#pragma unroll
  for (int s = 32; s >= 1; s >>= 1) {
    const bool up = (lane & s) != 0;
#pragma unroll
    for (int j = 0; j < s; ++j) {
      const float send = up ? v[j] : v[j + s];
      const float keep = up ? v[j + s] : v[j];
      v[j] = keep + __shfl_xor(send, s, 64);
    }
  }
  return v[0];
}

template <int R, int CPL>
__global__ __launch_bounds__(256) void corr_otf_fwd_kernel(const float* __restrict__ f1, F2Lvls f2,
                                                           const float* __restrict__ coords,
                                                           float* __restrict__ out, int B, int H,
                                                           int W, int levels, float inv_sqrt_c) {
  constexpr int D = 2 * R + 1;
  constexpr int E = D + 1;       // integer positions per axis
  constexpr int NP = E * E;      // <= 100
  constexpr int NB = (NP + 63) / 64;
  constexpr int C = CPL * 64;
  __shared__ float dots[4][NB * 64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int N = H * W;
  const int64_t pix = (int64_t)blockIdx.x * 4 + wv;
  const bool active = pix < (int64_t)B * N;
  const int b = active ? (int)(pix / N) : 0;
  const int i = active ? (int)(pix % N) : 0;

  float a[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) a[c] = active ? f1[((int64_t)b * N + i) * C + lane * CPL + c] : 0.f;
  const float x = active ? coords[((int64_t)b * 2) * N + i] : 0.f;
  const float y = active ? coords[((int64_t)b * 2 + 1) * N + i] : 0.f;
  const int ctot = levels * D * D;
  float* O = out + pix * ctot;

  for (int l = 0; l < levels; ++l) {
    const float inv = 1.f / (float)(1 << l);
    const float cx = clampc(x * inv), cy = clampc(y * inv);
    const float fx = floorf(cx), fy = floorf(cy);
    const float ax = cx - fx, ay = cy - fy;
    const int xs = (int)fx - R, ys = (int)fy - R;
    const int hl = f2.h[l], wl = f2.w[l];
    const float* F2 = f2.lvl[l] + (int64_t)b * hl * wl * C;
#pragma unroll
    for (int pb = 0; pb < NB; ++pb) {
      float v[64];
#pragma unroll
      for (int j = 0; j < 64; ++j) {
        const int p = pb * 64 + j;
        const int px = xs + p % E, py = ys + p / E;
        float s = 0.f;
        if (p < NP && px >= 0 && px < wl && py >= 0 && py < hl) {
          const float* row = F2 + ((int64_t)py * wl + px) * C + lane * CPL;
#pragma unroll
          for (int c = 0; c < CPL; ++c) s += a[c] * row[c];
        }
        v[j] = s;
      }
      dots[wv][pb * 64 + lane] = reduce_scatter64(v, lane);
    }
    __syncthreads();
    for (int t = lane; t < D * D; t += 64) {
      const int ix = t / D, iy = t % D;
      const float* d0 = &dots[wv][iy * E + ix];
      const float* d1 = d0 + E;
      const float val = (1.f - ay) * ((1.f - ax) * d0[0] + ax * d0[1]) +
                        ay * ((1.f - ax) * d1[0] + ax * d1[1]);
      if (active) O[l * D * D + t] = val * inv_sqrt_c;
    }
    __syncthreads();
  }
}

template <int R, int CPL>
__global__ __launch_bounds__(256) void corr_otf_bwd_kernel(const float* __restrict__ f1, F2Lvls f2,
                                                           const float* __restrict__ coords,
                                                           const float* __restrict__ dout,
                                                           float* __restrict__ df1, G2Lvls df2,
                                                           int B, int H, int W, int levels,
                                                           float inv_sqrt_c) {
  constexpr int D = 2 * R + 1;
  constexpr int E = D + 1;
  constexpr int NP = E * E;
  constexpr int C = CPL * 64;
  __shared__ float gpos[4][128];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int N = H * W;
  const int64_t pix = (int64_t)blockIdx.x * 4 + wv;
  const bool active = pix < (int64_t)B * N;
  const int b = active ? (int)(pix / N) : 0;
  const int i = active ? (int)(pix % N) : 0;

  float a[CPL], ga[CPL];
#pragma unroll
  for (int c = 0; c < CPL; ++c) {
    a[c] = active ? f1[((int64_t)b * N + i) * C + lane * CPL + c] : 0.f;
    ga[c] = 0.f;
  }
  const float x = active ? coords[((int64_t)b * 2) * N + i] : 0.f;
  const float y = active ? coords[((int64_t)b * 2 + 1) * N + i] : 0.f;
  const int ctot = levels * D * D;
  const float* dO = dout + pix * ctot;

  for (int l = 0; l < levels; ++l) {
    const float inv = 1.f / (float)(1 << l);
    const float cx = clampc(x * inv), cy = clampc(y * inv);
    const float fx = floorf(cx), fy = floorf(cy);
    const float ax = cx - fx, ay = cy - fy;
    const int xs = (int)fx - R, ys = (int)fy - R;
    const int hl = f2.h[l], wl = f2.w[l];
    // adjoint of the bilinear blend: position (px_i, py_i) collects from up to 4 taps
    for (int p = lane; p < 128; p += 64) {
      float g = 0.f;
      if (p < NP && active) {
        const int qx = p % E, qy = p / E;
#pragma unroll
        for (int dyi = 0; dyi < 2; ++dyi)
#pragma unroll
          for (int dxi = 0; dxi < 2; ++dxi) {
            const int ix = qx - dxi, iy = qy - dyi;
            if (ix >= 0 && ix < D && iy >= 0 && iy < D) {
              const float wx = dxi ? ax : 1.f - ax;
              const float wy = dyi ? ay : 1.f - ay;
              g += wx * wy * dO[l * D * D + ix * D + iy];
            }
          }
      }
      gpos[wv][p] = g * inv_sqrt_c;
    }
    __syncthreads();
    const float* F2 = f2.lvl[l] + (int64_t)b * hl * wl * C;
    float* G2 = df2.lvl[l] + (int64_t)b * hl * wl * C;
    for (int p = 0; p < NP; ++p) {
      const float g = gpos[wv][p];
      const int px = xs + p % E, py = ys + p / E;
      if (g != 0.f && px >= 0 && px < wl && py >= 0 && py < hl) {
        const int64_t off = ((int64_t)py * wl + px) * C + lane * CPL;
#pragma unroll
        for (int c = 0; c < CPL; ++c) {
          ga[c] += g * F2[off + c];
          atomicAdd(&G2[off + c], g * a[c]);
        }
      }
    }
    __syncthreads();
  }
  if (active) {
#pragma unroll
    for (int c = 0; c < CPL; ++c) df1[((int64_t)b * N + i) * C + lane * CPL + c] += ga[c];
  }
}

template <typename P, typename T>
P make_lvls(T* const* lvl, const int* hs, const int* ws, int levels) {
  P p;
  for (int l = 0; l < 4; ++l) {
    p.lvl[l] = l < levels ? lvl[l] : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
  }
  return p;
}

}  // namespace

#define OTF_DISPATCH(KERNEL, ...)                                                             \
  do {                                                                                        \
    if (radius == 4 && C == 256) { hipLaunchKernelGGL((KERNEL<4, 4>), __VA_ARGS__); return true; } \
    if (radius == 3 && C == 128) { hipLaunchKernelGGL((KERNEL<3, 2>), __VA_ARGS__); return true; } \
    if (radius == 4 && C == 128) { hipLaunchKernelGGL((KERNEL<4, 2>), __VA_ARGS__); return true; } \
    if (radius == 3 && C == 256) { hipLaunchKernelGGL((KERNEL<3, 4>), __VA_ARGS__); return true; } \
    return false;                                                                             \
  } while (0)

bool launch_corr_otf_fwd(const float* f1, const float* const* f2lvl, const int* hs, const int* ws,
                         int levels, const float* coords, float* out, int B, int C, int H, int W,
                         int radius, hipStream_t stream) {
  F2Lvls p = make_lvls<F2Lvls>(f2lvl, hs, ws, levels);
  dim3 grid(raft_cdiv((int64_t)B * H * W, 4));
  const float isc = 1.f / sqrtf((float)C);
  OTF_DISPATCH(corr_otf_fwd_kernel, grid, dim3(256), 0, stream, f1, p, coords, out, B, H, W, levels, isc);
}

bool launch_corr_otf_bwd(const float* f1, const float* const* f2lvl, const int* hs, const int* ws,
                         int levels, const float* coords, const float* dout, float* df1,
                         float* const* df2lvl, int B, int C, int H, int W, int radius,
                         hipStream_t stream) {
  F2Lvls p = make_lvls<F2Lvls>(f2lvl, hs, ws, levels);
  G2Lvls g = make_lvls<G2Lvls>(df2lvl, hs, ws, levels);
  dim3 grid(raft_cdiv((int64_t)B * H * W, 4));
  const float isc = 1.f / sqrtf((float)C);
  OTF_DISPATCH(corr_otf_bwd_kernel, grid, dim3(256), 0, stream, f1, p, coords, dout, df1, g, B, H, W, levels, isc);
}
