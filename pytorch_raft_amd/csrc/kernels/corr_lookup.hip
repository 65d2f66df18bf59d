// Fused multi-level (2r+1)^2 bilinear window lookup on the all-pairs pyramid (forward + backward).
//
// Replaces, per GRU iteration, the reference's per-level linspace/meshgrid + `F.grid_sample`
// (align_corners=True, zero padding) + view/cat/permute/contiguous chain (`core/corr.py:29-50`,
// `core/utils/utils.py:57-71`) -- 4 levels x ~8 ATen ops each -- with one launch.
//
// Semantics: a window's taps share one fractional offset, so each thread (one query pixel, one
// level) walks the (2r+2) x (2r+2) integer neighbourhood row by row, blends horizontally once per
// row and vertically between consecutive rows.  Output channel = level*(2r+1)^2 + ix*(2r+1) + iy
// (x-offset-major, `SURVEY.md` §2.7 item 7); taps outside the plane read 0.
//
// Backward: every query pixel owns its own correlation plane in every level, so the adjoint is a
// race-free read-modify-write of that pixel's (2r+2)^2 neighbourhood (no atomics, deterministic)
// into a pyramid-gradient buffer that persists across all iterations of the step; the reference
// instead materialises and zero-fills a dense plane-sized gradient per level per iteration.
#include "common.h"
#include "launchers.h"

namespace {

struct PyrC {
  const float* lvl[4];
  int h[4];
  int w[4];
};
struct PyrG {
  float* lvl[4];
  int h[4];
  int w[4];
};

__device__ __forceinline__ float clamp_coord(float v) { return fminf(fmaxf(v, -1.0e7f), 1.0e7f); }

// Output addressing: element (b, pixel i, channel ch) at b*os.b + i*os.p + ch*os.c, so one kernel
// writes NCHW fp32 (reference layout) or NHWC bf16 straight into the fused update block's input
// buffer (channel stride 1, zero-padded pixel stride).
struct OStride {
  int64_t b, p, c;
};

template <int R, typename TO>
__global__ __launch_bounds__(64) void corr_lookup_fwd_kernel(PyrC pyr, const float* __restrict__ coords,
                                                            TO* __restrict__ out, OStride os, int B,
                                                            int H, int W, int levels) {
  // one thread per (batch, level, tap row iy, query pixel): 9x the parallelism of a
  // thread-per-pixel walk, so the scattered window reads are latency-hidden
  constexpr int D = 2 * R + 1;
  const int N = H * W;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * levels * D * N) return;
  const int i = (int)(t % N);
  int64_t rest = t / N;
  const int iy = (int)(rest % D);
  rest /= D;
  const int l = (int)(rest % levels);
  const int b = (int)(rest / levels);
  const int hl = pyr.h[l], wl = pyr.w[l];
  const float inv = 1.0f / (float)(1 << l);
  const float cx = clamp_coord(coords[((int64_t)b * 2 + 0) * N + i] * inv);
  const float cy = clamp_coord(coords[((int64_t)b * 2 + 1) * N + i] * inv);
  const float fx = floorf(cx), fy = floorf(cy);
  const float ax = cx - fx, ay = cy - fy;
  const int xs = (int)fx - R, ys = (int)fy - R;
  const float* P = pyr.lvl[l] + ((int64_t)b * N + i) * hl * wl;
  TO* O = out + b * os.b + i * os.p + (int64_t)l * D * D * os.c;

  float hr[2][D];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const int gy = ys + iy + k;
    const bool rowok = (gy >= 0) && (gy < hl);
    float v[D + 1];
#pragma unroll
    for (int xx = 0; xx <= D; ++xx) {
      const int gx = xs + xx;
      v[xx] = (rowok && gx >= 0 && gx < wl) ? P[(int64_t)gy * wl + gx] : 0.f;
    }
#pragma unroll
    for (int ix = 0; ix < D; ++ix) hr[k][ix] = (1.f - ax) * v[ix] + ax * v[ix + 1];
  }
#pragma unroll
  for (int ix = 0; ix < D; ++ix)
    St<TO>::put(O, (int64_t)(ix * D + iy) * os.c, (1.f - ay) * hr[0][ix] + ay * hr[1][ix]);
}

template <int R>
__global__ __launch_bounds__(64) void corr_lookup_bwd_kernel(PyrG g, const float* __restrict__ coords,
                                                            const float* __restrict__ dout, OStride os,
                                                            int B, int H, int W, int levels) {
  // one thread per (batch, level, integer window row yy, query pixel); each thread owns one row
  // of the pixel's private plane, so the read-modify-writes never race
  constexpr int D = 2 * R + 1;
  constexpr int E = D + 1;
  const int N = H * W;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)B * levels * E * N) return;
  const int i = (int)(t % N);
  int64_t rest = t / N;
  const int yy = (int)(rest % E);
  rest /= E;
  const int l = (int)(rest % levels);
  const int b = (int)(rest / levels);
  const int hl = g.h[l], wl = g.w[l];
  const float inv = 1.0f / (float)(1 << l);
  const float cx = clamp_coord(coords[((int64_t)b * 2 + 0) * N + i] * inv);
  const float cy = clamp_coord(coords[((int64_t)b * 2 + 1) * N + i] * inv);
  const float fx = floorf(cx), fy = floorf(cy);
  const float ax = cx - fx, ay = cy - fy;
  const int xs = (int)fx - R, ys = (int)fy - R;
  const int gy = ys + yy;
  if (gy < 0 || gy >= hl) return;
  float* G = g.lvl[l] + ((int64_t)b * N + i) * hl * wl + (int64_t)gy * wl;
  const float* dO = dout + b * os.b + i * os.p + (int64_t)l * D * D * os.c;

  // row yy collects tap row yy (weight 1-ay) and tap row yy-1 (weight ay); horizontally the
  // adjoint of x-interpolation: hs[xx] = (1-ax) d[xx] + ax d[xx-1]
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
    for (int ix = 0; ix < D; ++ix) d[ix] = dO[(int64_t)(ix * D + iy) * os.c];
#pragma unroll
    for (int xx = 0; xx < E; ++xx) {
      float s = 0.f;
      if (xx < D) s += (1.f - ax) * d[xx];
      if (xx > 0) s += ax * d[xx - 1];
      acc[xx] += wy * s;
    }
  }
#pragma unroll
  for (int xx = 0; xx < E; ++xx) {
    const int gx = xs + xx;
    if (gx >= 0 && gx < wl) G[gx] += acc[xx];
  }
}

template <typename P>
P make_pyr(float* const* lvl, const int* hs, const int* ws, int levels) {
  P p;
  for (int l = 0; l < 4; ++l) {
    p.lvl[l] = l < levels ? lvl[l] : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
  }
  return p;
}

}  // namespace

// out layout: element (b, i, ch) at b*bs + i*ps + ch*cs; out_bf16 selects bf16 storage
bool launch_corr_lookup_fwd(const float* const* lvl, const int* hs, const int* ws, int levels,
                            const float* coords, void* out, int out_bf16, int64_t bs, int64_t ps,
                            int64_t cs, int B, int H, int W, int radius, hipStream_t stream) {
  PyrC p;
  for (int l = 0; l < 4; ++l) {
    p.lvl[l] = l < levels ? lvl[l] : nullptr;
    p.h[l] = l < levels ? hs[l] : 0;
    p.w[l] = l < levels ? ws[l] : 0;
  }
  OStride os{bs, ps, cs};
  const int64_t total = (int64_t)B * levels * (2 * radius + 1) * H * W;
  dim3 grid(raft_cdiv(total, 64));
#define LK(R, T) hipLaunchKernelGGL((corr_lookup_fwd_kernel<R, T>), grid, dim3(64), 0, stream, p, coords, (T*)out, os, B, H, W, levels)
  if (radius == 3) { if (out_bf16) LK(3, uint16_t); else LK(3, float); return true; }
  if (radius == 4) { if (out_bf16) LK(4, uint16_t); else LK(4, float); return true; }
#undef LK
  return false;
}

bool launch_corr_lookup_bwd(float* const* glvl, const int* hs, const int* ws, int levels,
                            const float* coords, const float* dout, int64_t bs, int64_t ps,
                            int64_t cs, int B, int H, int W, int radius, hipStream_t stream) {
  PyrG p = make_pyr<PyrG>(glvl, hs, ws, levels);
  OStride os{bs, ps, cs};
  const int64_t total = (int64_t)B * levels * (2 * radius + 2) * H * W;
  dim3 grid(raft_cdiv(total, 64));
  switch (radius) {
    case 3: hipLaunchKernelGGL(corr_lookup_bwd_kernel<3>, grid, dim3(64), 0, stream, p, coords, dout, os, B, H, W, levels); return true;
    case 4: hipLaunchKernelGGL(corr_lookup_bwd_kernel<4>, grid, dim3(64), 0, stream, p, coords, dout, os, B, H, W, levels); return true;
    default: return false;
  }
}
