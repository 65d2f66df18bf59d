// Fused NHWC normalisation + activation for the RAFT encoders (fnet: InstanceNorm, cnet: BatchNorm).
//
// Reference: `core/extractor.py:6-56,118-192` -- conv -> norm -> ReLU, residual add -> ReLU, run as
// NCHW PyTorch ops under autocast.  On ROCm that is MIOpen convs bracketed by NCHW<->NHWC transposes,
// InstanceNorm lowered to batch_norm on a (1, N*C, H, W) view, separate ReLU / add kernels and an
// ATen reduction per conv for the bias gradient.  Here the encoders run channels-last (MIOpen NHWC
// convs, no transposes) and every norm is four memory passes of bf16 NHWC data:
//
//   stats     per (image, channel) [instance] or per channel [batch] shifted sums  sum(x-K),
//             sum((x-K)^2) -> per-workgroup partials (deterministic, no atomics)
//   finalize  partials reduced (same launch) -> mean / invstd, the affine fold into one scale/shift per (image, channel),
//             BatchNorm running-stat update; the conv bias is folded here too (it cancels in a
//             training-mode norm, and shifts the eval-mode one), so the conv runs without bias
//   apply     y = act(x * scale + shift) [+ residual, ReLU]     (16-B vectors, 8 channels/thread)
//   backward  partial sums of g, g*xhat, xhat (g = dy masked by the ReLU, the mask recomputed from
//             x -- y is never read back) -> reduce + finalize (one launch) -> one pass
//             dx = A*g + B*xhat + C, whose first workgroup also sums the parameter gradients over
//             the groups.  The conv-bias gradient falls out of the same sums.
//
// Channel counts are multiples of 8 up to 256; a thread owns one 16-B channel group of a pixel.
#include "common.h"
#include "launchers.h"

#include <cstdlib>

namespace {

constexpr int NT = 256;

// f16 arguments of the launchers: the storage type TY below (0 bf16, 1 fp16, 2 fp32)
// 8 channels of one pixel in the storage type TY: 0 bf16, 1 fp16 (fp16 autocast), 2 fp32 (the
// fp32 schedule); element offsets, 16-B (32-B for fp32) aligned groups of 8
template <int TY> struct V8 { uint4 r; };
template <> struct V8<2> { uint4 a, b; };

template <int TY>
__device__ __forceinline__ V8<TY> ld8(const uint16_t* p, int64_t off) {
  V8<TY> v;
  if constexpr (TY == 2) {
    const uint4* q = reinterpret_cast<const uint4*>(reinterpret_cast<const float*>(p) + off);
    v.a = q[0];
    v.b = q[1];
  } else {
    v.r = *reinterpret_cast<const uint4*>(p + off);
  }
  return v;
}
template <int TY>
__device__ __forceinline__ void st8(uint16_t* p, int64_t off, const V8<TY>& v) {
  if constexpr (TY == 2) {
    uint4* q = reinterpret_cast<uint4*>(reinterpret_cast<float*>(p) + off);
    q[0] = v.a;
    q[1] = v.b;
  } else {
    *reinterpret_cast<uint4*>(p + off) = v.r;
  }
}
template <int TY>
__device__ __forceinline__ float ld1(const uint16_t* p, int64_t off) {
  if constexpr (TY == 2) return reinterpret_cast<const float*>(p)[off];
  else return raft_h2f<TY == 1>(p[off]);
}
template <int TY>
__device__ __forceinline__ void unpack8(const V8<TY>& v, float (&f)[8]) {
  if constexpr (TY == 2) {
    const uint32_t w[8] = {v.a.x, v.a.y, v.a.z, v.a.w, v.b.x, v.b.y, v.b.z, v.b.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) f[i] = __uint_as_float(w[i]);
  } else {
    const uint32_t w[4] = {v.r.x, v.r.y, v.r.z, v.r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if constexpr (TY == 1) {
        f[2 * i] = raft_h2f<true>((uint16_t)(w[i] & 0xffffu));
        f[2 * i + 1] = raft_h2f<true>((uint16_t)(w[i] >> 16));
      } else {
        f[2 * i] = __uint_as_float(w[i] << 16);
        f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
      }
    }
  }
}
template <int TY>
__device__ __forceinline__ V8<TY> pack8(const float (&f)[8]) {
  V8<TY> v;
  if constexpr (TY == 2) {
    v.a = make_uint4(__float_as_uint(f[0]), __float_as_uint(f[1]), __float_as_uint(f[2]), __float_as_uint(f[3]));
    v.b = make_uint4(__float_as_uint(f[4]), __float_as_uint(f[5]), __float_as_uint(f[6]), __float_as_uint(f[7]));
  } else {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
      w[i] = (uint32_t)raft_f2h<TY == 1>(f[2 * i]) | ((uint32_t)raft_f2h<TY == 1>(f[2 * i + 1]) << 16);
    v.r = make_uint4(w[0], w[1], w[2], w[3]);
  }
  return v;
}

// 16-bit value > 0 per half of a packed word: sign bit clear and magnitude non-zero (bf16 and
// fp16 alike)
__device__ __forceinline__ uint32_t pos_mask(uint32_t w) {
  const uint32_t lo = ((w & 0x8000u) == 0 && (w & 0x7fffu) != 0) ? 0xffffu : 0u;
  const uint32_t hi = ((w & 0x80000000u) == 0 && (w & 0x7fff0000u) != 0) ? 0xffff0000u : 0u;
  return lo | hi;
}
// d where o > 0, else 0 (the ReLU backward on the stored forward output o)
template <int TY>
__device__ __forceinline__ V8<TY> mask_pos(const V8<TY>& d, const V8<TY>& o) {
  V8<TY> r;
  if constexpr (TY == 2) {
    auto m = [](uint32_t dv, uint32_t ov) { return __uint_as_float(ov) > 0.f ? dv : 0u; };
    r.a = make_uint4(m(d.a.x, o.a.x), m(d.a.y, o.a.y), m(d.a.z, o.a.z), m(d.a.w, o.a.w));
    r.b = make_uint4(m(d.b.x, o.b.x), m(d.b.y, o.b.y), m(d.b.z, o.b.z), m(d.b.w, o.b.w));
  } else {
    r.r = make_uint4(d.r.x & pos_mask(o.r.x), d.r.y & pos_mask(o.r.y), d.r.z & pos_mask(o.r.z),
                     d.r.w & pos_mask(o.r.w));
  }
  return r;
}

// fp32 schedule: the 8 values of channel group g of pixel pix also as the split-bf16 operand of
// the consuming conv ([hi | lo] halves of a (P, 2 spad) bf16 buffer, ops/conv_fp32.py's
// split_hilo layout); the pixel's last group also zeroes the padding channels [C, spad) of both
// halves
__device__ __forceinline__ void store_split8(uint16_t* __restrict__ s, int spad, int64_t pix, int g,
                                             int cg, const float (&f)[8]) {
  uint32_t wh[4], wl[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const uint16_t h0 = raft_f32_to_bf16(f[2 * k]), h1 = raft_f32_to_bf16(f[2 * k + 1]);
    const uint16_t l0 = raft_f32_to_bf16(f[2 * k] - raft_bf16_to_f32(h0));
    const uint16_t l1 = raft_f32_to_bf16(f[2 * k + 1] - raft_bf16_to_f32(h1));
    wh[k] = (uint32_t)h0 | ((uint32_t)h1 << 16);
    wl[k] = (uint32_t)l0 | ((uint32_t)l1 << 16);
  }
  uint16_t* o = s + pix * 2 * spad + g * 8;
  *reinterpret_cast<uint4*>(o) = make_uint4(wh[0], wh[1], wh[2], wh[3]);
  *reinterpret_cast<uint4*>(o + spad) = make_uint4(wl[0], wl[1], wl[2], wl[3]);
  if (g == cg - 1)
    for (int c = cg * 8; c < spad; c += 8) {
      *reinterpret_cast<uint4*>(s + pix * 2 * spad + c) = make_uint4(0, 0, 0, 0);
      *reinterpret_cast<uint4*>(s + pix * 2 * spad + spad + c) = make_uint4(0, 0, 0, 0);
    }
}

// The forward's per-(group, channel) affine of the normalised value, evaluated with exactly the
// float expressions of norm_finalize_kernel (so a backward ReLU mask recomputed from x matches the
// forward's y > 0 without reading y).
__device__ __forceinline__ void norm_affine(int mode, const float* __restrict__ gamma,
                                            const float* __restrict__ beta, int c, float mean,
                                            float invstd, float& sc, float& sh) {
  const float gm = (mode == 1 || mode == 2) && gamma ? gamma[c] : 1.f;
  const float bt = (mode == 1 || mode == 2) && beta ? beta[c] : 0.f;
  sc = gm * invstd;
  sh = bt - mean * gm * invstd;
}

// grid.x = blocks per group-range, grid.y = image (instance) or 1 (batch: range = all images)
// partial layout [group_img][blk][2][C]
template <int TY>
__global__ __launch_bounds__(NT) void norm_stats_kernel(const uint16_t* __restrict__ x, int HW,
                                                        int C, int per_image, int pix_per_blk,
                                                        int total_pix, float* __restrict__ part) {
  __shared__ float red[2][NT * 8];
  const int cg = C / 8;
  const int lanes = NT / cg;
  const int tid = threadIdx.x;
  const int g = tid % cg, pl = tid / cg;
  const int img = blockIdx.y;
  const int64_t base = per_image ? (int64_t)img * HW : 0;
  const int range = per_image ? HW : total_pix;
  const int p0 = blockIdx.x * pix_per_blk, p1 = min(range, p0 + pix_per_blk);
  // shift: the group's first pixel (keeps the one-pass variance well conditioned)
  float K[8];
  unpack8<TY>(ld8<TY>(x, base * C + g * 8), K);
  float s1[8], s2[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s1[i] = s2[i] = 0.f;
  if (pl < lanes) {
    // 4 pixels per round with all four 16-B loads issued first: one outstanding load per
    // thread left this pass latency-bound at ~3 TB/s
    int p = p0 + pl;
    for (; p + 7 * lanes < p1; p += 8 * lanes) {
      V8<TY> raw[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) raw[u] = ld8<TY>(x, (base + p + u * lanes) * C + g * 8);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        float v[8];
        unpack8<TY>(raw[u], v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const float d = v[i] - K[i];
          s1[i] += d;
          s2[i] += d * d;
        }
      }
    }
    for (; p < p1; p += lanes) {
      float v[8];
      unpack8<TY>(ld8<TY>(x, (base + p) * C + g * 8), v);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = v[i] - K[i];
        s1[i] += d;
        s2[i] += d * d;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[0][tid * 8 + i] = s1[i];
    red[1][tid * 8 + i] = s2[i];
  }
  __syncthreads();
  // block combine: Q = NT / C threads per channel each sum every Q-th lane row, then one
  // thread per channel adds the Q partials (fixed order: deterministic)
  {
    __shared__ float red2[2][NT];
    const int Q = NT / C;
    const int c = tid % C, q = tid / C;
    float a = 0.f, b = 0.f;
    if (q < Q) {
      const int gg = c / 8, ii = c % 8;
      for (int l = q; l < lanes; l += Q) {
        a += red[0][(l * cg + gg) * 8 + ii];
        b += red[1][(l * cg + gg) * 8 + ii];
      }
      red2[0][q * C + c] = a;
      red2[1][q * C + c] = b;
    }
    __syncthreads();
    if (tid < C) {
      float sa = 0.f, sb = 0.f;
      for (int k = 0; k < Q; ++k) {
        sa += red2[0][k * C + tid];
        sb += red2[1][k * C + tid];
      }
      float* dst = part + ((int64_t)img * gridDim.x + blockIdx.x) * 2 * C;
      dst[tid] = sa;
      dst[C + tid] = sb;
    }
  }
}

// mode: 0 instance (train or eval: always batch statistics), 1 batch-train, 2 batch-eval, 3 none
// one thread per (group image, channel); the training-statistics modes run
// norm_reduce_finalize_kernel instead
template <int TY>
__global__ void norm_finalize_kernel(const float* __restrict__ part, const uint16_t* __restrict__ x,
                                     int HW, int C, int groups_img, int nblk, int cnt, int mode,
                                     const float* __restrict__ gamma, const float* __restrict__ beta,
                                     const float* __restrict__ cbias, float* __restrict__ rmean,
                                     float* __restrict__ rvar, float momentum, float eps,
                                     float* __restrict__ mean_out, float* __restrict__ invstd_out,
                                     float* __restrict__ scale, float* __restrict__ shift, int nimg) {
  const int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= groups_img * C) return;
  const int gi = idx / C, c = idx % C;
  const float b = cbias ? cbias[c] : 0.f;
  float mean = 0.f, invstd = 1.f;
  if (mode == 0 || mode == 1) {
    const double a = part[(int64_t)gi * 2 * C + c], q = part[(int64_t)gi * 2 * C + C + c];
    const float K = ld1<TY>(x, (int64_t)(mode == 0 ? gi : 0) * HW * C + c);
    const double m = a / cnt;
    double var = q / cnt - m * m;
    if (var < 0.0) var = 0.0;
    mean = (float)(m + K);
    invstd = (float)(1.0 / sqrt(var + (double)eps));
    if (mode == 1 && rmean != nullptr) {
      const double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
      rmean[c] = (1.f - momentum) * rmean[c] + momentum * (mean + b);
      rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
    }
  } else if (mode == 2) {
    mean = rmean[c] - b;  // (x + b - rm) = (x - (rm - b))
    invstd = 1.f / sqrtf(rvar[c] + eps);
  } else {
    mean = -b;  // y = x + b
    invstd = 1.f;
  }
  const float gm = (mode == 1 || mode == 2) && gamma ? gamma[c] : 1.f;
  const float bt = (mode == 1 || mode == 2) && beta ? beta[c] : 0.f;
  mean_out[idx] = mean;
  invstd_out[idx] = invstd;
  // per-image scale/shift table [nimg][C] (instance: its own group; batch/none: shared)
  for (int n = (mode == 0 ? gi : 0); n < (mode == 0 ? gi + 1 : nimg); ++n) {
    scale[(int64_t)n * C + c] = gm * invstd;
    shift[(int64_t)n * C + c] = bt - mean * gm * invstd;
  }
}

// Partial reduce + finalize of the training statistics in ONE launch: block = COLS channels x
// LANES lanes of one group (grid (groups, ceil(C / COLS))); the lanes stride over the group's
// per-workgroup partials, a fixed-order LDS combine (deterministic), then lane 0 finalizes its
// (group, channel).  64 lanes for the long batch-norm partial lists (4 channels per block: 8.3 ->
// 5.6 us per call vs 16 lanes' 4 blocks of 256 threads for a 64-channel batch norm; the backward
// finalize keeps 16 lanes: 64 gave 14.8 vs 9.2 us, 32 gave 7.8 / 9.0 vs 8.6 us on two boxes --
// noise, profiles/r6/norm_wg/, profiles/r6/final8/), 4 for per-image ones.
// TILED: the partials are a producing conv's per-tile rows [4][C] -- sum (x - K_t), sum
// (x - K_t)^2, K_t, count (conv_enc64.hip) -- re-shifted to the group's first tile's K in double
// (sum (x - K) = s1 + n d, sum (x - K)^2 = s2 + 2 d s1 + n d^2 with d = K_t - K), so the norm runs
// no statistics pass of its own
template <int LANES, int TY, bool TILED = false>
__global__ __launch_bounds__(256) void norm_reduce_finalize_kernel(
    const float* __restrict__ part, int nblk, const uint16_t* __restrict__ x, int HW, int C,
    int cnt, int mode, const float* __restrict__ gamma, const float* __restrict__ beta,
    const float* __restrict__ cbias, float* __restrict__ rmean, float* __restrict__ rvar,
    float momentum, float eps, float* __restrict__ mean_out, float* __restrict__ invstd_out,
    float* __restrict__ scale, float* __restrict__ shift, int nimg) {
  constexpr int COLS = 256 / LANES;
  __shared__ float red[2][LANES][COLS];
  const int gi = blockIdx.x;
  const int t = threadIdx.x % COLS, lane = threadIdx.x / COLS;
  const int c = blockIdx.y * COLS + t;
  const int SC = (TILED ? 4 : 2) * C;
  float a = 0.f, q = 0.f;
  float K0 = 0.f;
  if (c < C) {
    if constexpr (TILED) {
      K0 = part[(int64_t)gi * nblk * SC + 2 * C + c];
      double ad = 0.0, qd = 0.0;
      for (int k = lane; k < nblk; k += LANES) {
        const float* pk = part + ((int64_t)gi * nblk + k) * SC;
        const double s1 = pk[c], s2 = pk[C + c], n = pk[3 * C + c];
        const double d = (double)pk[2 * C + c] - (double)K0;
        ad += s1 + n * d;
        qd += s2 + 2.0 * d * s1 + n * d * d;
      }
      a = (float)ad;
      q = (float)qd;
    } else {
      for (int k = lane; k < nblk; k += LANES) {
        const float* pk = part + ((int64_t)gi * nblk + k) * SC;
        a += pk[c];
        q += pk[C + c];
      }
    }
  }
  red[0][lane][t] = a;
  red[1][lane][t] = q;
  __syncthreads();
  if (lane != 0 || c >= C) return;
  float sa = 0.f, sq = 0.f;
#pragma unroll
  for (int l = 0; l < LANES; ++l) {
    sa += red[0][l][t];
    sq += red[1][l][t];
  }
  const float b = cbias ? cbias[c] : 0.f;
  const double m = (double)sa / cnt;
  double var = (double)sq / cnt - m * m;
  if (var < 0.0) var = 0.0;
  const float K = TILED ? K0 : ld1<TY>(x, (int64_t)(mode == 0 ? gi : 0) * HW * C + c);
  const float mean = (float)(m + K);
  const float invstd = (float)(1.0 / sqrt(var + (double)eps));
  if (mode == 1 && rmean != nullptr) {
    const double unb = cnt > 1 ? var * cnt / (cnt - 1) : var;
    rmean[c] = (1.f - momentum) * rmean[c] + momentum * (mean + b);
    rvar[c] = (1.f - momentum) * rvar[c] + momentum * (float)unb;
  }
  const float gm = mode == 1 && gamma ? gamma[c] : 1.f;
  const float bt = mode == 1 && beta ? beta[c] : 0.f;
  const int idx = gi * C + c;
  mean_out[idx] = mean;
  invstd_out[idx] = invstd;
  for (int n = (mode == 0 ? gi : 0); n < (mode == 0 ? gi + 1 : nimg); ++n) {
    scale[(int64_t)n * C + c] = gm * invstd;
    shift[(int64_t)n * C + c] = bt - mean * gm * invstd;
  }
}

// y = act(x*scale + shift) [+ res -> relu];  act: relu when relu != 0.  Block size is a multiple
// of the channel-group count: each thread keeps one channel group and reloads its scale / shift
// only when the image changes.
template <int TY>
__global__ __launch_bounds__(NT) void norm_apply_kernel(const uint16_t* __restrict__ x,
                                                        const float* __restrict__ scale,
                                                        const float* __restrict__ shift, int HW,
                                                        int C, int64_t nvec, int relu,
                                                        const uint16_t* __restrict__ res,
                                                        uint16_t* __restrict__ y,
                                                        uint16_t* __restrict__ ys, int spad) {
  const int cg = C / 8;
  const int64_t step = (int64_t)gridDim.x * blockDim.x;
  int cur = -1;
  float sc[8], sh[8];
  for (int64_t v = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; v < nvec; v += step) {
    const int64_t pix = v / cg;
    const int g = (int)(v - pix * cg);
    const int n = (int)(pix / HW);
    if (n != cur) {
      cur = n;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        sc[i] = scale[(int64_t)n * C + g * 8 + i];
        sh[i] = shift[(int64_t)n * C + g * 8 + i];
      }
    }
    float f[8];
    unpack8<TY>(ld8<TY>(x, v * 8), f);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      f[i] = f[i] * sc[i] + sh[i];
      if (relu) f[i] = fmaxf(f[i], 0.f);
    }
    if (res) {
      float r[8];
      unpack8<TY>(ld8<TY>(res, v * 8), r);
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = fmaxf(f[i] + r[i], 0.f);
    }
    st8<TY>(y, v * 8, pack8<TY>(f));
    if (ys != nullptr) store_split8(ys, spad, pix, g, cg, f);
  }
}

// out = relu(a + b)
template <int TY>
__global__ __launch_bounds__(NT) void add_relu_kernel(const uint16_t* __restrict__ a,
                                                      const uint16_t* __restrict__ b,
                                                      uint16_t* __restrict__ out, int64_t nvec) {
  for (int64_t v = blockIdx.x * (int64_t)NT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * NT) {
    float fa[8], fb[8];
    unpack8<TY>(ld8<TY>(a, v * 8), fa);
    unpack8<TY>(ld8<TY>(b, v * 8), fb);
#pragma unroll
    for (int i = 0; i < 8; ++i) fa[i] = fmaxf(fa[i] + fb[i], 0.f);
    st8<TY>(out, v * 8, pack8<TY>(fa));
  }
}

// g = (dy [+ dy2]) * [y > 0]   (the ReLU backward, also the block-end residual ReLU)
template <int TY>
__global__ __launch_bounds__(NT) void relu_mask_kernel(const uint16_t* __restrict__ dy,
                                                       const uint16_t* __restrict__ dy2,
                                                       const uint16_t* __restrict__ y,
                                                       uint16_t* __restrict__ g, int64_t nvec) {
  for (int64_t v = blockIdx.x * (int64_t)NT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * NT) {
    V8<TY> d = ld8<TY>(dy, v * 8);
    if (dy2 != nullptr) {
      // g = (dy + dy2) * [y > 0]: the residual-branch gradient folded in (no separate add pass)
      float a[8], b[8];
      unpack8<TY>(d, a);
      unpack8<TY>(ld8<TY>(dy2, v * 8), b);
#pragma unroll
      for (int i = 0; i < 8; ++i) a[i] += b[i];
      d = pack8<TY>(a);
    }
    st8<TY>(g, v * 8, mask_pos<TY>(d, ld8<TY>(y, v * 8)));
  }
}

// The block-end ReLU of a residual block (out = relu(branch + res)) folded into the norm
// backward's statistics pass: g = (dy [+ dy2]) * [out > 0] is formed on load, written once (it
// is also the residual's gradient and the apply pass's input) and summed -- the separate
// relu_mask pass and its re-read of g are gone.
template <int TY>
__device__ __forceinline__ V8<TY> block_end_grad(V8<TY> d, const uint16_t* dy2, int64_t off, const V8<TY>& o) {
  if (dy2 != nullptr) {
    float a[8], b[8];
    unpack8<TY>(d, a);
    unpack8<TY>(ld8<TY>(dy2, off), b);
#pragma unroll
    for (int i = 0; i < 8; ++i) a[i] += b[i];
    d = pack8<TY>(a);
  }
  return mask_pos<TY>(d, o);
}

// backward partial sums per (group image, blk): sum g, sum g*xhat, sum xhat;
// g = dy * [y > 0] when relu; xhat = (x - mean) * invstd.  yres != null: dy is the block output's
// gradient, g0 = (dy [+ dy2]) * [yres > 0] is formed first and stored to gout (see above)
template <int TY>
__global__ __launch_bounds__(NT) void norm_bwd_stats_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma, const float* __restrict__ beta,
    int mode, int HW, int C, int per_image, int pix_per_blk, int total_pix, int relu,
    float* __restrict__ part, const uint16_t* __restrict__ dy2, const uint16_t* __restrict__ yres,
    uint16_t* __restrict__ gout) {
  __shared__ float red[3][NT * 8];
  const int cg = C / 8;
  const int lanes = NT / cg;
  const int tid = threadIdx.x;
  const int g = tid % cg, pl = tid / cg;
  const int img = blockIdx.y;
  const int64_t base = per_image ? (int64_t)img * HW : 0;
  const int range = per_image ? HW : total_pix;
  const int p0 = blockIdx.x * pix_per_blk, p1 = min(range, p0 + pix_per_blk);
  float mu[8], is[8], sc[8], sh[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int c = g * 8 + i;
    mu[i] = mean[(int64_t)(per_image ? img : 0) * C + c];
    is[i] = invstd[(int64_t)(per_image ? img : 0) * C + c];
    norm_affine(mode, gamma, beta, c, mu[i], is[i], sc[i], sh[i]);
  }
  float sg[8], sgx[8], sx[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) sg[i] = sgx[i] = sx[i] = 0.f;
  auto accum = [&](const V8<TY>& rd, const V8<TY>& rx) {
    float d[8], xv[8];
    unpack8<TY>(rd, d);
    unpack8<TY>(rx, xv);
    if (relu) {
      // the forward ReLU mask, recomputed from x with the forward's own scale / shift
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = xv[i] * sc[i] + sh[i] > 0.f ? d[i] : 0.f;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float xh = (xv[i] - mu[i]) * is[i];
      sg[i] += d[i];
      sgx[i] += d[i] * xh;
      sx[i] += xh;
    }
  };
  if (pl < lanes) {
    int p = p0 + pl;
    if (yres != nullptr) {
      // block-end ReLU: 4 pixels' dy, x, yres [, dy2] loads in flight per round, all issued
      // before any math (8 pixels x 4 streams would hold ~190 VGPRs: 2 waves per SIMD)
      for (; p + 3 * lanes < p1; p += 4 * lanes) {
        V8<TY> rd[4], rx[4], ry[4], r2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t off = (base + p + u * lanes) * C + g * 8;
          rd[u] = ld8<TY>(dy, off);
          rx[u] = ld8<TY>(x, off);
          ry[u] = ld8<TY>(yres, off);
          if (dy2 != nullptr) r2[u] = ld8<TY>(dy2, off);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int64_t off = (base + p + u * lanes) * C + g * 8;
          if (dy2 != nullptr) {
            float a[8], b[8];
            unpack8<TY>(rd[u], a);
            unpack8<TY>(r2[u], b);
#pragma unroll
            for (int i = 0; i < 8; ++i) a[i] += b[i];
            rd[u] = pack8<TY>(a);
          }
          rd[u] = mask_pos<TY>(rd[u], ry[u]);
          st8<TY>(gout, off, rd[u]);
          accum(rd[u], rx[u]);
        }
      }
    }
    // 8 pixels (16 loads) in flight per round (see norm_stats_kernel)
    for (; yres == nullptr && p + 7 * lanes < p1; p += 8 * lanes) {
      V8<TY> rd[8], rx[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int64_t off = (base + p + u * lanes) * C + g * 8;
        rd[u] = ld8<TY>(dy, off);
        rx[u] = ld8<TY>(x, off);
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) accum(rd[u], rx[u]);
    }
    for (; p < p1; p += lanes) {
      const int64_t off = (base + p) * C + g * 8;
      V8<TY> d = ld8<TY>(dy, off);
      if (yres != nullptr) {
        d = block_end_grad<TY>(d, dy2, off, ld8<TY>(yres, off));
        st8<TY>(gout, off, d);
      }
      accum(d, ld8<TY>(x, off));
    }
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[0][tid * 8 + i] = sg[i];
    red[1][tid * 8 + i] = sgx[i];
    red[2][tid * 8 + i] = sx[i];
  }
  __syncthreads();
  {
    __shared__ float red2[3][NT];
    const int Q = NT / C;
    const int c = tid % C, q = tid / C;
    if (q < Q) {
      const int gg = c / 8, ii = c % 8;
      float a = 0.f, b = 0.f, s = 0.f;
      for (int l = q; l < lanes; l += Q) {
        a += red[0][(l * cg + gg) * 8 + ii];
        b += red[1][(l * cg + gg) * 8 + ii];
        s += red[2][(l * cg + gg) * 8 + ii];
      }
      red2[0][q * C + c] = a;
      red2[1][q * C + c] = b;
      red2[2][q * C + c] = s;
    }
    __syncthreads();
    if (tid < C) {
      float sa = 0.f, sb = 0.f, ss = 0.f;
      for (int k = 0; k < Q; ++k) {
        sa += red2[0][k * C + tid];
        sb += red2[1][k * C + tid];
        ss += red2[2][k * C + tid];
      }
      float* dst = part + ((int64_t)img * gridDim.x + blockIdx.x) * 3 * C;
      dst[tid] = sa;
      dst[C + tid] = sb;
      dst[2 * C + tid] = ss;
    }
  }
}

// Backward partial reduce + per-group finalize in ONE launch: block =
// COLS channels x LANES lanes of one group (grid (groups, ceil(C / COLS))); lanes stride over the
// group's partials, fixed-order LDS combine, then lane 0 writes the group's coefficients and its
// contributions (sum g*xhat, sum g, conv-bias term) to pg [groups][3][C]; the apply kernel's
// first workgroup sums pg over the groups (fixed order) into dgamma / dbeta / dcbias.
template <int LANES, int TY>
__global__ __launch_bounds__(256) void norm_bwd_reduce_finalize_kernel(
    const float* __restrict__ part, int nblk, int C, int cnt, int mode,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ mean,
    const float* __restrict__ invstd, float* __restrict__ coef, float* __restrict__ pg) {
  constexpr int COLS = 256 / LANES;
  __shared__ float red[3][LANES][COLS];
  const int gi = blockIdx.x;
  const int t = threadIdx.x % COLS, lane = threadIdx.x / COLS;
  const int c = blockIdx.y * COLS + t;
  float a = 0.f, b = 0.f, s = 0.f;
  if (c < C)
    for (int k = lane; k < nblk; k += LANES) {
      const float* pk = part + ((int64_t)gi * nblk + k) * 3 * C;
      a += pk[c];
      b += pk[C + c];
      s += pk[2 * C + c];
    }
  red[0][lane][t] = a;
  red[1][lane][t] = b;
  red[2][lane][t] = s;
  __syncthreads();
  if (lane != 0 || c >= C) return;
  float fsg = 0.f, fsgx = 0.f, fsx = 0.f;
#pragma unroll
  for (int l = 0; l < LANES; ++l) {
    fsg += red[0][l][t];
    fsgx += red[1][l][t];
    fsx += red[2][l][t];
  }
  const double sg = fsg, sgx = fsgx, sx = fsx;
  const float gm = (mode == 1 || mode == 2) && gamma ? gamma[c] : 1.f;
  const float is = invstd[(int64_t)gi * C + c];
  float A, B, Cc;
  double dcb;
  if (mode == 0 || mode == 1) {
    const double mg = sg / cnt, mgx = sgx / cnt;
    A = gm * is;
    B = (float)(-gm * is * mgx);
    Cc = (float)(-gm * is * mg);
    dcb = A * sg + B * sx + (double)Cc * cnt;
  } else {
    A = gm * is;
    B = 0.f;
    Cc = 0.f;
    dcb = A * sg;
  }
  const float mu = mean[(int64_t)gi * C + c];
  float sc, sh;
  norm_affine(mode, gamma, beta, c, mu, is, sc, sh);
  float* co = coef + (int64_t)gi * 5 * C + c;
  co[0] = A;
  co[C] = B * is;
  co[2 * C] = Cc - B * is * mu;
  co[3 * C] = sc;
  co[4 * C] = sh;
  float* q = pg + (int64_t)gi * 3 * C + c;
  q[0] = fsgx;
  q[C] = fsg;
  q[2 * C] = (float)dcb;
}

// dx = A*g + B'*x + C' with g = dy masked by the forward ReLU (read from y when given, else
// recomputed from x with the forward's scale / shift); per-element coefficient reads (L1-resident
// table) measured faster than per-thread register caching across the grid-stride loop
template <int TY>
__global__ __launch_bounds__(NT) void norm_bwd_apply_kernel(
    const uint16_t* __restrict__ dy, const uint16_t* __restrict__ x, const uint16_t* __restrict__ y,
    const float* __restrict__ coef, int HW, int C, int per_image, int64_t nvec, int relu,
    uint16_t* __restrict__ dx, const float* __restrict__ pg, int groups, float* __restrict__ dgamma,
    float* __restrict__ dbeta, float* __restrict__ dcbias, uint16_t* __restrict__ dxs, int spad) {
  const int cg = C / 8;
  if (pg != nullptr && blockIdx.x == 0) {
    // parameter gradients: the groups' contributions summed in a fixed order
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
      double dg = 0.0, db = 0.0, dcb = 0.0;
      for (int gi = 0; gi < groups; ++gi) {
        const float* q = pg + (int64_t)gi * 3 * C + c;
        dg += q[0];
        db += q[C];
        dcb += q[2 * C];
      }
      if (dgamma) dgamma[c] = (float)dg;
      if (dbeta) dbeta[c] = (float)db;
      if (dcbias) dcbias[c] = (float)dcb;
    }
  }
  for (int64_t v = blockIdx.x * (int64_t)NT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * NT) {
    const int64_t pix = v / cg;
    const int g = (int)(v - pix * cg);
    const int gi = per_image ? (int)(pix / HW) : 0;
    float d[8], xv[8];
    unpack8<TY>(ld8<TY>(dy, v * 8), d);
    unpack8<TY>(ld8<TY>(x, v * 8), xv);
    const float* co = coef + (int64_t)gi * 5 * C + g * 8;
    auto ldc = [&](int f, float (&r)[8]) {
      const float4 a = *reinterpret_cast<const float4*>(co + f * C);
      const float4 b = *reinterpret_cast<const float4*>(co + f * C + 4);
      r[0] = a.x; r[1] = a.y; r[2] = a.z; r[3] = a.w; r[4] = b.x; r[5] = b.y; r[6] = b.z; r[7] = b.w;
    };
    if (relu && y != nullptr) {
      float yv[8];
      unpack8<TY>(ld8<TY>(y, v * 8), yv);
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = yv[i] > 0.f ? d[i] : 0.f;
    } else if (relu) {
      float sc[8], sh[8];
      ldc(3, sc);
      ldc(4, sh);
#pragma unroll
      for (int i = 0; i < 8; ++i) d[i] = xv[i] * sc[i] + sh[i] > 0.f ? d[i] : 0.f;
    }
    float A[8], Bp[8], Cp[8], o[8];
    ldc(0, A);
    ldc(1, Bp);
    ldc(2, Cp);
#pragma unroll
    for (int i = 0; i < 8; ++i) o[i] = A[i] * d[i] + Bp[i] * xv[i] + Cp[i];
    st8<TY>(dx, v * 8, pack8<TY>(o));
    if (dxs != nullptr) store_split8(dxs, spad, pix, g, cg, o);
  }
}

// Context-encoder output (`core/raft.py:111-113`): cnet (NHWC, C = hdim + cdim) -> h = tanh of
// channels [0, hdim), x = relu of [hdim, C), each written as its own contiguous NHWC tensor (the
// fused update block's operands); one pass instead of split + tanh + relu + two layout copies
template <int TY>
__global__ __launch_bounds__(NT) void ctx_act_kernel(const uint16_t* __restrict__ in, int C, int hdim,
                                                     int64_t nvec, uint16_t* __restrict__ h,
                                                     uint16_t* __restrict__ xo) {
  const int cg = C / 8, hg = hdim / 8, xg = cg - hg;
  for (int64_t v = blockIdx.x * (int64_t)NT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * NT) {
    const int64_t pix = v / cg;
    const int g = (int)(v - pix * cg);
    float f[8];
    unpack8<TY>(ld8<TY>(in, v * 8), f);
    if (g < hg) {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = tanhf(f[i]);
      st8<TY>(h, (pix * hg + g) * 8, pack8<TY>(f));
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) f[i] = f[i] > 0.f ? f[i] : 0.f;
      st8<TY>(xo, (pix * xg + g - hg) * 8, pack8<TY>(f));
    }
  }
}

// its backward: gin[..., :hdim] = gh * (1 - h^2), gin[..., hdim:] = gx * [x > 0]; a missing
// gradient (nullptr) is zero
template <int TY>
__global__ __launch_bounds__(NT) void ctx_act_bwd_kernel(const uint16_t* __restrict__ gh,
                                                         const uint16_t* __restrict__ gx,
                                                         const uint16_t* __restrict__ h,
                                                         const uint16_t* __restrict__ xo, int C, int hdim,
                                                         int64_t nvec, uint16_t* __restrict__ gin) {
  const int cg = C / 8, hg = hdim / 8, xg = cg - hg;
  for (int64_t v = blockIdx.x * (int64_t)NT + threadIdx.x; v < nvec; v += (int64_t)gridDim.x * NT) {
    const int64_t pix = v / cg;
    const int g = (int)(v - pix * cg);
    float d[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) d[i] = 0.f;
    if (g < hg) {
      if (gh != nullptr) {
        const int64_t off = (pix * hg + g) * 8;
        float hv[8];
        unpack8<TY>(ld8<TY>(gh, off), d);
        unpack8<TY>(ld8<TY>(h, off), hv);
#pragma unroll
        for (int i = 0; i < 8; ++i) d[i] = d[i] * (1.f - hv[i] * hv[i]);
      }
      st8<TY>(gin, v * 8, pack8<TY>(d));
    } else if (gx != nullptr) {
      const int64_t off = (pix * xg + g - hg) * 8;
      st8<TY>(gin, v * 8, mask_pos<TY>(ld8<TY>(gx, off), ld8<TY>(xo, off)));
    } else {
      st8<TY>(gin, v * 8, pack8<TY>(d));
    }
  }
}

unsigned grid_for(int64_t nvec) {
  const int64_t b = (nvec + NT - 1) / NT;
  return (unsigned)std::min<int64_t>(b, 256 * 16);
}

}  // namespace

int encoder_norm_blocks(int64_t range, int C, int groups, int* pix_per_blk) {
  // 32 pixels per lane: ~1 K workgroups for the 64-channel full-resolution layers, 70-400 for the
  // 96 / 128-channel stages and the batch-norm encoder's single group.  RAFT_NORM_MIN_WG = n > 0
  // halves the chunk (down to 8 pixels per lane, the statistics kernels' unrolled round) until a
  // launch has n workgroups: measured slower at chairs (encoder norms 4.01 -> 4.26 / 4.38 ms/step
  // at n = 1024 / 2048, profiles/r6/norm_wg/): the statistics passes did not speed up and the
  // finalize kernels pay for the extra partial rows
  static const int min_wg = [] {
    const char* e = std::getenv("RAFT_NORM_MIN_WG");
    return e ? std::atoi(e) : 0;
  }();
  const int cg = C / 8;
  const int lanes = NT / cg;
  int64_t ppb = (int64_t)lanes * 32;
  while ((range + ppb - 1) / ppb * groups < min_wg && ppb > (int64_t)lanes * 8) ppb /= 2;
  if (ppb < 64) ppb = 64;
  const int64_t nb = (range + ppb - 1) / ppb;
  *pix_per_blk = (int)ppb;
  return (int)nb;
}

void launch_norm_stats(const uint16_t* x, int N, int HW, int C, int per_image, float* part,
                       int nblk, int pix_per_blk, int f16, hipStream_t stream) {
  dim3 grid(nblk, per_image ? N : 1);
  if (f16 == 2) hipLaunchKernelGGL(norm_stats_kernel<2>, grid, dim3(NT), 0, stream, x, HW, C, per_image, pix_per_blk,
                     N * HW, part);
  else if (f16) hipLaunchKernelGGL(norm_stats_kernel<1>, grid, dim3(NT), 0, stream, x, HW, C, per_image, pix_per_blk,
                     N * HW, part);
  else hipLaunchKernelGGL(norm_stats_kernel<0>, grid, dim3(NT), 0, stream, x, HW, C, per_image, pix_per_blk,
                     N * HW, part);
}

void launch_norm_finalize(const float* part, const uint16_t* x, int N, int HW, int C, int mode,
                          int nblk, const float* gamma, const float* beta, const float* cbias,
                          float* rmean, float* rvar, float momentum, float eps, float* mean,
                          float* invstd, float* scale, float* shift, int f16, hipStream_t stream) {
  const int groups = mode == 0 ? N : 1;
  const int cnt = mode == 0 ? HW : N * HW;
  const int tot = groups * C;
  if (mode <= 1) {
    // training statistics: partial reduce + finalize in one launch
    if (nblk > 64) {
      if (f16 == 2) hipLaunchKernelGGL((norm_reduce_finalize_kernel<64, 2>), dim3(groups, (C + 3) / 4), dim3(256), 0,
                         stream, part, nblk, x, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                         momentum, eps, mean, invstd, scale, shift, N);
      else if (f16) hipLaunchKernelGGL((norm_reduce_finalize_kernel<64, 1>), dim3(groups, (C + 3) / 4), dim3(256), 0,
                         stream, part, nblk, x, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                         momentum, eps, mean, invstd, scale, shift, N);
      else hipLaunchKernelGGL((norm_reduce_finalize_kernel<64, 0>), dim3(groups, (C + 3) / 4), dim3(256), 0,
                         stream, part, nblk, x, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                         momentum, eps, mean, invstd, scale, shift, N);
    } else {
      if (f16 == 2) hipLaunchKernelGGL((norm_reduce_finalize_kernel<4, 2>), dim3(groups, (C + 63) / 64), dim3(256), 0,
                         stream, part, nblk, x, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                         momentum, eps, mean, invstd, scale, shift, N);
      else if (f16) hipLaunchKernelGGL((norm_reduce_finalize_kernel<4, 1>), dim3(groups, (C + 63) / 64), dim3(256), 0,
                         stream, part, nblk, x, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                         momentum, eps, mean, invstd, scale, shift, N);
      else hipLaunchKernelGGL((norm_reduce_finalize_kernel<4, 0>), dim3(groups, (C + 63) / 64), dim3(256), 0,
                         stream, part, nblk, x, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                         momentum, eps, mean, invstd, scale, shift, N);
    }
    return;
  }
  float* sums = nullptr;
  if (f16 == 2) hipLaunchKernelGGL(norm_finalize_kernel<2>, dim3((tot + 255) / 256), dim3(256), 0, stream, sums, x, HW,
                     C, groups, nblk, cnt, mode, gamma, beta, cbias, rmean, rvar, momentum, eps, mean,
                     invstd, scale, shift, N);
  else if (f16) hipLaunchKernelGGL(norm_finalize_kernel<1>, dim3((tot + 255) / 256), dim3(256), 0, stream, sums, x, HW,
                     C, groups, nblk, cnt, mode, gamma, beta, cbias, rmean, rvar, momentum, eps, mean,
                     invstd, scale, shift, N);
  else hipLaunchKernelGGL(norm_finalize_kernel<0>, dim3((tot + 255) / 256), dim3(256), 0, stream, sums, x, HW,
                     C, groups, nblk, cnt, mode, gamma, beta, cbias, rmean, rvar, momentum, eps, mean,
                     invstd, scale, shift, N);
}

void launch_norm_finalize_tiled(const float* part, int nblk, int N, int HW, int C, int mode,
                                const float* gamma, const float* beta, const float* cbias,
                                float* rmean, float* rvar, float momentum, float eps, float* mean,
                                float* invstd, float* scale, float* shift, hipStream_t stream) {
  const int groups = mode == 0 ? N : 1;
  const int cnt = mode == 0 ? HW : N * HW;
  // 64 lanes per channel: ~6 tile rows each at chairs (368 tiles per 184 x 248 image)
  hipLaunchKernelGGL((norm_reduce_finalize_kernel<64, 0, true>), dim3(groups, (C + 3) / 4), dim3(256), 0,
                     stream, part, nblk, nullptr, HW, C, cnt, mode, gamma, beta, cbias, rmean, rvar,
                     momentum, eps, mean, invstd, scale, shift, N);
}

void launch_norm_apply(const uint16_t* x, const float* scale, const float* shift, int N, int HW,
                       int C, int relu, const uint16_t* res, uint16_t* y, int f16, hipStream_t stream,
                       uint16_t* ys, int spad) {
  if (f16 != 2) ys = nullptr;   // split operands exist for the fp32 schedule only
  const int64_t nvec = (int64_t)N * HW * C / 8;
  const int bt = (NT / (C / 8)) * (C / 8);  // multiple of the channel-group count
  if (f16 == 2) hipLaunchKernelGGL(norm_apply_kernel<2>, dim3(grid_for(nvec)), dim3(bt), 0, stream, x, scale, shift, HW,
                     C, nvec, relu, res, y, ys, spad);
  else if (f16) hipLaunchKernelGGL(norm_apply_kernel<1>, dim3(grid_for(nvec)), dim3(bt), 0, stream, x, scale, shift, HW,
                     C, nvec, relu, res, y, ys, spad);
  else hipLaunchKernelGGL(norm_apply_kernel<0>, dim3(grid_for(nvec)), dim3(bt), 0, stream, x, scale, shift, HW,
                     C, nvec, relu, res, y, ys, spad);
}

void launch_add_relu(const uint16_t* a, const uint16_t* b, uint16_t* out, int64_t n,
                     int f16, hipStream_t stream) {
  const int64_t nvec = n / 8;
  if (f16 == 2) hipLaunchKernelGGL(add_relu_kernel<2>, dim3(grid_for(nvec)), dim3(NT), 0, stream, a, b, out, nvec);
  else if (f16) hipLaunchKernelGGL(add_relu_kernel<1>, dim3(grid_for(nvec)), dim3(NT), 0, stream, a, b, out, nvec);
  else hipLaunchKernelGGL(add_relu_kernel<0>, dim3(grid_for(nvec)), dim3(NT), 0, stream, a, b, out, nvec);
}

void launch_relu_mask(const uint16_t* dy, const uint16_t* dy2, const uint16_t* y, uint16_t* g, int64_t n,
                      int f16, hipStream_t stream) {
  const int64_t nvec = n / 8;
  if (f16 == 2) hipLaunchKernelGGL(relu_mask_kernel<2>, dim3(grid_for(nvec)), dim3(NT), 0, stream, dy, dy2, y, g, nvec);
  else if (f16) hipLaunchKernelGGL(relu_mask_kernel<1>, dim3(grid_for(nvec)), dim3(NT), 0, stream, dy, dy2, y, g, nvec);
  else hipLaunchKernelGGL(relu_mask_kernel<0>, dim3(grid_for(nvec)), dim3(NT), 0, stream, dy, dy2, y, g, nvec);
}

void launch_norm_bwd(const uint16_t* dy, const uint16_t* x, const uint16_t* y, const float* mean,
                     const float* invstd,
                     int N, int HW, int C, int mode, int relu, const float* gamma,
                     const float* beta, float* part, int nblk, int pix_per_blk, float* coef,
                     float* dgamma, float* dbeta, float* dcbias, uint16_t* dx,
                     const uint16_t* dy2, const uint16_t* yres, uint16_t* gout, int f16, hipStream_t stream,
                     uint16_t* dxs, int spad) {
  if (f16 != 2) dxs = nullptr;
  const int per_image = mode == 0 ? 1 : 0;
  const int groups = per_image ? N : 1;
  const int cnt = per_image ? HW : N * HW;
  if (mode == 0 || mode == 1) {
    dim3 grid(nblk, groups);
    if (f16 == 2) hipLaunchKernelGGL(norm_bwd_stats_kernel<2>, grid, dim3(NT), 0, stream, dy, x, mean, invstd, gamma,
                       beta, mode, HW, C, per_image, pix_per_blk, N * HW, relu, part, dy2, yres, gout);
    else if (f16) hipLaunchKernelGGL(norm_bwd_stats_kernel<1>, grid, dim3(NT), 0, stream, dy, x, mean, invstd, gamma,
                       beta, mode, HW, C, per_image, pix_per_blk, N * HW, relu, part, dy2, yres, gout);
    else hipLaunchKernelGGL(norm_bwd_stats_kernel<0>, grid, dim3(NT), 0, stream, dy, x, mean, invstd, gamma,
                       beta, mode, HW, C, per_image, pix_per_blk, N * HW, relu, part, dy2, yres, gout);
  } else {
    // eval / none: only sum(g) and sum(g*xhat) are needed for the parameter grads
    dim3 grid(nblk, 1);
    if (f16 == 2) hipLaunchKernelGGL(norm_bwd_stats_kernel<2>, grid, dim3(NT), 0, stream, dy, x, mean, invstd, gamma,
                       beta, mode, HW, C, 0, pix_per_blk, N * HW, relu, part, dy2, yres, gout);
    else if (f16) hipLaunchKernelGGL(norm_bwd_stats_kernel<1>, grid, dim3(NT), 0, stream, dy, x, mean, invstd, gamma,
                       beta, mode, HW, C, 0, pix_per_blk, N * HW, relu, part, dy2, yres, gout);
    else hipLaunchKernelGGL(norm_bwd_stats_kernel<0>, grid, dim3(NT), 0, stream, dy, x, mean, invstd, gamma,
                       beta, mode, HW, C, 0, pix_per_blk, N * HW, relu, part, dy2, yres, gout);
  }
  // the block-end ReLU ran in the statistics pass: the apply pass reads its result
  if (yres != nullptr) dy = gout;
  // per-group sums + coefficients in one launch; pg (the groups' parameter-gradient terms) sits
  // after the partials in `part`
  float* pg = part + (int64_t)groups * nblk * 3 * C;
  if (nblk > 64) {
    if (f16 == 2) hipLaunchKernelGGL((norm_bwd_reduce_finalize_kernel<16, 2>), dim3(groups, (C + 15) / 16), dim3(256), 0,
                       stream, part, nblk, C, cnt, mode, gamma, beta, mean, invstd, coef, pg);
    else if (f16) hipLaunchKernelGGL((norm_bwd_reduce_finalize_kernel<16, 1>), dim3(groups, (C + 15) / 16), dim3(256), 0,
                       stream, part, nblk, C, cnt, mode, gamma, beta, mean, invstd, coef, pg);
    else hipLaunchKernelGGL((norm_bwd_reduce_finalize_kernel<16, 0>), dim3(groups, (C + 15) / 16), dim3(256), 0,
                       stream, part, nblk, C, cnt, mode, gamma, beta, mean, invstd, coef, pg);
  } else {
    if (f16 == 2) hipLaunchKernelGGL((norm_bwd_reduce_finalize_kernel<4, 2>), dim3(groups, (C + 63) / 64), dim3(256), 0,
                       stream, part, nblk, C, cnt, mode, gamma, beta, mean, invstd, coef, pg);
    else if (f16) hipLaunchKernelGGL((norm_bwd_reduce_finalize_kernel<4, 1>), dim3(groups, (C + 63) / 64), dim3(256), 0,
                       stream, part, nblk, C, cnt, mode, gamma, beta, mean, invstd, coef, pg);
    else hipLaunchKernelGGL((norm_bwd_reduce_finalize_kernel<4, 0>), dim3(groups, (C + 63) / 64), dim3(256), 0,
                       stream, part, nblk, C, cnt, mode, gamma, beta, mean, invstd, coef, pg);
  }
  const int64_t nvec = (int64_t)N * HW * C / 8;
  if (f16 == 2) hipLaunchKernelGGL(norm_bwd_apply_kernel<2>, dim3(grid_for(nvec)), dim3(NT), 0, stream, dy, x, y, coef,
                     HW, C, per_image, nvec, relu, dx, pg, groups, dgamma, dbeta, dcbias, dxs, spad);
  else if (f16) hipLaunchKernelGGL(norm_bwd_apply_kernel<1>, dim3(grid_for(nvec)), dim3(NT), 0, stream, dy, x, y, coef,
                     HW, C, per_image, nvec, relu, dx, pg, groups, dgamma, dbeta, dcbias, dxs, spad);
  else hipLaunchKernelGGL(norm_bwd_apply_kernel<0>, dim3(grid_for(nvec)), dim3(NT), 0, stream, dy, x, y, coef,
                     HW, C, per_image, nvec, relu, dx, pg, groups, dgamma, dbeta, dcbias, dxs, spad);
}

void launch_ctx_act(const uint16_t* in, int64_t P, int C, int hdim, uint16_t* h, uint16_t* x, int f16,
                    hipStream_t stream) {
  const int64_t nvec = P * C / 8;
  if (f16) hipLaunchKernelGGL(ctx_act_kernel<1>, dim3(grid_for(nvec)), dim3(NT), 0, stream, in, C, hdim, nvec, h, x);
  else hipLaunchKernelGGL(ctx_act_kernel<0>, dim3(grid_for(nvec)), dim3(NT), 0, stream, in, C, hdim, nvec, h, x);
}

void launch_ctx_act_bwd(const uint16_t* gh, const uint16_t* gx, const uint16_t* h, const uint16_t* x,
                        int64_t P, int C, int hdim, uint16_t* gin, int f16, hipStream_t stream) {
  const int64_t nvec = P * C / 8;
  if (f16) hipLaunchKernelGGL(ctx_act_bwd_kernel<1>, dim3(grid_for(nvec)), dim3(NT), 0, stream, gh, gx, h, x, C,
                              hdim, nvec, gin);
  else hipLaunchKernelGGL(ctx_act_bwd_kernel<0>, dim3(grid_for(nvec)), dim3(NT), 0, stream, gh, gx, h, x, C,
                          hdim, nvec, gin);
}
