// Shared device code of the implicit-GEMM conv kernels (conv_igemm.hip: register-staged kernel +
// tile dispatch / autotune; conv_glds.hip: LDS-DMA pipelined kernel): LDS swizzle, buffer
// descriptors, branch-free fused epilogues.
#pragma once
#include "common.h"
#include "launchers.h"

namespace conv_detail {


typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
constexpr int BK = 64;   // K per pipeline step: one filter tap x 64 channels (128-B LDS rows)
constexpr int NT = 256;

// 16-B chunk `chunk` (0..7) of LDS row `row` (128 B).  A 256-B bank row holds two LDS rows; a
// ds_read_b128 fragment read serves 16 lanes = 16 consecutive rows at one logical chunk per pass, so
// the XOR key is (row >> 1) & 7: each row-parity class of the 16 rows lands on 8 distinct 16-B
// slots and the pass is conflict-free (the ds_write_b128 tile stores stay conflict-free too).
__device__ __forceinline__ int swz(int row, int chunk) { return row * 8 + (chunk ^ ((row >> 1) & 7)); }

__device__ __forceinline__ bf16x8_t zero_frag8() { return __builtin_bit_cast(bf16x8_t, make_uint4(0, 0, 0, 0)); }

// 16-bit operand type (common.h): fragments travel as bf16x8_t bit containers
template <bool F16>
__device__ __forceinline__ f32x16 mfma16(bf16x8_t a, bf16x8_t b, f32x16 c) { return raft_mfma32<F16>(a, b, c); }
template <bool F16>
__device__ __forceinline__ float cvt16(uint16_t v) { return raft_h2f<F16>(v); }
template <bool F16>
__device__ __forceinline__ uint16_t pack16(float v) { return raft_f2h<F16>(v); }

typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t OOB = 0x80000000u;  // voffset past every num_records: the load returns zeros

__device__ __forceinline__ rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 buf_load16(rsrc_t r, uint32_t voff) {
  auto v = __builtin_amdgcn_raw_buffer_load_b128(r, voff, 0, 0);
  return __builtin_bit_cast(uint4, v);
}

// XCD-aware tile order for a 1-D grid padded to a multiple of 8: the dispatcher deals
// consecutive workgroups round-robin over the 8 XCDs, so logical tile L = (id % 8) * (grid / 8) +
// id / 8 gives every XCD a contiguous run of tiles: the N tiles of one M tile (same input rows)
// and neighbouring M tiles (shared halo rows of the shifted taps) meet in the same L2.
// Returns false for the padding workgroups.
__device__ __forceinline__ bool conv_tile_coords(int n_m, int n_n, int& mt, int& nt) {
  const int L = (int)(blockIdx.x & 7) * (int)(gridDim.x >> 3) + (int)(blockIdx.x >> 3);
  if (L >= n_m * n_n) return false;
  mt = L / n_n;
  nt = L - mt * n_n;
  return true;
}
inline int conv_grid_1d(int n_m, int n_n) { return (n_m * n_n + 7) / 8 * 8; }

__device__ __forceinline__ float sigmoidf_(float v) { return 1.f / (1.f + __expf(-v)); }
__device__ __forceinline__ float tanhf_(float v) {
  const float e = __expf(-2.f * fabsf(v));
  const float t = (1.f - e) / (1.f + e);
  return copysignf(t, v);
}

// ---------------------------------------------------------------- fused epilogue
// Branch-free: every load and store goes through a range-checked buffer descriptor and invalid
// rows / columns get an out-of-range offset (loads read 0, stores are dropped).  With no exec-
// masked blocks around memory ops hipcc counts vmcnt exactly: one wait per 32x32 tile (for the
// tile's aux / accumulate loads) instead of an `s_waitcnt vmcnt(0)` before EVERY store, which
// serialized the 16-64 stores of a wave into dependent memory round trips.
// Column-wise choices (GRU z vs r half, dgrad output segment) are made on the wave-uniform tile
// column (segment / split boundaries are multiples of 32, checked on the host).
__device__ __forceinline__ float bld_f32(rsrc_t r, uint32_t off) {
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
template <bool F16 = false>
__device__ __forceinline__ float bld_bf16(rsrc_t r, uint32_t off) {
  return cvt16<F16>(__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0));
}
__device__ __forceinline__ void bst_f32(rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), r, off, 0, 0);
}
template <bool F16 = false>
__device__ __forceinline__ void bst_bf16(rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b16(pack16<F16>(v), r, off, 0, 0);
}
// 16-bit activation element of operand type OT (0 bf16, 1 fp16, 2 split: the fp32 value as a
// bf16 pair, hi at channel c and lo = bf16(v - hi) at channel c + stride / 2 of the same pixel
// row -- `lo` is that distance in bytes, i.e. the row stride in elements)
template <int OT>
__device__ __forceinline__ float ld16(rsrc_t r, uint32_t off, uint32_t lo) {
  float v = cvt16<OT == 1>(__builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0));
  if constexpr (OT == 2) v += cvt16<false>(__builtin_amdgcn_raw_buffer_load_b16(r, off + lo, 0, 0));
  return v;
}
template <int OT>
__device__ __forceinline__ void st16(rsrc_t r, uint32_t off, uint32_t lo, float v) {
  const uint16_t h = pack16<OT == 1>(v);
  __builtin_amdgcn_raw_buffer_store_b16(h, r, off, 0, 0);
  if constexpr (OT == 2)
    __builtin_amdgcn_raw_buffer_store_b16(pack16<false>(v - cvt16<false>(h)), r, off + lo, 0, 0);
}

// 64-channel K chunks of the workgroup whose N tile is [n0, n0 + BN): all of cin_pad unless the
// output segments it overlaps all read a K prefix (OSeg.kcin); then the longest of those prefixes
__device__ __forceinline__ int tile_nchunk(const ConvFwdArgs& a, int n0, int BN) {
  if (!a.kprefix) return a.cin_pad / BK;
  int base = 0, kc = 0;
#pragma unroll
  for (int s = 0; s < 3; ++s) {
    if (s < a.noseg) {
      const int hi = base + a.oseg[s].cnt;
      if (base < n0 + BN && hi > n0) kc = max(kc, a.oseg[s].kcin > 0 ? a.oseg[s].kcin : a.cin_pad);
      base = hi;
    }
  }
  return (kc > 0 ? kc : a.cin_pad) / BK;
}

template <int TM, int TN, int WM, int WN, int EPI>
__device__ __forceinline__ void conv_epilogue(const ConvFwdArgs& a, f32x16 (&acc)[TM][TN], int m0,
                                              int n0, int wm, int wn, int lane, int P, int HW) {
  constexpr int OT = epi_ot(EPI);
  constexpr int E = epi_kind(EPI);
  constexpr bool F32OUT = E == EPI_F32 || E == EPI_ACC_F32 || E == EPI_F32_NCHW;
  constexpr uint32_t ES = F32OUT ? 4u : 2u;
  const rsrc_t bias_rs = make_rsrc(a.bias, a.bias ? (uint32_t)a.cout * 4u : 0u);
  const uint32_t P_u = (uint32_t)P;
  const rsrc_t nul = make_rsrc(nullptr, 0u);
  rsrc_t o0 = nul, o1 = nul, o2 = nul, x0 = nul, x1 = nul;
  if constexpr (E == EPI_F32_NCHW) {
    o0 = make_rsrc(a.out0, P_u * (uint32_t)a.cout * 4u);
  } else if constexpr (E != EPI_DGRAD && E != EPI_DGRAD_GATE) {
    o0 = make_rsrc(a.out0, P_u * (uint32_t)a.out0_stride * ES);
  }
  if constexpr (E == EPI_GRU_ZR || E == EPI_GRU_Q) {
    o1 = make_rsrc(a.out1, P_u * (uint32_t)a.out1_stride * 2u);
    x0 = make_rsrc(a.aux0, P_u * (uint32_t)a.aux0_stride * 2u);
  }
  if constexpr (E == EPI_GRU_ZR) o2 = make_rsrc(a.out2, P_u * (uint32_t)a.out2_stride * 2u);
  if constexpr (E == EPI_GRU_Q) x1 = make_rsrc(a.aux1, P_u * (uint32_t)a.aux1_stride * 2u);
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int ncol0 = __builtin_amdgcn_readfirstlane(n0 + wn * WN + j * 32);
      if (ncol0 >= a.cout) continue;  // wave-uniform
      const int n = ncol0 + (lane & 31);
      const bool nok = n < a.cout;
      const float bias = bld_f32(bias_rs, nok ? (uint32_t)n * 4u : OOB);
      int mrow[16];
      bool ok[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        mrow[r] = m0 + wm * WM + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        ok[r] = nok && mrow[r] < P;
      }
      float v[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) v[r] = (acc[i][j][r] + bias) * a.scale;
      if constexpr (E == EPI_GRU_ZR || E == EPI_GRU_Q) {
        if (a.bmap != nullptr && a.bmap_bf16) {  // uniform
          const rsrc_t bm = make_rsrc(a.bmap, P_u * (uint32_t)a.bmap_stride * 2u);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            v[r] += ld16<OT>(bm, ok[r] ? (uint32_t)(mrow[r] * a.bmap_stride + n) * 2u : OOB, (uint32_t)a.bmap_stride);
        } else if (a.bmap != nullptr) {
          const rsrc_t bm = make_rsrc(a.bmap, P_u * (uint32_t)a.bmap_stride * 4u);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            v[r] += bld_f32(bm, ok[r] ? (uint32_t)(mrow[r] * a.bmap_stride + n) * 4u : OOB);
        }
      }

      if constexpr (E == EPI_BF16 || E == EPI_RELU_BF16 || E == EPI_F32) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const uint32_t off = ok[r] ? (uint32_t)(mrow[r] * a.out0_stride + n) * ES : OOB;
          if constexpr (E == EPI_F32) bst_f32(o0, off, v[r]);
          else st16<OT>(o0, off, (uint32_t)a.out0_stride, E == EPI_RELU_BF16 ? fmaxf(v[r], 0.f) : v[r]);
        }
      } else if constexpr (E == EPI_ACC_F32) {
        uint32_t off[16];
        float pre[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          off[r] = ok[r] ? (uint32_t)(mrow[r] * a.out0_stride + n) * 4u : OOB;
          pre[r] = bld_f32(o0, off[r]);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) bst_f32(o0, off[r], pre[r] + v[r]);
      } else if constexpr (E == EPI_F32_NCHW) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int b = mrow[r] / HW, yx = mrow[r] - b * HW;
          bst_f32(o0, ok[r] ? (uint32_t)((b * a.cout + n) * HW + yx) * 4u : OOB, v[r]);
        }
      } else if constexpr (E == EPI_GRU_ZR) {
        if (ncol0 < a.split) {  // z half
#pragma unroll
          for (int r = 0; r < 16; ++r)
            st16<OT>(o0, ok[r] ? (uint32_t)(mrow[r] * a.out0_stride + n) * 2u : OOB, (uint32_t)a.out0_stride, sigmoidf_(v[r]));
        } else {  // r half: r*h and r
          const int c = n - a.split;
          float h[16];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            h[r] = ld16<OT>(x0, ok[r] ? (uint32_t)(mrow[r] * a.aux0_stride + c) * 2u : OOB, (uint32_t)a.aux0_stride);
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const float g = sigmoidf_(v[r]);
            st16<OT>(o1, ok[r] ? (uint32_t)(mrow[r] * a.out1_stride + c) * 2u : OOB, (uint32_t)a.out1_stride, g * h[r]);
            st16<OT>(o2, ok[r] ? (uint32_t)(mrow[r] * a.out2_stride + c) * 2u : OOB, (uint32_t)a.out2_stride, g);
          }
        }
      } else if constexpr (E == EPI_GRU_Q) {
        float h[16], z[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          h[r] = ld16<OT>(x0, ok[r] ? (uint32_t)(mrow[r] * a.aux0_stride + n) * 2u : OOB, (uint32_t)a.aux0_stride);
          z[r] = ld16<OT>(x1, ok[r] ? (uint32_t)(mrow[r] * a.aux1_stride + n) * 2u : OOB, (uint32_t)a.aux1_stride);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float q = tanhf_(v[r]);
          st16<OT>(o0, ok[r] ? (uint32_t)(mrow[r] * a.out0_stride + n) * 2u : OOB, (uint32_t)a.out0_stride, h[r] + z[r] * (q - h[r]));
          st16<OT>(o1, ok[r] ? (uint32_t)(mrow[r] * a.out1_stride + n) * 2u : OOB, (uint32_t)a.out1_stride, q);
        }
      } else if constexpr (E == EPI_DGRAD || E == EPI_DGRAD_GATE) {
        // output segment of this 32-column tile (uniform)
        int s = 0, base = 0;
#pragma unroll
        for (int q = 0; q < 2; ++q)
          if (s + 1 < a.noseg && ncol0 >= base + a.oseg[s].cnt) { base += a.oseg[s].cnt; ++s; }
        const OSeg o = a.oseg[s];
        const int c = n - base;
        const bool cok = c < o.real;
        bool gated = false;
        if constexpr (E == EPI_DGRAD_GATE) {
          gated = o.gate != 0;
          if (o.gate == 1) {  // ConvGRU q / z gate backward on the final state gradient
            const rsrc_t od = make_rsrc(o.ptr, P_u * (uint32_t)o.stride * 4u);
            const uint32_t ab = P_u * (uint32_t)o.ga_stride * 2u;
            const rsrc_t rz = make_rsrc(o.ga0, ab), rq = make_rsrc(o.ga1, ab), rh = make_rsrc(o.ga2, ab);
            const rsrc_t gb = make_rsrc(o.gb, P_u * (uint32_t)o.gb_stride * 2u);
            const rsrc_t gz = make_rsrc(o.gz, P_u * (uint32_t)o.gz_stride * 2u);
            const rsrc_t f1 = make_rsrc(o.gf1, P_u * (uint32_t)o.gf_stride * 4u);
#pragma unroll
            for (int h8 = 0; h8 < 16; h8 += 8) {   // 8 rows at a time: bounded live registers
              float pre[8], zz[8], qq[8], hh[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int r = h8 + u;
                const bool e = ok[r] && cok;
                pre[u] = bld_f32(od, e ? (uint32_t)(mrow[r] * o.stride + c) * 4u : OOB);
                const uint32_t oa = e ? (uint32_t)(mrow[r] * o.ga_stride + c) * 2u : OOB;
                zz[u] = ld16<OT>(rz, oa, (uint32_t)o.ga_stride);
                qq[u] = ld16<OT>(rq, oa, (uint32_t)o.ga_stride);
                hh[u] = ld16<OT>(rh, oa, (uint32_t)o.ga_stride);
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int r = h8 + u;
                const bool e = ok[r] && cok;
                const float g = pre[u] + v[r];
                st16<OT>(gb, e ? (uint32_t)(mrow[r] * o.gb_stride + c) * 2u : OOB, (uint32_t)o.gb_stride,
                         g * zz[u] * (1.f - qq[u] * qq[u]));
                const float dz = g * (qq[u] - hh[u]);
                st16<OT>(gz, e ? (uint32_t)(mrow[r] * o.gz_stride + c) * 2u : OOB, (uint32_t)o.gz_stride,
                         dz * zz[u] * (1.f - zz[u]));
                bst_f32(f1, e ? (uint32_t)(mrow[r] * o.gf_stride + c) * 4u : OOB, g * (1.f - zz[u]));
              }
            }
          } else if (o.gate == 3) {  // last accumulation + ReLU backward: gb = bf16([y > 0](pre + v))
            const uint32_t ab = P_u * (uint32_t)o.ga_stride * 2u;
            const rsrc_t ry = make_rsrc(o.ga0, ab);
            const rsrc_t f1 = make_rsrc(o.gf1, P_u * (uint32_t)o.gf_stride * 4u);
            const rsrc_t gb = make_rsrc(o.gb, P_u * (uint32_t)o.gb_stride * 2u);
#pragma unroll
            for (int h8 = 0; h8 < 16; h8 += 8) {
              float pre[8], yv[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int r = h8 + u;
                const bool e = ok[r] && cok;
                pre[u] = bld_f32(f1, e ? (uint32_t)(mrow[r] * o.gf_stride + c) * 4u : OOB);
                yv[u] = ld16<OT>(ry, e ? (uint32_t)(mrow[r] * o.ga_stride + c) * 2u : OOB, (uint32_t)o.ga_stride);
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int r = h8 + u;
                const bool e = ok[r] && cok;
                st16<OT>(gb, e ? (uint32_t)(mrow[r] * o.gb_stride + c) * 2u : OOB, (uint32_t)o.gb_stride,
                         yv[u] > 0.f ? pre[u] + v[r] : 0.f);
              }
            }
          } else if (o.gate == 2) {  // ConvGRU r gate backward on d(r*h)
            const uint32_t ab = P_u * (uint32_t)o.ga_stride * 2u;
            const rsrc_t rr = make_rsrc(o.ga1, ab), rh = make_rsrc(o.ga2, ab);
            const rsrc_t gb = make_rsrc(o.gb, P_u * (uint32_t)o.gb_stride * 2u);
            const rsrc_t f1 = make_rsrc(o.gf1, P_u * (uint32_t)o.gf_stride * 4u);
#pragma unroll
            for (int h8 = 0; h8 < 16; h8 += 8) {
              float rv[8], hh[8], dh[8];
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int r = h8 + u;
                const bool e = ok[r] && cok;
                const uint32_t oa = e ? (uint32_t)(mrow[r] * o.ga_stride + c) * 2u : OOB;
                dh[u] = bld_f32(f1, e ? (uint32_t)(mrow[r] * o.gf_stride + c) * 4u : OOB);
                rv[u] = ld16<OT>(rr, oa, (uint32_t)o.ga_stride);
                hh[u] = ld16<OT>(rh, oa, (uint32_t)o.ga_stride);
              }
#pragma unroll
              for (int u = 0; u < 8; ++u) {
                const int r = h8 + u;
                const bool e = ok[r] && cok;
                st16<OT>(gb, e ? (uint32_t)(mrow[r] * o.gb_stride + o.real + c) * 2u : OOB, (uint32_t)o.gb_stride,
                         v[r] * hh[u] * rv[u] * (1.f - rv[u]));
                bst_f32(f1, e ? (uint32_t)(mrow[r] * o.gf_stride + c) * 4u : OOB,
                        dh[u] + v[r] * rv[u]);
              }
            }
          }
        }
        if (gated) {
          // the gate epilogue consumed this segment's values
        } else if (o.ob != nullptr && o.ry == nullptr) {  // plain bf16 gradient
          const rsrc_t ob = make_rsrc(o.ob, P_u * (uint32_t)o.ob_stride * 2u);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            st16<OT>(ob, ok[r] && cok ? (uint32_t)(mrow[r] * o.ob_stride + c) * 2u : OOB, (uint32_t)o.ob_stride, v[r]);
        } else if (o.ob != nullptr) {  // relu-gated bf16 gradient
          const rsrc_t ob = make_rsrc(o.ob, P_u * (uint32_t)o.ob_stride * 2u);
          const rsrc_t ry = make_rsrc(o.ry, P_u * (uint32_t)o.ry_stride * 2u);
          float y[16];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            y[r] = ld16<OT>(ry, ok[r] && cok ? (uint32_t)(mrow[r] * o.ry_stride + c) * 2u : OOB, (uint32_t)o.ry_stride);
#pragma unroll
          for (int r = 0; r < 16; ++r)
            st16<OT>(ob, ok[r] && cok ? (uint32_t)(mrow[r] * o.ob_stride + c) * 2u : OOB, (uint32_t)o.ob_stride,
                     y[r] > 0.f ? v[r] : 0.f);
        } else if (o.ptr != nullptr) {
          const rsrc_t od = make_rsrc(o.ptr, P_u * (uint32_t)o.stride * 4u);
          uint32_t off[16];
#pragma unroll
          for (int r = 0; r < 16; ++r)
            off[r] = ok[r] && cok ? (uint32_t)(mrow[r] * o.stride + c) * 4u : OOB;
          if (o.acc) {
            float pre[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) pre[r] = bld_f32(od, off[r]);
#pragma unroll
            for (int r = 0; r < 16; ++r) bst_f32(od, off[r], pre[r] + v[r]);
          } else {
#pragma unroll
            for (int r = 0; r < 16; ++r) bst_f32(od, off[r], v[r]);
          }
        }
      }
    }
}


template <int TM, int TN, int WVM>
struct ConvTile {
  static constexpr int WVN = 4 / WVM;
  static constexpr int BM = 32 * TM * WVM, BN = 32 * TN * WVN;
  static constexpr int LDS = 2 * (BM + BN) * 128;
  static constexpr int OCC = LDS <= 65536 && TM * TN <= 4 ? 2 : 1;
};

}  // namespace conv_detail
