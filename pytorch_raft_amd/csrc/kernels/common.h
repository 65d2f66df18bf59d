// Shared helpers for the gfx950 (MI355X / CDNA4) kernels of pytorch_raft_amd.
//
// Kernels are written for wave64 and compiled only with --offload-arch=gfx950.  They expose plain
// C++ launch functions (raw pointers + a hipStream_t) declared in launchers.h; the torch-facing
// validation / dispatch lives in ../bindings.cpp, so these translation units never include torch
// headers and compile in seconds.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#define RAFT_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float raft_bf16_to_f32(uint16_t v) {
  return __uint_as_float(((uint32_t)v) << 16);
}

// round-to-nearest-even f32 -> bf16 bits (inputs here are finite activations)
__device__ __forceinline__ uint16_t raft_f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// ---- 16-bit MFMA operand type: bf16 (F16 = false) or fp16 (fp16 autocast).  Operands travel as
// 16-bit bit containers; only the MFMA instruction and the conversions know the type.
typedef __bf16 raft_v8bf16 __attribute__((ext_vector_type(8)));
typedef _Float16 raft_v8f16 __attribute__((ext_vector_type(8)));
template <bool F16>
__device__ __forceinline__ f32x16 raft_mfma32(raft_v8bf16 a, raft_v8bf16 b, f32x16 c) {
  if constexpr (F16)
    return __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(raft_v8f16, a),
                                                 __builtin_bit_cast(raft_v8f16, b), c, 0, 0, 0);
  else
    return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
template <bool F16>
__device__ __forceinline__ float raft_h2f(uint16_t v) {
  if constexpr (F16) return (float)__builtin_bit_cast(_Float16, v);
  else return raft_bf16_to_f32(v);
}
template <bool F16>
__device__ __forceinline__ uint16_t raft_f2h(float v) {
  if constexpr (F16) return __builtin_bit_cast(uint16_t, (_Float16)v);
  else return raft_f32_to_bf16(v);
}

template <typename T> struct Ld;
template <> struct Ld<float> {
  __device__ __forceinline__ static float get(const float* p, int64_t i) { return p[i]; }
};
template <> struct Ld<uint16_t> {
  __device__ __forceinline__ static float get(const uint16_t* p, int64_t i) {
    return raft_bf16_to_f32(p[i]);
  }
};

template <typename T> struct St;
template <> struct St<float> {
  __device__ __forceinline__ static void put(float* p, int64_t i, float v) { p[i] = v; }
};
template <> struct St<uint16_t> {
  __device__ __forceinline__ static void put(uint16_t* p, int64_t i, float v) {
    p[i] = raft_f32_to_bf16(v);
  }
};
// fp16 bits (fp16 autocast outputs)
struct Fp16Bits { uint16_t v; };
template <> struct St<Fp16Bits> {
  __device__ __forceinline__ static void put(Fp16Bits* p, int64_t i, float v) {
    reinterpret_cast<uint16_t*>(p)[i] = raft_f2h<true>(v);
  }
};

// ---- cross-lane sums on DPP (VALU: no ds_bpermute traffic through the LDS pipe).  Fixed pairing
// order, and every lane of the group ends with the same bits (deterministic).  Used where it
// measured faster (the convex upsample backward); in the correlation build's epilogue the same
// lane-pair sum on DPP made the compiler spill 243 VGPRs (0.28 -> 0.98 ms), and the flow head's
// 32-lane sums showed no clear gain (20.1 vs 21.5 us, across boxes): both keep __shfl_xor.
template <int CTRL>
__device__ __forceinline__ float raft_dpp(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, true));
}
// sum over a 16-lane DPP row
__device__ __forceinline__ float raft_row16_sum(float v) {
  v += raft_dpp<0xB1>(v);   // quad_perm [1,0,3,2]: lane ^ 1
  v += raft_dpp<0x4E>(v);   // quad_perm [2,3,0,1]: lane ^ 2
  v += raft_dpp<0x141>(v);  // row_half_mirror: lane i <-> 7 - i of its 8
  v += raft_dpp<0x140>(v);  // row_mirror: lane i <-> 15 - i of its 16
  return v;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

static inline __host__ __device__ unsigned raft_cdiv(int64_t a, int64_t b) { return (unsigned)((a + b - 1) / b); }

// ---- LDS-DMA (buffer_load ... lds) helpers shared by the MFMA conv kernels
//
// s_waitcnt vmcnt(N) with the other counters left alone (gfx9 encoding: vmcnt[3:0] + [15:14]).
template <int N>
__device__ __forceinline__ void raft_wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// One 16-B-per-lane LDS-DMA: lane l's 16 bytes at voff land at LDS byte lds_addr + 16 l
// (lds_addr wave-uniform).  Issued from inline asm so hipcc does not treat the following
// ds_reads as dependent on it (it would otherwise insert `s_waitcnt vmcnt(0)` before the first
// LDS read after any LDS-DMA, draining the prefetch pipeline); completion is counted by the
// caller with raft_wait_vmcnt + a barrier.  M0 is saved and restored inside the statement.
__device__ __forceinline__ void raft_dma16(__amdgpu_buffer_rsrc_t r, uint32_t lds_addr, uint32_t voff) {
  uint32_t keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %1\n\t"
      "s_nop 4\n\t"
      "buffer_load_dwordx4 %2, %3, 0 offen lds\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "s"(lds_addr), "v"(voff), "s"(r)
      : "memory");
}

// LDS byte address of a __shared__ object (for raft_dma16)
__device__ __forceinline__ uint32_t raft_lds_addr(const void* p) {
  return (uint32_t)(size_t)(const __attribute__((address_space(3))) void*)p;
}
