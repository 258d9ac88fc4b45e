// lamm_device.h -- gfx950 device helpers shared by the lamm HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <utility>

#include "lamm_formats.h"

namespace lamm {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ float h2f(uint32_t h16) {
  return (float)__builtin_bit_cast(_Float16, (uint16_t)h16);
}

// Buffer resource over [base, base+bytes): loads past the end return 0 instead of
// faulting (gfx950 raw buffer range check), which is how ragged tails are handled
// without per-load branches (cdna_hip_programming.md §5.5 T8/T20).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* base, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ u32x4 bload16(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t bload4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
}
__device__ __forceinline__ uint16_t bload2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b16(r, off, 0, 0);
}

// Write-through vector stores (sc0 sc1): a short launch's results go straight past L2 instead of
// waiting in it, dirty, for the end-of-kernel write-back.  tools/write_probe.hip
// (profiles/r03/write_probe.json): 4 MB written by a 1024-workgroup pass 2.13 us per launch with
// plain stores, 1.85 us with sc0 sc1 (2 MB 1.99 -> 1.68, 8 MB 2.87 -> 2.52).
constexpr int kAuxWriteThrough = 1 | 16;   // sc0 | sc1
__device__ __forceinline__ void bstore4_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, kAuxWriteThrough);
}
__device__ __forceinline__ void bstore8_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, f32x2 v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, kAuxWriteThrough);
}
__device__ __forceinline__ void bstore16_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, u32x4 v) {
  __builtin_amdgcn_raw_buffer_store_b128(v, r, off, 0, kAuxWriteThrough);
}

// dword starting at byte offset O of a register-resident byte string (O compile-time).
template <int O, int NW>
__device__ __forceinline__ uint32_t get32(const uint32_t (&w)[NW]) {
  static_assert(O >= 0 && ((O & 3) == 0 ? (O >> 2) < NW : (O >> 2) + 1 < NW), "get32 range");
  if constexpr ((O & 3) == 0) {
    return w[O >> 2];
  } else {
    return __builtin_amdgcn_alignbit(w[(O >> 2) + 1], w[O >> 2], (O & 3) * 8);
  }
}
template <int O, int NW>
__device__ __forceinline__ uint32_t get16(const uint32_t (&w)[NW]) {
  return (w[O >> 2] >> ((O & 3) * 8)) & 0xffffu;
}

// Compile-time unrolled loop: unroll<N>([&](auto I) { constexpr int i = I; ... });
template <class Fn, int... I>
__device__ __forceinline__ void unroll_impl(Fn& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, class Fn>
__device__ __forceinline__ void unroll(Fn&& f) {
  unroll_impl(f, std::make_integer_sequence<int, N>{});
}

__device__ __forceinline__ int dot4(uint32_t a, uint32_t b, int c) {
  return __builtin_amdgcn_sdot4((int)a, (int)b, c, false);
}

// Sum over the 64 lanes of a wave in a fixed order (deterministic), returned in every lane:
// DPP within each row of 16 (pairs, quads, 8s via row_half_mirror, 16s via row_mirror), then
// the four row sums read back with v_readlane -- no LDS round trips (__shfl_xor compiles to
// ds_bpermute, ~100+ cycles each, 6 in a row).
template <int CTRL>
__device__ __forceinline__ float dpp_get(float x) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x), CTRL, 0xF, 0xF, false));
}
// No contraction: the first add must not fuse with the caller's product (hipcc contracts across the
// inlined call, so the same per-lane product would sum differently in two kernels -- a row's value
// would depend on the kernel its launch picks, tests/test_gpu_parity.py::test_gemv_row_slab_invariance).
__device__ __forceinline__ float wave_sum(float x) {
#pragma clang fp contract(off)
  x += dpp_get<0xB1>(x);    // quad_perm [1,0,3,2]
  x += dpp_get<0x4E>(x);    // quad_perm [2,3,0,1]
  x += dpp_get<0x141>(x);   // row_half_mirror
  x += dpp_get<0x140>(x);   // row_mirror
  const float r0 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 0));
  const float r1 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 16));
  const float r2 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 32));
  const float r3 = __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, x), 48));
  return (r0 + r1) + (r2 + r3);
}

// _mm256_cvtps_epi32 of an already rounded value: NaN and values outside int32 give INT_MIN (x86's
// "integer indefinite"; v_cvt_i32_f32 would saturate instead) -- an id of inf (0 < amax < ~3.7e-37)
// or NaN inputs then quantize to -128 after the packs, as on the reference's CPU
__device__ __forceinline__ int avx_cvt_i32(float r) {
  return (r >= -2147483648.f && r < 2147483648.f) ? (int)r : (int)0x80000000u;
}

// bit i (i<4) of x -> bit 4 of byte i  (the 5th quant bit of q5_0/q5_1)
__device__ __forceinline__ uint32_t spread4_hi(uint32_t x4) {
  return ((x4 * 0x00204081u) & 0x01010101u) << 4;
}

}  // namespace lamm
