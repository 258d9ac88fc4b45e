// lamm_gemv_dense.hip -- decode-shaped (N <= 8) mat-vec for the unquantized weight rows:
// F32 x F32 (src/lamm_kernel_f32.hpp, the reference's lamm_kernel_f32) and the §8f F16 x F16
// rows (ggml_vec_dot_f16, LC/ggml.c:1589-1629).
//
// The block-format GEMV (lamm_gemv.hip) gives each lane 1/16 of a row segment in VGPRs,
// which for 4-byte elements means 1024-element segments and a re-staged activation per
// segment.  Unquantized rows need no unpacking, so this kernel streams them directly:
//   * one WAVE owns RW rows at a time; each step its 64 lanes read 64 consecutive 16-byte
//     pieces of every row (1 KiB per row per step, fully coalesced, non-temporal: A is read
//     once), U steps in flight per row;
//   * the activation column(s) are staged once per workgroup into LDS (32 KiB budget, a
//     K-segment loop covers longer rows) and read back with ds_read_b128 at the same lane
//     offsets (conflict-free), shared by the RW rows;
//   * f32: 4 FMAs per piece per column; f16: 4 v_dot2_f32_f16 (exact products, fp32 sums);
//   * per-lane partials are reduced across the wave once per row (fixed shuffle order:
//     deterministic), elements past K are masked so row padding (possibly NaN) never
//     reaches the sum.
// Bytes per output row: K * 2|4 (A) -- B comes from LDS, C is 4 bytes: HBM-bound.
#include "lamm_device.h"
#include "lamm_kernels.h"

namespace lamm {
namespace {

constexpr int kDWaves = 8;                 // waves per workgroup
constexpr int kDThreads = 64 * kDWaves;
constexpr int kDLdsBytes = 32 * 1024;      // activation staging budget per workgroup
constexpr int kDU = 4;                     // steps (16-byte loads per row) in flight

template <int T> struct Dense;
template <> struct Dense<kF32> { static constexpr int EB = 4; };
template <> struct Dense<kF16> { static constexpr int EB = 2; };

typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// elements of one row consumed by one wave step
template <int T> constexpr int dstep() { return 64 * 16 / Dense<T>::EB; }

// elements per K-segment (multiple of a wave step) for NC staged columns
template <int T> constexpr int dseg(int nc) {
  return (kDLdsBytes / nc / Dense<T>::EB) / dstep<T>() * dstep<T>();
}

// a . b over one 16-byte piece, masked to the first nv elements when MASK
template <int T, bool MASK>
__device__ __forceinline__ float piece_dot(u32x4 a, u32x4 b, int nv, float acc) {
  if constexpr (MASK) {
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      uint32_t m;
      if constexpr (T == kF32) m = c < nv ? 0xffffffffu : 0u;
      else m = 2 * c + 1 < nv ? 0xffffffffu : (2 * c < nv ? 0x0000ffffu : 0u);
      a[c] &= m;
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    // copy the lanes out first: __builtin_bit_cast of an ext-vector element lvalue reads
    // the vector's first element (always component 0) with this compiler
    const uint32_t ac = a[c], bc = b[c];
    if constexpr (T == kF32)
      acc = __builtin_fmaf(__uint_as_float(ac), __uint_as_float(bc), acc);
    else
      acc = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, ac), __builtin_bit_cast(h2, bc), acc, false);
  }
  return acc;
}

template <int T, int NC, int RW>
__global__ __launch_bounds__(kDThreads) void gemv_dense_kernel(GemvArgs p) {
  constexpr int EB = Dense<T>::EB, EV = 16 / EB, STEP = dstep<T>(), SEGK = dseg<T>(NC);
  constexpr int SEGW = SEGK * EB / 4;       // LDS words per staged column
  __shared__ __attribute__((aligned(16))) uint32_t bs[NC * SEGW];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int K = p.K;
  const int ncols = p.N < NC ? p.N : NC;
  const int nseg = (K + SEGK - 1) / SEGK;
  const int bands = (p.M + kDWaves * RW - 1) / (kDWaves * RW);
  const int64_t bbytes = (int64_t)(p.N - 1) * p.ldb + (int64_t)K * EB;
  const auto rsb = make_rsrc(Bz, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));

  auto stage = [&](int seg) {
    const int64_t k0 = (int64_t)seg * SEGK;
    for (int it = t; it < NC * SEGW; it += kDThreads) {
      const int j = it / SEGW, wi = it % SEGW;
      uint32_t v = 0;
      if constexpr (T == kF32) {
        const int64_t e = k0 + wi;
        if (j < ncols && e < K) v = bload4(rsb, (uint32_t)(j * p.ldb + e * 4));
      } else {   // F16 rows need only be 2-byte aligned: two 2-byte loads per word
        const int64_t e = k0 + 2 * wi;
        uint32_t lo = 0, hi = 0;
        if (j < ncols && e < K) lo = bload2(rsb, (uint32_t)(j * p.ldb + e * 2));
        if (j < ncols && e + 1 < K) hi = bload2(rsb, (uint32_t)(j * p.ldb + e * 2 + 2));
        v = lo | (hi << 16);
      }
      bs[it] = v;
    }
  };

  if (nseg == 1) {
    stage(0);
    __syncthreads();
  }
  for (int band = blockIdx.x; band < bands; band += gridDim.x) {
    const int r0 = (band * kDWaves + w) * RW;
    const int rows = max(0, min(RW, p.M - r0));
    const int64_t avail = rows ? (int64_t)(rows - 1) * p.lda + (int64_t)K * EB : 0;
    const auto ra = make_rsrc(Az + (int64_t)r0 * p.lda, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
    uint32_t roff[RW];
#pragma unroll
    for (int i = 0; i < RW; ++i) roff[i] = i < rows ? (uint32_t)(i * p.lda) : 0x7ffffff0u;
    float acc[RW][NC];
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
      for (int j = 0; j < NC; ++j) acc[i][j] = 0.f;

    for (int seg = 0; seg < nseg; ++seg) {
      if (nseg > 1) {
        __syncthreads();   // previous segment's readers done
        stage(seg);
        __syncthreads();
      }
      const int k0 = seg * SEGK;
      const int klen = min(SEGK, K - k0);
      const int nfull = klen / STEP;            // steps with every lane in range
      auto step = [&](u32x4 (&a)[RW], int s, auto masked) {
        constexpr bool MASK = decltype(masked)::value;
        const int e = s * STEP + lane * EV;       // element within the segment
        const int nv = klen - e;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          if (j < ncols) {
            const u32x4 b = *(const u32x4*)&bs[j * SEGW + e * EB / 4];
#pragma unroll
            for (int i = 0; i < RW; ++i) acc[i][j] = piece_dot<T, MASK>(a[i], b, nv, acc[i][j]);
          }
        }
      };
      auto load = [&](u32x4 (&a)[RW], int s) {
        const uint32_t kb = (uint32_t)((k0 + s * STEP + lane * EV) * EB);
#pragma unroll
        for (int i = 0; i < RW; ++i) a[i] = __builtin_amdgcn_raw_buffer_load_b128(ra, roff[i] + kb, 0, 2);
      };
      int s = 0;
      for (; s + kDU <= nfull; s += kDU) {
        u32x4 a[kDU][RW];
#pragma unroll
        for (int u = 0; u < kDU; ++u) load(a[u], s + u);
#pragma unroll
        for (int u = 0; u < kDU; ++u) step(a[u], s + u, std::false_type{});
      }
      for (; s < nfull; ++s) {
        u32x4 a[RW];
        load(a, s);
        step(a, s, std::false_type{});
      }
      if (nfull * STEP < klen) {   // ragged tail: lanes past K masked (loads past the row read 0)
        u32x4 a[RW];
        load(a, nfull);
        step(a, nfull, std::true_type{});
      }
    }
#pragma unroll
    for (int i = 0; i < RW; ++i)
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        float x = acc[i][j];
        x += __shfl_xor(x, 32);
        x += __shfl_xor(x, 16);
        x += __shfl_xor(x, 8);
        x += __shfl_xor(x, 4);
        x += __shfl_xor(x, 2);
        x += __shfl_xor(x, 1);
        acc[i][j] = x;
      }
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < RW; ++i)
#pragma unroll
        for (int j = 0; j < NC; ++j)
          if (i < rows && j < ncols) Cz[(int64_t)j * p.ldc + r0 + i] = acc[i][j];
    }
  }
}

template <int T, int NC, int RW>
hipError_t launch_rw(const GemvArgs& p, hipStream_t s) {
  const int slices = p.ne12 * p.ne13;
  const int bands = (p.M + kDWaves * RW - 1) / (kDWaves * RW);
  // up to 4 workgroups per CU resident; a workgroup keeps its staged activation for every
  // band it visits (grid-stride), so launch no more than one resident round
  int gx = (256 * 4 + slices - 1) / slices;
  gx = gx < 1 ? 1 : (gx > bands ? bands : gx);
  hipLaunchKernelGGL((gemv_dense_kernel<T, NC, RW>), dim3(gx, slices), dim3(kDThreads), 0, s, p);
  return hipGetLastError();
}

template <int T, int NC>
hipError_t launch_dense_nc(const GemvArgs& p, hipStream_t s) {
  // 2 rows per wave once the grid has >= 8 bands per CU-round, else 1 (more waves)
  const int64_t rows = (int64_t)p.M * p.ne12 * p.ne13;
  if (rows >= (int64_t)256 * 4 * kDWaves * 2 * 2) return launch_rw<T, NC, 2>(p, s);
  return launch_rw<T, NC, 1>(p, s);
}

template <int T>
hipError_t launch_dense_t(const GemvArgs& p, hipStream_t s) {
  if (p.N <= 1) return launch_dense_nc<T, 1>(p, s);
  if (p.N <= 2) return launch_dense_nc<T, 2>(p, s);
  if (p.N <= 4) return launch_dense_nc<T, 4>(p, s);
  return launch_dense_nc<T, 8>(p, s);
}

}  // namespace

hipError_t launch_gemv_dense(int type, const GemvArgs& p, hipStream_t s) {
  if (p.M == 0 || p.N == 0) return hipSuccess;
  switch (type) {
    case kF32: return launch_dense_t<kF32>(p, s);
    case kF16: return launch_dense_t<kF16>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
