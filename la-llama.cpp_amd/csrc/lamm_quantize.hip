// lamm_quantize.hip -- activation (src1) quantizers on the GPU.
//
// ggml's INIT phase quantizes the F32 src1 rows into vec_dot_type blocks on host
// thread 0 (LC/ggml.c:10865-10887).  These kernels produce the same bytes on the
// device, bit-exact with either flavour of the reference:
//   flavour 0 (*_reference): q8_0 LC/ggml-quants.c:1182-1205, q8_1 :1396-1429
//                            (d = amax/127, id = 1/d, roundf)
//   flavour 1 (AVX2 from_float): q8_0 :1280-1330, q8_1 :1505-1575
//                            (d = amax/127.f, id = 127.f/amax, round-half-even)
//   q8_K (one flavour):      :3981-4018 (iscale = -127/max, nearest_int, bsums)
// Max / sum reductions are exact, so lane-parallel order does not change results.
#include "lamm_device.h"
#include "lamm_kernels.h"

namespace lamm {
namespace {

__device__ __forceinline__ void store_u16(unsigned char* p, uint32_t v) {
  *reinterpret_cast<uint16_t*>(p) = (uint16_t)v;  // blocks are 2-byte aligned
}
__device__ __forceinline__ uint32_t f2h(float f) {
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}

// 8 lanes per 32-element block, 4 floats each.
template <bool Q81>
__global__ __launch_bounds__(256) void quant_q8_32(const float* __restrict__ x, int64_t ldx,
                                                  unsigned char* __restrict__ y, int64_t ldy_bytes,
                                                  int K, int N, int flavour) {
  const int64_t gid = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int nb = K / 32;
  const int64_t blk = gid / 8;
  const int sub = (int)(gid % 8);
  const bool valid = blk < (int64_t)nb * N;
  const int64_t j = valid ? blk / nb : 0, b = valid ? blk % nb : 0;
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (valid) v = *reinterpret_cast<const f32x4*>(x + j * ldx + b * 32 + sub * 4);
  float amax = fmaxf(fmaxf(fabsf(v[0]), fabsf(v[1])), fmaxf(fabsf(v[2]), fabsf(v[3])));
  amax = fmaxf(amax, __shfl_xor(amax, 1));
  amax = fmaxf(amax, __shfl_xor(amax, 2));
  amax = fmaxf(amax, __shfl_xor(amax, 4));
  float d, id;
  if (flavour == 1) {
    d = amax / 127.f;
    id = (amax != 0.0f) ? 127.f / amax : 0.0f;
  } else {
    d = amax / 127.f;  // (1 << 7) - 1 promotes to float: same division
    id = d != 0.0f ? 1.0f / d : 0.0f;
  }
  int q[4];
  int sum = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const float s = v[k] * id;
    int r = flavour == 1 ? avx_cvt_i32(__builtin_rintf(s)) : (int)roundf(s);
    const int raw = r;
    r = r > 127 ? 127 : (r < -128 ? -128 : r);
    q[k] = r;
    // AVX2 q8_1: s sums the int32 values before the packs' saturation, wrapping (LC/ggml-quants.c
    // :1562); the scalar reference sums the stored quants
    sum = flavour == 1 ? (int)((uint32_t)sum + (uint32_t)raw) : sum + r;
  }
  if (Q81) {
    sum = (int)((uint32_t)sum + (uint32_t)__shfl_xor(sum, 1));
    sum = (int)((uint32_t)sum + (uint32_t)__shfl_xor(sum, 2));
    sum = (int)((uint32_t)sum + (uint32_t)__shfl_xor(sum, 4));
  }
  if (!valid) return;
  unsigned char* blkp = y + j * ldy_bytes + b * (Q81 ? 36 : 34);
  const uint32_t packed = (q[0] & 0xff) | ((q[1] & 0xff) << 8) | ((q[2] & 0xff) << 16) | ((uint32_t)(q[3] & 0xff) << 24);
  unsigned char* qs = blkp + (Q81 ? 4 : 2) + sub * 4;
  store_u16(qs, packed & 0xffff);
  store_u16(qs + 2, packed >> 16);
  if (sub == 0) {
    store_u16(blkp, f2h(d));
    if (Q81) store_u16(blkp + 2, f2h((float)sum * d));
  }
}

__device__ __forceinline__ int nearest_int(float f) {
  const float v = f + 12582912.f;
  return (int)(__builtin_bit_cast(uint32_t, v) & 0x007fffff) - 0x00400000;
}

// one wave per 256-element super-block, 4 floats per lane
__global__ __launch_bounds__(256) void quant_q8_K(const float* __restrict__ x, int64_t ldx,
                                                 unsigned char* __restrict__ y, int64_t ldy_bytes,
                                                 int K, int N) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = ((int64_t)blockIdx.x * 256 + threadIdx.x) / 64;
  const int nb = K / 256;
  if (wid >= (int64_t)nb * N) return;
  const int64_t j = wid / nb, b = wid % nb;
  const f32x4 v = *reinterpret_cast<const f32x4*>(x + j * ldx + b * 256 + lane * 4);
  // first element of largest magnitude (reference scans with strict '>')
  float am = -1.f;
  int ai = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k)
    if (fabsf(v[k]) > am) { am = fabsf(v[k]); ai = lane * 4 + k; }
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const float om = __shfl_xor(am, o);
    const int oi = __shfl_xor(ai, o);
    if (om > am || (om == am && oi < ai)) { am = om; ai = oi; }
  }
  const float vmax = __shfl(v[ai & 3], ai >> 2);  // lane ai/4 holds x[ai]
  unsigned char* blkp = y + j * ldy_bytes + b * 292;
  int q[4];
  float d = 0.f;
  if (am == 0.f) {
    q[0] = q[1] = q[2] = q[3] = 0;
  } else {
    const float iscale = -127.f / vmax;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int r = nearest_int(iscale * v[k]);
      q[k] = r < 127 ? r : 127;
    }
    d = 1.f / iscale;
  }
  int s = q[0] + q[1] + q[2] + q[3];
  s += __shfl_xor(s, 1);
  s += __shfl_xor(s, 2);  // 4 lanes = 16 elements = one bsum group
  const uint32_t packed = (q[0] & 0xff) | ((q[1] & 0xff) << 8) | ((q[2] & 0xff) << 16) | ((uint32_t)(q[3] & 0xff) << 24);
  *reinterpret_cast<uint32_t*>(blkp + 4 + lane * 4) = packed;  // q8_K is dword aligned
  if ((lane & 3) == 0) *reinterpret_cast<int16_t*>(blkp + 260 + (lane >> 2) * 2) = (int16_t)s;
  if (lane == 0) *reinterpret_cast<float*>(blkp) = d;
}

// F16 activations: ggml_fp32_to_fp16_row (LC/ggml.c), round-to-nearest-even per
// element -- v_cvt_f16_f32 in the default round mode, subnormals kept
__global__ __launch_bounds__(256) void cvt_f16(const float* __restrict__ x, int64_t ldx, unsigned char* __restrict__ y,
                                               int64_t ldy_bytes, int K, int N) {
  const int64_t it = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (it >= (int64_t)K * N) return;
  const int64_t j = it / K, e = it % K;
  const _Float16 h = (_Float16)x[j * ldx + e];
  *reinterpret_cast<_Float16*>(y + j * ldy_bytes + 2 * e) = h;
}

}  // namespace

hipError_t launch_quantize(int vec_type, int flavour, const float* x, int64_t ldx, void* y,
                           int64_t ldy_bytes, int K, int N, hipStream_t s) {
  unsigned char* yb = static_cast<unsigned char*>(y);
  if (vec_type == kQ8_0 || vec_type == kQ8_1) {
    const int64_t threads = (int64_t)(K / 32) * N * 8;
    const int grid = (int)((threads + 255) / 256);
    if (grid == 0) return hipSuccess;
    if (vec_type == kQ8_0)
      hipLaunchKernelGGL(quant_q8_32<false>, dim3(grid), dim3(256), 0, s, x, ldx, yb, ldy_bytes, K, N, flavour);
    else
      hipLaunchKernelGGL(quant_q8_32<true>, dim3(grid), dim3(256), 0, s, x, ldx, yb, ldy_bytes, K, N, flavour);
    return hipGetLastError();
  }
  if (vec_type == kQ8_K) {
    const int64_t threads = (int64_t)(K / 256) * N * 64;
    const int grid = (int)((threads + 255) / 256);
    if (grid == 0) return hipSuccess;
    hipLaunchKernelGGL(quant_q8_K, dim3(grid), dim3(256), 0, s, x, ldx, yb, ldy_bytes, K, N);
    return hipGetLastError();
  }
  if (vec_type == kF16) {
    const int64_t n = (int64_t)K * N;
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(cvt_f16, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, x, ldx, yb, ldy_bytes, K, N);
    return hipGetLastError();
  }
  return hipErrorInvalidValue;
}

}  // namespace lamm
