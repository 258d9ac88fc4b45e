// lamm_host_quant.cpp -- the activation quantizer ggml's INIT phase runs on x86, restated for the
// boundary's host side: F32 rows -> q8_0 / q8_1 blocks exactly as ggml's AVX2 from_float writes
// them (LC/ggml-quants.c:1277-1330 quantize_row_q8_0, :1505-1575 quantize_row_q8_1, the
// `__AVX2__ || __AVX__` branches; the same bytes lamm_quantize.hip's AVX2 flavour writes on the
// device):
//   amax = max |x| over the 32 values, d = amax / 127 (stored as fp16, round to nearest even),
//   id = amax != 0 ? 127 / amax : 0, q = round-half-even(x * id) (_mm256_round_ps NEAREST), then
//   the int32 -> int8 pack saturation; q8_1 also stores s = fp16(d * sum q).
// Used by prefill calls whose activations ggml's pool threads quantize in parallel before the
// upload (lamm_hip.cpp pool jobs): 2.2 MiB of q8_0 rows cross PCIe instead of 8 MiB of F32.
// host_stream_copy: the pool's C scatter (LAMM_HIP_POOL bit 2) with non-temporal stores.
// Built with -ffp-contract=off: x * id must round before the rounding step, as the AVX2 code's
// separate multiply does.
#include <immintrin.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>

#include "../../include/lamm_hip.h"
#include "lamm_formats.h"

namespace {

inline uint16_t to_f16(float v) { return __builtin_bit_cast(uint16_t, (_Float16)v); }

// x * id rounded to the nearest integer, ties to even: adding 1.5 * 2^23 leaves the integer part
// in the low mantissa bits under the default rounding mode (|v| <= 2^22; here |v| <= 127.x)
typedef float f8 __attribute__((ext_vector_type(8)));
typedef int32_t i8 __attribute__((ext_vector_type(8)));
typedef int8_t c8 __attribute__((ext_vector_type(8)));

// 8-wide vectors: one AVX2 register in the x86-64-v3 clone (whose F16C converts d and s), two SSE
// ones otherwise
__attribute__((target_clones("arch=x86-64-v3", "default"))) void quant_q8(const float* __restrict x, unsigned char* __restrict y,
                                                                 int64_t nb, bool sum) {
  const int OFF = sum ? 4 : 2, BPB = sum ? 36 : 34;
#pragma clang loop unroll_count(4)
  for (int64_t i = 0; i < nb; ++i, x += 32, y += BPB) {
    f8 v[4], a[4];
    for (int k = 0; k < 4; ++k) {
      memcpy(&v[k], x + 8 * k, 32);
      a[k] = __builtin_bit_cast(f8, __builtin_bit_cast(i8, v[k]) & 0x7fffffff);   // |x|
    }
    const f8 m = __builtin_elementwise_max(__builtin_elementwise_max(a[0], a[1]), __builtin_elementwise_max(a[2], a[3]));
    const float amax = __builtin_reduce_max(m);   // max is exact: any order gives the same amax
    // inf / NaN anywhere in the block (|x| as an integer above the largest finite float's)
    const i8 big = __builtin_elementwise_max(__builtin_elementwise_max(__builtin_bit_cast(i8, a[0]), __builtin_bit_cast(i8, a[1])),
                                             __builtin_elementwise_max(__builtin_bit_cast(i8, a[2]), __builtin_bit_cast(i8, a[3])));
    const bool finite = __builtin_reduce_max(big) < 0x7f800000;
    float d = amax / 127.f;
    float id = amax != 0.0f ? 127.f / amax : 0.0f;
    int8_t q[32];
    int s = 0;
    if (finite && id < INFINITY) {   // |x id| <= 127 + 1 ulp: no saturation
      i8 rs = 0;
      for (int k = 0; k < 4; ++k) {
        const f8 t = v[k] * id + 12582912.f;   // two roundings (-ffp-contract=off): the product, then the integer
        const i8 r = (__builtin_bit_cast(i8, t) & 0x007fffff) - 0x00400000;
        rs += r;
        const c8 c = __builtin_convertvector(r, c8);
        memcpy(q + 8 * k, &c, 8);
      }
      if (sum) s = __builtin_reduce_add(rs);
    } else {
      // inf / NaN in the block, or 0 < amax < ~3.7e-37 (id = inf): the AVX2 code step by step
      //  -- its amax reduction (_mm_max_ps(a, b) = a > b ? a : b, so a NaN's position
      // decides), then _mm256_cvtps_epi32 (NaN / out of range -> INT_MIN) and the packs' saturation;
      // q8_1's s sums the int32 values before the packs, wrapping (oracle/lamm_oracle.c quant_q8)
      float mx[8], q4[4], r2[4];
      for (int i = 0; i < 8; ++i) mx[i] = std::fabs(x[i]);
      for (int u = 1; u < 4; ++u)
        for (int i = 0; i < 8; ++i) {
          const float b = std::fabs(x[8 * u + i]);
          mx[i] = mx[i] > b ? mx[i] : b;
        }
      for (int i = 0; i < 4; ++i) q4[i] = mx[4 + i] > mx[i] ? mx[4 + i] : mx[i];
      for (int i = 0; i < 4; ++i) {
        const float b = q4[2 + (i & 1)];
        r2[i] = q4[i] > b ? q4[i] : b;
      }
      const float am = r2[0] > r2[1] ? r2[0] : r2[1];
      d = am / 127.f;
      id = am != 0.0f ? 127.f / am : 0.0f;
      uint32_t ws = 0;
      for (int j = 0; j < 32; ++j) {
        const float r = std::nearbyint(x[j] * id);
        const int32_t iv = (r >= -2147483648.f && r < 2147483648.f) ? (int32_t)r : INT32_MIN;
        ws += (uint32_t)iv;
        q[j] = (int8_t)(iv > 127 ? 127 : iv < -128 ? -128 : iv);
      }
      s = (int32_t)ws;
    }
    const uint16_t dh = to_f16(d);
    memcpy(y, &dh, 2);
    memcpy(y + OFF, q, 32);
    if (sum) {
      const uint16_t sh = to_f16(d * (float)s);
      memcpy(y + 2, &sh, 2);
    }
  }
}

// n bytes with non-temporal stores where the destination is 32-byte aligned (no read for ownership
// of lines the copy overwrites whole; ggml's dst is cold in the host caches)
__attribute__((target("avx2"))) void stream_copy_avx2(unsigned char* __restrict d, const unsigned char* __restrict s,
                                                        size_t n) {
  const size_t head = std::min(n, (size_t)((32 - ((uintptr_t)d & 31)) & 31));
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  size_t i = 0;
  for (; i + 128 <= n; i += 128) {
    const __m256i a = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i));
    const __m256i b = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 32));
    const __m256i c = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 64));
    const __m256i e = _mm256_loadu_si256(reinterpret_cast<const __m256i*>(s + i + 96));
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i), a);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 32), b);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 64), c);
    _mm256_stream_si256(reinterpret_cast<__m256i*>(d + i + 96), e);
  }
  memcpy(d + i, s + i, n - i);
  _mm_sfence();
}

}  // namespace

namespace lamm {

void host_stream_copy(void* dst, const void* src, size_t n) {
  static const bool avx2 = __builtin_cpu_supports("avx2");
  if (avx2) stream_copy_avx2(static_cast<unsigned char*>(dst), static_cast<const unsigned char*>(src), n);
  else memcpy(dst, src, n);
}

bool host_quant_supported(int type) { return type == kQ8_0 || type == kQ8_1; }

void host_quantize_row(int type, const float* x, void* y, int64_t nblk) {
  quant_q8(x, static_cast<unsigned char*>(y), nblk, type == kQ8_1);
}

}  // namespace lamm

extern "C" int lamm_hip_quantize_host(int type, const float* x, void* y, int64_t k) {
  if (!lamm::host_quant_supported(type)) return LAMM_ERR_TYPE;
  if (k < 0 || k % 32 || (k && (!x || !y))) return LAMM_ERR_SHAPE;
  lamm::host_quantize_row(type, x, y, k / 32);
  return LAMM_OK;
}
