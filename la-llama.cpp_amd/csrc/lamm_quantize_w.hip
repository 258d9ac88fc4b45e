// lamm_quantize_w.hip -- weight (src0) quantizers on the GPU: ggml_quantize_chunk
// (LC/ggml.c:20413) with no importance matrix, i.e. the *_reference row quantizers of
// LC/ggml-quants.c, producing the same bytes:
//   q4_0 :1002-1036   q4_1 :1044-1078   q5_0 :1086-1128   q5_1 :1134-1176
//   q2_K :2039-2114 (make_qkx2_quants :1945-2024, use_mad)
//   q4_K :2744-2849   q5_K :2992-3090 (make_qkx2_quants, weighted squared error)
//   q6_K :3301-3380 (make_qx_quants :1774-1841, rmse_type 1)
// (q8_0 weights are quantize_row_q8_0_reference = lamm_hip_quantize flavour 0.)
// One thread per block: the k-quant searches are sequential per super-block in the reference
// and their float sums are order-sensitive, so each thread replays one block's arithmetic in
// the reference's order.  This file is built with -ffp-contract=off (Makefile): a fused
// multiply-add would round differently from the reference's separate multiply and add.
// The quantizer prepares weights once (la-benchmark-matmult quantizes outside its timed loop,
// src/la-benchmark-matmult.cpp:294-303), so simplicity beats speed here.
#include "lamm_device.h"
#include "lamm_formats.h"
#include "lamm_kernels.h"

namespace lamm {
namespace {

// The register barrier keeps the f32 -> f16 conversion a separate v_cvt_f16_f32: without it the
// compiler folds `d = max / -8; f16(d)` into v_fma_mixlo_f16(max, -0.125, +0), whose +0 addend
// turns the reference's -0.0 scale of an all-zero block into +0.0 (0x0000 instead of 0x8000).
__device__ __forceinline__ uint16_t f2h(float f) {
  asm volatile("" : "+v"(f));
  return __builtin_bit_cast(uint16_t, (_Float16)f);
}
__device__ __forceinline__ float hf(uint16_t h) { return (float)__builtin_bit_cast(_Float16, h); }

__device__ __forceinline__ int nearest_int(float f) {   // LC/ggml-quants.c:1766-1772
  const float v = f + 12582912.f;
  return (int)(__builtin_bit_cast(uint32_t, v) & 0x007fffff) - 0x00400000;
}

__device__ __forceinline__ void put16(unsigned char* p, uint16_t v) { p[0] = (unsigned char)v; p[1] = (unsigned char)(v >> 8); }

// ------------------------------------------------------------------ 32-element blocks
// q4_0 / q5_0: symmetric, d = (signed absmax) / -2^(bits-1)
template <int BITS>
__device__ void quant_sym(const float* x, unsigned char* y) {
  float amax = 0.0f, mx = 0.0f;
  for (int j = 0; j < 32; ++j) {
    const float v = x[j];
    if (amax < fabsf(v)) { amax = fabsf(v); mx = v; }
  }
  const float d = mx / (BITS == 4 ? -8 : -16);
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  put16(y, f2h(d));
  unsigned char* qs = y + (BITS == 4 ? 2 : 6);
  uint32_t qh = 0;
  for (int j = 0; j < 16; ++j) {
    const float x0 = x[j] * id, x1 = x[16 + j] * id;
    constexpr float OFF = BITS == 4 ? 8.5f : 16.5f;
    constexpr int TOP = BITS == 4 ? 15 : 31;
    const int8_t i0 = (int8_t)(int)(x0 + OFF), i1 = (int8_t)(int)(x1 + OFF);
    const uint8_t v0 = (uint8_t)(i0 < TOP ? i0 : TOP), v1 = (uint8_t)(i1 < TOP ? i1 : TOP);
    qs[j] = (unsigned char)((v0 & 0x0f) | ((v1 & 0x0f) << 4));
    if (BITS == 5) {
      qh |= (uint32_t)((v0 & 0x10u) >> 4) << j;
      qh |= (uint32_t)((v1 & 0x10u) >> 4) << (j + 16);
    }
  }
  if (BITS == 5) { put16(y + 2, (uint16_t)qh); put16(y + 4, (uint16_t)(qh >> 16)); }
}

// q4_1 / q5_1: affine, d = (max - min) / (2^bits - 1), m = min
template <int BITS>
__device__ void quant_affine(const float* x, unsigned char* y) {
  float mn = 3.402823466e+38f, mx = -3.402823466e+38f;
  for (int j = 0; j < 32; ++j) {
    const float v = x[j];
    if (v < mn) mn = v;
    if (v > mx) mx = v;
  }
  const float d = (mx - mn) / ((1 << BITS) - 1);
  const float id = d != 0.0f ? 1.0f / d : 0.0f;
  put16(y, f2h(d));
  put16(y + 2, f2h(mn));
  unsigned char* qs = y + (BITS == 4 ? 4 : 8);
  uint32_t qh = 0;
  for (int j = 0; j < 16; ++j) {
    const float x0 = (x[j] - mn) * id, x1 = (x[16 + j] - mn) * id;
    uint8_t v0, v1;
    if (BITS == 4) {
      const int8_t i0 = (int8_t)(int)(x0 + 0.5f), i1 = (int8_t)(int)(x1 + 0.5f);
      v0 = (uint8_t)(i0 < 15 ? i0 : 15);
      v1 = (uint8_t)(i1 < 15 ? i1 : 15);
    } else {   // the q5_1 reference does not clamp
      v0 = (uint8_t)(int)(x0 + 0.5f);
      v1 = (uint8_t)(int)(x1 + 0.5f);
      qh |= (uint32_t)((v0 & 0x10u) >> 4) << j;
      qh |= (uint32_t)((v1 & 0x10u) >> 4) << (j + 16);
    }
    qs[j] = (unsigned char)((v0 & 0x0f) | ((v1 & 0x0f) << 4));
  }
  if (BITS == 5) { put16(y + 4, (uint16_t)qh); put16(y + 6, (uint16_t)(qh >> 16)); }
}

// ------------------------------------------------------------------ k-quant searches
// make_qkx2_quants: affine fit of n values to [0, nmax] minimising the weighted |err|
// (use_mad) or err^2, scanning nstep+1 candidate scales
__device__ float make_qkx2(int n, int nmax, const float* x, const float* w, uint8_t* L, float* the_min,
                           uint8_t* Laux, float rmin, float rdelta, int nstep, bool use_mad) {
  float mn = x[0], mx = x[0];
  float sum_w = w[0], sum_x = sum_w * x[0];
  for (int i = 1; i < n; ++i) {
    if (x[i] < mn) mn = x[i];
    if (x[i] > mx) mx = x[i];
    sum_w += w[i];
    sum_x += w[i] * x[i];
  }
  if (mn > 0) mn = 0;
  if (mx == mn) {
    for (int i = 0; i < n; ++i) L[i] = 0;
    *the_min = -mn;
    return 0.f;
  }
  float iscale = nmax / (mx - mn);
  float scale = 1 / iscale;
  float best = 0;
  for (int i = 0; i < n; ++i) {
    const int l = nearest_int(iscale * (x[i] - mn));
    L[i] = (uint8_t)(l < 0 ? 0 : (l > nmax ? nmax : l));
    float diff = scale * L[i] + mn - x[i];
    diff = use_mad ? fabsf(diff) : diff * diff;
    best += w[i] * diff;
  }
  for (int is = 0; is <= nstep; ++is) {
    iscale = (rmin + rdelta * is + nmax) / (mx - mn);
    float sum_l = 0, sum_l2 = 0, sum_xl = 0;
    for (int i = 0; i < n; ++i) {
      int l = nearest_int(iscale * (x[i] - mn));
      l = l < 0 ? 0 : (l > nmax ? nmax : l);
      Laux[i] = (uint8_t)l;
      sum_l += w[i] * l;
      sum_l2 += w[i] * l * l;
      sum_xl += w[i] * l * x[i];
    }
    const float D = sum_w * sum_l2 - sum_l * sum_l;
    if (D > 0) {
      float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
      float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
      if (this_min > 0) {
        this_min = 0;
        this_scale = sum_xl / sum_l2;
      }
      float mad = 0;
      for (int i = 0; i < n; ++i) {
        float diff = this_scale * Laux[i] + this_min - x[i];
        diff = use_mad ? fabsf(diff) : diff * diff;
        mad += w[i] * diff;
      }
      if (mad < best) {
        for (int i = 0; i < n; ++i) L[i] = Laux[i];
        best = mad;
        scale = this_scale;
        mn = this_min;
      }
    }
  }
  *the_min = -mn;
  return scale;
}

// q2_K (84 B: scales[16] | qs[64] | d | dmin)
__device__ void quant_q2_K(const float* x, unsigned char* y) {
  uint8_t L[256], Laux[16];
  float w[16], mins[16], scales[16];
  unsigned char* sc = y;
  float max_scale = 0, max_min = 0;
  for (int j = 0; j < 16; ++j) {
    for (int l = 0; l < 16; ++l) w[l] = fabsf(x[16 * j + l]);
    scales[j] = make_qkx2(16, 3, x + 16 * j, w, L + 16 * j, &mins[j], Laux, -0.5f, 0.1f, 15, true);
    if (scales[j] > max_scale) max_scale = scales[j];
    if (mins[j] > max_min) max_min = mins[j];
  }
  uint16_t dh, mh;
  if (max_scale > 0) {
    const float iscale = 15.f / max_scale;
    for (int j = 0; j < 16; ++j) sc[j] = (uint8_t)nearest_int(iscale * scales[j]);
    dh = f2h(max_scale / 15.f);
  } else {
    for (int j = 0; j < 16; ++j) sc[j] = 0;
    dh = f2h(0.f);
  }
  if (max_min > 0) {
    const float iscale = 15.f / max_min;
    for (int j = 0; j < 16; ++j) sc[j] |= (uint8_t)(nearest_int(iscale * mins[j]) << 4);
    mh = f2h(max_min / 15.f);
  } else {
    mh = f2h(0.f);
  }
  put16(y + 80, dh);
  put16(y + 82, mh);
  for (int j = 0; j < 16; ++j) {
    const float d = hf(dh) * (sc[j] & 0xF);
    if (!d) continue;
    const float dm = hf(mh) * (sc[j] >> 4);
    for (int ii = 0; ii < 16; ++ii) {
      const int l = nearest_int((x[16 * j + ii] + dm) / d);
      L[16 * j + ii] = (uint8_t)(l < 0 ? 0 : (l > 3 ? 3 : l));
    }
  }
  for (int j = 0; j < 256; j += 128)
    for (int l = 0; l < 32; ++l)
      y[16 + j / 4 + l] = (unsigned char)(L[j + l] | (L[j + l + 32] << 2) | (L[j + l + 64] << 4) | (L[j + l + 96] << 6));
}

// q4_K (144 B) / q5_K (176 B): 8 sub-blocks of 32, 6-bit scales and mins
template <bool Q5>
__device__ void quant_q45_K(const float* x, unsigned char* y) {
  constexpr int NMAX = Q5 ? 31 : 15;
  uint8_t L[256], Laux[32];
  float w[32], mins[8], scales[8];
  float max_scale = 0, max_min = 0;
  for (int j = 0; j < 8; ++j) {
    float sum_x2 = 0;
    for (int l = 0; l < 32; ++l) sum_x2 += x[32 * j + l] * x[32 * j + l];
    const float av_x = sqrtf(sum_x2 / 32);
    for (int l = 0; l < 32; ++l) w[l] = av_x + fabsf(x[32 * j + l]);
    scales[j] = make_qkx2(32, NMAX, x + 32 * j, w, L + 32 * j, &mins[j], Laux, Q5 ? -0.5f : -1.f, 0.1f,
                          Q5 ? 15 : 20, false);
    if (scales[j] > max_scale) max_scale = scales[j];
    if (mins[j] > max_min) max_min = mins[j];
  }
  const float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
  const float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
  uint8_t s12[12];
  for (int j = 0; j < 8; ++j) {
    uint8_t ls = (uint8_t)nearest_int(inv_scale * scales[j]);
    uint8_t lm = (uint8_t)nearest_int(inv_min * mins[j]);
    ls = ls < 63 ? ls : 63;
    lm = lm < 63 ? lm : 63;
    if (j < 4) {
      s12[j] = ls;
      s12[j + 4] = lm;
    } else {
      s12[j + 4] = (uint8_t)((ls & 0xF) | ((lm & 0xF) << 4));
      s12[j - 4] |= (uint8_t)((ls >> 4) << 6);
      s12[j] |= (uint8_t)((lm >> 4) << 6);
    }
  }
  const uint16_t dh = f2h(max_scale / 63.f), mh = f2h(max_min / 63.f);
  for (int j = 0; j < 8; ++j) {   // get_scale_min_k4, LC/ggml-quants.c:2027-2034
    uint8_t sc, m;
    if (j < 4) {
      sc = s12[j] & 63;
      m = s12[j + 4] & 63;
    } else {
      sc = (uint8_t)((s12[j + 4] & 0xF) | ((s12[j - 4] >> 6) << 4));
      m = (uint8_t)((s12[j + 4] >> 4) | ((s12[j] >> 6) << 4));
    }
    const float d = hf(dh) * sc;
    if (!d) continue;
    const float dm = hf(mh) * m;
    for (int ii = 0; ii < 32; ++ii) {
      const int l = nearest_int((x[32 * j + ii] + dm) / d);
      L[32 * j + ii] = (uint8_t)(l < 0 ? 0 : (l > NMAX ? NMAX : l));
    }
  }
  put16(y, dh);
  put16(y + 2, mh);
  for (int k = 0; k < 12; ++k) y[4 + k] = s12[k];
  unsigned char* qh = y + 16;
  unsigned char* ql = y + (Q5 ? 48 : 16);
  if (Q5)
    for (int k = 0; k < 32; ++k) qh[k] = 0;
  uint8_t m1 = 1, m2 = 2;
  for (int n = 0; n < 256; n += 64) {
    for (int j = 0; j < 32; ++j) {
      int l1 = L[n + j], l2 = L[n + j + 32];
      if (Q5) {
        if (l1 > 15) { l1 -= 16; qh[j] |= m1; }
        if (l2 > 15) { l2 -= 16; qh[j] |= m2; }
      }
      ql[j] = (unsigned char)(l1 | (l2 << 4));
    }
    m1 <<= 2;
    m2 <<= 2;
    ql += 32;
  }
}

// make_qx_quants(n, nmax, x, L, rmse_type = 1, qw = NULL): symmetric fit with x^2 weights
__device__ float make_qx_r1(int n, int nmax, const float* x, int8_t* L) {
  float mx = 0, amax = 0;
  for (int i = 0; i < n; ++i) {
    const float ax = fabsf(x[i]);
    if (ax > amax) { amax = ax; mx = x[i]; }
  }
  if (amax < 1e-30f) {
    for (int i = 0; i < n; ++i) L[i] = 0;
    return 0.f;
  }
  float iscale = -nmax / mx;
  float sumlx = 0, suml2 = 0;
  for (int i = 0; i < n; ++i) {
    int l = nearest_int(iscale * x[i]);
    l = l < -nmax ? -nmax : (l > nmax - 1 ? nmax - 1 : l);
    L[i] = (int8_t)(l + nmax);
    const float w = x[i] * x[i];
    sumlx += w * x[i] * l;
    suml2 += w * l * l;
  }
  float scale = sumlx / suml2;
  float best = scale * sumlx;
  for (int is = -9; is <= 9; ++is) {
    if (is == 0) continue;
    iscale = -(nmax + 0.1f * is) / mx;
    sumlx = suml2 = 0;
    for (int i = 0; i < n; ++i) {
      int l = nearest_int(iscale * x[i]);
      l = l < -nmax ? -nmax : (l > nmax - 1 ? nmax - 1 : l);
      const float w = x[i] * x[i];
      sumlx += w * x[i] * l;
      suml2 += w * l * l;
    }
    if (suml2 > 0 && sumlx * sumlx > best * suml2) {
      for (int i = 0; i < n; ++i) {
        const int l = nearest_int(iscale * x[i]);
        L[i] = (int8_t)(nmax + (l < -nmax ? -nmax : (l > nmax - 1 ? nmax - 1 : l)));
      }
      scale = sumlx / suml2;
      best = scale * sumlx;
    }
  }
  return scale;
}

// q6_K (210 B: ql[128] | qh[64] | scales[16] | d)
__device__ void quant_q6_K(const float* x, unsigned char* y) {
  int8_t L[256];
  float scales[16];
  float max_scale = 0, max_abs_scale = 0;
  for (int ib = 0; ib < 16; ++ib) {
    const float scale = make_qx_r1(16, 32, x + 16 * ib, L + 16 * ib);
    scales[ib] = scale;
    const float abs_scale = fabsf(scale);
    if (abs_scale > max_abs_scale) {
      max_abs_scale = abs_scale;
      max_scale = scale;
    }
  }
  if (!max_abs_scale) {
    for (int k = 0; k < 210; ++k) y[k] = 0;
    put16(y + 208, f2h(0.f));
    return;
  }
  const float iscale = -128.f / max_scale;
  const uint16_t dh = f2h(1 / iscale);
  int8_t sc[16];
  for (int ib = 0; ib < 16; ++ib) {
    const int v = nearest_int(iscale * scales[ib]);
    sc[ib] = (int8_t)(v < 127 ? v : 127);
  }
  for (int j = 0; j < 16; ++j) {
    const float d = hf(dh) * sc[j];
    if (!d) continue;
    for (int ii = 0; ii < 16; ++ii) {
      int l = nearest_int(x[16 * j + ii] / d);
      l = l < -32 ? -32 : (l > 31 ? 31 : l);
      L[16 * j + ii] = (int8_t)(l + 32);
    }
  }
  unsigned char* ql = y;
  unsigned char* qh = y + 128;
  for (int j = 0; j < 256; j += 128) {
    for (int l = 0; l < 32; ++l) {
      const uint8_t a = (uint8_t)L[j + l], b = (uint8_t)L[j + l + 32], c = (uint8_t)L[j + l + 64],
                    e = (uint8_t)L[j + l + 96];
      ql[l] = (unsigned char)((a & 0xF) | ((c & 0xF) << 4));
      ql[l + 32] = (unsigned char)((b & 0xF) | ((e & 0xF) << 4));
      qh[l] = (unsigned char)((a >> 4) | ((b >> 4) << 2) | ((c >> 4) << 4) | ((e >> 4) << 6));
    }
    ql += 64;
    qh += 32;
  }
  for (int k = 0; k < 16; ++k) y[192 + k] = (unsigned char)sc[k];
  put16(y + 208, dh);
}

// one thread per block: block b of row j reads x + j*ldx + b*QK, writes y + j*ldy_bytes + b*BPB
template <int T>
__global__ __launch_bounds__(64) void quant_w(const float* __restrict__ x, int64_t ldx, unsigned char* __restrict__ y,
                                              int64_t ldy_bytes, int K, int M) {
  constexpr int QK = T == kQ2_K || T == kQ4_K || T == kQ5_K || T == kQ6_K ? 256 : 32;
  constexpr int BPB = T == kQ4_0 ? 18 : T == kQ4_1 ? 20 : T == kQ5_0 ? 22 : T == kQ5_1 ? 24 : T == kQ2_K ? 84
                    : T == kQ4_K ? 144 : T == kQ5_K ? 176 : 210;
  const int nb = K / QK;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= (int64_t)nb * M) return;
  const int64_t j = g / nb, b = g % nb;
  const float* xb = x + j * ldx + b * QK;
  unsigned char* yb = y + j * ldy_bytes + b * BPB;
  if constexpr (T == kQ4_0) quant_sym<4>(xb, yb);
  else if constexpr (T == kQ5_0) quant_sym<5>(xb, yb);
  else if constexpr (T == kQ4_1) quant_affine<4>(xb, yb);
  else if constexpr (T == kQ5_1) quant_affine<5>(xb, yb);
  else if constexpr (T == kQ2_K) quant_q2_K(xb, yb);
  else if constexpr (T == kQ4_K) quant_q45_K<false>(xb, yb);
  else if constexpr (T == kQ5_K) quant_q45_K<true>(xb, yb);
  else quant_q6_K(xb, yb);
}

}  // namespace

bool quantize_weights_supported(int type) {
  return type == kQ4_0 || type == kQ4_1 || type == kQ5_0 || type == kQ5_1 || type == kQ2_K || type == kQ4_K ||
         type == kQ5_K || type == kQ6_K;
}

hipError_t launch_quantize_weights(int type, const float* x, int64_t ldx, void* y, int64_t ldy_bytes, int K, int M,
                                   hipStream_t s) {
  unsigned char* yb = static_cast<unsigned char*>(y);
  const int64_t n = (int64_t)(K / block_elems(type)) * M;
  if (n == 0) return hipSuccess;
  const dim3 grid((unsigned)((n + 63) / 64)), blk(64);
  switch (type) {
    case kQ4_0: hipLaunchKernelGGL(quant_w<kQ4_0>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ4_1: hipLaunchKernelGGL(quant_w<kQ4_1>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ5_0: hipLaunchKernelGGL(quant_w<kQ5_0>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ5_1: hipLaunchKernelGGL(quant_w<kQ5_1>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ2_K: hipLaunchKernelGGL(quant_w<kQ2_K>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ4_K: hipLaunchKernelGGL(quant_w<kQ4_K>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ5_K: hipLaunchKernelGGL(quant_w<kQ5_K>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ6_K: hipLaunchKernelGGL(quant_w<kQ6_K>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lamm
