// lamm_quantize_w.hip -- weight (src0) quantizers on the GPU: ggml_quantize_chunk
// (LC/ggml.c:20413) with no importance matrix, i.e. the *_reference row quantizers of
// LC/ggml-quants.c, producing the same bytes:
//   q4_0 :1002-1036   q4_1 :1044-1078   q5_0 :1086-1128   q5_1 :1134-1176
//   q2_K :2039-2114 (make_qkx2_quants :1945-2024, use_mad)
//   q4_K :2744-2849   q5_K :2992-3090 (make_qkx2_quants, weighted squared error)
//   q6_K :3301-3380 (make_qx_quants :1774-1841, rmse_type 1)
// (q8_0 weights are quantize_row_q8_0_reference = lamm_hip_quantize flavour 0.)
// The float sums are order-sensitive, so each thread replays the reference's arithmetic in its
// order: one thread per 32-element block, and for the k-quants one LANE per sub-block (the
// reference searches sub-block by sub-block and only then combines their scales).  This file is built with -ffp-contract=off (Makefile): a fused
// multiply-add would round differently from the reference's separate multiply and add.
// The quantizer prepares weights once (la-benchmark-matmult quantizes outside its timed loop,
// src/la-benchmark-matmult.cpp:294-303).
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
// (use_mad) or err^2, scanning nstep+1 candidate scales.  N is a template constant so the
// per-value arrays live in registers (every loop over the values is unrolled; the float
// operations stay in the reference's order).
template <int N>
__device__ float make_qkx2(int nmax, const float (&x)[N], const float (&w)[N], uint8_t (&L)[N], float* the_min,
                           float rmin, float rdelta, int nstep, bool use_mad) {
  float mn = x[0], mx = x[0];
  float sum_w = w[0], sum_x = sum_w * x[0];
#pragma unroll
  for (int i = 1; i < N; ++i) {
    if (x[i] < mn) mn = x[i];
    if (x[i] > mx) mx = x[i];
    sum_w += w[i];
    sum_x += w[i] * x[i];
  }
  if (mn > 0) mn = 0;
  if (mx == mn) {
#pragma unroll
    for (int i = 0; i < N; ++i) L[i] = 0;
    *the_min = -mn;
    return 0.f;
  }
  float iscale = nmax / (mx - mn);
  float scale = 1 / iscale;
  float best = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const int l = nearest_int(iscale * (x[i] - mn));
    L[i] = (uint8_t)(l < 0 ? 0 : (l > nmax ? nmax : l));
    float diff = scale * L[i] + mn - x[i];
    diff = use_mad ? fabsf(diff) : diff * diff;
    best += w[i] * diff;
  }
  for (int is = 0; is <= nstep; ++is) {
    iscale = (rmin + rdelta * is + nmax) / (mx - mn);
    uint8_t Laux[N];
    float sum_l = 0, sum_l2 = 0, sum_xl = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
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
#pragma unroll
      for (int i = 0; i < N; ++i) {
        float diff = this_scale * Laux[i] + this_min - x[i];
        diff = use_mad ? fabsf(diff) : diff * diff;
        mad += w[i] * diff;
      }
      if (mad < best) {
#pragma unroll
        for (int i = 0; i < N; ++i) L[i] = Laux[i];
        best = mad;
        scale = this_scale;
        mn = this_min;
      }
    }
  }
  *the_min = -mn;
  return scale;
}

// make_qx_quants(n, nmax, x, L, rmse_type = 1, qw = NULL): symmetric fit with x^2 weights
template <int N>
__device__ float make_qx_r1(int nmax, const float (&x)[N], int8_t (&L)[N]) {
  float mx = 0, amax = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    const float ax = fabsf(x[i]);
    if (ax > amax) { amax = ax; mx = x[i]; }
  }
  if (amax < 1e-30f) {
#pragma unroll
    for (int i = 0; i < N; ++i) L[i] = 0;
    return 0.f;
  }
  float iscale = -nmax / mx;
  float sumlx = 0, suml2 = 0;
#pragma unroll
  for (int i = 0; i < N; ++i) {
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
#pragma unroll
    for (int i = 0; i < N; ++i) {
      int l = nearest_int(iscale * x[i]);
      l = l < -nmax ? -nmax : (l > nmax - 1 ? nmax - 1 : l);
      const float w = x[i] * x[i];
      sumlx += w * x[i] * l;
      suml2 += w * l * l;
    }
    if (suml2 > 0 && sumlx * sumlx > best * suml2) {
#pragma unroll
      for (int i = 0; i < N; ++i) {
        const int l = nearest_int(iscale * x[i]);
        L[i] = (int8_t)(nmax + (l < -nmax ? -nmax : (l > nmax - 1 ? nmax - 1 : l)));
      }
      scale = sumlx / suml2;
      best = scale * sumlx;
    }
  }
  return scale;
}

// ------------------------------------------------------------------ k-quants, one lane per sub-block
// The reference's k-quant search runs per sub-block (16 of 16 values for q2_K / q6_K, 8 of 32
// for q4_K / q5_K) and only then combines the sub-blocks' scales, so a super-block maps onto a
// group of SUB lanes: each lane replays its own sub-block's search in the reference's order
// (make_qkx2 / make_qx_r1 above, same float arithmetic), the group combines the scales with
// cross-lane max reductions (order-free: max, and for q6_K the first sub-block of largest
// |scale|), each lane requantizes its own values, and the packed bits -- which interleave
// sub-blocks -- are assembled through LDS.  64 / SUB super-blocks per wave.
template <int T> struct KQ;
template <> struct KQ<kQ2_K> { static constexpr int SUB = 16, N = 16, BPB = 84; };
template <> struct KQ<kQ4_K> { static constexpr int SUB = 8, N = 32, BPB = 144; };
template <> struct KQ<kQ5_K> { static constexpr int SUB = 8, N = 32, BPB = 176; };
template <> struct KQ<kQ6_K> { static constexpr int SUB = 16, N = 16, BPB = 210; };

template <int SUB>
__device__ __forceinline__ float group_max(float v) {   // max over the lane's group of SUB lanes
#pragma unroll
  for (int o = 1; o < SUB; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

constexpr int KQ_NT = 256;

template <int T>
__global__ __launch_bounds__(KQ_NT) void quant_kq_wave(const float* __restrict__ x, int64_t ldx,
                                                       unsigned char* __restrict__ y, int64_t ldy_bytes, int K, int M) {
  using Q = KQ<T>;
  constexpr int SUB = Q::SUB, N = Q::N, SB_PER_WG = KQ_NT / SUB;
  __shared__ uint8_t Ls[SB_PER_WG][256];
  const int nb = K / 256;
  const int t = threadIdx.x, j = t % SUB, gl = t / SUB;   // sub-block, super-block within the WG
  const int64_t g = (int64_t)blockIdx.x * SB_PER_WG + gl;  // super-block index (row-major)
  const bool live = g < (int64_t)nb * M;
  const int64_t row = live ? g / nb : 0, b = live ? g % nb : 0;
  const float* xs = x + row * ldx + b * 256 + N * j;
  unsigned char* yb = y + row * ldy_bytes + b * Q::BPB;
  float xv[N];
#pragma unroll
  for (int i = 0; i < N; ++i) xv[i] = live ? xs[i] : 0.f;
  uint8_t L[N];
  uint8_t* Lg = Ls[gl];

  if constexpr (T == kQ6_K) {
    int8_t Li[N];
    const float scale = make_qx_r1<N>(32, xv, Li);
    // the first sub-block with the largest |scale| gives max_scale (its sign included)
    float ab = fabsf(scale);
    int who = j;
#pragma unroll
    for (int o = 1; o < SUB; o <<= 1) {
      const float ab2 = __shfl_xor(ab, o);
      const int who2 = __shfl_xor(who, o);
      if (ab2 > ab || (ab2 == ab && who2 < who)) { ab = ab2; who = who2; }
    }
    const float max_scale = __shfl(scale, (t & ~(SUB - 1) & 63) + who);
    if (ab == 0.f) {   // !max_abs_scale: the whole super-block is zero, d = +0
      if (live) {
        for (int k = j; k < 210; k += SUB) yb[k] = 0;
        if (j == 0) put16(yb + 208, f2h(0.f));
      }
      return;
    }
    const float iscale = -128.f / max_scale;
    const uint16_t dh = f2h(1 / iscale);
    const int v = nearest_int(iscale * scale);
    const int8_t sc = (int8_t)(v < 127 ? v : 127);
    const float d = hf(dh) * sc;
#pragma unroll
    for (int ii = 0; ii < N; ++ii) {
      if (d) {
        int l = nearest_int(xv[ii] / d);
        l = l < -32 ? -32 : (l > 31 ? 31 : l);
        L[ii] = (uint8_t)(l + 32);
      } else {
        L[ii] = (uint8_t)Li[ii];
      }
    }
#pragma unroll
    for (int ii = 0; ii < N; ++ii) Lg[N * j + ii] = L[ii];
    __syncthreads();
    if (!live) return;
    yb[192 + j] = (unsigned char)sc;
    if (j == 0) put16(yb + 208, dh);
    // ql[128] | qh[64]: 12 bytes per lane
    for (int k = j; k < 192; k += SUB) {
      if (k < 128) {   // ql[64 * h + l] (h: 128-value half, l < 64)
        const int h = k / 64, l = k % 64, base = 128 * h;
        const int lo = l < 32 ? base + l : base + l;   // a (l < 32) or b (l >= 32, = L[base + (l-32) + 32])
        yb[k] = (unsigned char)((Lg[lo] & 0xF) | ((Lg[lo + 64] & 0xF) << 4));
      } else {
        const int q = k - 128, h = q / 32, l = q % 32, base = 128 * h;
        yb[k] = (unsigned char)((Lg[base + l] >> 4) | ((Lg[base + l + 32] >> 4) << 2) | ((Lg[base + l + 64] >> 4) << 4) |
                                ((Lg[base + l + 96] >> 4) << 6));
      }
    }
  } else {
    float w[N];
    float sc_, mn_;
    if constexpr (T == kQ2_K) {
#pragma unroll
      for (int l = 0; l < N; ++l) w[l] = fabsf(xv[l]);
      sc_ = make_qkx2<N>(3, xv, w, L, &mn_, -0.5f, 0.1f, 15, true);
    } else {
      constexpr bool Q5 = T == kQ5_K;
      float sum_x2 = 0;
      for (int l = 0; l < 32; ++l) sum_x2 += xv[l] * xv[l];
      const float av_x = sqrtf(sum_x2 / 32);
#pragma unroll
      for (int l = 0; l < 32; ++l) w[l] = av_x + fabsf(xv[l]);
      sc_ = make_qkx2<N>(Q5 ? 31 : 15, xv, w, L, &mn_, Q5 ? -0.5f : -1.f, 0.1f, Q5 ? 15 : 20, false);
    }
    // max_scale / max_min start at 0 in the reference: max with 0
    // (+0 for non-positive values: fmaxf(-0, +0) may be -0, which would change f16(max / 63))
    const float max_scale = group_max<SUB>(sc_ > 0.f ? sc_ : 0.f), max_min = group_max<SUB>(mn_ > 0.f ? mn_ : 0.f);
    if constexpr (T == kQ2_K) {
      uint8_t scb = 0;
      uint16_t dh, mh;
      if (max_scale > 0) {
        const float iscale = 15.f / max_scale;
        scb = (uint8_t)nearest_int(iscale * sc_);
        dh = f2h(max_scale / 15.f);
      } else {
        dh = f2h(0.f);
      }
      if (max_min > 0) {
        const float iscale = 15.f / max_min;
        scb |= (uint8_t)(nearest_int(iscale * mn_) << 4);
        mh = f2h(max_min / 15.f);
      } else {
        mh = f2h(0.f);
      }
      const float d = hf(dh) * (scb & 0xF);
      if (d) {
        const float dm = hf(mh) * (scb >> 4);
#pragma unroll
        for (int ii = 0; ii < N; ++ii) {
          const int l = nearest_int((xv[ii] + dm) / d);
          L[ii] = (uint8_t)(l < 0 ? 0 : (l > 3 ? 3 : l));
        }
      }
#pragma unroll
      for (int ii = 0; ii < N; ++ii) Lg[N * j + ii] = L[ii];
      __syncthreads();
      if (!live) return;
      yb[j] = scb;
      if (j == 0) {
        put16(yb + 80, dh);
        put16(yb + 82, mh);
      }
      for (int k = j; k < 64; k += SUB) {   // qs[64]: 4 bytes per lane
        const int h = k / 32, l = k % 32, base = 128 * h;
        yb[16 + k] = (unsigned char)(Lg[base + l] | (Lg[base + l + 32] << 2) | (Lg[base + l + 64] << 4) |
                                     (Lg[base + l + 96] << 6));
      }
    } else {
      constexpr bool Q5 = T == kQ5_K;
      constexpr int NMAX = Q5 ? 31 : 15;
      const float inv_scale = max_scale > 0 ? 63.f / max_scale : 0.f;
      const float inv_min = max_min > 0 ? 63.f / max_min : 0.f;
      uint8_t ls = (uint8_t)nearest_int(inv_scale * sc_);
      uint8_t lm = (uint8_t)nearest_int(inv_min * mn_);
      ls = ls < 63 ? ls : 63;
      lm = lm < 63 ? lm : 63;
      const uint16_t dh = f2h(max_scale / 63.f), mh = f2h(max_min / 63.f);
      // get_scale_min_k4 of the packed scales gives back ls / lm exactly (6-bit values)
      const float d = hf(dh) * ls;
      if (d) {
        const float dm = hf(mh) * lm;
#pragma unroll
        for (int ii = 0; ii < N; ++ii) {
          const int l = nearest_int((xv[ii] + dm) / d);
          L[ii] = (uint8_t)(l < 0 ? 0 : (l > NMAX ? NMAX : l));
        }
      }
#pragma unroll
      for (int ii = 0; ii < N; ++ii) Lg[N * j + ii] = L[ii];
      // the 12 scale bytes: every lane's (ls, lm) to the group's first lane
      uint8_t lsv[8], lmv[8];
      const int base_lane = t & 63 & ~(SUB - 1);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        lsv[k] = (uint8_t)__shfl((int)ls, base_lane + k);
        lmv[k] = (uint8_t)__shfl((int)lm, base_lane + k);
      }
      __syncthreads();
      if (!live) return;
      if (j == 0) {
        uint8_t s12[12];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          if (k < 4) {
            s12[k] = lsv[k];
            s12[k + 4] = lmv[k];
          } else {
            s12[k + 4] = (uint8_t)((lsv[k] & 0xF) | ((lmv[k] & 0xF) << 4));
            s12[k - 4] |= (uint8_t)((lsv[k] >> 4) << 6);
            s12[k] |= (uint8_t)((lmv[k] >> 4) << 6);
          }
        }
        put16(yb, dh);
        put16(yb + 2, mh);
#pragma unroll
        for (int k = 0; k < 12; ++k) yb[4 + k] = s12[k];
      }
      unsigned char* qh = yb + 16;
      unsigned char* ql = yb + (Q5 ? 48 : 16);
      for (int k = j; k < 128; k += SUB) {   // ql[128]: 16 bytes per lane
        const int n = 64 * (k / 32), jj = k % 32;
        int l1 = Lg[n + jj], l2 = Lg[n + jj + 32];
        if (Q5) {
          l1 &= 15;
          l2 &= 15;
        }
        ql[k] = (unsigned char)(l1 | (l2 << 4));
      }
      if constexpr (Q5) {
        for (int k = j; k < 32; k += SUB) {   // qh[32]: bit 2i / 2i+1 = the 5th bit of chunk i's two halves
          uint8_t h = 0;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            if (Lg[64 * i + k] > 15) h |= (uint8_t)(1u << (2 * i));
            if (Lg[64 * i + k + 32] > 15) h |= (uint8_t)(2u << (2 * i));
          }
          qh[k] = h;
        }
      }
    }
  }
}

// 32-element formats, one thread per block: block b of row j reads x + j*ldx + b*32, writes
// y + j*ldy_bytes + b*BPB
template <int T>
__global__ __launch_bounds__(64) void quant_w(const float* __restrict__ x, int64_t ldx, unsigned char* __restrict__ y,
                                              int64_t ldy_bytes, int K, int M) {
  constexpr int QK = 32;
  constexpr int BPB = T == kQ4_0 ? 18 : T == kQ4_1 ? 20 : T == kQ5_0 ? 22 : 24;
  const int nb = K / QK;
  const int64_t g = (int64_t)blockIdx.x * 64 + threadIdx.x;
  if (g >= (int64_t)nb * M) return;
  const int64_t j = g / nb, b = g % nb;
  const float* xb = x + j * ldx + b * QK;
  unsigned char* yb = y + j * ldy_bytes + b * BPB;
  if constexpr (T == kQ4_0) quant_sym<4>(xb, yb);
  else if constexpr (T == kQ5_0) quant_sym<5>(xb, yb);
  else if constexpr (T == kQ4_1) quant_affine<4>(xb, yb);
  else quant_affine<5>(xb, yb);
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
  // k-quants: one lane per sub-block, KQ_NT / SUB super-blocks per workgroup
  auto kq = [&](auto kern, int sub) {
    const int per = KQ_NT / sub;
    hipLaunchKernelGGL(kern, dim3((unsigned)((n + per - 1) / per)), dim3(KQ_NT), 0, s, x, ldx, yb, ldy_bytes, K, M);
    return hipGetLastError();
  };
  switch (type) {
    case kQ4_0: hipLaunchKernelGGL(quant_w<kQ4_0>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ4_1: hipLaunchKernelGGL(quant_w<kQ4_1>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ5_0: hipLaunchKernelGGL(quant_w<kQ5_0>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ5_1: hipLaunchKernelGGL(quant_w<kQ5_1>, grid, blk, 0, s, x, ldx, yb, ldy_bytes, K, M); break;
    case kQ2_K: return kq(quant_kq_wave<kQ2_K>, KQ<kQ2_K>::SUB);
    case kQ4_K: return kq(quant_kq_wave<kQ4_K>, KQ<kQ4_K>::SUB);
    case kQ5_K: return kq(quant_kq_wave<kQ5_K>, KQ<kQ5_K>::SUB);
    case kQ6_K: return kq(quant_kq_wave<kQ6_K>, KQ<kQ6_K>::SUB);
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lamm
