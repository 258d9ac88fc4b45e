/*
 * lamm_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the thing
 * measured or shipped).  Plain-C restatement of the reference arithmetic on the
 * lamm_* mul_mat path:
 *
 *   * block formats            LC/ggml-common.h:144-225, 316-321
 *   * weight quantizers        LC/ggml-quants.c:1002-1180 (q4_0..q5_1 *_reference,
 *                              reached via ggml_quantize_chunk with imatrix==NULL,
 *                              :3569-3583), :1182-1205 (q8_0), :2039-2114 (q2_K,
 *                              with make_qkx2_quants :1945-2029, nearest_int :1767)
 *   * activation quantizers    q8_0 :1182-1205 (ref) / :1280-1330 (AVX2 from_float),
 *                              q8_1 :1396-1429 (ref) / :1505-1575 (AVX2),
 *                              q8_K :3981-4018
 *   * scalar vec_dot           q4_0 :4451-4469, q4_1 :4700-4718, q5_0 :4985-5008,
 *                              q5_1 :5290-5313, q8_0 :5300-5313, q2_K :5820-5860,
 *                              q4_K :7301-7358, q5_K :7968-8029, q6_K :8695-8738
 *                              (the SURVEY §8f "next" formats; no quantizer restated:
 *                              their test inputs are the reference's own bytes or
 *                              random bytes, for which vec_dot is equally defined)
 *                              f32 LC/ggml.c:1576-1581 (double accumulation),
 *                              f16 LC/ggml.c:1589-1629 (scalar branch: double accumulation)
 *   * mul_mat semantics        src/lamm_kernel_q4_0.hpp:21-37 (C[j*ldc+i], K blocks),
 *                              computing ALL M rows (not inheriting SURVEY §8a defect 1)
 *
 * Floating-point expressions are written in the reference's evaluation order and
 * compiled with -ffp-contract=off, so the results are bit-identical to a scalar
 * (-march=x86-64) build of ggml: tests/test_oracle_golden.py checks exactly that.
 */
#include "lamm_oracle.h"

#include <float.h>
#include <math.h>
#include <stdlib.h>
#include <string.h>

/* ---------------------------------------------------------------- fp16 */

static inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
static inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

float lo_fp16_to_fp32(uint16_t h) {
  const uint32_t sign = (uint32_t)(h & 0x8000u) << 16;
  const uint32_t e = (h >> 10) & 0x1f, m = h & 0x3ffu;
  if (e == 0) {                       /* zero / subnormal: m * 2^-24, exact */
    float v = (float)m * 5.9604644775390625e-08f;
    return u2f(f2u(v) | sign);
  }
  if (e == 31) return u2f(sign | 0x7f800000u | (m << 13));
  return u2f(sign | ((e + 112u) << 23) | (m << 13));
}

uint16_t lo_fp32_to_fp16(float f) {   /* IEEE round-to-nearest-even */
  uint32_t x = f2u(f);
  const uint16_t sign = (uint16_t)((x >> 16) & 0x8000u);
  uint32_t ax = x & 0x7fffffffu;
  if (ax >= 0x7f800000u) return sign | (ax > 0x7f800000u ? 0x7e00u : 0x7c00u);
  if (ax >= 0x477ff000u) return sign | 0x7c00u;           /* >= 65520 -> inf */
  if (ax < 0x38800000u) {                                  /* below 2^-14 */
    float r = rintf(u2f(ax) * 16777216.0f);                /* exact scale, RNE */
    return sign | (uint16_t)r;
  }
  ax += 0xc8000fffu + ((ax >> 13) & 1u);                   /* rebias + RNE */
  return sign | (uint16_t)(ax >> 13);
}

#define H2F(h) lo_fp16_to_fp32(h)
#define F2H(f) lo_fp32_to_fp16(f)

/* ------------------------------------------------------------ layout */

int lo_block_elems(int t) {
  switch (t) {
  case LO_F32: case LO_F16: return 1;
  case LO_Q2_K: case LO_Q4_K: case LO_Q5_K: case LO_Q6_K: case LO_Q8_K: return 256;
  default: return 32;
  }
}

size_t lo_block_bytes(int t) {
  switch (t) {
  case LO_F32: return 4;
  case LO_F16: return 2;
  case LO_Q4_0: return 18;
  case LO_Q4_1: return 20;
  case LO_Q5_0: return 22;
  case LO_Q5_1: return 24;
  case LO_Q8_0: return 34;
  case LO_Q8_1: return 36;
  case LO_Q2_K: return 84;
  case LO_Q4_K: return 144;
  case LO_Q5_K: return 176;
  case LO_Q6_K: return 210;
  case LO_Q8_K: return 292;
  default: return 0;
  }
}

int lo_vec_dot_type(int t) {
  switch (t) {
  case LO_F32: return LO_F32;
  case LO_F16: return LO_F16;
  case LO_Q4_0: case LO_Q5_0: case LO_Q8_0: return LO_Q8_0;
  case LO_Q4_1: case LO_Q5_1: return LO_Q8_1;
  case LO_Q2_K: case LO_Q4_K: case LO_Q5_K: case LO_Q6_K: return LO_Q8_K;
  default: return -1;
  }
}

size_t lo_row_bytes(int t, int k) { return (size_t)(k / lo_block_elems(t)) * lo_block_bytes(t); }

static inline uint16_t rd16(const uint8_t *p) { uint16_t v; memcpy(&v, p, 2); return v; }
static inline void wr16(uint8_t *p, uint16_t v) { memcpy(p, &v, 2); }

/* ------------------------------------------------------- quantizers */

/* first element of largest magnitude, as the reference scans (strict <) */
static void absmax_signed(const float *x, int n, float *amax, float *vmax) {
  float a = 0.0f, m = 0.0f;
  for (int j = 0; j < n; j++) {
    if (a < fabsf(x[j])) { a = fabsf(x[j]); m = x[j]; }
  }
  *amax = a; *vmax = m;
}

static void minmax(const float *x, int n, float *mn, float *mx) {
  float lo = FLT_MAX, hi = -FLT_MAX;
  for (int j = 0; j < n; j++) {
    if (x[j] < lo) lo = x[j];
    if (x[j] > hi) hi = x[j];
  }
  *mn = lo; *mx = hi;
}

/* q4_0 / q5_0 : symmetric, d = max / -(2^(bits-1)) */
static void quant_sym(const float *x, uint8_t *blk, int bits) {
  float amax, vmax;
  absmax_signed(x, 32, &amax, &vmax);
  const float d = vmax / (bits == 4 ? -8 : -16);
  const float id = d ? 1.0f / d : 0.0f;
  wr16(blk, F2H(d));
  uint32_t qh = 0;
  uint8_t *qs = blk + (bits == 4 ? 2 : 6);
  for (int j = 0; j < 16; j++) {
    const float x0 = x[j] * id, x1 = x[16 + j] * id;
    uint8_t v0, v1;
    if (bits == 4) {
      v0 = (uint8_t)((int8_t)(x0 + 8.5f)); if (v0 > 15) v0 = 15;
      v1 = (uint8_t)((int8_t)(x1 + 8.5f)); if (v1 > 15) v1 = 15;
    } else {
      v0 = (uint8_t)((int8_t)(x0 + 16.5f)); if (v0 > 31) v0 = 31;
      v1 = (uint8_t)((int8_t)(x1 + 16.5f)); if (v1 > 31) v1 = 31;
      qh |= (uint32_t)((v0 >> 4) & 1) << j;
      qh |= (uint32_t)((v1 >> 4) & 1) << (j + 16);
    }
    qs[j] = (uint8_t)((v0 & 0x0f) | ((v1 & 0x0f) << 4));
  }
  if (bits == 5) memcpy(blk + 2, &qh, 4);
}

/* q4_1 / q5_1 : affine, d = (max - min) / (2^bits - 1), m = min */
static void quant_affine(const float *x, uint8_t *blk, int bits) {
  float mn, mx;
  minmax(x, 32, &mn, &mx);
  const float d = (mx - mn) / ((1 << bits) - 1);
  const float id = d ? 1.0f / d : 0.0f;
  wr16(blk, F2H(d));
  wr16(blk + 2, F2H(mn));
  uint32_t qh = 0;
  uint8_t *qs = blk + (bits == 4 ? 4 : 8);
  for (int j = 0; j < 16; j++) {
    const float x0 = (x[j] - mn) * id, x1 = (x[16 + j] - mn) * id;
    uint8_t v0, v1;
    if (bits == 4) {
      v0 = (uint8_t)((int8_t)(x0 + 0.5f)); if (v0 > 15) v0 = 15;
      v1 = (uint8_t)((int8_t)(x1 + 0.5f)); if (v1 > 15) v1 = 15;
    } else {                            /* q5_1 reference has no clamp */
      v0 = (uint8_t)(x0 + 0.5f);
      v1 = (uint8_t)(x1 + 0.5f);
      qh |= (uint32_t)((v0 >> 4) & 1) << j;
      qh |= (uint32_t)((v1 >> 4) & 1) << (j + 16);
    }
    qs[j] = (uint8_t)((v0 & 0x0f) | ((v1 & 0x0f) << 4));
  }
  if (bits == 5) memcpy(blk + 4, &qh, 4);
}

/* q8_0 / q8_1 activations.  with_sum selects q8_1 (stores s = d*sum(q)). */
static void quant_q8(const float *x, uint8_t *blk, int flavour, int with_sum) {
  float amax = 0.0f;
  for (int j = 0; j < 32; j++) amax = fmaxf(amax, fabsf(x[j]));
  int8_t *qs = (int8_t *)(blk + (with_sum ? 4 : 2));
  float d;
  int sum = 0;
  if (flavour == LO_QUANT_AVX) {
    /* amax exactly as the AVX2 code reduces it (LC/ggml-quants.c:1286-1296): _mm_max_ps(a, b) is
       a > b ? a : b per lane (the second operand when either is NaN), so a NaN block's amax
       depends on where its NaNs sit -- restated step by step */
    float m[8], q4[4], r[4];
    for (int i = 0; i < 8; i++) m[i] = fabsf(x[i]);
    for (int v = 1; v < 4; v++)
      for (int i = 0; i < 8; i++) {
        const float b = fabsf(x[8 * v + i]);
        m[i] = m[i] > b ? m[i] : b;
      }
    for (int i = 0; i < 4; i++) q4[i] = m[4 + i] > m[i] ? m[4 + i] : m[i];   /* max(hi128, lo128) */
    for (int i = 0; i < 4; i++) {                                           /* max(., movehl) */
      const float b = q4[2 + (i & 1)];
      r[i] = q4[i] > b ? q4[i] : b;
    }
    amax = r[0] > r[1] ? r[0] : r[1];                                       /* max_ss(., movehdup) */
    d = amax / 127.f;
    const float id = (amax != 0.0f) ? 127.f / amax : 0.0f;
    uint32_t wsum = 0;   /* q8_1's s sums the int32 values before the packs, wrapping */
    for (int j = 0; j < 32; j++) {
      const float rv = rintf(x[j] * id);  /* _mm256_round_ps(_MM_ROUND_NEAREST) */
      /* _mm256_cvtps_epi32: NaN and out-of-range values (an id of inf: amax below ~3.7e-37) give
         INT_MIN, which the packs saturate to -128 */
      const int32_t v = (rv >= -2147483648.f && rv < 2147483648.f) ? (int32_t)rv : INT32_MIN;
      wsum += (uint32_t)v;
      qs[j] = (int8_t)(v > 127 ? 127 : v < -128 ? -128 : v);   /* packs saturation */
    }
    sum = (int32_t)wsum;
  } else {
    d = amax / ((1 << 7) - 1);
    const float id = d ? 1.0f / d : 0.0f;
    for (int j = 0; j < 32; j++) {
      qs[j] = (int8_t)roundf(x[j] * id);
      sum += qs[j];
    }
  }
  wr16(blk, F2H(d));
  if (with_sum) wr16(blk + 2, F2H(sum * d));
}

static inline int nearest_int(float f) {
  float v = f + 12582912.f;
  int i; memcpy(&i, &v, 4);
  return (i & 0x007fffff) - 0x00400000;
}

/* affine fit of n values to [0,nmax] minimising weighted |err| (use_mad) */
static float fit_affine(int n, int nmax, const float *x, const float *w, uint8_t *L,
                        float *the_min, uint8_t *Laux, float rmin, float rdelta,
                        int nstep, int use_mad) {
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
    int l = nearest_int(iscale * (x[i] - mn));
    l = l < 0 ? 0 : (l > nmax ? nmax : l);
    L[i] = (uint8_t)l;
    float diff = scale * L[i] + mn - x[i];
    diff = use_mad ? fabsf(diff) : diff * diff;
    best += w[i] * diff;
  }
  if (nstep < 1) { *the_min = -mn; return scale; }
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
    float D = sum_w * sum_l2 - sum_l * sum_l;
    if (D > 0) {
      float this_scale = (sum_w * sum_xl - sum_x * sum_l) / D;
      float this_min = (sum_l2 * sum_x - sum_l * sum_xl) / D;
      if (this_min > 0) { this_min = 0; this_scale = sum_xl / sum_l2; }
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

/* block_q2_K: scales[16] | qs[64] | d | dmin  (LC/ggml-common.h:199-209) */
static void quant_q2_K(const float *x, uint8_t *blk) {
  uint8_t L[256], Laux[16];
  float w[16], mins[16], scales[16];
  uint8_t *sc = blk, *qs = blk + 16;
  float max_scale = 0, max_min = 0;
  for (int j = 0; j < 16; ++j) {
    for (int l = 0; l < 16; ++l) w[l] = fabsf(x[16 * j + l]);
    scales[j] = fit_affine(16, 3, x + 16 * j, w, L + 16 * j, &mins[j], Laux, -0.5f, 0.1f, 15, 1);
    if (scales[j] > max_scale) max_scale = scales[j];
    if (mins[j] > max_min) max_min = mins[j];
  }
  if (max_scale > 0) {
    float iscale = 15.f / max_scale;
    for (int j = 0; j < 16; ++j) sc[j] = (uint8_t)nearest_int(iscale * scales[j]);
    wr16(blk + 80, F2H(max_scale / 15.f));
  } else {
    for (int j = 0; j < 16; ++j) sc[j] = 0;
    wr16(blk + 80, F2H(0.f));
  }
  if (max_min > 0) {
    float iscale = 15.f / max_min;
    for (int j = 0; j < 16; ++j) sc[j] |= (uint8_t)(nearest_int(iscale * mins[j]) << 4);
    wr16(blk + 82, F2H(max_min / 15.f));
  } else {
    wr16(blk + 82, F2H(0.f));
  }
  for (int j = 0; j < 16; ++j) {
    const float d = H2F(rd16(blk + 80)) * (sc[j] & 0xF);
    if (!d) continue;
    const float dm = H2F(rd16(blk + 82)) * (sc[j] >> 4);
    for (int ii = 0; ii < 16; ++ii) {
      int l = nearest_int((x[16 * j + ii] + dm) / d);
      L[16 * j + ii] = (uint8_t)(l < 0 ? 0 : (l > 3 ? 3 : l));
    }
  }
  for (int j = 0; j < 256; j += 128)
    for (int l = 0; l < 32; ++l)
      qs[j / 4 + l] = (uint8_t)(L[j + l] | (L[j + l + 32] << 2) | (L[j + l + 64] << 4) | (L[j + l + 96] << 6));
}

/* block_q8_K: f32 d | i8 qs[256] | i16 bsums[16] */
static void quant_q8_K(const float *x, uint8_t *blk) {
  float amax = 0, vmax = 0;
  for (int j = 0; j < 256; ++j) {
    float ax = fabsf(x[j]);
    if (ax > amax) { amax = ax; vmax = x[j]; }
  }
  int8_t *qs = (int8_t *)(blk + 4);
  if (!amax) {
    float z = 0; memcpy(blk, &z, 4);
    memset(qs, 0, 256);
    memset(blk + 260, 0, 32);
    return;
  }
  const float iscale = -127.f / vmax;
  for (int j = 0; j < 256; ++j) {
    int v = nearest_int(iscale * x[j]);
    qs[j] = (int8_t)(v < 127 ? v : 127);
  }
  for (int j = 0; j < 16; ++j) {
    int s = 0;
    for (int i = 0; i < 16; ++i) s += qs[16 * j + i];
    int16_t s16 = (int16_t)s;
    memcpy(blk + 260 + 2 * j, &s16, 2);
  }
  float d = 1 / iscale;
  memcpy(blk, &d, 4);
}

void lo_quantize_row(int type, int flavour, const float *x, void *y, int k) {
  const int qk = lo_block_elems(type);
  const size_t bb = lo_block_bytes(type);
  uint8_t *out = (uint8_t *)y;
  if (type == LO_F32) { memcpy(y, x, (size_t)k * 4); return; }
  if (type == LO_F16) {   /* ggml_fp32_to_fp16_row (LC/ggml.c): per element, round-to-nearest-even */
    for (int i = 0; i < k; i++) wr16(out + 2 * (size_t)i, lo_fp32_to_fp16(x[i]));
    return;
  }
  for (int b = 0; b < k / qk; b++) {
    const float *xb = x + (size_t)b * qk;
    uint8_t *yb = out + (size_t)b * bb;
    switch (type) {
    case LO_Q4_0: quant_sym(xb, yb, 4); break;
    case LO_Q5_0: quant_sym(xb, yb, 5); break;
    case LO_Q4_1: quant_affine(xb, yb, 4); break;
    case LO_Q5_1: quant_affine(xb, yb, 5); break;
    case LO_Q8_0: quant_q8(xb, yb, flavour, 0); break;
    case LO_Q8_1: quant_q8(xb, yb, flavour, 1); break;
    case LO_Q2_K: quant_q2_K(xb, yb); break;
    case LO_Q8_K: quant_q8_K(xb, yb); break;
    default: break;
    }
  }
}

/* ------------------------------------------------ k-quant element access */

/* 6-bit scales / mins of q4_K / q5_K from the 12 packed bytes: the utmp shuffle of
 * LC/ggml-quants.c:7324-7330 (kmask1 = 0x3f3f3f3f, kmask2 = 0x0f0f0f0f, kmask3 = 0x03030303) */
static void kq_scale_min(const uint8_t *s12, uint8_t sc[8], uint8_t mn[8]) {
  uint32_t u[4];
  memcpy(u, s12, 12);
  u[3] = ((u[2] >> 4) & 0x0f0f0f0fu) | (((u[1] >> 6) & 0x03030303u) << 4);
  const uint32_t uaux = u[1] & 0x3f3f3f3fu;
  u[1] = (u[2] & 0x0f0f0f0fu) | (((u[0] >> 6) & 0x03030303u) << 4);
  u[2] = uaux;
  u[0] &= 0x3f3f3f3fu;
  memcpy(sc, u, 8);
  memcpy(mn, u + 2, 8);
}

/* quant of element e (0..255) of a q4_K / q5_K block: :7316-7322 / :7983-7992 */
static int kq_nibble(const uint8_t *x, int type, int e) {
  const int g = e / 64, hi = (e % 64) >= 32, l = e % 32;
  const uint8_t *qs = x + (type == LO_Q5_K ? 48 : 16);
  int q = hi ? (qs[32 * g + l] >> 4) : (qs[32 * g + l] & 0xF);
  if (type == LO_Q5_K) q += (x[16 + l] >> (e / 32)) & 1 ? 16 : 0;
  return q;
}

/* q6_K element e: (ql | qh << 4) - 32, :8710-8720 */
static int q6_value(const uint8_t *x, int e) {
  const int hf = e / 128, r = e % 128, part = r / 32, l = r % 32;
  const uint8_t *ql = x + 64 * hf, *qh = x + 128 + 32 * hf;
  const int nib = (part & 1) ? ql[32 + l] : ql[l];
  const int q = (part < 2 ? (nib & 0xF) : (nib >> 4)) | (((qh[l] >> (2 * part)) & 3) << 4);
  return q - 32;
}

/* --------------------------------------------------------- dequant */

void lo_dequantize_row(int type, const void *vx, float *y, int k) {
  const uint8_t *x = (const uint8_t *)vx;
  const int qk = lo_block_elems(type);
  const size_t bb = lo_block_bytes(type);
  if (type == LO_F32) { memcpy(y, vx, (size_t)k * 4); return; }
  if (type == LO_F16) {
    for (int i = 0; i < k; i++) y[i] = H2F(rd16(x + 2 * (size_t)i));
    return;
  }
  for (int b = 0; b < k / qk; b++, x += bb, y += qk) {
    switch (type) {
    case LO_Q4_0: case LO_Q5_0: case LO_Q4_1: case LO_Q5_1: {
      const int aff = (type == LO_Q4_1 || type == LO_Q5_1);
      const int five = (type == LO_Q5_0 || type == LO_Q5_1);
      const float d = H2F(rd16(x)), m = aff ? H2F(rd16(x + 2)) : 0.f;
      uint32_t qh = 0;
      if (five) memcpy(&qh, x + (aff ? 4 : 2), 4);
      const uint8_t *qs = x + (aff ? 4 : 2) + (five ? 4 : 0);
      for (int j = 0; j < 32; j++) {
        int q = (j < 16) ? (qs[j] & 0xF) : (qs[j - 16] >> 4);
        if (five) q |= ((qh >> j) & 1) << 4;
        if (!aff) q -= five ? 16 : 8;
        y[j] = aff ? d * q + m : d * q;
      }
    } break;
    case LO_Q8_0: case LO_Q8_1: {
      const float d = H2F(rd16(x));
      const int8_t *qs = (const int8_t *)(x + (type == LO_Q8_1 ? 4 : 2));
      for (int j = 0; j < 32; j++) y[j] = d * qs[j];
    } break;
    case LO_Q2_K: {
      const float d = H2F(rd16(x + 80)), dmin = H2F(rd16(x + 82));
      for (int e = 0; e < 256; e++) {
        const int n = e / 128, j = (e % 128) / 32, l = e % 32;
        const int is = 8 * n + 2 * j + (l >= 16);
        const int q = (x[16 + 32 * n + l] >> (2 * j)) & 3;
        y[e] = d * (x[is] & 0xF) * q - dmin * (x[is] >> 4);
      }
    } break;
    case LO_Q4_K: case LO_Q5_K: {   /* LC/ggml-quants.c dequantize_row_q4_K / q5_K */
      uint8_t sc[8], mn[8];
      kq_scale_min(x + 4, sc, mn);
      const float d = H2F(rd16(x)), dmin = H2F(rd16(x + 2));
      for (int e = 0; e < 256; e++) {
        const int j = e / 32, l = e % 32;
        int q = kq_nibble(x, type, e);
        y[e] = d * sc[j] * q - dmin * mn[j];
        (void)l;
      }
    } break;
    case LO_Q6_K: {                  /* dequantize_row_q6_K */
      const float d = H2F(rd16(x + 208));
      for (int e = 0; e < 256; e++) y[e] = d * (int8_t)x[192 + e / 16] * q6_value(x, e);
    } break;
    case LO_Q8_K: {
      float d; memcpy(&d, x, 4);
      for (int j = 0; j < 256; j++) y[j] = d * ((const int8_t *)(x + 4))[j];
    } break;
    default: break;
    }
  }
}

/* --------------------------------------------------------- vec_dot */

static float dot_f32(int k, const float *a, const float *b) {
  double s = 0.0;
  for (int i = 0; i < k; ++i) s += (double)(a[i] * b[i]);
  return (float)s;
}

/* one 32-element block, (A, B) in the lamm pairs; returns the int dot */
static int blk_idot(int type, const uint8_t *a, const int8_t *bq) {
  int s = 0;
  switch (type) {
  case LO_Q4_0:
    for (int j = 0; j < 16; ++j)
      s += ((a[2 + j] & 0x0F) - 8) * bq[j] + ((a[2 + j] >> 4) - 8) * bq[j + 16];
    break;
  case LO_Q4_1:
    for (int j = 0; j < 16; ++j)
      s += (a[4 + j] & 0x0F) * bq[j] + (a[4 + j] >> 4) * bq[j + 16];
    break;
  case LO_Q5_0: {
    uint32_t qh; memcpy(&qh, a + 2, 4);
    for (int j = 0; j < 16; ++j) {
      const int h0 = ((qh >> j) & 1) << 4, h1 = ((qh >> (j + 16)) & 1) << 4;
      s += (((a[6 + j] & 0x0F) | h0) - 16) * bq[j] + (((a[6 + j] >> 4) | h1) - 16) * bq[j + 16];
    }
  } break;
  case LO_Q5_1: {
    uint32_t qh; memcpy(&qh, a + 4, 4);
    for (int j = 0; j < 16; ++j) {
      const int h0 = ((qh >> j) & 1) << 4, h1 = ((qh >> (j + 16)) & 1) << 4;
      s += ((a[8 + j] & 0x0F) | h0) * bq[j] + ((a[8 + j] >> 4) | h1) * bq[j + 16];
    }
  } break;
  case LO_Q8_0:
    for (int j = 0; j < 32; ++j) s += ((const int8_t *)(a + 2))[j] * bq[j];
    break;
  default: break;
  }
  return s;
}

float lo_vec_dot(int type, int k, const void *va, const void *vb) {
  const uint8_t *a = (const uint8_t *)va, *b = (const uint8_t *)vb;
  if (type == LO_F32) return dot_f32(k, (const float *)va, (const float *)vb);
  if (type == LO_F16) {   /* ggml_vec_dot_f16 scalar branch: ggml_float (double) sum of f32 products */
    double s = 0.0;
    for (int i = 0; i < k; ++i) s += (double)(H2F(rd16(a + 2 * (size_t)i)) * H2F(rd16(b + 2 * (size_t)i)));
    return (float)s;
  }
  const size_t ab = lo_block_bytes(type), bb = lo_block_bytes(lo_vec_dot_type(type));
  float sumf = 0.0f;
  if (type == LO_Q2_K) {
    for (int i = 0; i < k / 256; ++i, a += ab, b += bb) {
      const uint8_t *sc = a, *q2 = a + 16;
      float yd; memcpy(&yd, b, 4);
      const int8_t *q8 = (const int8_t *)(b + 4);
      int summs = 0;
      for (int j = 0; j < 16; ++j) {
        int16_t bs; memcpy(&bs, b + 260 + 2 * j, 2);
        summs += bs * (sc[j] >> 4);
      }
      const float dall = yd * H2F(rd16(a + 80));
      const float dmin = yd * H2F(rd16(a + 82));
      int isum = 0, is = 0;
      for (int n = 0; n < 2; ++n, q2 += 32) {
        for (int j = 0, shift = 0; j < 4; ++j, shift += 2, q8 += 32) {
          int d = sc[is++] & 0xF, part = 0;
          for (int l = 0; l < 16; ++l) part += q8[l] * ((q2[l] >> shift) & 3);
          isum += d * part;
          d = sc[is++] & 0xF;
          part = 0;
          for (int l = 16; l < 32; ++l) part += q8[l] * ((q2[l] >> shift) & 3);
          isum += d * part;
        }
      }
      sumf += dall * isum - dmin * summs;
    }
    return sumf;
  }
  if (type == LO_Q4_K || type == LO_Q5_K || type == LO_Q6_K) {
    /* the reference's 8-lane order: aux32[l] (int) per super-block, sums[l] += d*aux32[l],
     * sumf -= dmin*sumi per super-block, then sumf += sums[l] (:7301-7358, :8695-8738) */
    float sums[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = 0; i < k / 256; ++i, a += ab, b += bb) {
      float yd; memcpy(&yd, b, 4);
      const int8_t *q8 = (const int8_t *)(b + 4);
      int32_t aux32[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      int8_t av[256];
      for (int e = 0; e < 256; ++e) av[e] = (int8_t)(type == LO_Q6_K ? q6_value(a, e) : kq_nibble(a, type, e));
      if (type == LO_Q6_K) {
        for (int j = 0; j < 16; ++j) {
          const int scale = (int8_t)a[192 + j];
          for (int l = 0; l < 16; ++l) aux32[l % 8] += scale * (int16_t)(q8[16 * j + l] * av[16 * j + l]);
        }
        const float d = H2F(rd16(a + 208)) * yd;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
      } else {
        uint8_t sc[8], mn[8];
        kq_scale_min(a + 4, sc, mn);
        int sumi = 0;
        for (int j = 0; j < 16; ++j) {
          int16_t bs; memcpy(&bs, b + 260 + 2 * j, 2);
          sumi += bs * mn[j / 2];
        }
        for (int j = 0; j < 8; ++j) {
          const int32_t scale = sc[j];
          for (int l = 0; l < 32; ++l) aux32[l % 8] += scale * (int16_t)(q8[32 * j + l] * av[32 * j + l]);
        }
        const float d = H2F(rd16(a)) * yd;
        for (int l = 0; l < 8; ++l) sums[l] += d * aux32[l];
        const float dmin = H2F(rd16(a + 2)) * yd;
        sumf -= dmin * sumi;
      }
    }
    for (int l = 0; l < 8; ++l) sumf += sums[l];
    return sumf;
  }
  const int bq_off = (type == LO_Q4_1 || type == LO_Q5_1) ? 4 : 2;
  for (int i = 0; i < k / 32; ++i, a += ab, b += bb) {
    const int sumi = blk_idot(type, a, (const int8_t *)(b + bq_off));
    const float da = H2F(rd16(a)), db = H2F(rd16(b));
    switch (type) {
    case LO_Q4_0: sumf += sumi * da * db; break;                 /* :4466 order */
    case LO_Q8_0: sumf += sumi * (da * db); break;               /* :5310 order */
    case LO_Q5_0: sumf += (da * db) * sumi; break;
    case LO_Q4_1: case LO_Q5_1:
      sumf += (da * db) * sumi + H2F(rd16(a + 2)) * H2F(rd16(b + 2));
      break;
    default: break;
    }
  }
  return sumf;
}

void lo_mul_mat(int type, int M, int N, int K, const void *A, size_t lda_bytes,
                const void *B, size_t ldb_bytes, float *C, size_t ldc) {
  for (int j = 0; j < N; j++)
    for (int i = 0; i < M; i++)
      C[(size_t)j * ldc + i] = lo_vec_dot(type, K, (const uint8_t *)A + (size_t)i * lda_bytes,
                                          (const uint8_t *)B + (size_t)j * ldb_bytes);
}

/* --------------------------------------------------------- the AVX2 float order
 * The reference's CPU path on x86 (the lamm opt-3 AVX2 kernels, src/lamm_kernel_q*.hpp
 * lamm_simd_block_kernel / lamm_simd_kernel with src/lamm_simd_avx2.h, q2_K among them; for q4_K /
 * q5_K / q6_K, which lamm declines, ggml's AVX2 ggml_vec_dot_q*_K_q8_K, LC/ggml-quants.c:7082-7145,
 * :7696-7777, :8305-8385 -- their min terms are restated beside the lanes below) keeps EIGHT fp32
 * accumulators per output -- one per 32-bit lane of an __m256 -- and for every block / super-block
 * adds d * (float)X_l into lane l with a fused multiply-add (_mm256_fmadd_ps), where X_l is the
 * exact int32 sum of the 4 products (block formats: elements 4l..4l+3, through
 * mul_sum_i8_pairs_float / mul_sum_us8_pairs_float) or of the scaled group sums (q6_K: positions
 * 4l..4l+3 of each of the 8 32-element groups) that land in lane l, and d = fp32(d_a) * fp32(d_b)
 * rounded once.  The lanes then meet in reduce_sum's tree (src/lamm_simd_avx2.h:117-127, the same
 * as hsum_float_8): ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7)).  q4_1 / q5_1 add
 * sum_k fp32(m_a) * fp32(s_b) (a separate fp32 sum, :lamm_kernel_q4_1.hpp) after the tree; f32
 * keeps element 8i + l in lane l (src/lamm_kernel_f32.hpp).
 * q8_0 is not restated here: lamm's AVX2 q8_0 kernel treats the weight quants as unsigned
 * (mul_sum_us8_pairs_float, SURVEY §8a defect 2), so its output is not the product. */
static float tree8(const float *a) {
  const float x0 = a[0] + a[4], x1 = a[1] + a[5], x2 = a[2] + a[6], x3 = a[3] + a[7];
  return (x0 + x2) + (x1 + x3);
}

/* ggml's AVX2 ggml_vec_dot_f16 (LC/ggml.c:1589-1629; GGML_F16_STEP 32, GGML_F16_EPR 8 :979-1027):
 * FOUR __m256 accumulators, element i of each 32-element step into sum[(i % 32) / 8] lane i % 8,
 * sum = fma(x, y, sum) on the F16C-widened values; then GGML_F32x8_REDUCE (:946-964):
 * sum0 += sum2, sum1 += sum3, sum0 += sum1 lanewise, t0 = low half + high half, two hadds:
 * ((t0 + t1) + (t2 + t3)) with t_e = v_e + v_{e+4}.  The n % 32 leftovers are added after that in
 * double (ggml_float) and the result rounded to float. */
static float f16_dot_avx(int n, const uint16_t *x, const uint16_t *y) {
  float s[4][8];
  memset(s, 0, sizeof s);
  const int np = n & ~31;
  for (int i = 0; i < np; i += 32)
    for (int j = 0; j < 4; ++j)
      for (int e = 0; e < 8; ++e) {
        const int ii = i + 8 * j + e;
        s[j][e] = fmaf(H2F(x[ii]), H2F(y[ii]), s[j][e]);
      }
  float v[8], t[4];
  for (int e = 0; e < 8; ++e) v[e] = (s[0][e] + s[2][e]) + (s[1][e] + s[3][e]);
  for (int e = 0; e < 4; ++e) t[e] = v[e] + v[e + 4];
  double sumf = (double)((t[0] + t[1]) + (t[2] + t[3]));
  for (int i = np; i < n; ++i) sumf += (double)(H2F(x[i]) * H2F(y[i]));
  return (float)sumf;
}

/* quant e (0..31) of a 32-element block, with the format's offset (q4_0: q - 8, q5_0: q - 16) */
static int blk_q(int type, const uint8_t *a, int e) {
  const int j = e & 15, hi = e >= 16;
  switch (type) {
  case LO_Q4_0: return (hi ? a[2 + j] >> 4 : a[2 + j] & 0xF) - 8;
  case LO_Q4_1: return hi ? a[4 + j] >> 4 : a[4 + j] & 0xF;
  case LO_Q5_0: case LO_Q5_1: {
    const int qs = type == LO_Q5_0 ? 6 : 8;
    uint32_t qh; memcpy(&qh, a + (type == LO_Q5_0 ? 2 : 4), 4);
    const int q = (hi ? a[qs + j] >> 4 : a[qs + j] & 0xF) | (((qh >> e) & 1) << 4);
    return type == LO_Q5_0 ? q - 16 : q;
  }
  default: return 0;
  }
}

float lo_vec_dot_avx(int type, int k, const void *va, const void *vb) {
  const uint8_t *a = (const uint8_t *)va, *b = (const uint8_t *)vb;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  if (type == LO_F32) {
    const float *x = (const float *)va, *y = (const float *)vb;
    for (int i = 0; i < k; i += 8)
      for (int l = 0; l < 8; ++l) acc[l] = fmaf(x[i + l], y[i + l], acc[l]);
    return tree8(acc);
  }
  if (type == LO_F16) return f16_dot_avx(k, (const uint16_t *)va, (const uint16_t *)vb);
  const size_t ab = lo_block_bytes(type), bb = lo_block_bytes(lo_vec_dot_type(type));
  if (type == LO_Q6_K) {
    for (int i = 0; i < k / 256; ++i, a += ab, b += bb) {
      float yd; memcpy(&yd, b, 4);
      const int8_t *q8 = (const int8_t *)(b + 4);
      const float d = yd * H2F(rd16(a + 208));
      int32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int h = 0; h < 8; ++h)          /* 32-element group h = 4 j + g: elements 32 h .. */
        for (int e = 0; e < 32; ++e) {
          const int y = 32 * h + e;
          X[e / 4] += (int8_t)a[192 + y / 16] * (q6_value(a, y) * q8[y]);
        }
      for (int l = 0; l < 8; ++l) acc[l] = fmaf(d, (float)X[l], acc[l]);
    }
    return tree8(acc);
  }
  if (type == LO_Q2_K) {
    /* lamm's AVX2 q2_K block kernel (src/lamm_kernel_q2_k.hpp:163-307, the opt-3 tier's kernel for
     * every tile, src/lamm_impl.hpp:124-143): per super-block, lane l of sumi is the exact int sum over
     * the 8 32-element groups h of (scale nibble sc[2h + (l >= 4)]) * (the 4-element dot of q2 (0..3)
     * and q8 at positions 4l .. 4l+3 of group h) -- maddubs pairs, madd_epi16 with the shuffled
     * scales (:212-233); lane l of prod is mins[2l] bsums[2l] + mins[2l+1] bsums[2l+1] (madd_epi16,
     * :247); then acc = fma(fp32(d_a) * d_b, sumi, acc) and acc = fma(-fp32(dmin_a) * d_b, prod, acc)
     * (:245-248), in that order; reduce_sum's tree at the end */
    for (int i = 0; i < k / 256; ++i, a += ab, b += bb) {
      float yd; memcpy(&yd, b, 4);
      const int8_t *q8 = (const int8_t *)(b + 4);
      const float d1 = H2F(rd16(a + 80)) * yd;
      const float d2 = -H2F(rd16(a + 82)) * yd;
      int32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int h = 0; h < 8; ++h)          /* group h: elements 32 h .. 32 h + 31 */
        for (int e = 0; e < 32; ++e) {
          const int q = (a[16 + 32 * (h / 4) + e] >> (2 * (h % 4))) & 3;
          X[e / 4] += (a[2 * h + (e >= 16)] & 0xF) * q * q8[32 * h + e];
        }
      for (int l = 0; l < 8; ++l) {
        int16_t s0, s1;
        memcpy(&s0, b + 260 + 4 * l, 2);
        memcpy(&s1, b + 262 + 4 * l, 2);
        const int32_t Y = (a[2 * l] >> 4) * s0 + (a[2 * l + 1] >> 4) * s1;
        acc[l] = fmaf(d1, (float)X[l], acc[l]);
        acc[l] = fmaf(d2, (float)Y, acc[l]);
      }
    }
    return tree8(acc);
  }
  if (type == LO_Q4_K || type == LO_Q5_K) {
    /* ggml's AVX2 ggml_vec_dot_q4_K_q8_K (LC/ggml-quants.c:7082-7145) / q5_K (:7696-7777), which lamm
     * declines: per super-block lane l of sumi = sum over the 8 32-element groups g of sc[g] * (the
     * 4-element dot at positions 4l .. 4l+3 of group g), acc_l = fma(d_b * fp32(d_a), sumi_l, acc_l);
     * the mins: q8s = hadd(bsums) (pairs), prod_k = mn[2k] q8s[2k] + mn[2k+1] q8s[2k+1] (k = 0..3);
     * q4_K keeps them in a 4-lane fma chain reduced (m0 + m2) + (m1 + m3), q5_K adds dmin * (the int
     * sum of the four) into a scalar per super-block (product and sum rounded separately);
     * then hsum_float_8(acc) + that */
    float acc_m[4] = {0, 0, 0, 0}, summs = 0.0f;
    for (int i = 0; i < k / 256; ++i, a += ab, b += bb) {
      float yd; memcpy(&yd, b, 4);
      const int8_t *q8 = (const int8_t *)(b + 4);
      const float d = yd * H2F(rd16(a)), dmin = -yd * H2F(rd16(a + 2));
      uint8_t sc[8], mn[8];
      kq_scale_min(a + 4, sc, mn);
      int16_t bs[16];
      memcpy(bs, b + 260, 32);
      int32_t prod[4];
      for (int q = 0; q < 4; ++q)
        prod[q] = mn[2 * q] * (int16_t)(bs[4 * q] + bs[4 * q + 1]) + mn[2 * q + 1] * (int16_t)(bs[4 * q + 2] + bs[4 * q + 3]);
      if (type == LO_Q4_K) {
        for (int q = 0; q < 4; ++q) acc_m[q] = fmaf(dmin, (float)prod[q], acc_m[q]);
      } else {
        summs = summs + dmin * (float)((prod[0] + prod[1]) + (prod[2] + prod[3]));
      }
      int32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int e = 0; e < 256; ++e) X[(e % 32) / 4] += sc[e / 32] * kq_nibble(a, type, e) * q8[e];
      for (int l = 0; l < 8; ++l) acc[l] = fmaf(d, (float)X[l], acc[l]);
    }
    if (type == LO_Q4_K) return tree8(acc) + ((acc_m[0] + acc_m[2]) + (acc_m[1] + acc_m[3]));
    return tree8(acc) + summs;
  }
  if (type != LO_Q4_0 && type != LO_Q4_1 && type != LO_Q5_0 && type != LO_Q5_1) return 0.0f;
  const int aff = type == LO_Q4_1 || type == LO_Q5_1;
  const int8_t *bq;
  float summs = 0.0f;
  for (int i = 0; i < k / 32; ++i, a += ab, b += bb) {
    bq = (const int8_t *)(b + (aff ? 4 : 2));
    const float d = H2F(rd16(a)) * H2F(rd16(b));
    for (int l = 0; l < 8; ++l) {
      int X = 0;
      for (int e = 4 * l; e < 4 * l + 4; ++e) X += blk_q(type, a, e) * bq[e];
      acc[l] = fmaf(d, (float)X, acc[l]);
    }
    if (aff) summs += H2F(rd16(a + 2)) * H2F(rd16(b + 2));
  }
  return tree8(acc) + summs;
}

/* the same order as lo_vec_dot_avx, with each A row's quants decoded once for all N columns */
static void row_avx(int type, int N, int K, const uint8_t *a, const uint8_t *B, size_t ldb_bytes, float *C,
                    size_t ldc, int8_t *av) {
  const size_t ab = lo_block_bytes(type), bb = lo_block_bytes(lo_vec_dot_type(type));
  if (type == LO_Q6_K) {
    for (int e = 0; e < K; ++e) av[e] = (int8_t)q6_value(a + (size_t)(e / 256) * ab, e % 256);
    for (int j = 0; j < N; ++j) {
      const uint8_t *b = B + (size_t)j * ldb_bytes;
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int i = 0; i < K / 256; ++i) {
        const uint8_t *x = a + (size_t)i * ab, *y = b + (size_t)i * bb;
        float yd; memcpy(&yd, y, 4);
        const int8_t *q8 = (const int8_t *)(y + 4), *v = av + 256 * i;
        const float d = yd * H2F(rd16(x + 208));
        int32_t X[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        for (int e = 0; e < 256; ++e) X[(e % 32) / 4] += (int8_t)x[192 + e / 16] * (v[e] * q8[e]);
        for (int l = 0; l < 8; ++l) acc[l] = fmaf(d, (float)X[l], acc[l]);
      }
      C[(size_t)j * ldc] = tree8(acc);
    }
    return;
  }
  const int aff = type == LO_Q4_1 || type == LO_Q5_1;
  for (int e = 0; e < K; ++e) av[e] = (int8_t)blk_q(type, a + (size_t)(e / 32) * ab, e % 32);
  for (int j = 0; j < N; ++j) {
    const uint8_t *b = B + (size_t)j * ldb_bytes;
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, summs = 0.0f;
    for (int i = 0; i < K / 32; ++i) {
      const uint8_t *x = a + (size_t)i * ab, *y = b + (size_t)i * bb;
      const int8_t *bq = (const int8_t *)(y + (aff ? 4 : 2)), *v = av + 32 * i;
      const float d = H2F(rd16(x)) * H2F(rd16(y));
      for (int l = 0; l < 8; ++l) {
        const int X = v[4 * l] * bq[4 * l] + v[4 * l + 1] * bq[4 * l + 1] + v[4 * l + 2] * bq[4 * l + 2] +
                      v[4 * l + 3] * bq[4 * l + 3];
        acc[l] = fmaf(d, (float)X, acc[l]);
      }
      if (aff) summs += H2F(rd16(x + 2)) * H2F(rd16(y + 2));
    }
    C[(size_t)j * ldc] = tree8(acc) + summs;
  }
}

void lo_mul_mat_avx(int type, int M, int N, int K, const void *A, size_t lda_bytes,
                    const void *B, size_t ldb_bytes, float *C, size_t ldc) {
  if (type == LO_Q6_K || type == LO_Q4_0 || type == LO_Q4_1 || type == LO_Q5_0 || type == LO_Q5_1) {
    int8_t *av = (int8_t *)malloc((size_t)K);
    for (int i = 0; i < M; i++)
      row_avx(type, N, K, (const uint8_t *)A + (size_t)i * lda_bytes, (const uint8_t *)B, ldb_bytes, C + i, ldc, av);
    free(av);
    return;
  }
  for (int j = 0; j < N; j++)
    for (int i = 0; i < M; i++)
      C[(size_t)j * ldc + i] = lo_vec_dot_avx(type, K, (const uint8_t *)A + (size_t)i * lda_bytes,
                                              (const uint8_t *)B + (size_t)j * ldb_bytes);
}
