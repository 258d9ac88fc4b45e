// lamm_gemv.hip -- decode-shaped (N <= 8) quantized mat-vec for gfx950.
//
// Replaces the per-format block-dot kernels of the lamm plug-in
// (src/lamm_kernel_{f32,q4_0,q4_1,q5_0,q5_1,q8_0,q2_k}.hpp, driven by
// LAMMImpl<T>::matmul_simd_block, src/lamm_impl.hpp:90-147) for small N:
//
//   C[j*ldc + i] = sum_k A[i,k] * B[j,k]     (C stored N rows of M; lamm layout)
//
// Structure (one workgroup = 256 threads = 16 rows x 16 "chunks"):
//   * A is streamed from HBM once, as raw block_q* bytes, with coalesced 16-byte
//     buffer loads into LDS (AoS, no repack: 18/20/22/24/34/84-byte blocks are not
//     dword aligned, so each thread then reads its chunk of G blocks from LDS).
//   * B (the q8_0/q8_1/q8_K activation row(s)) is decoded once per workgroup into
//     LDS as int8 words + fp32 scales (+ sum(q) / s / bsums), XOR-swizzled so the 16
//     chunk-threads of a row read conflict-free.
//   * Each thread unpacks its blocks' 2/4/5/8-bit quants to int8 in registers and
//     accumulates exact per-block int32 dots with v_dot4_i32_i8, then applies the
//     fp16 scales in fp32 (d_a*d_b*S [+ m_a*s_b]).  The 16 chunk partials of a row
//     are reduced with wave shuffles in a fixed order (deterministic).
//   * K larger than one segment (4096 elements; 1024 for f32) loops over segments.
#include "lamm_device.h"
#include "lamm_kernels.h"

#include <cstdlib>
#include "lamm_knobs.h"

namespace lamm {
namespace {

constexpr int kThreads = 256;
constexpr int kSC = 16;                 // chunks per row per segment
constexpr int kRows = kThreads / kSC;   // rows per workgroup

template <int T> struct Fmt;
// QK: elems/block, BPB: bytes/block, G: blocks per chunk (G*BPB % 16 == 0 or G=1),
// VBPB: activation block bytes, VQK: activation elems/block
template <> struct Fmt<kQ4_0> { static constexpr int QK = 32, BPB = 18, G = 8, VBPB = 34, VQK = 32; };
template <> struct Fmt<kQ4_1> { static constexpr int QK = 32, BPB = 20, G = 8, VBPB = 36, VQK = 32; };
template <> struct Fmt<kQ5_0> { static constexpr int QK = 32, BPB = 22, G = 8, VBPB = 34, VQK = 32; };
template <> struct Fmt<kQ5_1> { static constexpr int QK = 32, BPB = 24, G = 8, VBPB = 36, VQK = 32; };
template <> struct Fmt<kQ8_0> { static constexpr int QK = 32, BPB = 34, G = 8, VBPB = 34, VQK = 32; };
template <> struct Fmt<kQ2_K> { static constexpr int QK = 256, BPB = 84, G = 1, VBPB = 292, VQK = 256; };
template <> struct Fmt<kQ4_K> { static constexpr int QK = 256, BPB = 144, G = 1, VBPB = 292, VQK = 256; };
template <> struct Fmt<kQ5_K> { static constexpr int QK = 256, BPB = 176, G = 1, VBPB = 292, VQK = 256; };
template <> struct Fmt<kQ6_K> { static constexpr int QK = 256, BPB = 210, G = 1, VBPB = 292, VQK = 256; };
template <> struct Fmt<kF32>  { static constexpr int QK = 1, BPB = 4, G = 64, VBPB = 4, VQK = 1; };
template <> struct Fmt<kF16>  { static constexpr int QK = 1, BPB = 2, G = 128, VBPB = 2, VQK = 1; };

template <int T> struct Geo {
  using F = Fmt<T>;
  static constexpr int CH_ELEMS = F::G * F::QK;          // 256 (64 for f32)
  static constexpr int CH_BYTES = F::G * F::BPB;
  static constexpr int CH_WORDS = (CH_BYTES + 3) / 4;
  static constexpr int SEG_ELEMS = kSC * CH_ELEMS;       // 4096 (1024 for f32)
  static constexpr int SEG_BLK = kSC * F::G;             // A blocks per row-segment
  static constexpr int ROW_BYTES = kSC * CH_BYTES;       // LDS bytes per row-segment
  static constexpr int A_PIECES = kRows * ROW_BYTES / 16;
  static constexpr int A_NPT = (A_PIECES + kThreads - 1) / kThreads;
  static constexpr int A_LDS = A_NPT * kThreads * 16;
  static constexpr int VBLK = SEG_ELEMS / F::VQK;        // activation blocks per segment
  static constexpr int BQ_WORDS = T == kF32 ? SEG_ELEMS : T == kF16 ? SEG_ELEMS / 2 : SEG_ELEMS / 4;  // int8 quads / f32 words / f16 pairs
};

// XOR swizzle of B word index: the 16 chunk-threads of a row read 16-byte
// piece p of chunk ch; piece p^ch spreads them over 16 bank slots.
__device__ __forceinline__ int swz(int wi) {
  return (wi & ~63) | ((((wi >> 2) & 15) ^ ((wi >> 6) & 15)) << 2) | (wi & 3);
}

template <int T, int NC>
struct Smem {
  using GG = Geo<T>;
  uint32_t a[GG::A_LDS / 4];
  uint32_t bq[NC][GG::BQ_WORDS];
  float bd[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  float bx[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];   // q8_0: sum(q) as float; q8_1: s
  int bs[NC][Fmt<T>::VQK == 256 ? GG::VBLK * 16 : 1];  // q8_K bsums
};

// ---- stage the activation segment (decoded) into LDS --------------------------
// ggml's INIT quantization of F32 activations (AVX2 from_float flavour: d = amax/127,
// id = 127/amax, round-half-even; q8_1 also s = fp16(d * sum q)), done per 32-block while
// staging B, so a decode GEMV needs no separate quantize launch.  Produces exactly the bytes
// quant_q8_32<.., flavour 1> writes (lamm_quantize.hip), then the same LDS image stage_b
// builds from them: quads, fp32(fp16 d), and sum q (q8_0) or fp32(fp16 s) (q8_1).
template <int T, int NC, class SM>
__device__ __forceinline__ void stage_b_f32(SM& sm, const GemvArgs& p, const unsigned char* Bz, int seg) {
  using GG = Geo<T>;
  using F = Fmt<T>;
  const int64_t bbytes = (int64_t)(p.N - 1) * p.ldb + (int64_t)p.K * 4;
  const auto rs = make_rsrc(Bz, (uint32_t)min(bbytes, (int64_t)0x7fffffff));
  for (int it = threadIdx.x; it < NC * GG::VBLK; it += kThreads) {
    const int j = it / GG::VBLK, bi = it % GG::VBLK;
    const int gb = seg * GG::VBLK + bi;
    const bool ok = j < p.N && gb * 32 < p.K;
    const uint32_t off = ok ? (uint32_t)(j * p.ldb + (int64_t)gb * 128) : 0x7ffffff0u;
    float x[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) x[k] = __builtin_bit_cast(float, bload4(rs, off + 4 * k));
    float amax = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k) amax = fmaxf(amax, fabsf(x[k]));
    const float d = amax / 127.f;
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    int sum = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      uint32_t qw = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int r = avx_cvt_i32(__builtin_rintf(x[4 * k + e] * id));
        sum = (int)((uint32_t)sum + (uint32_t)r);   // before the saturation, wrapping (AVX2 q8_1's s)
        r = r > 127 ? 127 : (r < -128 ? -128 : r);
        qw |= (uint32_t)(r & 0xff) << (8 * e);
      }
      sm.bq[j][swz(bi * 8 + k)] = qw;
    }
    float dh = d;
    asm volatile("" : "+v"(dh));   // keep the fp16 round trip a separate conversion
    sm.bd[j][bi] = (float)(_Float16)dh;
    if constexpr (F::VBPB == 36) {
      float sd = (float)sum * d;
      asm volatile("" : "+v"(sd));
      sm.bx[j][bi] = (float)(_Float16)sd;
    } else {
      sm.bx[j][bi] = (float)sum;
    }
  }
}

template <int T, int NC, class SM>
__device__ __forceinline__ void stage_b(SM& sm, const GemvArgs& p, const unsigned char* Bz, int seg) {
  using GG = Geo<T>;
  using F = Fmt<T>;
  const int t = threadIdx.x;
  if constexpr (T != kF32 && T != kF16 && F::VQK == 32) {
    if (p.b_f32) {   // F32 rows quantized here: quant_q8_32 flavour 1 (lamm_quantize.hip)
      stage_b_f32<T, NC>(sm, p, Bz, seg);
      return;
    }
  }
  const int64_t bbytes = (int64_t)(p.N - 1) * p.ldb + (int64_t)(p.K / F::VQK) * F::VBPB;
  // range-checked per dword: round up so a dword straddling the logical end is read
  // (allocations are readable to the next 4-byte boundary: include/lamm_hip.h)
  const auto rs = make_rsrc(Bz, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
  if constexpr (T == kF32) {
    // f32 activations: straight words
    for (int it = t; it < NC * GG::BQ_WORDS; it += kThreads) {
      const int j = it / GG::BQ_WORDS, w = it % GG::BQ_WORDS;
      const int64_t e = (int64_t)seg * GG::SEG_ELEMS + w;
      uint32_t v = 0;
      if (j < p.N && e < p.K) v = bload4(rs, (uint32_t)(j * p.ldb + e * 4));
      sm.bq[j][swz(w)] = v;
    }
  } else if constexpr (T == kF16) {
    // f16 rows (ggml INIT converted src1 with ggml_fp32_to_fp16_row): pairs of halves,
    // read with 2-byte loads (F16 rows need not be dword aligned); past K -> 0
    for (int it = t; it < NC * GG::BQ_WORDS; it += kThreads) {
      const int j = it / GG::BQ_WORDS, w = it % GG::BQ_WORDS;
      const int64_t e = (int64_t)seg * GG::SEG_ELEMS + 2 * w;
      uint32_t lo = 0, hi = 0;
      if (j < p.N && e < p.K) lo = bload2(rs, (uint32_t)(j * p.ldb + e * 2));
      if (j < p.N && e + 1 < p.K) hi = bload2(rs, (uint32_t)(j * p.ldb + e * 2 + 2));
      sm.bq[j][swz(w)] = lo | (hi << 16);
    }
  } else if constexpr (F::VQK == 256) {
    // q8_K: f32 d | 256 x i8 | 16 x i16 bsums  = 73 dwords, dword aligned
    for (int it = t; it < NC * GG::VBLK * 73; it += kThreads) {
      const int j = it / (GG::VBLK * 73), r = it % (GG::VBLK * 73);
      const int sb = r / 73, k = r % 73;
      const int gsb = seg * GG::VBLK + sb;
      uint32_t v = 0;
      if (j < p.N && gsb * 256 < p.K) v = bload4(rs, (uint32_t)(j * p.ldb + gsb * 292 + 4 * k));
      if (k == 0) {
        sm.bd[j][sb] = __builtin_bit_cast(float, v);
      } else if (k <= 64) {
        sm.bq[j][swz(sb * 64 + k - 1)] = v;
      } else {
        sm.bs[j][sb * 16 + 2 * (k - 65)] = (int)(int16_t)(v & 0xffff);
        sm.bs[j][sb * 16 + 2 * (k - 65) + 1] = (int)(int16_t)(v >> 16);
      }
    }
  } else {
    // q8_0 (34 B) / q8_1 (36 B): one block per item, 10 dword loads from the
    // dword-aligned address at or below the block.
    constexpr int VQS = F::VBPB == 36 ? 4 : 2;
    for (int it = t; it < NC * GG::VBLK; it += kThreads) {
      const int j = it / GG::VBLK, bi = it % GG::VBLK;
      const int gb = seg * GG::VBLK + bi;
      const bool ok = j < p.N && gb * 32 < p.K;
      const uint32_t off = ok ? (uint32_t)(j * p.ldb + (int64_t)gb * F::VBPB) : 0xfffffff0u;
      const uint32_t base = off & ~3u;
      const int sh = (int)(off & 3u);
      uint32_t w[10], m[10];
#pragma unroll
      for (int k = 0; k < 10; ++k) w[k] = bload4(rs, base + 4 * k);
      // realign: m = the block's bytes as dwords from its first byte
#pragma unroll
      for (int k = 0; k < 9; ++k) m[k] = __builtin_amdgcn_alignbit(w[k + 1], w[k], sh * 8);
      m[9] = 0;
      const uint32_t h0 = m[0];
      float sx = 0.f;
      unroll<8>([&](auto K) {
        constexpr int k = K;
        const uint32_t q = get32<VQS + 4 * k>(m);
        sm.bq[j][swz(bi * 8 + k)] = q;
        if constexpr (VQS == 2) sx += (float)dot4(q, 0x01010101u, 0);
      });
      sm.bd[j][bi] = h2f(h0 & 0xffff);
      if constexpr (VQS == 4) sx = h2f(h0 >> 16);
      sm.bx[j][bi] = sx;
    }
  }
}

// ---- one A block (compile-time position G_IDX in the chunk) x NC columns -------
template <int T, int NC, int GI, class SM>
__device__ __forceinline__ void block_dot(const uint32_t (&w)[Geo<T>::CH_WORDS + 1], const SM& sm,
                                          int ch, int ncols, float (&acc)[NC]) {
  using F = Fmt<T>;
  constexpr int O = GI * F::BPB;
  const int bi = ch * F::G + GI;                 // block index within segment
  if constexpr (T == kQ2_K) {
    // block_q2_K: scales[16] @0, qs[64] @16, d @80, dmin @82 ; B = q8_K
    uint32_t sc[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) sc[k] = w[k];
    const float da = h2f(w[20] & 0xffff), dm = h2f(w[20] >> 16);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j >= ncols) break;
      const uint32_t* bq = sm.bq[j];
      int isum = 0, summs = 0;
#pragma unroll
      for (int n = 0; n < 2; ++n) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int s = 8 * n + 2 * jj + h;
            const int scv = (sc[s >> 2] >> (8 * (s & 3))) & 0xff;
            const u32x4 b = *(const u32x4*)&bq[swz(ch * 64 + 32 * n + 8 * jj + 4 * h)];
            int part = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const uint32_t q = (w[4 + 8 * n + 4 * h + k] >> (2 * jj)) & 0x03030303u;
              part = dot4(q, b[k], part);
            }
            isum += (scv & 0xf) * part;
            summs += sm.bs[j][ch * 16 + s] * (scv >> 4);
          }
        }
      }
      const float yd = sm.bd[j][ch];
      acc[j] += (yd * da) * (float)isum - (yd * dm) * (float)summs;
    }
  } else if constexpr (T == kQ4_K || T == kQ5_K) {
    // block_q4_K: d, dmin @0 | scales[12] @4 | qs[128] @16 ; block_q5_K: qh[32] @16, qs @48.
    // 6-bit scales / mins: the utmp shuffle of LC/ggml-quants.c:7324-7330.  Element
    // 32*sb + l: nibble (sb & 1) of qs[32*(sb >> 1) + l] (+16 if bit sb of qh[l]).
    static_assert(O == 0, "k-quant chunks hold one super-block");
    constexpr bool Q5 = T == kQ5_K;
    constexpr int QS = Q5 ? 12 : 4;   // dword index of qs
    uint32_t u0 = w[1], u1 = w[2], u2 = w[3];
    const uint32_t u3 = ((u2 >> 4) & 0x0f0f0f0fu) | (((u1 >> 6) & 0x03030303u) << 4);
    const uint32_t uaux = u1 & 0x3f3f3f3fu;
    u1 = (u2 & 0x0f0f0f0fu) | (((u0 >> 6) & 0x03030303u) << 4);
    u2 = uaux;
    u0 &= 0x3f3f3f3fu;
    const float da = h2f(w[0] & 0xffff), dm = h2f(w[0] >> 16);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j >= ncols) break;
      const uint32_t* bq = sm.bq[j];
      int isum = 0, summ = 0;
#pragma unroll
      for (int sb = 0; sb < 8; ++sb) {
        const int sc = (int)(((sb < 4 ? u0 : u1) >> (8 * (sb & 3))) & 0xffu);
        const int mn = (int)(((sb < 4 ? u2 : u3) >> (8 * (sb & 3))) & 0xffu);
        int part = 0;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u32x4 b = *(const u32x4*)&bq[swz(ch * 64 + 8 * sb + 4 * h)];
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            uint32_t q = (w[QS + 8 * (sb >> 1) + 4 * h + k] >> (4 * (sb & 1))) & 0x0f0f0f0fu;
            if constexpr (Q5) q |= ((w[4 + 4 * h + k] >> sb) & 0x01010101u) << 4;
            part = dot4(q, b[k], part);
          }
        }
        isum += sc * part;
        summ += mn * (sm.bs[j][ch * 16 + 2 * sb] + sm.bs[j][ch * 16 + 2 * sb + 1]);
      }
      const float yd = sm.bd[j][ch];
      acc[j] += (yd * da) * (float)isum - (yd * dm) * (float)summ;
    }
  } else if constexpr (T == kQ6_K) {
    // block_q6_K: ql[128] @0 | qh[64] @128 | scales[16] (int8) @192 | d @208.  Element
    // 128*hf + 32*part + l = (nibble (part >> 1) of ql[64*hf + 32*(part & 1) + l]
    //   | ((qh[32*hf + l] >> 2*part) & 3) << 4) - 32     (LC/ggml-quants.c:8710-8720)
    static_assert(O == 0, "k-quant chunks hold one super-block");
    const float da = h2f(w[52] & 0xffff);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j >= ncols) break;
      const uint32_t* bq = sm.bq[j];
      int isum = 0;
#pragma unroll
      for (int sb = 0; sb < 8; ++sb) {
        const int hf = sb >> 2, part = sb & 3;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const u32x4 b = *(const u32x4*)&bq[swz(ch * 64 + 8 * sb + 4 * h)];
          int s16 = 0;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int kk = 4 * h + k;
            const uint32_t nw = w[16 * hf + 8 * (part & 1) + kk];
            const uint32_t nib = (part < 2 ? nw : (nw >> 4)) & 0x0f0f0f0fu;
            const uint32_t hb = ((w[32 + 8 * hf + kk] >> (2 * part)) & 0x03030303u) << 4;
            // per byte (q - 32) with q = nib | hb in [0, 63]: no borrow crosses a byte
            const uint32_t q = (((nib | hb) | 0x80808080u) - 0x20202020u) ^ 0x80808080u;
            s16 = dot4(q, b[k], s16);
          }
          const int si = 2 * sb + h;
          const int scale = (int)(int8_t)((w[48 + (si >> 2)] >> (8 * (si & 3))) & 0xffu);
          isum += scale * s16;
        }
      }
      acc[j] += (sm.bd[j][ch] * da) * (float)isum;
    }
  } else {
    // 32-element blocks.  Unpack to 8 int8 words (elements 0-15 = low nibbles,
    // 16-31 = high nibbles; the 5th bit from qh), exact int32 dot with v_dot4.
    uint32_t q[8];
    float da, ma = 0.f;
    if constexpr (T == kQ8_0) {
      da = h2f(get16<O>(w));
      unroll<8>([&](auto K) { q[K] = get32<O + 2 + 4 * K>(w); });
    } else {
      constexpr bool AFF = (T == kQ4_1 || T == kQ5_1);
      constexpr bool FIVE = (T == kQ5_0 || T == kQ5_1);
      constexpr int QS = (AFF ? 4 : 2) + (FIVE ? 4 : 0);
      da = h2f(get16<O>(w));
      if constexpr (AFF) ma = h2f(get16<O + 2>(w));
      uint32_t qh = 0;
      if constexpr (FIVE) qh = get32<O + (AFF ? 4 : 2)>(w);
      unroll<4>([&](auto K) {
        constexpr int k = K;
        const uint32_t x = get32<O + QS + 4 * k>(w);
        q[k] = x & 0x0f0f0f0fu;
        q[4 + k] = (x >> 4) & 0x0f0f0f0fu;
        if constexpr (FIVE) {
          q[k] |= spread4_hi((qh >> (4 * k)) & 0xf);
          q[4 + k] |= spread4_hi((qh >> (16 + 4 * k)) & 0xf);
        }
      });
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      if (j >= ncols) break;
      const uint32_t* bq = sm.bq[j];
      const u32x4 b0 = *(const u32x4*)&bq[swz(ch * 64 + 8 * GI)];
      const u32x4 b1 = *(const u32x4*)&bq[swz(ch * 64 + 8 * GI + 4)];
      int s = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) s = dot4(q[k], b0[k], s);
#pragma unroll
      for (int k = 0; k < 4; ++k) s = dot4(q[4 + k], b1[k], s);
      const float db = sm.bd[j][bi], bx = sm.bx[j][bi];
      if constexpr (T == kQ4_0) {
        acc[j] += (da * db) * ((float)s - 8.f * bx);     // sum (q-8) b = sum q b - 8 sum b
      } else if constexpr (T == kQ5_0) {
        acc[j] += (da * db) * ((float)s - 16.f * bx);
      } else if constexpr (T == kQ8_0) {
        acc[j] += (da * db) * (float)s;
      } else {  // q4_1 / q5_1 against q8_1: d_a d_b S + m_a s_b
        acc[j] += (da * db) * (float)s + ma * bx;
      }
    }
  }
}

// f32: the chunk is 64 consecutive floats; elements past K (nvalid) are masked so
// row padding (possibly NaN) never reaches the sum.
template <int NC, class SM>
__device__ __forceinline__ void chunk_dot_f32(const uint32_t (&w)[Geo<kF32>::CH_WORDS + 1],
                                              const SM& sm, int ch, int nvalid, int ncols,
                                              float (&acc)[NC]) {
  float a[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) a[i] = i < nvalid ? __builtin_bit_cast(float, w[i]) : 0.f;
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (j >= ncols) break;
    const uint32_t* bq = sm.bq[j];
    float s = 0.f;
#pragma unroll
    for (int pc = 0; pc < 16; ++pc) {
      const u32x4 b = *(const u32x4*)&bq[swz(ch * 64 + 4 * pc)];
#pragma unroll
      for (int k = 0; k < 4; ++k) s = __builtin_fmaf(a[4 * pc + k], __uint_as_float((uint32_t)b[k]), s);
    }
    acc[j] += s;
  }
}

// f16 (e.g. the F16 KV cache of the attention matmuls): 128 halves per chunk,
// exact fp16 x fp16 products with fp32 accumulation (v_dot2_f32_f16); halves past K masked.
template <int NC, class SM>
__device__ __forceinline__ void chunk_dot_f16(const uint32_t (&w)[Geo<kF16>::CH_WORDS + 1],
                                              const SM& sm, int ch, int nvalid, int ncols,
                                              float (&acc)[NC]) {
  typedef _Float16 h2 __attribute__((ext_vector_type(2)));
  uint32_t a[64];
#pragma unroll
  for (int i = 0; i < 64; ++i) {
    const uint32_t m = 2 * i + 1 < nvalid ? 0xffffffffu : (2 * i < nvalid ? 0x0000ffffu : 0u);
    a[i] = w[i] & m;
  }
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    if (j >= ncols) break;
    const uint32_t* bq = sm.bq[j];
    float s = 0.f;
#pragma unroll
    for (int pc = 0; pc < 16; ++pc) {
      const u32x4 b = *(const u32x4*)&bq[swz(ch * 64 + 4 * pc)];
#pragma unroll
      for (int k = 0; k < 4; ++k)
        s = __builtin_amdgcn_fdot2(__builtin_bit_cast(h2, a[4 * pc + k]), __builtin_bit_cast(h2, (uint32_t)b[k]), s,
                                   false);
    }
    acc[j] += s;
  }
}

template <int T, int NC, int GI, class SM>
__device__ __forceinline__ void chunk_dot(const uint32_t (&w)[Geo<T>::CH_WORDS + 1], const SM& sm,
                                          int ch, int nvalid, int ncols, float (&acc)[NC]) {
  if constexpr (T == kF32) {
    chunk_dot_f32<NC>(w, sm, ch, nvalid, ncols, acc);
  } else if constexpr (T == kF16) {
    chunk_dot_f16<NC>(w, sm, ch, nvalid, ncols, acc);
  } else if constexpr (GI < Fmt<T>::G) {
    if (GI < nvalid) block_dot<T, NC, GI>(w, sm, ch, ncols, acc);
    chunk_dot<T, NC, GI + 1>(w, sm, ch, nvalid, ncols, acc);
  }
}

// V (A staging variant): 0 = 16-byte buffer loads to VGPRs + ds_write;
// 1 = LDS-DMA (buffer_load_dwordx4 ... lds) with the non-temporal policy (A is read
// once); 2 = LDS-DMA, default policy; 3 = VGPR staging with non-temporal loads.
template <int T, int NC, int V = 0>
__global__ __launch_bounds__(kThreads) void gemv_kernel(GemvArgs p) {
  using GG = Geo<T>;
  using F = Fmt<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  Smem<T, NC>& sm = *reinterpret_cast<Smem<T, NC>*>(smem_raw);

  const int t = threadIdx.x;
  const int row = t / kSC, ch = t % kSC;
  const int64_t r0 = (int64_t)blockIdx.x * kRows;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int rows = (int)min((int64_t)kRows, (int64_t)p.M - r0);
  const int row_bytes = p.nblk * F::BPB;                   // bytes of one A row
  const int nseg = (p.nblk + GG::SEG_BLK - 1) / GG::SEG_BLK;
  const int ncols = p.N < NC ? p.N : NC;

  float acc[NC];
#pragma unroll
  for (int j = 0; j < NC; ++j) acc[j] = 0.f;

  for (int seg = 0; seg < nseg; ++seg) {
    // ---- issue the A segment loads (HBM stream) ----
    const unsigned char* abase = Az + r0 * p.lda + (int64_t)seg * GG::ROW_BYTES;
    const int64_t avail = (int64_t)(rows - 1) * p.lda + row_bytes - (int64_t)seg * GG::ROW_BYTES;
    const auto ra = make_rsrc(abase, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
    [[maybe_unused]] u32x4 v[GG::A_NPT];
#pragma unroll
    for (int k = 0; k < GG::A_NPT; ++k) {
      const int pc = t + k * kThreads;
      const int rr = pc / (GG::ROW_BYTES / 16), oo = pc % (GG::ROW_BYTES / 16);
      const uint32_t off = (pc < GG::A_PIECES && rr < rows) ? (uint32_t)(rr * p.lda + 16 * oo) : 0x7ffffff0u;
      if constexpr (V == 1 || V == 2 || V >= 4) {
        // lane-linear LDS destination: wave-uniform base + 16 * lane
        const int wbase = k * kThreads + (t & ~63);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            ra, (__attribute__((address_space(3))) void*)(sm.a + 4 * wbase), 16, off, 0, 0, V == 2 ? 0 : 2);
      } else if constexpr (V == 3) {
        v[k] = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 2);
      } else {
        v[k] = bload16(ra, off);
      }
    }
    // ---- activations (L2-resident) decoded into LDS ----
    if constexpr (V != 5) stage_b<T, NC>(sm, p, Bz, seg);
    if constexpr (V == 0 || V == 3) {
#pragma unroll
      for (int k = 0; k < GG::A_NPT; ++k) *(u32x4*)&sm.a[4 * (t + k * kThreads)] = v[k];
    }
    __syncthreads();

    // ---- compute this thread's chunk ----
    const int cb0 = seg * GG::SEG_BLK + ch * F::G;           // first A block of chunk
    if (V != 4 && row < rows && cb0 < p.nblk) {
      uint32_t w[GG::CH_WORDS + 1];
      const int cbyte = row * GG::ROW_BYTES + ch * GG::CH_BYTES;
      const uint32_t* src = &sm.a[cbyte / 4];
      if constexpr (GG::CH_BYTES % 4 != 0) {   // q6_K: 210-byte chunks, 2-byte aligned
        const int sh = (cbyte & 3) * 8;
#pragma unroll
        for (int k = 0; k < GG::CH_WORDS; ++k) w[k] = __builtin_amdgcn_alignbit(src[k + 1], src[k], sh);
      } else if constexpr (GG::CH_BYTES % 16 == 0) {
#pragma unroll
        for (int k = 0; k < GG::CH_WORDS / 4; ++k) {
          const u32x4 x = *(const u32x4*)&src[4 * k];
          w[4 * k] = x[0]; w[4 * k + 1] = x[1]; w[4 * k + 2] = x[2]; w[4 * k + 3] = x[3];
        }
      } else {
#pragma unroll
        for (int k = 0; k < GG::CH_WORDS; ++k) w[k] = src[k];
      }
      w[GG::CH_WORDS] = 0;
      const int nvalid = min(F::G, p.nblk - cb0);
      chunk_dot<T, NC, 0>(w, sm, ch, nvalid, ncols, acc);
    }
    __syncthreads();
  }

  // ---- reduce the 16 chunk partials of each row (fixed order) ----
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    float x = acc[j];
    x += __shfl_xor(x, 8);
    x += __shfl_xor(x, 4);
    x += __shfl_xor(x, 2);
    x += __shfl_xor(x, 1);
    acc[j] = x;
  }
  if (ch == 0 && row < rows) {
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (j < ncols) Cz[(int64_t)j * p.ldc + r0 + row] = acc[j];
  }
}

// ---- wave-streaming single-segment kernel (K <= one segment: 4096 elements) --------
// Each WAVE owns groups of 4 rows (its 64 lanes = 4 rows x 16 chunks).  Group g+1 is
// loaded HBM -> VGPRs (non-temporal 16-byte buffer loads) while group g is computed
// from the wave's private LDS slot, so every wave keeps a group in flight during its
// compute and the register file (3x the LDS) is the landing zone.  A wave reads only
// the LDS bytes it wrote itself: no workgroup barrier in the loop, the waves of a CU
// desynchronise.  B is decoded once per workgroup and reused by all its groups.
constexpr int kWRows = 4;   // rows per wave group

template <int T> struct WGeo {
  using GG = Geo<T>;
  static constexpr int BYTES = kWRows * GG::ROW_BYTES;    // one wave group
  static constexpr int NPW = (BYTES + 1023) / 1024;       // 16-byte loads per lane
  static constexpr int SLOT = NPW * 1024;
};

template <int T, int NC, int WAVES>
struct SmemStream {
  using GG = Geo<T>;
  uint32_t a[WAVES][WGeo<T>::SLOT / 4];
  uint32_t bq[NC][GG::BQ_WORDS];
  float bd[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  float bx[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  int bs[NC][Fmt<T>::VQK == 256 ? GG::VBLK * 16 : 1];
};

template <int T, int NC, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void gemv_stream_kernel(GemvArgs p) {
  using GG = Geo<T>;
  using WG = WGeo<T>;
  using F = Fmt<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SmemStream<T, NC, WAVES>& sm = *reinterpret_cast<SmemStream<T, NC, WAVES>*>(smem_raw);

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int row = lane / kSC, ch = lane % kSC;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int row_bytes = p.nblk * F::BPB;
  const int ncols = p.N < NC ? p.N : NC;
  const int stride = gridDim.x * WAVES;

  u32x4 v[WG::NPW];
  auto load = [&](int q) {
    const int64_t r0 = (int64_t)q * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    const int64_t avail = (int64_t)(rows - 1) * p.lda + row_bytes;
    const auto ra = make_rsrc(Az + r0 * p.lda, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
#pragma unroll
    for (int k = 0; k < WG::NPW; ++k) {
      const int pc = lane + 64 * k;
      const int rr = pc / (GG::ROW_BYTES / 16), oo = pc % (GG::ROW_BYTES / 16);
      const uint32_t off = (pc * 16 < WG::BYTES && rr < rows) ? (uint32_t)(rr * p.lda + 16 * oo) : 0x7ffffff0u;
      v[k] = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 2);   // nt: streamed once
    }
  };

  int q = blockIdx.x * WAVES + w;
  if (q < ngroups) load(q);
  stage_b<T, NC>(sm, p, Bz, 0);
  __syncthreads();   // B visible to every wave

  for (; q < ngroups; q += stride) {
#pragma unroll
    for (int k = 0; k < WG::NPW; ++k) *(u32x4*)&sm.a[w][4 * (lane + 64 * k)] = v[k];
    const int qn = q + stride;
    if (qn < ngroups) load(qn);      // in flight during this group's compute

    const int64_t r0 = (int64_t)q * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = 0.f;
    const int cb0 = ch * F::G;
    if (row < rows && cb0 < p.nblk) {
      uint32_t wv[GG::CH_WORDS + 1];
      const int cbyte = row * GG::ROW_BYTES + ch * GG::CH_BYTES;
      const uint32_t* src = &sm.a[w][cbyte / 4];
      if constexpr (GG::CH_BYTES % 4 != 0) {   // q6_K: 210-byte chunks, 2-byte aligned
        const int sh = (cbyte & 3) * 8;
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = __builtin_amdgcn_alignbit(src[c + 1], src[c], sh);
      } else if constexpr (GG::CH_BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS / 4; ++c) {
          const u32x4 x = *(const u32x4*)&src[4 * c];
          wv[4 * c] = x[0]; wv[4 * c + 1] = x[1]; wv[4 * c + 2] = x[2]; wv[4 * c + 3] = x[3];
        }
      } else {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = src[c];
      }
      wv[GG::CH_WORDS] = 0;
      chunk_dot<T, NC, 0>(wv, sm, ch, min(F::G, p.nblk - cb0), ncols, acc);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      float x = acc[j];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 4);
      x += __shfl_xor(x, 2);
      x += __shfl_xor(x, 1);
      acc[j] = x;
    }
    if (ch == 0 && row < rows) {
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if (j < ncols) Cz[(int64_t)j * p.ldc + r0 + row] = acc[j];
    }
  }
}

// ---- LDS-DMA variant of the streaming kernel (A/B: LAMM_GEMV_VARIANT=8 / 9) ----------------
// Group bytes go HBM -> LDS directly (buffer_load ... lds, non-temporal), NS slots per wave, NS-1
// groups in flight; no VGPR landing zone and no ds_write pass.  A wave reads only the slots its
// own DMAs filled, so its counted vmcnt is the only ordering needed (no barrier in the loop).
template <int T, int NC, int WAVES, int NS>
struct SmemStreamD {
  using GG = Geo<T>;
  uint32_t a[WAVES][NS][WGeo<T>::SLOT / 4];
  uint32_t bq[NC][GG::BQ_WORDS];
  float bd[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  float bx[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  int bs[NC][Fmt<T>::VQK == 256 ? GG::VBLK * 16 : 1];
};

template <int T, int NC>
struct alignas(16) BPart {   // 16-byte aligned: a part at index > 0 is read with ds_read_b128
  using GG = Geo<T>;
  uint32_t bq[NC][GG::BQ_WORDS];
  float bd[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  float bx[NC][(T == kF32 || T == kF16) ? 1 : GG::VBLK];
  int bs[NC][Fmt<T>::VQK == 256 ? GG::VBLK * 16 : 1];
};

template <int N_>
__device__ __forceinline__ void gv_wait_vm() {   // s_waitcnt vmcnt(N) (lgkmcnt untouched)
  static_assert(N_ >= 0 && N_ < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N_ & 0xF) | ((N_ >> 4) << 14) | (0x7 << 4) | (0xF << 8));
  asm volatile("" ::: "memory");
}

template <int T, int NC, int WAVES, int NS>
__global__ __launch_bounds__(64 * WAVES) void gemv_stream_dma_kernel(GemvArgs p) {
  using GG = Geo<T>;
  using WG = WGeo<T>;
  using F = Fmt<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SmemStreamD<T, NC, WAVES, NS>& sm = *reinterpret_cast<SmemStreamD<T, NC, WAVES, NS>*>(smem_raw);
  static_assert(WG::NPW * (NS - 1) < 64, "vmcnt range");

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int row = lane / kSC, ch = lane % kSC;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int row_bytes = p.nblk * F::BPB;
  const int ncols = p.N < NC ? p.N : NC;
  const int stride = gridDim.x * WAVES;

  auto issue = [&](int q, int slot) {
    const int64_t r0 = (int64_t)q * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    const int64_t avail = (int64_t)(rows - 1) * p.lda + row_bytes;
    const auto ra = make_rsrc(Az + r0 * p.lda, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
#pragma unroll
    for (int k = 0; k < WG::NPW; ++k) {
      const int pc = lane + 64 * k;
      const int rr = pc / (GG::ROW_BYTES / 16), oo = pc % (GG::ROW_BYTES / 16);
      const uint32_t off = (pc * 16 < WG::BYTES && rr < rows) ? (uint32_t)(rr * p.lda + 16 * oo) : 0x7ffffff0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)&sm.a[w][slot][4 * 64 * k], 16, off, 0, 0, 2);
    }
  };

  const int q0 = blockIdx.x * WAVES + w;
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (q0 + k * stride < ngroups) issue(q0 + k * stride, k);
  stage_b<T, NC>(sm, p, Bz, 0);
  __syncthreads();   // B visible to every wave

  int it = 0;
  for (int q = q0; q < ngroups; q += stride, ++it) {
    const int slot = it % NS;
    {   // refill the slot consumed one iteration ago (its LDS reads retired: lgkmcnt(0))
      const int qn = q + (NS - 1) * stride;
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (qn < ngroups) issue(qn, (it + NS - 1) % NS);
    }
    // groups issued after q that are still allowed in flight
    const int after = min(NS - 1, (ngroups - 1 - q) / stride);
    if constexpr (NS >= 4) {
      if (after >= 3) gv_wait_vm<3 * WG::NPW>();
      else if (after == 2) gv_wait_vm<2 * WG::NPW>();
      else if (after == 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    } else if constexpr (NS == 3) {
      if (after >= 2) gv_wait_vm<2 * WG::NPW>();
      else if (after == 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    } else {
      if (after >= 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    }

    const int64_t r0 = (int64_t)q * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = 0.f;
    const int cb0 = ch * F::G;
    if (row < rows && cb0 < p.nblk) {
      uint32_t wv[GG::CH_WORDS + 1];
      const int cbyte = row * GG::ROW_BYTES + ch * GG::CH_BYTES;
      const uint32_t* src = &sm.a[w][slot][cbyte / 4];
      if constexpr (GG::CH_BYTES % 4 != 0) {
        const int sh = (cbyte & 3) * 8;
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = __builtin_amdgcn_alignbit(src[c + 1], src[c], sh);
      } else if constexpr (GG::CH_BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS / 4; ++c) {
          const u32x4 x = *(const u32x4*)&src[4 * c];
          wv[4 * c] = x[0]; wv[4 * c + 1] = x[1]; wv[4 * c + 2] = x[2]; wv[4 * c + 3] = x[3];
        }
      } else {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = src[c];
      }
      wv[GG::CH_WORDS] = 0;
      chunk_dot<T, NC, 0>(wv, sm, ch, min(F::G, p.nblk - cb0), ncols, acc);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      float x = acc[j];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 4);
      x += __shfl_xor(x, 2);
      x += __shfl_xor(x, 1);
      acc[j] = x;
    }
    if (ch == 0 && row < rows) {
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if (j < ncols) Cz[(int64_t)j * p.ldc + r0 + row] = acc[j];
    }
  }
}

template <int T, int NC, int WAVES, int NS>
hipError_t launch_stream_dma(const GemvArgs& p, hipStream_t s) {
  constexpr size_t lds = sizeof(SmemStreamD<T, NC, WAVES, NS>);
  static_assert(lds <= 160 * 1024, "LDS");
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int slices = p.ne12 * p.ne13;
  const int per_cu = (int)((160 * 1024) / lds) < 1 ? 1 : (int)((160 * 1024) / lds);
  int gx = (256 * per_cu) / slices;
  const int gmax = (ngroups + WAVES - 1) / WAVES;
  gx = gx < 1 ? 1 : (gx > gmax ? gmax : gx);
  set_max_lds((const void*)gemv_stream_dma_kernel<T, NC, WAVES, NS>, (int)lds);
  hipLaunchKernelGGL((gemv_stream_dma_kernel<T, NC, WAVES, NS>), dim3(gx, slices), dim3(64 * WAVES), lds, s, p);
  return hipGetLastError();
}

// ---- multi-segment LDS-DMA streaming kernel (K up to NSEG x 4096: e.g. ffn_down's 11008) ---
// Work items are (4-row group, K-segment) pairs in group-major order per wave; the activation
// of every segment is staged once (one 16-byte aligned part per segment), partial sums carry
// across a group's segments, C is written after its last one.  Pieces past the row's last
// byte (ragged last segment) are pointed out of range, so they land as zeros.
template <int T, int NC, int WAVES, int NS, int NSEG>
struct SmemSegD {
  uint32_t a[WAVES][NS][WGeo<T>::SLOT / 4];
  BPart<T, NC> b[NSEG];
};

template <int T, int NC, int WAVES, int NS, int NSEG>
__global__ __launch_bounds__(64 * WAVES) void gemv_seg_dma_kernel(GemvArgs p) {
  using GG = Geo<T>;
  using WG = WGeo<T>;
  using F = Fmt<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SmemSegD<T, NC, WAVES, NS, NSEG>& sm = *reinterpret_cast<SmemSegD<T, NC, WAVES, NS, NSEG>*>(smem_raw);
  static_assert(WG::NPW * (NS - 1) < 64, "vmcnt range");

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int row = lane / kSC, ch = lane % kSC;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int row_bytes = p.nblk * F::BPB;
  const int nseg = (p.nblk + GG::SEG_BLK - 1) / GG::SEG_BLK;   // <= NSEG (launcher)
  const int ncols = p.N < NC ? p.N : NC;
  const int stride = gridDim.x * WAVES;
  const int q0 = blockIdx.x * WAVES + w;
  // this wave's items: k -> (group q0 + (k / nseg) * stride, segment k % nseg)
  const int ngw = q0 < ngroups ? (ngroups - 1 - q0) / stride + 1 : 0;
  const int nitems = ngw * nseg;

  auto issue = [&](int k, int slot) {
    const int q = q0 + (k / nseg) * stride, sg = k % nseg;
    const int64_t r0 = (int64_t)q * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    const int64_t avail = (int64_t)(rows - 1) * p.lda + row_bytes;
    const auto ra = make_rsrc(Az + r0 * p.lda, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
#pragma unroll
    for (int kk = 0; kk < WG::NPW; ++kk) {
      const int pc = lane + 64 * kk;
      const int rr = pc / (GG::ROW_BYTES / 16), oo = pc % (GG::ROW_BYTES / 16);
      const int cbyte = sg * GG::ROW_BYTES + 16 * oo;   // byte within the row
      const uint32_t off =
          (pc * 16 < WG::BYTES && rr < rows && cbyte < row_bytes) ? (uint32_t)(rr * p.lda + cbyte) : 0x7ffffff0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)&sm.a[w][slot][4 * 64 * kk], 16, off, 0, 0, 2);
    }
  };

#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (k < nitems) issue(k, k);
  for (int sg = 0; sg < nseg; ++sg) stage_b<T, NC>(sm.b[sg], p, Bz, sg);
  __syncthreads();   // B visible to every wave

  float acc[NC];
  for (int k = 0; k < nitems; ++k) {
    const int slot = k % NS;
    {
      const int kn = k + NS - 1;
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (kn < nitems) issue(kn, kn % NS);
    }
    const int after = min(NS - 1, nitems - 1 - k);
    if constexpr (NS >= 3) {
      if (after >= 2) gv_wait_vm<2 * WG::NPW>();
      else if (after == 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    } else {
      if (after >= 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    }
    const int q = q0 + (k / nseg) * stride, sg = k % nseg;
    if (sg == 0) {
#pragma unroll
      for (int j = 0; j < NC; ++j) acc[j] = 0.f;
    }
    const int64_t r0 = (int64_t)q * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    const int cb0 = sg * GG::SEG_BLK + ch * F::G;
    if (row < rows && cb0 < p.nblk) {
      uint32_t wv[GG::CH_WORDS + 1];
      const int cbyte = row * GG::ROW_BYTES + ch * GG::CH_BYTES;
      const uint32_t* src = &sm.a[w][slot][cbyte / 4];
      if constexpr (GG::CH_BYTES % 4 != 0) {
        const int sh = (cbyte & 3) * 8;
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = __builtin_amdgcn_alignbit(src[c + 1], src[c], sh);
      } else if constexpr (GG::CH_BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS / 4; ++c) {
          const u32x4 x = *(const u32x4*)&src[4 * c];
          wv[4 * c] = x[0]; wv[4 * c + 1] = x[1]; wv[4 * c + 2] = x[2]; wv[4 * c + 3] = x[3];
        }
      } else {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = src[c];
      }
      wv[GG::CH_WORDS] = 0;
      chunk_dot<T, NC, 0>(wv, sm.b[sg], ch, min(F::G, p.nblk - cb0), ncols, acc);
    }
    if (sg == nseg - 1) {
      float o[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        float x = acc[j];
        x += __shfl_xor(x, 8);
        x += __shfl_xor(x, 4);
        x += __shfl_xor(x, 2);
        x += __shfl_xor(x, 1);
        o[j] = x;
      }
      if (ch == 0 && row < rows) {
#pragma unroll
        for (int j = 0; j < NC; ++j)
          if (j < ncols) Cz[(int64_t)j * p.ldc + r0 + row] = o[j];
      }
    }
  }
}

template <int T, int NC, int WAVES, int NS, int NSEG>
hipError_t launch_seg_dma(const GemvArgs& p, hipStream_t s) {
  const size_t lds = sizeof(SmemSegD<T, NC, WAVES, NS, NSEG>);
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int slices = p.ne12 * p.ne13;
  int gx = 256 / slices;
  const int gmax = (ngroups + WAVES - 1) / WAVES;
  gx = gx < 1 ? 1 : (gx > gmax ? gmax : gx);
  set_max_lds((const void*)gemv_seg_dma_kernel<T, NC, WAVES, NS, NSEG>, (int)lds);
  hipLaunchKernelGGL((gemv_seg_dma_kernel<T, NC, WAVES, NS, NSEG>), dim3(gx, slices), dim3(64 * WAVES), lds, s, p);
  return hipGetLastError();
}

// ---- flattened LDS-DMA streaming kernel: one workgroup per CU over ALL slices -----------
// With one 149 KiB workgroup per CU, a (groups-per-slice x slices) grid cannot match 256 CUs
// (33 slices -> 7 workgroups each = 231 busy CUs).  Here the (slice, group) list is flattened
// and cut into exactly one contiguous range per workgroup; a range spans at most two slices
// (the launcher guarantees it), whose activation rows are both staged in LDS.
template <int T, int NC, int WAVES, int NS>
struct SmemFlat {
  uint32_t a[WAVES][NS][WGeo<T>::SLOT / 4];
  BPart<T, NC> b[2];
};

template <int T, int NC, int WAVES, int NS>
__global__ __launch_bounds__(64 * WAVES) void gemv_flat_dma_kernel(GemvArgs p) {
  using GG = Geo<T>;
  using WG = WGeo<T>;
  using F = Fmt<T>;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  SmemFlat<T, NC, WAVES, NS>& sm = *reinterpret_cast<SmemFlat<T, NC, WAVES, NS>*>(smem_raw);
  static_assert(WG::NPW * (NS - 1) < 64, "vmcnt range");

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int row = lane / kSC, ch = lane % kSC;
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  // 32-bit (q, slice) arithmetic: the launcher bounds the flattened list below 2^31, and
  // 64-bit divides per group cost more than the group's decode
  const int total = ngroups * p.ne12 * p.ne13;
  const int g0 = (int)((int64_t)blockIdx.x * total / gridDim.x), g1 = (int)((int64_t)(blockIdx.x + 1) * total / gridDim.x);
  const int z0 = g0 / ngroups;
  const int row_bytes = p.nblk * F::BPB;
  const int ncols = p.N < NC ? p.N : NC;

  // (the slice base is computed inline: a lambda called from this lambda makes the host
  // pass of hipcc drop the kernel template as a substitution failure -- an undefined stub)
  auto issue = [&](int q, int slot) {
    const int z = q / ngroups, grp = q - z * ngroups;
    const int zi12 = z % p.ne12, zi13 = z / p.ne12;
    const unsigned char* Az = p.A + (int64_t)(zi12 / p.r2) * p.sa2 + (int64_t)(zi13 / p.r3) * p.sa3;
    const int64_t r0 = (int64_t)grp * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    const int64_t avail = (int64_t)(rows - 1) * p.lda + row_bytes;
    const auto ra = make_rsrc(Az + r0 * p.lda, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
#pragma unroll
    for (int k = 0; k < WG::NPW; ++k) {
      const int pc = lane + 64 * k;
      const int rr = pc / (GG::ROW_BYTES / 16), oo = pc % (GG::ROW_BYTES / 16);
      const uint32_t off = (pc * 16 < WG::BYTES && rr < rows) ? (uint32_t)(rr * p.lda + 16 * oo) : 0x7ffffff0u;
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          ra, (__attribute__((address_space(3))) void*)&sm.a[w][slot][4 * 64 * k], 16, off, 0, 0, 2);
    }
  };

  const int q0 = g0 + w;
#pragma unroll
  for (int k = 0; k < NS - 1; ++k)
    if (q0 + k * WAVES < g1) issue(q0 + k * WAVES, k);
  // activation rows of the (at most two) slices this range touches
  for (int k = 0; k < 2; ++k) {
    const int z = z0 + k;
    if (z < p.ne12 * p.ne13 && z * ngroups < g1) {
      const int i12 = z % p.ne12, i13 = z / p.ne12;
      stage_b<T, NC>(sm.b[k], p, p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3, 0);
    }
  }
  __syncthreads();

  int it = 0;
  for (int q = q0; q < g1; q += WAVES, ++it) {
    const int slot = it % NS;
    {
      const int qn = q + (NS - 1) * WAVES;
      __builtin_amdgcn_s_waitcnt(0xC07F);
      if (qn < g1) issue(qn, (it + NS - 1) % NS);
    }
    const int after = min(NS - 1, (g1 - 1 - q) / WAVES);
    if constexpr (NS >= 3) {
      if (after >= 2) gv_wait_vm<2 * WG::NPW>();
      else if (after == 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    } else {
      if (after >= 1) gv_wait_vm<WG::NPW>();
      else gv_wait_vm<0>();
    }
    const int z = q / ngroups, grp = q - z * ngroups;
    const BPart<T, NC>& bp = sm.b[z - z0];
    const int64_t r0 = (int64_t)grp * kWRows;
    const int rows = (int)min((int64_t)kWRows, (int64_t)p.M - r0);
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) acc[j] = 0.f;
    const int cb0 = ch * F::G;
    if (row < rows && cb0 < p.nblk) {
      uint32_t wv[GG::CH_WORDS + 1];
      const int cbyte = row * GG::ROW_BYTES + ch * GG::CH_BYTES;
      const uint32_t* src = &sm.a[w][slot][cbyte / 4];
      if constexpr (GG::CH_BYTES % 4 != 0) {
        const int sh = (cbyte & 3) * 8;
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = __builtin_amdgcn_alignbit(src[c + 1], src[c], sh);
      } else if constexpr (GG::CH_BYTES % 16 == 0) {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS / 4; ++c) {
          const u32x4 x = *(const u32x4*)&src[4 * c];
          wv[4 * c] = x[0]; wv[4 * c + 1] = x[1]; wv[4 * c + 2] = x[2]; wv[4 * c + 3] = x[3];
        }
      } else {
#pragma unroll
        for (int c = 0; c < GG::CH_WORDS; ++c) wv[c] = src[c];
      }
      wv[GG::CH_WORDS] = 0;
      chunk_dot<T, NC, 0>(wv, bp, ch, min(F::G, p.nblk - cb0), ncols, acc);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      float x = acc[j];
      x += __shfl_xor(x, 8);
      x += __shfl_xor(x, 4);
      x += __shfl_xor(x, 2);
      x += __shfl_xor(x, 1);
      acc[j] = x;
    }
    if (ch == 0 && row < rows) {
      const int i12 = z % p.ne12, i13 = z / p.ne12;
      float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if (j < ncols) Cz[(int64_t)j * p.ldc + r0 + row] = acc[j];
    }
  }
}

// one workgroup per CU when every range stays within two slices; false -> caller falls back
template <int T, int NC, int WAVES, int NS>
bool launch_flat_dma(const GemvArgs& p, hipStream_t s, hipError_t* err) {
  const size_t lds = sizeof(SmemFlat<T, NC, WAVES, NS>);
  if (lds > 160 * 1024) return false;
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int64_t total = (int64_t)ngroups * p.ne12 * p.ne13;
  const int nwg = 256;
  if (total < (int64_t)nwg * WAVES * 2 || total >= (int64_t)1 << 31) return false;   // small calls: the 2-D grid
  if ((total + nwg - 1) / nwg > ngroups) return false;         // a range would span > 2 slices
  set_max_lds((const void*)gemv_flat_dma_kernel<T, NC, WAVES, NS>, (int)lds);
  hipLaunchKernelGGL((gemv_flat_dma_kernel<T, NC, WAVES, NS>), dim3(nwg), dim3(64 * WAVES), lds, s, p);
  *err = hipGetLastError();
  return true;
}

template <int T, int NC, int WAVES>
constexpr bool stream_fits() { return sizeof(SmemStream<T, NC, WAVES>) <= 160 * 1024; }

template <int T, int NC, int WAVES>
hipError_t launch_stream_w(const GemvArgs& p, hipStream_t s, int gx) {
  const size_t lds = sizeof(SmemStream<T, NC, WAVES>);
  set_max_lds((const void*)gemv_stream_kernel<T, NC, WAVES>, (int)lds);
  hipLaunchKernelGGL((gemv_stream_kernel<T, NC, WAVES>), dim3(gx, p.ne12 * p.ne13), dim3(64 * WAVES), lds, s, p);
  return hipGetLastError();
}

template <int T, int NC>
hipError_t launch_stream(const GemvArgs& p, hipStream_t s) {
  const int ngroups = (p.M + kWRows - 1) / kWRows;
  const int slices = p.ne12 * p.ne13;
  // 8-wave workgroups when there is enough work for >= 2 per CU, else 4-wave ones
  constexpr bool fit8 = stream_fits<T, NC, 8>();
  const bool big = fit8 && (int64_t)ngroups * slices >= 2 * 256 * 8 * 2;
  const int waves = big ? 8 : 4;
  const size_t lds = big ? sizeof(SmemStream<T, NC, 8>) : sizeof(SmemStream<T, NC, 4>);
  int per_cu = (int)((160 * 1024) / lds);
  per_cu = per_cu < 1 ? 1 : (per_cu > 4 ? 4 : per_cu);
  // all workgroups resident in ONE round (no tail round): floor, not ceil
  int gx = (256 * per_cu) / slices;
  const int gmax = (ngroups + waves - 1) / waves;
  gx = gx < 1 ? 1 : (gx > gmax ? gmax : gx);
  if constexpr (fit8) {
    if (big) return launch_stream_w<T, NC, 8>(p, s, gx);
  }
  return launch_stream_w<T, NC, 4>(p, s, gx);
}

template <int T, int NC, int V = 0>
hipError_t launch_v(const GemvArgs& p, hipStream_t s) {
  const size_t lds = sizeof(Smem<T, NC>);
  const int grid = (int)((p.M + kRows - 1) / kRows);
  if (grid == 0) return hipSuccess;
  set_max_lds((const void*)gemv_kernel<T, NC, V>, (int)lds);
  hipLaunchKernelGGL((gemv_kernel<T, NC, V>), dim3(grid, p.ne12 * p.ne13), dim3(kThreads), lds, s, p);
  return hipGetLastError();
}

int variant() { return knobs().gemv_variant; }

template <int T, int NC>
hipError_t launch_t(const GemvArgs& p, hipStream_t s) {
  const int v = variant();
  // the 256-element super-block formats decode a whole super-block per lane: with more than
  // one activation column their stream kernel outgrows 256 VGPRs (spills), so only NC == 1
  // (the decode GEMV) streams; wider N takes the LDS-staged segment kernel
  // single-column decode with a group small enough for 8 waves x 2 LDS slots (q4_0, q4_K):
  // the LDS-DMA streaming kernel (+2 %, profiles/r01/ab_gemv.txt); q2_K's decode is heavier
  // per byte and keeps the 16-wave VGPR-landing kernel (DMA -12 %).  LAMM_GEMV_VARIANT=10
  // forces the VGPR-landing stream kernel for A/B
  if constexpr (NC == 1 && T != kQ2_K && sizeof(SmemStreamD<T, NC, 8, 2>) <= 160 * 1024) {
    if (p.nblk <= Geo<T>::SEG_BLK && (v == 0 || v == 12)) {
      hipError_t e;
      // LAMM_GEMV_VARIANT=12: the flattened one-workgroup-per-CU grid (all 256 CUs instead of
      // 231 at 33 slices) -- measured equal (q4_0 -1 %, q4_K +1 %, profiles/r01/ab_gemv.txt):
      // the decode is HBM-bound chip-wide, not per CU, so the 2-D grid stays the default
      if (v == 12 && launch_flat_dma<T, NC, 8, 2>(p, s, &e)) return e;
      return launch_stream_dma<T, NC, 8, 2>(p, s);
    }
  }
  // single-column decode with 2-3 K-segments (e.g. ffn_down K = 11008): the multi-segment
  // DMA streaming kernel (8 waves x 2 slots + 3 staged activation segments <= 160 KiB);
  // LAMM_GEMV_VARIANT=13 forces the LDS-staged segment kernel for A/B
  if constexpr (NC == 1 && T != kQ2_K && sizeof(SmemSegD<T, NC, 8, 2, 3>) <= 160 * 1024) {
    const int nseg = (p.nblk + Geo<T>::SEG_BLK - 1) / Geo<T>::SEG_BLK;
    if (nseg > 1 && nseg <= 3 && v == 0) return launch_seg_dma<T, NC, 8, 2, 3>(p, s);
  }
  if constexpr (stream_fits<T, NC, 4>() && (Fmt<T>::VQK != 256 || NC == 1)) {
    if (p.nblk <= Geo<T>::SEG_BLK && (v == 0 || v == 10)) return launch_stream<T, NC>(p, s);
  }
  if constexpr (T == kQ4_0 && NC == 1) {
    if (v == 8) return launch_stream_dma<T, NC, 4, 4>(p, s);   // A/B: LDS-DMA streaming, 4 waves x 4 slots
#ifdef LAMM_AB_VARIANTS
    switch (v) {   // variant build only
      case 1: return launch_v<T, NC, 1>(p, s);
      case 2: return launch_v<T, NC, 2>(p, s);
      case 3: return launch_v<T, NC, 3>(p, s);
      case 4: return launch_v<T, NC, 4>(p, s);   // ablation: no compute (timing only)
      case 5: return launch_v<T, NC, 5>(p, s);   // ablation: no B staging (timing only)
      default: break;
    }
#endif
  }
  return launch_v<T, NC, 0>(p, s);
}

template <int T>
hipError_t launch_nc(const GemvArgs& p, hipStream_t s) {
  if (p.N <= 1) return launch_t<T, 1>(p, s);
  if (p.N <= 2) return launch_t<T, 2>(p, s);
  if (p.N <= 4) return launch_t<T, 4>(p, s);
  return launch_t<T, 8>(p, s);
}

}  // namespace

size_t gemv_lds_bytes(int type, int nc) {
#define LDS_CASE(T)                                                            \
  case T:                                                                      \
    return nc <= 1 ? sizeof(Smem<T, 1>) : nc <= 2 ? sizeof(Smem<T, 2>)         \
         : nc <= 4 ? sizeof(Smem<T, 4>) : sizeof(Smem<T, 8>);
  switch (type) {
    LDS_CASE(kQ4_0) LDS_CASE(kQ4_1) LDS_CASE(kQ5_0) LDS_CASE(kQ5_1)
    LDS_CASE(kQ8_0) LDS_CASE(kQ2_K) LDS_CASE(kQ4_K) LDS_CASE(kQ5_K) LDS_CASE(kQ6_K) LDS_CASE(kF32) LDS_CASE(kF16)
    default: return 0;
  }
#undef LDS_CASE
}

// Row-per-wave kernel (lamm_gemv_rpw.hip) for the 32-element formats at N <= 2 on launches of
// up to 32768 rows (one decode projection; a 4-slice batch of them): the wave-group kernels
// below leave half the chip idle on one 4096-row slice (1024 four-row groups) and only pay off
// once several slices share a launch.  hipGraph-replayed single calls, q4_0 (tools/
// ab_gemv_single.py, profiles/r02/ab_gemv_single.json): 4096x4096 6.03 -> 4.67 us, 11008x4096
// 8.81 -> 7.78, 4096x11008 11.34 -> 8.25; 33 stacked slices stay on the wave-group kernel
// (52 vs 75 us).  Workgroup size: for K > 4096 8 waves (16 with F32 activations); otherwise 16 up
// to 12288 rows per launch (4096 with F32 activations, which every workgroup quantizes once), 8
// beyond.
// LAMM_GEMV_RPW=0 off, =4/8/16 forces.
int rpw_waves(const GemvArgs& p) {
  if (knobs().gemv_rpw >= 0) return knobs().gemv_rpw;
  const int64_t rows = (int64_t)p.M * p.ne12 * p.ne13;
  if (rows > 32768) return 0;
  // K > 4096: 8 waves; F32 rows 16, so two lanes per block stage the row in one pass
  // (4096 x 11008 F32 9.8 -> 8.7 us, profiles/r02/ab_gemv_f32_staging.txt)
  if (p.nblk > 128) return p.b_f32 ? 16 : 8;
  // fewer rows than one per wave of 256 sixteen-wave workgroups (a row slab of a sharded
  // weight, bench.py --gpus N): smaller workgroups spread the rows over more CUs
  if (rows < 4096) return rows >= 2048 ? 8 : 4;
  // 8 waves: with the slim prologue (round 3) the 512-workgroup grid beats 256 x 16 waves on
  // config 2 (probe clones R8 3.74-3.89 vs R16 3.99-4.07 us, profiles/r03/gemv_probe_*.json)
  return 8;
}

hipError_t launch_gemv(int type, const GemvArgs& p, hipStream_t s) {
  // q2_K / q4_K / q5_K single columns: the row-per-wave kernel (LAMM_GEMV_RPW=0 or a
  // LAMM_GEMV_VARIANT keep the wave-group ones)
  if (gemv_kq_supported(type, p) && knobs().gemv_variant == 0 && knobs().gemv_rpw != 0)
    return launch_gemv_kq(type, p, s);
  if (gemv_rpw_supported(type, p)) {
    const int w = rpw_waves(p);
    if (w > 0) return launch_gemv_rpw(type, p, s, w);
  }
  switch (type) {
    case kQ4_0: return launch_nc<kQ4_0>(p, s);
    case kQ4_1: return launch_nc<kQ4_1>(p, s);
    case kQ5_0: return launch_nc<kQ5_0>(p, s);
    case kQ5_1: return launch_nc<kQ5_1>(p, s);
    case kQ8_0: return launch_nc<kQ8_0>(p, s);
    case kQ2_K: return launch_nc<kQ2_K>(p, s);
    case kQ4_K: return launch_nc<kQ4_K>(p, s);
    case kQ5_K: return launch_nc<kQ5_K>(p, s);
    case kQ6_K: return launch_nc<kQ6_K>(p, s);
    // unquantized rows stream through lamm_gemv_dense.hip (LAMM_GEMV_VARIANT=7: this file's
    // segmented kernel, kept for A/B)
    case kF32:  return variant() == 7 ? launch_nc<kF32>(p, s) : launch_gemv_dense(kF32, p, s);
    case kF16:  return variant() == 7 ? launch_nc<kF16>(p, s) : launch_gemv_dense(kF16, p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
