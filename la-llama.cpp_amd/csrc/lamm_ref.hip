// lamm_ref.hip -- mul_mat in the reference's own x86 float order, bit for bit.
//
// The reference's CPU path (the lamm opt-3 AVX2 kernels, src/lamm_kernel_q*.hpp
// lamm_simd_block_kernel with src/lamm_simd_avx2.h; for q6_K, which lamm declines, ggml's AVX2
// ggml_vec_dot_q6_K_q8_K, LC/ggml-quants.c:8305-8385) computes every output with EIGHT fp32
// accumulators -- the lanes of one __m256 -- and per block (super-block for q6_K):
//     acc_l = fma(d, (float)X_l, acc_l),   l = 0..7
// with d = fp32(d_a) * fp32(d_b) rounded once and X_l the exact int32 sum of what lands in lane l:
//     q4_0 / q4_1 / q5_0 / q5_1 : elements 4l .. 4l+3 of the 32-element block
//                                 (mul_sum_i8_pairs_float / mul_sum_us8_pairs_float)
//     q6_K                      : positions 4l .. 4l+3 of each of the 8 32-element groups h,
//                                 times the group half's int8 scale sc[2h + (l >= 4)]
// then the fixed tree ((a0+a4) + (a2+a6)) + ((a1+a5) + (a3+a7)) (reduce_sum / hsum_float_8);
// q4_1 / q5_1 add the separate fp32 sum of fp32(m_a) * fp32(s_b) after it.  oracle/lamm_oracle.c
// lo_vec_dot_avx restates this and is pinned bit-exact to the reference's own lamm3 output
// (tests/test_oracle_golden.py::test_avx_order_matches_lamm3_bit_exact).
//
// The ggml boundary runs its calls here by default (LAMM_HIP_ORDER=reference), so
// llama.cpp through the boundary computes the same bits as the reference's CPU build; the device
// API keeps the fast engines (lamm_hip_matmul) and offers this order as lamm_hip_matmul_ex(...,
// LAMM_ORDER_REFERENCE, ...).
//
// Roundings that must stay separate (d = d_a * d_b before the chain's fma) sit behind an empty
// NON-volatile asm: it hides the value from contraction, and unlike a volatile one it does not
// order every memory access around it (which serialised the MFMA kernels' LDS reads behind the
// previous block's FMAs).
//
// Layout: a workgroup owns 16 / 32 rows x NCOL columns (1, 2, 4 or 8 by N); thread (row r, lane l)
// runs the NCOL column chains of lane l for row r (the A quads it decodes are shared by the columns).
// Per chunk of K both operands come through LDS: the rows' raw block bytes by coalesced 16-byte
// loads (the 2-byte aligned blocks read back with a realignment), the activation columns as quads
// laid out [column][lane][unit].  The quants are turned into signed bytes (q - 8,
// q - 16, q - 32) so each X_l is one v_dot4 -- integer, exact, any order.
#include <hip/hip_ext.h>

#include "lamm_aql.h"
#include "lamm_device.h"
#include "lamm_kernels.h"
#include "lamm_rowdot.h"
#include "lamm_knobs.h"

namespace lamm {
namespace {

constexpr int RR = 32;           // rows per workgroup (16 for decode calls: launch_ref)

template <int T> struct RefFmt;
// BPB: A block bytes; QS / QH / M: byte offsets of the quants, the 5th bits, m (-1: none);
// OFF: the signed-byte offset of the quants (their unsigned maximum + 1, halved); UE: elements per unit;
// D / DM: byte offsets of the (super-)block's d and dmin (-1: none)
template <> struct RefFmt<kQ4_0> { static constexpr int BPB = 18, QS = 2, QH = -1, M = -1, OFF = 8, UE = 32, VB = 34, D = 0, DM = -1; };
template <> struct RefFmt<kQ4_1> { static constexpr int BPB = 20, QS = 4, QH = -1, M = 2, OFF = 0, UE = 32, VB = 36, D = 0, DM = -1; };
template <> struct RefFmt<kQ5_0> { static constexpr int BPB = 22, QS = 6, QH = 2, M = -1, OFF = 16, UE = 32, VB = 34, D = 0, DM = -1; };
template <> struct RefFmt<kQ5_1> { static constexpr int BPB = 24, QS = 8, QH = 4, M = 2, OFF = 0, UE = 32, VB = 36, D = 0, DM = -1; };
template <> struct RefFmt<kQ6_K> { static constexpr int BPB = 210, QS = 0, QH = 128, M = -1, OFF = 32, UE = 256, VB = 292, D = 208, DM = -1; };
// the super-block formats with mins (round 6): q2_K in lamm's AVX2 block kernel's order
// (src/lamm_kernel_q2_k.hpp:163-307), q4_K / q5_K in ggml's AVX2 vec_dot's (LC/ggml-quants.c:7082-7145,
// :7696-7777); their quants are unsigned (0..3 / 0..15 / 0..31), every dot4 stays exact as is
template <> struct RefFmt<kQ2_K> { static constexpr int BPB = 84, QS = 16, QH = -1, M = -1, OFF = 0, UE = 256, VB = 292, D = 80, DM = 82; };
template <> struct RefFmt<kQ4_K> { static constexpr int BPB = 144, QS = 16, QH = -1, M = -1, OFF = 0, UE = 256, VB = 292, D = 0, DM = 2; };
template <> struct RefFmt<kQ5_K> { static constexpr int BPB = 176, QS = 48, QH = 16, M = -1, OFF = 0, UE = 256, VB = 292, D = 0, DM = 2; };

// units of K per LDS chunk, and the dwords of quads one (column, lane, unit) holds
template <int T> constexpr int ref_kch() { return RefFmt<T>::UE == 256 ? 8 : 64; }
template <int T> constexpr int ref_qw() { return RefFmt<T>::UE / 32; }   // groups per lane: 1 or 8

// unsigned quant bytes (0 .. 2 OFF - 1) -> signed (q - OFF), bytewise: flip the top bit of the
// field, then copy it into the bits above (the multiply stays inside each byte)
template <int OFF>
__device__ __forceinline__ uint32_t to_signed(uint32_t q) {
  if constexpr (OFF == 0) {
    return q;
  } else {
    constexpr uint32_t top = (uint32_t)OFF * 0x01010101u;                  // the field's top bit per byte
    constexpr uint32_t ext = (uint32_t)(0x100 - 2 * OFF) / (uint32_t)OFF;   // top bit * ext = the bits above it
    const uint32_t t = q ^ top;
    return t | ((t & top) * ext);
  }
}

// one dword at a 2-byte aligned byte offset of an LDS row image
__device__ __forceinline__ uint32_t lds32(const uint32_t* row, int byte) {
  const int i = byte >> 2;
  return __builtin_amdgcn_alignbit(row[i + 1], row[i], (byte & 3) * 8);
}

template <int T, int RR, int NCOL, bool ONE_SLICE>
__global__ __launch_bounds__(RR * 8) void ref_kernel(GemvArgs p) {
  using F = RefFmt<T>;
  constexpr int NT = RR * 8;
  constexpr int KCH = ref_kch<T>(), QW = ref_qw<T>();
  constexpr int U = QW == 1 ? 4 : 1;                 // units per batch of LDS reads
  constexpr bool AFF = F::M >= 0;
  constexpr bool KQ = F::UE == 256;
  // mins terms: q2_K a second fma per super-block on the lane chains (Y_l = mins[2l] bsums[2l] +
  // mins[2l+1] bsums[2l+1]); q4_K a 4-lane fma chain of prod_q = mn[2q] q8s[2q] + mn[2q+1] q8s[2q+1]
  // (q8s = pairwise sums of the bsums) reduced (m0 + m2) + (m1 + m3); q5_K one scalar sum of dmin * the
  // four prods' int sum, product and sum rounded separately -- each added after the lane tree
  constexpr bool K2 = T == kQ2_K, K45 = T == kQ4_K || T == kQ5_K, MINS = K2 || K45;
  constexpr int SEG = KCH * F::BPB;                  // bytes of a row's chunk (a multiple of 16)
  constexpr int SEGW = SEG / 4 + 1;                  // dwords per LDS row (+1: realignment reads)
  static_assert(SEG % 16 == 0, "chunks start 16-byte aligned");
  __shared__ __attribute__((aligned(16))) uint32_t sa[RR * SEGW];               // A rows, raw bytes
  __shared__ __attribute__((aligned(16))) uint32_t sq[NCOL * 8 * KCH * QW];   // [col][lane][unit][group]
  __shared__ __attribute__((aligned(16))) float sd[NCOL * KCH];               // d_b     [col][unit]
  __shared__ __attribute__((aligned(16))) float ss[AFF ? NCOL * KCH : 1];     // s_b (q8_1)
  __shared__ __attribute__((aligned(16))) uint32_t sbs[MINS ? NCOL * KCH * 8 : 1];   // q8_K bsums [col][unit]

  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if constexpr (!ONE_SLICE) {
    const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  const int t = threadIdx.x, l = t & 7, rloc = t >> 3;
  const int row0 = blockIdx.x * RR, row = row0 + rloc;
  const int nrows = p.M - row0 < RR ? p.M - row0 : RR;
  const int n0 = blockIdx.y * NCOL;
  const int ncols = p.N - n0 < NCOL ? p.N - n0 : NCOL;
  const int nunits = p.nblk;
  // A: the workgroup's rows, from its first row to its last row's last byte (wave-uniform base)
  const auto ra = make_rsrc(Az + (int64_t)row0 * p.lda,
                            (uint32_t)(((int64_t)(nrows - 1) * p.lda + (int64_t)nunits * F::BPB + 3) & ~int64_t(3)));
  const int64_t bbytes = (int64_t)(ncols - 1) * p.ldb + (int64_t)nunits * F::VB;
  const auto rb = make_rsrc(Bz + (int64_t)n0 * p.ldb, (uint32_t)((bbytes + 3) & ~int64_t(3)));

  // the reference's lane l of each column's __m256 accumulator: one fp32 chain per column here
  // (the 8 lanes of a row sit in 8 threads)
  float chain[NCOL], summs[AFF || K45 ? NCOL : 1];   // K45: the mins' chain (q4_K lanes 0-3, q5_K lane 0)
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    chain[c] = 0.f;
    if constexpr (AFF || K45) summs[c] = 0.f;
  }
  const uint32_t* arow = &sa[rloc * SEGW];

  for (int u0 = 0; u0 < nunits; u0 += KCH) {
    const int nu = nunits - u0 < KCH ? nunits - u0 : KCH;
    // ---- stage the A chunk: each row's bytes [u0 BPB, (u0 + KCH) BPB) as coalesced 16-byte loads
    for (int it = t; it < RR * (SEG / 16); it += NT) {
      const int r = it / (SEG / 16), o = it % (SEG / 16);
      const uint32_t off = r < nrows ? (uint32_t)((int64_t)r * p.lda + (int64_t)u0 * F::BPB) + 16 * o : 0x7ffffff0u;
      const u32x4 v = bload16(ra, off);   // past the rows / the row's end: zeros (never summed)
      uint32_t* dst = &sa[r * SEGW + 4 * o];
      dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
    }
    // ---- stage the activation chunk: columns n0 .. n0 + NCOL, units u0 .. u0 + nu
    if constexpr (!KQ) {
      for (int it = t; it < NCOL * KCH; it += NT) {
        const int c = it / KCH, k = it % KCH;
        const bool ok = c < ncols && k < nu;
        const uint32_t off = (uint32_t)((int64_t)c * p.ldb + (int64_t)(u0 + k) * F::VB);
        uint32_t w[10];
        const uint32_t base = ok ? (off & ~3u) : 0x7ffffff0u;
#pragma unroll
        for (int i = 0; i < 10; ++i) w[i] = bload4(rb, base + 4 * i);
        const int sh = (int)(off & 3u) * 8;
        uint32_t m[9];
#pragma unroll
        for (int i = 0; i < 9; ++i) m[i] = __builtin_amdgcn_alignbit(w[i + 1], w[i], sh);
#pragma unroll
        for (int q = 0; q < 8; ++q) {   // quad q = quants 4q .. 4q+3 (q8_0: from byte 2; q8_1: d, s, then byte 4)
          const uint32_t v = AFF ? m[1 + q] : __builtin_amdgcn_alignbit(m[q + 1], m[q], 16);
          sq[((c * 8 + q) * KCH + k) * QW] = ok ? v : 0u;
        }
        sd[c * KCH + k] = ok ? h2f(m[0] & 0xffffu) : 0.f;
        if constexpr (AFF) ss[c * KCH + k] = ok ? h2f(m[0] >> 16) : 0.f;
      }
    } else {
      // q8_K super-block: float d, 256 quants, bsums; 4 threads per (column, unit), 16 quads each
      for (int it = t; it < NCOL * KCH * 4; it += NT) {
        const int item = it >> 2, part = it & 3, c = item / KCH, k = item % KCH;
        const bool ok = c < ncols && k < nu;
        const uint32_t base = ok ? (uint32_t)((int64_t)c * p.ldb + (int64_t)(u0 + k) * F::VB) : 0x7ffffff0u;
#pragma unroll
        for (int i = 0; i < 4; ++i) {   // past the range (base 0x7ffffff0): zeros
          const u32x4 v = bload16(rb, base + 4 + 64 * part + 16 * i);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const int qd = 16 * part + 4 * i + e, h = qd >> 3, ln = qd & 7;   // position 4 qd = 32 h + 4 ln
            sq[((c * 8 + ln) * KCH + k) * QW + h] = v[e];
          }
        }
        if (part == 0) sd[c * KCH + k] = ok ? __builtin_bit_cast(float, bload4(rb, base)) : 0.f;
        if (MINS && part == 1) {   // the 16 int16 bsums (bytes 260 .. 291) as 8 dwords
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            const u32x4 v = bload16(rb, ok ? base + 260 + 16 * i : 0x7ffffff0u);
#pragma unroll
            for (int e = 0; e < 4; ++e) sbs[(c * KCH + k) * 8 + 4 * i + e] = v[e];
          }
        }
      }
    }
    __syncthreads();
    // ---- the chains: units u0 .. u0 + nu, this thread's lane l, its row, every column
    if (row < p.M) {
      for (int k0 = 0; k0 < nu; k0 += U) {
        uint32_t aq[U][QW];
        int sc[U][QW];
        float da[U], ma[U], dm[U];
        int mn[U][K45 ? 8 : 2];   // q2_K: this lane's two min nibbles; q4_K / q5_K: the 8 mins
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int ub = (k0 + u) * F::BPB;   // this unit's bytes in the row's LDS image
          da[u] = h2f(lds32(arow, ub + F::D) & 0xffffu);
          ma[u] = AFF ? h2f(lds32(arow, ub + (AFF ? F::M : 0)) & 0xffffu) : 0.f;
          dm[u] = MINS ? h2f(lds32(arow, ub + (MINS ? F::DM : 0)) & 0xffffu) : 0.f;
          if constexpr (K2) {
            // group h = elements 32 h ..: quants (qs[32 (h / 4) + e] >> 2 (h % 4)) & 3, scale nibble
            // sc[2 h + (e >= 16)] (lane l: e = 4 l .. 4 l + 3)
            const uint32_t s4[4] = {lds32(arow, ub), lds32(arow, ub + 4), lds32(arow, ub + 8), lds32(arow, ub + 12)};
#pragma unroll
            for (int h = 0; h < 8; ++h) {
              const uint32_t w = lds32(arow, ub + F::QS + 32 * (h >> 2) + 4 * l);
              static_assert(F::QH < 0 && F::OFF == 0, "q2_K: two-bit unsigned quants, no high bits");
              aq[u][h] = to_signed<F::OFF>((w >> (2 * (h & 3))) & 0x03030303u);
              const int si = 2 * h + (l < 4 ? 0 : 1);
              sc[u][h] = (int)((s4[si >> 2] >> (8 * (si & 3))) & 0xfu);
            }
            const uint32_t mw = (s4[l >> 1] >> (16 * (l & 1))) & 0xffffu;   // bytes 2l, 2l + 1
            mn[u][0] = (int)((mw >> 4) & 0xfu);
            mn[u][1] = (int)((mw >> 12) & 0xfu);
          } else if constexpr (K45) {
            // ggml's utmp unpacking of the 12 scale bytes (LC/ggml-quants.c:7093-7098): 8 six-bit scales
            // and mins; group h = elements 32 h ..: nibble (h odd: high) of qs[32 (h / 2) + e] (+ 16 x
            // bit h of qh[e] for q5_K)
            uint32_t u0 = lds32(arow, ub + 4), u1 = lds32(arow, ub + 8), u2 = lds32(arow, ub + 12), u3;
            u3 = ((u2 >> 4) & 0x0f0f0f0fu) | (((u1 >> 6) & 0x03030303u) << 4);
            const uint32_t uaux = u1 & 0x3f3f3f3fu;
            u1 = (u2 & 0x0f0f0f0fu) | (((u0 >> 6) & 0x03030303u) << 4);
            u2 = uaux;
            u0 &= 0x3f3f3f3fu;
            const uint32_t qh = F::QH >= 0 ? lds32(arow, ub + (F::QH >= 0 ? F::QH : 0) + 4 * l) : 0u;
#pragma unroll
            for (int h = 0; h < 8; ++h) {
              const uint32_t w = lds32(arow, ub + F::QS + 32 * (h >> 1) + 4 * l);
              uint32_t q = ((h & 1) ? w >> 4 : w) & 0x0f0f0f0fu;
              if constexpr (F::QH >= 0) q |= ((qh >> h) & 0x01010101u) << 4;
              aq[u][h] = to_signed<F::OFF>(q);
              sc[u][h] = (int)((((h < 4) ? u0 : u1) >> (8 * (h & 3))) & 0xffu);
              mn[u][h] = (int)((((h < 4) ? u2 : u3) >> (8 * (h & 3))) & 0xffu);
            }
          } else if constexpr (!KQ) {
            const uint32_t qw = lds32(arow, ub + F::QS + 4 * (l & 3));
            uint32_t q = l < 4 ? qw & 0x0f0f0f0fu : (qw >> 4) & 0x0f0f0f0fu;
            if constexpr (F::QH >= 0) {
              const uint32_t qh = lds32(arow, ub + (F::QH >= 0 ? F::QH : 0));
              q |= spread4_hi((qh >> (4 * l)) & 0xfu);
            }
            aq[u][0] = to_signed<F::OFF>(q);
            sc[u][0] = 1;
          } else {
            const uint32_t sc0 = lds32(arow, ub + 192), sc1 = lds32(arow, ub + 196);
            const uint32_t sc2 = lds32(arow, ub + 200), sc3 = lds32(arow, ub + 204);
            const uint32_t scw[4] = {sc0, sc1, sc2, sc3};
#pragma unroll
            for (int h = 0; h < 8; ++h) {   // group h = 4 j + g: ql[64 j + 32 (g & 1) + 4 l], qh[32 j + 4 l] >> 2 g
              const int j = h >> 2, g = h & 3;
              const uint32_t ql = lds32(arow, ub + F::QS + 64 * j + 32 * (g & 1) + 4 * l);
              const uint32_t qh = lds32(arow, ub + F::QH + 32 * j + 4 * l);
              const uint32_t q = ((g < 2 ? ql : ql >> 4) & 0x0f0f0f0fu) | (((qh >> (2 * g)) & 0x03030303u) << 4);
              aq[u][h] = to_signed<F::OFF>(q);
              const int si = 2 * h + (l < 4 ? 0 : 1);   // scale byte 2h + (l >= 4)
              sc[u][h] = (int)(int8_t)((scw[si >> 2] >> (8 * (si & 3))) & 0xffu);
            }
          }
        }
#pragma unroll
        for (int c = 0; c < NCOL; ++c) {
          uint32_t bq[U][QW];
          float db[U], sb[U];
          int ym[U];   // q2_K: Y_l; q4_K: prod_l (lanes 0-3); q5_K: the four prods' sum
#pragma unroll
          for (int u = 0; u < U; ++u) {
#pragma unroll
            for (int h = 0; h < QW; ++h) bq[u][h] = sq[((c * 8 + l) * KCH + k0 + u) * QW + h];
            db[u] = sd[c * KCH + k0 + u];
            sb[u] = AFF ? ss[c * KCH + k0 + u] : 0.f;
            ym[u] = 0;
            if constexpr (MINS) {
              const uint32_t* bs = &sbs[(c * KCH + k0 + u) * 8];
              auto lo16 = [](uint32_t x) { return (int)(int16_t)(x & 0xffffu); };
              auto hi16 = [](uint32_t x) { return (int)(int16_t)(x >> 16); };
              if constexpr (K2) {   // madd_epi16(mins, bsums), lane l: bsums 2l, 2l + 1
                const uint32_t w = bs[l];
                ym[u] = mn[u][0] * lo16(w) + mn[u][1] * hi16(w);
              } else {   // prod_q = mn[2q] (bs[4q] + bs[4q+1]) + mn[2q+1] (bs[4q+2] + bs[4q+3])
                auto prod = [&](int q) {
                  const uint32_t w0 = bs[2 * q], w1 = bs[2 * q + 1];
                  return mn[u][2 * q] * (int)(int16_t)(lo16(w0) + hi16(w0)) +
                         mn[u][2 * q + 1] * (int)(int16_t)(lo16(w1) + hi16(w1));
                };
                if constexpr (T == kQ4_K) ym[u] = l < 4 ? prod(l & 3) : 0;
                else ym[u] = (prod(0) + prod(1)) + (prod(2) + prod(3));
              }
            }
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            if (k0 + u >= nu) break;   // (uniform)
            int X = 0;
#pragma unroll
            for (int h = 0; h < QW; ++h) {
              const int d4 = dot4(aq[u][h], bq[u][h], 0);
              X = KQ ? X + sc[u][h] * d4 : d4;
            }
            // d = fp32(d_a) * fp32(d_b) rounded once (q6_K: y.d * fp32(x.d)), then one fused step
            float d = KQ ? db[u] * da[u] : da[u] * db[u];
            asm("" : "+v"(d));   // a separate rounding of the product: never contracted into the fma
            chain[c] = __builtin_fmaf(d, (float)X, chain[c]);
            if constexpr (AFF) {
              float pm = ma[u] * sb[u];
              asm("" : "+v"(pm));
              summs[c] = summs[c] + pm;
            }
            if constexpr (K2) {   // lamm: acc = fma(-fp32(dmin_a) * d_b, prod, acc) after the d term
              float d2 = -dm[u] * db[u];
              asm("" : "+v"(d2));
              chain[c] = __builtin_fmaf(d2, (float)ym[u], chain[c]);
            }
            if constexpr (K45) {   // ggml: dmin = -y.d * fp32(x.dmin)
              float d2 = -db[u] * dm[u];
              asm("" : "+v"(d2));
              if constexpr (T == kQ4_K) {
                if (l < 4) summs[c] = __builtin_fmaf(d2, (float)ym[u], summs[c]);
              } else if (l == 0) {
                float pm = d2 * (float)ym[u];
                asm("" : "+v"(pm));
                summs[c] = summs[c] + pm;
              }
            }
          }
        }
      }
    }
    __syncthreads();
  }
  // ---- the tree over the row's 8 lanes: ((a0 + a4) + (a2 + a6)) + ((a1 + a5) + (a3 + a7))
#pragma unroll
  for (int c = 0; c < NCOL; ++c) {
    float v = chain[c];
    {
#pragma clang fp contract(off)
      v = v + __shfl_down(v, 4, 8);   // lanes 0..3: a_l + a_{l+4}
      v = v + __shfl_down(v, 2, 8);   // lanes 0, 1: x_l + x_{l+2}
      v = v + __shfl_down(v, 1, 8);   // lane 0: (x0 + x2) + (x1 + x3)
      if constexpr (AFF) v = v + summs[c];
      if constexpr (T == kQ4_K) {   // the mins' 4-lane chain: (m0 + m2) + (m1 + m3)
        float m = summs[c] + __shfl_down(summs[c], 2, 8);
        m = m + __shfl_down(m, 1, 8);
        v = v + m;
      }
      if constexpr (T == kQ5_K) v = v + summs[c];
    }
    if (l == 0 && row < p.M && c < ncols) Cz[(int64_t)(n0 + c) * p.ldc + row] = v;
  }
}

// ---------------------------------------------------------------- decode: producers and chains
// A one-column call has only 8 chains per weight row -- 32768 for a 4096-row GEMV, half a wave
// per SIMD -- so ref_kernel (each chain thread also decoding its own quads) ran one long
// dependent stream per thread: 28 us per 4096 x 4096 call in llama.cpp's decode (rocprofv3,
// profiles/r04/ref_order/).  Here the chains only do the part that must be sequential:
//   producers  all 256 threads of the workgroup: 4 consecutive blocks of one of its 8 rows per
//              thread (one wide load of 4 BPB bytes), each block's 8 exact lane sums X_l and
//              d = fp32(d_a) * fp32(d_b) (and m_a * s_b) into LDS, a chunk of GKC blocks at a time;
//   chains     wave 0, lane (row, l): acc_l = fma(d, X_l, acc_l) over the chunk (b128 LDS reads),
//              then reduce_sum's tree across the row's 8 lanes.
// The activation column is staged once per workgroup (ActStage; F32 rows quantized there, ggml's
// AVX2 from_float bit for bit -- the boundary's fused INIT).  The chunk's A loads for the next
// chunk are in flight while the chains run.
// GKC: blocks per chunk of a single-weight launch with K > 4096 (each workgroup's long chain then
// runs over fewer, longer chunks); everything else takes chunks of GKC_S = 64 -- 256-thread
// workgroups of a third of the LDS, so a grouped launch keeps ~2x the workgroups resident
// (tools/ref_group_ab.py, profiles/r05/ref_gemv_occupancy/: q|k|v 9.1 -> 7.7 us, gate|up 16.4 -> 14.0,
// wo 4.45 -> 4.33; down 8.6 at 128 vs 9.1 at 64)
#ifndef REF_GKC_S
#define REF_GKC_S 64   // probe builds: the short chunk (a multiple of 4 and of 2 x blocks per producer)
#endif
constexpr int GR = 8, GKC = 128, GKC_S = REF_GKC_S;   // rows, blocks per chunk (the LDS pitch is the chunk + 4)

// dword at byte O of a register byte string, zero past its end (the last block's slack bytes)
template <int O, int NW>
__device__ __forceinline__ uint32_t get32z(const uint32_t (&w)[NW]) {
  if constexpr ((O >> 2) >= NW) return 0u;
  else if constexpr ((O & 3) == 0) return w[O >> 2];
  else if constexpr ((O >> 2) + 1 < NW) return __builtin_amdgcn_alignbit(w[(O >> 2) + 1], w[O >> 2], (O & 3) * 8);
  else return w[O >> 2] >> ((O & 3) * 8);
}

#ifndef REF_NEG_LDS
// probe builds: the q4_0 / q5_0 offset dots once per block in the staging instead of per row --
// measured SLOWER (q|k|v 7.8 -> 9.2 us, wo 4.3 -> 4.7; the extra barrier and LDS reads cost more than
// the 8 dot4 per block and row: the kernel is not VALU-bound, profiles/r05/ref_gemv_occupancy/)
#define REF_NEG_LDS 0
#endif
size_t ref_gemv_lds(int type, int nblk, int ck = GKC, int rg = GR) {
  const bool aff = type == kQ4_1 || type == kQ5_1;
  const size_t neg = REF_NEG_LDS && (type == kQ4_0 || type == kQ5_0) ? (size_t)nblk * 32 : 0;
  return (((size_t)nblk * 40 + 15) & ~size_t(15)) + sizeof(float) * (ck + 4) * (rg * 8 + rg + (aff ? rg : 0)) + neg;
}
#ifndef REF_GROUP_RG
#define REF_GROUP_RG 8   // rows per workgroup of the grouped launch (probe builds: 16)
#endif

#ifndef REF_GAB
// probe builds only (ablations of ref_gemv_kernel): 1 no chains, 2 no producer arithmetic,
// 3 no activation staging
#define REF_GAB 0
#endif
// MODE 0: one slice; 1: ggml's batch slices over blockIdx.z; 2: blockIdx.z picks one of up to
// kRefSegs weights sharing the activation column (lamm_hip_matmul_group)
template <int T, bool BF32, int MODE, int BPT, int CK, int RG = GR>
__device__ __forceinline__ void ref_gemv_body(const GemvArgs& p, const RefSegs& sg) {
  using F = RFmt<T>;
  constexpr int GKC = CK, GP = CK + 4, GR = RG;   // this instance's chunk and rows (hide the defaults)
  // BPT consecutive blocks of one row per producer thread (one wide load of BPT * BPB bytes, dword
  // aligned: BPB is even); NT threads cover the chunk's GR x GKC blocks.  Config 2 (q4_0 4096 x 4096,
  // F32 row, profiles/r05/ref_gemv/): BPT 2 (512 threads) 5.1-5.4 us, 4 (256) 5.9-6.0, 1 (1024
  // threads, realigned 18-byte loads) 6.4-6.6 -- the producers' arithmetic runs after the one
  // chunk's loads land, so more, shorter producer streams finish it sooner, until the realigning
  // single-block loads cost more than they save
  static_assert(BPT == 2 || BPT == 4, "blocks per producer thread");
  constexpr int NT = GR * GKC / BPT, TPR = GKC / BPT;   // threads, threads per row
  constexpr bool AFF = T == kQ4_1 || T == kQ5_1;
  // -OFF as four int8: sum (q - OFF) b = sum q b + sum (-OFF) b, both exact
  constexpr uint32_t NEG = T == kQ4_0 ? 0xf8f8f8f8u : T == kQ5_0 ? 0xf0f0f0f0u : 0u;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nb = p.nblk;
  u32x4* sq0 = reinterpret_cast<u32x4*>(smem_raw);
  u32x4* sq1 = sq0 + nb;
  float* sbd = reinterpret_cast<float*>(sq1 + nb);
  float* sbs = sbd + nb;
  float* xs = reinterpret_cast<float*>(smem_raw + ((nb * 40 + 15) & ~15));   // [row * 8 + l][GP]
  float* dsm = xs + GR * 8 * GP;                                             // [row][GP]
  float* pms = dsm + GR * GP;                                                // [row][GP] (q4_1 / q5_1)

  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  int Mz = p.M;
  if constexpr (MODE == 1) {
    const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  } else if constexpr (MODE == 2) {   // uniform selects: no dynamic index into the kernargs
    const int z = blockIdx.z;
#pragma unroll
    for (int i = 1; i < kRefSegs; ++i)
      if (z == i) {
        Az = sg.A[i];
        Cz = sg.C[i];
        Mz = sg.M[i];
      }
  }
  const int t = threadIdx.x;
  const int row0 = blockIdx.x * GR;
  if (MODE == 2 && row0 >= Mz) return;   // a shorter weight of the group (whole workgroup)
  const int nrows = Mz - row0 < GR ? Mz - row0 : GR;
  const auto ra = make_rsrc(Az + (int64_t)row0 * p.lda,
                            (uint32_t)(((int64_t)(nrows - 1) * p.lda + (int64_t)nb * F::BPB + 3) & ~int64_t(3)));
  // producer: row pr, blocks BPT pg .. BPT pg + BPT - 1 of each chunk
  const int pr = t / TPR, pg = t % TPR;
  uint32_t w[BPT * F::BPB / 4];   // BPT blocks: BPT BPB bytes
  auto issue = [&](int u0) {
    const int u = u0 + BPT * pg;
    const uint32_t off = pr < nrows && u < nb ? (uint32_t)((int64_t)pr * p.lda + (int64_t)u * F::BPB) : 0x7ffffff0u;
    load_words<BPT * F::BPB / 4, 2>(ra, off, w);   // non-temporal: A is read once
  };
  issue(0);
  // ---- the activation column, once per workgroup
  const auto rb = act_rsrc<T, 1, BF32>(p, Bz);
  if constexpr (REF_GAB == 3) {
  } else if constexpr (BF32) {
    for (int it = t; it < 2 * nb; it += NT) {   // two lanes per block (pairs stay together: NT even)
      ActStageL<T, 2> sl;
      sl.template load<1>(p, rb, it);
      sl.store(it, sq0, sq1, sbd, sbs);
    }
  } else {
    for (int it = t; it < nb; it += NT) {
      ActStage<T, false> st;
      st.template load<1>(p, rb, it);
      st.store(it, sq0, sq1, sbd, sbs);
    }
  }
  __syncthreads();
  // the offset term's 8 lane dots depend on the activation only: once per block, not per row
  u32x4* sng = reinterpret_cast<u32x4*>(pms);   // (q4_0 / q5_0 leave pms unused)
  if constexpr (REF_NEG_LDS && NEG != 0) {
    for (int it = t; it < nb; it += NT) {
      const u32x4 b0 = sq0[it], b1 = sq1[it];
      u32x4 n0, n1;
#pragma unroll
      for (int l = 0; l < 4; ++l) {
        n0[l] = (uint32_t)dot4(b0[l], NEG, 0);
        n1[l] = (uint32_t)dot4(b1[l], NEG, 0);
      }
      sng[2 * it] = n0;
      sng[2 * it + 1] = n1;
    }
    __syncthreads();
  }

  const int cl = t & 7, cr = t >> 3;   // chain lane (wave 0): row cr, lane cl
  float chain = 0.f, summs = 0.f;
  for (int u0 = 0; u0 < nb; u0 += GKC) {
    // ---- producers: 4 blocks of row pr
    typedef float fv __attribute__((ext_vector_type(BPT)));
    if constexpr (REF_GAB == 2) {
      fv xv;
#pragma unroll
      for (int j = 0; j < BPT; ++j) xv[j] = (float)w[j];
#pragma unroll
      for (int l = 0; l < 8; ++l) *reinterpret_cast<fv*>(&xs[(pr * 8 + l) * GP + BPT * pg]) = xv;
      *reinterpret_cast<fv*>(&dsm[pr * GP + BPT * pg]) = xv;
    } else {
      fv xv[8], dv, pv;
      unroll<BPT>([&](auto J) {
        constexpr int j = J;
        const int u = u0 + BPT * pg + j;
        const bool ok = pr < nrows && u < nb;
        uint32_t m[F::BPB / 4 + 1];
        unroll<F::BPB / 4 + 1>([&](auto K) { m[K] = get32z<j * F::BPB + 4 * K>(w); });
        uint32_t q[8];
        float da, ma;
        unpack_a<T>(m, q, da, ma);
        const int ub = ok ? u : 0;
        const u32x4 b0 = sq0[ub], b1 = sq1[ub];
        const uint32_t bq[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        int negc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if constexpr (REF_NEG_LDS && NEG != 0) {
          const u32x4 n0 = sng[2 * ub], n1 = sng[2 * ub + 1];
#pragma unroll
          for (int l = 0; l < 4; ++l) {
            negc[l] = (int)n0[l];
            negc[4 + l] = (int)n1[l];
          }
        }
        float d = da * sbd[ub];
        asm("" : "+v"(d));   // rounded on its own: never contracted into the chain's fma
        // past nb / nrows only d is zeroed: X is a finite integer whatever the (zero or clamped)
        // operands, and fma(0, X, acc) == acc (no chain is ever -0)
#pragma unroll
        for (int l = 0; l < 8; ++l) {
          const int c = REF_NEG_LDS ? negc[l] : NEG ? dot4(bq[l], NEG, 0) : 0;
          xv[l][j] = (float)dot4(q[l], bq[l], c);
        }
        dv[j] = ok ? d : 0.f;
        if constexpr (AFF) {
          float pm = ma * sbs[ub];
          asm("" : "+v"(pm));
          pv[j] = ok ? pm : 0.f;
        }
      });
#pragma unroll
      for (int l = 0; l < 8; ++l) *reinterpret_cast<fv*>(&xs[(pr * 8 + l) * GP + BPT * pg]) = xv[l];
      *reinterpret_cast<fv*>(&dsm[pr * GP + BPT * pg]) = dv;
      if constexpr (AFF) *reinterpret_cast<fv*>(&pms[pr * GP + BPT * pg]) = pv;
    }
    if (u0 + GKC < nb) issue(u0 + GKC);   // the next chunk's A under the chains
    __syncthreads();
    // ---- chains: wave 0, the chunk's blocks in order (zeros past nb leave a chain unchanged:
    // fma(0, 0, acc) == acc, and no chain is ever -0)
    if (t < 8 * GR && REF_GAB != 1) {   // (GR / 8 chain waves)
      // the whole chunk, always: the producers zero-filled it past nb, and a fixed trip count
      // lets the LDS reads run ahead of the chain instead of one wait per 4 blocks
      const float* xr = &xs[(cr * 8 + cl) * GP];
      const float* dr = &dsm[cr * GP];
#pragma unroll 8
      for (int k = 0; k < GKC; k += 4) {
        const f32x4 x4 = *reinterpret_cast<const f32x4*>(&xr[k]);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(&dr[k]);
        chain = __builtin_fmaf(d4[0], x4[0], chain);
        chain = __builtin_fmaf(d4[1], x4[1], chain);
        chain = __builtin_fmaf(d4[2], x4[2], chain);
        chain = __builtin_fmaf(d4[3], x4[3], chain);
        if constexpr (AFF) {
          const f32x4 p4 = *reinterpret_cast<const f32x4*>(&pms[cr * GP + k]);
          summs = summs + p4[0];   // one rounding per block, in block order (no products here)
          summs = summs + p4[1];
          summs = summs + p4[2];
          summs = summs + p4[3];
        }
      }
    }
    __syncthreads();
  }
  if (t < 8 * GR) {
    float v = chain;
    {
#pragma clang fp contract(off)
      v = v + __shfl_down(v, 4, 8);
      v = v + __shfl_down(v, 2, 8);
      v = v + __shfl_down(v, 1, 8);
      if constexpr (AFF) v = v + summs;
    }
    if (cl == 0 && cr < nrows) Cz[row0 + cr] = v;
  }
  if (MODE != 2 && p.flag) signal_done(p);
}

template <int T, bool BF32, bool ONE_SLICE, int BPT = 4, int CK = GKC>
#ifndef REF_GEMV_WPE
#define REF_GEMV_WPE 6   // waves per SIMD the register budget is cut for (probe builds: 5 = unconstrained)
#endif
// 512-thread form (BPT 2): 86 -> <= 80 VGPRs, so three workgroups (24 waves) share a CU instead of
// two -- a grouped launch (lamm_hip_matmul_group, 1536 / 2752 workgroups) runs in fewer rounds.  The
// 256-thread form would spill under the same cut and keeps its budget.
__global__ __launch_bounds__(GR * CK / BPT) __attribute__((amdgpu_waves_per_eu(BPT == 2 ? REF_GEMV_WPE : 1)))
void ref_gemv_kernel(GemvArgs p) {
  ref_gemv_body<T, BF32, ONE_SLICE ? 0 : 1, BPT, CK>(p, RefSegs{});
}

// several weights times one activation column in one launch (segment 0 in p.A / p.C / p.M)
template <int T, bool BF32, int BPT = 4, int CK = GKC_S, int RG = REF_GROUP_RG>
__global__ __launch_bounds__(RG * CK / BPT) __attribute__((amdgpu_waves_per_eu(BPT == 2 ? REF_GEMV_WPE : 1)))
void ref_gemv_group_kernel(GemvArgs p, RefSegs sg) {
  ref_gemv_body<T, BF32, 2, BPT, CK, RG>(p, sg);
}

// ---------------------------------------------------------------- F16 x F16: ggml_vec_dot_f16's order
// The attention mul_mats (KQ over the F16 K cache, KQV over the F16 V cache) in ggml's AVX2
// ggml_vec_dot_f16 order (LC/ggml.c:1589-1629, GGML_F32x8_REDUCE :946-964; oracle
// f16_dot_avx, pinned to the reference's own attention nodes): element i of each 32-element step
// feeds accumulator slot i % 32 (sum[(i % 32) / 8] lane i % 8) through one fp32 fma on the
// F16-widened values (v_fma_mix_f32: the widening is exact, one rounding), then
//     v_e = (s_e + s_{16+e}) + (s_{8+e} + s_{24+e}),  t_e = v_e + v_{e+4},  (t0 + t1) + (t2 + t3)
// and the n % 32 leftovers in double.  Slots are independent chains, so a thread keeps all 32 of
// each of its 2 x 2 outputs (128 accumulators) and the tree runs in registers; 32 x 32 outputs
// per workgroup, K through LDS in steps of 64 halves (16-byte rows when the pitches allow).
constexpr int FT = 32, FKC = 64, FNT = 256, FPITCH = FKC + 8;   // tile, K step, threads, LDS pitch (halves)

// acc = fma(f16 half H of a, f16 half H of b, acc) with one rounding: v_fma_mix_f32 widens its f16
// sources exactly (hipcc widens with separate v_cvt_f32_f16 instead, one per operand)
template <int H>
__device__ __forceinline__ void fma_mix(float& acc, uint32_t a, uint32_t b) {
  if constexpr (H == 0)
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(a), "v"(b));
  else
    asm("v_fma_mix_f32 %0, %1, %2, %0 op_sel:[1,1,0] op_sel_hi:[1,1,0]" : "+v"(acc) : "v"(a), "v"(b));
}

template <bool VEC, bool ONE_SLICE>
__global__ __launch_bounds__(FNT) void ref_f16_kernel(GemvArgs p) {
  __shared__ __attribute__((aligned(16))) _Float16 sa[FT * FPITCH];
  __shared__ __attribute__((aligned(16))) _Float16 sb[FT * FPITCH];
  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if constexpr (!ONE_SLICE) {
    const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  const int t = threadIdx.x, tc = t & 15, tr = t >> 4;
  const int m0 = blockIdx.x * FT, n0 = blockIdx.y * FT;
  const int nrows = p.M - m0 < FT ? p.M - m0 : FT;
  const int ncols = p.N - n0 < FT ? p.N - n0 : FT;
  const int K = p.K, np = K & ~31;
  const auto ra = make_rsrc(Az + (int64_t)m0 * p.lda, (uint32_t)((int64_t)(nrows - 1) * p.lda + 2 * (int64_t)K));
  const auto rb = make_rsrc(Bz + (int64_t)n0 * p.ldb, (uint32_t)((int64_t)(ncols - 1) * p.ldb + 2 * (int64_t)K));

  float acc[2][2][32];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int s = 0; s < 32; ++s) acc[i][j][s] = 0.f;

  // staging: thread t moves 8 halves of row / column t >> 3, elements 8 (t & 7) .. of the step
  const int sr = t >> 3, se = 8 * (t & 7);
  for (int k0 = 0; k0 < np; k0 += FKC) {
    const int k = k0 + se;
    const bool kin = k < np;   // np % 32 == 0: a group of 8 is wholly in or out
    u32x4 va = {0u, 0u, 0u, 0u}, vb = {0u, 0u, 0u, 0u};
    if constexpr (VEC) {
      va = bload16(ra, sr < nrows && kin ? (uint32_t)((int64_t)sr * p.lda + 2 * k) : 0x7ffffff0u);
      vb = bload16(rb, sr < ncols && kin ? (uint32_t)((int64_t)sr * p.ldb + 2 * k) : 0x7ffffff0u);
    } else {
#pragma unroll
      for (int e = 0; e < 8; e += 2) {
        const uint32_t oa = sr < nrows && kin ? (uint32_t)((int64_t)sr * p.lda + 2 * (k + e)) : 0x7ffffff0u;
        const uint32_t ob = sr < ncols && kin ? (uint32_t)((int64_t)sr * p.ldb + 2 * (k + e)) : 0x7ffffff0u;
        va[e / 2] = (uint32_t)bload2(ra, oa) | ((uint32_t)bload2(ra, oa + 2) << 16);
        vb[e / 2] = (uint32_t)bload2(rb, ob) | ((uint32_t)bload2(rb, ob + 2) << 16);
      }
    }
    __syncthreads();   // the previous step's reads are done
    *reinterpret_cast<u32x4*>(&sa[sr * FPITCH + se]) = va;
    *reinterpret_cast<u32x4*>(&sb[sr * FPITCH + se]) = vb;
    __syncthreads();
#pragma unroll
    for (int g = 0; g < FKC / 8; ++g) {
      const int s0 = (8 * g) & 31;
      const u32x4 a0 = *reinterpret_cast<const u32x4*>(&sa[(2 * tr) * FPITCH + 8 * g]);
      const u32x4 a1 = *reinterpret_cast<const u32x4*>(&sa[(2 * tr + 1) * FPITCH + 8 * g]);
      const u32x4 b0 = *reinterpret_cast<const u32x4*>(&sb[(2 * tc) * FPITCH + 8 * g]);
      const u32x4 b1 = *reinterpret_cast<const u32x4*>(&sb[(2 * tc + 1) * FPITCH + 8 * g]);
#pragma unroll
      for (int w = 0; w < 4; ++w) {   // halves 2w (low) and 2w + 1 (high) of the group
        fma_mix<0>(acc[0][0][s0 + 2 * w], a0[w], b0[w]);
        fma_mix<0>(acc[0][1][s0 + 2 * w], a0[w], b1[w]);
        fma_mix<0>(acc[1][0][s0 + 2 * w], a1[w], b0[w]);
        fma_mix<0>(acc[1][1][s0 + 2 * w], a1[w], b1[w]);
        fma_mix<1>(acc[0][0][s0 + 2 * w + 1], a0[w], b0[w]);
        fma_mix<1>(acc[0][1][s0 + 2 * w + 1], a0[w], b1[w]);
        fma_mix<1>(acc[1][0][s0 + 2 * w + 1], a1[w], b0[w]);
        fma_mix<1>(acc[1][1][s0 + 2 * w + 1], a1[w], b1[w]);
      }
    }
  }
  // GGML_F32x8_REDUCE per output, then the leftovers in double
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int m = m0 + 2 * tr + i, n = n0 + 2 * tc + j;
      const float* s = acc[i][j];
      float r;
      {
#pragma clang fp contract(off)
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (s[e] + s[16 + e]) + (s[8 + e] + s[24 + e]);
        const float t0 = v[0] + v[4], t1 = v[1] + v[5], t2 = v[2] + v[6], t3 = v[3] + v[7];
        r = (t0 + t1) + (t2 + t3);
      }
      if (m < p.M && n < p.N) {
        if (np < K) {
          double sumf = (double)r;
          for (int kk = np; kk < K; ++kk) {
            const float x = h2f(bload2(ra, (uint32_t)((int64_t)(2 * tr + i) * p.lda + 2 * kk)));
            const float y = h2f(bload2(rb, (uint32_t)((int64_t)(2 * tc + j) * p.ldb + 2 * kk)));
            float xy = x * y;   // exact (11-bit significands), as the reference's float product
            asm("" : "+v"(xy));
            sumf += (double)xy;
          }
          r = (float)sumf;
        }
        Cz[(int64_t)n * p.ldc + m] = r;
      }
    }
}

// ---------------------------------------------------------------- prefill: the same order on MFMA
// The lane sums X_l come from v_mfma_f32_32x32x16_f16 with a block-diagonal activation operand:
// its 32 rows are (column n, lane l) pairs, row (n, l) carrying b_n's 4 quants of lane l (as f16,
// the rest of its K zero), so C[(n, l)][m] = X_l(m, n) -- 16 integer products, exact in fp32 --
// for the 16 elements of a half block; the other half block is a second MFMA.  Each lane (weight
// row m) then holds all 8 lanes' sums of its 4 columns per n-group, so the reference's
// acc_l = fma(d, X_l, acc_l) chains and the final reduce_sum tree run in registers, with
// d = fp32(d_a) * fp32(d_b) rounded once on the VALU.
//   workgroup: 4 waves = 2 (64 weight rows) x 2 (32 activation columns); a wave: 32 rows (its
//   lanes) x 2 n-groups of 8 columns; K in chunks of 8 blocks through LDS (the rows' raw block
//   bytes; the activation columns converted to f16 once per workgroup)
typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 half2v __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));
constexpr int MR = 64, MC = 32, MKB = 8, MNT = 256;   // rows, columns, blocks per chunk, threads

// four unsigned bytes q (0 .. 255) -> f16 (q - OFF) pairs: {lo dword: q0, q1; hi dword: q2, q3}
template <int OFF>
__device__ __forceinline__ void q4_to_f16(uint32_t q, uint32_t& lo, uint32_t& hi) {
  // f16 bit pattern 0x6400 | q is 1024 + q exactly; subtract 1024 + OFF in f16 (exact: integers)
  const uint32_t a = __builtin_amdgcn_perm(0u, q, 0x0c010c00u) | 0x64006400u;   // bytes 0, 1 -> halves
  const uint32_t b = __builtin_amdgcn_perm(0u, q, 0x0c030c02u) | 0x64006400u;   // bytes 2, 3
  const half2v off = {(_Float16)(-(1024 + OFF)), (_Float16)(-(1024 + OFF))};
  lo = __builtin_bit_cast(uint32_t, __builtin_bit_cast(half2v, a) + off);
  hi = __builtin_bit_cast(uint32_t, __builtin_bit_cast(half2v, b) + off);
}

template <int T, bool ONE_SLICE>
__global__ __launch_bounds__(MNT) void ref_mfma_kernel(GemvArgs p) {
  using F = RefFmt<T>;
  static_assert(F::UE == 32, "32-element block formats");
  constexpr bool AFF = F::M >= 0;
  constexpr int SEG = MKB * F::BPB;                 // a row's chunk bytes
  static_assert(SEG % 16 == 0, "chunks start 16-byte aligned");
  constexpr int SEGW = SEG / 4 + 1;
  constexpr int BP = MKB * 32 + 8;                  // f16 activation row pitch (halves)
  __shared__ __attribute__((aligned(16))) uint32_t sa[MR * SEGW];
  __shared__ __attribute__((aligned(16))) _Float16 sb[MC * BP];
  __shared__ float sdb[MC][MKB];
  __shared__ float ssb[AFF ? MC : 1][MKB];

  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if constexpr (!ONE_SLICE) {
    const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  const int t = threadIdx.x, lane = t & 63, lr = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), wm = w & 1, wn = w >> 1;
  const int m0 = blockIdx.x * MR, n0 = blockIdx.y * MC;
  const int nrows = p.M - m0 < MR ? p.M - m0 : MR;
  const int ncols = p.N - n0 < MC ? p.N - n0 : MC;
  const int nunits = p.nblk;
  const auto ra = make_rsrc(Az + (int64_t)m0 * p.lda,
                            (uint32_t)(((int64_t)(nrows - 1) * p.lda + (int64_t)nunits * F::BPB + 3) & ~int64_t(3)));
  const int64_t bbytes = (int64_t)(ncols - 1) * p.ldb + (int64_t)nunits * F::VB;
  const auto rb = make_rsrc(Bz + (int64_t)n0 * p.ldb, (uint32_t)((bbytes + 3) & ~int64_t(3)));
  const int ml = 32 * wm + lr;                      // this lane's weight row in the tile

  // acc[g][half][r]: n-group g (columns 16 wn + 8 g ..), block half (lanes l = 4 half + (r & 3)),
  // MFMA output element r: column 16 wn + 8 g + 2 (r >> 2) + h, lane 4 half + (r & 3)
  f32x16 acc[2][2];
  float summs[2][4];
#pragma unroll
  for (int g = 0; g < 2; ++g) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[g][q][r] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) summs[g][c] = 0.f;
  }
  const uint32_t* arow = &sa[ml * SEGW];

  for (int u0 = 0; u0 < nunits; u0 += MKB) {
    const int nu = nunits - u0 < MKB ? nunits - u0 : MKB;
    // ---- stage: the rows' raw chunk bytes; the columns' quants as f16, d_b (and s_b)
    for (int it = t; it < MR * (SEG / 16); it += MNT) {
      const int r = it / (SEG / 16), o = it % (SEG / 16);
      const uint32_t off = r < nrows ? (uint32_t)((int64_t)r * p.lda + (int64_t)u0 * F::BPB) + 16 * o : 0x7ffffff0u;
      const u32x4 v = bload16(ra, off);
      uint32_t* dst = &sa[r * SEGW + 4 * o];
      dst[0] = v[0]; dst[1] = v[1]; dst[2] = v[2]; dst[3] = v[3];
    }
    {
      const int c = t >> 3, k = t & 7;              // 256 threads = 32 columns x 8 blocks
      const bool ok = c < ncols && k < nu;
      const uint32_t off = (uint32_t)((int64_t)c * p.ldb + (int64_t)(u0 + k) * F::VB);
      const uint32_t base = ok ? (off & ~3u) : 0x7ffffff0u;
      uint32_t wv[10];
#pragma unroll
      for (int i = 0; i < 10; ++i) wv[i] = bload4(rb, base + 4 * i);
      const int sh = (int)(off & 3u) * 8;
      uint32_t m[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) m[i] = __builtin_amdgcn_alignbit(wv[i + 1], wv[i], sh);
      uint32_t* dst = reinterpret_cast<uint32_t*>(&sb[c * BP + 32 * k]);
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // quad q (signed bytes) -> 4 f16
        const uint32_t qd = AFF ? m[1 + q] : __builtin_amdgcn_alignbit(m[q + 1], m[q], 16);
        uint32_t lo, hi;
        q4_to_f16<128>(qd ^ 0x80808080u, lo, hi);   // int8 b: b + 128 as an unsigned byte, less 128
        dst[2 * q] = ok ? lo : 0u;
        dst[2 * q + 1] = ok ? hi : 0u;
      }
      sdb[c][k] = ok ? h2f(m[0] & 0xffffu) : 0.f;
      if constexpr (AFF) ssb[c][k] = ok ? h2f(m[0] >> 16) : 0.f;
    }
    __syncthreads();
    for (int k = 0; k < nu; ++k) {
      // ---- the weight operand: row ml, elements 8h .. 8h + 7 (half 0) and 16 + 8h .. (half 1)
      const int ub = k * F::BPB;
      const float da = h2f(lds32(arow, ub) & 0xffffu);
      const float ma = AFF ? h2f(lds32(arow, ub + (AFF ? F::M : 0)) & 0xffffu) : 0.f;
      uint32_t q0 = lds32(arow, ub + F::QS + 8 * h), q1 = lds32(arow, ub + F::QS + 8 * h + 4);
      uint32_t wlo[2] = {q0 & 0x0f0f0f0fu, q1 & 0x0f0f0f0fu};            // elements 8h ..
      uint32_t whi[2] = {(q0 >> 4) & 0x0f0f0f0fu, (q1 >> 4) & 0x0f0f0f0fu};   // elements 16 + 8h ..
      if constexpr (F::QH >= 0) {
        const uint32_t qh = lds32(arow, ub + (F::QH >= 0 ? F::QH : 0));
        wlo[0] |= spread4_hi((qh >> (8 * h)) & 0xfu);
        wlo[1] |= spread4_hi((qh >> (8 * h + 4)) & 0xfu);
        whi[0] |= spread4_hi((qh >> (16 + 8 * h)) & 0xfu);
        whi[1] |= spread4_hi((qh >> (16 + 8 * h + 4)) & 0xfu);
      }
      uint32_t wf[2][4];
      q4_to_f16<F::OFF>(wlo[0], wf[0][0], wf[0][1]);
      q4_to_f16<F::OFF>(wlo[1], wf[0][2], wf[0][3]);
      q4_to_f16<F::OFF>(whi[0], wf[1][0], wf[1][1]);
      q4_to_f16<F::OFF>(whi[1], wf[1][2], wf[1][3]);
#pragma unroll
      for (int g = 0; g < 2; ++g) {
        const int nb = 16 * wn + 8 * g;             // the n-group's first column in the tile
        // the block-diagonal activation operand: row lr = (column nb + lr / 4, lane lr % 4 of the
        // half); this lane holds K = 8h .. 8h + 7 of it: that lane's 4 quants when lr % 4 is 2h or
        // 2h + 1, else zeros
        const int nn = nb + (lr >> 2), lq = lr & 3;
        const bool mine = (lq >> 1) == h;
        f32x16 S[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const uint2 v = *reinterpret_cast<const uint2*>(&sb[nn * BP + 32 * k + 16 * q + 4 * lq]);
          uint32_t af[4] = {0u, 0u, 0u, 0u};
          af[2 * (lq & 1)] = mine ? v.x : 0u;
          af[2 * (lq & 1) + 1] = mine ? v.y : 0u;
          const half8 A8 = __builtin_bit_cast(half8, u32x4{af[0], af[1], af[2], af[3]});
          const half8 W8 = __builtin_bit_cast(half8, u32x4{wf[q][0], wf[q][1], wf[q][2], wf[q][3]});
          const f32x16 zero = {};
          S[q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(A8, W8, zero, 0, 0, 0);
        }
        // d per output column: 2 (r >> 2) + h of the group; one fused step per lane sum
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          float d = da * sdb[nb + 2 * c + h][k];
          asm("" : "+v"(d));
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            acc[g][0][4 * c + e] = __builtin_fmaf(d, S[0][4 * c + e], acc[g][0][4 * c + e]);
            acc[g][1][4 * c + e] = __builtin_fmaf(d, S[1][4 * c + e], acc[g][1][4 * c + e]);
          }
          if constexpr (AFF) {
            float pm = ma * ssb[nb + 2 * c + h][k];
            asm("" : "+v"(pm));
            summs[g][c] = summs[g][c] + pm;
          }
        }
      }
    }
    __syncthreads();
  }
  // ---- reduce_sum's tree per output, in registers: lanes l = e (half 0) and 4 + e (half 1)
  const int m = m0 + ml;
#pragma unroll
  for (int g = 0; g < 2; ++g)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int n = 16 * wn + 8 * g + 2 * c + h;
      float v;
      {
#pragma clang fp contract(off)
        const float x0 = acc[g][0][4 * c + 0] + acc[g][1][4 * c + 0], x1 = acc[g][0][4 * c + 1] + acc[g][1][4 * c + 1];
        const float x2 = acc[g][0][4 * c + 2] + acc[g][1][4 * c + 2], x3 = acc[g][0][4 * c + 3] + acc[g][1][4 * c + 3];
        v = (x0 + x2) + (x1 + x3);
        if constexpr (AFF) v = v + summs[g][c];
      }
      if (m < p.M && n < ncols) Cz[(int64_t)(n0 + n) * p.ldc + m] = v;
    }
}

// The same arithmetic, pipelined (ref_mfma_kernel measured ~0.4 ms per Llama-7B prefill
// projection in llama.cpp, profiles/r04/ref_order/: every chunk waited for its own HBM loads and
// built the block-diagonal operand with four per-lane selects per MFMA):
//   * the next chunk's A and activation bytes are loaded into registers while the current chunk
//     computes, then written to LDS between two barriers;
//   * the activation image in LDS is already block-diagonal: per (column, block, half) the four
//     quads as f16, each in its own 16-byte slot at the position its lanes need ({q, 0} for even
//     lanes l % 4, {0, q} for odd) -- one ds_read_b128 per MFMA operand, lanes whose slot is zero
//     read a shared zero quad;
//   * G groups of 8 columns per wave (G = 4: 64 columns per workgroup, the weight operand built
//     once per block for 4 groups).
//   * SW (LAMM_REF_MFMA=5): the per-chunk image stores without bank conflicts -- a thread's
//     (column, block) item puts columns 2 apart in each 16-lane group, and a block's 16 slots
//     are XOR-swizzled by 4 k dwords, so the 8 blocks of a column land in distinct banks (the
//     unswizzled stores hit 2 of the 64 banks' 16-dword groups: half the LDS cycles were
//     conflicts, profiles/r04/ref_order/kernels/); the reads stay conflict-free (the swizzle
//     only permutes a wave's 16-byte slots within each column).
#ifndef REF_AB
// probe builds only (ablations of the interleaved kernel, LAMM_REF_MFMA=6): 1 no chain steps, 2 no
// weight unpacking, 3 no chunk refills after the first (every chunk computed from the first image)
#define REF_AB 0
#endif
template <int T, int G, bool ONE_SLICE, bool SW = false, bool PIPE = false>
__global__ __launch_bounds__(MNT) void ref_mfma2_kernel(GemvArgs p) {
  using F = RefFmt<T>;
  static_assert(F::UE == 32, "32-element block formats");
  constexpr bool AFF = F::M >= 0;
  constexpr int MC2 = 16 * G;                       // columns per workgroup
  constexpr int SEG = MKB * F::BPB;
  static_assert(SEG % 16 == 0, "chunks start 16-byte aligned");
  constexpr int SEGW = SEG / 4 + 1;
  constexpr int NAL = MR * (SEG / 16);              // A b128 loads per chunk
  constexpr int NA = (NAL + MNT - 1) / MNT;
  constexpr int NITEM = MC2 * MKB;                  // activation blocks per chunk
  constexpr int NB = (NITEM + MNT - 1) / MNT;       // per thread
  static_assert(NITEM % MNT == 0 || NITEM < MNT, "whole activation items per thread");
  // the padded image: per column, block, half and k-group h of the MFMA operand, the 4 slots
  // (16 bytes each) lanes (slot, h) read: the quad for slots of that k-group, zeros otherwise --
  // the zero slots are written once; column pitch = 16 banks mod 64, so a ds_read_b128 lane
  // group (4 columns x 4 slots) covers the 64 banks once
  constexpr int NPC = MKB * 64 + 16;
  __shared__ __attribute__((aligned(16))) uint32_t sa[MR * SEGW];
  __shared__ __attribute__((aligned(16))) uint32_t sbp[MC2 * NPC];
  __shared__ float sdb[MKB][MC2];
  __shared__ float ssb[AFF ? MKB : 1][AFF ? MC2 : 1];

  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if constexpr (!ONE_SLICE) {
    const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  const int t = threadIdx.x, lane = t & 63, lr = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), wm = w & 1, wn = w >> 1;
  const int m0 = blockIdx.x * MR, n0 = blockIdx.y * MC2;
  const int nrows = p.M - m0 < MR ? p.M - m0 : MR;
  const int ncols = p.N - n0 < MC2 ? p.N - n0 : MC2;
  const int nunits = p.nblk;
  const auto ra = make_rsrc(Az + (int64_t)m0 * p.lda,
                            (uint32_t)(((int64_t)(nrows - 1) * p.lda + (int64_t)nunits * F::BPB + 3) & ~int64_t(3)));
  const int64_t bbytes = (int64_t)(ncols - 1) * p.ldb + (int64_t)nunits * F::VB;
  const auto rb = make_rsrc(Bz + (int64_t)n0 * p.ldb, (uint32_t)((bbytes + 3) & ~int64_t(3)));
  const int ml = 32 * wm + lr;

  static_assert(!SW || (MKB == 8 && MC2 % 4 == 0), "the swizzled item order");
  // packed chain steps where they cost no occupancy (the swizzled q4_0 kernel with them: 265 VGPRs)
  constexpr bool PK = (T == kQ4_0 || T == kQ5_1) && !SW;
  // item -> (column c, block k of the chunk)
  auto item_ck = [](int item, int& c, int& k) __attribute__((always_inline)) {
    if constexpr (SW) {
      const int u = item >> 3;
      k = item & 7;
      c = (u & ~3) | ((u & 1) << 1) | ((u >> 1) & 1);   // lanes' columns 2 apart per 16-lane group
    } else {
      c = item / MKB;
      k = item % MKB;
    }
  };
  // dword of slot L (0 .. 63) of block k in a column's image
  auto slot = [](int k, int L) __attribute__((always_inline)) { return k * 64 + (SW ? (L ^ (4 * k)) : L); };
  u32x4 pa[NA];
  uint32_t pb[NB][10];
  auto fetch = [&](int u0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int it = t + i * MNT, r = it / (SEG / 16), o = it % (SEG / 16);
      const uint32_t off = it < NAL && r < nrows ? (uint32_t)((int64_t)r * p.lda + (int64_t)u0 * F::BPB) + 16 * o
                                                 : 0x7ffffff0u;
      pa[i] = bload16(ra, off);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int item = t + j * MNT;
      int c, k;
      item_ck(item, c, k);
      const bool ok = item < NITEM && c < ncols && u0 + k < nunits;
      const uint32_t off = (uint32_t)((int64_t)c * p.ldb + (int64_t)(u0 + k) * F::VB);
      const uint32_t base = ok ? (off & ~3u) : 0x7ffffff0u;
#pragma unroll
      for (int i = 0; i < 10; ++i) pb[j][i] = bload4(rb, base + 4 * i);
    }
  };
  auto commit = [&](int u0) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int it = t + i * MNT, r = it / (SEG / 16), o = it % (SEG / 16);
      if (it < NAL) {
        uint32_t* dst = &sa[r * SEGW + 4 * o];
        dst[0] = pa[i][0]; dst[1] = pa[i][1]; dst[2] = pa[i][2]; dst[3] = pa[i][3];
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int item = t + j * MNT;
      int c, k;
      item_ck(item, c, k);
      if (item >= NITEM) break;
      const bool ok = c < ncols && u0 + k < nunits;
      const int sh = (int)((uint32_t)((int64_t)c * p.ldb + (int64_t)(u0 + k) * F::VB) & 3u) * 8;
      uint32_t m[9];
#pragma unroll
      for (int i = 0; i < 9; ++i) m[i] = __builtin_amdgcn_alignbit(pb[j][i + 1], pb[j][i], sh);
#pragma unroll
      for (int q = 0; q < 8; ++q) {   // quad q = lane q of the block: half q >> 2, slot q & 3
        const uint32_t qd = AFF ? m[1 + q] : __builtin_amdgcn_alignbit(m[q + 1], m[q], 16);
        uint32_t lo, hi;
        q4_to_f16<128>(qd ^ 0x80808080u, lo, hi);
        if (!ok) lo = hi = 0u;
        const u32x4 v = (q & 1) ? u32x4{0u, 0u, lo, hi} : u32x4{lo, hi, 0u, 0u};
        *reinterpret_cast<u32x4*>(&sbp[c * NPC + slot(k, ((q >> 2) * 2 + ((q & 3) >> 1)) * 16 + (q & 3) * 4)]) = v;
      }
      sdb[k][c] = ok ? h2f(m[0] & 0xffffu) : 0.f;
      if constexpr (AFF) ssb[k][c] = ok ? h2f(m[0] >> 16) : 0.f;
    }
  };

  f32x16 acc[G][2];
  float summs[G][4];
#pragma unroll
  for (int g = 0; g < G; ++g) {
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[g][q][r] = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) summs[g][c] = 0.f;
  }
  // this lane's operand slot in the padded image: row lr = (column lr / 4, slot lr % 4) of the
  // group, K = 8h .. 8h + 7 of the half -- nonzero only when the slot's quad lies there
  const int lq = lr & 3;
  const uint32_t* arow = &sa[ml * SEGW];
  const uint32_t* blc = &sbp[(8 * G * wn + (lr >> 2)) * NPC];   // + g, block, slot offsets
  const int lb = h * 16 + lq * 4;                                  // this lane's slot in half 0
  const uint32_t* bl = blc + lb;                                   // (unswizzled: + g, block offsets)
  for (int z = t; z < MC2 * MKB * 16; z += MNT) {   // the slots of the other k-group: zero for good
    const int c = z / (MKB * 16), rest = z % (MKB * 16), kh = rest >> 2, s = rest & 3;   // kh = (block, half, h)
    if ((s >> 1) != (kh & 1))
      *reinterpret_cast<u32x4*>(&sbp[c * NPC + slot(kh >> 2, (kh & 3) * 16 + s * 4)]) = u32x4{0u, 0u, 0u, 0u};
  }
  fetch(0);
  for (int u0 = 0; u0 < nunits; u0 += MKB) {
    const int nu = nunits - u0 < MKB ? nunits - u0 : MKB;
    if (!(PIPE && REF_AB == 3) || u0 == 0) {
      if (u0 > 0) __syncthreads();   // every wave is done reading the previous chunk
      commit(u0);
      __syncthreads();
      if (u0 + MKB < nunits) fetch(u0 + MKB);   // the next chunk's bytes fly under this one's math
    }
    // swizzled: this lane's slot per block, recomputed every chunk (one v_xor per block) rather than
    // eight hoisted addresses held across the loop (VGPRs past 256: occupancy 1)
    int lbs = lb;
    if constexpr (SW) asm volatile("" : "+v"(lbs));
    auto block = [&](int k) {
      const int ub = k * F::BPB;
      const float da = h2f(lds32(arow, ub) & 0xffffu);
      const float ma = AFF ? h2f(lds32(arow, ub + (AFF ? F::M : 0)) & 0xffffu) : 0.f;
      uint32_t q0 = lds32(arow, ub + F::QS + 8 * h), q1 = lds32(arow, ub + F::QS + 8 * h + 4);
      uint32_t wlo[2] = {q0 & 0x0f0f0f0fu, q1 & 0x0f0f0f0fu};
      uint32_t whi[2] = {(q0 >> 4) & 0x0f0f0f0fu, (q1 >> 4) & 0x0f0f0f0fu};
      if constexpr (F::QH >= 0) {
        const uint32_t qh = lds32(arow, ub + (F::QH >= 0 ? F::QH : 0));
        wlo[0] |= spread4_hi((qh >> (8 * h)) & 0xfu);
        wlo[1] |= spread4_hi((qh >> (8 * h + 4)) & 0xfu);
        whi[0] |= spread4_hi((qh >> (16 + 8 * h)) & 0xfu);
        whi[1] |= spread4_hi((qh >> (16 + 8 * h + 4)) & 0xfu);
      }
      uint32_t wf[2][4];
      if constexpr (PIPE && REF_AB == 2) {
        wf[0][0] = wf[0][1] = wlo[0]; wf[0][2] = wf[0][3] = wlo[1];
        wf[1][0] = wf[1][1] = whi[0]; wf[1][2] = wf[1][3] = whi[1];
      } else {
        q4_to_f16<F::OFF>(wlo[0], wf[0][0], wf[0][1]);
        q4_to_f16<F::OFF>(wlo[1], wf[0][2], wf[0][3]);
        q4_to_f16<F::OFF>(whi[0], wf[1][0], wf[1][1]);
        q4_to_f16<F::OFF>(whi[1], wf[1][2], wf[1][3]);
      }
      const half8 W0 = __builtin_bit_cast(half8, u32x4{wf[0][0], wf[0][1], wf[0][2], wf[0][3]});
      const half8 W1 = __builtin_bit_cast(half8, u32x4{wf[1][0], wf[1][1], wf[1][2], wf[1][3]});
      if constexpr (PIPE) {
        // the chain steps of group g wait on that group's MFMAs; issue group g + 1's MFMAs between
        // group g's two halves of chain steps so each half finds its MFMA result done (a half's
        // results: 16 VGPRs; at most 3 halves live, +16 VGPRs over the plain order)
        f32x16 S[G][2];
        float d[G][4];
        const f32x16 zero = {};
        auto issue = [&](int g, int q) {
          const uint32_t* bk = SW ? &blc[g * 8 * NPC + k * 64 + (lbs ^ (4 * k))] : &bl[g * 8 * NPC + k * 64];
          const u32x4 a = *reinterpret_cast<const u32x4*>(bk + 32 * q);
          S[g][q] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a), q ? W1 : W0, zero, 0, 0, 0);
        };
        auto chains = [&](int g, int q) {
          if constexpr (REF_AB == 1) {
#pragma unroll
            for (int i = 0; i < 16; ++i) asm volatile("" ::"v"(S[g][q][i]));
            return;
          }
#pragma unroll
          for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int e = 0; e < 4; ++e)
              acc[g][q][4 * c + e] = __builtin_fmaf(d[g][c], S[g][q][4 * c + e], acc[g][q][4 * c + e]);
        };
#pragma unroll
        for (int g = 0; g < G; ++g) {
          const int nb = 8 * G * wn + 8 * g;
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            d[g][c] = da * sdb[k][nb + 2 * c + h];
            asm("" : "+v"(d[g][c]));
            if constexpr (AFF) {
              float pm = ma * ssb[k][nb + 2 * c + h];
              asm("" : "+v"(pm));
              summs[g][c] = summs[g][c] + pm;
            }
          }
        }
        issue(0, 0);
        issue(0, 1);
#pragma unroll
        for (int g = 0; g < G; ++g) {
          if (g + 1 < G) issue(g + 1, 0);
          __builtin_amdgcn_sched_barrier(0);
          chains(g, 0);
          if (g + 1 < G) issue(g + 1, 1);
          __builtin_amdgcn_sched_barrier(0);
          chains(g, 1);
        }
      } else {
  #pragma unroll
        for (int g = 0; g < G; ++g) {
          const int nb = 8 * G * wn + 8 * g;
          // half 1's slot is half 0's + 32: the swizzle (4 k < 32) leaves bit 5 alone
          const uint32_t* bk = SW ? &blc[g * 8 * NPC + k * 64 + (lbs ^ (4 * k))] : &bl[g * 8 * NPC + k * 64];
          const u32x4 a0 = *reinterpret_cast<const u32x4*>(bk);
          const u32x4 a1 = *reinterpret_cast<const u32x4*>(bk + 32);
          const f32x16 zero = {};
          const f32x16 S0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a0), W0, zero, 0, 0, 0);
          const f32x16 S1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a1), W1, zero, 0, 0, 0);
  #pragma unroll
          for (int c = 0; c < 4; ++c) {
            float d = da * sdb[k][nb + 2 * c + h];
            asm("" : "+v"(d));
            // lanes e, e + 1 of a column share d: one packed fp32 fma per pair (v_pk_fma_f32, each
            // element one IEEE fma -- the same bits as two v_fma_f32).  q4_1 / q5_0: single fmas
            // (the packed form's register pairs push those kernels past 256 VGPRs: one wave per SIMD)
            if constexpr (PK) {
              const f32x2 d2 = {d, d};
  #pragma unroll
              for (int e = 0; e < 4; e += 2) {
                const int i = 4 * c + e;
                const f32x2 r0 = __builtin_elementwise_fma(d2, f32x2{S0[i], S0[i + 1]}, f32x2{acc[g][0][i], acc[g][0][i + 1]});
                const f32x2 r1 = __builtin_elementwise_fma(d2, f32x2{S1[i], S1[i + 1]}, f32x2{acc[g][1][i], acc[g][1][i + 1]});
                acc[g][0][i] = r0[0], acc[g][0][i + 1] = r0[1];
                acc[g][1][i] = r1[0], acc[g][1][i + 1] = r1[1];
              }
            } else {
  #pragma unroll
              for (int e = 0; e < 4; ++e) {
                acc[g][0][4 * c + e] = __builtin_fmaf(d, S0[4 * c + e], acc[g][0][4 * c + e]);
                acc[g][1][4 * c + e] = __builtin_fmaf(d, S1[4 * c + e], acc[g][1][4 * c + e]);
              }
            }
            if constexpr (AFF) {
              float pm = ma * ssb[k][nb + 2 * c + h];
              asm("" : "+v"(pm));
              summs[g][c] = summs[g][c] + pm;
            }
          }
        }
      }
    };
    if (nu == MKB) {   // a whole chunk: unrolled, so the next block's LDS reads run ahead
#pragma unroll
      for (int k = 0; k < MKB; ++k) block(k);
    } else {
      for (int k = 0; k < nu; ++k) block(k);
    }
  }
  const int m = m0 + ml;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int n = 8 * G * wn + 8 * g + 2 * c + h;
      float v;
      {
#pragma clang fp contract(off)
        const float x0 = acc[g][0][4 * c + 0] + acc[g][1][4 * c + 0], x1 = acc[g][0][4 * c + 1] + acc[g][1][4 * c + 1];
        const float x2 = acc[g][0][4 * c + 2] + acc[g][1][4 * c + 2], x3 = acc[g][0][4 * c + 3] + acc[g][1][4 * c + 3];
        v = (x0 + x2) + (x1 + x3);
        if constexpr (AFF) v = v + summs[g][c];
      }
      if (m < p.M && n < ncols) Cz[(int64_t)(n0 + n) * p.ldc + m] = v;
    }
}

// q6_K x q8_K prefill in ggml's AVX2 order (ggml_vec_dot_q6_K_q8_K): per super-block
//   X_l = sum_h sc[2h + (l >= 4)] * (4-element dot of group h, lane l)   (exact int32)
//   acc_l = fma(y.d * fp32(x.d), (float)X_l, acc_l)
// Each 32-element group h is one "block" of ref_mfma2_kernel's block-diagonal MFMA (the lane dots
// of 32 weight rows x 8 columns, two MFMAs per group); X accumulates in fp32 registers
// (X += sc * S: integers below 2^24, exact) and the chain step runs once per super-block.
// One super-block per chunk: the rows' 210 bytes come by dword loads from the dword below their
// start (a 2-byte shift on odd super-blocks), the activation quads go to the padded f16 image.
template <int G, bool ONE_SLICE>
__global__ __launch_bounds__(MNT) void ref_mfma_kq_kernel(GemvArgs p) {
  constexpr int MC2 = 16 * G;
  constexpr int AW = 54;                            // dwords per row image (210 bytes + a 2-byte shift)
  constexpr int NAL = MR * AW;
  constexpr int NA = (NAL + MNT - 1) / MNT;
  constexpr int NQ = MC2 * 64;                      // activation quads per super-block
  constexpr int NB = NQ / MNT;
  static_assert(NQ % MNT == 0, "whole quads per thread");
  constexpr int NPC = 512 + 16;                     // per column: 8 groups x 2 halves x 2 k-groups x 4 slots x 4
  __shared__ __attribute__((aligned(16))) uint32_t sa[MR * (AW + 1)];
  __shared__ __attribute__((aligned(16))) uint32_t sbp[MC2 * NPC];
  __shared__ float sdb[MC2];

  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if constexpr (!ONE_SLICE) {
    const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  const int t = threadIdx.x, lane = t & 63, lr = lane & 31, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6), wm = w & 1, wn = w >> 1;
  const int m0 = blockIdx.x * MR, n0 = blockIdx.y * MC2;
  const int nrows = p.M - m0 < MR ? p.M - m0 : MR;
  const int ncols = p.N - n0 < MC2 ? p.N - n0 : MC2;
  const int nsb = p.nblk;
  const auto ra = make_rsrc(Az + (int64_t)m0 * p.lda,
                            (uint32_t)(((int64_t)(nrows - 1) * p.lda + (int64_t)nsb * 210 + 3) & ~int64_t(3)));
  const auto rb = make_rsrc(Bz + (int64_t)n0 * p.ldb, (uint32_t)((int64_t)(ncols - 1) * p.ldb + (int64_t)nsb * 292));
  const int ml = 32 * wm + lr;

  uint32_t pa[NA], pb[NB];
  float pd = 0.f;
  auto fetch = [&](int u) {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int it = t + i * MNT, r = it / AW, o = it % AW;
      const uint32_t off = it < NAL && r < nrows ? (uint32_t)(((int64_t)r * p.lda + (int64_t)u * 210) & ~int64_t(3)) + 4 * o
                                                 : 0x7ffffff0u;
      pa[i] = bload4(ra, off);
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int item = t + j * MNT, c = item >> 6, qi = item & 63;
      pb[j] = bload4(rb, c < ncols ? (uint32_t)((int64_t)c * p.ldb + (int64_t)u * 292 + 4 + 4 * qi) : 0x7ffffff0u);
    }
    if (t < MC2) pd = __builtin_bit_cast(float, bload4(rb, t < ncols ? (uint32_t)((int64_t)t * p.ldb + (int64_t)u * 292)
                                                                      : 0x7ffffff0u));
  };
  auto commit = [&]() {
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int it = t + i * MNT, r = it / AW, o = it % AW;
      if (it < NAL) sa[r * (AW + 1) + o] = pa[i];
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int item = t + j * MNT, c = item >> 6, qi = item & 63;   // quad qi: group qi / 8, lane qi % 8
      uint32_t lo, hi;
      q4_to_f16<128>(pb[j] ^ 0x80808080u, lo, hi);
      const int l = qi & 7;
      const u32x4 v = (l & 1) ? u32x4{0u, 0u, lo, hi} : u32x4{lo, hi, 0u, 0u};
      *reinterpret_cast<u32x4*>(&sbp[c * NPC + (((qi >> 3) * 2 + (l >> 2)) * 2 + ((l & 3) >> 1)) * 16 + (l & 3) * 4]) = v;
    }
    if (t < MC2) sdb[t] = pd;
  };

  f32x16 acc[G][2];
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[g][q][r] = 0.f;
  const int lq = lr & 3;
  const uint32_t* arow = &sa[ml * (AW + 1)];
  const uint32_t* bl = &sbp[(8 * G * wn + (lr >> 2)) * NPC + h * 16 + lq * 4];
  for (int z = t; z < MC2 * 128; z += MNT) {   // the other k-group's slots: zero for good
    const int c = z >> 7, kh = (z & 127) >> 2, s = z & 3;
    if ((s >> 1) != (kh & 1)) *reinterpret_cast<u32x4*>(&sbp[c * NPC + kh * 16 + s * 4]) = u32x4{0u, 0u, 0u, 0u};
  }
  fetch(0);
  for (int u = 0; u < nsb; ++u) {
    const int sh = (int)(((int64_t)ml * p.lda + (int64_t)u * 210) & 3);   // this row's shift in its image
    if (u > 0) __syncthreads();
    commit();
    __syncthreads();
    if (u + 1 < nsb) fetch(u + 1);
    const float da = h2f(lds32(arow, sh + 208) & 0xffffu);
    const uint32_t scw[4] = {lds32(arow, sh + 192), lds32(arow, sh + 196), lds32(arow, sh + 200), lds32(arow, sh + 204)};
    f32x16 X[G][2];
#pragma unroll
    for (int g = 0; g < G; ++g)
#pragma unroll
      for (int q = 0; q < 2; ++q)
#pragma unroll
        for (int r = 0; r < 16; ++r) X[g][q][r] = 0.f;
#pragma unroll 1
    for (int gh = 0; gh < 8; ++gh) {   // group gh = 4 j + gg: ql[64 j + 32 (gg & 1) + e], qh[32 j + e] >> 2 gg
      const int j = gh >> 2, gg = gh & 3;
      uint32_t wf[2][4];
#pragma unroll
      for (int q = 0; q < 2; ++q) {   // half q: elements 16 q + 8 h .. + 7 of the group
        const int e0 = 16 * q + 8 * h;
        const uint32_t l0 = lds32(arow, sh + 64 * j + 32 * (gg & 1) + e0), l1 = lds32(arow, sh + 64 * j + 32 * (gg & 1) + e0 + 4);
        const uint32_t h0 = lds32(arow, sh + 128 + 32 * j + e0), h1 = lds32(arow, sh + 128 + 32 * j + e0 + 4);
        const uint32_t v0 = ((gg < 2 ? l0 : l0 >> 4) & 0x0f0f0f0fu) | (((h0 >> (2 * gg)) & 0x03030303u) << 4);
        const uint32_t v1 = ((gg < 2 ? l1 : l1 >> 4) & 0x0f0f0f0fu) | (((h1 >> (2 * gg)) & 0x03030303u) << 4);
        q4_to_f16<32>(v0, wf[q][0], wf[q][1]);
        q4_to_f16<32>(v1, wf[q][2], wf[q][3]);
      }
      const half8 W0 = __builtin_bit_cast(half8, u32x4{wf[0][0], wf[0][1], wf[0][2], wf[0][3]});
      const half8 W1 = __builtin_bit_cast(half8, u32x4{wf[1][0], wf[1][1], wf[1][2], wf[1][3]});
      // scales of the group's two 16-element halves (lanes 0-3 / 4-7): sc[2 gh], sc[2 gh + 1]
      const float s0 = (float)(int8_t)((scw[gh >> 1] >> (16 * (gh & 1))) & 0xffu);
      const float s1 = (float)(int8_t)((scw[gh >> 1] >> (16 * (gh & 1) + 8)) & 0xffu);
#pragma unroll
      for (int g = 0; g < G; ++g) {
        const u32x4 a0 = *reinterpret_cast<const u32x4*>(&bl[g * 8 * NPC + gh * 64]);
        const u32x4 a1 = *reinterpret_cast<const u32x4*>(&bl[g * 8 * NPC + gh * 64 + 32]);
        const f32x16 zero = {};
        const f32x16 S0 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a0), W0, zero, 0, 0, 0);
        const f32x16 S1 = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, a1), W1, zero, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 16; ++r) {   // exact: |X| < 2^24
          X[g][0][r] = __builtin_fmaf(s0, S0[r], X[g][0][r]);
          X[g][1][r] = __builtin_fmaf(s1, S1[r], X[g][1][r]);
        }
      }
    }
#pragma unroll
    for (int g = 0; g < G; ++g) {
      const int nb = 8 * G * wn + 8 * g;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        float d = sdb[nb + 2 * c + h] * da;   // y.d * fp32(x.d)
        asm("" : "+v"(d));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          acc[g][0][4 * c + e] = __builtin_fmaf(d, X[g][0][4 * c + e], acc[g][0][4 * c + e]);
          acc[g][1][4 * c + e] = __builtin_fmaf(d, X[g][1][4 * c + e], acc[g][1][4 * c + e]);
        }
      }
    }
  }
  const int m = m0 + ml;
#pragma unroll
  for (int g = 0; g < G; ++g)
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int n = 8 * G * wn + 8 * g + 2 * c + h;
      float v;
      {
#pragma clang fp contract(off)
        const float x0 = acc[g][0][4 * c + 0] + acc[g][1][4 * c + 0], x1 = acc[g][0][4 * c + 1] + acc[g][1][4 * c + 1];
        const float x2 = acc[g][0][4 * c + 2] + acc[g][1][4 * c + 2], x3 = acc[g][0][4 * c + 3] + acc[g][1][4 * c + 3];
        v = (x0 + x2) + (x1 + x3);
      }
      if (m < p.M && n < ncols) Cz[(int64_t)(n0 + n) * p.ldc + m] = v;
    }
}

}  // namespace

bool ref_order_supported(int type, int btype) {
  switch (type) {
    case kQ4_0: case kQ5_0: return btype == kQ8_0;
    case kQ4_1: case kQ5_1: return btype == kQ8_1;
    case kQ2_K: case kQ4_K: case kQ5_K: case kQ6_K: return btype == kQ8_K;
    case kF16: return btype == kF16;
    default: return false;
  }
}

bool ref_gemv_supported(int type, const GemvArgs& p) {
  const bool fmt = type == kQ4_0 || type == kQ4_1 || type == kQ5_0 || type == kQ5_1;
  return fmt && p.N == 1 && p.nblk <= 576 && ref_gemv_lds(type, p.nblk) <= 65536;
}

hipError_t launch_ref(int type, const GemvArgs& p, hipStream_t s) {
  const int slices = p.ne12 * p.ne13;
  if (ref_gemv_supported(type, p)) {   // one column: ref_gemv_kernel (F32 rows quantized in its staging)
    const dim3 g((unsigned)((p.M + GR - 1) / GR), 1, (unsigned)slices);
    const bool long_k = p.nblk > GKC;   // K > 4096: chunks of GKC, else GKC_S
    const size_t lds = ref_gemv_lds(type, p.nblk, long_k ? GKC : GKC_S);
    const LaunchTiming tm = take_launch_timing();
    auto gov = [&](auto tc) {
      constexpr int T = decltype(tc)::value;
      auto go3 = [&](auto kern, int nt) {
        if (tm.start) hipExtLaunchKernelGGL(kern, g, dim3(nt), lds, s, tm.start, tm.stop, 0, p);
        else if (!direct_launch(reinterpret_cast<const void*>(kern), g, dim3(nt), (uint32_t)lds, &p, sizeof p))
          hipLaunchKernelGGL(kern, g, dim3(nt), lds, s, p);   // (direct: the library's own queue, lamm_aql.cpp)
      };
      auto go1 = [&](auto bc, auto cc) {
        constexpr int BPT = decltype(bc)::value, CK = decltype(cc)::value, nt = GR * CK / BPT;
        if (p.b_f32) {
          if (slices == 1) go3(ref_gemv_kernel<T, true, true, BPT, CK>, nt);
          else go3(ref_gemv_kernel<T, true, false, BPT, CK>, nt);
        } else {
          if (slices == 1) go3(ref_gemv_kernel<T, false, true, BPT, CK>, nt);
          else go3(ref_gemv_kernel<T, false, false, BPT, CK>, nt);
        }
      };
      auto go2 = [&](auto bc) {
        if (long_k) go1(bc, std::integral_constant<int, GKC>{});
        else go1(bc, std::integral_constant<int, GKC_S>{});
      };
      if (knobs().ref_gemv_bpt == 4) go2(std::integral_constant<int, 4>{});
      else go2(std::integral_constant<int, 2>{});
    };
    switch (type) {
      case kQ4_0: gov(std::integral_constant<int, kQ4_0>{}); break;
      case kQ4_1: gov(std::integral_constant<int, kQ4_1>{}); break;
      case kQ5_0: gov(std::integral_constant<int, kQ5_0>{}); break;
      case kQ5_1: gov(std::integral_constant<int, kQ5_1>{}); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  if (p.b_f32) return hipErrorInvalidValue;   // F32 activations: the one-column kernel only
  if (type == kF16) {   // ggml_vec_dot_f16's order (ref_f16_kernel); 16-byte rows take wide loads
    const dim3 g((unsigned)((p.M + FT - 1) / FT), (unsigned)((p.N + FT - 1) / FT), (unsigned)slices);
    const bool vec = ((uintptr_t)p.B & 15) == 0 && (p.ldb & 15) == 0 && (p.sb2 & 15) == 0 && (p.sb3 & 15) == 0 &&
                     (p.lda & 15) == 0 && ((uintptr_t)p.A & 15) == 0;
    if (vec) {
      if (slices == 1) hipLaunchKernelGGL((ref_f16_kernel<true, true>), g, dim3(FNT), 0, s, p);
      else hipLaunchKernelGGL((ref_f16_kernel<true, false>), g, dim3(FNT), 0, s, p);
    } else {
      if (slices == 1) hipLaunchKernelGGL((ref_f16_kernel<false, true>), g, dim3(FNT), 0, s, p);
      else hipLaunchKernelGGL((ref_f16_kernel<false, false>), g, dim3(FNT), 0, s, p);
    }
    return hipGetLastError();
  }
  // prefill-sized calls on the 32-element formats: the MFMA form (ref_mfma_kernel)
  if (p.N > 8 && type == kQ6_K && knobs().ref_mfma != 1) {   // q6_K prefill: ref_mfma_kq_kernel
    const dim3 gm((unsigned)((p.M + MR - 1) / MR), (unsigned)((p.N + 31) / 32), (unsigned)slices);
    if (slices == 1) hipLaunchKernelGGL((ref_mfma_kq_kernel<2, true>), gm, dim3(MNT), 0, s, p);
    else hipLaunchKernelGGL((ref_mfma_kq_kernel<2, false>), gm, dim3(MNT), 0, s, p);
    return hipGetLastError();
  }
  if (p.N > 8 && type != kQ6_K && type != kQ2_K && type != kQ4_K && type != kQ5_K) {
    // ref_mfma2_kernel, 2 column groups per wave (LAMM_REF_MFMA=4: 4 groups, one wave per SIMD; =1:
    // the unpipelined ref_mfma_kernel)
    // default per format (tools/ref_ab.py, profiles/r04/ref_order/pk_fma/, profiles/r05/ref_pipe/):
    // the swizzled 2-group kernel with each group's chain steps behind the next group's MFMAs for
    // q4_0 / q5_0 (6); q4_1 without that (its extra VGPRs cost a wave per SIMD: 5); q5_1's larger
    // chunk keeps ref_mfma2 at one wave per SIMD, so it runs the unpipelined ref_mfma_kernel (1)
    const int sel = knobs().ref_mfma > 0 ? knobs().ref_mfma : type == kQ5_1 ? 1 : type == kQ4_1 ? 5 : 6;
    const int mc = sel == 4 ? 64 : sel == 3 ? 16 : 32;   // 5: the 2-group kernel, swizzled image
    const dim3 gm((unsigned)((p.M + MR - 1) / MR), (unsigned)((p.N + mc - 1) / mc), (unsigned)slices);
    auto gom = [&](auto tc) {
      constexpr int T = decltype(tc)::value;
      if (sel == 1) {
        if (slices == 1) hipLaunchKernelGGL((ref_mfma_kernel<T, true>), gm, dim3(MNT), 0, s, p);
        else hipLaunchKernelGGL((ref_mfma_kernel<T, false>), gm, dim3(MNT), 0, s, p);
      } else if (sel == 4) {
        if (slices == 1) hipLaunchKernelGGL((ref_mfma2_kernel<T, 4, true>), gm, dim3(MNT), 0, s, p);
        else hipLaunchKernelGGL((ref_mfma2_kernel<T, 4, false>), gm, dim3(MNT), 0, s, p);
      } else if (sel == 3) {   // one column group per wave (occupancy over reuse)
        if (slices == 1) hipLaunchKernelGGL((ref_mfma2_kernel<T, 1, true>), gm, dim3(MNT), 0, s, p);
        else hipLaunchKernelGGL((ref_mfma2_kernel<T, 1, false>), gm, dim3(MNT), 0, s, p);
      } else if (sel == 6) {   // swizzled, chain steps interleaved with the next group's MFMAs
        if (slices == 1) hipLaunchKernelGGL((ref_mfma2_kernel<T, 2, true, true, true>), gm, dim3(MNT), 0, s, p);
        else hipLaunchKernelGGL((ref_mfma2_kernel<T, 2, false, true, true>), gm, dim3(MNT), 0, s, p);
      } else if (sel == 5) {
        if (slices == 1) hipLaunchKernelGGL((ref_mfma2_kernel<T, 2, true, true>), gm, dim3(MNT), 0, s, p);
        else hipLaunchKernelGGL((ref_mfma2_kernel<T, 2, false, true>), gm, dim3(MNT), 0, s, p);
      } else {
        if (slices == 1) hipLaunchKernelGGL((ref_mfma2_kernel<T, 2, true>), gm, dim3(MNT), 0, s, p);
        else hipLaunchKernelGGL((ref_mfma2_kernel<T, 2, false>), gm, dim3(MNT), 0, s, p);
      }
    };
    switch (type) {
      case kQ4_0: gom(std::integral_constant<int, kQ4_0>{}); break;
      case kQ4_1: gom(std::integral_constant<int, kQ4_1>{}); break;
      case kQ5_0: gom(std::integral_constant<int, kQ5_0>{}); break;
      case kQ5_1: gom(std::integral_constant<int, kQ5_1>{}); break;
      default: return hipErrorInvalidValue;
    }
    return hipGetLastError();
  }
  // columns per workgroup: the N of a decode call (1, 2, 4), else 8
  const int nc = p.N <= 1 ? 1 : p.N <= 2 ? 2 : p.N <= 4 ? 4 : 8;
  const dim3 g((unsigned)((p.M + RR - 1) / RR), (unsigned)((p.N + nc - 1) / nc), (unsigned)slices);
  auto go = [&](auto tc) {
    constexpr int T = decltype(tc)::value;
    auto go2 = [&](auto ncc) {
      constexpr int NC = decltype(ncc)::value;
      // 16 rows per workgroup for one or two columns (a decode GEMV: twice the workgroups) and for
      // q6_K (8 super-blocks of 32 rows would not fit the 64 KiB of static LDS), else 32
      constexpr int R = NC <= 2 || RefFmt<T>::UE == 256 ? 16 : 32;
      const dim3 gr((unsigned)((p.M + R - 1) / R), g.y, g.z);
      if (slices == 1) hipLaunchKernelGGL((ref_kernel<T, R, NC, true>), gr, dim3(R * 8), 0, s, p);
      else hipLaunchKernelGGL((ref_kernel<T, R, NC, false>), gr, dim3(R * 8), 0, s, p);
    };
    if (nc == 1) go2(std::integral_constant<int, 1>{});
    else if (nc == 2) go2(std::integral_constant<int, 2>{});
    else if (nc == 4) go2(std::integral_constant<int, 4>{});
    else go2(std::integral_constant<int, 8>{});
  };
  switch (type) {
    case kQ4_0: go(std::integral_constant<int, kQ4_0>{}); break;
    case kQ4_1: go(std::integral_constant<int, kQ4_1>{}); break;
    case kQ5_0: go(std::integral_constant<int, kQ5_0>{}); break;
    case kQ5_1: go(std::integral_constant<int, kQ5_1>{}); break;
    case kQ2_K: go(std::integral_constant<int, kQ2_K>{}); break;
    case kQ4_K: go(std::integral_constant<int, kQ4_K>{}); break;
    case kQ5_K: go(std::integral_constant<int, kQ5_K>{}); break;
    case kQ6_K: go(std::integral_constant<int, kQ6_K>{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_ref_group(int type, const GemvArgs& p, const RefSegs& sg, int nseg, hipStream_t s) {
  if (nseg < 1 || nseg > kRefSegs || !ref_gemv_supported(type, p) || p.ne12 * p.ne13 != 1 || p.flag)
    return hipErrorInvalidValue;
  int mmax = 0;
  for (int i = 0; i < nseg; ++i) mmax = sg.M[i] > mmax ? sg.M[i] : mmax;
  const dim3 g((unsigned)((mmax + REF_GROUP_RG - 1) / REF_GROUP_RG), 1, (unsigned)nseg);
  const size_t lds = ref_gemv_lds(type, p.nblk, GKC_S, REF_GROUP_RG);
  auto gov = [&](auto tc) {
    constexpr int T = decltype(tc)::value;
    auto go2 = [&](auto bc) {
      constexpr int BPT = decltype(bc)::value, nt = REF_GROUP_RG * GKC_S / BPT;
      if (p.b_f32) hipLaunchKernelGGL((ref_gemv_group_kernel<T, true, BPT>), g, dim3(nt), lds, s, p, sg);
      else hipLaunchKernelGGL((ref_gemv_group_kernel<T, false, BPT>), g, dim3(nt), lds, s, p, sg);
    };
    if (knobs().ref_gemv_bpt == 4) go2(std::integral_constant<int, 4>{});
    else go2(std::integral_constant<int, 2>{});
  };
  switch (type) {
    case kQ4_0: gov(std::integral_constant<int, kQ4_0>{}); break;
    case kQ4_1: gov(std::integral_constant<int, kQ4_1>{}); break;
    case kQ5_0: gov(std::integral_constant<int, kQ5_0>{}); break;
    case kQ5_1: gov(std::integral_constant<int, kQ5_1>{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace lamm
