// lamm_gemm_dq.hip -- prefill GEMM (N > 8) for the 32-element block formats (q4_0, q4_1, q5_0,
// q5_1, q8_0 weights x q8_0 / q8_1 activation rows) on f16 MFMAs, the block scales folded into
// the operands while the raw blocks are unpacked in registers: one launch, no packing pass.
//
// Contract: the lamm block kernels (src/lamm_kernel_q4_0.hpp:59-128, q4_1 :46-116, q5_0 :69-139,
// q5_1 :80-153, q8_0 :50-117 via LAMMImpl<T>::matmul_simd_block, src/lamm_impl.hpp:90-147):
//   C[j*ldc + i] = sum_blocks d_a*d_b*S (+ m_a*s_b),   S = the int block dot
// within the north star's 1e-3 relative bar, NOT bit for bit: every weight element
// becomes ONE f16 value d_a*(q - c) (or d_a*q + m_a), every activation element ONE f16 value d_b*b,
// each rounded once (relative error <= 2^-11 each, so <= 2^-10 + 2^-22 per product, below the bar
// before the fp32 accumulation; random operands ~1e-5).  The exact engine (block-scaled fp6 MFMA +
// per-block fp32 epilogue, lamm_gemm_fp6.hip) stays selectable (LAMM_GEMM_PATH=fp6).
//
// Why.  With exact block dots every 32-element block needs its own fp32 scale per OUTPUT element
// (a 32x32 tile: 16 FMAs per lane per block); here the scales cost per LOADED element (3 VALU per
// pair of values), and a CU's 128 x 64 tile loads 42x fewer elements than it outputs per block.
// The raw AoS blocks are read as they lie (0.56 B / element for q4_0 instead of the fp6 planes'
// 1.0), so a CU streams 573 KB at config 3 instead of 1 MiB, with no activation-packing launch.
//
// Unpacking (per pair of values, both in one dword at an even byte offset):
//   v_perm_b32(0x64646464, bytes, sel) -> f16 bits 0x64XY = 1024 + u   (u = the quant as unsigned)
//   v_pk_add_f16(v, -(1024 + c))       -> u - c exactly (small integers)
//   v_pk_mul_f16(., {d, d})            -> d (u - c), one rounding     [affine: v_pk_fma_f16(q, d, m)]
// 4-bit quants are split into low / high nibble dwords first (and / shift+and per 4 bytes), q5's
// 5th bits OR'ed in, q8 bytes xor 0x80 (u = b + 128, c = 128).
//
// Tiling: 128 weight rows x 64 activation rows per workgroup (one per CU), 4 waves = 4 K-groups:
// wave g takes quads (4 consecutive blocks) g, g + 4, ...; in a quad, lane (r, h) holds blocks
// 2h, 2h + 1 of its row's quad (both operands, the same element order), so each of the quad's 8
// v_mfma_f32_32x32x16_f16 k-steps covers element group s % 4 of block s / 4 in the h = 0 lanes and
// of block 2 + s / 4 in the h = 1 lanes.  A wave owns the whole 128 x 64 tile (8 tiles of 32x32,
// 128 f32 accumulators): no operand is unpacked twice.  The quads' raw bytes come straight into
// VGPRs (NBUF quads in flight); at the end the 4 partial tiles meet in LDS and are summed in group
// order (deterministic, and independent of M: a row's value does not depend on how the rows of C
// are split over launches or ranks).
#include "lamm_device.h"
#include "lamm_kernels.h"
#include "lamm_rowdot.h"

namespace lamm {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));

// block layout of a weight / activation format: bytes per block, offset of qs / qh / m, 4-bit
// quants, the unsigned-quant offset c (value = d (u - c) [+ m])
template <int T> struct DqFmt;
template <> struct DqFmt<kQ4_0> { static constexpr int BPB = 18, QS = 2, QH = -1, MO = -1, C = 8; static constexpr bool NIB = true; };
template <> struct DqFmt<kQ4_1> { static constexpr int BPB = 20, QS = 4, QH = -1, MO = 2, C = 0; static constexpr bool NIB = true; };
template <> struct DqFmt<kQ5_0> { static constexpr int BPB = 22, QS = 6, QH = 2, MO = -1, C = 16; static constexpr bool NIB = true; };
template <> struct DqFmt<kQ5_1> { static constexpr int BPB = 24, QS = 8, QH = 4, MO = 2, C = 0; static constexpr bool NIB = true; };
template <> struct DqFmt<kQ8_0> { static constexpr int BPB = 34, QS = 2, QH = -1, MO = -1, C = 128; static constexpr bool NIB = false; };
// q8_1: its s = d * sum(q) is implied by the unpacked values (sum_k (d_a q_k + m_a) d_b b_k)
template <> struct DqFmt<kQ8_1> { static constexpr int BPB = 36, QS = 4, QH = -1, MO = -1, C = 128; static constexpr bool NIB = false; };

#ifndef DQ_AB
// probe builds only (tools/build_dq_var.sh): 1 loads only, 2 unpack + MFMA only (no loads after the
// first quads)
#define DQ_AB 0
#endif

constexpr int DQ_TI = 128, DQ_TJ = 64, DQ_KG = 4, DQ_NT = 256;
constexpr int DQ_PI = DQ_TI + 8;   // LDS pitch of a parked partial row: the two half-waves' rows j, j + 4
                                   // fall on disjoint banks
constexpr size_t DQ_LDS = (size_t)DQ_KG * DQ_TJ * DQ_PI * 4;
// weights are pre-scaled by 2^8 and activations by 2^4 (both exact) so the block scales of real
// operands stay in f16's normal range; C is scaled back by 2^-12 (exact) in the epilogue.  The
// window this leaves -- weight d in [2^-22, 2^8), activation d in [2^-18, 2^5) -- is enforced at run
// time by the range guard below, not assumed.
constexpr float DQ_ASCALE = 256.f, DQ_BSCALE = 16.f, DQ_CSCALE = 1.f / 4096.f;

// ---------------------------------------------------------------- range guard
// dq16 is exact to 2^-10 per product only while every unpacked f16 value is normal and finite.  Each
// lane tracks the range of the pre-scaled block scales it unpacks (DqRange: a subnormal, inf or NaN
// scale -> bad); an operand value that overflows f16 (|d * q| > 65504) turns its MFMA results into
// inf / NaN, which the tile's final accumulators show.  A workgroup that sees either recomputes its
// whole tile with exact int8 block dots (dq_exact_tile: d_a * d_b * S [+ m_a * s_b] in fp32, the
// reference's lamm_kernel_q*.hpp arithmetic) -- slow, but only such tiles pay it, and the result is
// finite wherever the reference's is (src/lamm_kernel_q8_0.hpp:50-117: any magnitude).
constexpr int kDqNonFinite = 0x207;          // +-inf, NaN (v_cmp_class_f32 mask)

// Scale tracking in VGPRs: per lane the largest |d| bits and the smallest nonzero |d| bits seen (the
// packed u16 halves of a {d, d} pair; |d| - 1 wraps a zero to 0xffff): three packed ops per scale.
// bad: an inf / NaN (>= 0x7c00) or a nonzero subnormal (< 0x0400) among them.
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
struct DqRange {
  u16x2 hi = {0, 0}, lo = {0xffff, 0xffff};
  __device__ __forceinline__ void see(uint32_t d2) {
    const u16x2 a = __builtin_bit_cast(u16x2, d2 & 0x7fff7fffu);
    hi = __builtin_elementwise_max(hi, a);
    lo = __builtin_elementwise_min(lo, a - u16x2{1, 1});
  }
  __device__ __forceinline__ bool bad() const { return hi[0] >= 0x7c00 || lo[0] < 0x03ff; }
};

// the 16-bit word at byte offset o (even) of x
__device__ __forceinline__ uint32_t ld16(const unsigned char* x, int o) {
  return *reinterpret_cast<const uint16_t*>(x + o);
}
__device__ __forceinline__ uint32_t ld32(const unsigned char* x, int o) {   // o even
  return ld16(x, o) | (ld16(x, o + 2) << 16);
}

// One weight block as 8 dwords of signed int8 values (q - c), d and m (0 unless affine)
template <int T>
__device__ __forceinline__ void exact_a(const unsigned char* a, uint32_t (&q)[8], float& d, float& m) {
  using F = DqFmt<T>;
  d = h2f(ld16(a, 0));
  m = F::MO >= 0 ? h2f(ld16(a, F::MO >= 0 ? F::MO : 0)) : 0.f;
  if constexpr (!F::NIB) {
#pragma unroll
    for (int w = 0; w < 8; ++w) q[w] = ld32(a, F::QS + 4 * w);
  } else {
    const uint32_t qh = F::QH >= 0 ? ld32(a, F::QH >= 0 ? F::QH : 0) : 0u;
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      const uint32_t x = ld32(a, F::QS + 4 * w);
      uint32_t lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
      if constexpr (F::QH >= 0) {
        lo |= spread4_hi((qh >> (4 * w)) & 0xfu);
        hi |= spread4_hi((qh >> (16 + 4 * w)) & 0xfu);
      }
      // bytes u in [0, 31] -> u - c as signed bytes (no borrow crosses a byte: u + 128 - c >= 0)
      constexpr uint32_t cc = 0x01010101u * (uint32_t)F::C;
      q[w] = ((lo | 0x80808080u) - cc) ^ 0x80808080u;
      q[4 + w] = ((hi | 0x80808080u) - cc) ^ 0x80808080u;
    }
  }
}

// The tile [i0, i0 + arows) x [j0, j0 + bcols) with exact int8 block dots, every block in order:
// per block the 64 activation blocks are staged in LDS (int8 quads, d, s), then each thread
// accumulates its weight row against its columns.  NT threads, NT / DQ_TI columns each step.
template <int T, int V, int NT>
__device__ void dq_exact_tile(const unsigned char* A, int64_t lda, const unsigned char* B, int64_t ldb, float* C,
                              int64_t ldc, int arows, int bcols, int nblk, unsigned char* smem) {
  using FA = DqFmt<T>;
  using FB = DqFmt<V>;
  constexpr int CJ = NT / DQ_TI, NJ = DQ_TJ / CJ;
  static_assert(NT % DQ_TI == 0 && DQ_TJ % CJ == 0, "tile split");
  uint32_t* bq = reinterpret_cast<uint32_t*>(smem);    // [64][8] int8 quads
  float* bd = reinterpret_cast<float*>(bq + DQ_TJ * 8);   // [64] d, then [64] s
  const int t = threadIdx.x, i = t % DQ_TI, jc = t / DQ_TI;
  float acc[NJ];
#pragma unroll
  for (int k = 0; k < NJ; ++k) acc[k] = 0.f;
  for (int b = 0; b < nblk; ++b) {
    __syncthreads();   // the previous block's LDS reads are done
    if (t < DQ_TJ) {
      uint32_t w[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      float d = 0.f, sb = 0.f;
      if (t < bcols) {
        const unsigned char* x = B + (int64_t)t * ldb + (int64_t)b * FB::BPB;
        d = h2f(ld16(x, 0));
        if constexpr (FB::QS == 4) sb = h2f(ld16(x, 2));
#pragma unroll
        for (int k = 0; k < 8; ++k) w[k] = ld32(x, FB::QS + 4 * k);
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) bq[t * 8 + k] = w[k];
      bd[t] = d;
      bd[DQ_TJ + t] = sb;
    }
    __syncthreads();
    if (i < arows) {
      uint32_t qa[8];
      float da, ma;
      exact_a<T>(A + (int64_t)i * lda + (int64_t)b * FA::BPB, qa, da, ma);
#pragma unroll
      for (int k = 0; k < NJ; ++k) {
        const int j = jc + CJ * k;
        int sumi = 0;
#pragma unroll
        for (int w = 0; w < 8; ++w) sumi = dot4(qa[w], bq[j * 8 + w], sumi);
        acc[k] += da * bd[j] * (float)sumi;
        if constexpr (FA::MO >= 0) acc[k] += ma * bd[DQ_TJ + j];
      }
    }
  }
  if (i < arows)
#pragma unroll
    for (int k = 0; k < NJ; ++k) {
      const int j = jc + CJ * k;
      if (j < bcols) C[(int64_t)j * ldc + i] = acc[k];
    }
}

// load_words' vector-memory instructions for NW dwords (b128s, then b64 / b32)
[[maybe_unused]] constexpr int vm_ops(int nw) { return nw / 4 + (nw % 4 >= 2 ? 1 : 0) + (nw % 2 ? 1 : 0); }

__device__ __forceinline__ uint32_t perm(uint32_t s0, uint32_t s1, uint32_t sel) {
  return __builtin_amdgcn_perm(s0, s1, sel);
}

template <int N_>
__device__ __forceinline__ void wait_vm() {   // s_waitcnt vmcnt(N) (lgkmcnt untouched)
  static_assert(N_ >= 0 && N_ < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N_ & 0xF) | ((N_ >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// {x, x} for the 16-bit field at byte offset O (even) of a register-resident byte string
template <int O, int NW>
__device__ __forceinline__ uint32_t splat16(const uint32_t (&w)[NW]) {
  constexpr uint32_t b = O & 3;
  return perm(0u, w[O >> 2], b | ((b + 1) << 8) | (b << 16) | ((b + 1) << 24));
}

// the 32-bit field at byte offset O (even) of a register-resident byte string
template <int O, int NW>
__device__ __forceinline__ uint32_t field32(const uint32_t (&w)[NW]) {
  if constexpr ((O & 3) == 0) return w[O >> 2];
  else return __builtin_amdgcn_alignbit(w[(O >> 2) + 1], w[O >> 2], 16);
}

// One operand of a k-step: element group c (elements 8c .. 8c + 7) of block JB of the pair in w,
// as 8 f16 values d (u - C) [+ m].  d2 / m2: {d, d} / {m, m} (f16 bits, already pre-scaled).
template <int T, int JB, int CG, int NW>
__device__ __forceinline__ half8 dq_operand(const uint32_t (&w)[NW], uint32_t d2, uint32_t m2, uint32_t qh) {
  using F = DqFmt<T>;
  constexpr int QS0 = JB * F::BPB + F::QS;   // window byte of this block's qs[0]
  uint32_t o[4];
  unroll<4>([&](auto P) {
    constexpr int p = P;
    constexpr int bq = F::NIB ? 8 * (CG % 2) + 2 * p : 8 * CG + 2 * p;   // qs byte of the pair
    constexpr int a = QS0 + bq;                                           // its window byte
    constexpr int k = a >> 2;
    uint32_t src;
    if constexpr (F::NIB) {
      src = CG < 2 ? (w[k] & 0x0f0f0f0fu) : ((w[k] >> 4) & 0x0f0f0f0fu);
      if constexpr (F::QH >= 0) {   // the 5th bits of the dword's elements (bytes 4k .. 4k + 3)
        constexpr int e0 = 4 * k - QS0 + (CG < 2 ? 0 : 16);   // element of byte 0 of the dword
        const uint32_t bits = e0 >= 0 ? (qh >> (e0 >= 0 ? e0 : 0)) : (qh << (e0 < 0 ? -e0 : 0));
        src |= spread4_hi(bits & 0xfu);
      }
    } else {
      src = w[k] ^ 0x80808080u;
    }
    o[p] = perm(0x64646464u, src, (a & 2) ? 0x04030402u : 0x04010400u);   // {1024 + u, 1024 + u'}
  });
  half8 r;
  const h2 d = __builtin_bit_cast(h2, d2);
  constexpr _Float16 off = (_Float16)(-(1024 + F::C));
  unroll<4>([&](auto P) {
    constexpr int p = P;
    const h2 u = __builtin_bit_cast(h2, o[p]) + h2{off, off};
    h2 v;
    if constexpr (F::MO >= 0) v = __builtin_elementwise_fma(u, d, __builtin_bit_cast(h2, m2));
    else v = u * d;
    r[2 * p] = v[0];
    r[2 * p + 1] = v[1];
  });
  return r;
}

// per-block scalars of block JB of the pair in w: {d, d} (x scale), {m, m} (x scale), qh
template <int T, int JB, int NW>
__device__ __forceinline__ void dq_scalars(const uint32_t (&w)[NW], bool valid, _Float16 scale, uint32_t& d2,
                                           uint32_t& m2, uint32_t& qh) {
  using F = DqFmt<T>;
  constexpr int O = JB * F::BPB;
  const h2 sc = {scale, scale};
  h2 d = __builtin_bit_cast(h2, splat16<O>(w));
  if (scale != (_Float16)1) d = d * sc;
  d2 = valid ? __builtin_bit_cast(uint32_t, d) : 0u;
  m2 = 0;
  if constexpr (F::MO >= 0) {
    h2 m = __builtin_bit_cast(h2, splat16<O + F::MO>(w));
    if (scale != (_Float16)1) m = m * sc;
    m2 = valid ? __builtin_bit_cast(uint32_t, m) : 0u;
  }
  qh = 0;
  if constexpr (F::QH >= 0) qh = field32<O + F::QH>(w);
}

// ---------------------------------------------------------------- LDS-staged form (v2)
// The same unpacking and MFMA steps, but each wave's quad arrives by COALESCED loads: consecutive
// lanes take consecutive 8-byte pieces of a row's (column's) quad -- 9 pieces of a q4_0 row, 17 of a
// q8_0 column -- so one load instruction touches ~8 rows' contiguous bytes instead of 64 rows'
// scattered windows (v1: one row per lane, every lane its own cache lines).  The pieces go to the
// wave's private LDS image of the quad (rows at a 4*BPB-byte pitch: the lanes' pair windows read
// back conflict-free, 18r + 9h / 34c + 17h dwords), and the NEXT quads are already in flight in
// VGPRs while this one is unpacked and multiplied.
template <int T, int V, int NBV, int WH>
__global__ __launch_bounds__(DQ_NT * WH) void gemm_dq2_kernel(GemvArgs p) {
  // WH waves per K-group, each owning 128 / WH of the tile's weight rows (2: two waves per SIMD, the
  // activation quad unpacked by both)
  constexpr int NT = DQ_NT * WH, TIW = DQ_TI / WH, YW = 4 / WH;
  using FA = DqFmt<T>;
  using FB = DqFmt<V>;
  constexpr int NWA = FA::BPB / 2, NWB = FB::BPB / 2;
  constexpr int QA = 4 * FA::BPB, QB = 4 * FB::BPB;   // bytes of a row's / a column's quad
  constexpr int PA = QA / 8, PB = QB / 8;             // its 8-byte pieces
  constexpr int LA = TIW * PA / 64, LB = DQ_TJ * PB / 64;   // piece loads per lane per quad
  static_assert((TIW * PA) % 64 == 0 && (DQ_TJ * PB) % 64 == 0, "whole loads");
  constexpr int QBYTES = 8 * 64 * (LA + LB);          // a wave's LDS image of one quad
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int t = threadIdx.x, lane = t & 63, lr = lane & 31, h = lane >> 5;
  const int wid = __builtin_amdgcn_readfirstlane(t >> 6), g = wid / WH, mh = wid % WH;
  const int nsi = (p.M + DQ_TI - 1) / DQ_TI, nsj = (p.N + DQ_TJ - 1) / DQ_TJ;
  int ti, tj, z;
  {   // XCD-aware order (gemm_dq_kernel)
    const int ntile = nsi * nsj * p.ne12 * p.ne13;
    const int id = blockIdx.x, x = id & 7, k = id >> 3, q = ntile >> 3, rmd = ntile & 7;
    const int wv = x < rmd ? x * (q + 1) + k : rmd * (q + 1) + (x - rmd) * q + k;
    const int per = nsi * nsj;
    z = wv / per;
    ti = (wv % per) / nsj;
    tj = (wv % per) % nsj;
  }
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const int i02 = i12 / p.r2, i03 = i13 / p.r3;
  const int64_t i0 = (int64_t)ti * DQ_TI, j0 = (int64_t)tj * DQ_TJ;
  const int64_t arows = min((int64_t)DQ_TI, (int64_t)p.M - i0), bcols = min((int64_t)DQ_TJ, (int64_t)p.N - j0);
  const auto ra = make_rsrc(p.A + (int64_t)i02 * p.sa2 + (int64_t)i03 * p.sa3 + i0 * p.lda,
                            (uint32_t)min(arows * p.lda, (int64_t)0x7fffffff));
  const auto rb = make_rsrc(p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3 + j0 * p.ldb,
                            (uint32_t)min(bcols * p.ldb, (int64_t)0x7fffffff));
  const int nblk = p.nblk;   // (no lambda captures p, see gemm_dq_kernel)
  const int nq = (nblk + 3) / 4;
  const int mine = nq > g ? (nq - g + DQ_KG - 1) / DQ_KG : 0;
  // this lane's pieces: load i covers piece i * 64 + lane -> (row, piece in row)
  uint32_t a_off[LA], b_off[LB];
  {
    const uint32_t lda = (uint32_t)p.lda, ldb = (uint32_t)p.ldb;
#pragma unroll
    for (int i = 0; i < LA; ++i) {
      const int pc = i * 64 + lane;
      a_off[i] = (uint32_t)(mh * TIW + pc / PA) * lda + (uint32_t)(pc % PA) * 8;
    }
#pragma unroll
    for (int i = 0; i < LB; ++i) {
      const int pc = i * 64 + lane;
      b_off[i] = (uint32_t)(pc / PB) * ldb + (uint32_t)(pc % PB) * 8;
    }
  }
  unsigned char* img = smem + wid * QBYTES;   // rows [TIW][QA], then columns [64][QB]
  u32x2 st[NBV][LA + LB];
  auto issue = [&](int u, auto S_) __attribute__((always_inline)) {
    constexpr int S = decltype(S_)::value;
    const int q = g + DQ_KG * min(u, mine - 1);
    const uint32_t qa = (uint32_t)q * QA, qb = (uint32_t)q * QB;
#pragma unroll
    for (int i = 0; i < LA; ++i) st[S][i] = __builtin_amdgcn_raw_buffer_load_b64(ra, a_off[i] + qa, 0, 0);
#pragma unroll
    for (int i = 0; i < LB; ++i) st[S][LA + i] = __builtin_amdgcn_raw_buffer_load_b64(rb, b_off[i] + qb, 0, 0);
  };
  auto stage = [&](auto S_) __attribute__((always_inline)) {   // the landed pieces into the image
    constexpr int S = decltype(S_)::value;
#pragma unroll
    for (int i = 0; i < LA + LB; ++i) *reinterpret_cast<u32x2*>(img + 8 * (i * 64 + lane)) = st[S][i];
  };

  f32x16 acc[2][YW];
  unroll<2>([&](auto X) __attribute__((always_inline)) { unroll<YW>([&](auto Y) __attribute__((always_inline)) { acc[X][Y] = f32x16{}; }); });

  DqRange range;   // the range guard: the scales this lane unpacked
  auto quad = [&](int u) __attribute__((always_inline)) {
    const int q = g + DQ_KG * u;
    uint32_t wa[YW][NWA], wb[2][NWB];   // this lane's pair windows, from the image
#pragma unroll
    for (int y = 0; y < YW; ++y) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(img + (32 * y + lr) * QA + h * 2 * FA::BPB);
#pragma unroll
      for (int k = 0; k < NWA; ++k) wa[y][k] = src[k];
    }
#pragma unroll
    for (int x = 0; x < 2; ++x) {
      const uint32_t* src = reinterpret_cast<const uint32_t*>(img + TIW * QA + (32 * x + lr) * QB + h * 2 * FB::BPB);
#pragma unroll
      for (int k = 0; k < NWB; ++k) wb[x][k] = src[k];
    }
    if constexpr (DQ_AB == 1) {
#pragma unroll
      for (int y = 0; y < YW; ++y)
#pragma unroll
        for (int i = 0; i < NWA; ++i) asm volatile("" ::"v"(wa[y][i]));
#pragma unroll
      for (int x = 0; x < 2; ++x)
#pragma unroll
        for (int i = 0; i < NWB; ++i) asm volatile("" ::"v"(wb[x][i]));
      return;
    }
    unroll<2>([&](auto JB_) __attribute__((always_inline)) {
      constexpr int JB = JB_;
      const bool valid = 4 * q + 2 * h + JB < nblk;
      uint32_t ad[YW], am[YW], aq[YW], bd[2], bm[2], bq[2];
      unroll<YW>([&](auto Y) __attribute__((always_inline)) { dq_scalars<T, JB>(wa[Y], valid, (_Float16)DQ_ASCALE, ad[Y], am[Y], aq[Y]); });
      unroll<2>([&](auto X) __attribute__((always_inline)) { dq_scalars<V, JB>(wb[X], valid, (_Float16)DQ_BSCALE, bd[X], bm[X], bq[X]); });
      unroll<YW>([&](auto Y) __attribute__((always_inline)) {
        range.see(ad[Y]);
        if constexpr (FA::MO >= 0) range.see(am[Y]);
      });
      unroll<2>([&](auto X) __attribute__((always_inline)) { range.see(bd[X]); });
      unroll<4>([&](auto CG_) __attribute__((always_inline)) {
        constexpr int CG = CG_;
        half8 bo[2];
        unroll<2>([&](auto X) __attribute__((always_inline)) { bo[X] = dq_operand<V, JB, CG>(wb[X], bd[X], 0u, 0u); });
        unroll<YW>([&](auto Y) __attribute__((always_inline)) {
          const half8 ao = dq_operand<T, JB, CG>(wa[Y], ad[Y], am[Y], aq[Y]);
          unroll<2>([&](auto X) __attribute__((always_inline)) { acc[X][Y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(bo[X], ao, acc[X][Y], 0, 0, 0); });
        });
      });
    });
  };

  constexpr int LPQ = LA + LB;
  if constexpr (DQ_AB == 2) {   // probe: unpack + MFMA only, on the first quad's image (no loads after it)
    if (mine > 0) {
      issue(0, std::integral_constant<int, 0>{});
      wait_vm<0>();
      stage(std::integral_constant<int, 0>{});
      for (int u = 0; u < mine; ++u) {
        asm volatile("" ::: "memory");
        quad(u);
      }
    }
  } else if (mine > 0) {
    unroll<NBV>([&](auto K) __attribute__((always_inline)) { issue(K, K); });
    int u0 = 0;
    for (; u0 + NBV <= mine; u0 += NBV) {
      unroll<NBV>([&](auto K) __attribute__((always_inline)) {
        wait_vm<LPQ * (NBV - 1)>();   // quad u0 + k's pieces landed
        stage(K);
        issue(u0 + K + NBV, K);
        quad(u0 + K);
      });
    }
    unroll<NBV>([&](auto K) __attribute__((always_inline)) {
      if (u0 + (int)K < mine) {
        wait_vm<LPQ * (NBV - 1)>();
        stage(K);
        issue(u0 + K + NBV, K);
        quad(u0 + K);
      }
    });
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  // range guard: any bad scale or non-finite accumulator in any wave -> the exact tile
  bool bad = range.bad();
  unroll<2>([&](auto X) __attribute__((always_inline)) {
    unroll<YW>([&](auto Y) __attribute__((always_inline)) {
      unroll<16>([&](auto E) __attribute__((always_inline)) { constexpr int e = E; bad |= __builtin_amdgcn_class(acc[X][Y][e], kDqNonFinite); });
    });
  });
  __shared__ int wave_bad[NT / 64];
  if (lane == 0) wave_bad[wid] = 0;
  __syncthreads();   // every wave past its last image read: the partial tiles reuse the LDS
  if (bad) wave_bad[wid] = 1;   // (any lane; the same value)
  __syncthreads();
  int any_bad = 0;
#pragma unroll
  for (int w = 0; w < NT / 64; ++w) any_bad |= wave_bad[w];
  if (any_bad) {
    dq_exact_tile<T, V, NT>(p.A + (int64_t)i02 * p.sa2 + (int64_t)i03 * p.sa3 + i0 * p.lda, p.lda,
                            p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3 + j0 * p.ldb, p.ldb,
                            p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3 + j0 * p.ldc + i0, p.ldc, (int)arows,
                            (int)bcols, nblk, smem);
    return;
  }
  float* red = reinterpret_cast<float*>(smem);
  unroll<2>([&](auto X) __attribute__((always_inline)) {
    unroll<YW>([&](auto Y) __attribute__((always_inline)) {
      unroll<16>([&](auto E) __attribute__((always_inline)) {
        constexpr int e = E;
        const int j = 32 * X + (e & 3) + 8 * (e >> 2) + 4 * h, i = TIW * mh + 32 * Y + lr;
        red[(g * DQ_TJ + j) * DQ_PI + i] = acc[X][Y][e];
      });
    });
  });
  __syncthreads();
  float* C = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const bool pair = (p.ldc & 1) == 0 && ((uintptr_t)C & 7) == 0;
#pragma unroll
  for (int r = 0; r < DQ_TJ * DQ_TI / (2 * NT); ++r) {
    const int idx = 2 * (r * NT + t), jl = idx / DQ_TI, il = idx % DQ_TI;
    f32x2 v = *reinterpret_cast<const f32x2*>(&red[jl * DQ_PI + il]);
#pragma unroll
    for (int g_ = 1; g_ < DQ_KG; ++g_) v += *reinterpret_cast<const f32x2*>(&red[(g_ * DQ_TJ + jl) * DQ_PI + il]);
    v *= DQ_CSCALE;
    const int64_t j = j0 + jl, i = i0 + il;
    if (j < p.N) {
      float* c = C + j * p.ldc + i;
      if (pair && i + 1 < p.M) {
        __builtin_nontemporal_store(v, reinterpret_cast<f32x2*>(c));
      } else {
        if (i < p.M) c[0] = v[0];
        if (i + 1 < p.M) c[1] = v[1];
      }
    }
  }
}

template <int T, int V, int WH>
constexpr size_t dq2_lds() {
  constexpr size_t img =
      (size_t)8 * DQ_KG * WH * (DQ_TI / WH * (4 * DqFmt<T>::BPB / 8) + DQ_TJ * (4 * DqFmt<V>::BPB / 8));
  return img > DQ_LDS ? img : DQ_LDS;
}

#ifndef DQ_WH
#define DQ_WH 1     // waves per K-group (2: two waves per SIMD; measured no faster, profiles/r04/dq16/)
#endif
#ifndef DQ_NBV
#define DQ_NBV 1    // quads in flight in VGPRs
#endif

template <int T, int V>
hipError_t launch_dq_t(const GemvArgs& p, hipStream_t s) {
  const int tiles = gemm_dq_tiles(p);
  auto kern = gemm_dq2_kernel<T, V, DQ_NBV, DQ_WH>;
  constexpr size_t lds = dq2_lds<T, V, DQ_WH>();
  static_assert(lds <= 160 * 1024, "LDS");
  set_max_lds((const void*)kern, (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)tiles), dim3(DQ_NT * DQ_WH), lds, s, p);
  return hipGetLastError();
}

}  // namespace

int gemm_dq_tiles(const GemvArgs& p) {
  return ((p.M + DQ_TI - 1) / DQ_TI) * ((p.N + DQ_TJ - 1) / DQ_TJ) * p.ne12 * p.ne13;
}

bool gemm_dq_supported(int type) {
  return type == kQ4_0 || type == kQ4_1 || type == kQ5_0 || type == kQ5_1 || type == kQ8_0;
}

// B rows must be 4-byte aligned (pair windows are read as dwords): every q8_0 / q8_1 row pitch is
// a whole number of pairs only when even, so check the pitch, the base and the slice strides
bool gemm_dq_args_ok(const GemvArgs& p) {
  return ((uintptr_t)p.B & 3) == 0 && (p.ldb & 3) == 0 && (p.sb2 & 3) == 0 && (p.sb3 & 3) == 0 && !p.b_f32 &&
         (int64_t)DQ_TI * p.lda < 0x7fffffff && (int64_t)DQ_TJ * p.ldb < 0x7fffffff;
}

size_t gemm_dq_workspace_bytes(const GemvArgs&) { return 0; }

hipError_t launch_gemm_dq(int type, const GemvArgs& p, void*, hipStream_t s) {
  switch (type) {
    case kQ4_0: return launch_dq_t<kQ4_0, kQ8_0>(p, s);
    case kQ4_1: return launch_dq_t<kQ4_1, kQ8_1>(p, s);
    case kQ5_0: return launch_dq_t<kQ5_0, kQ8_0>(p, s);
    case kQ5_1: return launch_dq_t<kQ5_1, kQ8_1>(p, s);
    case kQ8_0: return launch_dq_t<kQ8_0, kQ8_0>(p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
