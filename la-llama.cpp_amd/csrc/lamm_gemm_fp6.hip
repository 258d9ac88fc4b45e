// lamm_gemm_fp6.hip -- prefill GEMM (N > 8) for q4_0 / q4_1 / q5_0 weights whose block dots
// run on gfx950's block-scaled f8f6f4 matrix path with EXACT integer operands.
//
// Contract: the lamm block kernels (src/lamm_kernel_q4_0.hpp:59-128, q4_1 :46-116,
// q5_0 :69-139, via LAMMImpl<T>::matmul_simd_block, src/lamm_impl.hpp:90-147):
//   C[j*ldc + i] = sum_blocks d_a*d_b*S (+ m_a*s_b),   S = exact int32 block dot.
//
// Why fp6.  Every 32-element block needs its own fp32 scale d_a*d_b, so each int32 block
// dot costs the VALU a convert and an FMA per output element; on gfx950 that epilogue, not
// the matrix core, bounds an i8 GEMM (tools/mfma_probe.hip, profiles/r01/mfma_probe.txt:
// i8 S + cvt + fma 57 ns per 32x32 block per SIMD vs 37-40 ns for fp6 S + fma).  The quants
// are small integers, and e2m3 (fp6) encodes n/8 EXACTLY as sign|n for |n| <= 16
// (subnormals 0..7/8, then 1.0..1.875, then 2.0), so with E8M0 block scales the fp6 MFMA
// computes the same integer S as an i8 MFMA -- bit for bit, in fp32 (|S| < 2^24) -- and
// hands it to the epilogue already as a float:
//   weight quant  n = q-8 (q4_0), q (q4_1), q-16 (q5_0)        -> code sign|n,  scale 2^3
//   activation    b = 16*h + l,  h = b>>4 in [-8,7], l = b&15    -> hi code sign|h, scale 2^7
//                                                                    lo code l,      scale 2^3
// One v_mfma_scale_f32_32x32x64_f8f6f4 per block: k-group 0 = (hi x n), k-group 1 = (lo x n),
// i.e. S = sum n*(16h + l) = sum n*b.  Its C/D layout is the 32x32 one of every gfx950 MFMA
// (lane map verified: tools/mfma_probe.hip layout check, "k = 32h + e").
//
// Two passes per call:
//   prep_w_fp6 / prep_b_fp6 : AoS block_q* -> MFMA-ready tiles in a workspace, laid out as the
//       GEMM's LDS image so each K-step's tile moves with plain LDS-DMA (buffer_load ... lds)
//       and every fragment is two conflict-free ds_read_b128;
//   gemm_fp6_kernel : 256(i) x 128(j) tile per workgroup, 8 waves = 2(j) x 4(i), a wave owns
//       64(j) x 64(i) = 2 x 2 tiles of 32x32.  Per block and tile ("unit"): fp6 S-MFMA, f16
//       P-MFMA (P = 2 d_b d_a, exact) and 16 FMAs acc += S*P; unit n+1's MFMAs are issued
//       before unit n's FMAs so the matrix core and the VALU overlap.  q4_1: sum m_a*s_b is
//       one rank-2 f16 MFMA per K-step.
// Ragged M / N / K are zero-padded by the prep passes, so the main loop has no bounds checks.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>

#include "lamm_device.h"
#include "lamm_kernels.h"
#include "lamm_knobs.h"
#include "lamm_rowdot.h"

namespace lamm {
namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

#ifndef F6_KB_CFG
#define F6_KB_CFG 2
#endif
#ifndef F6_NBUF_CFG
#define F6_NBUF_CFG 4
#endif
constexpr int F6_KB = F6_KB_CFG;   // 32-element blocks per K-step (4 with 2 stages: A/B builds)
constexpr int F6_TI = 256;      // weight rows per tile
constexpr int F6_TJ = 128;      // activation rows per tile
constexpr int F6_PIECE = 1024;  // bytes one wave moves per LDS-DMA instruction (64 lanes x 16 B)
constexpr int F6_NBUF = F6_NBUF_CFG;   // LDS stages (3 K-steps of DMA in flight)
constexpr int SCALE_W = 130, SCALE_HI = 134, SCALE_LO = 130;   // E8M0: 2^(s-127)
#ifndef F6_C_NT
// The K-group epilogue's C stores are non-temporal: C is written once and not re-read by this
// launch, so streaming it past L2 leaves the end-of-launch L2 write-back nothing of it to flush
// (config 3, one slice: whole launch 36.2 -> 35.1 us on one box, profiles/r02/ab_c_nt/).
// 0: cached stores (A/B build, tools/ab_c_nt.sh).
#define F6_C_NT 1
#endif
#ifndef F6_CT_NT
// The whole-tile (KG = 1) epilogue's C / split-K partial stores are non-temporal too (config 3,
// four slices: 93.0 -> 89.7 us whole launch, mean of 3 alternating pairs on one box,
// profiles/r02/ab_c_nt/ab_ct_nt.txt).  0: cached stores (A/B build, tools/ab_ct_nt.sh).
#define F6_CT_NT 1
#endif
#ifndef F6_KV_ORDER
#define F6_KV_ORDER 0   // gemm_fp6_kv_kernel's issue order per unit (probe builds only, see block())
#endif
#ifndef F6_PD
#define F6_PD 1   // MFMA pipeline depth: unit n+PD's MFMAs are issued before unit n's FMAs (2: no gain, +20 VGPRs)
#endif

template <int T> struct F6;
// SH16 (q5_1): the quant q in [0, 31] is coded as n = q - 16 (|n| <= 16, exact in e2m3) and the
// block's affine term carries the shift back: d q + m = d n + (m + 16 d).  The reference multiplies
// d_a d_b sum q b, so the shift's share is 16 d_a (d_b sum q_b) -- the activation block's fp16 s_b
// is that product ROUNDED (and from ggml's fp32 d), off by up to ~2^-10 of s_b, which at small K with
// activations that do not cancel reached 1.1e-3 of sum |a b|.  So the activation prep
// also stores the residual r_b = d_b sum q_b - s_b (exact in fp32, kept as fp16 -- its own rounding is
// ~2^-11 of a residual that is ~2^-11 of s_b) and the m * s MFMA adds, per block,
//   2 m_a s_b + 32 d_a s_b + 32 d_a r_b = 2 (m_a s_b + 16 d_a d_b sum q_b)
// over its eight k slots (lanes 0-31: {2 m_a, 32 d_a} x {s_b, s_b}, lanes 32-63: {32 d_a} x {r_b}; the
// x2 matches the P-MFMA's 2 d_a d_b), each product f16 x f16 exact in fp32.  32 d_a and 2 m_a are
// exact in f16 for |d_a| <= 2047 and |m_a| <= 32752: prepare_fp6_weights reports a weight outside
// that range, which then stays on the range-guarded dq16 engine.
// WP: weight code planes per block.  q8_0 (round 6): its quants q in [-127, 127] do not
// fit e2m3, so the weight is split like the activations, q = 16 h + l (h = q >> 4 in [-8, 7], l = q & 15),
// into a hi and a lo code plane; the S of a unit is then two chained scale MFMAs, the hi one with its
// weight scale x16 (E8M0 +4) accumulating into the lo one -- S = sum (16 h + l) b, every partial an
// integer below 2^24, exact in fp32.  Only the 128 x 64 K-group plan (gemm_fp6_kv_kernel) takes it, and
// only with prepared weights; other q8_0 calls stay on dq16.
template <> struct F6<kQ4_0> { static constexpr int ABPB = 18, VBPB = 34, WP = 1; static constexpr bool AFF = false, SH16 = false; };
template <> struct F6<kQ4_1> { static constexpr int ABPB = 20, VBPB = 36, WP = 1; static constexpr bool AFF = true, SH16 = false; };
template <> struct F6<kQ5_0> { static constexpr int ABPB = 22, VBPB = 34, WP = 1; static constexpr bool AFF = false, SH16 = false; };
template <> struct F6<kQ5_1> { static constexpr int ABPB = 24, VBPB = 36, WP = 1; static constexpr bool AFF = true, SH16 = true; };
template <> struct F6<kQ8_0> { static constexpr int ABPB = 34, VBPB = 34, WP = 2; static constexpr bool AFF = false, SH16 = false; };
static_assert(F6_KB == 2, "q5_1's shift term uses the m * s MFMA's k slots 2..3");
static_assert(!F6<kQ4_0>::SH16 && !F6<kQ4_1>::SH16 && !F6<kQ5_0>::SH16 && !F6<kQ8_0>::SH16, "only q5_1 shifts its quants");

// 16 * h for an f16 bit pattern h (exact below 4096); the f16 bits of the result
__device__ __forceinline__ uint32_t f16_times16(uint32_t h) {
  const _Float16 v = __builtin_bit_cast(_Float16, (uint16_t)(h & 0xffffu));
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(v * (_Float16)16.0f));
}

__device__ __forceinline__ uint32_t f16_times2(uint32_t h) {   // 2 * h (exact below 32768)
  const _Float16 v = __builtin_bit_cast(_Float16, (uint16_t)(h & 0xffffu));
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)(v * (_Float16)2.0f));
}

// q8_1 activation blocks (d, s fp16 bits, the 32 int8 quants as 8 dwords): the fp16 bits of the residual
// r = d * sum q - s (SH16 above), 0 when s or the product is not finite (the term then falls back to
// 16 d_a s_b, as the reference's own s overflows there)
__device__ __forceinline__ uint32_t s_residual(uint32_t dbits, uint32_t sbits, const uint32_t (&q)[8]) {
  int sum = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) sum = __builtin_amdgcn_sdot4((int)q[k], 0x01010101, sum, false);
  const float e = h2f(dbits & 0xffffu) * (float)sum;   // 11 x 12 significant bits: exact
  const float r = e - h2f(sbits & 0xffffu);             // within a factor 2 of each other: exact
  if (!__builtin_isfinite(r)) return 0u;
  return (uint32_t)__builtin_bit_cast(uint16_t, (_Float16)r);
}

// A fragment = 8 dwords = two 16-byte planes: p0 = fp6 code dwords 0-3,
// p1 = {code dwords 4-5, scale dword ({d, 0} fp16 pair), m (q4_1) / s (q8_1) fp16 or 0; q8_1 B planes
// carry s's residual r (SH16) in the upper half of that last dword}.
// Chunk = one K-step of one tile, exactly the GEMM's LDS image:
//   A chunk: [p 2][b KB][r TI] x 16 B            B chunk: [p 2][b KB][h 2][r TJ] x 16 B
// (h = k-group: 0 = hi codes, 1 = lo codes; both copies carry d_b and s_b)
constexpr int F6_A_BYTES = 2 * F6_KB * F6_TI * 16;
constexpr int F6_B_BYTES = 2 * F6_KB * 2 * F6_TJ * 16;

// byte offset of plane p (16 bytes) of the fragment of (block b, [k-group h,] row r).  Planes
// are separate arrays, so the 32 lanes of a half-wave read 512 contiguous bytes per plane:
// conflict-free ds_read_b128 (a 32-byte-per-lane image costs a 2-way conflict on every read,
// measured +20 % kernel time).
__host__ __device__ constexpr int f6_aoff(int p, int b, int r) { return ((p * F6_KB + b) * F6_TI + r) * 16; }
__host__ __device__ constexpr int f6_boff(int p, int b, int h, int r) {
  return (((p * F6_KB + b) * 2 + h) * F6_TJ + r) * 16;
}

struct F6Layout {
  int nsteps, nit, njt, na;
  int64_t a_slice, b_slice, a_bytes;
  // wp: weight code planes (F6<T>::WP): a K-step's A chunk is wp x F6_A_BYTES (q8_0: hi then lo)
  __host__ __device__ static F6Layout of(const GemvArgs& p, int wp = 1) {
    F6Layout L;
    L.nsteps = (p.nblk + F6_KB - 1) / F6_KB;
    L.nit = (p.M + F6_TI - 1) / F6_TI;
    L.njt = (p.N + F6_TJ - 1) / F6_TJ;
    L.na = (p.ne12 / p.r2) * (p.ne13 / p.r3);
    L.a_slice = (int64_t)L.nit * L.nsteps * F6_A_BYTES * wp;
    L.b_slice = (int64_t)L.njt * L.nsteps * F6_B_BYTES;
    L.a_bytes = (int64_t)L.na * L.a_slice;
    return L;
  }
};

// 32 six-bit codes -> the 192-bit fragment (code e at bit 6e)
__device__ __forceinline__ void pack_fp6(const uint32_t (&c)[32], uint32_t (&o)[6]) {
#pragma unroll
  for (int k = 0; k < 6; ++k) o[k] = 0;
#pragma unroll
  for (int e = 0; e < 32; ++e) {
    const int bit = 6 * e, w = bit >> 5, sh = bit & 31;
    o[w] |= c[e] << sh;
    if (sh > 26) o[w + 1] |= c[e] >> (32 - sh);
  }
}

__device__ __forceinline__ uint32_t sm_code(int n) {   // e2m3 code of n/8, |n| <= 16
  return n < 0 ? (32u | (uint32_t)(-n)) : (uint32_t)n;
}

// Read a block starting at (2-byte aligned) byte offset `off` of a buffer into dwords.
template <int NW>
__device__ __forceinline__ void load_block(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t (&m)[NW]) {
  const uint32_t base = off & ~3u;
  const int sh = (int)(off & 3u) * 8;
  uint32_t w[NW + 1];
  load_words<NW + 1, 0>(r, base, w);   // wide loads (b128 / b64 / b32) from the dword below
#pragma unroll
  for (int k = 0; k < NW; ++k) m[k] = __builtin_amdgcn_alignbit(w[k + 1], w[k], sh);
}

// Each prep thread streams PREP_NB consecutive blocks of ONE row (its loads walk the row's
// bytes in order, so cache lines are used whole) and writes them to the K-step chunks;
// across a wave the rows are consecutive, so every 16-byte plane store is coalesced.
constexpr int PREP_NB = 4;
constexpr int PREP_NT = 256;   // rows per prep workgroup

// ---------------------------------------------------------------- weight prep
// A workgroup converts 64 rows x 16 blocks: the rows' raw AoS bytes are first staged in LDS
// with coalesced 16-byte loads (a row's 16 blocks are 288/320/352 contiguous, 16-byte aligned
// bytes), then each thread converts 4 (row, block) items; lanes own consecutive rows, so the
// 16-byte plane stores of a wave are contiguous.
constexpr int PW_ROWS = 64, PW_NB = 16, PW_NT = 256;

template <int T>
__global__ __launch_bounds__(PW_NT) void prep_w_fp6(GemvArgs p, unsigned char* ws, unsigned* big_d) {
  using F = F6<T>;
  constexpr int SEG = PW_NB * F::ABPB;            // bytes per row segment (multiple of 16)
  constexpr int SEGW = SEG / 4 + 1;                // + 1 dword so unaligned block reads stay inside
  __shared__ uint32_t raw[PW_ROWS * SEGW];
  const F6Layout L = F6Layout::of(p, F::WP);
  const int nkg = (L.nsteps * F6_KB + PW_NB - 1) / PW_NB;
  const int64_t i0 = (int64_t)(blockIdx.x / nkg) * PW_ROWS;
  const int kb0 = (blockIdx.x % nkg) * PW_NB;
  const int a = blockIdx.y, ne02 = p.ne12 / p.r2, i02 = a % ne02, i03 = a / ne02;
  // resource based at this workgroup's first row: offsets stay < 2^31 for any slice size
  const unsigned char* Az = p.A + (int64_t)i02 * p.sa2 + (int64_t)i03 * p.sa3 + min(i0, (int64_t)p.M) * p.lda;
  const int64_t nrow = min((int64_t)PW_ROWS, (int64_t)p.M - i0);
  const int64_t abytes = nrow > 0 ? (nrow - 1) * p.lda + (int64_t)p.nblk * F::ABPB : 0;
  const auto rs = make_rsrc(Az, (uint32_t)min((abytes + 15) & ~int64_t(15), (int64_t)0x7fffffff));
  const int t = threadIdx.x;
  constexpr int PIECES = PW_ROWS * SEG / 16;
#pragma unroll
  for (int k = 0; k < (PIECES + PW_NT - 1) / PW_NT; ++k) {
    const int pc = t + k * PW_NT;
    if (pc < PIECES) {
      const int r = pc / (SEG / 16), o = pc % (SEG / 16);
      const int64_t i = i0 + r;
      const uint32_t off = i < p.M ? (uint32_t)((int64_t)r * p.lda + (int64_t)kb0 * F::ABPB + 16 * o) : 0x7ffffff0u;
      const u32x4 v = bload16(rs, off);
#pragma unroll
      for (int q = 0; q < 4; ++q) raw[r * SEGW + 4 * o + q] = v[q];
    }
  }
  __syncthreads();
#pragma unroll 1
  for (int k = 0; k < PW_ROWS * PW_NB / PW_NT; ++k) {
    const int item = t + k * PW_NT, r = item % PW_ROWS, bl = item / PW_ROWS;
    const int64_t i = i0 + r;
    const int kb = kb0 + bl;
    if (i >= (int64_t)L.nit * F6_TI || kb >= L.nsteps * F6_KB) continue;
    uint32_t code[32], code2[32];   // code2: q8_0's lo plane
    uint32_t d = 0, mv = 0;
    if (T == kQ8_0 && i < p.M && kb < p.nblk) {
      uint32_t m[9];
      const int bo = bl * F::ABPB;
      const uint32_t* src = &raw[r * SEGW + (bo >> 2)];
      const int sh = (bo & 3) * 8;
#pragma unroll
      for (int q = 0; q < 9; ++q) m[q] = __builtin_amdgcn_alignbit(src[q + 1], src[q], sh);
      d = m[0] & 0xffffu;
#pragma unroll
      for (int e = 0; e < 32; ++e) {
        const int q = (int)(int8_t)((m[(2 + e) >> 2] >> (8 * ((2 + e) & 3))) & 0xffu);
        code[e] = sm_code(q >> 4);          // h = floor(q / 16) in [-8, 7]
        code2[e] = (uint32_t)(q & 15);      // l in [0, 15]
      }
    } else if (T != kQ8_0 && i < p.M && kb < p.nblk) {
      constexpr int NW = (F::ABPB + 3) / 4;
      uint32_t m[NW];
      const int bo = bl * F::ABPB;
      const uint32_t* src = &raw[r * SEGW + (bo >> 2)];
      const int sh = (bo & 3) * 8;
#pragma unroll
      for (int q = 0; q < NW; ++q) m[q] = __builtin_amdgcn_alignbit(src[q + 1], src[q], sh);
      d = m[0] & 0xffffu;
      if constexpr (F::AFF) mv = m[0] >> 16;
      constexpr int QS = T == kQ4_0 ? 2 : T == kQ4_1 ? 4 : T == kQ5_0 ? 6 : 8;
      constexpr int OFF = T == kQ4_0 ? 8 : T == kQ4_1 ? 0 : 16;
      constexpr bool Q5 = T == kQ5_0 || T == kQ5_1;
      uint32_t qh = 0;
      if constexpr (T == kQ5_0) qh = get32<2>(m);
      if constexpr (T == kQ5_1) {
        qh = get32<4>(m);
        // |d| > 2047 or |m| > 32752 (incl. inf / NaN): 32 d or 2 m leaves f16
        if ((d & 0x7fffu) > 0x67ffu || ((m[0] >> 16) & 0x7fffu) > 0x77ffu) *big_d = 1u;
      }
      uint32_t qs[4];
      unroll<4>([&](auto K) { qs[K] = get32<QS + 4 * K>(m); });
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const uint32_t byte = (qs[e >> 2] >> (8 * (e & 3))) & 0xffu;
        int lo = (int)(byte & 15u), hi = (int)(byte >> 4);
        if constexpr (Q5) {
          lo |= (int)((qh >> e) & 1u) << 4;
          hi |= (int)((qh >> (e + 16)) & 1u) << 4;
        }
        code[e] = sm_code(lo - OFF);
        code[e + 16] = sm_code(hi - OFF);
      }
    } else {
#pragma unroll
      for (int e = 0; e < 32; ++e) code[e] = code2[e] = 0;
    }
    uint32_t o[6];
    pack_fp6(code, o);
    const int it = (int)(i / F6_TI), rr = (int)(i % F6_TI);
    unsigned char* ch = ws + (int64_t)a * L.a_slice + ((int64_t)it * L.nsteps + kb / F6_KB) * (F6_A_BYTES * F::WP);
    const int b = kb % F6_KB;
    *(u32x4*)(ch + f6_aoff(0, b, rr)) = u32x4{o[0], o[1], o[2], o[3]};
    *(u32x4*)(ch + f6_aoff(1, b, rr)) = u32x4{o[4], o[5], d, mv};
    if constexpr (F::WP == 2) {   // the lo plane: the second half of the K-step's chunk
      pack_fp6(code2, o);
      *(u32x4*)(ch + F6_A_BYTES + f6_aoff(0, b, rr)) = u32x4{o[0], o[1], o[2], o[3]};
      *(u32x4*)(ch + F6_A_BYTES + f6_aoff(1, b, rr)) = u32x4{o[4], o[5], d, mv};
    }
  }
}

// ---------------------------------------------------------------- activation prep
// grid: x = row group of PREP_NT rows * kgroups + kgroup, y = B slice z
// NB blocks per thread: PREP_NB on batched calls, 1 when a single slice would leave the grid
// at a few dozen workgroups (one 4096x512 slice: 64 -> 256)
// BF32: B holds F32 rows (ldb bytes apart) -- ggml's INIT quantization (AVX2 flavour, the bits
// lamm_hip_quantize(.., 1, ..) writes) runs here, straight into the fp6 planes, instead of a
// separate pass writing q8 rows for this kernel to re-read
template <int T, int NB, bool BF32>
__global__ __launch_bounds__(PREP_NT) void prep_b_fp6(GemvArgs p, unsigned char* ws) {
  using F = F6<T>;
  constexpr int VBPB = F::VBPB, VQS = VBPB == 36 ? 4 : 2;
  const F6Layout L = F6Layout::of(p);
  const int nkg = (F6Layout::of(p).nsteps * F6_KB + NB - 1) / NB;
  const int64_t j = (int64_t)(blockIdx.x / nkg) * PREP_NT + threadIdx.x;
  const int kb0 = (blockIdx.x % nkg) * NB;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  if (j >= (int64_t)L.njt * F6_TJ) return;
  const int jt = (int)(j / F6_TJ), r = (int)(j % F6_TJ);
  unsigned char* wsb = ws + (int64_t)z * L.b_slice + (int64_t)jt * L.nsteps * F6_B_BYTES;
  // resource based at the workgroup's first row: wave-uniform (a per-lane base would turn
  // every buffer load into a waterfall loop) and offsets < 2^31 for any slice size
  const int64_t jw = (int64_t)(blockIdx.x / nkg) * PREP_NT;
  const int64_t nrow = min((int64_t)PREP_NT, (int64_t)p.N - jw);
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3 + min(jw, (int64_t)p.N) * p.ldb;
  const int64_t bbytes = nrow > 0 ? (nrow - 1) * p.ldb + (int64_t)p.nblk * (BF32 ? 128 : VBPB) : 0;
  const auto rs = make_rsrc(Bz, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
  for (int kb = kb0; kb < kb0 + NB && kb < L.nsteps * F6_KB; ++kb) {
    uint32_t chi[32], clo[32];
    uint32_t d = 0, sv = 0;
    if (j < p.N && kb < p.nblk) {
      if constexpr (BF32) {
        uint32_t x[32], q8[8];
        uint16_t dh, sh;
        load_words<32, 0>(rs, (uint32_t)((j - jw) * p.ldb + (int64_t)kb * 128), x);
        q8_from_f32<VBPB == 36>(x, q8, dh, sh);
        d = dh;
        sv = sh;
        if constexpr (VBPB == 36) sv |= s_residual(d, sv, q8) << 16;
#pragma unroll
        for (int e = 0; e < 32; ++e) {
          const int q = (int)(int8_t)((q8[e >> 2] >> (8 * (e & 3))) & 0xffu);
          chi[e] = sm_code(q >> 4);
          clo[e] = (uint32_t)(q & 15);
        }
      } else {
        uint32_t m[9];
        load_block<9>(rs, (uint32_t)((j - jw) * p.ldb + (int64_t)kb * VBPB), m);
        d = m[0] & 0xffffu;
        if constexpr (VBPB == 36) {
          sv = m[0] >> 16;
          uint32_t q8[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) q8[k] = m[1 + k];   // q8_1: the quants from byte 4
          sv |= s_residual(d, sv, q8) << 16;
        }
#pragma unroll
        for (int e = 0; e < 32; ++e) {
          const int q = (int)(int8_t)((m[(VQS + e) >> 2] >> (8 * ((VQS + e) & 3))) & 0xffu);
          chi[e] = sm_code(q >> 4);   // floor(q / 16) in [-8, 7]
          clo[e] = (uint32_t)(q & 15);
        }
      }
    } else {
#pragma unroll
      for (int e = 0; e < 32; ++e) chi[e] = clo[e] = 0;
    }
    uint32_t oh[6], ol[6];
    pack_fp6(chi, oh);
    pack_fp6(clo, ol);
    unsigned char* ch = wsb + (int64_t)(kb / F6_KB) * F6_B_BYTES;
    const int b = kb % F6_KB;
    *(u32x4*)(ch + f6_boff(0, b, 0, r)) = u32x4{oh[0], oh[1], oh[2], oh[3]};
    *(u32x4*)(ch + f6_boff(1, b, 0, r)) = u32x4{oh[4], oh[5], d, sv};
    *(u32x4*)(ch + f6_boff(0, b, 1, r)) = u32x4{ol[0], ol[1], ol[2], ol[3]};
    *(u32x4*)(ch + f6_boff(1, b, 1, r)) = u32x4{ol[4], ol[5], d, sv};
  }
}

// Activation prep, q8 rows (the default path), tiled: a workgroup takes 32 rows x 8 blocks; the
// rows' raw block bytes come in by coalesced 16-byte loads (consecutive lanes, consecutive bytes
// of one row) through LDS, then thread (row r, block b) encodes one block.  The per-row kernel
// above reads 34 bytes per lane at a 4352-byte lane stride -- every lane a different cache line,
// 3 instructions per block -- which made it 6.4 us for config 3's 2.2 MB (profiles/r02/
// full_run_6/kernel_stats_bench.csv).  Codes by SWAR, 4 per dword:
//   lo = q & 15 (e2m3 code n/8 = n for 0 <= n <= 15)
//   hi = u < 8 ? u : 48 - u, u = q >> 4 as a nibble (sign | |h| for h = floor(q / 16) in [-8, 7])
#ifndef F6_PB_NB
#define F6_PB_NB 8   // blocks per row of a prep workgroup (A/B builds: 4, 2 -- more, smaller workgroups)
#endif
constexpr int PB_ROWS = 32, PB_NB = F6_PB_NB, PB_NT = PB_ROWS * PB_NB;

// 32 six-bit codes held as bytes (code e = byte e % 4 of c[e / 4]) -> the 192-bit fragment
__device__ __forceinline__ void pack_fp6_bytes(const uint32_t (&c)[8], uint32_t (&o)[6]) {
  uint32_t t[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const uint32_t x = c[k];
    t[k] = (x & 0x3fu) | ((x >> 2) & 0xfc0u) | ((x >> 4) & 0x3f000u) | ((x >> 6) & 0xfc0000u);
  }
  o[0] = t[0] | (t[1] << 24);
  o[1] = (t[1] >> 8) | (t[2] << 16);
  o[2] = (t[2] >> 16) | (t[3] << 8);
  o[3] = t[4] | (t[5] << 24);
  o[4] = (t[5] >> 8) | (t[6] << 16);
  o[5] = (t[6] >> 16) | (t[7] << 8);
}

// one activation block (32 int8 quants as 8 dwords, fp16 d / s bits) -> its hi / lo fragments, at
// byte offset `ch` of the slice's workspace `ws` (write-through: the planes are read by the next
// launch, not this one -- nothing of them should wait dirty in L2 for the end-of-kernel write-back)
template <class Put>
__device__ __forceinline__ void store_b_fp6(Put&& put, int b, int r, const uint32_t (&q)[8], uint32_t d,
                                            uint32_t sv) {
  uint32_t hi[8], lo[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    lo[k] = q[k] & 0x0f0f0f0fu;
    const uint32_t u = (q[k] >> 4) & 0x0f0f0f0fu;
    const uint32_t neg = ((u >> 3) & 0x01010101u) * 0xffu;
    hi[k] = u + ((0x30303030u - (u << 1)) & neg);
  }
  uint32_t oh[6], ol[6];
  pack_fp6_bytes(hi, oh);
  pack_fp6_bytes(lo, ol);
  put(f6_boff(0, b, 0, r), u32x4{oh[0], oh[1], oh[2], oh[3]});
  put(f6_boff(1, b, 0, r), u32x4{oh[4], oh[5], d, sv});
  put(f6_boff(0, b, 1, r), u32x4{ol[0], ol[1], ol[2], ol[3]});
  put(f6_boff(1, b, 1, r), u32x4{ol[4], ol[5], d, sv});
}

#ifndef F6_PREP_AB
// probe builds only (tools/build_fp6_var.sh): 1 no plane stores, 2 no encoding (raw words stored),
// 3 no loads (zero pieces)
#define F6_PREP_AB 0
#endif
template <int T>
__global__ __launch_bounds__(PB_NT) void prep_b_fp6_tile(GemvArgs p, unsigned char* ws) {
  using F = F6<T>;
  constexpr int VBPB = F::VBPB, VQS = VBPB == 36 ? 4 : 2;
  constexpr int SEG = PB_NB * VBPB;                // bytes of a row's 8 blocks (272 / 288)
  constexpr int PIECES = (SEG + 3 + 15) / 16;      // 16-byte pieces from the dword below the start
  constexpr int SEGW = PIECES * 4 + 4;             // dwords per LDS row: 16-byte aligned, realign slack
  __shared__ uint32_t raw[PB_ROWS * SEGW];
  const F6Layout L = F6Layout::of(p);
  const int nbg = (L.nsteps * F6_KB + PB_NB - 1) / PB_NB;
  const int64_t j0 = (int64_t)(blockIdx.x / nbg) * PB_ROWS;
  const int kb0 = (blockIdx.x % nbg) * PB_NB;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  const int64_t nrow = min((int64_t)PB_ROWS, (int64_t)p.N - j0);
  // resource from the tile's first row: offsets < 2^31 for any slice size
  const int64_t base = min(j0, (int64_t)p.N) * p.ldb;
  const int64_t bbytes = nrow > 0 ? (nrow - 1) * p.ldb + (int64_t)p.nblk * VBPB : 0;
  const auto rs = make_rsrc(Bz + base, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
  const int t = threadIdx.x;
  // every piece load of the thread issued before the first wait (round 5: a loop of load -> LDS
  // store waited for each load in turn, three HBM round trips per thread)
  constexpr int NPT = (PB_ROWS * PIECES + PB_NT - 1) / PB_NT;
  u32x4 pc[NPT];
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int idx = t + i * PB_NT, r = idx / PIECES, o = idx % PIECES;
    const uint32_t start = (uint32_t)((int64_t)r * p.ldb + (int64_t)kb0 * VBPB);
    const uint32_t off =
        idx < PB_ROWS * PIECES && r < nrow && kb0 < p.nblk && F6_PREP_AB != 3 ? (start & ~3u) + 16 * o : 0x7ffffff0u;
    pc[i] = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
  }
#pragma unroll
  for (int i = 0; i < NPT; ++i) {
    const int idx = t + i * PB_NT, r = idx / PIECES, o = idx % PIECES;
    if (idx < PB_ROWS * PIECES) *reinterpret_cast<u32x4*>(&raw[r * SEGW + 4 * o]) = pc[i];
  }
  __syncthreads();
  const int r = t % PB_ROWS, bl = t / PB_ROWS;
  const int64_t j = j0 + r;
  const int kb = kb0 + bl;
  if (j >= (int64_t)L.njt * F6_TJ || kb >= L.nsteps * F6_KB) return;
  uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0}, d = 0, sv = 0;
  if (j < p.N && kb < p.nblk) {
    const uint32_t start = (uint32_t)((int64_t)r * p.ldb + (int64_t)kb0 * VBPB);
    const int byte = (int)(start & 3u) + bl * VBPB;
    const uint32_t* src = &raw[r * SEGW + (byte >> 2)];
    const int sh = (byte & 3) * 8;
    constexpr int NWM = (VBPB + 3) / 4 + 1;
    uint32_t m[NWM];
#pragma unroll
    for (int k = 0; k < NWM; ++k) m[k] = __builtin_amdgcn_alignbit(src[k + 1], src[k], sh);
    d = m[0] & 0xffffu;
    if constexpr (VBPB == 36) sv = m[0] >> 16;
    unroll<8>([&](auto K) { q[K] = get32<VQS + 4 * K>(m); });
    if constexpr (VBPB == 36) sv |= s_residual(d, sv, q) << 16;
  }
  unsigned char* wz = ws + (int64_t)z * L.b_slice;
  const int64_t ch = ((int64_t)(j / F6_TJ) * L.nsteps + kb / F6_KB) * F6_B_BYTES;
  if constexpr (F6_PREP_AB == 1) {
    uint32_t x = d ^ sv;
#pragma unroll
    for (int k = 0; k < 8; ++k) x ^= q[k];
    asm volatile("" ::"v"(x));
    return;
  }
  if constexpr (F6_PREP_AB == 2) {
    const auto wr = make_rsrc(wz, (uint32_t)L.b_slice);
    const int b_ = kb % F6_KB, r_ = (int)(j % F6_TJ);
    bstore16_wt(wr, (uint32_t)(ch + f6_boff(0, b_, 0, r_)), u32x4{q[0], q[1], q[2], q[3]});
    bstore16_wt(wr, (uint32_t)(ch + f6_boff(1, b_, 0, r_)), u32x4{q[4], q[5], d, sv});
    bstore16_wt(wr, (uint32_t)(ch + f6_boff(0, b_, 1, r_)), u32x4{q[0], q[1], q[2], q[3]});
    bstore16_wt(wr, (uint32_t)(ch + f6_boff(1, b_, 1, r_)), u32x4{q[4], q[5], d, sv});
    return;
  }
  if (L.b_slice <= 0x7fffffff) {   // write-through buffer stores from a wave-uniform base
    const auto wr = make_rsrc(wz, (uint32_t)L.b_slice);
    store_b_fp6([&](int o, u32x4 v) { bstore16_wt(wr, (uint32_t)(ch + o), v); }, kb % F6_KB, (int)(j % F6_TJ), q, d, sv);
  } else {
    store_b_fp6([&](int o, u32x4 v) { *(u32x4*)(wz + ch + o) = v; }, kb % F6_KB, (int)(j % F6_TJ), q, d, sv);
  }
}

// ---------------------------------------------------------------- GEMM
template <int N_>
__device__ __forceinline__ void f6_wait_vm() {   // s_waitcnt vmcnt(N) (lgkmcnt untouched)
  static_assert(N_ >= 0 && N_ < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N_ & 0xF) | ((N_ >> 4) << 14) | (0x7 << 4) | (0xF << 8));
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void f6_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS reads retired
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// One fragment = 8 consecutive VGPRs: dwords 0-5 are the fp6 operand itself, dwords 6-7 are
// {d, 0} (or {d, m/s} for the affine formats) -- for q4_0 / q5_0 the f16 scale MFMA reads
// dwords 6-7 as its {d, 0, 0, 0} operand with no register moves.
struct F6Frag { i32x8 v; };
struct F6Res { f32x16 s, pr; };    // S (exact block dots) and P = 2 d_b d_a

__device__ __forceinline__ void f6_load(F6Frag& f, const unsigned char* p0, const unsigned char* p1) {
  const u32x4 a = *(const u32x4*)p0, b = *(const u32x4*)p1;
  f.v = i32x8{(int)a[0], (int)a[1], (int)a[2], (int)a[3], (int)b[0], (int)b[1], (int)b[2], (int)b[3]};
}
template <bool AFF>
__device__ __forceinline__ half4 f6_dq(const F6Frag& f) {   // {d, 0, 0, 0}
  if constexpr (AFF) return __builtin_bit_cast(half4, uint2{(uint32_t)f.v[6], 0u});
  else return __builtin_bit_cast(half4, uint2{(uint32_t)f.v[6], (uint32_t)f.v[7]});
}

// V: ablations for tools/ab_gemm.py (0 production, 1 no compute, 2 no DMA, 3 no epilogue FMAs,
//    4 no DMA + no LDS fragment reads (operands from registers), 5 no DMA + no barrier,
//    6 no P-MFMA, 7 no S-MFMA)
// WJ: 32-row activation sub-tiles per wave (2: 64x64 per wave; 1: 32x64).
// SI / SJ: the workgroup's tile is 1/SI x 1/SJ of a packed 256 x 128 chunk (the packed layout,
// and so the stationary weights, stay the same: a sub-tile's rows of one plane are contiguous
// 1 KiB DMA pieces).  KG: K-groups -- the workgroup's waves form KG groups that compute
// consecutive K-steps of the same output tile side by side (one LDS stage = KG K-steps) and
// sum their accumulators through LDS at the end in group order: small grids fill the chip
// without split-K partials in HBM or a reduce launch.
template <int WJ, int SI = 1, int SJ = 1, int KG = 1> struct F6Waves {
  static constexpr int TI = F6_TI / SI, TJ = F6_TJ / SJ;   // workgroup tile
  static constexpr int NWJ = TJ / (32 * WJ), NWI = TI / 64, NWG = NWJ * NWI, NW = NWG * KG, NT = 64 * NW;
  static constexpr int A_SUB = 2 * F6_KB * TI * 16, B_SUB = 2 * F6_KB * 2 * TJ * 16, SUB = A_SUB + B_SUB;
  static constexpr int STAGE = KG * SUB;
  static constexpr int NBUF = STAGE * F6_NBUF <= 128 * 1024 ? F6_NBUF : 128 * 1024 / STAGE;
  static constexpr int PA = A_SUB / F6_PIECE, PSUB = SUB / F6_PIECE;
  static_assert(TI % 64 == 0 && TJ % 64 == 0 && NWJ >= 1, "tile");
  static_assert(NBUF >= 2, "LDS stages");
  static_assert(STAGE % (NW * F6_PIECE) == 0, "every wave moves the same number of DMA pieces");
  // K-group epilogue: every wave's partial tile as [group][j][i] rows padded by 8 floats (the
  // two half-waves' rows j and j+4 then fall on disjoint banks)
  static constexpr int RED = KG > 1 ? KG * TJ * (TI + 8) * 4 : 0;
  static constexpr int LDS = NBUF * STAGE > RED ? NBUF * STAGE : RED;
  static_assert(LDS <= 160 * 1024, "LDS");
  static_assert(KG == 1 || (TI == 128 && TJ % NW == 0), "K-group epilogue: a lane stores 2 of a 128-float row");
  static constexpr int PPW = STAGE / F6_PIECE / NW;   // DMA pieces per wave per stage
  // LDS byte offsets inside one K-step's sub-stage (the chunk image with TI / TJ rows)
  __device__ static constexpr int aoff(int p, int b, int r) { return ((p * F6_KB + b) * TI + r) * 16; }
  __device__ static constexpr int boff(int p, int b, int h, int r) { return A_SUB + (((p * F6_KB + b) * 2 + h) * TJ + r) * 16; }
};

// Split-K (grids with too few 256x128 tiles to fill 256 CUs and no sub-tile plan): split s of
// nsplit runs K-steps [s*nsteps/nsplit, (s+1)*nsteps/nsplit) and writes its partial tile to
// part[s][z][j][i]; f6_reduce then sums the splits in order 0..nsplit-1 (deterministic).
// nsplit == 1 writes C directly.
template <int T, int V_, int WJ, int SI = 1, int SJ = 1, int KG = 1>
__global__ __launch_bounds__((F6Waves<WJ, SI, SJ, KG>::NT)) void gemm_fp6_kernel(GemvArgs p, const unsigned char* wsA,
                                                                                const unsigned char* wsB, int nsplit,
                                                                                float* part, unsigned* tile_ctr) {
  // V_ >= 20: clock probe of ablation V_ - 20 (tools/clk_probe.py): instead of C, thread 0 of
  // workgroup b writes C[2b] = shader clocks (s_memtime) and C[2b+1] = 100 MHz ticks
  // (s_memrealtime) spent from entry to the end of the main loop
  constexpr int V = V_ >= 20 ? V_ - 20 : V_;
  constexpr bool CLK = V_ >= 20;
  const uint64_t clk0 = CLK ? __builtin_readcyclecounter() : 0, rt0 = CLK ? __builtin_amdgcn_s_memrealtime() : 0;
  using F = F6<T>;
  using WV = F6Waves<WJ, SI, SJ, KG>;
  constexpr int F6_NW = WV::NW, F6_PPW = WV::PPW, UPB = 2 * WJ;   // UPB: units per block
  constexpr int NBUF = WV::NBUF, TI = WV::TI, TJ = WV::TJ;
  constexpr bool AFF = F::AFF;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const F6Layout L = F6Layout::of(p);

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const int g = w / WV::NWG, wl = w % WV::NWG;   // K-group, wave within the group
  const int wj = wl % WV::NWJ, wi = wl / WV::NWJ;   // NWJ (j) x NWI (i) waves
  // XCD-aware tile order: workgroup id -> tile index so that the workgroups one XCD runs at
  // once are neighbouring tiles of one slice (their DMA chunks meet in that XCD's L2).
  const int nsi = (p.M + TI - 1) / TI, nsj = (p.N + TJ - 1) / TJ;   // workgroup tiles per slice
  int ti, tj, z, sp;
  {
    const int ntile = nsi * nsj * p.ne12 * p.ne13;
    const int nwg = ntile * nsplit;
    const int id = blockIdx.x, x = id & 7, k = id >> 3, q = nwg >> 3, rmd = nwg & 7;
    int wv = x < rmd ? x * (q + 1) + k : rmd * (q + 1) + (x - rmd) * q + k;
    sp = wv / ntile;   // split-major: one XCD's neighbouring tiles share a K range
    wv %= ntile;
    const int per = nsi * nsj;
    z = wv / per;
    const int ws_ = wv % per, ib = ws_ / (8 * nsj), rem = ws_ % (8 * nsj);
    const int width = min(8, nsi - ib * 8);
    tj = rem / width;
    ti = ib * 8 + rem % width;
  }
  const int it = ti / SI, jt = tj / SJ;   // packed chunk and the tile's rows inside it
  const int ri0 = (ti % SI) * TI, rj0 = (tj % SJ) * TJ;
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const int ne02 = p.ne12 / p.r2, a = (i12 / p.r2) + (i13 / p.r3) * ne02;
  const unsigned char* wa = wsA + (int64_t)a * L.a_slice + (int64_t)it * L.nsteps * F6_A_BYTES;
  const unsigned char* wb = wsB + (int64_t)z * L.b_slice + (int64_t)jt * L.nsteps * F6_B_BYTES;
  const int nsteps = L.nsteps;
  const int k0 = (int)((int64_t)sp * nsteps / nsplit), k1 = (int)((int64_t)(sp + 1) * nsteps / nsplit);
  // stages: KG consecutive K-steps each (KG > 1 runs unsplit)
  const int s0 = KG == 1 ? k0 : 0, s1 = KG == 1 ? k1 : (nsteps + KG - 1) / KG;

  // ---- LDS-DMA: piece pc = k*NW + w of a stage = K-group pc / PSUB, piece pc % PSUB of its
  // K-step (A pieces first, then B); a K-step past the end re-loads the last one (its group
  // skips the compute), so every wave moves PPW pieces per stage and the vmcnt counts hold.
  // The piece's offset is wave-uniform (soffset); the lane's 16 bytes are the only VGPR ----
  const auto ra = make_rsrc(wa, (uint32_t)(nsteps * F6_A_BYTES));
  const auto rb = make_rsrc(wb, (uint32_t)(nsteps * F6_B_BYTES));
  auto issue = [&](int ss) {
    unsigned char* dst = smem + (ss % NBUF) * WV::STAGE;
#pragma unroll
    for (int k = 0; k < F6_PPW; ++k) {
      const int pc = k * F6_NW + w;   // wave-uniform
      const int kg = pc / WV::PSUB, q = pc % WV::PSUB;
      const int ks = min(KG * ss + kg, nsteps - 1);
      auto* d = (__attribute__((address_space(3))) void*)(dst + pc * F6_PIECE);
      if (q < WV::PA) {
        const int plane = q / (TI / 64), part_ = q % (TI / 64);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, d, 16, lane * 16,
                                                 ks * F6_A_BYTES + (plane * F6_TI + ri0 + 64 * part_) * 16, 0, 0);
      } else {
        const int plane = (q - WV::PA) / (TJ / 64), part_ = (q - WV::PA) % (TJ / 64);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, d, 16, lane * 16,
                                                 ks * F6_B_BYTES + (plane * F6_TJ + rj0 + 64 * part_) * 16, 0, 0);
      }
    }
  };

  const int sc_a = h ? SCALE_LO : SCALE_HI;   // MFMA A operand = activations (k-group h)
  f32x16 acc[WJ][2];   // [jt][it]: 2 * sum d_a d_b S (+ 2 * sum m_a s_b)
#pragma unroll
  for (int x = 0; x < WJ; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
  const f32x16 fz = {};

  constexpr bool NODMA = V == 2 || V == 4 || V == 5;
  if (!NODMA)
    for (int k = s0; k < s0 + NBUF - 1 && k < s1; ++k) issue(k);
  F6Frag fb[2][WJ], fa[2][2];   // [block slot][sub-tile]
  F6Res rr[F6_PD + 1];   // results of the units in flight
  constexpr int NU = UPB * F6_KB;   // units per K-step
  auto epi = [&](int n, const F6Res& R) {
    f32x16& c = acc[(n / 2) % WJ][n & 1];
    if constexpr (V == 3) {
      c[0] += R.s[0] + R.pr[0];
    } else {
#pragma unroll
      for (int e = 0; e < 16; ++e) c[e] = __builtin_fmaf(R.s[e], R.pr[e], c[e]);
    }
  };
  // Every wave defers its last unit's FMAs of a K-step across the barrier: they run while the
  // next step's first fragments load (-2.7 % main-kernel time, profiles/r01/ab_sched.txt).
  // A/B variants: 8 = + waves 4-7 at s_setprio 1 (no gain); 10 = only waves 4-7 defer (a
  // stagger: two code paths, 256 VGPRs, +65 %); 12 = no deferral (the previous schedule)
  const bool defer = V != 12 && (V != 10 || w >= 4);
  if constexpr (V == 8) {
    if (w >= 4) __builtin_amdgcn_s_setprio(1);
  }
  bool pend = false;
  for (int ss = s0; ss < s1; ++ss) {
    if (!NODMA) {   // this wave's pieces of stage ss landed (younger stages may stay in flight)
      const int ahead = min(NBUF - 2, s1 - 1 - ss);
      if (ahead >= 2) f6_wait_vm<2 * F6_PPW>();
      else if (ahead == 1) f6_wait_vm<F6_PPW>();
      else f6_wait_vm<0>();
    }
    if (V != 5) f6_barrier();   // stage ss visible to all waves; stage ss-1 no longer read
    if (!NODMA && ss + NBUF - 1 < s1) issue(ss + NBUF - 1);
    if constexpr (V == 1) continue;
    const int ks = KG * ss + g;
    if (KG > 1 && ks >= nsteps) continue;   // this group's K-step is past the end (wave-uniform)
    const unsigned char* sA = smem + (ss % NBUF) * WV::STAGE + g * WV::SUB;
    const unsigned char* sB = sA;

    // fragments are read from LDS one block ahead of their MFMAs, not as one burst per K-step
    // (8 waves x 4*KB ds_read_b128 pairs right after the barrier queue hundreds of LDS cycles
    // in front of every wave's first MFMA).  Block b lives in register slot b & 1.
    auto ldB = [&](int b, int x) {
      if constexpr (V == 4 || V == 11) {   // 11: DMA on, fragments read once
        if (ss > s0) return;
      }
      const int r = 32 * WJ * wj + 32 * x + lr;
      f6_load(fb[b & 1][x], sB + WV::boff(0, b, h, r), sB + WV::boff(1, b, h, r));
    };
    auto ldA = [&](int b, int y) {
      if constexpr (V == 4 || V == 11) {   // 11: DMA on, fragments read once
        if (ss > s0) return;
      }
      const int r = 64 * wi + 32 * y + lr;
      f6_load(fa[b & 1][y], sA + WV::aoff(0, b, r), sA + WV::aoff(1, b, r));
    };
    // unit n = (block n / UPB, j sub-tile (n / 2) % WJ, i sub-tile n % 2)
    auto ld_unit = [&](int n) {   // the fragments unit n uses first
      const int b = n / UPB, u = n % UPB, x = (n / 2) % WJ;
      if (u == 0) { ldB(b, 0); ldA(b, 0); }
      else if (u == 1) ldA(b, 1);
      else if ((u & 1) == 0) ldB(b, x);
    };
    auto mfmas = [&](int n, F6Res& R) {
      const F6Frag& fB = fb[(n / UPB) & 1][(n / 2) % WJ];
      const F6Frag& fA = fa[(n / UPB) & 1][n & 1];
      if constexpr (V != 7)
        R.s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(fB.v, fA.v, fz, 2, 2, 0, sc_a, 0, SCALE_W);
      if constexpr (V != 6)
        R.pr = __builtin_amdgcn_mfma_f32_32x32x8f16(f6_dq<AFF>(fB), f6_dq<AFF>(fA), fz, 0, 0, 0);
      if constexpr (V == 6) R.pr = R.s;   // ablation: no P-MFMA
      if constexpr (V == 7) R.s = R.pr;   // ablation: no S-MFMA
    };
    uint32_t msA[2][2] = {{0, 0}, {0, 0}}, msB[WJ][2] = {};   // q4_1: m_a / s_b per block
    auto keep_ms = [&](int b) {
      if constexpr (AFF) {
#pragma unroll
        for (int y = 0; y < 2; ++y) msA[y][b >> 1] |= ((uint32_t)fa[b & 1][y].v[7] & 0xffffu) << (16 * (b & 1));
#pragma unroll
        for (int x = 0; x < WJ; ++x) msB[x][b >> 1] |= ((uint32_t)fb[b & 1][x].v[7] & 0xffffu) << (16 * (b & 1));
        if constexpr (F::SH16) {   // [0]: 2 m_a / s_b, [1]: 32 d_a / s's residual r_b (SH16 above)
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            msA[y][0] = (msA[y][0] & ~(0xffffu << (16 * (b & 1)))) |
                        f16_times2((uint32_t)fa[b & 1][y].v[7]) << (16 * (b & 1));
            msA[y][1] |= f16_times2(f16_times16((uint32_t)fa[b & 1][y].v[6])) << (16 * (b & 1));
          }
#pragma unroll
          for (int x = 0; x < WJ; ++x) msB[x][1] |= ((uint32_t)fb[b & 1][x].v[7] >> 16) << (16 * (b & 1));
        }
      }
    };

    static_assert(F6_KB == 2 || F6_KB == 4, "the m*s rank-KB MFMA packs <= 4 blocks per k half");
    constexpr int LDA = UPB;          // fragment prefetch distance in units (one block)
    static_assert((NU - 1) % (F6_PD + 1) >= F6_PD, "deferred unit's result slot is reused too early");
    unroll<LDA>([&](auto NN) { ld_unit(NN); });
    if (pend) {   // previous step's last unit, under this step's first LDS reads
      __builtin_amdgcn_sched_barrier(0);
      epi(NU - 1, rr[(NU - 1) % (F6_PD + 1)]);
      __builtin_amdgcn_sched_barrier(0);
    }
    unroll<F6_PD>([&](auto NN) { mfmas(NN, rr[NN]); });
    unroll<NU>([&](auto NN) {
      constexpr int n = NN;
      if constexpr (n % UPB == UPB - 1) keep_ms(n / UPB);
      if constexpr (n + LDA < NU) ld_unit(n + LDA);
      if constexpr (n + F6_PD < NU) mfmas(n + F6_PD, rr[(n + F6_PD) % (F6_PD + 1)]);
      __builtin_amdgcn_sched_barrier(0);
      if (n != NU - 1 || !defer) epi(n, rr[n % (F6_PD + 1)]);
      __builtin_amdgcn_sched_barrier(0);
    });
    pend = defer;
    if constexpr (AFF) {   // sum_b m_a * s_b: rank-KB per K-step, both k halves carry it (x2 like P)
#pragma unroll
      for (int x = 0; x < WJ; ++x) {
        // SH16: lanes 0-31 {s_b, s_b} x {2 m_a, 32 d_a}, lanes 32-63 {r_b, 0} x {32 d_a, 0}
        const half4 sf = F::SH16 ? __builtin_bit_cast(half4, uint2{h ? msB[x][1] : msB[x][0], h ? 0u : msB[x][0]})
                                 : __builtin_bit_cast(half4, uint2{msB[x][0], msB[x][1]});
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          const half4 mf = F::SH16 ? __builtin_bit_cast(half4, uint2{h ? msA[y][1] : msA[y][0], h ? 0u : msA[y][1]})
                                   : __builtin_bit_cast(half4, uint2{msA[y][0], msA[y][1]});
          acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x8f16(sf, mf, acc[x][y], 0, 0, 0);
        }
      }
    }
  }

  if (pend) epi(NU - 1, rr[(NU - 1) % (F6_PD + 1)]);
  if constexpr (CLK) {
    float sink = 0.f;   // keep the main loop's arithmetic alive and ordered before the stamp
#pragma unroll
    for (int x = 0; x < WJ; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) sink += acc[x][y][e];
    asm volatile("s_nop 0" ::"v"(sink) : "memory");
    const uint64_t clk1 = __builtin_readcyclecounter(), rt1 = __builtin_amdgcn_s_memrealtime();
    if (sink == -1.2345e-30f) p.C[4096 + t] = sink;
    if (t == 0) {
      p.C[2 * blockIdx.x] = (float)(clk1 - clk0);
      p.C[2 * blockIdx.x + 1] = (float)(rt1 - rt0);
    }
    return;
  }
  if constexpr (KG > 1) {
    // Every wave parks its partial tile in the (now idle) stages; then the tile's rows are split
    // over ALL waves: wave w sums rows j = w*RPW.. over the groups in group order (the bits of
    // "group 0 adds groups 1, 2, 3"), and stores them as 512-byte runs of C (2 floats a lane)
    // -- instead of group 0's two waves alone adding and storing 4-byte pieces
    // (profiles/r02/fp6_kgroups_ablation.txt: that epilogue cost ~4 us of a 30 us kernel).
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    float* red = reinterpret_cast<float*>(smem);
    constexpr int PI = TI + 8, RPW = TJ / F6_NW;
#pragma unroll
    for (int x = 0; x < WJ; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int i = 64 * wi + 32 * y + lr, j = 32 * WJ * wj + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
          red[(g * TJ + j) * PI + i] = acc[x][y][e];
        }
    __syncthreads();
    float* C = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
    const int64_t i = (int64_t)ti * TI + 2 * lane;
    const bool pair = i + 1 < p.M && (p.ldc & 1) == 0 && ((uintptr_t)C & 7) == 0;
#pragma unroll
    for (int q = 0; q < RPW; ++q) {
      const int jl = w * RPW + q;
      const int64_t j = (int64_t)tj * TJ + jl;
      f32x2 v = *reinterpret_cast<const f32x2*>(&red[jl * PI + 2 * lane]);
#pragma unroll
      for (int g_ = 1; g_ < KG; ++g_) v += *reinterpret_cast<const f32x2*>(&red[(g_ * TJ + jl) * PI + 2 * lane]);
      v *= 0.5f;
      if (j < p.N) {
        float* c = C + j * p.ldc + i;
        if (pair) {
#if F6_C_NT
          __builtin_nontemporal_store(v, reinterpret_cast<f32x2*>(c));
#else
          *reinterpret_cast<f32x2*>(c) = v;
#endif
        } else {
          if (i < p.M) c[0] = v[0];
          if (i + 1 < p.M) c[1] = v[1];
        }
      }
    }
    return;
  }
  float* Cz;
  int64_t ldc;
  if (nsplit == 1) {
    Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
    ldc = p.ldc;
  } else {
    Cz = part + ((int64_t)sp * p.ne12 * p.ne13 + z) * p.N * p.M;
    ldc = p.M;
  }
  const bool fused = SI == 1 && SJ == 1 && KG == 1 && nsplit > 1 && tile_ctr != nullptr;
  if (!fused) {
#pragma unroll
    for (int x = 0; x < WJ; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        const int64_t i = (int64_t)ti * TI + 64 * wi + 32 * y + lr;
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int64_t j = (int64_t)tj * TJ + 32 * WJ * wj + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
          if (i < p.M && j < p.N) {
#if F6_CT_NT
            __builtin_nontemporal_store(0.5f * acc[x][y][e], &Cz[j * ldc + i]);
#else
            Cz[j * ldc + i] = 0.5f * acc[x][y][e];
#endif
          }
        }
      }
    return;
  }
  // Split-K fixup inside the launch (no reduce kernel): every split's workgroup publishes its
  // partial tile, then counts itself in on the tile's counter; the one that arrives last sums
  // the partials in split order 0..nsplit-1 -- the order f6_reduce adds them in, so C has the
  // same bits -- and resets the counter for the next launch.  Nobody waits for anybody:
  // correctness does not depend on which workgroups are resident.  The partials are kept in
  // the accumulators' own register layout (each lane's 16 values as 4 x 16 B, a wave's
  // instruction 1 KiB contiguous) and stored write-through (sc1), so the last workgroup reads
  // them from any XCD with 16-byte loads (4-byte write-through stores cost one fabric write
  // per lane).
  constexpr int kAuxSc1 = 16;
  constexpr int TILE_FLOATS = F6_TI * F6_TJ;
  const int tile = (int)(((int64_t)z * L.njt + jt) * L.nit + it);
  const int ntile = L.nit * L.njt * p.ne12 * p.ne13;
  auto slab = [&](int s_) {   // split s_'s partial of this tile: [wave][x][y][q][lane][4]
    return make_rsrc(part + ((int64_t)s_ * ntile + tile) * TILE_FLOATS, TILE_FLOATS * 4u);
  };
  auto foff = [&](int x, int y, int q) { return (uint32_t)(((((w * WJ + x) * 2 + y) * 4 + q) * 64 + lane) * 16); };
  {
    const auto mine = slab(sp);
#pragma unroll
    for (int x = 0; x < WJ; ++x)
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const f32x4 v = {0.5f * acc[x][y][4 * q], 0.5f * acc[x][y][4 * q + 1], 0.5f * acc[x][y][4 * q + 2],
                           0.5f * acc[x][y][4 * q + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), mine, foff(x, y, q), 0, kAuxSc1);
        }
  }
  __shared__ int last_arrival;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's partial stores have landed
  __syncthreads();
  if (t == 0) last_arrival = atomicAdd(&tile_ctr[tile], 1u) == (unsigned)(nsplit - 1);
  __syncthreads();
  if (!last_arrival) return;
  float* C = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
#pragma unroll
  for (int x = 0; x < WJ; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      f32x16 sum;
#pragma unroll
      for (int e = 0; e < 16; ++e) sum[e] = sp == 0 ? 0.5f * acc[x][y][e] : 0.f;
      for (int s2 = (sp == 0 ? 1 : 0); s2 < nsplit; ++s2) {
        const auto r = slab(s2);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          f32x4 v;
          if (s2 == sp) {
            v = f32x4{0.5f * acc[x][y][4 * q], 0.5f * acc[x][y][4 * q + 1], 0.5f * acc[x][y][4 * q + 2],
                      0.5f * acc[x][y][4 * q + 3]};
          } else {
            v = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, foff(x, y, q), 0, kAuxSc1));
          }
#pragma unroll
          for (int k = 0; k < 4; ++k) sum[4 * q + k] = s2 == 0 ? v[k] : sum[4 * q + k] + v[k];
        }
      }
      const int64_t i = (int64_t)it * F6_TI + 64 * wi + 32 * y + lr;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int64_t j = (int64_t)jt * F6_TJ + 32 * WJ * wj + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (i < p.M && j < p.N) C[j * p.ldc + i] = sum[e];
      }
    }
  if (t == 0) __hip_atomic_store(&tile_ctr[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// K-group plan without workgroup barriers in the main loop.  The workgroup's 128 x 64 tile and
// waves as gemm_fp6_kernel<.., 2, 2, 2, 4> (4 K-groups x 2 row halves), but every wave streams its
// own blocks:
//   weights   : its 64 rows by LDS-DMA into a ring of its OWN (P x 2 KiB) -- only this wave writes
//               and reads it, so its vmcnt is the only synchronisation -- read back by ds_read
//               with both half-waves on the same rows (the MFMA wants each weight row in both
//               K halves; LDS serves the duplicate addresses, no cross-lane VALU)
//   activations: the group's 64 rows straight into VGPRs in fragment order (lane (r, h) = row r,
//               hi / lo plane h; the group's second wave hits L1)
// P blocks in flight per wave.  A fragment's six code dwords and its {d, m / s} pair are separate
// operands (scale MFMA / f16 MFMA), assembled from the two 16-byte planes at use.
// AB (ablations, tools/prep_probe.hip only): 1 loads only; 2 compute only (no loads after the first
// P blocks); 3 compute only with half the FMAs; 4 compute only, one FMA per unit; 5 / 6 / 7 the
// production loop without the activations' / the weights' / both second 16-byte planes (the
// operand bytes' share of the time; the results are not meaningful).
// AD (probe): the weight fragments by buffer loads straight into VGPRs (both half-waves load the same
// rows; the L1 merges the duplicate addresses) instead of the LDS-DMA ring.
template <int T, int P, int AB = 0, int AD = 0>
__global__ __launch_bounds__(512) void gemm_fp6_kv_kernel(GemvArgs p, const unsigned char* wsA,
                                                          const unsigned char* wsB) {
  using F = F6<T>;
  constexpr bool AFF = F::AFF;
  constexpr int WP = F::WP;   // weight code planes (q8_0: hi, lo)
  constexpr int KG = 4, TI = 128, TJ = 64, NW = 8, WJ = 2, UPB = 2 * WJ;
  // vmem ops per block: 2 weight DMA pieces per plane (AD: 2 sub-tiles x 2 loads per plane), WJ x 2
  // activation loads
  constexpr bool CO = AB >= 2 && AB <= 4;            // compute-only ablations
  constexpr bool SKA = AB == 5 || AB == 7, SKW = AB == 6 || AB == 7;
  constexpr int APB = (SKA ? 1 : 2) * WJ;             // activation loads per block
  constexpr int LPB = (AD ? 4 * WP : (SKW ? 1 : 2) * WP) + APB;
  constexpr int RING = P * 2 * WP * F6_PIECE;   // bytes of a wave's weight ring
  constexpr int ABY = WP * F6_A_BYTES;          // bytes of a K-step's A chunk
  static_assert(P >= 2 && P <= 6, "blocks in flight");
  static_assert(NW * RING <= 4 * 64 * (128 + 8) * 4, "the rings live under the epilogue's LDS");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const F6Layout L = F6Layout::of(p, WP);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const int g = w / 2, wi = w % 2;
  const int nsi = (p.M + TI - 1) / TI, nsj = (p.N + TJ - 1) / TJ;
  int ti, tj, z;
  {   // XCD-aware tile order (gemm_fp6_kernel)
    const int ntile = nsi * nsj * p.ne12 * p.ne13;
    const int id = blockIdx.x, x = id & 7, k = id >> 3, q = ntile >> 3, rmd = ntile & 7;
    const int wv = x < rmd ? x * (q + 1) + k : rmd * (q + 1) + (x - rmd) * q + k;
    const int per = nsi * nsj;
    z = wv / per;
    const int ws_ = wv % per, ib = ws_ / (8 * nsj), rem = ws_ % (8 * nsj);
    const int width = min(8, nsi - ib * 8);
    tj = rem / width;
    ti = ib * 8 + rem % width;
  }
  const int it = ti / 2, jt = tj / 2, ri0 = (ti % 2) * TI, rj0 = (tj % 2) * TJ;
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const int ne02 = p.ne12 / p.r2, a = (i12 / p.r2) + (i13 / p.r3) * ne02;
  const unsigned char* wa = wsA + (int64_t)a * L.a_slice + (int64_t)it * L.nsteps * ABY;
  const unsigned char* wb = wsB + (int64_t)z * L.b_slice + (int64_t)jt * L.nsteps * F6_B_BYTES;
  const int nsteps = L.nsteps;
  const int nbw = nsteps > g ? (nsteps - g + KG - 1) / KG * F6_KB : 0;   // this wave's blocks
  const auto ra = make_rsrc(wa, (uint32_t)(nsteps * ABY));
  const auto rb = make_rsrc(wb, (uint32_t)(nsteps * F6_B_BYTES));
  const int a0 = (ri0 + 64 * wi) * 16;                         // f6_aoff(0, 0, first row)
  const uint32_t b0 = (uint32_t)(h * F6_TJ + rj0 + lr) * 16;   // f6_boff(0, 0, h, row)
  unsigned char* ring = smem + w * RING;

  u32x4 rb_[P][WJ][2];   // activation ring: sub-tile x, plane
  if constexpr (SKA)
    for (int s_ = 0; s_ < P; ++s_)
      for (int x = 0; x < WJ; ++x) rb_[s_][x][1] = u32x4{0u, 0u, 0u, 0u};
  u32x4 ra_[AD ? P : 1][2][2 * WP];   // AD: weight fragments: sub-tile y, (code plane, 16-byte plane)
  const uint32_t arow = (uint32_t)(ri0 + 64 * wi + lr) * 16;   // AD: the lane's weight row
  // block u of this wave (K-step g + KG (u / KB), block u % KB) into ring slot S; past the end the
  // last block is fetched again (unused) so every slot's wait count stays the same
  auto issue = [&](int u, auto S_) {
    constexpr int S = decltype(S_)::value;
    const int uu = min(u, nbw - 1);
    const int ks = g + KG * (uu / F6_KB), b = uu % F6_KB;
    const int ka = ks * ABY, kb = ks * F6_B_BYTES;
    if constexpr (AD) {
#pragma unroll
      for (int y = 0; y < 2; ++y)
#pragma unroll
        for (int pl = 0; pl < 2 * WP; ++pl) {
          const uint32_t o = arow + (uint32_t)((pl / 2) * F6_A_BYTES + ((pl % 2) * F6_KB + b) * F6_TI * 16 + 32 * y * 16);
          // a second plane without m (all but q4_1 / q5_1): its last dword is 0, 12 bytes suffice
          if (pl % 2 == 1 && !AFF) {
            const auto v = __builtin_amdgcn_raw_buffer_load_b96(ra, o, ka, 0);
            ra_[S][y][pl] = u32x4{v[0], v[1], v[2], 0u};
          } else {
            ra_[S][y][pl] = __builtin_amdgcn_raw_buffer_load_b128(ra, o, ka, 0);
          }
        }
    } else {
#pragma unroll
      for (int pl = 0; pl < 2 * WP; ++pl) {   // (code plane pl / 2) x (16-byte plane pl % 2)
        if (SKW && pl % 2 == 1) continue;
        auto* d = (__attribute__((address_space(3))) void*)(ring + (S * 2 * WP + pl) * F6_PIECE);
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, d, 16, lane * 16,
                                                 ka + (pl / 2) * F6_A_BYTES + a0 + ((pl % 2) * F6_KB + b) * F6_TI * 16, 0, 0);
      }
    }
#pragma unroll
    for (int x = 0; x < WJ; ++x)
#pragma unroll
      for (int pl = 0; pl < 2; ++pl) {
        if (SKA && pl == 1) continue;
        const uint32_t o = b0 + (uint32_t)((((pl * F6_KB + b) * 2) * F6_TJ + 32 * x) * 16);
        if (AD && pl == 1 && F::VBPB != 36) {   // q8_0 activations: no s, the plane's last dword is 0
          const auto v = __builtin_amdgcn_raw_buffer_load_b96(rb, o, kb, 0);
          rb_[S][x][pl] = u32x4{v[0], v[1], v[2], 0u};
        } else {
          rb_[S][x][pl] = __builtin_amdgcn_raw_buffer_load_b128(rb, o, kb, 0);
        }
      }
  };

  const int sc_a = h ? SCALE_LO : SCALE_HI;
  f32x16 acc[WJ][2];
#pragma unroll
  for (int x = 0; x < WJ; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
  const f32x16 fz = {};
  F6Res rr[2];
  bool pend = false;
  uint32_t msA[2] = {0, 0}, msB[WJ] = {};   // q4_1: the K-step's m_a / s_b (16 bits per block)
  uint32_t dsA[2] = {0, 0};                 // q5_1: the K-step's 32 d_a
  uint32_t rsB[WJ] = {};                    // q5_1: the K-step's residuals r_b of s_b
  // a fragment's operands from its two 16-byte planes: the scale MFMA's six code dwords, the f16
  // MFMA's {d, 0, 0, 0} (q4_1: {d, m} -> {d, 0, 0, 0} too)
  auto codes = [](const u32x4& p0, const u32x4& p1) {
    return i32x8{(int)p0[0], (int)p0[1], (int)p0[2], (int)p0[3], (int)p1[0], (int)p1[1], 0, 0};
  };
  auto dq = [](const u32x4& p1) {
    if constexpr (AFF) return __builtin_bit_cast(half4, uint2{p1[2], 0u});
    else return __builtin_bit_cast(half4, uint2{p1[2], p1[3]});
  };

  // a block's weight fragments from its ring slot: per sub-tile y (rows 32 y + lr in both half-waves)
  // the scale MFMA's six code dwords and the f16 MFMA's {d, m} pair
  struct WFrag { i32x8 c[2]; i32x2 d[2]; i32x8 c2[WP == 2 ? 2 : 1]; };   // c2: q8_0's lo codes
  const int lo = (32 * 0 + lr) * 16;
  auto wread = [&](int slot, WFrag& f) {
    const unsigned char* r0 = ring + slot * 2 * WP * F6_PIECE;
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int o = lo + 32 * y * 16;
      const i32x4 q0 = *reinterpret_cast<const i32x4*>(r0 + o);
      const i32x4 q1 = *reinterpret_cast<const i32x4*>(r0 + F6_PIECE + o);
      f.d[y] = i32x2{q1[2], q1[3]};
      f.c[y] = i32x8{q0[0], q0[1], q0[2], q0[3], q1[0], q1[1], 0, 0};
      if constexpr (WP == 2) {
        const i32x4 q2 = *reinterpret_cast<const i32x4*>(r0 + 2 * F6_PIECE + o);
        const i32x4 q3 = *reinterpret_cast<const i32x4*>(r0 + 3 * F6_PIECE + o);
        f.c2[y] = i32x8{q2[0], q2[1], q2[2], q2[3], q3[0], q3[1], 0, 0};
      }
    }
  };
  WFrag wc;   // the current block's weight fragments (read during the block before)

  int sink = 0;
  auto block = [&](int u, auto S_) {
    constexpr int S = decltype(S_)::value;
    constexpr int SN = (S + 1) % P;
    f6_wait_vm<LPB * (P - 1)>();   // block u's activations landed; the P - 1 younger may fly
    if constexpr (AB == 1) {
#pragma unroll
      for (int x = 0; x < WJ; ++x) sink ^= (int)(rb_[S][x][0][0] ^ rb_[S][x][1][0]);
      if constexpr (AD) {   // every load's first dword (a load whose value is unused would be dropped)
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int pl = 0; pl < 2 * WP; ++pl) sink ^= (int)ra_[S][y][pl][0];
      } else {
        sink ^= *(const int*)(ring + S * 2 * F6_PIECE + lane * 4);
      }
      issue(u + P, S_);
      return;
    }
    if constexpr (CO || SKA) {
#pragma unroll
      for (int x = 0; x < WJ; ++x) asm volatile("" : "+v"(rb_[S][x][0]), "+v"(rb_[S][x][1]));
      if constexpr (AD) {
#pragma unroll
        for (int y = 0; y < 2; ++y)
#pragma unroll
          for (int pl = 0; pl < 2 * WP; ++pl) asm volatile("" : "+v"(ra_[S][y][pl]));
      }
    }
    if constexpr (AD) {   // this block's weight fragments: landed with its activations
#pragma unroll
      for (int y = 0; y < 2; ++y) {
        wc.d[y] = i32x2{(int)ra_[S][y][1][2], (int)ra_[S][y][1][3]};
        wc.c[y] = codes(ra_[S][y][0], ra_[S][y][1]);
        if constexpr (WP == 2) wc.c2[y] = codes(ra_[S][y][2], ra_[S][y][3]);
      }
    }
    WFrag wn;   // the next block's, read half-way through this one
    // unit n: S = the exact block dots (scale MFMA), P = 2 d_b d_a (f16 MFMA), then acc += S * P.
    // Issue order per unit: S(n+1), half of unit n's FMAs, P(n+1), the other half -- each MFMA's 32
    // cycles in the matrix pipe covered by 8 FMAs (32 issue cycles) of the unit before
    auto mfma_s = [&](int n, F6Res& R) {
      const int x = (n / 2) % WJ, y = n & 1;
      if constexpr (WP == 2) {   // q8_0: S = sum 16 h b (hi codes, weight scale x16) + sum l b
        const i32x8 bc = codes(rb_[S][x][0], rb_[S][x][1]);
        R.s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bc, wc.c[y], fz, 2, 2, 0, sc_a, 0, SCALE_W + 4);
        R.s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bc, wc.c2[y], R.s, 2, 2, 0, sc_a, 0, SCALE_W);
      } else {
        R.s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(codes(rb_[S][x][0], rb_[S][x][1]), wc.c[y], fz, 2, 2, 0,
                                                              sc_a, 0, SCALE_W);
      }
    };
    auto mfma_p = [&](int n, F6Res& R) {
      const int x = (n / 2) % WJ, y = n & 1;
      const half4 da = AFF ? __builtin_bit_cast(half4, i32x2{wc.d[y][0], 0}) : __builtin_bit_cast(half4, wc.d[y]);
      R.pr = __builtin_amdgcn_mfma_f32_32x32x8f16(dq(rb_[S][x][1]), da, fz, 0, 0, 0);
    };
    auto epi = [&](int n, const F6Res& R, int half) {
      f32x16& c = acc[(n / 2) % WJ][n & 1];
      if constexpr (AB == 4) {
        if (half == 0) c[0] = __builtin_fmaf(R.s[0], R.pr[0], c[0]);
        return;
      }
      if (AB == 3 && half == 1) return;
#pragma unroll
      for (int e = 8 * half; e < 8 * half + 8; ++e) c[e] = __builtin_fmaf(R.s[e], R.pr[e], c[e]);
    };
    auto sb = [] { __builtin_amdgcn_sched_barrier(0); };
    // issue order of one unit step (F6_KV_ORDER, probe builds): 0 S, E/2, P, E/2 (production);
    // 1 P, E/2, S, E/2; 2 S, P, E
    auto unit = [&](auto do_s, auto do_p, auto do_e0, auto do_e1) {
      if constexpr (F6_KV_ORDER == 1) {
        do_p(); sb(); do_e0(); sb(); do_s(); sb(); do_e1(); sb();
      } else if constexpr (F6_KV_ORDER == 2) {
        do_s(); sb(); do_p(); sb(); do_e0(); sb(); do_e1(); sb();
      } else {
        do_s(); sb(); do_e0(); sb(); do_p(); sb(); do_e1(); sb();
      }
    };
    sb();
    unit([&] { mfma_s(0, rr[0]); }, [&] { mfma_p(0, rr[0]); },
         [&] { if (pend) epi(UPB - 1, rr[(UPB - 1) % 2], 0); },   // the previous block's last unit
         [&] { if (pend) epi(UPB - 1, rr[(UPB - 1) % 2], 1); });
    unroll<UPB - 1>([&](auto NN) {
      constexpr int n = NN;
      if constexpr (n == 1 && !AD) {   // the next block's weights: its DMA pieces landed (the oldest vmem
        // ops but this block's activation loads are older still -- all landed at the top)
        if constexpr (!CO) f6_wait_vm<LPB * (P - 2) + APB>();
        wread(SN, wn);
        sb();
      }
      unit([&] { mfma_s(n + 1, rr[(n + 1) % 2]); }, [&] { mfma_p(n + 1, rr[(n + 1) % 2]); },
           [&] { epi(n, rr[n % 2], 0); }, [&] { epi(n, rr[n % 2], 1); });
    });
    pend = true;
    if constexpr (AFF) {   // sum_b m_a s_b per K-step: rank-KB, both k halves carry it (x2 like P)
      const int bk = u % F6_KB;
#pragma unroll
      for (int y = 0; y < 2; ++y) msA[y] |= ((uint32_t)wc.d[y][1] & 0xffffu) << (16 * bk);
#pragma unroll
      for (int x = 0; x < WJ; ++x) msB[x] |= (rb_[S][x][1][3] & 0xffffu) << (16 * bk);
      if constexpr (F::SH16) {   // 2 m_a (in msA), 32 d_a, s's residual r_b (SH16 above)
#pragma unroll
        for (int y = 0; y < 2; ++y) {
          msA[y] = (msA[y] & ~(0xffffu << (16 * bk))) | f16_times2((uint32_t)wc.d[y][1]) << (16 * bk);
          dsA[y] |= f16_times2(f16_times16((uint32_t)wc.d[y][0])) << (16 * bk);
        }
#pragma unroll
        for (int x = 0; x < WJ; ++x) rsB[x] |= (rb_[S][x][1][3] >> 16) << (16 * bk);
      }
      if (bk == F6_KB - 1) {
#pragma unroll
        for (int x = 0; x < WJ; ++x) {
          // k slots 0, 1: (m_a, s_b) of the two blocks, both k halves (x2 like P); q5_1: lanes 0-31
          // {s_b, s_b} x {2 m_a, 32 d_a}, lanes 32-63 {r_b, 0} x {32 d_a, 0}
          const half4 sf = F::SH16 ? __builtin_bit_cast(half4, uint2{h ? rsB[x] : msB[x], h ? 0u : msB[x]})
                                   : __builtin_bit_cast(half4, uint2{msB[x], 0u});
#pragma unroll
          for (int y = 0; y < 2; ++y) {
            const half4 mf = F::SH16 ? __builtin_bit_cast(half4, uint2{h ? dsA[y] : msA[y], h ? 0u : dsA[y]})
                                     : __builtin_bit_cast(half4, uint2{msA[y], dsA[y]});
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x8f16(sf, mf, acc[x][y], 0, 0, 0);
          }
          msB[x] = 0;
          rsB[x] = 0;
        }
        msA[0] = msA[1] = 0;
        dsA[0] = dsA[1] = 0;
      }
    }
    sb();
    // this slot's registers were read by the MFMAs above and its LDS by the ds_reads they waited
    // for: refill it P blocks ahead
    if constexpr (!CO) issue(u + P, S_);
    if constexpr (!AD) wc = wn;
  };
  if (nbw > 0) {
    // whole rounds of the ring without branches (the wait-count pass stays exact), then the
    // remaining nbw % P blocks (a multiple of KB = 2)
    unroll<P>([&](auto K) { issue(K, K); });
    if constexpr (!AD) {
      f6_wait_vm<LPB * (P - 1) + APB>();   // block 0's weight pieces
      wread(0, wc);
    }
    int u0 = 0;
    for (; u0 + P <= nbw; u0 += P) unroll<P>([&](auto K) { block(u0 + K, K); });
    unroll<P - 1>([&](auto K) {
      if (u0 + (int)K < nbw) block(u0 + K, K);
    });
  }
  if (pend) {
    f32x16& c = acc[((UPB - 1) / 2) % WJ][(UPB - 1) & 1];
#pragma unroll
    for (int e = 0; e < 16; ++e) c[e] = __builtin_fmaf(rr[(UPB - 1) % 2].s[e], rr[(UPB - 1) % 2].pr[e], c[e]);
  }
  if constexpr (AB == 1)
    if (sink == 0x9e3779b9) acc[0][0][0] = 1.f;
  // K-group epilogue (gemm_fp6_kernel's), over the rings: every wave past its last ring read
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  float* red = reinterpret_cast<float*>(smem);
  constexpr int PI = TI + 8, RPW = TJ / NW;
#pragma unroll
  for (int x = 0; x < WJ; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int i = 64 * wi + 32 * y + lr, j = 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
        red[(g * TJ + j) * PI + i] = acc[x][y][e];
      }
  __syncthreads();
  float* C = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int64_t i = (int64_t)ti * TI + 2 * lane;
  const bool pair = i + 1 < p.M && (p.ldc & 1) == 0 && ((uintptr_t)C & 7) == 0;
  // the tile's C rows through a write-through resource from the tile's first row (wave-uniform)
  const bool wt = (int64_t)TJ * p.ldc * 4 < 0x7fffffff;
  const auto cr = make_rsrc(C + (int64_t)tj * TJ * p.ldc, wt ? (uint32_t)(TJ * p.ldc * 4) : 0u);
#pragma unroll
  for (int q = 0; q < RPW; ++q) {
    const int jl = w * RPW + q;
    const int64_t j = (int64_t)tj * TJ + jl;
    f32x2 v = *reinterpret_cast<const f32x2*>(&red[jl * PI + 2 * lane]);
#pragma unroll
    for (int g_ = 1; g_ < KG; ++g_) v += *reinterpret_cast<const f32x2*>(&red[(g_ * TJ + jl) * PI + 2 * lane]);
    v *= 0.5f;
    if (j < p.N) {
      float* c = C + j * p.ldc + i;
      if (pair && wt) {
        bstore8_wt(cr, (uint32_t)((jl * p.ldc + i) * 4), v);
      } else if (pair) {
        __builtin_nontemporal_store(v, reinterpret_cast<f32x2*>(c));
      } else {
        if (i < p.M) c[0] = v[0];
        if (i + 1 < p.M) c[1] = v[1];
      }
    }
  }
}

// C[z][j][i] = sum_{s < nsplit} part[s][z][j][i], in split order; V4: 4 consecutive i per
// thread (M, ldc and the C slice strides multiples of 4, so every float4 is aligned)
template <bool V4>
__global__ __launch_bounds__(256) void f6_reduce(GemvArgs p, int nsplit, const float* __restrict__ part) {
  constexpr int W = V4 ? 4 : 1;
  const int64_t per = (int64_t)p.N * p.M, slices = (int64_t)p.ne12 * p.ne13;
  const int64_t g = ((int64_t)blockIdx.x * 256 + threadIdx.x) * W;
  if (g >= per * slices) return;
  const int64_t z = g / per, r = g % per, j = r / p.M, i = r % p.M;
  const int i12 = (int)(z % p.ne12), i13 = (int)(z / p.ne12);
  float* c = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3 + j * p.ldc + i;
  if constexpr (V4) {
    f32x4 acc = *(const f32x4*)(part + g);
    for (int s = 1; s < nsplit; ++s) acc += *(const f32x4*)(part + (int64_t)s * per * slices + g);
    *(f32x4*)c = acc;
  } else {
    float acc = part[g];
    for (int s = 1; s < nsplit; ++s) acc += part[(int64_t)s * per * slices + g];
    *c = acc;
  }
}

}  // namespace

void launch_splitk_reduce(const GemvArgs& p, int nsplit, const float* part, hipStream_t s) {
  const int64_t n = (int64_t)p.N * p.M * p.ne12 * p.ne13;
  const bool v4 = p.M % 4 == 0 && p.ldc % 4 == 0 && p.sc2 % 4 == 0 && p.sc3 % 4 == 0 && ((uintptr_t)p.C & 15) == 0;
  if (v4)
    hipLaunchKernelGGL(f6_reduce<true>, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, s, p, nsplit, part);
  else
    hipLaunchKernelGGL(f6_reduce<false>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, p, nsplit, part);
}

namespace {

// Per (device, stream) tile counters for the in-launch split-K fixup: zeroed once when made,
// left zero by every launch (the last workgroup of a tile resets its counter).  Launches on one
// stream are ordered, so one set per stream is never shared by two running launches.
constexpr size_t kTileCounters = 1 << 16;
unsigned* tile_counters(hipStream_t s) {
  static std::mutex mu;
  static std::map<std::pair<int, hipStream_t>, unsigned*> bufs;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  unsigned*& b = bufs[{dev, s}];
  if (!b) {
    if (hipMalloc(&b, kTileCounters * sizeof(unsigned)) != hipSuccess) return b = nullptr;
    if (hipMemset(b, 0, kTileCounters * sizeof(unsigned)) != hipSuccess) {
      (void)hipFree(b);
      return b = nullptr;
    }
  }
  return b;
}

// K-splits for a grid of `tiles` workgroups: double until 256 CUs have one each, keeping
// >= 8 K-steps per split, at most 16 (K=11008, 16 tiles: 8 splits 247, 16 splits 288, 21
// splits 230 TFLOP/s, profiles/r01/ab_driver_split.txt).  LAMM_FP6_SPLIT=n forces n (A/B).
int f6_nsplit_for(const GemvArgs& p, const F6Layout& L) {
  const int tiles = L.nit * L.njt * p.ne12 * p.ne13;
  int n = 1;
  if (knobs().fp6_split > 0) {
    n = knobs().fp6_split;
  } else {
    while (tiles * n < 256 && n < 16 && L.nsteps / (2 * n) >= 8) n *= 2;
  }
  return n < 1 ? 1 : (n > L.nsteps ? L.nsteps : n);
}

// Launch plan.  A grid of fewer 256x128 tiles than CUs runs 128x64 workgroup tiles with
// K-groups (F6Waves) when that fills the chip -- no split-K partials, no reduce launch -- and
// splits K otherwise.  LAMM_FP6_SUB=0 keeps split-K (A/B), =2 picks the 2-group / 32x64-wave
// form instead of the 4-group / 64x64-wave one; LAMM_FP6_SPLIT=n forces split-K with n.
struct F6Plan {
  int sub;      // 0: 256x128 tiles (+ split-K), 1: 128x64 tiles x 4 K-groups, 2: 128x64 x 2 K-groups
  int nsplit;
  int grid;
};
constexpr int kSubTilesMin = 256;
F6Plan f6_plan(const GemvArgs& p, const F6Layout& L) {
  const int tiles = L.nit * L.njt * p.ne12 * p.ne13;
  const int sub = knobs().fp6_sub;   // -1: automatic; 1 / 2 force that form (tests, A/B)
  const int64_t subt = (int64_t)((p.M + 127) / 128) * ((p.N + 63) / 64) * p.ne12 * p.ne13;
  if (knobs().fp6_split <= 0 && sub != 0 && subt < (1 << 30)) {
    if (sub > 0) return {sub == 2 ? 2 : 1, 1, (int)subt};
    if (tiles < 256 && subt >= kSubTilesMin) return {1, 1, (int)subt};
  }
  const int n = f6_nsplit_for(p, L);
  return {0, n, tiles * n};
}
int f6_nsplit(const GemvArgs& p, const F6Layout& L) { return f6_plan(p, L).nsplit; }

template <int T>
void launch_prep_w(const GemvArgs& p, unsigned char* wsA, hipStream_t s, unsigned* big_d = nullptr) {
  const F6Layout L = F6Layout::of(p);
  const int nkw = (L.nsteps * F6_KB + PW_NB - 1) / PW_NB;
  hipLaunchKernelGGL(prep_w_fp6<T>, dim3((unsigned)(((L.nit * F6_TI) / PW_ROWS) * nkw), (unsigned)L.na), dim3(PW_NT),
                     0, s, p, wsA, big_d);
}

// Workspace: [packed A (unless prepared weights are given)] [packed B] [split-K partials]
template <int T>
hipError_t launch_fp6_t(const GemvArgs& p, const void* prepA, void* ws, hipStream_t s) {
  const F6Layout L = F6Layout::of(p);
  auto* w = static_cast<unsigned char*>(ws);
  unsigned char* wsA = prepA ? nullptr : w;
  unsigned char* wsB = w + (prepA ? 0 : L.a_bytes);
#ifdef LAMM_AB_VARIANTS
  // LAMM_GEMM_SKIP_PREP=1 (variant build only): re-run the main kernel on the workspace the
  // previous identical call prepared, so its own duration can be event-timed
  const char* sp = getenv("LAMM_GEMM_SKIP_PREP");
  if (!(sp && sp[0] == '1'))
#endif
  {
    if (!prepA) launch_prep_w<T>(p, wsA, s);
    const int rgroups = (L.njt * F6_TJ + PREP_NT - 1) / PREP_NT, nb_all = L.nsteps * F6_KB;
    auto prep = [&](auto kmulti, auto kone) {
      if ((int64_t)rgroups * ((nb_all + PREP_NB - 1) / PREP_NB) * p.ne12 * p.ne13 >= 256)
        hipLaunchKernelGGL(kmulti,
                           dim3((unsigned)(rgroups * ((nb_all + PREP_NB - 1) / PREP_NB)), (unsigned)(p.ne12 * p.ne13)),
                           dim3(PREP_NT), 0, s, p, wsB);
      else
        hipLaunchKernelGGL(kone, dim3((unsigned)(rgroups * nb_all), (unsigned)(p.ne12 * p.ne13)), dim3(PREP_NT), 0, s,
                           p, wsB);
    };
    if (p.b_f32) {
      prep(prep_b_fp6<T, PREP_NB, true>, prep_b_fp6<T, 1, true>);
    } else {
      const int nbg = (nb_all + PB_NB - 1) / PB_NB, rg = (L.njt * F6_TJ + PB_ROWS - 1) / PB_ROWS;
      hipLaunchKernelGGL(prep_b_fp6_tile<T>, dim3((unsigned)(rg * nbg), (unsigned)(p.ne12 * p.ne13)), dim3(PB_NT), 0,
                         s, p, wsB);
    }
  }
  const F6Plan plan = f6_plan(p, L);
  const int nsplit = plan.nsplit;
  float* part = reinterpret_cast<float*>(wsB + (size_t)(p.ne12 * p.ne13) * (size_t)L.b_slice);
  const unsigned char* kA = prepA ? static_cast<const unsigned char*>(prepA) : wsA;
  // LAMM_FP6_FUSED_REDUCE=1: split-K partials summed inside the launch by each tile's last
  // workgroup instead of the f6_reduce launch.  Measured SLOWER on config 3 (main kernel 25.7 ->
  // 40.9 us vs 7.7 us for f6_reduce, profiles/r02/fp6_single_slice_ablation.txt): publishing
  // 128 KiB per workgroup write-through and reading three partials on only the 64 last
  // workgroups costs more than a reduce pass over all CUs.  Kept as an A/B switch.
  const int64_t tiles = (int64_t)L.nit * L.njt * p.ne12 * p.ne13;
  unsigned* ctr = nsplit > 1 && tiles <= (int64_t)kTileCounters && knobs().fp6_fused_reduce ? tile_counters(s) : nullptr;
  auto go = [&](auto kern, auto waves) {
    using WV = decltype(waves);
    const size_t lds = (size_t)WV::LDS;
    set_max_lds((const void*)kern, (int)lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)plan.grid), dim3(WV::NT), lds, s, p, kA,
                       static_cast<const unsigned char*>(wsB), nsplit, part, ctr);
  };
#ifdef LAMM_AB_VARIANTS
  const char* ev = getenv("LAMM_GEMM_VARIANT");
#endif
  if (plan.sub == 1 && knobs().fp6_av) {   // LAMM_FP6_AV=0: the LDS-staged form below
    constexpr size_t lds = (size_t)4 * 64 * (128 + 8) * 4;   // the epilogue's parked tiles
    // two blocks in flight per wave: config 3 whole launch 27.84-28.12 us against 27.94-28.34 with three
    // (q4_0; q5_0 28.22 vs 28.39; alternating processes, profiles/r06/kv_p/); the affine formats and
    // q8_0 spill with three.  LAMM_FP6_KV_P=3: three (A/B, q4_0 / q5_0 only)
    constexpr bool P3OK = !F6<T>::AFF && F6<T>::WP == 1;
    auto kern = knobs().fp6_kv_p == 3 && P3OK ? gemm_fp6_kv_kernel<T, P3OK ? 3 : 2> : gemm_fp6_kv_kernel<T, 2>;
    set_max_lds((const void*)kern, (int)lds);
    hipLaunchKernelGGL(kern, dim3((unsigned)plan.grid), dim3(512), lds, s, p, kA, static_cast<const unsigned char*>(wsB));
    return hipGetLastError();
  }
  if constexpr (F6<T>::WP == 2) {
    return hipErrorInvalidValue;   // q8_0: the K-group plan only (f6_kv_plan)
  } else {
  if (plan.sub == 1) {
    using WK = F6Waves<2, 2, 2, 4>;
#ifdef LAMM_AB_VARIANTS
    // ablations of the K-group form (variant build, q4_0 only, tools/ab_kg.sh,
    // profiles/r02/fp6_kgroups_ablation.txt): 1 no compute, 2 no DMA, 3 no epilogue FMAs,
    // 4 no DMA + no LDS fragment reads, 6 no P-MFMA, 7 no S-MFMA, 11 DMA but no LDS fragment
    // reads; 20 + V: in-kernel clock probe of V
    switch (T == kQ4_0 && ev ? atoi(ev) : 0) {
      case 1: go(gemm_fp6_kernel<T, 1, 2, 2, 2, 4>, WK{}); break;
      case 2: go(gemm_fp6_kernel<T, 2, 2, 2, 2, 4>, WK{}); break;
      case 3: go(gemm_fp6_kernel<T, 3, 2, 2, 2, 4>, WK{}); break;
      case 4: go(gemm_fp6_kernel<T, 4, 2, 2, 2, 4>, WK{}); break;
      case 6: go(gemm_fp6_kernel<T, 6, 2, 2, 2, 4>, WK{}); break;
      case 7: go(gemm_fp6_kernel<T, 7, 2, 2, 2, 4>, WK{}); break;
      case 20: go(gemm_fp6_kernel<T, 20, 2, 2, 2, 4>, WK{}); break;
      case 21: go(gemm_fp6_kernel<T, 21, 2, 2, 2, 4>, WK{}); break;
      case 22: go(gemm_fp6_kernel<T, 22, 2, 2, 2, 4>, WK{}); break;
      case 24: go(gemm_fp6_kernel<T, 24, 2, 2, 2, 4>, WK{}); break;
      case 11: go(gemm_fp6_kernel<T, 11, 2, 2, 2, 4>, WK{}); break;
      case 31: go(gemm_fp6_kernel<T, 31, 2, 2, 2, 4>, WK{}); break;
      default: go(gemm_fp6_kernel<T, 0, 2, 2, 2, 4>, WK{});
    }
#else
    go(gemm_fp6_kernel<T, 0, 2, 2, 2, 4>, WK{});
#endif
    return hipGetLastError();
  }
  if (plan.sub == 2) {
    go(gemm_fp6_kernel<T, 0, 1, 2, 2, 2>, F6Waves<1, 2, 2, 2>{});
    return hipGetLastError();
  }
  using W2 = F6Waves<2>;
  if (knobs().fp6_wj == 1) {   // A/B: 16 waves of 32x64
    go(gemm_fp6_kernel<T, 0, 1>, F6Waves<1>{});
  } else {
#ifdef LAMM_AB_VARIANTS
  switch (ev ? atoi(ev) : 0) {
    case 1: go(gemm_fp6_kernel<T, 1, 2>, W2{}); break;
    case 2: go(gemm_fp6_kernel<T, 2, 2>, W2{}); break;
    case 3: go(gemm_fp6_kernel<T, 3, 2>, W2{}); break;
    case 5: go(gemm_fp6_kernel<T, 5, 2>, W2{}); break;
    case 6: go(gemm_fp6_kernel<T, 6, 2>, W2{}); break;
    case 7: go(gemm_fp6_kernel<T, 7, 2>, W2{}); break;
    case 8: go(gemm_fp6_kernel<T, 8, 2>, W2{}); break;
    case 10: go(gemm_fp6_kernel<T, 10, 2>, W2{}); break;
    case 12: go(gemm_fp6_kernel<T, 12, 2>, W2{}); break;
    default: go(gemm_fp6_kernel<T, 0, 2>, W2{});
  }
#else
  go(gemm_fp6_kernel<T, 0, 2>, W2{});
#endif
  }
  if (nsplit > 1 && !ctr) launch_splitk_reduce(p, nsplit, part, s);
  return hipGetLastError();
  }
}

}  // namespace

bool gemm_fp6_kv_plan(const GemvArgs& p) {
  const F6Plan plan = f6_plan(p, F6Layout::of(p));
  return plan.sub == 1 && knobs().fp6_av;
}

bool gemm_fp6_supported(int type) {
  return type == kQ4_0 || type == kQ4_1 || type == kQ5_0 || type == kQ5_1 || type == kQ8_0;
}

int gemm_fp6_tiles(const GemvArgs& p) {
  const F6Layout L = F6Layout::of(p);
  return L.nit * L.njt * p.ne12 * p.ne13;
}

int gemm_fp6_grid(const GemvArgs& p) {
  const F6Layout L = F6Layout::of(p);
  return f6_plan(p, L).grid;
}

size_t gemm_fp6_workspace_bytes(int type, const GemvArgs& p, bool prepared) {
  const F6Layout L = F6Layout::of(p, type == kQ8_0 ? 2 : 1);
  const int nsplit = f6_nsplit(p, L);
  // split-K partials: C-shaped for f6_reduce, or whole 256 x 128 tiles for the in-launch fixup
  const size_t tiles = (size_t)L.nit * L.njt * p.ne12 * p.ne13;
  const size_t per_split = std::max((size_t)p.ne12 * p.ne13 * (size_t)p.N * p.M, tiles * F6_TI * F6_TJ);
  const size_t part = nsplit > 1 ? (size_t)nsplit * per_split * sizeof(float) : 0;
  return (prepared ? 0 : (size_t)L.a_bytes) + (size_t)(p.ne12 * p.ne13) * (size_t)L.b_slice + part + 256;
}

size_t gemm_fp6_weight_bytes(int type, const GemvArgs& p) {
  return (size_t)F6Layout::of(p, type == kQ8_0 ? 2 : 1).a_bytes;
}

hipError_t prepare_fp6_weights(int type, const GemvArgs& p, void* wsA, hipStream_t s, bool* in_range) {
  auto* w = static_cast<unsigned char*>(wsA);
  if (in_range) *in_range = true;
  switch (type) {
    case kQ4_0: launch_prep_w<kQ4_0>(p, w, s); break;
    case kQ4_1: launch_prep_w<kQ4_1>(p, w, s); break;
    case kQ5_0: launch_prep_w<kQ5_0>(p, w, s); break;
    case kQ8_0: launch_prep_w<kQ8_0>(p, w, s); break;
    case kQ5_1: {   // reports block scales past 16 d's f16 range (the packed form is then unusable)
      unsigned* flag = nullptr;
      if (hipMalloc(&flag, sizeof(unsigned)) != hipSuccess) return hipErrorOutOfMemory;
      unsigned h = 0;
      hipError_t e = hipMemsetAsync(flag, 0, sizeof(unsigned), s);
      if (e == hipSuccess) {
        launch_prep_w<kQ5_1>(p, w, s, flag);
        e = hipGetLastError();
      }
      if (e == hipSuccess) e = hipMemcpyAsync(&h, flag, sizeof(unsigned), hipMemcpyDeviceToHost, s);
      if (e == hipSuccess) e = hipStreamSynchronize(s);
      (void)hipFree(flag);
      if (in_range) *in_range = h == 0;
      return e;
    }
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_gemm_fp6(int type, const GemvArgs& p, const void* prepA, void* ws, hipStream_t s) {
  switch (type) {
    case kQ4_0: return launch_fp6_t<kQ4_0>(p, prepA, ws, s);
    case kQ4_1: return launch_fp6_t<kQ4_1>(p, prepA, ws, s);
    case kQ5_0: return launch_fp6_t<kQ5_0>(p, prepA, ws, s);
    case kQ5_1:   // prepared (range-checked) weights only: the per-call form has no range check
      if (!prepA) return hipErrorInvalidValue;
      return launch_fp6_t<kQ5_1>(p, prepA, ws, s);
    case kQ8_0:   // prepared weights (the two code planes) and the K-group plan only
      if (!prepA || !gemm_fp6_kv_plan(p)) return hipErrorInvalidValue;
      return launch_fp6_t<kQ8_0>(p, prepA, ws, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
