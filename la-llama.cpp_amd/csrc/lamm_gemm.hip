// lamm_gemm.hip -- prefill-shaped (N > 8) quantized GEMM on the MFMA-i8 matrix cores.
//
// Same contract as the lamm block kernels (src/lamm_kernel_*.hpp via
// LAMMImpl<T>::matmul_simd_block, src/lamm_impl.hpp:90-147): C[j*ldc+i] = A_i . B_j.
//
// Orientation: the MFMA's row dimension is the activation index j (B columns) and its
// column dimension is the weight row i, so each lane owns one i and the C stores are
// 128-byte row segments.  One workgroup = 4 waves = a 128(j) x 64(i) tile; each wave
// owns 64(j) x 32(i) = two 32x32 MFMA tiles.
//
// Per K-step (8 blocks = 256 elements):
//   1. raw block_q* bytes of A (64 rows) and B (128 rows) -> LDS with coalesced 16-byte
//      buffer loads (AoS as stored in HBM, no repack);
//   2. unpack to int8 in LDS: q4_0 -> q-8, q5_0 -> q-16 (5th bit from qh), q4_1/q5_1 ->
//      0..31, q8_0 as is; scales to fp32 (d) / fp16 (m, s);
//   3. per block: v_mfma_i32_32x32x32_i8 (K = 32 = exactly one block) gives the exact
//      int32 block dots S; the epilogue applies the block scales in fp32:
//      acc += (d_a * d_b) * float(S).  For q4_1/q5_1 the m_a * s_b term is a rank-8
//      product per K-step, done exactly on v_mfma_f32_32x32x8_f16 (fp16 x fp16 products
//      are exact in fp32).
// q2_K (256-element super-blocks) has its own kernel: the 4-bit sub-block scale is
// folded into the int8 A operand (q2 * sc <= 45), 8 chained i8 MFMAs give one exact
// int32 per super-block, and the min term sum_s mn_s * bsums_s is one
// v_mfma_f32_32x32x16_f16 (K = 16 sub-blocks, exact).
#include "lamm_device.h"
#include "lamm_kernels.h"

namespace lamm {
namespace {

typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int GT = 256;    // threads per workgroup
constexpr int TJ = 128;    // activation rows per tile
constexpr int TI = 64;     // weight rows per tile
constexpr int KBLK = 8;    // 32-element blocks per K-step
constexpr int ROWB = KBLK * 32 + 16;   // unpacked int8 row pitch (272 B): conflict-free b128 reads

template <int T> struct GF;
template <> struct GF<kQ4_0> { static constexpr int ABPB = 18, VBPB = 34; };
template <> struct GF<kQ4_1> { static constexpr int ABPB = 20, VBPB = 36; };
template <> struct GF<kQ5_0> { static constexpr int ABPB = 22, VBPB = 34; };
template <> struct GF<kQ5_1> { static constexpr int ABPB = 24, VBPB = 36; };
template <> struct GF<kQ8_0> { static constexpr int ABPB = 34, VBPB = 34; };

// ---- 32-element block formats ----------------------------------------------------
// 512 threads = 8 waves laid out 4 (j) x 2 (i); each wave owns one 32x32 MFMA tile.
constexpr int GT8 = 512;

template <int T>
struct GemmSmem {
  static constexpr int RA = TI * KBLK * GF<T>::ABPB;   // raw A bytes per K-step
  static constexpr int RB = TJ * KBLK * GF<T>::VBPB;   // raw B bytes per K-step
  static constexpr int RA_PIECES = RA / 16, RB_PIECES = RB / 16;
  static constexpr int RA_NPT = (RA_PIECES + GT8 - 1) / GT8, RB_NPT = (RB_PIECES + GT8 - 1) / GT8;
  uint32_t rawA[RA_NPT * GT8 * 4 + 4];
  uint32_t rawB[RB_NPT * GT8 * 4 + 4];
  uint32_t wt[TI * ROWB / 4];
  uint32_t act[TJ * ROWB / 4];
  _Float16 dah[KBLK][TI];       // fp16 scales, exactly as stored in the blocks
  _Float16 dbh[KBLK][TJ];
  _Float16 mah[TI][KBLK];
  _Float16 sbh[TJ][KBLK];
};

__device__ __forceinline__ uint32_t sub_bytes(uint32_t x, uint32_t off4) {
  // per-byte x - off (x < 0x80 per byte): no borrow crosses a byte
  return ((x | 0x80808080u) - off4) ^ 0x80808080u;
}

// Read NW dwords of an (only 2-byte aligned) block from LDS, realigned to its first byte.
template <int NW>
__device__ __forceinline__ void lds_block(const uint32_t* base, int byte_off, uint32_t (&m)[NW]) {
  const uint32_t* p = base + (byte_off >> 2);
  const int sh = (byte_off & 3) * 8;
  uint32_t w[NW + 1];
#pragma unroll
  for (int k = 0; k <= NW; ++k) w[k] = p[k];
#pragma unroll
  for (int k = 0; k < NW; ++k) m[k] = __builtin_amdgcn_alignbit(w[k + 1], w[k], sh);
}

template <int T>
__device__ __forceinline__ void unpack_weight(const uint32_t (&m)[(GF<T>::ABPB + 3) / 4], uint32_t (&q)[8]) {
  if constexpr (T == kQ8_0) {
    unroll<8>([&](auto K) { q[K] = get32<2 + 4 * K>(m); });
  } else {
    constexpr bool AFF = (T == kQ4_1 || T == kQ5_1);
    constexpr bool FIVE = (T == kQ5_0 || T == kQ5_1);
    constexpr int QS = (AFF ? 4 : 2) + (FIVE ? 4 : 0);
    uint32_t qh = 0;
    if constexpr (FIVE) qh = get32<AFF ? 4 : 2>(m);
    unroll<4>([&](auto K) {
      constexpr int k = K;
      const uint32_t x = get32<QS + 4 * k>(m);
      uint32_t lo = x & 0x0f0f0f0fu, hi = (x >> 4) & 0x0f0f0f0fu;
      if constexpr (FIVE) {
        lo |= spread4_hi((qh >> (4 * k)) & 0xf);
        hi |= spread4_hi((qh >> (16 + 4 * k)) & 0xf);
      }
      if constexpr (T == kQ4_0) { lo = sub_bytes(lo, 0x08080808u); hi = sub_bytes(hi, 0x08080808u); }
      if constexpr (T == kQ5_0) { lo = sub_bytes(lo, 0x10101010u); hi = sub_bytes(hi, 0x10101010u); }
      q[k] = lo;
      q[4 + k] = hi;
    });
  }
}

template <int T>
__global__ __launch_bounds__(GT8) void gemm_kernel(GemvArgs p) {
  using S = GemmSmem<T>;
  constexpr int ABPB = GF<T>::ABPB, VBPB = GF<T>::VBPB;
  constexpr bool AFF = (T == kQ4_1 || T == kQ5_1);
  constexpr int APR = KBLK * ABPB / 16, BPR = KBLK * VBPB / 16;   // 16-byte pieces per row
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  S& sm = *reinterpret_cast<S*>(smem_raw);

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int lr = lane & 31, h = lane >> 5;
  const int wj = w >> 1, wi = w & 1;             // wave tile: rows jb..jb+31, cols ib..ib+31
  const int jb = 32 * wj, ib = 32 * wi;
  const int64_t i0 = (int64_t)blockIdx.x * TI, j0 = (int64_t)blockIdx.y * TJ;
  const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3 + i0 * p.lda;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3 + j0 * p.ldb;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int rowsA = (int)min((int64_t)TI, (int64_t)p.M - i0);
  const int rowsB = (int)min((int64_t)TJ, (int64_t)p.N - j0);
  const int64_t a_end = (int64_t)(rowsA - 1) * p.lda + (int64_t)p.nblk * ABPB;   // bytes readable from Az
  const int64_t b_end = (int64_t)(rowsB - 1) * p.ldb + (int64_t)p.nblk * VBPB;

  // per-thread piece offsets within a K-step (constant over K)
  uint32_t aoff[S::RA_NPT], boff[S::RB_NPT];
#pragma unroll
  for (int k = 0; k < S::RA_NPT; ++k) {
    const int pc = t + k * GT8, rr = pc / APR, oo = pc % APR;
    aoff[k] = (pc < S::RA_PIECES && rr < rowsA) ? (uint32_t)(rr * p.lda + 16 * oo) : 0x7ffffff0u;
  }
#pragma unroll
  for (int k = 0; k < S::RB_NPT; ++k) {
    const int pc = t + k * GT8, rr = pc / BPR, oo = pc % BPR;
    boff[k] = (pc < S::RB_PIECES && rr < rowsB) ? (uint32_t)(rr * p.ldb + 16 * oo) : 0x7ffffff0u;
  }

  u32x4 va[S::RA_NPT], vb[S::RB_NPT];
  auto issue = [&](int ks) {   // global -> registers for K-step ks (OOB reads return 0)
    const int64_t ka = (int64_t)ks * KBLK * ABPB, kbb = (int64_t)ks * KBLK * VBPB;
    const auto ra = make_rsrc(Az + ka, (uint32_t)min((a_end - ka + 3) & ~int64_t(3), (int64_t)0x7fffffff));
    const auto rb = make_rsrc(Bz + kbb, (uint32_t)min((b_end - kbb + 3) & ~int64_t(3), (int64_t)0x7fffffff));
#pragma unroll
    for (int k = 0; k < S::RA_NPT; ++k) va[k] = bload16(ra, aoff[k]);
#pragma unroll
    for (int k = 0; k < S::RB_NPT; ++k) vb[k] = bload16(rb, boff[k]);
  };

  f32x16 acc, macc;
#pragma unroll
  for (int e = 0; e < 16; ++e) { acc[e] = 0.f; macc[e] = 0.f; }

  const int nsteps = (p.nblk + KBLK - 1) / KBLK;
  issue(0);
  for (int ks = 0; ks < nsteps; ++ks) {
    const int kb0 = ks * KBLK;
    // ---- registers (loaded during the previous step's MFMAs) -> raw LDS ----
#pragma unroll
    for (int k = 0; k < S::RA_NPT; ++k) *(u32x4*)&sm.rawA[4 * (t + k * GT8)] = va[k];
#pragma unroll
    for (int k = 0; k < S::RB_NPT; ++k) *(u32x4*)&sm.rawB[4 * (t + k * GT8)] = vb[k];
    __syncthreads();
    // ---- unpack to int8 + fp16 scales (one item = one (row, block)) ----
    for (int it = t; it < TI * KBLK; it += GT8) {
      const int il = it / KBLK, b = it % KBLK;
      uint32_t m[(ABPB + 3) / 4], q[8];
      lds_block(sm.rawA, il * KBLK * ABPB + b * ABPB, m);
      unpack_weight<T>(m, q);
      const bool ok = il < rowsA && kb0 + b < p.nblk;
      u32x4* dst = (u32x4*)&sm.wt[(il * ROWB + 32 * b) / 4];
      dst[0] = ok ? u32x4{q[0], q[1], q[2], q[3]} : u32x4{0, 0, 0, 0};
      dst[1] = ok ? u32x4{q[4], q[5], q[6], q[7]} : u32x4{0, 0, 0, 0};
      sm.dah[b][il] = __builtin_bit_cast(_Float16, (uint16_t)(ok ? (m[0] & 0xffff) : 0));
      if constexpr (AFF) sm.mah[il][b] = __builtin_bit_cast(_Float16, (uint16_t)(ok ? (m[0] >> 16) : 0));
    }
    for (int it = t; it < TJ * KBLK; it += GT8) {
      const int jl = it / KBLK, b = it % KBLK;
      uint32_t m[(VBPB + 3) / 4];
      lds_block(sm.rawB, jl * KBLK * VBPB + b * VBPB, m);
      constexpr int VQS = VBPB == 36 ? 4 : 2;
      const bool ok = jl < rowsB && kb0 + b < p.nblk;
      u32x4* dst = (u32x4*)&sm.act[(jl * ROWB + 32 * b) / 4];
      dst[0] = ok ? u32x4{get32<VQS>(m), get32<VQS + 4>(m), get32<VQS + 8>(m), get32<VQS + 12>(m)} : u32x4{0, 0, 0, 0};
      dst[1] = ok ? u32x4{get32<VQS + 16>(m), get32<VQS + 20>(m), get32<VQS + 24>(m), get32<VQS + 28>(m)}
                  : u32x4{0, 0, 0, 0};
      sm.dbh[b][jl] = __builtin_bit_cast(_Float16, (uint16_t)(ok ? (m[0] & 0xffff) : 0));
      if constexpr (AFF) sm.sbh[jl][b] = __builtin_bit_cast(_Float16, (uint16_t)(ok ? (m[0] >> 16) : 0));
    }
    __syncthreads();
    // ---- next step's global loads fly during this step's MFMAs ----
    if (ks + 1 < nsteps) issue(ks + 1);
    // ---- MFMA: exact int32 block dots; d_a*d_b on the fp16 MFMA; acc += P * S ----
#pragma unroll 2
    for (int b = 0; b < KBLK; ++b) {
      const i32x4 wf = *(const i32x4*)&sm.wt[((ib + lr) * ROWB + 32 * b + 16 * h) / 4];
      const i32x4 af = *(const i32x4*)&sm.act[((jb + lr) * ROWB + 32 * b + 16 * h) / 4];
      const i32x16 zero = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
      const i32x16 sdot = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, wf, zero, 0, 0, 0);
      // outer product d_b[j] * d_a[i] (k = 0 only): fp16 x fp16 is exact in fp32
      const _Float16 hz = (_Float16)0.f;
      const half8 dbv = {h == 0 ? sm.dbh[b][jb + lr] : hz, hz, hz, hz, hz, hz, hz, hz};
      const half8 dav = {h == 0 ? sm.dah[b][ib + lr] : hz, hz, hz, hz, hz, hz, hz, hz};
      const f32x16 fz = {};
      const f32x16 sc = __builtin_amdgcn_mfma_f32_32x32x16_f16(dbv, dav, fz, 0, 0, 0);
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] = __builtin_fmaf((float)sdot[r], sc[r], acc[r]);
    }
    if constexpr (AFF) {
      // sum_b m_a[i,b] * s_b[j,b] over this K-step's 8 blocks: one exact fp16 MFMA
      const half4 mf = *(const half4*)&sm.mah[ib + lr][4 * h];
      const half4 sf = *(const half4*)&sm.sbh[jb + lr][4 * h];
      macc = __builtin_amdgcn_mfma_f32_32x32x8f16(sf, mf, macc, 0, 0, 0);
    }
    __syncthreads();
  }

  // ---- epilogue: C[j*ldc + i], lanes own i (128-byte segments) ----
  const int64_t i = i0 + ib + lr;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int64_t j = j0 + jb + (r & 3) + 8 * (r >> 2) + 4 * h;
    if (i < p.M && j < p.N) Cz[j * p.ldc + i] = acc[r] + (AFF ? macc[r] : 0.f);
  }
}

// ------------------------------------------------------------------ q2_K x q8_K
constexpr int QK2_RAWA = TI * 84, QK2_RAWB = TJ * 292;
struct Q2KSmem {
  uint32_t rawA[(QK2_RAWA / 16 + GT - 1) / GT * GT * 4 + 4];
  uint32_t rawB[(QK2_RAWB / 16 + GT - 1) / GT * GT * 4 + 4];
  uint32_t wt[TI * ROWB / 4];     // q2 * (sc & 15), 256 int8 per row
  uint32_t act[TJ * ROWB / 4];    // q8_K quants
  float da[TI], dmn[TI], yd[TJ];
  _Float16 mn[TI][16];            // sc >> 4
  _Float16 bs[TJ][16];            // bsums (|bsum| <= 2032: exact in fp16)
};

__global__ __launch_bounds__(GT) void gemm_q2k_kernel(GemvArgs p) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  Q2KSmem& sm = *reinterpret_cast<Q2KSmem*>(smem_raw);
  constexpr int RA_P = QK2_RAWA / 16, RB_P = QK2_RAWB / 16;
  constexpr int RA_NPT = (RA_P + GT - 1) / GT, RB_NPT = (RB_P + GT - 1) / GT;

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int lr = lane & 31, h = lane >> 5;
  const int wj = w >> 1, wi = w & 1;
  const int64_t i0 = (int64_t)blockIdx.x * TI, j0 = (int64_t)blockIdx.y * TJ;
  const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int rowsA = (int)min((int64_t)TI, (int64_t)p.M - i0);
  const int rowsB = (int)min((int64_t)TJ, (int64_t)p.N - j0);

  f32x16 acc[2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;

  for (int sb = 0; sb < p.nblk; ++sb) {
    {
      // raw rows: A 84 B/row (pieces may straddle rows: gather by dword), B 292 B/row
      const unsigned char* abase = Az + i0 * p.lda + (int64_t)sb * 84;
      const int64_t avail = (int64_t)(rowsA - 1) * p.lda + (int64_t)(p.nblk - sb) * 84;
      const auto ra = make_rsrc(abase, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
      const unsigned char* bbase = Bz + j0 * p.ldb + (int64_t)sb * 292;
      const int64_t bavail = (int64_t)(rowsB - 1) * p.ldb + (int64_t)(p.nblk - sb) * 292;
      const auto rb = make_rsrc(bbase, (uint32_t)min((bavail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
      uint32_t va[RA_NPT * 4], vb[RB_NPT * 4];
#pragma unroll
      for (int k = 0; k < RA_NPT * 4; ++k) {
        const int dw = t + k * GT;                // dword index in the packed [TI][84] image
        const int rr = dw / 21, oo = dw % 21;
        const uint32_t off = (dw < TI * 21 && rr < rowsA) ? (uint32_t)(rr * p.lda + 4 * oo) : 0x7ffffff0u;
        va[k] = bload4(ra, off);
      }
#pragma unroll
      for (int k = 0; k < RB_NPT * 4; ++k) {
        const int dw = t + k * GT;                // [TJ][73]
        const int rr = dw / 73, oo = dw % 73;
        const uint32_t off = (dw < TJ * 73 && rr < rowsB) ? (uint32_t)(rr * p.ldb + 4 * oo) : 0x7ffffff0u;
        vb[k] = bload4(rb, off);
      }
#pragma unroll
      for (int k = 0; k < RA_NPT * 4; ++k) sm.rawA[t + k * GT] = va[k];
#pragma unroll
      for (int k = 0; k < RB_NPT * 4; ++k) sm.rawB[t + k * GT] = vb[k];
    }
    __syncthreads();
    // unpack A: 64 rows x 16 sub-blocks; a = q2 * (sc & 15), element order of
    // src/lamm_kernel_q2_k.hpp:52-71 (element n*128 + jj*32 + l, sub-block 8n+2jj+(l>=16))
    for (int it = t; it < TI * 16; it += GT) {
      const int il = it / 16, s = it % 16;
      const uint32_t* blk = &sm.rawA[il * 21];
      const int n = s >> 3, jj = (s >> 1) & 3, hh = s & 1;
      const uint32_t scw = blk[s >> 2];
      const int sc = (scw >> (8 * (s & 3))) & 0xff;
      const uint32_t mul = (uint32_t)(sc & 15) * 0x01010101u;
      uint32_t q[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t x = (blk[4 + 8 * n + 4 * hh + k] >> (2 * jj)) & 0x03030303u;
        q[k] = x * (uint32_t)(sc & 15);            // per byte <= 45: no carries
      }
      (void)mul;
      const bool ok = il < rowsA;
      // element e = n*128 + jj*32 + hh*16 + 0..15  -> int8 offset e in the row
      *(u32x4*)&sm.wt[(il * ROWB + n * 128 + jj * 32 + hh * 16) / 4] = ok ? u32x4{q[0], q[1], q[2], q[3]}
                                                                            : u32x4{0, 0, 0, 0};
      sm.mn[il][s] = ok ? (_Float16)(float)(sc >> 4) : (_Float16)0.f;
      if (s == 0) {
        sm.da[il] = ok ? h2f(blk[20] & 0xffff) : 0.f;
        sm.dmn[il] = ok ? h2f(blk[20] >> 16) : 0.f;
      }
    }
    for (int it = t; it < TJ * 16; it += GT) {
      const int jl = it / 16, q16 = it % 16;
      const uint32_t* blk = &sm.rawB[jl * 73];
      const bool ok = jl < rowsB;
      *(u32x4*)&sm.act[(jl * ROWB + 16 * q16) / 4] =
          ok ? u32x4{blk[1 + 4 * q16], blk[2 + 4 * q16], blk[3 + 4 * q16], blk[4 + 4 * q16]} : u32x4{0, 0, 0, 0};
      const uint32_t bw = blk[65 + (q16 >> 1)];
      sm.bs[jl][q16] = ok ? (_Float16)(float)(int16_t)((q16 & 1) ? (bw >> 16) : (bw & 0xffff)) : (_Float16)0.f;
      if (q16 == 0) sm.yd[jl] = ok ? __builtin_bit_cast(float, blk[0]) : 0.f;
    }
    __syncthreads();
    // 8 chained i8 MFMAs = exact int32 super-block dot; min term via one fp16 MFMA
    const float dai = sm.da[32 * wi + lr], dmi = sm.dmn[32 * wi + lr];
    const half8 mnf = *(const half8*)&sm.mn[32 * wi + lr][8 * h];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int jb = 64 * wj + 32 * rt;
      i32x16 s = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const i32x4 wf = *(const i32x4*)&sm.wt[((32 * wi + lr) * ROWB + 32 * kk + 16 * h) / 4];
        const i32x4 af = *(const i32x4*)&sm.act[((jb + lr) * ROWB + 32 * kk + 16 * h) / 4];
        s = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, wf, s, 0, 0, 0);
      }
      const half8 bsf = *(const half8*)&sm.bs[jb + lr][8 * h];
      f32x16 zero = {};
      const f32x16 mins = __builtin_amdgcn_mfma_f32_32x32x16_f16(bsf, mnf, zero, 0, 0, 0);
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 ydv = *(const f32x4*)&sm.yd[jb + 8 * g + 4 * h];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          acc[rt][r] += (ydv[e] * dai) * (float)s[r] - (ydv[e] * dmi) * mins[r];
        }
      }
    }
    __syncthreads();
  }

  const int64_t i = i0 + 32 * wi + lr;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t j = j0 + 64 * wj + 32 * rt + (r & 3) + 8 * (r >> 2) + 4 * h;
      if (i < p.M && j < p.N) Cz[j * p.ldc + i] = acc[rt][r];
    }
}

template <class K>
hipError_t launch_with(K kern, size_t lds, int threads, const GemvArgs& p, hipStream_t s) {
  const dim3 grid((unsigned)((p.M + TI - 1) / TI), (unsigned)((p.N + TJ - 1) / TJ), (unsigned)(p.ne12 * p.ne13));
  (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(kern, grid, dim3(threads), lds, s, p);
  return hipGetLastError();
}

}  // namespace

bool gemm_supported(int type) {
  return type == kQ4_0 || type == kQ4_1 || type == kQ5_0 || type == kQ5_1 || type == kQ8_0 || type == kQ2_K;
}

bool gemm_args_ok(int type, const GemvArgs& p) {
  // B rows are staged with 16-byte (32-block formats) or 4-byte (q8_K) loads
  const int64_t a = type == kQ2_K ? 4 : 16;
  return (p.ldb % a) == 0 && ((uintptr_t)p.B % a) == 0 && (p.sb2 % a) == 0 && (p.sb3 % a) == 0;
}

hipError_t launch_gemm(int type, const GemvArgs& p, hipStream_t s) {
  switch (type) {
    case kQ4_0: return launch_with(gemm_kernel<kQ4_0>, sizeof(GemmSmem<kQ4_0>), GT8, p, s);
    case kQ4_1: return launch_with(gemm_kernel<kQ4_1>, sizeof(GemmSmem<kQ4_1>), GT8, p, s);
    case kQ5_0: return launch_with(gemm_kernel<kQ5_0>, sizeof(GemmSmem<kQ5_0>), GT8, p, s);
    case kQ5_1: return launch_with(gemm_kernel<kQ5_1>, sizeof(GemmSmem<kQ5_1>), GT8, p, s);
    case kQ8_0: return launch_with(gemm_kernel<kQ8_0>, sizeof(GemmSmem<kQ8_0>), GT8, p, s);
    case kQ2_K: return launch_with(gemm_q2k_kernel, sizeof(Q2KSmem), GT, p, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
