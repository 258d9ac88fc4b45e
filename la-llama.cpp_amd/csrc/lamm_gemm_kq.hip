// lamm_gemm_kq.hip -- prefill GEMM (N > 8) for the super-block weights q4_K / q5_K / q6_K
// (§8f; vec_dot LC/ggml-quants.c:7301-7358 q4_K, :7968-8029 q5_K, :8695-8738 q6_K) and the
// reference's own q2_K (src/lamm_kernel_q2_k.hpp:28-307), against q8_K activations.  Without
// it the §8f formats ran as N/8 grouped GEMV launches (~30x slower); q2_K had the simpler
// single-pass kernel of lamm_gemm.hip (still reachable with LAMM_KQ_GEMM=0).
//
// Per 256-element super-block the reference computes exact integer sub-block dots, scales
// them by the INTEGER 6-bit (q4_K/q5_K) or int8 (q6_K) sub-block scales, and applies the fp16
// super-block scale(s) once:
//   q4_K/q5_K:  d_b * ( d_a * sum_e sc(e) q(e) b(e)  -  dmin_a * sum_s m_s * bsum_s )
//   q6_K:       d_b *   d_a * sum_e sc(e) (q(e) - 32) b(e)
// Folding the integer scale into the weight operand makes the whole super-block ONE exact
// integer dot: A'(e) = sc(e) * q(e) (<= 1953; q2_K: <= 45) or sc(e) * (q(e) - 32) (|.| <= 4096).
// A' does not fit int8 (except q2_K's), so it is split exactly as A' = 128 * hi + lo, lo = A' & 127 in [0, 127],
// hi = A' >> 7 in [-32, 31]: two chains of 8 v_mfma_i32_32x32x32_i8 (K = 32 each) per 32x32
// tile and super-block give S = 128 * S_hi + S_lo bit-exactly (|S| < 2^28).  The min term is
// one v_mfma_f32_32x32x16_f16 over the 16 q8_K bsums (|bsum| <= 2048 and m <= 63: exact in
// fp16, products and sums exact in fp32).  Only the final fp32 scaling differs in rounding
// order from the reference (d_b is f32, d_a / dmin fp16).
//
// Two kernels, both 256 threads = 4 waves as 2 (j) x 2 (i), tile 128 (j) x 64 (i), one
// super-block per step, each wave 2 tiles:
//   gemm_kq_kernel (default): prep passes write the int8 planes / scales as the kernel's LDS
//     image (weights once for stationary callers), a double-buffered LDS-DMA ring feeds the
//     MFMA chains;
//   gemm_kq_simple_kernel (LAMM_KQ_VARIANT=1): stages raw A / q8_K rows into LDS with dword
//     loads and unpacks them in place every step (no workspace).
#include <cstdlib>

#include "lamm_device.h"
#include "lamm_kernels.h"
#include "lamm_knobs.h"

namespace lamm {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int KQ_T = 256;              // threads
constexpr int KQ_TI = 64, KQ_TJ = 128;
constexpr int KQ_ROWB = 256 + 16;      // int8 plane row pitch: conflict-free b128 reads

template <int T> struct KQ;
// HI: A' needs the hi plane (q2_K: q * sc <= 45 fits int8, one MFMA chain)
template <> struct KQ<kQ4_K> { static constexpr int ABPB = 144; static constexpr bool MIN = true, HI = true; };
template <> struct KQ<kQ5_K> { static constexpr int ABPB = 176; static constexpr bool MIN = true, HI = true; };
template <> struct KQ<kQ6_K> { static constexpr int ABPB = 210; static constexpr bool MIN = false, HI = true; };
template <> struct KQ<kQ2_K> { static constexpr int ABPB = 84; static constexpr bool MIN = true, HI = false; };

template <int T>
struct KQSmem {
  static constexpr int RAWW = KQ<T>::ABPB / 4 + 1;           // dwords per staged A row (+1: q6_K is 2-aligned)
  uint32_t rawA[((KQ_TI * RAWW + KQ_T - 1) / KQ_T) * KQ_T];
  uint32_t rawB[((KQ_TJ * 73 + KQ_T - 1) / KQ_T) * KQ_T];  // q8_K: f32 d | 256 x i8 | 16 x i16 = 73 dwords
  uint32_t wlo[KQ_TI * KQ_ROWB / 4];
  uint32_t whi[KQ_TI * KQ_ROWB / 4];
  uint32_t act[KQ_TJ * KQ_ROWB / 4];
  float da[KQ_TI], dmn[KQ_TI], yd[KQ_TJ];
  _Float16 mn[KQ_TI][16];   // m of the 32-sub-block each 16-element bsum belongs to
  _Float16 bs[KQ_TJ][16];
};

// scales / mins of sub-block j (0..7) from the 12 packed bytes (LC/ggml-quants.c
// get_scale_min_k4, as the utmp shuffle of the vec_dot)
__device__ __forceinline__ void kq_sm(const uint32_t (&u)[3], int j, int& sc, int& m) {
  auto byte = [&](int b) { return (int)((u[b >> 2] >> (8 * (b & 3))) & 0xffu); };
  if (j < 4) {
    sc = byte(j) & 63;
    m = byte(j + 4) & 63;
  } else {
    sc = (byte(j + 4) & 0xF) | ((byte(j - 4) >> 6) << 4);
    m = (byte(j + 4) >> 4) | ((byte(j) >> 6) << 4);
  }
}

template <int T>
__global__ __launch_bounds__(KQ_T) void gemm_kq_simple_kernel(GemvArgs p) {
  using F = KQ<T>;
  using S = KQSmem<T>;
  constexpr int ABPB = F::ABPB, RAWW = S::RAWW;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  S& sm = *reinterpret_cast<S*>(smem_raw);

  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int lr = lane & 31, h = lane >> 5;
  const int wj = w >> 1, wi = w & 1;
  const int64_t i0 = (int64_t)blockIdx.x * KQ_TI, j0 = (int64_t)blockIdx.y * KQ_TJ;
  const int z = blockIdx.z, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int rowsA = (int)min((int64_t)KQ_TI, (int64_t)p.M - i0);
  const int rowsB = (int)min((int64_t)KQ_TJ, (int64_t)p.N - j0);

  f32x16 acc[2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;

  for (int sb = 0; sb < p.nblk; ++sb) {
    // ---- stage raw A (row r: dwords from the 4-aligned address at or below its block) and B
    const int ash = (sb * ABPB) & 3;   // lda is a multiple of 16: same shift for every row
    {
      const unsigned char* abase = Az + i0 * p.lda + (((int64_t)sb * ABPB) & ~int64_t(3));
      const int64_t avail = (int64_t)(rowsA - 1) * p.lda + (int64_t)p.nblk * ABPB - (((int64_t)sb * ABPB) & ~int64_t(3));
      const auto ra = make_rsrc(abase, (uint32_t)min((avail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
      const unsigned char* bbase = Bz + j0 * p.ldb + (int64_t)sb * 292;
      const int64_t bavail = (int64_t)(rowsB - 1) * p.ldb + (int64_t)(p.nblk - sb) * 292;
      const auto rb = make_rsrc(bbase, (uint32_t)min((bavail + 3) & ~int64_t(3), (int64_t)0x7fffffff));
      constexpr int NA = sizeof(sm.rawA) / 4 / KQ_T, NB = sizeof(sm.rawB) / 4 / KQ_T;
      uint32_t va[NA], vb[NB];
#pragma unroll
      for (int k = 0; k < NA; ++k) {
        const int dw = t + k * KQ_T, rr = dw / RAWW, oo = dw % RAWW;
        const uint32_t off = (dw < KQ_TI * RAWW && rr < rowsA) ? (uint32_t)(rr * p.lda + 4 * oo) : 0x7ffffff0u;
        va[k] = bload4(ra, off);
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int dw = t + k * KQ_T, rr = dw / 73, oo = dw % 73;
        const uint32_t off = (dw < KQ_TJ * 73 && rr < rowsB) ? (uint32_t)(rr * p.ldb + 4 * oo) : 0x7ffffff0u;
        vb[k] = bload4(rb, off);
      }
#pragma unroll
      for (int k = 0; k < NA; ++k) sm.rawA[t + k * KQ_T] = va[k];
#pragma unroll
      for (int k = 0; k < NB; ++k) sm.rawB[t + k * KQ_T] = vb[k];
    }
    __syncthreads();

    // ---- unpack A: 64 rows x 16 groups of 16 elements; A' = sc * q split into lo / hi ----
    for (int it = t; it < KQ_TI * 16; it += KQ_T) {
      const int il = it / 16, g = it % 16;
      const uint32_t* row = &sm.rawA[il * RAWW];
      auto rd8 = [&](int b) { const int o = b + ash; return (int)((row[o >> 2] >> (8 * (o & 3))) & 0xffu); };
      int aval[16];
      if constexpr (T == kQ6_K) {
        const int sc = (int)(int8_t)rd8(192 + g);
        const int hf = g / 8, part = (g % 8) / 2, l0 = (g % 2) * 16;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int l = l0 + k;
          const int nib = (part & 1) ? rd8(64 * hf + 32 + l) : rd8(64 * hf + l);
          const int q = (part < 2 ? (nib & 0xF) : (nib >> 4)) | (((rd8(128 + 32 * hf + l) >> (2 * part)) & 3) << 4);
          aval[k] = sc * (q - 32);
        }
      } else {
        uint32_t u[3];
#pragma unroll
        for (int k = 0; k < 3; ++k) u[k] = (uint32_t)rd8(4 + 4 * k) | ((uint32_t)rd8(5 + 4 * k) << 8) |
                                           ((uint32_t)rd8(6 + 4 * k) << 16) | ((uint32_t)rd8(7 + 4 * k) << 24);
        int sc, m;
        kq_sm(u, g / 2, sc, m);
        const int e0 = 16 * g, G = e0 / 64, hi = (e0 % 64) >= 32, l0 = e0 % 32;
        constexpr int QS = T == kQ5_K ? 48 : 16;
#pragma unroll
        for (int k = 0; k < 16; ++k) {
          const int l = l0 + k;
          const int b = rd8(QS + 32 * G + l);
          int q = hi ? (b >> 4) : (b & 0xF);
          if constexpr (T == kQ5_K) q += ((rd8(16 + l) >> (e0 / 32)) & 1) << 4;
          aval[k] = sc * q;
        }
        if (il < rowsA) sm.mn[il][g] = (_Float16)(float)m;
        else sm.mn[il][g] = (_Float16)0.f;
      }
      uint32_t lo[4], hi8[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        lo[k] = 0;
        hi8[k] = 0;
#pragma unroll
        for (int c = 0; c < 4; ++c) {
          const int a = aval[4 * k + c];
          lo[k] |= (uint32_t)(a & 127) << (8 * c);
          hi8[k] |= ((uint32_t)(a >> 7) & 0xffu) << (8 * c);
        }
      }
      const bool ok = il < rowsA;
      *(u32x4*)&sm.wlo[(il * KQ_ROWB + 16 * g) / 4] = ok ? u32x4{lo[0], lo[1], lo[2], lo[3]} : u32x4{0, 0, 0, 0};
      *(u32x4*)&sm.whi[(il * KQ_ROWB + 16 * g) / 4] = ok ? u32x4{hi8[0], hi8[1], hi8[2], hi8[3]} : u32x4{0, 0, 0, 0};
      if (g == 0) {
        if constexpr (T == kQ6_K) {
          sm.da[il] = ok ? h2f((uint32_t)rd8(208) | ((uint32_t)rd8(209) << 8)) : 0.f;
          sm.dmn[il] = 0.f;
        } else {
          sm.da[il] = ok ? h2f((uint32_t)rd8(0) | ((uint32_t)rd8(1) << 8)) : 0.f;
          sm.dmn[il] = ok ? h2f((uint32_t)rd8(2) | ((uint32_t)rd8(3) << 8)) : 0.f;
        }
      }
    }
    // ---- unpack B: 128 rows x 16 pieces of 16 quants; bsums to fp16 (exact), d_b f32 ----
    for (int it = t; it < KQ_TJ * 16; it += KQ_T) {
      const int jl = it / 16, q16 = it % 16;
      const uint32_t* blk = &sm.rawB[jl * 73];
      const bool ok = jl < rowsB;
      *(u32x4*)&sm.act[(jl * KQ_ROWB + 16 * q16) / 4] =
          ok ? u32x4{blk[1 + 4 * q16], blk[2 + 4 * q16], blk[3 + 4 * q16], blk[4 + 4 * q16]} : u32x4{0, 0, 0, 0};
      if constexpr (F::MIN) {
        const uint32_t bw = blk[65 + (q16 >> 1)];
        sm.bs[jl][q16] = ok ? (_Float16)(float)(int16_t)((q16 & 1) ? (bw >> 16) : (bw & 0xffff)) : (_Float16)0.f;
      }
      if (q16 == 0) sm.yd[jl] = ok ? __uint_as_float(blk[0]) : 0.f;
    }
    __syncthreads();

    // ---- 2 x 8 chained i8 MFMAs per tile: S = 128 S_hi + S_lo; mins by one f16 MFMA ----
    const int ia = 32 * wi + lr;
    const float dai = sm.da[ia], dmi = sm.dmn[ia];
    half8 mnf = {};
    if constexpr (F::MIN) mnf = *(const half8*)&sm.mn[ia][8 * h];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int jb = 64 * wj + 32 * rt;
      i32x16 slo = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, shi = slo;
#pragma unroll
      for (int kk = 0; kk < 8; ++kk) {
        const int o = (32 * kk + 16 * h) / 4;
        const i32x4 af = *(const i32x4*)&sm.act[(jb + lr) * KQ_ROWB / 4 + o];
        const i32x4 wl = *(const i32x4*)&sm.wlo[ia * KQ_ROWB / 4 + o];
        const i32x4 wh = *(const i32x4*)&sm.whi[ia * KQ_ROWB / 4 + o];
        slo = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, wl, slo, 0, 0, 0);
        shi = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, wh, shi, 0, 0, 0);
      }
      f32x16 mins = {};
      if constexpr (F::MIN) {
        const half8 bsf = *(const half8*)&sm.bs[jb + lr][8 * h];
        mins = __builtin_amdgcn_mfma_f32_32x32x16_f16(bsf, mnf, mins, 0, 0, 0);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 ydv = *(const f32x4*)&sm.yd[jb + 8 * g4 + 4 * h];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g4 + e;
          const float s = (float)(shi[r] * 128 + slo[r]);
          if constexpr (F::MIN)
            acc[rt][r] += (ydv[e] * dai) * s - (ydv[e] * dmi) * mins[r];
          else
            acc[rt][r] += (ydv[e] * dai) * s;
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

template <int T>
hipError_t launch_kq_simple(const GemvArgs& p, hipStream_t s) {
  const dim3 grid((unsigned)((p.M + KQ_TI - 1) / KQ_TI), (unsigned)((p.N + KQ_TJ - 1) / KQ_TJ),
                  (unsigned)(p.ne12 * p.ne13));
  constexpr size_t lds = sizeof(KQSmem<T>);
  static_assert(lds <= 160 * 1024, "LDS");
  set_max_lds((const void*)gemm_kq_simple_kernel<T>, (int)lds);
  hipLaunchKernelGGL(gemm_kq_simple_kernel<T>, grid, dim3(KQ_T), lds, s, p);
  return hipGetLastError();
}

// =================================================================== pipelined engine
// The weights' integer-scaled planes (A lo / hi), the per-row fp scales and the min rows are
// made by prep_w_kq -- once per weight for stationary callers (lamm_hip_weights), per call
// otherwise -- and the q8_K rows are decoded by prep_b_kq, both straight into the main
// kernel's LDS image: one chunk per (tile, super-block), moved by LDS-DMA (buffer_load ...
// lds) into a double-buffered ring, so the main loop only reads fragments and issues MFMAs.
//   A chunk (64 rows):  lo [64][256] | hi [64][256] | d f32 [64] | dmin f32 [64] | mn f16 [64][16]
//   B chunk (128 rows): q8 [128][256] | d_b f32 [128] | bsums f16 [128][16]
// The int8 planes are XOR-swizzled per row (16-byte slot c of row r stored at c ^ (r & 15)),
// so a ds_read_b128 lane group (16 rows, one slot) hits 16 distinct bank quads.
constexpr int KQC_A = 35840;    // 35 KiB: 32768 + 256 + 256 + 2048 (+ pad)
constexpr int KQC_B = 37888;    // 37 KiB: 32768 + 512 + 4096 (+ pad)
constexpr int KQ_PIECES = (KQC_A + KQC_B) / 1024;   // 72 LDS-DMA pieces per step
constexpr int KQ_PA = KQC_A / 1024;
static_assert(KQ_PIECES % 4 == 0, "pieces split evenly over the 4 waves");

struct KQLayout {
  int nit, njt, nsb, na;
  int64_t a_bytes, b_slice;
  __host__ __device__ static KQLayout of(const GemvArgs& p) {
    KQLayout L;
    L.nit = (p.M + KQ_TI - 1) / KQ_TI;
    L.njt = (p.N + KQ_TJ - 1) / KQ_TJ;
    L.nsb = p.nblk;
    L.na = (p.ne12 / p.r2) * (p.ne13 / p.r3);
    L.a_bytes = (int64_t)L.na * L.nit * L.nsb * KQC_A;
    L.b_slice = (int64_t)L.njt * L.nsb * KQC_B;
    return L;
  }
};

__host__ __device__ constexpr int kq_swz(int r, int c) { return r * 256 + 16 * (c ^ (r & 15)); }

// one thread per (weight row, super-block): decode the block once, write its 16 groups
template <int T>
__global__ __launch_bounds__(256) void prep_w_kq(GemvArgs p, unsigned char* wsA) {
  constexpr int ABPB = KQ<T>::ABPB, NW = ABPB / 4 + 2;
  const KQLayout L = KQLayout::of(p);
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (int64_t)L.nit * KQ_TI * L.nsb) return;
  const int sb = (int)(g % L.nsb);
  const int64_t i = g / L.nsb;
  const int a = blockIdx.y, ne02 = p.ne12 / p.r2, i02 = a % ne02, i03 = a / ne02;
  const unsigned char* Az = p.A + (int64_t)i02 * p.sa2 + (int64_t)i03 * p.sa3;
  unsigned char* ch = wsA + (((int64_t)a * L.nit + i / KQ_TI) * L.nsb + sb) * KQC_A;
  const int r = (int)(i % KQ_TI);
  const bool ok = i < p.M;
  uint32_t raw[NW];
  int sh = 0;
  {
    // resource based at the workgroup's first row: wave-uniform (a per-lane base would turn
    // every buffer load into a waterfall loop) and offsets < 2^31 for any slice size
    const int64_t iw = min(((int64_t)blockIdx.x * 256) / L.nsb, (int64_t)p.M - 1);
    const int64_t il = min((int64_t)p.M - 1, ((int64_t)blockIdx.x * 256 + 255) / L.nsb);
    const int64_t abytes = (il - iw) * p.lda + (int64_t)p.nblk * ABPB;
    const auto ra = make_rsrc(Az + iw * p.lda, (uint32_t)min((abytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
    const int64_t off = ok ? (i - iw) * p.lda + (int64_t)sb * ABPB : 0x7fffff00;
    sh = (int)(off & 3);
#pragma unroll
    for (int k = 0; k < NW; ++k) raw[k] = bload4(ra, (uint32_t)((off & ~int64_t(3)) + 4 * k));
  }
  auto rd8 = [&](int b) { const int o = b + sh; return (int)((raw[o >> 2] >> (8 * (o & 3))) & 0xffu); };
  uint32_t u[3] = {0, 0, 0};
  if constexpr (T == kQ4_K || T == kQ5_K) {
#pragma unroll
    for (int k = 0; k < 3; ++k)
      u[k] = (uint32_t)rd8(4 + 4 * k) | ((uint32_t)rd8(5 + 4 * k) << 8) | ((uint32_t)rd8(6 + 4 * k) << 16) |
             ((uint32_t)rd8(7 + 4 * k) << 24);
  }
#pragma unroll 2
  for (int gi = 0; gi < 16; ++gi) {
    int aval[16];
    int m = 0;
    if constexpr (T == kQ6_K) {
      const int sc = (int)(int8_t)rd8(192 + gi);
      const int hf = gi / 8, part = (gi % 8) / 2, l0 = (gi % 2) * 16;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int l = l0 + k;
        const int nib = (part & 1) ? rd8(64 * hf + 32 + l) : rd8(64 * hf + l);
        const int q = (part < 2 ? (nib & 0xF) : (nib >> 4)) | (((rd8(128 + 32 * hf + l) >> (2 * part)) & 3) << 4);
        aval[k] = sc * (q - 32);
      }
    } else if constexpr (T == kQ2_K) {
      // element e = 128 n + 32 jj + l: (qs[32 n + l] >> 2 jj) & 3, sub-block e / 16 = gi
      // (src/lamm_kernel_q2_k.hpp:52-71); scale / min nibbles of scales[gi]
      const int scb = rd8(gi), sc = scb & 15;
      m = scb >> 4;
      const int n = gi / 8, jj = (gi % 8) / 2, l0 = (gi % 2) * 16;
#pragma unroll
      for (int k = 0; k < 16; ++k) aval[k] = sc * ((rd8(16 + 32 * n + l0 + k) >> (2 * jj)) & 3);
    } else {
      int sc;
      kq_sm(u, gi / 2, sc, m);
      const int e0 = 16 * gi, G = e0 / 64, hi = (e0 % 64) >= 32, l0 = e0 % 32;
      constexpr int QS = T == kQ5_K ? 48 : 16;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        const int l = l0 + k;
        const int b = rd8(QS + 32 * G + l);
        int q = hi ? (b >> 4) : (b & 0xF);
        if constexpr (T == kQ5_K) q += ((rd8(16 + l) >> (e0 / 32)) & 1) << 4;
        aval[k] = sc * q;
      }
    }
    uint32_t lo[4], hi8[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      lo[k] = 0;
      hi8[k] = 0;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int av = ok ? aval[4 * k + c] : 0;
        lo[k] |= (uint32_t)(av & 127) << (8 * c);
        hi8[k] |= ((uint32_t)(av >> 7) & 0xffu) << (8 * c);
      }
    }
    *(u32x4*)(ch + kq_swz(r, gi)) = u32x4{lo[0], lo[1], lo[2], lo[3]};
    if constexpr (KQ<T>::HI) *(u32x4*)(ch + 16384 + kq_swz(r, gi)) = u32x4{hi8[0], hi8[1], hi8[2], hi8[3]};
    *(_Float16*)(ch + 33280 + 32 * r + 2 * gi) = (_Float16)(float)(ok ? m : 0);
  }
  float d = 0.f, dm = 0.f;
  if (ok) {
    if constexpr (T == kQ6_K) {
      d = h2f((uint32_t)rd8(208) | ((uint32_t)rd8(209) << 8));
    } else if constexpr (T == kQ2_K) {
      d = h2f((uint32_t)rd8(80) | ((uint32_t)rd8(81) << 8));
      dm = h2f((uint32_t)rd8(82) | ((uint32_t)rd8(83) << 8));
    } else {
      d = h2f((uint32_t)rd8(0) | ((uint32_t)rd8(1) << 8));
      dm = h2f((uint32_t)rd8(2) | ((uint32_t)rd8(3) << 8));
    }
  }
  *(float*)(ch + 32768 + 4 * r) = d;
  *(float*)(ch + 33024 + 4 * r) = dm;
}

// 18 threads per (activation row, super-block): 16 copy a 16-quant piece each, one the f32
// d_b, one the 16 bsums (as exact fp16); consecutive threads read consecutive 16-byte pieces
__global__ __launch_bounds__(256) void prep_b_kq(GemvArgs p, unsigned char* wsB) {
  const KQLayout L = KQLayout::of(p);
  const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (g >= (int64_t)L.njt * KQ_TJ * L.nsb * 18) return;
  const int q = (int)(g % 18);
  const int64_t rest = g / 18;
  const int sb = (int)(rest % L.nsb);
  const int64_t j = rest / L.nsb;
  const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  unsigned char* ch = wsB + (int64_t)z * L.b_slice + ((j / KQ_TJ) * L.nsb + sb) * KQC_B;
  const int r = (int)(j % KQ_TJ);
  const bool ok = j < p.N;
  // resource based at the workgroup's first row: wave-uniform (a per-lane base would turn
  // every buffer load into a waterfall loop) and offsets < 2^31 for any slice size
  const int64_t jw = min(((int64_t)blockIdx.x * 256 / 18) / L.nsb, (int64_t)p.N - 1);
  const int64_t jl = min((int64_t)p.N - 1, (((int64_t)blockIdx.x * 256 + 255) / 18) / L.nsb);
  const int64_t bbytes = (jl - jw) * p.ldb + (int64_t)p.nblk * 292;
  const auto rb = make_rsrc(Bz + jw * p.ldb, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
  const uint32_t off = ok ? (uint32_t)((j - jw) * p.ldb + (int64_t)sb * 292) : 0x7ffffe00u;
  if (q < 16) {   // quants 16q .. 16q+15 (dwords 1 + 4q ..)
    u32x4 v;
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = bload4(rb, off + 4 * (1 + 4 * q + k));
    *(u32x4*)(ch + kq_swz(r, q)) = v;
  } else if (q == 16) {
    *(float*)(ch + 32768 + 4 * r) = __uint_as_float(bload4(rb, off));
  } else {
    uint32_t hb[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint32_t v = bload4(rb, off + 4 * (65 + k));
      const _Float16 lo = (_Float16)(float)(int16_t)(v & 0xffff), hi = (_Float16)(float)(int16_t)(v >> 16);
      hb[k] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
    }
    *(u32x4*)(ch + 33280 + 32 * r) = u32x4{hb[0], hb[1], hb[2], hb[3]};
    *(u32x4*)(ch + 33280 + 32 * r + 16) = u32x4{hb[4], hb[5], hb[6], hb[7]};
  }
}

template <int N_>
__device__ __forceinline__ void kq_wait_vm() {   // s_waitcnt vmcnt(N) (lgkmcnt untouched)
  static_assert(N_ >= 0 && N_ < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N_ & 0xF) | ((N_ >> 4) << 14) | (0x7 << 4) | (0xF << 8));
  asm volatile("" ::: "memory");
}
__device__ __forceinline__ void kq_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0)
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

template <int T>
__global__ __launch_bounds__(KQ_T) void gemm_kq_kernel(GemvArgs p, const unsigned char* wsA,
                                                       const unsigned char* wsB, int nsplit, float* part) {
  constexpr bool MIN = KQ<T>::MIN;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const KQLayout L = KQLayout::of(p);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const int wj = w >> 1, wi = w & 1;
  // blockIdx.z = split * slices + slice: split sp runs super-blocks [k0, k1) and writes a
  // partial tile (summed in split order by launch_splitk_reduce); nsplit 1 writes C
  const int nz = p.ne12 * p.ne13, z = (int)blockIdx.z % nz, sp = (int)blockIdx.z / nz;
  const int it = blockIdx.x, jt = blockIdx.y;
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const int ne02 = p.ne12 / p.r2, a = (i12 / p.r2) + (i13 / p.r3) * ne02;
  const unsigned char* ga = wsA + ((int64_t)a * L.nit + it) * L.nsb * KQC_A;
  const unsigned char* gb = wsB + (int64_t)z * L.b_slice + (int64_t)jt * L.nsb * KQC_B;
  const auto ra = make_rsrc(ga, (uint32_t)((int64_t)L.nsb * KQC_A));
  const auto rb = make_rsrc(gb, (uint32_t)((int64_t)L.nsb * KQC_B));
  const int nsb = L.nsb;

  // q2_K (no hi plane: q * sc <= 45 fits int8) skips the A chunk's hi-plane pieces 16..31 -- 56 instead
  // of 72 KiB per step
  constexpr int SKIP = KQ<T>::HI ? 0 : 16, PPW = (KQ_PIECES - SKIP) / 4;
  static_assert((KQ_PIECES - SKIP) % 4 == 0, "pieces split evenly over the 4 waves");
  auto issue = [&](int sb) {
    unsigned char* dst = smem + (sb & 1) * (KQC_A + KQC_B);
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      const int pc0 = k * 4 + w;   // wave-uniform
      const int pc = pc0 < 16 ? pc0 : pc0 + SKIP;
      if (pc < KQ_PA)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16,
                                                 (uint32_t)(sb * KQC_A + pc * 1024 + lane * 16), 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16,
                                                 (uint32_t)(sb * KQC_B + (pc - KQ_PA) * 1024 + lane * 16), 0, 0, 0);
    }
  };

  f32x16 acc[2];
#pragma unroll
  for (int r = 0; r < 2; ++r)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[r][e] = 0.f;

  const int k0 = (int)((int64_t)sp * nsb / nsplit), k1 = (int)((int64_t)(sp + 1) * nsb / nsplit);
  issue(k0);
  if (k1 - k0 > 1) issue(k0 + 1);
  const int ia = 32 * wi + lr;
  for (int sb = k0; sb < k1; ++sb) {
    if (sb + 1 < k1) kq_wait_vm<PPW>(); else kq_wait_vm<0>();
    kq_barrier();   // step sb's chunks visible to every wave
    const unsigned char* sA = smem + (sb & 1) * (KQC_A + KQC_B);
    const unsigned char* sB = sA + KQC_A;
    i32x16 slo[2], shi[2];
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int e = 0; e < 16; ++e) slo[rt][e] = shi[rt][e] = 0;
#pragma unroll
    for (int kk = 0; kk < 8; ++kk) {
      const int c = 2 * kk + h;
      const i32x4 wl = *(const i32x4*)(sA + kq_swz(ia, c));
      i32x4 wh = {};
      if constexpr (KQ<T>::HI) wh = *(const i32x4*)(sA + 16384 + kq_swz(ia, c));
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const int jr = 64 * wj + 32 * rt + lr;
        const i32x4 af = *(const i32x4*)(sB + kq_swz(jr, c));
        slo[rt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, wl, slo[rt], 0, 0, 0);
        if constexpr (KQ<T>::HI) shi[rt] = __builtin_amdgcn_mfma_i32_32x32x32_i8(af, wh, shi[rt], 0, 0, 0);
      }
    }
    const float dai = *(const float*)(sA + 32768 + 4 * ia);
    const float dmi = MIN ? *(const float*)(sA + 33024 + 4 * ia) : 0.f;
    half8 mnf = {};
    if constexpr (MIN) mnf = *(const half8*)(sA + 33280 + 32 * ia + 16 * h);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) {
      const int jb = 64 * wj + 32 * rt;
      f32x16 mins = {};
      if constexpr (MIN) {
        const half8 bsf = *(const half8*)(sB + 33280 + 32 * (jb + lr) + 16 * h);
        mins = __builtin_amdgcn_mfma_f32_32x32x16_f16(bsf, mnf, mins, 0, 0, 0);
      }
#pragma unroll
      for (int g4 = 0; g4 < 4; ++g4) {
        const f32x4 ydv = *(const f32x4*)(sB + 32768 + 4 * (jb + 8 * g4 + 4 * h));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g4 + e;
          const float sv = (float)(shi[rt][r] * 128 + slo[rt][r]);
          if constexpr (MIN)
            acc[rt][r] += (ydv[e] * dai) * sv - (ydv[e] * dmi) * mins[r];
          else
            acc[rt][r] += (ydv[e] * dai) * sv;
        }
      }
    }
    kq_barrier();   // every wave is done with buffer sb & 1
    if (sb + 2 < k1) issue(sb + 2);
  }

  float* Cz = nsplit == 1 ? p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3
                          : part + ((int64_t)sp * nz + z) * p.N * p.M;
  const int64_t ldc = nsplit == 1 ? p.ldc : p.M;
  const int64_t i = (int64_t)it * KQ_TI + ia;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int64_t j = (int64_t)jt * KQ_TJ + 64 * wj + 32 * rt + (r & 3) + 8 * (r >> 2) + 4 * h;
      // non-temporal: C is written once (Q6_K output.weight 32000x512: 292 -> 280 us whole
      // launch, profiles/r02/ab_gemm_store.txt)
      if (i < p.M && j < p.N) __builtin_nontemporal_store(acc[rt][r], &Cz[j * ldc + i]);
    }
}

// K-splits (in super-blocks) for small grids, e.g. one 4096 x 128 GEMM = 64 tiles: double until
// 256 workgroups, >= 4 super-blocks per split, at most 16.  LAMM_KQ_SPLIT=n forces n (A/B).
int kq_nsplit(const GemvArgs& p) {
  const KQLayout L = KQLayout::of(p);
  const int tiles = L.nit * L.njt * p.ne12 * p.ne13;
  int n = 1;
  if (knobs().kq_split > 0) {
    n = knobs().kq_split;
  } else {
    while (tiles * n < 256 && n < 16 && L.nsb / (2 * n) >= 4) n *= 2;
  }
  return n < 1 ? 1 : (n > L.nsb ? L.nsb : n);
}

size_t kq_part_offset(const GemvArgs& p, bool prepared) {
  const KQLayout L = KQLayout::of(p);
  return ((prepared ? 0 : (size_t)L.a_bytes) + (size_t)(p.ne12 * p.ne13) * (size_t)L.b_slice + 255) & ~(size_t)255;
}

template <int T>
void launch_prep_w_kq(const GemvArgs& p, unsigned char* wsA, hipStream_t s) {
  const KQLayout L = KQLayout::of(p);
  const int64_t n = (int64_t)L.nit * KQ_TI * L.nsb;
  hipLaunchKernelGGL(prep_w_kq<T>, dim3((unsigned)((n + 255) / 256), (unsigned)L.na), dim3(256), 0, s, p, wsA);
}

template <int T>
hipError_t launch_kq(const GemvArgs& p, const void* prepA, void* ws, hipStream_t s) {
  const KQLayout L = KQLayout::of(p);
  auto* w = static_cast<unsigned char*>(ws);
  unsigned char* wsA = prepA ? nullptr : w;
  unsigned char* wsB = w + (prepA ? 0 : L.a_bytes);
  if (!prepA) launch_prep_w_kq<T>(p, wsA, s);
  const int64_t nb = (int64_t)L.njt * KQ_TJ * L.nsb * 18;
  hipLaunchKernelGGL(prep_b_kq, dim3((unsigned)((nb + 255) / 256), (unsigned)(p.ne12 * p.ne13)), dim3(256), 0, s, p,
                     wsB);
  constexpr size_t lds = 2 * (KQC_A + KQC_B);
  static_assert(lds <= 160 * 1024, "LDS");
  set_max_lds((const void*)gemm_kq_kernel<T>, (int)lds);
  const int nsplit = kq_nsplit(p);
  float* part = reinterpret_cast<float*>(w + kq_part_offset(p, prepA != nullptr));
  hipLaunchKernelGGL(gemm_kq_kernel<T>, dim3((unsigned)L.nit, (unsigned)L.njt, (unsigned)(p.ne12 * p.ne13 * nsplit)),
                     dim3(KQ_T), lds, s, p, prepA ? static_cast<const unsigned char*>(prepA) : wsA,
                     static_cast<const unsigned char*>(wsB), nsplit, part);
  if (nsplit > 1) launch_splitk_reduce(p, nsplit, part, s);
  return hipGetLastError();
}

}  // namespace

bool gemm_kq_supported(int type) { return type == kQ4_K || type == kQ5_K || type == kQ6_K || type == kQ2_K; }

size_t gemm_kq_weight_bytes(int type, const GemvArgs& p) {
  (void)type;
  return (size_t)KQLayout::of(p).a_bytes;
}

size_t gemm_kq_workspace_bytes(int type, const GemvArgs& p, bool prepared) {
  (void)type;
  const int nsplit = kq_nsplit(p);
  const size_t part = nsplit > 1 ? (size_t)nsplit * p.ne12 * p.ne13 * (size_t)p.N * p.M * sizeof(float) : 0;
  return kq_part_offset(p, prepared) + part + 256;
}

hipError_t prepare_kq_weights(int type, const GemvArgs& p, void* wsA, hipStream_t s) {
  auto* w = static_cast<unsigned char*>(wsA);
  switch (type) {
    case kQ4_K: launch_prep_w_kq<kQ4_K>(p, w, s); break;
    case kQ5_K: launch_prep_w_kq<kQ5_K>(p, w, s); break;
    case kQ6_K: launch_prep_w_kq<kQ6_K>(p, w, s); break;
    case kQ2_K: launch_prep_w_kq<kQ2_K>(p, w, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// LAMM_KQ_VARIANT=1: the single-pass kernel that unpacks raw blocks in LDS (A/B)
hipError_t launch_gemm_kq(int type, const GemvArgs& p, const void* prepA, void* ws, hipStream_t s) {
  if (p.M == 0 || p.N == 0) return hipSuccess;
  if ((p.ldb & 3) || ((uintptr_t)p.B & 3) || (p.sb2 & 3) || (p.sb3 & 3)) return hipErrorInvalidValue;
  if (knobs().kq_variant == 1 && type != kQ2_K) {
    switch (type) {
      case kQ4_K: return launch_kq_simple<kQ4_K>(p, s);
      case kQ5_K: return launch_kq_simple<kQ5_K>(p, s);
      case kQ6_K: return launch_kq_simple<kQ6_K>(p, s);
      default: return hipErrorInvalidValue;
    }
  }
  switch (type) {
    case kQ4_K: return launch_kq<kQ4_K>(p, prepA, ws, s);
    case kQ5_K: return launch_kq<kQ5_K>(p, prepA, ws, s);
    case kQ6_K: return launch_kq<kQ6_K>(p, prepA, ws, s);
    case kQ2_K: return launch_kq<kQ2_K>(p, prepA, ws, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
