// lamm_gemm_i8kv.hip -- prefill GEMM (N > 8) for q4_0 / q5_0 / q8_0 weights with NO activation
// prep: the K-group plan of lamm_gemm_fp6.hip (gemm_fp6_kv_kernel) with the block dots on the int8
// matrix path, reading ggml's q8_0 activation rows exactly as they are stored.
//
// Contract: the lamm block kernels (src/lamm_kernel_q4_0.hpp:59-128, q5_0 :69-139, q8_0 :50-117, via
// LAMMImpl<T>::matmul_simd_block, src/lamm_impl.hpp:90-147): C[j*ldc + i] = sum_blocks d_a d_b S,
// S = the exact int32 block dot of the weight quants (q - 8 / q - 16 / q) with the q8_0 quants.
//
// Why a second engine.  The fp6 engine's activations must be re-coded per call into two 6-bit code
// planes (prep_b_fp6_tile): a separate launch, ~6 us of config 3's 27.8 us whole launch, most of it
// the dispatch itself.  v_mfma_i32_32x32x32_i8 (K = 32 = one block) takes the q8_0
// quants as they are: lane (r, h) of an activation fragment holds bytes 2 + 16 h .. 17 + 16 h of row
// r's 34-byte block (2-byte aligned: one alignbit per dword realigns them).  The weights are prepared
// once (weight-stationary callers) as int8 planes.  The block dot S is then the same exact integer
// the fp6 engine computes, as an int32; the epilogue converts it (v_cvt_f32_i32) and applies the same
// P-MFMA (P = 2 d_a d_b, exact) and FMA in the same order -- C is bit-identical to the fp6 engine's.
// The price is one convert per output element and block beside the FMA; the gains are no prep launch
// and 34 instead of 64 bytes of activation operand per row and block.
//
// Layout of the prepared weights (per 256-row tile and K-step of I8_KB = 2 blocks, one chunk):
//   plane 0 [b][r] x 16 B : quants 0..15 of block b of row r, int8
//   plane 1 [b][r] x 16 B : quants 16..31
//   d       [b][r] x 4 B  : the block's fp16 d in the low half (0 above)
// Rows past M and blocks past K are zero (the MFMA then adds nothing; d = 0 keeps P finite).
#include "lamm_device.h"
#include "lamm_kernels.h"
#include "lamm_knobs.h"

namespace lamm {
namespace {

typedef _Float16 half4 __attribute__((ext_vector_type(4)));

constexpr int I8_TI = 256;                             // rows per prepared tile (two workgroup tiles)
constexpr int I8_KB = 2;                               // blocks per K-step
constexpr int I8_PLANE = I8_KB * I8_TI * 16;           // one 16-byte plane of a K-step
constexpr int I8_CH = 2 * I8_PLANE + I8_KB * I8_TI * 4;   // a K-step's chunk: two planes + d
constexpr int I8_PIECE = 1024;                         // one wave's LDS-DMA instruction (64 lanes x 16 B)

template <int T> struct I8F;
template <> struct I8F<kQ4_0> { static constexpr int ABPB = 18; };
template <> struct I8F<kQ5_0> { static constexpr int ABPB = 22; };
template <> struct I8F<kQ8_0> { static constexpr int ABPB = 34; };

struct I8Layout {
  int nsteps, nit, na;
  int64_t a_slice, a_bytes;
  __host__ __device__ static I8Layout of(const GemvArgs& p) {
    I8Layout L;
    L.nsteps = (p.nblk + I8_KB - 1) / I8_KB;
    L.nit = (p.M + I8_TI - 1) / I8_TI;
    L.na = (p.ne12 / p.r2) * (p.ne13 / p.r3);
    L.a_slice = (int64_t)L.nit * L.nsteps * I8_CH;
    L.a_bytes = (int64_t)L.na * L.a_slice;
    return L;
  }
};

// ---------------------------------------------------------------- weight prep (once per weight)
// thread = (row i, block kb); consecutive threads take consecutive rows, so every plane store of a
// wave is 1 KiB contiguous
template <int T>
__global__ __launch_bounds__(256) void prep_w_i8(GemvArgs p, unsigned char* ws) {
  const I8Layout L = I8Layout::of(p);
  const int64_t rows = (int64_t)L.nit * I8_TI;
  const int64_t gi = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t i = gi % rows;
  const int kb = (int)(gi / rows);
  if (kb >= L.nsteps * I8_KB) return;
  const int a = blockIdx.y, ne02 = p.ne12 / p.r2, i02 = a % ne02, i03 = a / ne02;
  uint32_t q[8] = {0, 0, 0, 0, 0, 0, 0, 0}, d = 0;
  if (i < p.M && kb < p.nblk) {
    const unsigned char* blk =
        p.A + (int64_t)i02 * p.sa2 + (int64_t)i03 * p.sa3 + i * p.lda + (int64_t)kb * I8F<T>::ABPB;
    auto byte = [&](int o) { return (uint32_t)blk[o]; };
    d = byte(0) | (byte(1) << 8);
#pragma unroll
    for (int e = 0; e < 32; ++e) {
      int n;
      if constexpr (T == kQ8_0) {
        n = (int)(int8_t)byte(2 + e);
      } else if constexpr (T == kQ4_0) {
        n = (int)(e < 16 ? byte(2 + e) & 15u : byte(2 + e - 16) >> 4) - 8;
      } else {   // q5_0: the 5th bit from qh (bytes 2..5)
        const uint32_t qh = byte(2) | (byte(3) << 8) | (byte(4) << 16) | (byte(5) << 24);
        const uint32_t lo = e < 16 ? byte(6 + e) & 15u : byte(6 + e - 16) >> 4;
        n = (int)(lo | (((qh >> e) & 1u) << 4)) - 16;
      }
      q[e >> 2] |= ((uint32_t)n & 0xffu) << (8 * (e & 3));
    }
  }
  unsigned char* ch = ws + (int64_t)a * L.a_slice + ((int64_t)(i / I8_TI) * L.nsteps + kb / I8_KB) * I8_CH;
  const int b = kb % I8_KB, r = (int)(i % I8_TI);
  *(u32x4*)(ch + (b * I8_TI + r) * 16) = u32x4{q[0], q[1], q[2], q[3]};
  *(u32x4*)(ch + I8_PLANE + (b * I8_TI + r) * 16) = u32x4{q[4], q[5], q[6], q[7]};
  *(uint32_t*)(ch + 2 * I8_PLANE + (b * I8_TI + r) * 4) = d;
}

// ---------------------------------------------------------------- GEMM
template <int N_>
__device__ __forceinline__ void i8_wait_vm() {   // s_waitcnt vmcnt(N) (lgkmcnt untouched)
  static_assert(N_ >= 0 && N_ < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N_ & 0xF) | ((N_ >> 4) << 14) | (0x7 << 4) | (0xF << 8));
  asm volatile("" ::: "memory");
}

// The workgroup's 128 (i) x 64 (j) tile, 8 waves = 4 K-groups x 2 row halves; a wave owns 64 x 64 =
// 2 x 2 units of 32 x 32 per block and streams its own blocks (g, g + 4, ... in K-steps):
//   weights     : its 64 rows' two int8 planes and d by LDS-DMA into a ring of its own (P slots;
//                 only this wave writes and reads it, so its vmcnt is the only synchronisation),
//                 read back with both half-waves on the same rows -- plane h for half-wave h
//   activations : the group's 64 q8_0 rows straight into VGPRs: per lane the block's d dword and
//                 the five dwords around its 16 quants, realigned at use
// Per unit: S = the exact block dot (int8 MFMA), P = 2 d_b d_a (f16 MFMA), acc += float(S) * P --
// unit n + 1's MFMAs issued before unit n's converts and FMAs.
template <int T, int P>
__global__ __launch_bounds__(512) void gemm_i8_kv_kernel(GemvArgs p, const unsigned char* wsA) {
  constexpr int KG = 4, TI = 128, TJ = 64, NW = 8, WJ = 2, UPB = 2 * WJ;
  constexpr int NBW = 3;                         // activation loads per sub-tile and block
  constexpr int LPB = 3 + NBW * WJ;              // vmem ops per block: 3 DMA pieces + the activation loads
  constexpr int SLOT = 2 * I8_PIECE + 256;       // a ring slot: two plane pieces and the d piece
  constexpr int RING = P * SLOT;
  static_assert(P >= 2 && P <= 4, "blocks in flight");
  static_assert(NW * RING <= 4 * 64 * (128 + 8) * 4, "the rings live under the epilogue's LDS");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const I8Layout L = I8Layout::of(p);
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const int g = w / 2, wi = w % 2;
  const int nsi = (p.M + TI - 1) / TI, nsj = (p.N + TJ - 1) / TJ;
  int ti, tj, z;
  {   // XCD-aware tile order (gemm_fp6_kv_kernel's): one XCD's workgroups on neighbouring tiles
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
  const int it = ti / 2, ri0 = (ti % 2) * TI;
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const int ne02 = p.ne12 / p.r2, a = (i12 / p.r2) + (i13 / p.r3) * ne02;
  const unsigned char* wa = wsA + (int64_t)a * L.a_slice + (int64_t)it * L.nsteps * I8_CH;
  const int nsteps = L.nsteps;
  const int nbw = nsteps > g ? (nsteps - g + KG - 1) / KG * I8_KB : 0;   // this wave's blocks
  const auto ra = make_rsrc(wa, (uint32_t)(nsteps * I8_CH));
  // the group's activation rows from row j0: a wave-uniform base, offsets < 2^31; rows past N and
  // blocks past K read as zeros (offsets past the resource)
  const int64_t j0 = (int64_t)tj * TJ;
  const int64_t nrow = min((int64_t)TJ, (int64_t)p.N - j0);
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3 + j0 * p.ldb;
  const int64_t bbytes = (nrow - 1) * p.ldb + (int64_t)p.nblk * 34;
  const auto rb = make_rsrc(Bz, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
  const int ldb4 = (int)(p.ldb & 3);
  const int a0 = (ri0 + 64 * wi) * 16, d0 = (ri0 + 64 * wi) * 4;
  unsigned char* ring = smem + w * RING;

  uint32_t rq[P][WJ][NBW + 3];   // per slot and sub-tile: d dword, then 5 dwords around the quants
  // block u of this wave (K-step g + KG (u / KB), block u % KB) into slot S; past the end the last
  // block is fetched again (unused) so every slot's wait count stays the same
  auto issue = [&](int u, auto S_) {
    constexpr int S = decltype(S_)::value;
    const int uu = min(u, nbw - 1);
    const int ks = g + KG * (uu / I8_KB), b = uu % I8_KB;
    const int kb = ks * I8_KB + b;
    const int ka = ks * I8_CH;
    unsigned char* sl = ring + S * SLOT;
#pragma unroll
    for (int pl = 0; pl < 2; ++pl)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(sl + pl * I8_PIECE), 16,
                                               lane * 16, ka + pl * I8_PLANE + b * I8_TI * 16 + a0, 0, 0);
    __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(sl + 2 * I8_PIECE), 4,
                                             lane * 4, ka + 2 * I8_PLANE + b * I8_TI * 4 + d0, 0, 0);
#pragma unroll
    for (int x = 0; x < WJ; ++x) {
      const bool ok = kb < p.nblk;
      const uint32_t o = (uint32_t)((32 * x + lr) * p.ldb + (int64_t)kb * 34);
      const uint32_t od = ok ? (o & ~3u) : 0x7ffffff0u;
      const uint32_t oq = ok ? ((o + 2 + 16 * h) & ~3u) : 0x7ffffff0u;
      rq[S][x][0] = __builtin_amdgcn_raw_buffer_load_b32(rb, od, 0, 0);
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rb, oq, 0, 0);
      rq[S][x][1] = v[0];
      rq[S][x][2] = v[1];
      rq[S][x][3] = v[2];
      rq[S][x][4] = v[3];
      rq[S][x][5] = __builtin_amdgcn_raw_buffer_load_b32(rb, oq + 16, 0, 0);
    }
  };

  f32x16 acc[WJ][2];
#pragma unroll
  for (int x = 0; x < WJ; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;
  const f32x16 fz = {};
  const i32x16 iz = {};
  struct Res { i32x16 s; f32x16 pr; };
  // the previous block's last unit is finished under the next block's first MFMAs; before the first
  // block it is a zero unit (acc += 0 * 0), so no branch keeps two schedules' registers alive
  Res rr[2];
  rr[0] = Res{iz, fz};
  rr[1] = Res{iz, fz};

  auto block = [&](int u, auto S_) {
    constexpr int S = decltype(S_)::value;
    i8_wait_vm<LPB * (P - 1)>();   // block u's DMA pieces and activation loads landed
    const unsigned char* sl = ring + S * SLOT;
    i32x4 wq[2];
    uint32_t wd[2];
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      wq[y] = *reinterpret_cast<const i32x4*>(sl + h * I8_PIECE + (32 * y + lr) * 16);
      wd[y] = *reinterpret_cast<const uint32_t*>(sl + 2 * I8_PIECE + (32 * y + lr) * 4);
    }
    // the activation fragments: this block's byte shift is ((32 x + lr) ldb + 34 kb) & 3 in {0, 2}
    const int uu = min(u, nbw - 1);
    const int kb = (g + KG * (uu / I8_KB)) * I8_KB + uu % I8_KB;
    i32x4 af[WJ];
    uint32_t db[WJ];
#pragma unroll
    for (int x = 0; x < WJ; ++x) {
      const int sh = ((32 * x + lr) * ldb4 + 2 * kb) & 3;   // the block's start within its dword
      const int sq = (sh + 2) & 3;                          // the quants' start (16 h keeps it)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        af[x][k] = (int)__builtin_amdgcn_alignbit(rq[S][x][k + 2], rq[S][x][k + 1], 8 * sq);
      db[x] = (rq[S][x][0] >> (8 * sh)) & 0xffffu;
    }
    auto mfmas = [&](int n, Res& R) {
      const int x = (n / 2) % WJ, y = n & 1;
      R.s = __builtin_amdgcn_mfma_i32_32x32x32_i8(af[x], wq[y], iz, 0, 0, 0);
      R.pr = __builtin_amdgcn_mfma_f32_32x32x8f16(__builtin_bit_cast(half4, uint2{db[x], 0u}),
                                                  __builtin_bit_cast(half4, uint2{wd[y], 0u}), fz, 0, 0, 0);
    };
    auto epi = [&](int n, const Res& R) {
      f32x16& c = acc[(n / 2) % WJ][n & 1];
#pragma unroll
      for (int e = 0; e < 16; ++e) c[e] = __builtin_fmaf((float)R.s[e], R.pr[e], c[e]);
      asm volatile("" : "+v"(c));   // here, not sunk to the loop's end (that keeps every unit's S and P live)
    };
    auto sb = [] { __builtin_amdgcn_sched_barrier(0); };
    sb();
    mfmas(0, rr[0]);
    sb();
    epi(UPB - 1, rr[(UPB - 1) % 2]);   // the previous block's last unit
    sb();
    unroll<UPB - 1>([&](auto NN) {
      constexpr int n = NN;
      mfmas(n + 1, rr[(n + 1) % 2]);
      sb();
      epi(n, rr[n % 2]);
      sb();
    });
    // this slot's registers were read by the MFMAs above and its LDS by the reads they waited
    // for: refill it P blocks ahead
    issue(u + P, S_);
  };
  if (nbw > 0) {
    unroll<P>([&](auto K) { issue(K, K); });
    int u0 = 0;
    for (; u0 + P <= nbw; u0 += P) unroll<P>([&](auto K) { block(u0 + K, K); });
    unroll<P - 1>([&](auto K) {
      if (u0 + (int)K < nbw) block(u0 + K, K);
    });
  }
  {   // the last block's last unit
    f32x16& c = acc[((UPB - 1) / 2) % WJ][(UPB - 1) & 1];
#pragma unroll
    for (int e = 0; e < 16; ++e) c[e] = __builtin_fmaf((float)rr[(UPB - 1) % 2].s[e], rr[(UPB - 1) % 2].pr[e], c[e]);
  }
  // K-group epilogue (gemm_fp6_kv_kernel's): every wave parks its partial tile, then the tile's
  // rows are summed over the groups in group order and stored as 512-byte runs of C
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

template <int T>
hipError_t launch_i8kv_t(const GemvArgs& p, const void* prepA, hipStream_t s) {
  constexpr size_t lds = (size_t)4 * 64 * (128 + 8) * 4;   // the epilogue's parked tiles (rings below it)
  const int grid = ((p.M + 127) / 128) * ((p.N + 63) / 64) * p.ne12 * p.ne13;
  auto kern = gemm_i8_kv_kernel<T, 3>;
  set_max_lds((const void*)kern, (int)lds);
  hipLaunchKernelGGL(kern, dim3((unsigned)grid), dim3(512), lds, s, p, static_cast<const unsigned char*>(prepA));
  return hipGetLastError();
}

template <int T>
void launch_prep_w_i8(const GemvArgs& p, unsigned char* ws, hipStream_t s) {
  const I8Layout L = I8Layout::of(p);
  const int64_t n = (int64_t)L.nit * I8_TI * L.nsteps * I8_KB;
  hipLaunchKernelGGL(prep_w_i8<T>, dim3((unsigned)((n + 255) / 256), (unsigned)L.na), dim3(256), 0, s, p, ws);
}

}  // namespace

bool gemm_i8kv_supported(int type) { return type == kQ4_0 || type == kQ5_0 || type == kQ8_0; }

size_t gemm_i8kv_weight_bytes(int type, const GemvArgs& p) {
  (void)type;
  return (size_t)I8Layout::of(p).a_bytes;
}

hipError_t prepare_i8kv_weights(int type, const GemvArgs& p, void* ws, hipStream_t s) {
  auto* w = static_cast<unsigned char*>(ws);
  switch (type) {
    case kQ4_0: launch_prep_w_i8<kQ4_0>(p, w, s); break;
    case kQ5_0: launch_prep_w_i8<kQ5_0>(p, w, s); break;
    case kQ8_0: launch_prep_w_i8<kQ8_0>(p, w, s); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// q8_0 activation rows only (4-byte aligned row starts not required: the loads realign)
hipError_t launch_gemm_i8kv(int type, const GemvArgs& p, const void* prepA, hipStream_t s) {
  if (!prepA || p.b_f32) return hipErrorInvalidValue;
  // the realignment of the 2-byte aligned blocks counts from a dword-aligned row / slice base
  if (((uintptr_t)p.B & 3) || (p.sb2 & 3) || (p.sb3 & 3)) return hipErrorInvalidValue;
  if (p.M == 0 || p.N == 0) return hipSuccess;
  switch (type) {
    case kQ4_0: return launch_i8kv_t<kQ4_0>(p, prepA, s);
    case kQ5_0: return launch_i8kv_t<kQ5_0>(p, prepA, s);
    case kQ8_0: return launch_i8kv_t<kQ8_0>(p, prepA, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
