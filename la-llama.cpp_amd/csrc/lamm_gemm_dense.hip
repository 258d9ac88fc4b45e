// lamm_gemm_dense.hip -- prefill GEMM (N > 8) for unquantized rows: F32 x F32 (the reference's
// lamm_kernel_f32, src/lamm_kernel_f32.hpp, which it runs as a scalar/SIMD dot per (i, j)) and
// the §8f F16 x F16 rows (ggml_vec_dot_f16, LC/ggml.c:1589-1629: the attention matmuls of an
// F16 KV cache).  Without it these shapes ran as N/8 grouped GEMV launches.
//
//   C[j*ldc + i] = sum_k A[i,k] * B[j,k]
//
// Matrix cores, exact products, fp32 accumulation:
//   f32: v_mfma_f32_32x32x2_f32  (f32 in, f32 acc: each product and sum is an fp32 fmaf)
//   f16: v_mfma_f32_32x32x16_f16 (exact f16 x f16 products, fp32 accumulation)
// Tile: 128 (i) x 128 (j) per 256-thread workgroup, a wave owns 64 x 64 = 2 x 2 MFMA tiles.
// K-step = 128 bytes of every row (32 f32 / 64 f16).  The MFMA's k index is a free
// relabelling as long as both operands agree, so lane half h consumes bytes [64h, 64h+64) of
// its row chunk: four ds_read_b128 per fragment, contiguous per lane.  LDS rows are padded to
// 144 bytes, which spreads any 16 consecutive rows over all 64 banks (ds_read_b128 reads in
// 16-lane groups): conflict-free reads.  Global -> registers (next step, in flight during this
// step's MFMAs) -> ds_write_b128, double-buffered LDS, one barrier per step.
// Ragged M / N are zero-filled by the loads, ragged K masked per element (row padding may be
// NaN), so every lane runs the same MFMA stream.
#include <cstdlib>

#include "lamm_device.h"
#include "lamm_kernels.h"
#include "lamm_knobs.h"

namespace lamm {
namespace {

typedef _Float16 half8 __attribute__((ext_vector_type(8)));

constexpr int DG_T = 128;                 // tile rows (i) and columns (j)
constexpr int DG_NT = 256;                // threads: 4 waves, 2 (i) x 2 (j)
constexpr int DG_ROW = 144;               // LDS bytes per row chunk (128 + 16 pad)
constexpr int DG_OP = DG_T * DG_ROW;      // one operand tile in LDS
constexpr int DG_STAGE = 2 * DG_OP;       // A + B
constexpr int DG_PPT = DG_T * 8 / DG_NT;  // 16-byte pieces per thread per operand (4)

template <int T> struct DenseG;
template <> struct DenseG<kF32> { static constexpr int EB = 4; };
template <> struct DenseG<kF16> { static constexpr int EB = 2; };

// keep the first nv elements of a 16-byte piece (nv may be <= 0 or >= the piece's count)
template <int EB>
__device__ __forceinline__ u32x4 mask_piece(u32x4 v, int nv) {
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    uint32_t m;
    if constexpr (EB == 4) m = c < nv ? 0xffffffffu : 0u;
    else m = 2 * c + 1 < nv ? 0xffffffffu : (2 * c < nv ? 0x0000ffffu : 0u);
    v[c] &= m;
  }
  return v;
}

// BAL: B rows 16-byte aligned (b128 loads); else dword (f32) / halfword (f16) loads
template <int T, bool BAL>
__global__ __launch_bounds__(DG_NT) void gemm_dense_kernel(GemvArgs p, int nsplit, float* part) {
  constexpr int EB = DenseG<T>::EB, KS = 128 / EB, EPP = 16 / EB;   // elems per step / piece
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const int wi = w & 1, wj = w >> 1;
  const int nit = (p.M + DG_T - 1) / DG_T, njt = (p.N + DG_T - 1) / DG_T;
  // XCD-aware order: the 8 workgroups dealt to the 8 XCDs in one round take 8 different
  // column groups, and consecutive ids on one XCD walk neighbouring tiles (shared L2 lines)
  int it, jt, z, sp;
  {
    const int ntile = nit * njt * p.ne12 * p.ne13, nwg = ntile * nsplit;
    const int id = blockIdx.x, x = id & 7, k = id >> 3, q = nwg >> 3, rmd = nwg & 7;
    int wv = x < rmd ? x * (q + 1) + k : rmd * (q + 1) + (x - rmd) * q + k;
    sp = wv / ntile;   // split-major (K-splits of a tile run on different XCDs' rounds)
    wv %= ntile;
    z = wv / (nit * njt);
    const int r = wv % (nit * njt);
    jt = r / nit;
    it = r % nit;
  }
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int K = p.K, nsteps = (K + KS - 1) / KS;
  const int k0 = (int)((int64_t)sp * nsteps / nsplit), k1 = (int)((int64_t)(sp + 1) * nsteps / nsplit);
  const int i0 = it * DG_T, j0 = jt * DG_T;
  const int mrows = min(DG_T, p.M - i0), ncols = min(DG_T, p.N - j0);
  const int64_t abytes = (int64_t)(mrows - 1) * p.lda + (int64_t)K * EB;
  const int64_t bbytes = (int64_t)(ncols - 1) * p.ldb + (int64_t)K * EB;
  const auto ra = make_rsrc(Az + (int64_t)i0 * p.lda, (uint32_t)min((abytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
  const auto rb = make_rsrc(Bz + (int64_t)j0 * p.ldb, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));

  // piece q = t + 256*r of a tile: row q / 8, 16-byte piece q % 8 of the row's 128-byte chunk
  u32x4 ga[DG_PPT], gb[DG_PPT];
  auto gload = [&](int ks) {
#pragma unroll
    for (int r = 0; r < DG_PPT; ++r) {
      const int q = t + DG_NT * r, row = q >> 3, pc = q & 7;
      const int e = ks * KS + pc * EPP;   // first element of the piece
      const int nv = K - e;
      {
        const uint32_t off = row < mrows && nv > 0 ? (uint32_t)(row * p.lda + e * EB) : 0x7ffffff0u;
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
        ga[r] = nv < EPP ? mask_piece<EB>(v, nv) : v;
      }
      const bool ok = row < ncols && nv > 0;
      if constexpr (BAL) {
        const uint32_t off = ok ? (uint32_t)(row * p.ldb + e * EB) : 0x7ffffff0u;
        u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0);
        gb[r] = nv < EPP ? mask_piece<EB>(v, nv) : v;
      } else {
        u32x4 v = {0u, 0u, 0u, 0u};
        if (ok) {
          const uint32_t base = (uint32_t)(row * p.ldb + e * EB);
#pragma unroll
          for (int c = 0; c < 4; ++c) {
            if constexpr (EB == 4) {
              if (c < nv) v[c] = bload4(rb, base + 4 * c);
            } else {
              uint32_t lo = 0, hi = 0;
              if (2 * c < nv) lo = bload2(rb, base + 4 * c);
              if (2 * c + 1 < nv) hi = bload2(rb, base + 4 * c + 2);
              v[c] = lo | (hi << 16);
            }
          }
        }
        gb[r] = v;
      }
    }
  };
  auto swrite = [&](int buf) {
    unsigned char* sA = smem + buf * DG_STAGE;
    unsigned char* sB = sA + DG_OP;
#pragma unroll
    for (int r = 0; r < DG_PPT; ++r) {
      const int q = t + DG_NT * r, row = q >> 3, pc = q & 7;
      *(u32x4*)(sA + row * DG_ROW + pc * 16) = ga[r];
      *(u32x4*)(sB + row * DG_ROW + pc * 16) = gb[r];
    }
  };

  f32x16 acc[2][2];   // [j sub-tile][i sub-tile]
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[x][y][e] = 0.f;

  gload(k0);
  swrite(k0 & 1);
  __syncthreads();
  for (int ks = k0; ks < k1; ++ks) {
    if (ks + 1 < k1) gload(ks + 1);   // in flight during this step's MFMAs
    const unsigned char* sA = smem + (ks & 1) * DG_STAGE;
    const unsigned char* sB = sA + DG_OP;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {   // 16-byte quarter of this lane half's 64 bytes
      u32x4 fa[2], fb[2];
#pragma unroll
      for (int y = 0; y < 2; ++y) fa[y] = *(const u32x4*)(sA + (64 * wi + 32 * y + lr) * DG_ROW + 64 * h + 16 * qq);
#pragma unroll
      for (int x = 0; x < 2; ++x) fb[x] = *(const u32x4*)(sB + (64 * wj + 32 * x + lr) * DG_ROW + 64 * h + 16 * qq);
      if constexpr (T == kF16) {
#pragma unroll
        for (int x = 0; x < 2; ++x)
#pragma unroll
          for (int y = 0; y < 2; ++y)
            acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x16_f16(__builtin_bit_cast(half8, fb[x]),
                                                               __builtin_bit_cast(half8, fa[y]), acc[x][y], 0, 0, 0);
      } else {   // 4 k-pairs per 16 bytes; the 4 accumulators interleave so no MFMA waits on its predecessor
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
          for (int x = 0; x < 2; ++x)
#pragma unroll
            for (int y = 0; y < 2; ++y) {
              const uint32_t bc = fb[x][c], ac = fa[y][c];
              acc[x][y] = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(bc), __uint_as_float(ac), acc[x][y],
                                                               0, 0, 0);
            }
      }
    }
    if (ks + 1 < k1) swrite((ks + 1) & 1);   // the buffer everyone finished reading at step ks-1
    __syncthreads();
  }

  // D layout (srcA = activation rows j, srcB = weight rows i): lane -> i = lr, element e ->
  // j = (e & 3) + 8 (e >> 2) + 4 h.  For each e the 32 lanes of a half store 128 contiguous bytes.
  float* Co = Cz;
  int64_t ldo = p.ldc;
  if (nsplit > 1) {   // partial tile of split sp -> part[sp][z][j][i]
    Co = part + ((int64_t)sp * p.ne12 * p.ne13 + z) * p.N * p.M;
    ldo = p.M;
  }
#pragma unroll
  for (int x = 0; x < 2; ++x)
#pragma unroll
    for (int y = 0; y < 2; ++y) {
      const int i = i0 + 64 * wi + 32 * y + lr;
#pragma unroll
      for (int e = 0; e < 16; ++e) {
        const int j = j0 + 64 * wj + 32 * x + (e & 3) + 8 * (e >> 2) + 4 * h;
        if (i < p.M && j < p.N) Co[(int64_t)j * ldo + i] = acc[x][y][e];
      }
    }
}

// Small F32 GEMMs (BASELINE config 1: 512^3 is 16 of the 128 x 128 tiles above, which needed split-K
// partials and a reduce launch, 18.3 us): one 32 x 32 output tile per 256-thread workgroup -- 256
// workgroups for 512^3 -- whose 4 waves take a quarter of K each (K-groups), every operand straight
// from HBM / L2 into VGPRs (lane (r, h) takes row r's elements [128 c + 64 h, + 64) of chunk c: 16
// b128 loads per operand, no LDS staging), one v_mfma_f32_32x32x2_f32 chain per wave, and the four
// partial tiles summed through LDS in group order before one store per output.  No partials in HBM,
// no second launch.  K % 4 == 0 (whole 16-byte pieces; the tail past K is zeroed per piece).
constexpr int SF_CH = 128;   // floats of K per chunk (lane half h: 64 of them)

__global__ __launch_bounds__(256) void gemm_f32_small_kernel(GemvArgs p) {
  __shared__ float red[4][32][33];
  const int t = threadIdx.x, lane = t & 63;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int lr = lane & 31, h = lane >> 5;
  const int nit = (p.M + 31) / 32, njt = (p.N + 31) / 32;
  const int per = nit * njt, z = blockIdx.x / per, r = blockIdx.x % per;
  const int it = r % nit, jt = r / nit;
  const int i12 = z % p.ne12, i13 = z / p.ne12;
  const unsigned char* Az = p.A + (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
  const unsigned char* Bz = p.B + (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
  float* Cz = p.C + (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  const int K = p.K, i0 = it * 32, j0 = jt * 32;
  const int mrows = min(32, p.M - i0), ncols = min(32, p.N - j0);
  const int64_t abytes = (int64_t)(mrows - 1) * p.lda + (int64_t)K * 4;
  const int64_t bbytes = (int64_t)(ncols - 1) * p.ldb + (int64_t)K * 4;
  const auto ra = make_rsrc(Az + (int64_t)i0 * p.lda, (uint32_t)min(abytes, (int64_t)0x7fffffff));
  const auto rb = make_rsrc(Bz + (int64_t)j0 * p.ldb, (uint32_t)min(bbytes, (int64_t)0x7fffffff));
  const int nch = (K + SF_CH - 1) / SF_CH, c0 = w * nch / 4, c1 = (w + 1) * nch / 4;
  f32x16 acc = {};
  for (int c = c0; c < c1; ++c) {
    u32x4 a[16], b[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const int e = c * SF_CH + 64 * h + 4 * q;   // the piece's first element
      const bool in = e < K;                       // K % 4 == 0: a piece is all in or all out
      a[q] = __builtin_amdgcn_raw_buffer_load_b128(
          ra, in && lr < mrows ? (uint32_t)(lr * p.lda + 4 * e) : 0x7ffffff0u, 0, 0);
      b[q] = __builtin_amdgcn_raw_buffer_load_b128(
          rb, in && lr < ncols ? (uint32_t)(lr * p.ldb + 4 * e) : 0x7ffffff0u, 0, 0);
    }
#pragma unroll
    for (int q = 0; q < 16; ++q)
#pragma unroll
      for (int k = 0; k < 4; ++k)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(__uint_as_float(b[q][k]), __uint_as_float(a[q][k]), acc, 0, 0, 0);
  }
  // D layout (srcA = activation rows j, srcB = weight rows i): lane -> i = lr, e -> j = (e & 3) + 8 (e >> 2) + 4 h
#pragma unroll
  for (int e = 0; e < 16; ++e) red[w][(e & 3) + 8 * (e >> 2) + 4 * h][lr] = acc[e];
  __syncthreads();
  const int jl = t >> 3, il = 4 * (t & 7);   // 4 consecutive outputs of row jl per thread
  float v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) v[k] = ((red[0][jl][il + k] + red[1][jl][il + k]) + red[2][jl][il + k]) + red[3][jl][il + k];
  if (jl < ncols) {
    float* o = Cz + (int64_t)(j0 + jl) * p.ldc + i0 + il;
    if (il + 3 < mrows && ((uintptr_t)o & 15) == 0) {
      *reinterpret_cast<f32x4*>(o) = f32x4{v[0], v[1], v[2], v[3]};
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        if (il + k < mrows) o[k] = v[k];
    }
  }
}

// K-splits: double until the grid covers 256 CUs, keeping >= 4 K-steps per split
// (LAMM_DENSE_SPLIT=n forces n)
int dg_nsplit(const GemvArgs& p, int eb) {
  const int nit = (p.M + DG_T - 1) / DG_T, njt = (p.N + DG_T - 1) / DG_T;
  const int tiles = nit * njt * p.ne12 * p.ne13;
  const int nsteps = (p.K + 128 / eb - 1) / (128 / eb);
  int n = 1;
  if (knobs().dense_split > 0) {
    n = knobs().dense_split;
  } else {
    while (tiles * n < 256 && n < 8 && nsteps / (2 * n) >= 4) n *= 2;
  }
  return n < 1 ? 1 : (n > nsteps ? (nsteps < 1 ? 1 : nsteps) : n);
}

// the small-tile F32 form: grids the 128 x 128 tiles would split (fewer than 64 of them), K % 4 == 0
bool f32_small(const GemvArgs& p) {
  const int64_t tiles = (int64_t)((p.M + DG_T - 1) / DG_T) * ((p.N + DG_T - 1) / DG_T) * p.ne12 * p.ne13;
  const int64_t small = (int64_t)((p.M + 31) / 32) * ((p.N + 31) / 32) * p.ne12 * p.ne13;
  return knobs().dense_split <= 0 && tiles < 64 && p.K % 4 == 0 && small <= 4096 && (p.lda & 15) == 0 &&
         (p.ldb & 15) == 0 && ((uintptr_t)p.A & 15) == 0 && ((uintptr_t)p.B & 15) == 0 && (p.sa2 & 15) == 0 &&
         (p.sa3 & 15) == 0 && (p.sb2 & 15) == 0 && (p.sb3 & 15) == 0;
}

template <int T, bool BAL>
hipError_t launch_dg(const GemvArgs& p, void* ws, hipStream_t s) {
  if (T == kF32 && f32_small(p)) {
    const int64_t nwg = (int64_t)((p.M + 31) / 32) * ((p.N + 31) / 32) * p.ne12 * p.ne13;
    hipLaunchKernelGGL(gemm_f32_small_kernel, dim3((unsigned)nwg), dim3(256), 0, s, p);
    return hipGetLastError();
  }
  const int nit = (p.M + DG_T - 1) / DG_T, njt = (p.N + DG_T - 1) / DG_T;
  const int nsplit = dg_nsplit(p, DenseG<T>::EB);
  const int64_t nwg = (int64_t)nit * njt * p.ne12 * p.ne13 * nsplit;
  float* part = static_cast<float*>(ws);
  if (nwg > 0x7fffffff) return hipErrorInvalidValue;
  constexpr size_t lds = 2 * DG_STAGE;
  set_max_lds((const void*)gemm_dense_kernel<T, BAL>, (int)lds);
  hipLaunchKernelGGL((gemm_dense_kernel<T, BAL>), dim3((unsigned)nwg), dim3(DG_NT), lds, s, p, nsplit, part);
  if (nsplit > 1) launch_splitk_reduce(p, nsplit, part, s);
  return hipGetLastError();
}

}  // namespace

bool gemm_dense_supported(int type) { return type == kF32 || type == kF16; }
// a 128-row tile's bytes addressable by the kernels' 32-bit buffer offsets (other calls: grouped GEMV)
bool gemm_dense_args_ok(const GemvArgs& p) {
  return (int64_t)DG_T * p.lda < 0x7fffffff && (int64_t)DG_T * p.ldb < 0x7fffffff;
}

size_t gemm_dense_workspace_bytes(int type, const GemvArgs& p) {
  if (type == kF32 && f32_small(p)) return 0;
  const int n = dg_nsplit(p, type == kF32 ? 4 : 2);
  return n > 1 ? (size_t)n * p.ne12 * p.ne13 * (size_t)p.N * p.M * sizeof(float) + 256 : 0;
}

hipError_t launch_gemm_dense(int type, const GemvArgs& p, void* ws, hipStream_t s) {
  if (p.M == 0 || p.N == 0) return hipSuccess;
  const bool bal = ((uintptr_t)p.B & 15) == 0 && (p.ldb & 15) == 0 && (p.sb2 & 15) == 0 && (p.sb3 & 15) == 0;
  switch (type) {
    case kF32: return bal ? launch_dg<kF32, true>(p, ws, s) : launch_dg<kF32, false>(p, ws, s);
    case kF16: return bal ? launch_dg<kF16, true>(p, ws, s) : launch_dg<kF16, false>(p, ws, s);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
