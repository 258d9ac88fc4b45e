// rpw_probe.hip -- where the single-call decode GEMV's time goes (BASELINE config 2: one
// 4096 x 4096 q4_0 row set = 9.44 MB per launch), as the row-per-wave kernel
// (csrc/lamm_gemv_rpw.hip) lays it out: one wave per row, 4 waves per workgroup, 1024
// workgroups.  Each mode adds one piece; launches back to back over 33 weight copies (> MALL),
// hipEvent-timed per launch.
//   0 coalesced : the row as 16-byte chunks per lane (lane l: chunks l, l+64, l+128), xor-reduce
//   1 blocks    : the kernel's pattern -- lane l takes blocks l and l+64 whole (b128 + b64 at the
//                 block's dword-aligned start), xor-reduce
//   2 + staging : mode 1 + the activation row (q8_0, 4352 B) staged into LDS by 128 threads and a
//                 workgroup barrier before the reduce
//   3 + compute : mode 2 + the real q4_0 x q8_0 block dots, fixed-order wave reduction, C store
//   4 blocks + per-lane B : mode 1 + each lane loading its own two activation blocks (L2-served)
//                 instead of the LDS staging and barrier
//   5 coalesced + LDS     : mode 0's loads, the row written to a per-wave LDS slice, each lane then
//                 reading its two blocks back (dword reads + realignment), xor-reduce
//   hipcc --offload-arch=gfx950 -O3 tools/rpw_probe.hip -o tools/rpw_probe && tools/rpw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                               \
    }                                                        \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

constexpr int M = 4096, NB = 128, BPB = 18, ROW = NB * BPB;   // q4_0 row: 2304 B
constexpr int WAVES = 4;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p, uint32_t n) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)n, 0x00020000);
}

__device__ __forceinline__ float wave_sum(float x) {
  for (int o = 32; o >= 1; o >>= 1) x += __shfl_xor(x, o);
  return x;
}

template <int MODE>
__global__ __launch_bounds__(64 * WAVES) void probe(const unsigned char* A, const unsigned char* B, float* C) {
  __shared__ uint32_t sb[NB * 9 + 1];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int row = blockIdx.x * WAVES + wave;
  const auto ra = rsrc(A + (size_t)row * ROW, ROW);
  uint32_t w[2][6];
  u32x4 c[3];
  __shared__ uint32_t rowbuf[WAVES][ROW / 4 + 16];
  uint32_t bw[2][10];
  if constexpr (MODE == 4) {   // activation blocks l and l+64 straight into registers (before A)
    const auto rb = rsrc(B, NB * 34);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const uint32_t off = ((lane + 64 * it) * 34) & ~3u;
      const u32x4 v0 = __builtin_amdgcn_raw_buffer_load_b128(rb, off, 0, 0);
      const u32x4 v1 = __builtin_amdgcn_raw_buffer_load_b128(rb, off + 16, 0, 0);
      const u32x2 v2 = __builtin_amdgcn_raw_buffer_load_b64(rb, off + 32, 0, 0);
      bw[it][0] = v0[0]; bw[it][1] = v0[1]; bw[it][2] = v0[2]; bw[it][3] = v0[3];
      bw[it][4] = v1[0]; bw[it][5] = v1[1]; bw[it][6] = v1[2]; bw[it][7] = v1[3];
      bw[it][8] = v2[0]; bw[it][9] = v2[1];
    }
  }
  if constexpr (MODE == 0 || MODE == 5) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int ch = lane + 64 * k;
      c[k] = __builtin_amdgcn_raw_buffer_load_b128(ra, ch < ROW / 16 ? ch * 16 : 0x7ffffff0, 0, 2);
    }
  } else {
    if constexpr (MODE == 2 || MODE == 3) {   // activation loads first (vmcnt order), like the kernel
      if (threadIdx.x < NB) {
        const auto rb = rsrc(B, NB * 34);
        const uint32_t off = (threadIdx.x * 34) & ~3u;
#pragma unroll
        for (int k = 0; k < 9; ++k) sb[threadIdx.x * 9 + k] = __builtin_amdgcn_raw_buffer_load_b32(rb, off + 4 * k, 0, 0);
      }
    }
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const uint32_t off = ((lane + 64 * it) * BPB) & ~3u;
      const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 2);
      const u32x2 u = __builtin_amdgcn_raw_buffer_load_b64(ra, off + 16, 0, 2);
      w[it][0] = v[0]; w[it][1] = v[1]; w[it][2] = v[2]; w[it][3] = v[3]; w[it][4] = u[0]; w[it][5] = u[1];
    }
    if constexpr (MODE == 2 || MODE == 3) __syncthreads();
  }
  float acc = 0.f;
  if constexpr (MODE == 5) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const int ch = lane + 64 * k;
      if (ch < ROW / 16)
#pragma unroll
        for (int q = 0; q < 4; ++q) rowbuf[wave][ch * 4 + q] = c[k][q];
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);   // lgkmcnt(0): this wave's LDS writes done (wave-local slice)
    uint32_t x = 0;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int o = ((lane + 64 * it) * BPB) >> 2;
#pragma unroll
      for (int k = 0; k < 6; ++k) x ^= rowbuf[wave][o + k];
    }
    acc = (float)(x & 0xff);
  } else if constexpr (MODE == 4) {
    uint32_t x = 0;
#pragma unroll
    for (int it = 0; it < 2; ++it)
#pragma unroll
      for (int k = 0; k < 6; ++k) x ^= w[it][k] ^ bw[it][k] ^ bw[it][k + 4];
    acc = (float)(x & 0xff);
  } else if constexpr (MODE == 0) {
    uint32_t x = 0;
#pragma unroll
    for (int k = 0; k < 3; ++k) x ^= c[k][0] ^ c[k][1] ^ c[k][2] ^ c[k][3];
    acc = (float)(x & 0xff);
  } else if constexpr (MODE < 3) {
    uint32_t x = 0;
#pragma unroll
    for (int it = 0; it < 2; ++it)
#pragma unroll
      for (int k = 0; k < 6; ++k) x ^= w[it][k];
    if constexpr (MODE == 2) x ^= sb[lane];
    acc = (float)(x & 0xff);
  } else {
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int b = lane + 64 * it;
      const int sh = ((b * BPB) & 3) * 8;
      uint32_t m[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) m[k] = __builtin_amdgcn_alignbit(w[it][k + 1], w[it][k], sh);
      const float da = (float)__builtin_bit_cast(_Float16, (uint16_t)(m[0] & 0xffff));
      uint32_t qs[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) qs[k] = __builtin_amdgcn_alignbit(m[k + 1], m[k], 16);
      // activation block b: d (2 B) + 32 int8 at byte 34 * b of the staged row
      const uint32_t* s = &sb[b * 9];
      const int bs = ((b * 34) & 3) * 8;
      uint32_t bm[9];
#pragma unroll
      for (int k = 0; k < 9; ++k) bm[k] = __builtin_amdgcn_alignbit(s[k + 1], s[k], bs);
      const float db = (float)__builtin_bit_cast(_Float16, (uint16_t)(bm[0] & 0xffff));
      int sum = 0, sq = 0;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t bl = __builtin_amdgcn_alignbit(bm[k + 1], bm[k], 16);
        const uint32_t bh = __builtin_amdgcn_alignbit(bm[k + 5], bm[k + 4], 16);
        sum = __builtin_amdgcn_sdot4((int)(qs[k] & 0x0f0f0f0fu), (int)bl, sum, false);
        sum = __builtin_amdgcn_sdot4((int)((qs[k] >> 4) & 0x0f0f0f0fu), (int)bh, sum, false);
        sq = __builtin_amdgcn_sdot4((int)bl, 0x01010101, sq, false);
        sq = __builtin_amdgcn_sdot4((int)bh, 0x01010101, sq, false);
      }
      acc = __builtin_fmaf(da * db, (float)(sum - 8 * sq), acc);
    }
  }
  acc = wave_sum(acc);
  if (MODE == 3 ? lane == 0 : acc == 1234567.f) C[row] = acc;
}

int main() {
  const size_t bytes = (size_t)M * ROW, slots = 33;
  unsigned char *pool, *B;
  float* C;
  CK(hipMalloc(&pool, bytes * slots));
  CK(hipMemset(pool, 0x35, bytes * slots));
  CK(hipMalloc(&B, 8192));
  CK(hipMemset(B, 0x11, 8192));
  CK(hipMalloc(&C, M * 4));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 330;
  auto time_us = [&](auto launch) {
    for (int w = 0; w < 33; ++w) launch(w);
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch(r);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.0 / reps;
  };
  const dim3 g(M / WAVES), b(64 * WAVES);
  printf("{\"coalesced_us\": %.3f", time_us([&](int r) { probe<0><<<g, b, 0, s>>>(pool + (r % slots) * bytes, B, C); }));
  printf(", \"blocks_us\": %.3f", time_us([&](int r) { probe<1><<<g, b, 0, s>>>(pool + (r % slots) * bytes, B, C); }));
  printf(", \"blocks_staging_us\": %.3f", time_us([&](int r) { probe<2><<<g, b, 0, s>>>(pool + (r % slots) * bytes, B, C); }));
  printf(", \"blocks_staging_compute_us\": %.3f", time_us([&](int r) { probe<3><<<g, b, 0, s>>>(pool + (r % slots) * bytes, B, C); }));
  printf(", \"blocks_lane_b_us\": %.3f", time_us([&](int r) { probe<4><<<g, b, 0, s>>>(pool + (r % slots) * bytes, B, C); }));
  printf(", \"coalesced_lds_transpose_us\": %.3f", time_us([&](int r) { probe<5><<<g, b, 0, s>>>(pool + (r % slots) * bytes, B, C); }));
  printf(", \"bytes_per_launch\": %zu}\n", bytes);
  return 0;
}
