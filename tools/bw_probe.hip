// bw_probe.hip -- what one kernel launch can stream from HBM on MI355X (gfx950): the ceiling
// for a single decode-sized GEMV call (BASELINE config 2: 9.46 MB per call).
// A read-only reduction kernel (dwordx4 loads, non-temporal, each workgroup a contiguous
// chunk, one 4-byte store per workgroup) over buffers rotated beyond the 256 MiB MALL;
// event-timed per launch over back-to-back launches, and an empty kernel for the fixed cost.
//   hipcc --offload-arch=gfx950 -O3 tools/bw_probe.hip -o tools/bw_probe && tools/bw_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                   \
  do {                                                          \
    hipError_t e = (x);                                         \
    if (e != hipSuccess) {                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));    \
      exit(1);                                                  \
    }                                                           \
  } while (0)

__global__ void empty_kernel(float*) {}

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

// UNROLL dwordx4 loads in flight per lane per iteration
template <int UNROLL>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ p, size_t n16_per_wg, float* out) {
  const u32x4* base = p + (size_t)blockIdx.x * n16_per_wg;
  uint32_t acc = 0;
  for (size_t i = threadIdx.x; i < n16_per_wg; i += 256 * UNROLL) {
    u32x4 v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) {
      const size_t j = i + (size_t)u * 256;
      v[u] = j < n16_per_wg ? __builtin_nontemporal_load(base + j) : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) out[blockIdx.x] = (float)acc;   // keeps the loads live
}

int main() {
  const size_t total = 1ull << 30;   // 1 GiB pool: rotation beyond the 256 MiB MALL
  char* pool;
  float* out;
  CK(hipMalloc(&pool, total));
  CK(hipMemset(pool, 1, total));
  CK(hipMalloc(&out, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 200;
  auto time_us = [&](auto launch) {
    for (int w = 0; w < 20; ++w) launch(w);
    CK(hipEventRecord(e0, s));
    for (int r = 0; r < reps; ++r) launch(r);
    CK(hipEventRecord(e1, s));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    return ms * 1000.0 / reps;
  };
  printf("{\"empty_kernel_us\": %.3f", time_us([&](int) { empty_kernel<<<256, 256, 0, s>>>(out); }));
  const size_t sizes[] = {9437184, 4 * 9437184ull, 33 * 9437184ull};
  const int wgs[] = {256, 512, 1024, 2048};
  for (size_t bytes : sizes) {
    const size_t slots = total / bytes;
    for (int wg : wgs) {
      const size_t n16 = bytes / 16 / wg;
      auto go = [&](int r) {
        const u32x4* p = (const u32x4*)(pool + (size_t)(r % slots) * bytes);
        read_kernel<4><<<wg, 256, 0, s>>>(p, n16, out);
      };
      const double us = time_us(go);
      printf(", \"read_%zuB_wg%d_us\": %.3f, \"read_%zuB_wg%d_TBs\": %.3f", bytes, wg, us, bytes, wg,
             (double)n16 * 16 * wg / us * 1e-6);
    }
  }
  printf("}\n");
  return 0;
}
