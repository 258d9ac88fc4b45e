// floor_probe.hip -- the single-launch read floor of BASELINE config 2 by launch shape.
// bench.py's roofline.single_launch_floor_us times a read-only kernel on the config-2 GEMV's own
// grid (512 x 512 threads, 36 B per thread) and found it no faster than the GEMV (round 6).  This
// probe asks which launch shape reads the same 9,437,184 weight bytes fastest: workgroup size x
// b128 loads per thread (grid = bytes / (block x 16 x loads)), workgroup b on chunk b or XCD-
// contiguous chunks; each launch timed alone by its own dispatch timestamps (hipExtLaunchKernelGGL
// events, the kernel tracer's duration), over copies rotated through a 1 GiB pool (> MALL), the
// median of 200.  An empty kernel on each grid gives the dispatch cost alone.
//   hipcc --offload-arch=gfx950 -O3 tools/floor_probe.hip -o tools/floor_probe && tools/floor_probe
#include <hip/hip_ext.h>
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                \
  do {                                                       \
    hipError_t e_ = (x);                                     \
    if (e_ != hipSuccess) {                                  \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); \
      exit(1);                                               \
    }                                                        \
  } while (0)

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int BLOCK>
__global__ __launch_bounds__(BLOCK) void empty_k(uint32_t*) {}

// LOADS b128 per thread, all issued before any is used; chunk = BLOCK * 16 * LOADS bytes
template <int BLOCK, int LOADS, bool XCD>
__global__ __launch_bounds__(BLOCK) void read_k(const unsigned char* A, uint32_t bytes, uint32_t* sink) {
  int b = blockIdx.x;
  if (XCD) {   // XCD x (= b % 8 under round-robin dispatch) reads a contiguous range of chunks
    const int n = gridDim.x, x = b & 7, k = b >> 3, q = n >> 3, r = n & 7;
    b = x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
  }
  const uint32_t base = (uint32_t)b * BLOCK * 16 * LOADS + 16 * threadIdx.x;
  u32x4 v[LOADS];
#pragma unroll
  for (int u = 0; u < LOADS; ++u) {
    const uint32_t o = base + (uint32_t)u * BLOCK * 16;
    v[u] = o + 16 <= bytes ? *reinterpret_cast<const u32x4*>(A + o) : u32x4{0, 0, 0, 0};
  }
  uint32_t x = 0;
#pragma unroll
  for (int u = 0; u < LOADS; ++u) x ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  if (x == 0x9e3779b9u) sink[blockIdx.x] = x;
}

int main() {
  const size_t pool_bytes = 1ull << 30, unit = 9437184;   // config 2's weight bytes
  const int copies = (int)(pool_bytes / unit);
  unsigned char* pool;
  uint32_t* sink;
  CK(hipMalloc(&pool, pool_bytes));
  CK(hipMemset(pool, 1, pool_bytes));
  CK(hipMalloc(&sink, 1 << 20));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  int c = 0;
  auto med = [&](auto launch) {
    std::vector<float> v;
    for (int i = 0; i < 220; ++i) {
      launch(pool + (size_t)(c++ % copies) * unit);
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (i >= 20) v.push_back(ms * 1e3f);
    }
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
  };
  printf("{\"probe\": \"floor_probe\", \"bytes\": %zu, \"rows\": [\n", unit);
  bool first = true;
  auto run = [&](auto kread, auto kempty, int block, int loads, bool xcd) {
    const unsigned grid = (unsigned)((unit + (size_t)block * 16 * loads - 1) / ((size_t)block * 16 * loads));
    const float tr = med([&](const unsigned char* a) {
      hipExtLaunchKernelGGL(kread, dim3(grid), dim3(block), 0, s, e0, e1, 0, a, (uint32_t)unit, sink);
    });
    const float te = med([&](const unsigned char*) {
      hipExtLaunchKernelGGL(kempty, dim3(grid), dim3(block), 0, s, e0, e1, 0, sink);
    });
    printf("%s{\"block\": %d, \"loads\": %d, \"xcd\": %d, \"grid\": %u, \"waves_per_simd\": %.2f, \"read_us\": %.3f, "
           "\"empty_us\": %.3f, \"TBps\": %.3f}",
           first ? "" : ",\n", block, loads, (int)xcd, grid, grid * (block / 64.0) / 1024.0, tr, te, unit / tr / 1e6);
    first = false;
    fflush(stdout);
  };
#define RUN(B, L)                                                                              \
  run(read_k<B, L, false>, empty_k<B>, B, L, false);                                           \
  run(read_k<B, L, true>, empty_k<B>, B, L, true);
  RUN(256, 1) RUN(256, 2) RUN(256, 3) RUN(256, 4) RUN(256, 6) RUN(256, 8) RUN(256, 16)
  RUN(512, 1) RUN(512, 2) RUN(512, 3) RUN(512, 4) RUN(512, 6) RUN(512, 8)
  RUN(1024, 1) RUN(1024, 2) RUN(1024, 3) RUN(1024, 4)
  printf("\n]}\n");
  return 0;
}
