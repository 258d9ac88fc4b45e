// write_probe.hip -- what a short write-heavy launch costs on this chip (config 3's activation
// prep writes ~4 MB of fp6 planes from ~2 MB of q8 rows and takes ~6.4 us).  Each variant is
// hipGraph-replayed 1000 times, per-launch us = graph time / launches:
//   rd<MB>        : read-only pass (b128 per lane, nt)
//   wr<MB>-<pol>  : write-only pass, b128 stores with cache policy pol (0 default, nt, sc0sc1 =
//                   write-through, ntsc = nt + sc0 + sc1)
//   rw<MB>        : read 2 MB + write <MB> (the prep's shape), default stores
//   empty
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I la-llama.cpp_amd/csrc tools/write_probe.hip -o tools/write_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>

#include "lamm_device.h"

using namespace lamm;

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e_ = (x);                                                                           \
    if (e_ != hipSuccess) {                                                                        \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));           \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

constexpr int REPS = 1000;

// one b128 per thread per pass; grid-stride over n16 16-byte chunks
template <int POL>
__global__ __launch_bounds__(256) void kWrite(u32x4* __restrict__ dst, int64_t n16, uint32_t salt) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = u32x4{(uint32_t)i, salt, (uint32_t)i ^ salt, 7u};
    if constexpr (POL == 0) dst[i] = v;
    else if constexpr (POL == 1) __builtin_nontemporal_store(v, dst + i);
    else {
      const auto r = make_rsrc(dst, 0x7fffffffu);
      // buffer_store_dwordx4 with aux bits: 1 = sc0, 2 = nt, 16 = sc1 (gfx950)
      __builtin_amdgcn_raw_buffer_store_b128(v, r, (uint32_t)(i * 16), 0, POL == 2 ? (1 | 16) : (1 | 2 | 16));
    }
  }
}

__global__ __launch_bounds__(256) void kRead(const u32x4* __restrict__ src, int64_t n16, uint32_t* out) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  uint32_t x = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n16; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(src + i);
    x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (x == 0x12345678u) out[0] = x;
}

__global__ __launch_bounds__(256) void kReadWrite(const u32x4* __restrict__ src, int64_t n16r, u32x4* __restrict__ dst,
                                                  int64_t n16w) {
  const int64_t stride = (int64_t)gridDim.x * 256;
  const int64_t i0 = (int64_t)blockIdx.x * 256 + threadIdx.x;
  uint32_t x = 0;
  for (int64_t i = i0; i < n16r; i += stride) {
    const u32x4 v = __builtin_nontemporal_load(src + i);
    x ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  for (int64_t i = i0; i < n16w; i += stride) dst[i] = u32x4{x, (uint32_t)i, 1u, 2u};
}

__global__ void kEmpty(uint32_t* out) {
  if (threadIdx.x == 1023) out[0] = 1;
}

int main() {
  const size_t cap = (size_t)64 << 20;   // rotate writes over 64 MiB x 8 = beyond the MALL
  constexpr int NBUF = 8;
  unsigned char* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, cap * NBUF));
  CK(hipMalloc(&out, 64));
  CK(hipMemset(buf, 1, cap * NBUF));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  using L = std::function<void(int)>;
  auto time_graph = [&](const L& f) {
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < REPS; ++r) f(r);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return best * 1000.0 / REPS;
  };
  bool first = true;
  auto run = [&](const char* name, const L& f) {
    printf("%s\"%s\": %.3f", first ? "{" : ", ", name, time_graph(f));
    first = false;
    fflush(stdout);
  };
  const int grid = 1024;
  auto at = [&](int r) { return buf + (size_t)(r % NBUF) * cap; };
  run("empty", [&](int) { kEmpty<<<1024, 256, 0, s>>>(out); });
  for (int mb : {2, 4, 8}) {
    const int64_t n16 = ((int64_t)mb << 20) / 16;
    char nm[64];
    snprintf(nm, sizeof nm, "rd%d", mb);
    run(nm, [&](int r) { kRead<<<grid, 256, 0, s>>>((const u32x4*)at(r), n16, out); });
    snprintf(nm, sizeof nm, "wr%d-default", mb);
    run(nm, [&](int r) { kWrite<0><<<grid, 256, 0, s>>>((u32x4*)at(r), n16, r); });
    snprintf(nm, sizeof nm, "wr%d-nt", mb);
    run(nm, [&](int r) { kWrite<1><<<grid, 256, 0, s>>>((u32x4*)at(r), n16, r); });
    snprintf(nm, sizeof nm, "wr%d-sc0sc1", mb);
    run(nm, [&](int r) { kWrite<2><<<grid, 256, 0, s>>>((u32x4*)at(r), n16, r); });
    snprintf(nm, sizeof nm, "wr%d-ntsc", mb);
    run(nm, [&](int r) { kWrite<3><<<grid, 256, 0, s>>>((u32x4*)at(r), n16, r); });
    snprintf(nm, sizeof nm, "rw2_%d", mb);
    run(nm, [&](int r) {
      kReadWrite<<<grid, 256, 0, s>>>((const u32x4*)at(r + 1), ((int64_t)2 << 20) / 16, (u32x4*)at(r), n16);
    });
    snprintf(nm, sizeof nm, "wr%d-default-g256", mb);
    run(nm, [&](int r) { kWrite<0><<<256, 256, 0, s>>>((u32x4*)at(r), n16, r); });
    snprintf(nm, sizeof nm, "wr%d-default-g4096", mb);
    run(nm, [&](int r) { kWrite<0><<<4096, 256, 0, s>>>((u32x4*)at(r), n16, r); });
  }
  printf("}\n");
  return 0;
}
