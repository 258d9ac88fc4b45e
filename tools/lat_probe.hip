// lat_probe.hip -- host<->device round-trip latencies that bound one ggml-boundary call
// (lamm_mul_mat: activations up, one kernel, C down, stream synchronised).  Each line is the
// median of 2000 repetitions of: <operation(s)> on one stream + hipStreamSynchronize.
//   hipcc --offload-arch=gfx950 -O2 tools/lat_probe.hip -o tools/lat_probe && tools/lat_probe [spin|yield|block]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                                   \
  do {                                                                          \
    hipError_t e = (x);                                                         \
    if (e != hipSuccess) {                                                      \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                    \
      exit(1);                                                                  \
    }                                                                           \
  } while (0)

__global__ void empty_kernel() {}

// one lane stores `seq` to a host-mapped flag (system-scope release); the host spins on it
__global__ void flag_kernel(volatile unsigned* flag, unsigned seq) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    __threadfence_system();
    *flag = seq;
    __threadfence_system();
  }
}

// one workgroup per 4 KiB: write n floats (C) with plain vector stores
__global__ void write_kernel(float* __restrict__ c, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) c[i] = (float)i;
}

// read n floats from src (host or device) once, write them to dst
__global__ void copy_kernel(const float4* __restrict__ src, float4* __restrict__ dst, int n4) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n4) dst[i] = src[i];
}

template <class F>
double median_us(F&& f, hipStream_t s, int reps = 2000) {
  std::vector<double> t(reps);
  for (int w = 0; w < 50; ++w) { f(); CK(hipStreamSynchronize(s)); }
  for (int r = 0; r < reps; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    CK(hipStreamSynchronize(s));
    t[r] = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
  }
  std::sort(t.begin(), t.end());
  return t[reps / 2];
}

int main(int argc, char** argv) {
  const char* mode = argc > 1 ? argv[1] : "auto";
  if (!strcmp(mode, "spin")) CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
  if (!strcmp(mode, "yield")) CK(hipSetDeviceFlags(hipDeviceScheduleYield));
  if (!strcmp(mode, "block")) CK(hipSetDeviceFlags(hipDeviceScheduleBlockingSync));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const int n = 4096;                       // one decode C / F32 activation row (16 KiB)
  const size_t bytes = n * sizeof(float);
  float *d0, *d1, *hp, *hc, *hcd;
  std::vector<float> pageable(n);
  CK(hipMalloc(&d0, bytes));
  CK(hipMalloc(&d1, bytes));
  CK(hipHostMalloc(&hp, bytes, hipHostMallocDefault));
  CK(hipHostMalloc(&hc, bytes, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&hcd, hc, 0));
  printf("{\"mode\": \"%s\"", mode);
  printf(", \"empty_kernel\": %.2f", median_us([&] { empty_kernel<<<1, 64, 0, s>>>(); }, s));
  printf(", \"empty_kernel_256wg\": %.2f", median_us([&] { empty_kernel<<<256, 256, 0, s>>>(); }, s));
  printf(", \"h2d_16k_pinned\": %.2f", median_us([&] { CK(hipMemcpyAsync(d0, hp, bytes, hipMemcpyHostToDevice, s)); }, s));
  printf(", \"h2d_4k_pinned\": %.2f", median_us([&] { CK(hipMemcpyAsync(d0, hp, 4352, hipMemcpyHostToDevice, s)); }, s));
  printf(", \"h2d_16k_pageable\": %.2f",
         median_us([&] { CK(hipMemcpyAsync(d0, pageable.data(), bytes, hipMemcpyHostToDevice, s)); }, s));
  printf(", \"d2h_16k_pinned\": %.2f", median_us([&] { CK(hipMemcpyAsync(hp, d0, bytes, hipMemcpyDeviceToHost, s)); }, s));
  printf(", \"d2h_16k_pageable\": %.2f",
         median_us([&] { CK(hipMemcpyAsync(pageable.data(), d0, bytes, hipMemcpyDeviceToHost, s)); }, s));
  printf(", \"kernel_write_16k_to_host\": %.2f", median_us([&] { write_kernel<<<n / 256, 256, 0, s>>>(hcd, n); }, s));
  printf(", \"kernel_copy_16k_from_host\": %.2f",
         median_us([&] { copy_kernel<<<n / 4 / 256, 256, 0, s>>>((const float4*)hcd, (float4*)d1, n / 4); }, s));
  printf(", \"h2d_then_kernel_then_d2h\": %.2f", median_us([&] {
           CK(hipMemcpyAsync(d0, hp, bytes, hipMemcpyHostToDevice, s));
           empty_kernel<<<256, 256, 0, s>>>();
           CK(hipMemcpyAsync(hp, d0, bytes, hipMemcpyDeviceToHost, s));
         }, s));
  printf(", \"copyk_then_kernel_write_host\": %.2f", median_us([&] {
           copy_kernel<<<n / 4 / 256, 256, 0, s>>>((const float4*)hcd, (float4*)d1, n / 4);
           write_kernel<<<n / 256, 256, 0, s>>>(hcd, n);
         }, s));
  unsigned* hflag;
  unsigned* dflag;
  CK(hipHostMalloc((void**)&hflag, 64, hipHostMallocCoherent | hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&dflag, hflag, 0));
  *hflag = 0;
  unsigned seq = 0;
  {   // launch -> host sees the kernel's flag (no stream synchronisation in the timed path)
    std::vector<double> t(2000);
    for (int r = -50; r < 2000; ++r) {
      ++seq;
      const auto t0 = std::chrono::steady_clock::now();
      flag_kernel<<<1, 64, 0, s>>>(dflag, seq);
      while (*(volatile unsigned*)hflag != seq) {
      }
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 0) t[r] = us;
      CK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    printf(", \"flag_kernel_spin\": %.2f", t[1000]);
  }
  printf(", \"flag_kernel_sync\": %.2f", median_us([&] { flag_kernel<<<1, 64, 0, s>>>(dflag, ++seq); }, s));
  // the same completion signal written by the command processor (hipStreamWriteValue32), no kernel
  {
    std::vector<double> t(2000);
    for (int r = -50; r < 2000; ++r) {
      ++seq;
      const auto t0 = std::chrono::steady_clock::now();
      CK(hipStreamWriteValue32(s, dflag, seq, 0));
      while (*(volatile unsigned*)hflag != seq) {
      }
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 0) t[r] = us;
      CK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    printf(", \"write_value_spin\": %.2f", t[1000]);
  }
  // a 256-workgroup kernel then the completion signal: signal kernel vs stream write-value
  for (int mode = 0; mode < 2; ++mode) {
    std::vector<double> t(2000);
    for (int r = -50; r < 2000; ++r) {
      ++seq;
      const auto t0 = std::chrono::steady_clock::now();
      write_kernel<<<n / 256, 256, 0, s>>>(d0, n);
      if (mode == 0) flag_kernel<<<1, 64, 0, s>>>(dflag, seq);
      else CK(hipStreamWriteValue32(s, dflag, seq, 0));
      while (*(volatile unsigned*)hflag != seq) {
      }
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
      if (r >= 0) t[r] = us;
      CK(hipStreamSynchronize(s));
    }
    std::sort(t.begin(), t.end());
    printf(mode == 0 ? ", \"kernel_then_flag_kernel_spin\": %.2f" : ", \"kernel_then_write_value_spin\": %.2f", t[1000]);
  }
  printf("}\n");
  return 0;
}
