// bar_probe.hip -- where a decode call's activation row should live: the boundary hands over one F32
// row (16 KiB) per call, and every workgroup of the GEMV reads all of it.  Per strategy, median of
// 300 calls of [host writes the row; kernel: 512 workgroups read it and write 8 floats of C each to
// pinned host memory; signal kernel stores a flag into host-coherent memory; host spins on it]:
//   pinned : the row in coherent pinned host memory, read by the kernel over PCIe
//   pinned_nc : the same in non-coherent pinned memory (cached in the device's L2; the boundary's form)
//   vram   : the row in fine-grained device memory the host writes through the BAR (+ HDP flush)
// plus each kernel's own duration by HIP events (row already written).
// Usage: bar_probe [kib=16]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

__global__ __launch_bounds__(256) void read_row(const float* __restrict__ x, int n, float* __restrict__ c) {
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) s += x[i];
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (threadIdx.x < 8) {
    float v = 0.f;
    for (int k = threadIdx.x; k < 256; k += 8) v += red[k];
    c[blockIdx.x * 8 + threadIdx.x] = v;
  }
}

__global__ void signal(volatile unsigned* flag, unsigned seq) {
  if (threadIdx.x == 0) __hip_atomic_store(flag, seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const int kib = argc > 1 ? atoi(argv[1]) : 16;
  const int n = kib * 256;
  const int grid = 512;
  std::vector<float> src(n);
  for (int i = 0; i < n; ++i) src[i] = (float)(i % 7);
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float *h_row, *d_row_h, *h_c, *d_c_h, *v_row, *nc_row, *d_nc_row;
  CK(hipHostMalloc(&h_row, n * 4, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&d_row_h, h_row, 0));
  CK(hipHostMalloc(&nc_row, n * 4, hipHostMallocMapped | hipHostMallocNonCoherent));
  CK(hipHostGetDevicePointer((void**)&d_nc_row, nc_row, 0));
  CK(hipHostMalloc(&h_c, grid * 8 * 4, hipHostMallocMapped));
  CK(hipHostGetDevicePointer((void**)&d_c_h, h_c, 0));
  unsigned *h_flag, *d_flag;
  CK(hipHostMalloc(&h_flag, 64, hipHostMallocMapped | hipHostMallocCoherent));
  CK(hipHostGetDevicePointer((void**)&d_flag, h_flag, 0));
  *h_flag = 0;
  CK(hipExtMallocWithFlags((void**)&v_row, n * 4, hipDeviceMallocFinegrained));
  printf("{\"kib\": %d", kib);
  fflush(stdout);
  // can the host write the fine-grained VRAM row? (a fault here ends the probe: no BAR mapping)
  memcpy(v_row, src.data(), n * 4);
  float chk = v_row[n - 1];
  printf(", \"vram_host_write\": %s", chk == src[n - 1] ? "true" : "false");
  fflush(stdout);
  unsigned seq = 0;
  for (int mode = 0; mode < 3; ++mode) {
    float* dst_host = mode == 0 ? h_row : mode == 1 ? v_row : nc_row;
    const float* row_dev = mode == 0 ? d_row_h : mode == 1 ? v_row : d_nc_row;
    std::vector<double> call, write;
    for (int it = 0; it < 330; ++it) {
      const double t0 = now_us();
      memcpy(dst_host, src.data(), n * 4);
      if (mode == 1) std::atomic_thread_fence(std::memory_order_seq_cst);
      const double t1 = now_us();
      hipLaunchKernelGGL(read_row, dim3(grid), dim3(256), 0, s, row_dev, n, d_c_h);
      hipLaunchKernelGGL(signal, dim3(1), dim3(64), 0, s, d_flag, ++seq);
      while (__atomic_load_n(h_flag, __ATOMIC_ACQUIRE) != seq) {
      }
      const double t2 = now_us();
      if (it >= 30) {
        call.push_back(t2 - t0);
        write.push_back(t1 - t0);
      }
    }
    std::sort(call.begin(), call.end());
    std::sort(write.begin(), write.end());
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    std::vector<double> kern;
    for (int it = 0; it < 100; ++it) {
      CK(hipEventRecord(e0, s));
      hipLaunchKernelGGL(read_row, dim3(grid), dim3(256), 0, s, row_dev, n, d_c_h);
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      kern.push_back(ms * 1e3);
    }
    std::sort(kern.begin(), kern.end());
    printf(", \"%s\": {\"call_us\": %.2f, \"host_write_us\": %.2f, \"kernel_us\": %.2f}",
           mode == 0 ? "pinned" : mode == 1 ? "vram" : "pinned_nc",
           call[call.size() / 2], write[write.size() / 2], kern[kern.size() / 2]);
    fflush(stdout);
  }
  printf("}\n");
  return 0;
}
