// steps_loop.hip -- a C caller of the plug-in API for bench.py and the measurement tools: K
// lamm_hip_matmul calls issued from C (what a C host such as llama.cpp does per token), without
// Python/ctypes submission (~5-20 us per call) in the way.
//   lamm_steps_matmul        : back to back (host-bound at the library's ~4 us per call)
//   lamm_steps_matmul_paced  : launches paced slower than the kernel, so a kernel tracer times
//                              every dispatch on its own (no dispatch queued behind it to fold the
//                              tracer's per-dispatch cost into)
//   lamm_steps_isolated      : per-launch durations by HIP events, each launch isolated: behind a
//                              gate kernel that holds the stream until the host has enqueued the
//                              events and the launch, so e1 - e0 is the device's own time for one
//                              dispatch with nothing queued behind it -- what the kernel tracer
//                              reports for the same dispatch (bench.py's roofline)
// hipcc --offload-arch=gfx950 -O2 -shared -fPIC -I include tools/steps_loop.hip -L la-llama.cpp_amd -llamm_hip
#include <hip/hip_runtime.h>

#include <chrono>
#include <vector>

#include "lamm_hip.h"

namespace {

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

// one wave: wait until *flag >= want (host-coherent memory) or ~0.2 s have passed (s_memrealtime,
// 100 MHz), whichever comes first -- every launch of it ends
__global__ void gate_kernel(const unsigned* flag, unsigned want) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__hip_atomic_load(flag, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) < want) {
    if (__builtin_amdgcn_s_memrealtime() - t0 > 20000000ull) break;
    __builtin_amdgcn_s_sleep(8);
  }
}

}  // namespace

extern "C" {

// step s multiplies A[(first + s) % nA] by B into C; returns the first non-OK status
int lamm_steps_matmul(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first, int steps,
                      void* stream) {
  for (int s = 0; s < steps; ++s) {
    const int rc = lamm_hip_matmul(&A[(first + s) % nA], B, C, stream);
    if (rc != LAMM_OK) return rc;
  }
  return LAMM_OK;
}

// sync_each: wait for every launch to complete, then idle gap_us (the device idles >= one
// synchronize round trip); otherwise spin gap_us after each launch call, so the launches come at
// the host's own pace plus the gap -- slower than the kernel, so none queues behind another
int lamm_steps_matmul_paced(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first,
                            int steps, void* stream, double gap_us, int sync_each) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  for (int i = 0; i < steps; ++i) {
    const int rc = lamm_hip_matmul(&A[(first + i) % nA], B, C, stream);
    if (rc != LAMM_OK) return rc;
    if (sync_each && hipStreamSynchronize(s) != hipSuccess) return -2;
    const double t0 = now_us();
    while (now_us() - t0 < gap_us) {
    }
  }
  return hipStreamSynchronize(s) == hipSuccess ? LAMM_OK : -2;
}

// out_us[i] = device time of launch i alone (events around it, the stream held by a gate kernel
// until the host has enqueued both events and the launch)
int lamm_steps_isolated(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first,
                        int launches, void* stream, float* out_us) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  unsigned* flag = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&flag), sizeof(unsigned), hipHostMallocCoherent) != hipSuccess) return -3;
  __atomic_store_n(flag, 0u, __ATOMIC_RELEASE);
  std::vector<hipEvent_t> e0(launches), e1(launches);
  int rc = LAMM_OK;
  for (int i = 0; i < launches; ++i) {
    (void)hipEventCreate(&e0[i]);
    (void)hipEventCreate(&e1[i]);
  }
  for (int i = 0; i < launches && rc == LAMM_OK; ++i) {
    hipLaunchKernelGGL(gate_kernel, dim3(1), dim3(64), 0, s, flag, (unsigned)(i + 1));
    (void)hipEventRecord(e0[i], s);
    rc = lamm_hip_matmul(&A[(first + i) % nA], B, C, stream);
    (void)hipEventRecord(e1[i], s);
    __atomic_store_n(flag, (unsigned)(i + 1), __ATOMIC_RELEASE);   // open the gate
    if (hipEventSynchronize(e1[i]) != hipSuccess) rc = -2;
  }
  __atomic_store_n(flag, 0xffffffffu, __ATOMIC_RELEASE);
  if (hipStreamSynchronize(s) != hipSuccess && rc == LAMM_OK) rc = -2;
  for (int i = 0; i < launches; ++i) {
    float ms = 0.f;
    if (rc == LAMM_OK && hipEventElapsedTime(&ms, e0[i], e1[i]) != hipSuccess) rc = -2;
    out_us[i] = ms * 1e3f;
    (void)hipEventDestroy(e0[i]);
    (void)hipEventDestroy(e1[i]);
  }
  (void)hipHostFree(flag);
  return rc;
}

}  // extern "C"
