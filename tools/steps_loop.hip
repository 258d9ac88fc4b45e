// steps_loop.hip -- a C caller of the plug-in API for bench.py and the measurement tools: K
// lamm_hip_matmul calls issued from C (what a C host such as llama.cpp does per token), without
// Python/ctypes submission (~5-20 us per call) in the way.
//   lamm_steps_matmul        : back to back (host-bound at the library's ~4 us per call)
//   lamm_steps_matmul_paced  : launches paced slower than the kernel, so a kernel tracer times
//                              every dispatch on its own (no dispatch queued behind it to fold the
//                              tracer's per-dispatch cost into)
//   lamm_steps_isolated[_ex] : per-launch durations from the dispatches' own timestamps
//                              (lamm_hip_profile_next), launches isolated or back to back --
//                              what the kernel tracer reports for the same dispatch (bench.py's
//                              roofline)
//   lamm_steps_direct        : K calls inside one direct-dispatch region (lamm_hip_direct_begin /
//                              end: the library's own AQL queue), completed before it returns
//   lamm_steps_graph         : the K calls captured from C as one hipGraph (instantiated, uploaded),
//                              replayed; wall time of launch -> synchronize per replay
//   lamm_read_floor          : the single-launch floor of config 2: a read-only
//                              kernel on the GEMV's grid (512 workgroups of 512 threads, 36 bytes per
//                              thread as the GEMV's two 18-byte blocks per lane) over the same bytes,
//                              timed per isolated launch like lamm_steps_isolated
// hipcc --offload-arch=gfx950 -O2 -shared -fPIC -I include tools/steps_loop.hip -L la-llama.cpp_amd -llamm_hip
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <chrono>
#include <vector>

#include "lamm_hip.h"

namespace {

// 512 threads x 36 B per workgroup, coalesced: b128 at [t], b128 at [512 + t], b32 at 16 KiB + 4 t
constexpr uint32_t kFloorWgBytes = 512 * 36;
__global__ __launch_bounds__(512) void read_floor_kernel(const unsigned char* A, uint32_t bytes, uint32_t* sink) {
  const uint32_t base = blockIdx.x * kFloorWgBytes, t = threadIdx.x;
  const uint32_t o0 = base + 16 * t, o1 = base + 8192 + 16 * t, o2 = base + 16384 + 4 * t;
  uint32_t x = 0;
  if (o0 + 16 <= bytes) {
    const uint4 v = *reinterpret_cast<const uint4*>(A + o0);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (o1 + 16 <= bytes) {
    const uint4 v = *reinterpret_cast<const uint4*>(A + o1);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (o2 + 4 <= bytes) x ^= *reinterpret_cast<const uint32_t*>(A + o2);
  if (x == 0x9e3779b9u) sink[blockIdx.x] = x;   // (never in practice: keeps the loads)
}

__global__ __launch_bounds__(512) void empty_floor_kernel(uint32_t*) {}

double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
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

// out_us[i] = the dispatch's own duration (start / end timestamps of the kernel dispatch,
// lamm_hip_profile_next -> hipExtLaunchKernel: what a kernel tracer reports) of launch i.
// sync_each: each launch alone (completed before the next is issued); otherwise back to back.
int lamm_steps_isolated_ex(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first,
                           int launches, void* stream, float* out_us, int sync_each, int flags) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  std::vector<hipEvent_t> e0(launches), e1(launches);
  int rc = LAMM_OK;
  for (int i = 0; i < launches; ++i) {
    (void)hipEventCreate(&e0[i]);
    (void)hipEventCreate(&e1[i]);
  }
  for (int i = 0; i < launches && rc == LAMM_OK; ++i) {
    (void)lamm_hip_profile_next(e0[i], e1[i]);
    rc = lamm_hip_matmul_ex(&A[(first + i) % nA], B, C, nullptr, flags, stream);
    if (sync_each && hipEventSynchronize(e1[i]) != hipSuccess) rc = -2;
  }
  if (hipStreamSynchronize(s) != hipSuccess && rc == LAMM_OK) rc = -2;
  for (int i = 0; i < launches; ++i) {
    float ms = 0.f;
    if (rc == LAMM_OK && hipEventElapsedTime(&ms, e0[i], e1[i]) != hipSuccess) rc = -2;
    out_us[i] = ms * 1e3f;
    (void)hipEventDestroy(e0[i]);
    (void)hipEventDestroy(e1[i]);
  }
  return rc;
}

// the same with flags = 0 (lamm_hip_matmul)
int lamm_steps_isolated(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first,
                        int launches, void* stream, float* out_us, int sync_each) {
  return lamm_steps_isolated_ex(A, nA, B, C, first, launches, stream, out_us, sync_each, 0);
}

// K calls in one direct region on `device`: returns the number of direct dispatches (K when every
// call's kernel went onto the library's queue), or a negative status; *wall_us = the region's
// host wall time, from before the first call to the end of the wait for the last kernel
int lamm_steps_direct(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first, int steps,
                      int device, int flags, double* wall_us) {
  const double t0 = now_us();
  if (lamm_hip_direct_begin(device) != LAMM_OK) return -1;
  int rc = LAMM_OK;
  for (int s = 0; s < steps && rc == LAMM_OK; ++s) rc = lamm_hip_matmul_ex(&A[(first + s) % nA], B, C, nullptr, flags, nullptr);
  const int n = lamm_hip_direct_end();
  if (wall_us) *wall_us = now_us() - t0;
  return rc != LAMM_OK ? -100 - rc : n;
}

// K = steps calls A[(first + s) % nA] * B -> C captured on a fresh stream as one hipGraph, instantiated and
// uploaded; one untimed replay, then `reps` replays each timed on the host from hipGraphLaunch to the
// end of hipStreamSynchronize (out_us[r]).  Returns LAMM_OK or a negative status.
int lamm_steps_graph(const lamm_matrix* A, int nA, const lamm_matrix* B, const lamm_matrix* C, int first, int steps,
                     int reps, float* out_us) {
  hipStream_t s;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return -2;
  int rc = LAMM_OK;
  // warm: every kernel of the steps launched once, outside the capture
  for (int i = 0; i < steps && rc == LAMM_OK; ++i) rc = lamm_hip_matmul(&A[(first + i) % nA], B, C, s);
  if (rc != LAMM_OK || hipStreamSynchronize(s) != hipSuccess) {
    (void)hipStreamDestroy(s);
    return rc != LAMM_OK ? rc : -2;
  }
  hipGraph_t g = nullptr;
  hipGraphExec_t ge = nullptr;
  if (hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal) != hipSuccess) rc = -3;
  for (int i = 0; i < steps && rc == LAMM_OK; ++i) rc = lamm_hip_matmul(&A[(first + i) % nA], B, C, s);
  if (hipStreamEndCapture(s, &g) != hipSuccess && rc == LAMM_OK) rc = -4;
  if (rc == LAMM_OK && hipGraphInstantiate(&ge, g, nullptr, nullptr, 0) != hipSuccess) rc = -5;
  if (rc == LAMM_OK && hipGraphUpload(ge, s) != hipSuccess) rc = -6;
  if (rc == LAMM_OK && (hipGraphLaunch(ge, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess)) rc = -7;
  for (int r = 0; r < reps && rc == LAMM_OK; ++r) {
    const double t0 = now_us();
    if (hipGraphLaunch(ge, s) != hipSuccess || hipStreamSynchronize(s) != hipSuccess) rc = -8;
    out_us[r] = (float)(now_us() - t0);
  }
  if (ge) (void)hipGraphExecDestroy(ge);
  if (g) (void)hipGraphDestroy(g);
  (void)hipStreamDestroy(s);
  return rc;
}

// out_us[i] = the dispatch's own duration of an EMPTY kernel on `grid` workgroups of 512 threads, each
// launch completed before the next: what the timestamps report for a dispatch that does nothing
int lamm_empty_floor(int grid, int launches, void* stream, float* out_us) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = LAMM_OK;
  for (int i = 0; i < launches && rc == LAMM_OK; ++i) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipExtLaunchKernelGGL(empty_floor_kernel, dim3(grid), dim3(512), 0, s, e0, e1, 0, nullptr);
    float ms = 0.f;
    if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
      rc = -2;
    out_us[i] = ms * 1e3f;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  return rc;
}

// out_us[i] = the dispatch's own duration of read_floor_kernel over [A + ((first + i) % nA) * stride,
// + bytes), each launch completed before the next (as lamm_steps_isolated with sync_each)
int lamm_read_floor(const unsigned char* A, size_t stride, int nA, size_t bytes, int first, int launches, void* stream,
                    float* out_us) {
  const hipStream_t s = static_cast<hipStream_t>(stream);
  uint32_t* sink = nullptr;
  const unsigned grid = (unsigned)((bytes + kFloorWgBytes - 1) / kFloorWgBytes);
  if (bytes >= (1ull << 32) || hipMalloc(&sink, grid * sizeof(uint32_t)) != hipSuccess) return -2;
  int rc = LAMM_OK;
  for (int i = 0; i < launches && rc == LAMM_OK; ++i) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    hipExtLaunchKernelGGL(read_floor_kernel, dim3(grid), dim3(512), 0, s, e0, e1, 0,
                          A + (size_t)((first + i) % nA) * stride, (uint32_t)bytes, sink);
    float ms = 0.f;
    if (hipGetLastError() != hipSuccess || hipEventSynchronize(e1) != hipSuccess ||
        hipEventElapsedTime(&ms, e0, e1) != hipSuccess)
      rc = -2;
    out_us[i] = ms * 1e3f;
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
  }
  (void)hipFree(sink);
  return rc;
}

}  // extern "C"
