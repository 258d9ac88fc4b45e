// lamm_signal.hip -- completion flag for the ggml boundary's synchronous calls.
//
// lamm_mul_mat must return with dst filled, i.e. wait for its kernels.  hipStreamSynchronize
// after a launch costs ~10 us on MI355X even for an empty kernel; a one-lane kernel enqueued
// behind the work that stores a sequence number into pinned, host-coherent memory lets the host
// see completion by spinning on that word instead: 6 us launch-to-flag (tools/lat_probe.hip,
// profiles/r02/lat_probe.txt).  The store is a plain vector store after a system-scope release,
// so everything the stream's earlier kernels wrote (C in pinned host memory included) is
// visible to the host once the flag is.
#include <hip/hip_runtime.h>

#include "lamm_kernels.h"

namespace lamm {
namespace {

__global__ void signal_kernel(volatile unsigned* flag, unsigned seq) {
  if (threadIdx.x == 0) {
    __threadfence_system();
    *flag = seq;
    __threadfence_system();
  }
}

}  // namespace

hipError_t launch_signal(unsigned* flag_dev, unsigned seq, hipStream_t s) {
  hipLaunchKernelGGL(signal_kernel, dim3(1), dim3(64), 0, s, flag_dev, seq);
  return hipGetLastError();
}

}  // namespace lamm
