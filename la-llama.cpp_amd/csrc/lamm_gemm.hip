// lamm_gemm.hip -- prefill-shaped (N > 8) MFMA-i8 GEMM (placeholder until implemented).
#include "lamm_device.h"
#include "lamm_kernels.h"

namespace lamm {
bool gemm_supported(int) { return false; }
hipError_t launch_gemm(int, const GemvArgs&, hipStream_t) { return hipErrorInvalidValue; }
}  // namespace lamm
