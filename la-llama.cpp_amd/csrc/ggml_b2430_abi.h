// ggml_b2430_abi.h -- the two ggml structs the lamm boundary reads, at the exact
// llama.cpp-b2430 binary layout (LC/ggml.h:552-590 ggml_tensor, :668-677
// ggml_compute_params), so liblamm_hip.so can be linked into an unchanged b2430
// build without compiling against ggml's headers.  Offsets were checked against the
// real header with offsetof (tests/test_host_abi.py re-checks when the reference is
// present); the static_asserts pin them here.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace lamm {
namespace ggml {

enum : int32_t { TASK_INIT = 0, TASK_COMPUTE = 1, TASK_FINALIZE = 2 };
enum : int32_t { OP_MUL_MAT = 23 };
constexpr int kMaxDims = 4, kMaxSrc = 10, kMaxName = 64, kMaxOpParams = 64;

struct tensor {
  int32_t type;
  int32_t backend;
  void* buffer;
  int64_t ne[kMaxDims];
  size_t nb[kMaxDims];
  int32_t op;
  int32_t op_params[kMaxOpParams / 4];
  int32_t flags;
  tensor* grad;
  tensor* src[kMaxSrc];
  int32_t perf_runs;
  int64_t perf_cycles;
  int64_t perf_time_us;
  tensor* view_src;
  size_t view_offs;
  void* data;
  char name[kMaxName];
  void* extra;
  char padding[8];
};

struct compute_params {
  int32_t type;   // ggml_task_type
  int32_t ith, nth;
  size_t wsize;
  void* wdata;
};

static_assert(sizeof(tensor) == 368, "ggml_tensor size (b2430)");
static_assert(offsetof(tensor, ne) == 16 && offsetof(tensor, nb) == 48, "ne/nb");
static_assert(offsetof(tensor, op) == 80 && offsetof(tensor, src) == 160, "op/src");
static_assert(offsetof(tensor, data) == 280 && offsetof(tensor, name) == 288, "data/name");
static_assert(sizeof(compute_params) == 32 && offsetof(compute_params, wdata) == 24, "params");

}  // namespace ggml
}  // namespace lamm
