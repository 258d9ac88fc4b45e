// lamm_hip.cpp -- host side of liblamm_hip.so: the C ABI of include/lamm_hip.h.
//
//   * lamm_hip_matmul  : the operator API on device memory (mirrors
//                        LAMMImpl<T>::matmul, src/lamm_impl.hpp:20-29) -> kernel dispatch
//   * lamm_can_mul_mat / lamm_mul_mat / lamm_get_opt_level : the ggml boundary
//                        (src/loongarch_matmul.cpp:10-145) on top of it, with a
//                        device-resident weight cache and strided B/C transfers.
#include <hip/hip_runtime.h>

#include <linux/futex.h>
#include <sched.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <list>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/lamm_hip.h"
#include "ggml_b2430_abi.h"
#include "lamm_aql.h"
#include "lamm_formats.h"
#include "lamm_kernels.h"
#include "lamm_knobs.h"

namespace lamm {
hipError_t launch_quantize(int vec_type, int flavour, const float* x, int64_t ldx, void* y,
                           int64_t ldy_bytes, int K, int N, hipStream_t s);
}

using namespace lamm;

namespace {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}

}  // namespace

namespace {

struct DeviceProbe {
  int count = 0;          // gfx950 devices visible
  int device = 0;         // the first of them (the ggml boundary's default device)
  std::vector<int> ids;   // every gfx950 device
};

const DeviceProbe& probe() {
  static DeviceProbe p = [] {
    DeviceProbe d;
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) { (void)hipGetLastError(); return d; }
    for (int i = 0; i < n; ++i) {
      hipDeviceProp_t prop;
      if (hipGetDeviceProperties(&prop, i) == hipSuccess && strncmp(prop.gcnArchName, "gfx950", 6) == 0) {
        if (d.count == 0) d.device = i;
        ++d.count;
        d.ids.push_back(i);
      }
    }
    return d;
  }();
  return p;
}

// Device scratch of the GEMM engines (packed activations, split-K partials): grow-only, one
// per (device, stream), so calls on different streams never share one (work on ONE stream is
// ordered by the stream itself).  Growing synchronises that stream before the old buffer is
// released.
struct WsKey {
  int dev;
  hipStream_t stream;
  bool operator==(const WsKey& o) const { return dev == o.dev && stream == o.stream; }
};
struct WsKeyHash {
  size_t operator()(const WsKey& k) const { return std::hash<const void*>()(k.stream) ^ (size_t)k.dev * 0x9e3779b9u; }
};
struct WsBuf {
  void* ptr = nullptr;
  size_t bytes = 0;
};
std::mutex g_ws_mu;
std::unordered_map<WsKey, WsBuf, WsKeyHash> g_ws;

void* workspace(size_t bytes, hipStream_t s) {
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(g_ws_mu);
  WsBuf& b = g_ws[WsKey{dev, s}];
  if (b.ptr && b.bytes >= bytes) return b.ptr;
  if (b.ptr) {
    (void)hipStreamSynchronize(s);
    (void)hipFree(b.ptr);
    b = WsBuf{};
  }
  const size_t want = bytes + bytes / 4;
  if (hipMalloc(&b.ptr, want) != hipSuccess) { b = WsBuf{}; return nullptr; }
  b.bytes = want;
  return b.ptr;
}

// GEMM engine for the q4_0 / q4_1 / q5_0 prefill path: 0 = block-scaled fp6 MFMA
// (lamm_gemm_fp6.hip), 1 = MFMA-i8 (lamm_gemm.hip).  The fp6 kernel's 256x128 tiles only pay
// off once they fill the chip (>= one tile per CU); smaller calls take the i8 kernel's
// 128x64 tiles.  With weight-stationary callers (lamm_hip_weights: the packed weights are
// resident) the fp6 kernel's K-split fills the chip from 64 tiles up and wins there too
// (profiles/r01/ab_stationary.txt: one 4096x512x4096 slice 44.4 us at 4 splits vs 48.2 us
// on i8; two slices 65.1 vs 88.1); per call, re-packing the weights costs it that margin on
// a single slice (53.8 vs 47.9).  Both engines split K on small grids: la-benchmark-matmult's
// own shape K=11008, M=4096, N=128 (64 i8 tiles, 16 fp6 tiles) measures 231 TFLOP/s on i8 at 4
// splits (93 unsplit), 199 on fp6 re-packing per call at 16 splits, 286 with the packed weights
// resident (profiles/r01/ab_driver_split.txt).  LAMM_GEMM_PATH=fp6 / i8 forces one (A/B).
int gemm_path(const GemvArgs& p, bool stationary) {
  if (knobs().gemm_path >= 0) return knobs().gemm_path;
  return (stationary ? gemm_fp6_grid(p) : gemm_fp6_tiles(p)) >= 256 ? 0 : 1;
}

}  // namespace

void lamm::set_max_lds(const void* kernel, int bytes) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> done[64];   // per device: the largest size set
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lock(mu);
  int& have = done[dev & 63][kernel];
  if (have >= bytes) return;
  (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
  have = bytes;
}

// =============================================================== traits
extern "C" int lamm_blck_size(int type) { return block_bytes(type) ? block_elems(type) : 0; }
extern "C" size_t lamm_type_size(int type) { return block_bytes(type); }
extern "C" int lamm_vec_dot_type(int type) { return vec_dot_type(type); }
extern "C" const char* lamm_hip_last_error(void) { return g_err.c_str(); }
extern "C" int lamm_hip_device_count(void) { return probe().count; }
#ifndef LAMM_BUILD_ID
#define LAMM_BUILD_ID "unknown"
#endif
extern "C" const char* lamm_hip_build_id(void) { return LAMM_BUILD_ID; }

// ======================================================== operator API
struct lamm_weights {
  lamm_matrix A;
  int64_t ne02, ne03;
  size_t nba2, nba3;
  void* packed = nullptr;    // fp6 GEMM form of A (q4_0 / q4_1 / q5_0), null otherwise
  size_t packed_bytes = 0;
};

namespace {

GemvArgs weight_args(const lamm_matrix* A, int64_t ne02, int64_t ne03, size_t nba2, size_t nba3) {
  GemvArgs p{static_cast<const unsigned char*>(A->data), A->ld * (int64_t)block_bytes(A->type), nullptr, 0,
             nullptr, 0, A->row, 1, A->col * block_elems(A->type), A->col};
  p.ne12 = (int)ne02;
  p.ne13 = (int)ne03;
  p.sa2 = (int64_t)nba2;
  p.sa3 = (int64_t)nba3;
  return p;
}

// Widest activation count the GEMV kernels take; wider calls go to the prefill GEMM engines.
// The super-block formats' GEMV decodes a whole super-block per lane, and F16 rows carry no
// block scale to amortise, so their per-column cost grows faster than the matrix cores':
// measured crossovers (us per 4096 x 4096 slice, stationary weights, > MALL per launch,
// profiles/r01/gemv_vs_gemm_n.txt): q2_K GEMM from N = 6 (9.69 vs 8.83), q4_K from 7
// (11.56 vs 10.51), q5_K / q6_K / f16 from 5 (16.67 / 18.56 / 9.63 vs 10.72 / 10.19 / 7.59);
// the 32-block formats stay on the GEMV up to 8 (q4_0 N = 8: 4.74 vs 6.50).
// LAMM_GEMV_MAX_N=n overrides (A/B).
int gemv_max_n(int type) {
  int n = 8;
  if (knobs().gemv_max_n >= 0) n = knobs().gemv_max_n;
  else if (type == kQ2_K) n = 5;
  else if (type == kQ4_K) n = 6;
  else if (type == kQ5_K || type == kQ6_K || type == kF16) n = 4;
  return n < 1 ? 1 : (n > 8 ? 8 : n);
}

// Which engine lamm_hip_matmul* runs a call on (lamm_hip_engine reports the same choice to
// callers and tests).  stationary: the weights' packed prefill form is resident (lamm_weights);
// b_al4: B and its slice strides are 4-byte aligned (the super-block GEMM reads q8_K as dwords).
enum Engine { kEngGemv, kEngDense, kEngKq, kEngFp6, kEngI8, kEngGemvGroups, kEngDq };
// The dequantizing f16 GEMM (lamm_gemm_dq.hip) runs every 32-element format; by default it takes the
// q5_1 / q8_0 prefill calls whose 128 x 64 tiles fill at least half the chip (it has no K-split):
// there it beats the exact MFMA-i8 engine (config 4, 4096 x 512 x 4096: q5_1 37.7 vs 49.5 us, q8_0
// 39.6 vs 47.3 us, profiles/r04/dq16/), while for q4_0 / q4_1 / q5_0 the exact fp6 engine stays ahead
// (q4_0 28.5 vs 34.4 us).  q5_1 with prepared weights (lamm_weights) runs on the fp6 engine too
// (F6<kQ5_1>: its quants shifted into e2m3's range, the shift carried by the affine term), its
// per-call form stays here.  LAMM_GEMM_PATH=dq16 forces it for every format, fp6 / i8 force the
// exact engines.
constexpr int kDqMinTiles = 128;
bool use_dq(int type, const GemvArgs& p, bool stationary) {
  if (!gemm_dq_supported(type) || !gemm_dq_args_ok(p)) return false;
  if (knobs().gemm_path == 2) return true;
  // q8_0 with prepared weights on the K-group plan: the exact fp6 engine's two-plane form (round 6)
  const bool q8_fp6 = type == kQ8_0 && stationary && gemm_fp6_kv_plan(p);
  return knobs().gemm_path < 0 && ((type == kQ5_1 && !stationary) || (type == kQ8_0 && !q8_fp6)) &&
         gemm_dq_tiles(p) >= kDqMinTiles;
}
Engine pick_engine(int type, const GemvArgs& p, bool stationary, bool b_al4) {
  if (p.N <= gemv_max_n(type) || (p.b_f32 && p.N <= 8)) return kEngGemv;
  if (gemm_dense_supported(type) && knobs().dense_gemm && gemm_dense_args_ok(p)) return kEngDense;
  if (gemm_kq_supported(type) && knobs().kq_gemm && b_al4) return kEngKq;
  if (use_dq(type, p, stationary)) return kEngDq;
  if (gemm_fp6_supported(type) && (type != kQ5_1 || stationary) && gemm_path(p, stationary) == 0 &&
      (type != kQ8_0 || (stationary && gemm_fp6_kv_plan(p))))
    return kEngFp6;
  if (gemm_supported(type) && gemm_args_ok(type, p)) return kEngI8;
  return kEngGemvGroups;
}

// A completion signal the ggml boundary asks of the next matmul on this thread (decode calls):
// the row-per-wave GEMV writes it itself when it takes the call (signaled = true); otherwise the
// boundary launches the signal kernel after the call.
struct Completion {
  unsigned* ctr;
  unsigned* flag;
  unsigned seq;
  bool signaled;
};
thread_local Completion* g_completion = nullptr;
// lamm_hip_profile_next's events, for the next launch on this thread that records them
thread_local LaunchTiming g_timing;

int matmul_impl_(const lamm_matrix* A, const lamm_matrix* B, const lamm_matrix* C, const lamm_batch* batch,
                 void* hip_stream, const lamm_weights* W, int flags);

int matmul_impl(const lamm_matrix* A, const lamm_matrix* B, const lamm_matrix* C, const lamm_batch* batch,
                void* hip_stream, const lamm_weights* W, int flags = 0) {
  // a profiling request (lamm_hip_profile_next) holds for this call only: kernels launched with
  // hipExtLaunchKernel take it and record the dispatch's own start / end; for any other engine the
  // two events bracket the call's launches on the stream instead
  const LaunchTiming tm = g_timing;
  if (tm.start) (void)hipEventRecord(tm.start, static_cast<hipStream_t>(hip_stream));
  const int direct0 = lamm::direct_active() ? lamm::direct_launches() : -1;
  const int rc = matmul_impl_(A, B, C, batch, hip_stream, W, flags);
  if (direct0 >= 0 && rc == LAMM_OK && lamm::direct_launches() == direct0) {
    // a call in a direct region that launched through HIP: say which one and why it could
    char why[160];
    snprintf(why, sizeof why, "A type %d, %d x %d x %d%s%s: its kernel is not one the queue takes", A->type, A->row,
             B->col, A->col, tm.start ? ", with a profiling request pending" : "", flags ? ", flags set" : "");
    lamm::direct_note(why);
  }
  if (g_timing.start) (void)hipEventRecord(tm.stop, static_cast<hipStream_t>(hip_stream));
  g_timing = LaunchTiming{};
  return rc;
}

int matmul_impl_(const lamm_matrix* A, const lamm_matrix* B, const lamm_matrix* C, const lamm_batch* batch,
                 void* hip_stream, const lamm_weights* W, int flags) {
  Completion* done = g_completion;
  g_completion = nullptr;
  if (!A || !B || !C) return fail(LAMM_ERR_SHAPE, "null matrix");
  if (!is_weight_type(A->type)) return fail(LAMM_ERR_TYPE, "unsupported A type %d", A->type);
  // F32 activations for a q8_0 / q8_1 weight type: ggml's INIT quantization (AVX2 flavour) runs
  // on the device inside the kernels that read B, bit-exact with lamm_hip_quantize(.., 1, ..) +
  // matmul -- the GEMV's staging (N <= 8), the fp6 / i8 GEMMs' activation prep (N > 8)
  const int vdt = vec_dot_type(A->type);
  const bool b_f32 = B->type == kF32 && (vdt == kQ8_0 || vdt == kQ8_1);
  if (B->type != vdt && !b_f32)
    return fail(LAMM_ERR_TYPE, "B type %d is not vec_dot_type(%d)=%d", B->type, A->type, vdt);
  if (C->type != kF32) return fail(LAMM_ERR_TYPE, "C must be f32");
  const int M = A->row, N = B->col, Kb = A->col;
  const int brows = b_f32 ? Kb * block_elems(A->type) : Kb;   // B.row: K in blocks of B's own type
  if (M < 0 || N < 0 || Kb < 0 || B->row != brows || C->row != M || C->col != N)
    return fail(LAMM_ERR_SHAPE, "shape mismatch A(%d,%d) B(%d,%d) C(%d,%d)", A->row, A->col, B->row, B->col,
                C->row, C->col);
  if (A->ld < Kb || (N > 1 && B->ld < brows) || (N > 1 && C->ld < M))
    return fail(LAMM_ERR_SHAPE, "leading dimension too small");
  lamm_batch bt{1, 1, 1, 1, 0, 0, 0, 0, 0, 0};
  if (batch) bt = *batch;
  if (bt.ne02 < 1 || bt.ne03 < 1 || bt.ne12 < 1 || bt.ne13 < 1 || bt.ne12 % bt.ne02 || bt.ne13 % bt.ne03)
    return fail(LAMM_ERR_SHAPE, "batch dims must be >= 1 and ne12 %% ne02 == ne13 %% ne03 == 0");
  if (bt.ne12 * bt.ne13 > 65535) return fail(LAMM_ERR_SHAPE, "too many batch slices");
  if (M == 0 || N == 0) return LAMM_OK;
  const size_t abpb = block_bytes(A->type), bbpb = block_bytes(B->type);
  const int64_t lda = A->ld * (int64_t)abpb, ldb = B->ld * (int64_t)bbpb;
  if (((uintptr_t)A->data & 15) || (lda & 15) || (bt.nba2 & 15) || (bt.nba3 & 15))
    return fail(LAMM_ERR_ALIGN, "A must be 16-byte aligned with 16-byte row/slice pitches (pitch %lld)",
                (long long)lda);
  if ((bt.nbc2 & 3) || (bt.nbc3 & 3) || ((uintptr_t)C->data & 3)) return fail(LAMM_ERR_ALIGN, "C must be f32-aligned");
  if (B->type == kQ8_K && (((uintptr_t)B->data & 3) || (ldb & 3) || (bt.nbb2 & 3) || (bt.nbb3 & 3)))
    return fail(LAMM_ERR_ALIGN, "q8_K B must be 4-byte aligned");
  if (B->type == kF32 && (((uintptr_t)B->data & 3) || (bt.nbb2 & 3) || (bt.nbb3 & 3)))
    return fail(LAMM_ERR_ALIGN, "f32 B must be 4-byte aligned");
  if (probe().count == 0) return fail(LAMM_ERR_NODEV, "no gfx950 device");

  hipStream_t s = static_cast<hipStream_t>(hip_stream);
  GemvArgs p{static_cast<const unsigned char*>(A->data), lda, static_cast<const unsigned char*>(B->data), ldb,
             static_cast<float*>(C->data), C->ld, M, N, Kb * block_elems(A->type), Kb};
  p.ne12 = (int)bt.ne12;
  p.ne13 = (int)bt.ne13;
  p.r2 = (int)(bt.ne12 / bt.ne02);
  p.r3 = (int)(bt.ne13 / bt.ne03);
  p.sa2 = (int64_t)bt.nba2;
  p.sa3 = (int64_t)bt.nba3;
  p.sb2 = (int64_t)bt.nbb2;
  p.sb3 = (int64_t)bt.nbb3;
  p.sc2 = (int64_t)(bt.nbc2 / 4);
  p.sc3 = (int64_t)(bt.nbc3 / 4);
  p.b_f32 = b_f32 ? 1 : 0;
  hipError_t e;
  if (flags & LAMM_ORDER_REFERENCE) {   // the reference's x86 float order (lamm_ref.hip), bit for bit
    if (!ref_order_supported(A->type, vdt) || (b_f32 && !ref_gemv_supported(A->type, p)))
      return fail(LAMM_ERR_TYPE, "no reference-order kernel for A type %d with B type %d (N %d)", A->type, B->type, N);
    if (done && ref_gemv_supported(A->type, p) && p.ne12 * p.ne13 == 1) {
      p.done_ctr = done->ctr;
      p.flag = done->flag;
      p.seq = done->seq;
      done->signaled = true;
    }
    e = launch_ref(A->type, p, s);
    if (e != hipSuccess) return fail(LAMM_ERR_HIP, "kernel launch: %s", hipGetErrorString(e));
    return LAMM_OK;
  }
  const bool b_al4 = (ldb & 3) == 0 && ((uintptr_t)B->data & 3) == 0 && (bt.nbb2 & 3) == 0 && (bt.nbb3 & 3) == 0;
  switch (pick_engine(A->type, p, W && W->packed, b_al4)) {
    case kEngGemv:
      if (done && gemv_rpw_supported(A->type, p) && rpw_waves(p) > 0) {
        p.done_ctr = done->ctr;
        p.flag = done->flag;
        p.seq = done->seq;
        done->signaled = true;
      }
      e = launch_gemv(A->type, p, s);
      break;
    case kEngDense: {
      const size_t wsb = gemm_dense_workspace_bytes(A->type, p);
      void* ws = nullptr;
      if (wsb && !(ws = workspace(wsb, s))) return fail(LAMM_ERR_HIP, "workspace allocation of %zu bytes failed", wsb);
      e = launch_gemm_dense(A->type, p, ws, s);
      break;
    }
    case kEngKq: {
      const void* prepA = W ? W->packed : nullptr;
      const size_t wsb = gemm_kq_workspace_bytes(A->type, p, prepA != nullptr);
      void* ws = workspace(wsb, s);
      if (!ws) return fail(LAMM_ERR_HIP, "workspace allocation of %zu bytes failed", wsb);
      e = launch_gemm_kq(A->type, p, prepA, ws, s);
      break;
    }
    case kEngFp6: {
      const void* prepA = W ? W->packed : nullptr;
      const size_t wsb = gemm_fp6_workspace_bytes(A->type, p, prepA != nullptr);
      void* ws = workspace(wsb, s);
      if (!ws) return fail(LAMM_ERR_HIP, "workspace allocation of %zu bytes failed", wsb);
      e = launch_gemm_fp6(A->type, p, prepA, ws, s);
      break;
    }
    case kEngDq: {
      const size_t wsb = gemm_dq_workspace_bytes(p);
      void* ws = nullptr;
      if (wsb && !(ws = workspace(wsb, s))) return fail(LAMM_ERR_HIP, "workspace allocation of %zu bytes failed", wsb);
      e = launch_gemm_dq(A->type, p, ws, s);
      break;
    }
    case kEngI8: {
      void* ws = nullptr;
      const size_t wsb = gemm_workspace_bytes(A->type, p);
      if (wsb && !(ws = workspace(wsb, s))) return fail(LAMM_ERR_HIP, "workspace allocation of %zu bytes failed", wsb);
      e = launch_gemm(A->type, p, ws, s);
      break;
    }
    default:   // kEngGemvGroups: GEMV launches of 8 columns
      e = hipSuccess;
      for (int j0 = 0; j0 < N && e == hipSuccess; j0 += 8) {
        GemvArgs q = p;
        q.B = p.B + (int64_t)j0 * ldb;
        q.C = p.C + (int64_t)j0 * p.ldc;
        q.N = N - j0 < 8 ? N - j0 : 8;
        e = launch_gemv(A->type, q, s);
      }
  }
  if (e != hipSuccess) return fail(LAMM_ERR_HIP, "kernel launch: %s", hipGetErrorString(e));
  return LAMM_OK;
}

}  // namespace

LaunchTiming lamm::take_launch_timing() {
  const LaunchTiming t = g_timing;
  g_timing = LaunchTiming{};
  return t;
}

extern "C" int lamm_hip_profile_next(void* start_event, void* stop_event) {
  g_timing = LaunchTiming{static_cast<hipEvent_t>(start_event), static_cast<hipEvent_t>(stop_event)};
  return LAMM_OK;
}

extern "C" int lamm_hip_direct_begin(int device) {
  const std::vector<int>& ids = probe().ids;
  if (std::find(ids.begin(), ids.end(), device) == ids.end())
    return fail(LAMM_ERR_NODEV, "lamm_hip_direct_begin: no gfx950 device %d", device);
  if (!lamm::direct_begin(device))
    return fail(LAMM_ERR_HIP, "lamm_hip_direct_begin: no direct queue on device %d: %s", device,
                lamm::direct_reason().c_str());
  return LAMM_OK;
}

extern "C" int lamm_hip_direct_end(void) {
  if (!lamm::direct_active()) return -fail(LAMM_ERR_HIP, "lamm_hip_direct_end: no region open");
  const int n = lamm::direct_end();
  // calls whose kernel could not go onto the queue ran through HIP: say why (round 5's driver box
  // dispatched nothing directly with no reason given)
  if (lamm::direct_fallbacks() > 0)
    fail(LAMM_ERR_HIP, "lamm_hip_direct_end: %d call(s) launched through HIP: %s", lamm::direct_fallbacks(),
         lamm::direct_reason().c_str());
  else if (n == 0)
    fail(LAMM_ERR_HIP, "lamm_hip_direct_end: no call was made in the region");
  return n;
}

extern "C" int lamm_hip_matmul_batched(const lamm_matrix* A, const lamm_matrix* B, const lamm_matrix* C,
                                       const lamm_batch* batch, void* hip_stream) {
  return matmul_impl(A, B, C, batch, hip_stream, nullptr);
}

extern "C" const char* lamm_hip_engine(int type, int64_t M, int N, int K, int slices, int stationary, int b_f32) {
  static const char* const names[] = {"gemv", "dense", "superblock", "fp6", "i8", "gemv-groups", "dq16"};
  if (!is_weight_type(type) || M < 1 || N < 1 || K < 1 || slices < 1 || K % block_elems(type)) return "";
  const int kb = K / block_elems(type);
  GemvArgs p{nullptr, (int64_t)kb * (int64_t)block_bytes(type), nullptr, 0, nullptr, M, (int)M, N, K, kb};
  p.ne12 = slices;
  p.r2 = 1;
  p.b_f32 = b_f32 && (vec_dot_type(type) == kQ8_0 || vec_dot_type(type) == kQ8_1) ? 1 : 0;
  const bool packs = gemm_fp6_supported(type) || gemm_kq_supported(type);
  return names[pick_engine(type, p, stationary && packs, true)];
}

extern "C" int lamm_hip_weights_create(const lamm_matrix* A, int64_t ne02, int64_t ne03, size_t nba2, size_t nba3,
                                       void* hip_stream, lamm_weights** out) {
  if (!A || !out) return fail(LAMM_ERR_SHAPE, "null argument");
  *out = nullptr;
  if (!is_weight_type(A->type)) return fail(LAMM_ERR_TYPE, "unsupported A type %d", A->type);
  if (A->row < 0 || A->col < 0 || A->ld < A->col) return fail(LAMM_ERR_SHAPE, "bad A shape");
  if (ne02 < 1 || ne03 < 1 || ne02 * ne03 > 65535) return fail(LAMM_ERR_SHAPE, "bad A slice counts");
  const int64_t lda = A->ld * (int64_t)block_bytes(A->type);
  if (((uintptr_t)A->data & 15) || (lda & 15) || (nba2 & 15) || (nba3 & 15))
    return fail(LAMM_ERR_ALIGN, "A must be 16-byte aligned with 16-byte row/slice pitches");
  if (probe().count == 0) return fail(LAMM_ERR_NODEV, "no gfx950 device");
  auto* W = new lamm_weights{*A, ne02, ne03, nba2, nba3};
  const bool fp6 = gemm_fp6_supported(A->type), kq = gemm_kq_supported(A->type);
  if ((fp6 || kq) && A->row > 0 && A->col > 0) {
    const GemvArgs p = weight_args(A, ne02, ne03, nba2, nba3);
    W->packed_bytes = fp6 ? gemm_fp6_weight_bytes(A->type, p) : gemm_kq_weight_bytes(A->type, p);
    if (hipMalloc(&W->packed, W->packed_bytes) != hipSuccess) {
      const size_t nb = W->packed_bytes;
      delete W;
      return fail(LAMM_ERR_HIP, "hipMalloc of %zu packed weight bytes failed", nb);
    }
    bool in_range = true;
    const hipError_t e = fp6 ? prepare_fp6_weights(A->type, p, W->packed, static_cast<hipStream_t>(hip_stream), &in_range)
                             : prepare_kq_weights(A->type, p, W->packed, static_cast<hipStream_t>(hip_stream));
    if (e != hipSuccess) {
      (void)hipFree(W->packed);
      delete W;
      return fail(LAMM_ERR_HIP, "weight packing: %s", hipGetErrorString(e));
    }
    if (!in_range) {   // q5_1 block scales past the packed form's range: the unpacked engines take it
      (void)hipFree(W->packed);
      W->packed = nullptr;
      W->packed_bytes = 0;
    }
  }
  *out = W;
  return LAMM_OK;
}

extern "C" int lamm_hip_matmul_weights(const lamm_weights* W, const lamm_matrix* B, const lamm_matrix* C,
                                       const lamm_batch* batch, void* hip_stream) {
  if (!W) return fail(LAMM_ERR_SHAPE, "null weights");
  lamm_batch bt{W->ne02, W->ne03, W->ne02, W->ne03, W->nba2, W->nba3, 0, 0, 0, 0};
  if (batch) {
    if (batch->ne02 != W->ne02 || batch->ne03 != W->ne03 || batch->nba2 != W->nba2 || batch->nba3 != W->nba3)
      return fail(LAMM_ERR_SHAPE, "batch A dims differ from the prepared weights'");
    bt = *batch;
  }
  return matmul_impl(&W->A, B, C, &bt, hip_stream, W);
}

extern "C" size_t lamm_hip_weights_bytes(const lamm_weights* W) { return W ? W->packed_bytes : 0; }

extern "C" void lamm_hip_weights_destroy(lamm_weights* W) {
  if (!W) return;
  if (W->packed) {
    (void)hipDeviceSynchronize();   // no launch may still read the packed form
    (void)hipFree(W->packed);
  }
  delete W;
}

extern "C" int lamm_hip_matmul(const lamm_matrix* A, const lamm_matrix* B, const lamm_matrix* C,
                               void* hip_stream) {
  return lamm_hip_matmul_batched(A, B, C, nullptr, hip_stream);
}

extern "C" int lamm_hip_matmul_ex(const lamm_matrix* A, const lamm_matrix* B, const lamm_matrix* C,
                                  const lamm_batch* batch, int flags, void* hip_stream) {
  return matmul_impl(A, B, C, batch, hip_stream, nullptr, flags);
}

extern "C" int lamm_hip_matmul_group(const lamm_matrix* A, int n, const lamm_matrix* B, const lamm_matrix* C,
                                     int flags, void* hip_stream) {
  if (!A || !B || !C) return fail(LAMM_ERR_SHAPE, "null matrix");
  if (n < 1 || n > LAMM_GROUP_MAX) return fail(LAMM_ERR_SHAPE, "group of %d weights (1..%d)", n, LAMM_GROUP_MAX);
  // one launch: the one-column kernel of the call's order over every weight of one type and row
  // length (the reference order: ref_gemv_group_kernel; the fast engines: gemv_flat_group_kernel for
  // the K = 4096 weights their single calls run on gemv_flat1_kernel)
  const bool ref = (flags & LAMM_ORDER_REFERENCE) != 0;
  bool one = n > 1 && B->col == 1;
  for (int i = 0; i < n && one; ++i)
    one = A[i].type == A[0].type && A[i].col == A[0].col && A[i].ld == A[0].ld && A[i].row > 0 &&
          C[i].type == kF32 && C[i].row == A[i].row && C[i].col == 1 && ((uintptr_t)A[i].data & 15) == 0 &&
          ((uintptr_t)C[i].data & 3) == 0;
  if (one) {
    const int t = A[0].type, vdt = vec_dot_type(t), Kb = A[0].col;
    const bool b_f32 = B->type == kF32 && (vdt == kQ8_0 || vdt == kQ8_1);
    const int64_t lda = A[0].ld * (int64_t)block_bytes(t);
    one = is_weight_type(t) && (!ref || ref_order_supported(t, vdt)) && (B->type == vdt || b_f32) &&
          B->row == (b_f32 ? Kb * block_elems(t) : Kb) && A[0].ld >= Kb && (lda & 15) == 0 &&
          ((uintptr_t)B->data & (b_f32 ? 3 : 0)) == 0;
    if (one) {
      GemvArgs p{static_cast<const unsigned char*>(A[0].data), lda, static_cast<const unsigned char*>(B->data),
                 B->ld * (int64_t)block_bytes(B->type), static_cast<float*>(C[0].data), C[0].ld, A[0].row, 1,
                 Kb * block_elems(t), Kb};
      p.b_f32 = b_f32 ? 1 : 0;
      RefSegs sg{};
      for (int i = 0; i < n; ++i) {
        sg.A[i] = static_cast<const unsigned char*>(A[i].data);
        sg.C[i] = static_cast<float*>(C[i].data);
        sg.M[i] = A[i].row;
      }
      if ((ref ? ref_gemv_supported(t, p) : gemv_group_supported(t, p, sg, n)) && probe().count > 0) {
        // a lamm_hip_profile_next request brackets the one launch, as matmul_impl brackets its
        // launches (it used to be dropped here)
        const LaunchTiming tm = g_timing;
        g_timing = LaunchTiming{};
        g_completion = nullptr;
        const hipStream_t s = static_cast<hipStream_t>(hip_stream);
        if (tm.start) (void)hipEventRecord(tm.start, s);
        const hipError_t e = ref ? launch_ref_group(t, p, sg, n, s) : launch_gemv_group(t, p, sg, n, s);
        if (tm.start) (void)hipEventRecord(tm.stop, s);
        if (e != hipSuccess) return fail(LAMM_ERR_HIP, "kernel launch: %s", hipGetErrorString(e));
        return LAMM_OK;
      }
    }
  }
  for (int i = 0; i < n; ++i) {   // anything else: one call per weight (the same kernels, the same bits)
    const int rc = matmul_impl(&A[i], B, &C[i], nullptr, hip_stream, nullptr, flags);
    if (rc != LAMM_OK) return rc;
  }
  return LAMM_OK;
}

extern "C" int lamm_hip_quantize(int vec_type, int flavour, const float* x, int64_t ldx, void* y,
                                 int64_t ldy, int K, int N, void* hip_stream) {
  const bool wq = quantize_weights_supported(vec_type);
  if (!wq && vec_type != kQ8_0 && vec_type != kQ8_1 && vec_type != kQ8_K && vec_type != kF16)
    return fail(LAMM_ERR_TYPE, "quantize: unsupported type %d", vec_type);
  if (K % block_elems(vec_type)) return fail(LAMM_ERR_SHAPE, "quantize: K %% block != 0");
  if (((uintptr_t)x & 15) || (ldx & 3)) return fail(LAMM_ERR_ALIGN, "quantize: x must be 16B aligned, ldx %% 4 == 0");
  if (probe().count == 0) return fail(LAMM_ERR_NODEV, "no gfx950 device");
  const int64_t ldyb = ldy * (int64_t)block_bytes(vec_type);
  hipError_t e = wq ? launch_quantize_weights(vec_type, x, ldx, y, ldyb, K, N, static_cast<hipStream_t>(hip_stream))
                    : launch_quantize(vec_type, flavour, x, ldx, y, ldyb, K, N, static_cast<hipStream_t>(hip_stream));
  if (e != hipSuccess) return fail(LAMM_ERR_HIP, "quantize launch: %s", hipGetErrorString(e));
  return LAMM_OK;
}

// ===================================================== ggml boundary
namespace {

[[noreturn]] void die(const char* what, hipError_t e) {
  fprintf(stderr, "lamm_hip: %s failed: %s\n", what, hipGetErrorString(e));
  std::abort();
}
#define HIPCHK(x)                           \
  do {                                      \
    hipError_t _e = (x);                    \
    if (_e != hipSuccess) die(#x, _e);      \
  } while (0)

// Device copy of one weight slice, keyed by the host slice it came from.
struct WeightKey {
  const void* host;
  int type;
  int64_t rows, kb;
  size_t host_pitch, host_s2, host_s3;   // nb[1], nb[2], nb[3]
  bool operator==(const WeightKey& o) const {
    return host == o.host && type == o.type && rows == o.rows && kb == o.kb && host_pitch == o.host_pitch &&
           host_s2 == o.host_s2 && host_s3 == o.host_s3;
  }
};
struct WeightKeyHash {
  size_t operator()(const WeightKey& k) const {
    size_t h = std::hash<const void*>()(k.host);
    h ^= std::hash<int64_t>()(k.rows * 1315423911ll + k.kb * 2654435761ll + k.type) + 0x9e3779b9 + (h << 6);
    h ^= std::hash<size_t>()(k.host_s2 * 40503u + k.host_s3) + 0x9e3779b9 + (h << 6);
    return h;
  }
};
struct WeightEntry {
  void* dev = nullptr;
  int64_t dev_pitch = 0;
  size_t bytes = 0;
  lamm_weights* prepared = nullptr;   // packed GEMM form, made on the first prefill call
  uint64_t fingerprint = 0;
  std::list<WeightKey>::iterator lru;
};

uint64_t fingerprint(const unsigned char* p, size_t pitch, size_t row_bytes, int64_t rows) {
  // FNV-1a over 16 sampled 8-byte windows spread over the slice, plus the shape (each window is a
  // host cache miss on every decode call: 64 of them cost ~1.5 us of a ~20 us call,
  // profiles/r02/ab_zero_copy_spin.txt "weights lookup")
  uint64_t h = 1469598103934665603ull ^ (row_bytes * 31 + (uint64_t)rows);
  const size_t total = (size_t)(rows - 1) * pitch + row_bytes;
  const size_t win = total < 8 ? total : 8;
  for (int s = 0; s < 16; ++s) {
    const size_t pos = (size_t)((double)(total - win) * s / 15.0);
    uint64_t v = 0;
    memcpy(&v, p + pos, win);
    for (int b = 0; b < 8; ++b) { h ^= (v >> (8 * b)) & 0xff; h *= 1099511628211ull; }
  }
  return h;
}

// LAMM_HIP_STATS=1: per-category count and wall time of lamm_mul_mat (thread 0, entry to
// return: transfers, kernels, synchronisation), printed to stderr at exit -- how much of a
// llama.cpp token the boundary accounts for.
// Also the medians of a call's wall time and of the gap since thread 0 left the previous call
// (ggml's barriers and CPU ops in between; gaps over 5 ms -- between passes -- left out).
struct CallStats {
  const char* name;
  uint64_t calls = 0;
  double us = 0;
  double phase_us[7] = {0, 0, 0, 0, 0, 0, 0};
  std::vector<float> call_us, gap_us;
};
std::chrono::steady_clock::time_point g_last_return{};
// per-call samples kept for the medians: the first kSamples, then a ring over them (bounded memory
// in a long LAMM_HIP_STATS run)
constexpr size_t kSamples = 1 << 16;
void sample(std::vector<float>& v, uint64_t n, float x) {
  if (v.size() < kSamples) v.push_back(x);
  else v[n % kSamples] = x;
}
double median(std::vector<float> v) {
  if (v.empty()) return 0.0;
  std::nth_element(v.begin(), v.begin() + v.size() / 2, v.end());
  return v[v.size() / 2];
}
constexpr int kPhases = 7;
const char* kPhase[kPhases] = {"host staging", "src0", "B up", "launch", "C down", "device sync", "C to dst"};
CallStats g_stats[4] = {{"weights N<=8"}, {"weights N>8"}, {"views N<=8"}, {"views N>8"}};
bool stats_on() { return knobs().stats; }
void print_sibling_stats();
void print_stats() {
  for (const auto& c : g_stats)
    if (c.calls)
    {
      fprintf(stderr, "lamm_hip stats: %-13s %8llu calls %12.1f us total %8.2f us/call  (", c.name,
              (unsigned long long)c.calls, c.us, c.us / (double)c.calls);
      for (int k = 0; k < kPhases; ++k) fprintf(stderr, "%s%s %.2f", k ? ", " : "", kPhase[k], c.phase_us[k] / c.calls);
      fprintf(stderr, ")  median call %.2f us, median gap before it %.2f us\n", median(c.call_us), median(c.gap_us));
    }
  print_sibling_stats();
}
struct StatScope {
  CallStats* c;
  std::chrono::steady_clock::time_point t0, tp;
  explicit StatScope(CallStats* cs) : c(cs), t0(std::chrono::steady_clock::now()), tp(t0) {
    if (c && g_last_return.time_since_epoch().count()) {
      const double gap = std::chrono::duration<double, std::micro>(t0 - g_last_return).count();
      if (gap < 5000.0) sample(c->gap_us, c->calls, (float)gap);
    }
  }
  void phase(int k) {   // time since the previous mark -> phase k
    if (!c) return;
    const auto now = std::chrono::steady_clock::now();
    c->phase_us[k] += std::chrono::duration<double, std::micro>(now - tp).count();
    tp = now;
  }
  ~StatScope() {
    if (c) {
      g_last_return = std::chrono::steady_clock::now();
      const double us = std::chrono::duration<double, std::micro>(g_last_return - t0).count();
      sample(c->call_us, c->calls, (float)us);
      c->calls++;
      c->us += us;
    }
  }
};


// One device of the ggml boundary: its stream, its weight cache (LRU under the per-device budget)
// and grow-only scratch.  With LAMM_HIP_DEVICES listing several devices, every weight's rows are
// split over them (SURVEY §8e "host consumes C": each device computes its row slab of C and
// copies it straight into dst's rows -- no collective); device ids may repeat (a rehearsal of the
// multi-GPU path on one GPU).
struct Dev {
  int id = 0;
  hipStream_t stream = nullptr;
  hipStream_t stream2 = nullptr;  // the pipelined prefill's second column chunk (LAMM_HIP_POOL bit 4)
  hipEvent_t upload = nullptr;    // stream2 waits on it: the weight upload enqueued on stream
  unsigned* flag = nullptr;       // pinned, host-coherent completion word (lamm_signal.hip)
  unsigned* flag_dev = nullptr;   // its device address
  unsigned seq = 0;
  unsigned* done_ctr = nullptr;   // device counter for the GEMV's own completion signal
  unsigned pending = 0;           // seq the last call's kernel signals itself (0: none)
  bool enqueued = false;          // an upload went onto `stream` since the last direct region (lamm_aql.cpp)
  unsigned char* xv = nullptr;    // decode activations in fine-grained device memory, written by the host
  size_t xv_cap = 0;              // through the BAR (LAMM_HIP_VRAM_X); xv_ok -1: not available here
  int xv_ok = 0;

  // the activation buffer in device memory the host writes directly (nullptr: not available)
  unsigned char* vram_x(size_t bytes) {
    if (xv_ok < 0) return nullptr;
    if (xv_cap < bytes) {
      // on this device, the first allocation too (the caller's current device can be
      // another one, and the buffer and its HDP flush must be this device's)
      (void)hipSetDevice(id);
      if (xv) {
        (void)hipStreamSynchronize(stream);
        (void)hipFree(xv);
        xv = nullptr;
        xv_cap = 0;
      }
      void* p = nullptr;
      if (!lamm::vram_host_writable(id) || hipExtMallocWithFlags(&p, bytes + 256, hipDeviceMallocFinegrained) != hipSuccess) {
        xv_ok = -1;
        return nullptr;
      }
      xv = static_cast<unsigned char*>(p);
      xv_cap = bytes;
      xv_ok = 1;
    }
    return xv;
  }
  std::unordered_map<WeightKey, WeightEntry, WeightKeyHash> cache;
  std::list<WeightKey> lru;
  size_t cached = 0;
  void* buf[4] = {nullptr, nullptr, nullptr, nullptr};   // B, C, F32 src1, transient src0
  size_t cap[4] = {0, 0, 0, 0};

  void* scratch(int which, size_t bytes) {
    if (cap[which] < bytes) {
      if (buf[which]) HIPCHK(hipFree(buf[which]));
      HIPCHK(hipMalloc(&buf[which], bytes + 256));
      cap[which] = bytes;
    }
    return buf[which];
  }
  void evict(std::unordered_map<WeightKey, WeightEntry, WeightKeyHash>::iterator it) {
    if (it == cache.end()) return;
    (void)hipSetDevice(id);
    (void)hipStreamSynchronize(stream);
    (void)hipFree(it->second.dev);
    if (it->second.prepared) {
      cached -= lamm_hip_weights_bytes(it->second.prepared);
      lamm_hip_weights_destroy(it->second.prepared);
    }
    cached -= it->second.bytes;
    lru.erase(it->second.lru);
    cache.erase(it);
  }
};

// A src0 that is not a weight -- a view of the KV cache or an intermediate -- is uploaded on
// EVERY call and never cached: b2430's K/V views keep one data pointer while single token
// rows change inside them (llama.cpp:5322-5372 views, :8887 kv_self.n padded to 32), which no
// sampled fingerprint can see.  Device layout (pitch, slice strides in bytes):
//   rows stacked (nb2 = nb1*ne1, nb3 = nb2*ne2; the transposed V view): one 2D copy;
//   dense interleaved slices (the K view: the heads of a token side by side in one cache
//     row, nb1 = n_embd_k_gqa*2, nb2 = 256): one linear copy of the byte span, host strides;
//   anything else: a 2D copy per slice.
struct Transient {
  void* dev;
  int64_t pitch;
  size_t s2, s3;
};
Transient upload_transient(Dev& d, const ggml::tensor* src0, size_t row_bytes) {
  d.enqueued = true;
  const int64_t ne1 = src0->ne[1], ne2 = src0->ne[2], ne3 = src0->ne[3];
  const size_t nb1 = src0->nb[1], nb2 = src0->nb[2], nb3 = src0->nb[3];
  const auto* host = static_cast<const unsigned char*>(src0->data);
  const size_t bpb = block_bytes(src0->type);
  const size_t span = (size_t)(ne1 - 1) * nb1 + (size_t)(ne2 - 1) * nb2 + (size_t)(ne3 - 1) * nb3 + row_bytes;
  const size_t payload = row_bytes * (size_t)(ne1 * ne2 * ne3);
  const bool stacked = nb2 == nb1 * (size_t)ne1 && nb3 == nb2 * (size_t)ne2;
  // the whole span in one linear copy, host strides kept (the K view: heads interleaved; the
  // transposed V view: rows of n_kv cells at an n_ctx pitch) -- a 2D copy from pageable memory
  // goes row by row
  if (nb1 % 16 == 0 && nb2 % 16 == 0 && nb3 % 16 == 0 && nb1 % bpb == 0 && nb1 >= row_bytes && span <= 2 * payload) {
    void* dev = d.scratch(3, span + 64);
    HIPCHK(hipMemcpyAsync(dev, host, span, hipMemcpyHostToDevice, d.stream));
    return Transient{dev, (int64_t)nb1, nb2, nb3};
  }
  size_t pb = row_bytes / bpb;
  while ((pb * bpb) % 16) ++pb;
  const int64_t pitch = (int64_t)(pb * bpb);
  void* dev = d.scratch(3, (size_t)pitch * (size_t)(ne1 * ne2 * ne3) + 64);
  auto* dp = static_cast<unsigned char*>(dev);
  if (stacked) {
    HIPCHK(hipMemcpy2DAsync(dp, pitch, host, nb1, row_bytes, (size_t)(ne1 * ne2 * ne3), hipMemcpyHostToDevice,
                            d.stream));
  } else {
    for (int64_t i3 = 0; i3 < ne3; ++i3)
      for (int64_t i2 = 0; i2 < ne2; ++i2)
        HIPCHK(hipMemcpy2DAsync(dp + (i3 * ne2 + i2) * ne1 * pitch, pitch, host + i2 * nb2 + i3 * nb3, nb1, row_bytes,
                                (size_t)ne1, hipMemcpyHostToDevice, d.stream));
  }
  return Transient{dev, pitch, (size_t)pitch * ne1, (size_t)pitch * ne1 * ne2};
}

// the fingerprint of every (i02, i03) slice of a weight (sampled bytes + shape), host side
uint64_t weight_fingerprint(const ggml::tensor* src0, size_t row_bytes) {
  uint64_t fp = 0;
  for (int64_t i3 = 0; i3 < src0->ne[3]; ++i3)
    for (int64_t i2 = 0; i2 < src0->ne[2]; ++i2)
      fp = fp * 1099511628211ull ^ fingerprint(static_cast<const unsigned char*>(src0->data) + i2 * src0->nb[2] +
                                                   i3 * src0->nb[3],
                                               src0->nb[1], row_bytes, src0->ne[1]);
  return fp;
}

class Runtime {
 public:
  static Runtime& get() {
    static Runtime* r = new Runtime();  // leaked on purpose: no teardown-order issues
    return *r;
  }

  std::mutex mu;
  std::vector<Dev> devs;

  // LAMM_HIP_DEVICES: unset = the one boundary device (LAMM_HIP_DEVICE / the first gfx950);
  // "all" = every gfx950 device; "0,1,2,3" = that list (repeats allowed: one-GPU rehearsal)
  void ensure_init() {
    if (!devs.empty()) return;
    std::vector<int> ids;
    const char* e = knobs().devices;
    int nvis = 0;
    (void)hipGetDeviceCount(&nvis);
    if (e && !strcmp(e, "all")) {
      ids = probe().ids;
    } else if (e && *e) {
      for (const char* c = e; *c;) {
        char* end = nullptr;
        const long v = strtol(c, &end, 10);
        if (end == c) break;
        if (v < 0 || v >= nvis) {
          fprintf(stderr, "lamm_hip: LAMM_HIP_DEVICES lists device %ld of %d\n", v, nvis);
          std::abort();
        }
        ids.push_back((int)v);
        c = *end == ',' ? end + 1 : end;
      }
    }
    if (ids.empty()) ids.push_back(knobs().device >= 0 ? knobs().device : probe().device);
    devs.resize(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
      devs[i].id = ids[i];
      HIPCHK(hipSetDevice(ids[i]));
      HIPCHK(hipStreamCreateWithFlags(&devs[i].stream, hipStreamNonBlocking));
      HIPCHK(hipStreamCreateWithFlags(&devs[i].stream2, hipStreamNonBlocking));
      HIPCHK(hipEventCreateWithFlags(&devs[i].upload, hipEventDisableTiming));
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&devs[i].flag), 64, hipHostMallocCoherent | hipHostMallocMapped));
      HIPCHK(hipHostGetDevicePointer(reinterpret_cast<void**>(&devs[i].flag_dev), devs[i].flag, 0));
      *(volatile unsigned*)devs[i].flag = 0;
      HIPCHK(hipMalloc(reinterpret_cast<void**>(&devs[i].done_ctr), 64));
      HIPCHK(hipMemset(devs[i].done_ctr, 0, 64));
    }
    budget_ = (size_t)(knobs().cache_gb * (1ull << 30));
    static bool stats_registered = false;
    if (stats_on() && !stats_registered) {
      stats_registered = true;
      atexit(print_stats);
    }
  }

  // rows [r0, r0 + rows) of every (i02, i03) slice of a weight on device d, re-pitched to 16 B
  WeightEntry& weights(Dev& d, const WeightKey& k, size_t row_bytes, const ggml::tensor* src0, int64_t r0,
                       int64_t rows, uint64_t fp) {
    const int64_t ne02 = src0->ne[2], ne03 = src0->ne[3];
    auto it = d.cache.find(k);
    if (it != d.cache.end()) {
      if (it->second.fingerprint == fp) {
        d.lru.splice(d.lru.begin(), d.lru, it->second.lru);
        return it->second;
      }
      d.evict(it);
    }
    WeightEntry e;
    d.enqueued = true;   // the upload below goes onto d.stream
    const size_t bpb = block_bytes(k.type);
    size_t pitch_blocks = (size_t)k.kb;
    while ((pitch_blocks * bpb) % 16) ++pitch_blocks;
    e.dev_pitch = (int64_t)(pitch_blocks * bpb);
    e.bytes = (size_t)e.dev_pitch * (size_t)(rows * ne02 * ne03) + 64;
    while (d.cached + e.bytes > budget_ && !d.lru.empty()) d.evict(d.cache.find(d.lru.back()));
    HIPCHK(hipMalloc(&e.dev, e.bytes));
    for (int64_t i3 = 0; i3 < ne03; ++i3)
      for (int64_t i2 = 0; i2 < ne02; ++i2)
        HIPCHK(hipMemcpy2DAsync(static_cast<unsigned char*>(e.dev) + (i3 * ne02 + i2) * rows * e.dev_pitch,
                                e.dev_pitch,
                                static_cast<const unsigned char*>(k.host) + i2 * src0->nb[2] + i3 * src0->nb[3] +
                                    r0 * src0->nb[1],
                                k.host_pitch, row_bytes, rows, hipMemcpyHostToDevice, d.stream));
    e.fingerprint = fp;
    d.lru.push_front(k);
    e.lru = d.lru.begin();
    d.cached += e.bytes;
    return d.cache.emplace(k, e).first->second;
  }

  // the entry's weight-stationary handle (packed GEMM form), created on first use
  lamm_weights* prepared(Dev& d, WeightEntry& e, const lamm_matrix& A, int64_t ne02, int64_t ne03) {
    if (!e.prepared) {
      const size_t pitch = (size_t)e.dev_pitch * A.row;
      if (lamm_hip_weights_create(&A, ne02, ne03, pitch, pitch * ne02, d.stream, &e.prepared) != LAMM_OK) {
        fprintf(stderr, "lamm_hip: lamm_hip_weights_create failed: %s\n", g_err.c_str());
        std::abort();
      }
      d.cached += lamm_hip_weights_bytes(e.prepared);
    }
    return e.prepared;
  }

  // pinned host staging (grow-only), mapped into the device's address space: 0 = activations
  // the kernels read in place (non-coherent: the GPU may cache them in L2; every launch's
  // acquire drops stale lines), 1 = C the kernels write in place; pinned_dev = the device
  // address of the same bytes.  LAMM_HIP_PINNED=0 turns staging off (A/B).
  unsigned char* pinned(int which, size_t bytes) {
    if (hcap_[which] < bytes) {
      if (hbuf_[which]) {
        for (Dev& d : devs) {
          (void)hipSetDevice(d.id);
          (void)hipStreamSynchronize(d.stream);
        }
        HIPCHK(hipHostFree(hbuf_[which]));
      }
      // 2: the prefill pool's upload image (DMA only, not mapped); 0: activations, cached in the
      // device's L2 (every launch's acquire drops stale lines); 1: C, non-coherent (written back
      // by the kernel's end-of-kernel release) -- coherent under LAMM_HIP_C_WATCH=1, whose stores
      // then go straight to host memory while watch_c spins on them
      const unsigned flags = which == 2 ? hipHostMallocPortable
                                        : hipHostMallocMapped | hipHostMallocPortable |
                                              (which == 0 || knobs().c_watch != 1 ? hipHostMallocNonCoherent
                                                                                  : hipHostMallocCoherent);
      HIPCHK(hipHostMalloc(reinterpret_cast<void**>(&hbuf_[which]), bytes + 256, flags));
      if (which != 2) HIPCHK(hipHostGetDevicePointer(&hdev_[which], hbuf_[which], 0));
      hcap_[which] = bytes;
    }
    return hbuf_[which];
  }
  void* pinned_dev(int which) const { return hdev_[which]; }
  // the staging buffer (grown to `bytes`) has one address on every device: what zero-copy over
  // several devices needs (ROCm maps pinned host memory at its host address)
  bool pinned_shared(int which, size_t bytes) {
    pinned(which, bytes);
    return hdev_[which] == static_cast<void*>(hbuf_[which]);
  }

  void clear() {
    for (Dev& d : devs)
      while (!d.lru.empty()) d.evict(d.cache.find(d.lru.back()));
  }
  // drop every device's cache, scratch and stream; the next call re-reads the environment
  void reset() {
    clear();
    for (Dev& d : devs) {
      (void)hipSetDevice(d.id);
      (void)hipStreamSynchronize(d.stream);
      for (void* b : d.buf)
        if (b) (void)hipFree(b);
      if (d.xv) (void)hipFree(d.xv);
      (void)hipHostFree(d.flag);
      if (d.done_ctr) (void)hipFree(d.done_ctr);
      (void)hipStreamDestroy(d.stream);
      (void)hipStreamSynchronize(d.stream2);
      (void)hipStreamDestroy(d.stream2);
      (void)hipEventDestroy(d.upload);
    }
    devs.clear();
  }
  size_t cached_bytes() const {
    size_t n = 0;
    for (const Dev& d : devs) n += d.cached;
    return n;
  }

 private:
  size_t budget_ = 0;
  unsigned char* hbuf_[4] = {nullptr, nullptr, nullptr, nullptr};   // 3: sibling results (Siblings)
  void* hdev_[4] = {nullptr, nullptr, nullptr, nullptr};
  size_t hcap_[4] = {0, 0, 0, 0};
};

bool use_pinned(size_t bytes) {
  const bool on = knobs().pinned;
  // decode-sized transfers only: through the unchanged ggml (tools/ab_pinned.sh,
  // profiles/r01/ab_pinned.txt) Q4_0 4096x1x4096 27.7 -> 23.3 us, but N = 8 (128 KiB of C)
  // 41.8 -> 46 us and N = 512 (8 MiB) 367 -> 691 us: the host-side strided copy out of the
  // pinned buffer costs more than HIP's own pageable path saves
  return on && bytes <= ((size_t)32 << 10);
}

int opt_level() { return knobs().opt_level; }

bool is_contiguous(const ggml::tensor* t) {
  const size_t ts = block_bytes(t->type);
  const int be = block_elems(t->type);
  return t->nb[0] == ts && t->nb[1] == t->nb[0] * (size_t)(t->ne[0] / be) && t->nb[2] == t->nb[1] * (size_t)t->ne[1] &&
         t->nb[3] == t->nb[2] * (size_t)t->ne[2];
}

// A real weight: a leaf tensor that owns its bytes (GGML_OP_NONE = 0, not a view).  Only those
// are kept device-resident across calls; KV-cache views and intermediates are re-uploaded.
bool is_weight(const ggml::tensor* t) { return t->view_src == nullptr && t->op == 0; }

// Non-weight src0 (the F16 KV-cache attention matmuls KQ / KQV, llama.cpp:5329,5372) costs a
// host->device copy of the viewed cache on every call.  LAMM_HIP_VIEWS=0 leaves them to ggml's
// CPU loop (the reference's routing for F16), =1 always takes them; unset: taken from
// kViewMinRows activation rows (prefill), left to the CPU for decode.
constexpr int64_t kViewMinRows = 8;
bool views_accepted(const ggml::tensor* src0, const ggml::tensor* src1) {
  if (is_weight(src0)) return true;
  if (knobs().views >= 0) return knobs().views == 1;
  // (in the reference's order the views compute in ggml_vec_dot_f16's order: ref_f16_kernel)
  return src1->ne[1] >= kViewMinRows;
}

bool extra_types_enabled() { return knobs().extra_types; }

// The boundary computes in the reference's own x86 float order (lamm_ref.hip: the lamm opt-3 AVX2
// lanes; ggml's AVX2 q6_K) for every format that has that kernel, so llama.cpp through the hook
// produces the bits the reference's CPU build produces.  LAMM_HIP_ORDER=fast: the
// fast engines (exact block dots, another fp32 summation order).
bool boundary_ref_order(const ggml::tensor* src0) {
  return knobs().ref_order && ref_order_supported(src0->type, vec_dot_type(src0->type));
}

// How an F32 src1 reaches the kernels (ggml's INIT phase quantizes it on thread 0, serially:
// LC/ggml.c:10865-10887).  Whenever the GPU takes it over, the hook claims the INIT phase too
// (and does nothing in it) so ggml never quantizes; the INIT and COMPUTE answers come from the
// same function.
//   kCpuInit  : ggml's CPU INIT, as in the reference; COMPUTE uploads wdata
//   kFused    : decode-sized (N <= 8) weight matmuls on q8_0 / q8_1 activations: the GEMV
//               quantizes the F32 rows while staging them (AVX2 from_float flavour, bit-exact,
//               lamm_gemv*.hip) -- no quantizer launch, no CPU INIT
//   kGpuQuant : from 8 activation rows up: F32 rows up, lamm_hip_quantize (AVX2 flavour), then
//               the GEMM engines (profiles/r01/e2e_gpu_quant.txt: Q4_0 4096x512x4096 528 -> 376 us)
// LAMM_HIP_GPU_QUANT=0: always ggml's CPU INIT; =1: kGpuQuant for every row count.
// kFused is opt-in since round 5 (LAMM_HIP_FUSED=1): through llama.cpp's decode every one of the
// GEMV's 8 XCDs pulls the zero-copy F32 row (16 KiB) over PCIe into its own L2, where ggml's INIT
// leaves 4.25 KiB of q8_0 -- the boundary call 24.4 -> 20.3 us in the reference order, 20.7 ->
// 18.2 us in the fast order, tg +7 % (profiles/r05/decode_init/)
enum ActMode { kCpuInit, kFused, kGpuQuant };
ActMode act_mode(const ggml::tensor* src0, const ggml::tensor* src1) {
  const int vdt = vec_dot_type(src0->type);
  if (src1->type != kF32 || vdt == kF32) return kCpuInit;
  const bool f32_rows = src1->nb[0] == sizeof(float) && (src1->nb[1] & 3) == 0 && (src1->nb[2] & 3) == 0 &&
                        (src1->nb[3] & 3) == 0;
  if (!f32_rows) return kCpuInit;
  const int gq = knobs().gpu_quant;
  if (gq == 0) return kCpuInit;
  // in the reference's order only the one-column kernel (ref_gemv_kernel) quantizes in its staging;
  // 2 .. 7 rows take ggml's own INIT, 8 and more the GPU quantizer (the same AVX2-flavour bytes)
  const bool ref_fused = src1->ne[1] == 1 && src1->ne[2] * src1->ne[3] == 1 && src0->ne[0] / 32 <= 576;
  if (knobs().fused && gq != 1 && (vdt == kQ8_0 || vdt == kQ8_1) && src1->ne[1] <= 8 && is_weight(src0) &&
      (!boundary_ref_order(src0) || ref_fused))
    return kFused;
  const int64_t rows = src1->ne[1] * src1->ne[2] * src1->ne[3];
  if (gq != 1 && rows < 8) return kCpuInit;
  return (vdt == kQ8_0 || vdt == kQ8_1 || vdt == kQ8_K || vdt == kF16) ? kGpuQuant : kCpuInit;
}

}  // namespace

extern "C" int lamm_get_opt_level(void) { return probe().count ? (opt_level() > 0 ? 3 : 0) : 0; }

extern "C" bool lamm_can_mul_mat(const struct ggml_compute_params* vparams, const struct ggml_tensor* vdst) {
  const auto* params = reinterpret_cast<const ggml::compute_params*>(vparams);
  const auto* dst = reinterpret_cast<const ggml::tensor*>(vdst);
  if (opt_level() == 0) return false;                       // :12-14
  const ggml::tensor* src0 = dst->src[0];
  const ggml::tensor* src1 = dst->src[1];
  if (!src0 || !src1) return false;
  // :15-17: INIT belongs to ggml (it quantizes src1) unless the GPU quantizes it; the INIT
  // and COMPUTE answers must agree, so INIT re-runs every COMPUTE check below
  if (params->type == ggml::TASK_INIT) {
    if (act_mode(src0, src1) == kCpuInit) return false;
  } else if (params->type != ggml::TASK_COMPUTE) {
    return false;
  }
  const int vdt = vec_dot_type(src0->type);
  if (vdt < 0) return false;                                 // :37-52 supported pairs
  // q4_K / q5_K / q6_K / f16 are beyond the reference's lamm set (a Q4_0
  // model's Q6_K output.weight, the F16 KV-cache attention matmuls);
  // LAMM_HIP_EXTRA_TYPES=0 restores the reference's exact set
  if ((src0->type == kQ4_K || src0->type == kQ5_K || src0->type == kQ6_K || src0->type == kF16) &&
      !extra_types_enabled())
    return false;
  if (src1->type == vdt && !is_contiguous(src1)) return false;  // :23-28
  if (src1->nb[0] != block_bytes(src1->type)) return false;  // :29-31
  if (dst->type != kF32) return false;                       // :34-36
  if (src1->type != vdt && src1->type != kF32) return false; // wdata holds vdt rows
  if (src0->ne[0] % block_elems(src0->type)) return false;
  if (src0->nb[0] != block_bytes(src0->type)) return false;
  if (dst->nb[0] != sizeof(float)) return false;
  if (!views_accepted(src0, src1)) return false;
  return probe().count > 0;                                  // no GPU: ggml's CPU loop
}

namespace {

// Wait for everything queued on d's stream: a completion flag the GPU writes (lamm_signal.hip),
// spun on by the host -- ~4 us per call under hipStreamSynchronize.  If the flag has not arrived
// after a second (a fault, a hang) the stream is synchronised, which reports the error.
// LAMM_HIP_SPIN=0: hipStreamSynchronize only (A/B).
bool spin_enabled() { return knobs().spin; }

// LAMM_HIP_KERNEL_SIGNAL=1: the GEMV's last workgroup writes the completion flag itself instead
// of a signal launch behind it.  Measured no faster through llama.cpp (profiles/r02/
// ab_kernel_signal.txt: device wait 15.8 vs 15.1 us per decode call) -- the last workgroup's
// counter round trip and system fence cost what the second launch costs -- so it is an A/B switch.
bool kernel_signal_enabled() { return knobs().kernel_signal; }

void wait_device(Dev& d) {
  if (spin_enabled()) {
    // with LAMM_HIP_KERNEL_SIGNAL=1 the call's GEMV signals completion itself when it can
    // (Completion: zero-copy C with nothing queued behind it)
    unsigned seq = d.pending;
    d.pending = 0;
    if (!seq) {
      seq = ++d.seq;
      // LAMM_HIP_SIGNAL_WRITE=1 (A/B): HIP's stream write-value op instead of the one-lane kernel
      if (knobs().signal_write) HIPCHK(hipStreamWriteValue32(d.stream, d.flag_dev, seq, 0));
      else HIPCHK(launch_signal(d.flag_dev, seq, d.stream));
    }
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
      if (*(volatile unsigned*)d.flag == seq) return;
      if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) break;
      __builtin_ia32_pause();
    }
  }
  HIPCHK(hipStreamSynchronize(d.stream));
}

// Completion from C itself (LAMM_HIP_C_WATCH=1: coherent C, =2: non-coherent C, visible at the end-
// of-kernel release; default 0: the signal launch): a decode-sized call whose C goes straight into
// pinned host memory fills that C with a sentinel before the launch and spins until every word has
// been overwritten -- no signal launch behind the matmul.  In llama.cpp's decode the one-lane signal
// kernel shows 3.9 us of device time per call in the trace, but the boundary call measured the same
// with either form (18.4-20.3 us, three alternating runs, profiles/r05/decode_init/): the flag lands
// as soon as C does, so the signal is an A/B switch, not the default.  The sentinel is a
// signalling NaN: every C word is the result of a float add (the kernels' final reduction), and
// arithmetic never returns a signalling NaN, so no computed value can look unwritten.  Every word
// is written exactly once, after the workgroup's reads of A and B (C depends on them), so the
// activation buffer is free again when the last word lands.  After a second without progress the
// stream is synchronised (which reports a fault) and C must then be complete.
constexpr uint32_t kCSentinel = 0x7f80a5a5u;   // exponent all ones, quiet bit 0, payload != 0

void watch_c(Dev& d, const unsigned char* c, size_t words) {
  const uint32_t* w = reinterpret_cast<const uint32_t*>(c);
  const auto t0 = std::chrono::steady_clock::now();
  size_t i = 0;
  for (unsigned it = 0; i < words; ++it) {
    if (__atomic_load_n(&w[i], __ATOMIC_ACQUIRE) != kCSentinel) {
      ++i;
      continue;
    }
    if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(1)) {
      HIPCHK(hipStreamSynchronize(d.stream));
      for (; i < words; ++i)
        if (__atomic_load_n(&w[i], __ATOMIC_ACQUIRE) == kCSentinel) {
          fprintf(stderr, "lamm_hip: C word %zu of %zu was never written\n", i, words);
          std::abort();
        }
      return;
    }
    __builtin_ia32_pause();
  }
}

// Decode-sized calls read their activations from, and write C to, pinned host memory mapped into
// the device (tools/lat_probe.hip: every HIP copy op costs the host ~5 us to enqueue and the
// round trip ~2.5 us, against a 10 us floor for one launch + synchronise): one launch + one
// synchronise per call, host memcpys either side.  LAMM_HIP_ZERO_COPY=0 restores device copies.
constexpr size_t kZeroCopyMax = (size_t)256 << 10;
// LAMM_HIP_ZERO_COPY: "both" (default) / "in" / "out" / "0": which direction is read / written
// in place.  llama.cpp decode through the boundary (tools/ab_zero_copy.sh,
// profiles/r02/ab_zero_copy.txt, p=32 tg, -t 8): device copies 66 tok/s (34.5 us per matmul
// call: the D2H into ggml's pageable dst blocks), in only 72, out only 74, both 89 (24.4 us).
bool zero_copy(size_t bytes, bool in) { return (knobs().zero_copy & (in ? 1 : 2)) && bytes <= kZeroCopyMax; }

// ggml's pool threads other than 0 have nothing to do in a claimed COMPUTE phase.  Returning at once
// (the default) parks them in ggml's node barrier, which spins without yielding
// (LC/ggml.c:18440-18447, ggml_graph_compute_thread_sync_task(.., false)); LAMM_HIP_HELPERS=1 / 2
// keeps them here instead, yielding / asleep on a futex, until thread 0 publishes the node as done,
// so a pool as wide as the cores leaves the CPU to thread 0 and the HIP runtime.  A helper never
// waits more than 20 ms (a node thread 0 does not compute -- none exists -- cannot hang the pool).
std::atomic<const void*> g_node_done{nullptr};
std::atomic<uint32_t> g_node_gen{0};

void helper_wait(const void* dst, int mode) {
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    const uint32_t gen = g_node_gen.load(std::memory_order_acquire);
    if (g_node_done.load(std::memory_order_acquire) == dst) return;
    if ((i & 15) == 15 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(20)) return;
    if (mode == 2) {
      const timespec ts{0, 200000};   // re-check at least every 0.2 ms
      syscall(SYS_futex, reinterpret_cast<uint32_t*>(&g_node_gen), FUTEX_WAIT_PRIVATE, gen, &ts, nullptr, 0);
    } else {
      sched_yield();
    }
  }
}

// Prefill-sized calls put ggml's other pool threads to work (LAMM_HIP_POOL): they enter the same
// COMPUTE call as thread 0 (LC/ggml.c:18404-18421), wait here instead of spinning in ggml's
// barrier, and claim chunks of the row jobs thread 0 posts -- bit 1: quantize the F32 activation
// rows to q8_0 / q8_1 in pinned memory (lamm_host_quant.cpp, the bytes ggml's AVX2 INIT and the
// device quantizer write), so 2.2 MiB cross PCIe instead of 8 MiB of F32 (pageable: ~400 us per
// 4096 x 512 call); bit 2: C down into pinned memory and scattered into dst by the pool (measured
// slower than HIP's pageable download, profiles/r04/e2e_pool/: off).  Every thread decides from
// the call's shapes alone (pool_call) whether the node is a pool node; a helper that arrives after
// thread 0 has finished (or never sees it start within 2 s) returns, and thread 0 runs every chunk
// nobody claimed -- the jobs are complete whoever does them.
struct RowJob {   // rows r = (i3 * n2 + i2) * n1 + j: dst + off(r, d*) <- src + off(r, s*)
  const unsigned char* src = nullptr;
  unsigned char* dst = nullptr;
  size_t bytes = 0, s1 = 0, s2 = 0, s3 = 0, d1 = 0, d2 = 0, d3 = 0;   // bytes: per row (a copy)
  int64_t n1 = 1, n2 = 1, rows = 0, per_chunk = 1;
  int qtype = -1;        // >= 0: quantize each F32 row to nblk blocks of qtype instead of copying
  int64_t nblk = 0;
};
RowJob g_job;
std::atomic<uint64_t> g_ctl{0};             // job sequence (24 bits) | chunks (20) | next chunk (20)
std::atomic<int64_t> g_done{0};             // chunks of the current job completed
std::atomic<const void*> g_pool_dst{nullptr};
std::atomic<int> g_pool_finished{1};
std::atomic<const void*> g_pool_last{nullptr};   // the node whose last job has been posted
uint64_t g_pool_seq = 0;                    // thread 0's

void run_rows(const RowJob& jb, int64_t c) {
  const int64_t r1 = std::min(jb.rows, (c + 1) * jb.per_chunk);
  for (int64_t r = c * jb.per_chunk; r < r1; ++r) {
    const int64_t j = r % jb.n1, q = r / jb.n1, i2 = q % jb.n2, i3 = q / jb.n2;
    unsigned char* y = jb.dst + j * jb.d1 + i2 * jb.d2 + i3 * jb.d3;
    const unsigned char* x = jb.src + j * jb.s1 + i2 * jb.s2 + i3 * jb.s3;
    if (jb.qtype >= 0) host_quantize_row(jb.qtype, reinterpret_cast<const float*>(x), y, jb.nblk);
    else host_stream_copy(y, x, jb.bytes);
  }
}

void pool_work() {   // claim and run chunks of the posted job until none is left
  for (;;) {
    uint64_t v = g_ctl.load(std::memory_order_acquire);
    if ((v & 0xFFFFF) >= ((v >> 20) & 0xFFFFF)) return;
    if (!g_ctl.compare_exchange_weak(v, v + 1, std::memory_order_acq_rel)) continue;
    run_rows(g_job, (int64_t)(v & 0xFFFFF));   // g_job is rewritten only after every chunk is done
    g_done.fetch_add(1, std::memory_order_acq_rel);
  }
}

void pool_run(const RowJob& jb, int nth) {   // thread 0: post, take part, wait for the stragglers
  if (jb.rows <= 0) return;
  RowJob j = jb;
  const int64_t want = std::max<int64_t>(1, std::min<int64_t>(((int64_t)256 << 10) / (int64_t)std::max<size_t>(jb.bytes, 1),
                                                              jb.rows / (2 * (int64_t)nth)));
  j.per_chunk = std::max<int64_t>(want, (jb.rows + 0xFFFFE) / 0xFFFFF);
  const uint64_t n = (uint64_t)((jb.rows + j.per_chunk - 1) / j.per_chunk);
  g_job = j;
  g_done.store(0, std::memory_order_relaxed);
  ++g_pool_seq;
  g_ctl.store(((g_pool_seq & 0xFFFFFF) << 40) | (n << 20), std::memory_order_release);
  pool_work();
  while ((uint64_t)g_done.load(std::memory_order_acquire) < n) __builtin_ia32_pause();
}

// sleep: once this call's last job is posted and claimed, wait asleep (futex) for thread 0 instead
// of spinning (LAMM_HIP_HELPERS=2, or 3: asleep here only, decode nodes as with 0)
void pool_help(const void* dst, bool sleep) {
  const auto t0 = std::chrono::steady_clock::now();
  for (unsigned it = 0;; ++it) {
    const uint32_t gen = g_node_gen.load(std::memory_order_acquire);
    if (g_pool_dst.load(std::memory_order_acquire) == dst) {
      if (g_pool_finished.load(std::memory_order_acquire)) return;
      pool_work();
      if (sleep && g_pool_last.load(std::memory_order_acquire) == dst) {
        const timespec ts{0, 500000};
        syscall(SYS_futex, reinterpret_cast<uint32_t*>(&g_node_gen), FUTEX_WAIT_PRIVATE, gen, &ts, nullptr, 0);
      }
    }
    if ((it & 1023) == 1023 && std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) return;
    __builtin_ia32_pause();
  }
}

// Whether a COMPUTE call is a pool node -- the same answer in every thread (shapes and knobs only).
constexpr size_t kPoolMin = (size_t)1 << 20;
// A pool node is one where thread 0 will post a job (every prefill-sized node used to
// be one, and on nodes with no job -- ggml's own INIT, q8_K / F16 activations -- the helpers spun in
// pool_help with LAMM_HIP_HELPERS' yield / sleep turned off): bit 1 with F32 rows the host
// quantizer takes (the hostq condition of mul_mat_thread0), or bit 2 (the C scatter).
bool pool_call(const ggml::compute_params* params, const ggml::tensor* dst) {
  if (!knobs().pool || params->nth < 2) return false;
  const ggml::tensor* src0 = dst->src[0];
  const ggml::tensor* src1 = dst->src[1];
  const int64_t rows = src1->ne[1] * src1->ne[2] * src1->ne[3];
  if (!(rows > 8 && (size_t)dst->ne[0] * rows * sizeof(float) >= kPoolMin)) return false;
  const int vdt = vec_dot_type(src0->type);
  const bool quant_job = (knobs().pool & 1) && src1->type != vdt && act_mode(src0, src1) == kGpuQuant &&
                         host_quant_supported(vdt);
  return quant_job || (knobs().pool & 2);
}

void mul_mat_thread0(const ggml::compute_params* params, ggml::tensor* dst, bool pool);

}  // namespace

extern "C" void lamm_mul_mat(const struct ggml_compute_params* vparams, struct ggml_tensor* vdst) {
  const auto* params = reinterpret_cast<const ggml::compute_params*>(vparams);
  auto* dst = reinterpret_cast<ggml::tensor*>(vdst);
  if (params->type != ggml::TASK_COMPUTE) return;  // INIT claimed for the GPU quantizer: nothing to do
  const bool pool = pool_call(params, dst);
  const int helpers = pool || knobs().helpers == 3 ? 0 : knobs().helpers;   // 3: asleep in pool nodes only
  if (params->ith != 0) {   // thread 0 owns the device work; ggml's barrier follows
    if (pool) pool_help(dst, knobs().helpers >= 2);
    else if (helpers > 0 && params->nth > 1) helper_wait(dst, helpers);
    return;
  }
  if (helpers > 0) g_node_done.store(nullptr, std::memory_order_release);
  if (pool) {
    g_pool_finished.store(0, std::memory_order_release);
    g_pool_last.store(nullptr, std::memory_order_release);
    g_pool_dst.store(dst, std::memory_order_release);
  }
  mul_mat_thread0(params, dst, pool);
  if (pool) {
    g_pool_finished.store(1, std::memory_order_release);
    if (knobs().helpers >= 2) {
      g_node_gen.fetch_add(1, std::memory_order_acq_rel);
      syscall(SYS_futex, reinterpret_cast<uint32_t*>(&g_node_gen), FUTEX_WAKE_PRIVATE, INT32_MAX, nullptr, nullptr, 0);
    }
  }
  if (helpers > 0) {
    g_node_done.store(dst, std::memory_order_release);
    g_node_gen.fetch_add(1, std::memory_order_acq_rel);
    if (helpers == 2) syscall(SYS_futex, reinterpret_cast<uint32_t*>(&g_node_gen), FUTEX_WAKE_PRIVATE, INT32_MAX, nullptr, nullptr, 0);
  }
}

namespace {

// Siblings (LAMM_HIP_SIBLINGS, default on): decode calls that multiply the SAME activation row by
// different weights -- llama.cpp's wq / wk / wv on the attention norm, ffn_gate / ffn_up on the
// ffn norm (LC/llama.cpp build_llama), each its own mul_mat node, each its own round trip through
// the hook.  The boundary learns such groups from what it sees (a call whose src1 has the same
// address and the same bytes as the group's first call joins it), and on the next token, when a
// group's first call arrives, it runs the learned siblings' GEMVs in the same device round trip
// (same activation buffer, results into pinned memory) and keeps the results.  A sibling's own
// call then takes its result only if its src1 has the bytes it was computed from (compared in
// full), its weight is the same cache entry with the same fingerprint, and the shape matches;
// anything else discards it and computes as usual.  The kernels are the ones the call would run
// (the same bits; tests/test_gpu_ggml_boundary.py::test_sibling_calls).
struct SibKey {
  WeightKey key;
  int64_t M = 0;
};
struct SibResult {
  WeightKey key{};                    // the sibling's weight (type, shape, strides)
  const void* x = nullptr;            // src1 data pointer the result was computed for
  std::vector<unsigned char> xbytes;  // and its bytes
  uint64_t fp = 0;                    // the weight's fingerprint at that time
  size_t slot = 0;                    // float offset into the sibling result buffer
  int64_t M = 0;
};
struct Siblings {
  // learning: the current group (first call's key, its src1 pointer and bytes)
  bool have_group = false;
  WeightKey leader{};
  const void* gx = nullptr;
  std::vector<unsigned char> gbytes;
  std::unordered_map<WeightKey, std::vector<SibKey>, WeightKeyHash> followers;
  std::unordered_map<const void*, SibResult> pending;   // by the sibling's src0 data pointer
  uint64_t launched = 0, taken = 0;                     // lamm_hip_sibling_stats
  void clear() {
    have_group = false;
    followers.clear();
    pending.clear();
  }
};
Siblings g_sib;
void print_sibling_stats() {
  if (g_sib.launched)
    fprintf(stderr, "lamm_hip stats: sibling GEMVs %llu run ahead, %llu taken\n", (unsigned long long)g_sib.launched,
            (unsigned long long)g_sib.taken);
}

void mul_mat_thread0(const ggml::compute_params* params, ggml::tensor* dst, bool pool) {

  const ggml::tensor* src0 = dst->src[0];
  const ggml::tensor* src1 = dst->src[1];
  const int t0 = src0->type, vdt = vec_dot_type(t0);
  const int64_t ne00 = src0->ne[0], ne01 = src0->ne[1], ne02 = src0->ne[2], ne03 = src0->ne[3];
  const int64_t ne11 = src1->ne[1], ne12 = src1->ne[2], ne13 = src1->ne[3];
  const int qk = block_elems(t0);
  const int64_t kb = ne00 / qk;                                 // K in blocks (A.col)
  const size_t a_row = (size_t)kb * block_bytes(t0);
  const size_t b_row = (size_t)kb * block_bytes(vdt);           // ggml_row_size(vdt, ne10)
  const bool use_wdata = src1->type != vdt;
  const ActMode act = use_wdata ? act_mode(src0, src1) : kCpuInit;
  const bool ref = boundary_ref_order(src0);
  const int64_t M = ne01, N = ne11, nslices = ne12 * ne13;

  Runtime& rt = Runtime::get();
  std::lock_guard<std::mutex> lock(rt.mu);
  rt.ensure_init();
  const bool weight = is_weight(src0);
  StatScope stat(stats_on() ? &g_stats[(weight ? 0 : 2) + (N > 8 ? 1 : 0)] : nullptr);
  // weights: rows split over the boundary's devices (one device: all rows); other src0
  // (KV-cache views, intermediates): uploaded afresh, on the first device
  const int G = weight ? (int)rt.devs.size() : 1;
  const uint64_t fp = weight ? weight_fingerprint(src0, a_row) : 0;
  // a one-row decode call on one device with ggml's INIT (the form siblings are computed in)
  const bool sib_form = knobs().siblings && weight && G == 1 && N == 1 && nslices == 1 && use_wdata &&
                        act == kCpuInit && src1->type == kF32 && src1->nb[0] == sizeof(float) && params->wdata;
  const WeightKey wkey{src0->data, t0, M * ne02 * ne03, kb, src0->nb[1], src0->nb[2], src0->nb[3]};
  const size_t xb = (size_t)ne00 * sizeof(float);
  if (sib_form) {
    auto it = g_sib.pending.find(src0->data);
    if (it != g_sib.pending.end()) {
      const SibResult r = std::move(it->second);
      g_sib.pending.erase(it);
      if (r.key == wkey && r.x == src1->data && r.fp == fp && r.M == M && r.xbytes.size() == xb &&
          memcmp(r.xbytes.data(), src1->data, xb) == 0) {
        memcpy(dst->data, reinterpret_cast<const float*>(rt.pinned(3, 0)) + r.slot, (size_t)M * sizeof(float));
        ++g_sib.taken;
        return;
      }
    }
    // learning: does this call join the current group?
    if (g_sib.have_group && src1->data == g_sib.gx && !(wkey == g_sib.leader) && g_sib.gbytes.size() == xb &&
        memcmp(g_sib.gbytes.data(), src1->data, xb) == 0) {
      auto& f = g_sib.followers[g_sib.leader];
      bool known = false;
      for (const SibKey& k : f) known |= k.key == wkey;
      if (!known && f.size() < 4) f.push_back(SibKey{wkey, M});
    } else {
      g_sib.have_group = true;
      g_sib.leader = wkey;
      g_sib.gx = src1->data;
      g_sib.gbytes.assign(static_cast<const unsigned char*>(src1->data), static_cast<const unsigned char*>(src1->data) + xb);
    }
  }
  // activation bytes as the kernels read them: F32 rows (kFused, kGpuQuant; packed [slice][N][K])
  // or vec_dot_type rows (wdata / a vec_dot-typed src1)
  const int64_t ldx = (ne00 + 3) & ~int64_t(3);                 // the quantizer reads rows as float4
  // prefill q8_0 / q8_1 activations quantized by ggml's pool threads (LAMM_HIP_POOL bit 1): the
  // kernels then read vdt rows, as after ggml's own INIT
  const bool hostq = pool && (knobs().pool & 1) && act == kGpuQuant && host_quant_supported(vdt);
  const size_t x_row = act == kCpuInit || hostq ? b_row : (size_t)ldx * sizeof(float);
  const size_t x_bytes = x_row * (size_t)(N * nslices);
  const size_t c_bytes = (size_t)M * N * nslices * sizeof(float);
  // zero copy on several devices (LAMM_HIP_ZERO_COPY_SPLIT=1): every device reads the one pinned
  // activation buffer and writes its own rows of the one pinned C (mapped pinned memory has one
  // address on every device).  Off by default: it has only run with one GPU listed several times,
  // and with N > 1 and M not a multiple of 16 two devices' rows of C can share a host cache line
  const bool zc_split = G == 1 || knobs().zero_copy_split;
  const bool zc_in = zc_split && zero_copy(x_bytes, true) && act != kGpuQuant && (G == 1 || rt.pinned_shared(0, x_bytes));
  const bool zc_out = zc_split && zero_copy(c_bytes, false) && (G == 1 || rt.pinned_shared(1, c_bytes));
  const unsigned char* x_host = nullptr;   // the bytes every device uploads (or reads in place)
  // LAMM_HIP_POOL bit 4 (default on): a reference-order prefill call on one device runs as two column chunks on
  // two streams -- the pool quantizes chunk 2 while chunk 1 uploads and multiplies, and chunk 1's C
  // comes down while chunk 2 multiplies (the reference-order kernels compute every output in the
  // same order whatever the chunking: the same bits)
  const bool pipe = hostq && ref && weight && G == 1 && nslices == 1 && !zc_out && (knobs().pool & 4) &&
                    !(knobs().pool & 2) && N >= 64 && dst->nb[1] == (size_t)M * sizeof(float);
  const bool c_pool = pool && (knobs().pool & 2) && !zc_out && G == 1;   // C: pinned + the pool's scatter
  // completion from C's own words (watch_c): one device, C zero-copy, decode-sized
  const bool watch = zc_out && G == 1 && N <= 8 && spin_enabled() && knobs().c_watch;
  // LAMM_HIP_DIRECT=1: decode-sized, everything in place in pinned memory, one device -- the GEMV
  // goes onto the library's own AQL queue (lamm_aql.cpp), its completion signal replaces the signal
  // launch.  Off by default: through llama.cpp's decode it measured 22.5-23 us per call against
  // 20.3-21.1 through HIP (the host's launch cost drops 3 -> 0.6 us, the device wait grows by more;
  // profiles/r05/direct/)
  const bool direct = G == 1 && zc_in && zc_out && N <= 8 && act != kGpuQuant && spin_enabled() && knobs().direct &&
                      !kernel_signal_enabled() && !watch;
  bool in_direct = false;
  auto gather_f32 = [&](unsigned char* out) {   // F32 src1 rows (any strides) -> [slice][N][ldx]
    for (int64_t i13 = 0; i13 < ne13; ++i13)
      for (int64_t i12 = 0; i12 < ne12; ++i12)
        for (int64_t j = 0; j < N; ++j)
          memcpy(out + ((i13 * ne12 + i12) * N + j) * x_row,
                 static_cast<const unsigned char*>(src1->data) + i12 * src1->nb[2] + i13 * src1->nb[3] + j * src1->nb[1],
                 (size_t)ne00 * sizeof(float));
  };
  // one device: the decode activations go straight into device memory through the BAR (a kernel
  // read them zero-copy from pinned host memory before, every XCD pulling them over PCIe;
  // LAMM_HIP_VRAM_X=0 restores that)
  unsigned char* xv = zc_in && G == 1 && knobs().vram_x ? rt.devs[0].vram_x(x_bytes) : nullptr;
  if (zc_in) {
    unsigned char* h = xv ? xv : rt.pinned(0, x_bytes);
    if (act == kFused) gather_f32(h);
    else if (use_wdata) memcpy(h, params->wdata, x_bytes);
    else
      for (int64_t r = 0; r < N * nslices; ++r)
        memcpy(h + r * b_row, static_cast<const unsigned char*>(src1->data) + r * src1->nb[1], b_row);
    if (xv) lamm::hdp_flush(rt.devs[0].id, xv + ((x_bytes - 4) & ~size_t(3)));
    x_host = h;
  } else if (pipe) {
    Dev& d = rt.devs[0];
    HIPCHK(hipSetDevice(d.id));
    WeightEntry& w = rt.weights(d, WeightKey{src0->data, t0, M, kb, src0->nb[1], src0->nb[2], src0->nb[3]}, a_row, src0,
                                0, M, fp);
    // a cold weight's upload was enqueued on d.stream: chunk 2's kernel on stream2 must not start
    // before it lands (a pageable H2D copy may still be in flight when hipMemcpy2DAsync returns)
    HIPCHK(hipEventRecord(d.upload, d.stream));
    HIPCHK(hipStreamWaitEvent(d.stream2, d.upload, 0));
    stat.phase(1);
    unsigned char* h = rt.pinned(2, x_bytes);
    unsigned char* dB = static_cast<unsigned char*>(d.scratch(0, x_bytes + 64));
    float* dC = static_cast<float*>(d.scratch(1, c_bytes + 64));
    const int64_t per = ((N + 1) / 2 + 31) / 32 * 32;   // column chunks, whole 32-column tiles
    const hipStream_t ss[2] = {d.stream, d.stream2};
    const lamm_matrix A{w.dev, t0, (int)M, (int)kb, w.dev_pitch / (int64_t)block_bytes(t0)};
    for (int c = 0; c < 2; ++c) {
      const int64_t n0 = c * per, nc = std::min<int64_t>(per, N - n0);
      if (nc <= 0) break;
      RowJob jb;
      jb.src = static_cast<const unsigned char*>(src1->data) + n0 * src1->nb[1];
      jb.dst = h + n0 * b_row;
      jb.qtype = vdt, jb.nblk = kb;
      jb.bytes = (size_t)ne00 * sizeof(float);
      jb.s1 = src1->nb[1], jb.d1 = b_row;
      jb.n1 = nc, jb.rows = nc;
      if (n0 + nc >= N) g_pool_last.store(dst, std::memory_order_release);
      pool_run(jb, params->nth);
      HIPCHK(hipMemcpyAsync(dB + n0 * b_row, jb.dst, (size_t)nc * b_row, hipMemcpyHostToDevice, ss[c]));
      const lamm_matrix B{dB + n0 * b_row, vdt, (int)kb, (int)nc, (int64_t)kb};
      const lamm_matrix C{dC + n0 * M, kF32, (int)M, (int)nc, M};
      const int rc = lamm_hip_matmul_ex(&A, &B, &C, nullptr, LAMM_ORDER_REFERENCE, ss[c]);
      if (rc != LAMM_OK) {
        fprintf(stderr, "lamm_hip: lamm_hip_matmul_ex failed (%d): %s\n", rc, g_err.c_str());
        std::abort();
      }
    }
    stat.phase(3);
    for (int c = 0; c < 2; ++c) {
      const int64_t n0 = c * per, nc = std::min<int64_t>(per, N - n0);
      if (nc <= 0) break;
      HIPCHK(hipMemcpyAsync(static_cast<unsigned char*>(dst->data) + n0 * dst->nb[1], dC + n0 * M,
                            (size_t)nc * M * sizeof(float), hipMemcpyDeviceToHost, ss[c]));
    }
    stat.phase(4);
    HIPCHK(hipStreamSynchronize(d.stream2));
    wait_device(d);
    stat.phase(5);
    return;
  } else if (hostq) {   // the pool quantizes the F32 rows -> pinned [slice][N] vdt rows
    unsigned char* h = rt.pinned(2, x_bytes);
    RowJob jb;
    jb.src = static_cast<const unsigned char*>(src1->data);
    jb.dst = h;
    jb.qtype = vdt, jb.nblk = kb;
    jb.bytes = (size_t)ne00 * sizeof(float);
    jb.s1 = src1->nb[1], jb.s2 = src1->nb[2], jb.s3 = src1->nb[3];
    jb.d1 = b_row, jb.d2 = b_row * (size_t)N, jb.d3 = b_row * (size_t)(N * ne12);
    jb.n1 = N, jb.n2 = ne12, jb.rows = N * nslices;
    if (!c_pool) g_pool_last.store(dst, std::memory_order_release);   // no C job follows
    pool_run(jb, params->nth);
    x_host = h;
  } else if (act == kCpuInit && use_wdata) {
    x_host = static_cast<const unsigned char*>(params->wdata);
    if (use_pinned(x_bytes)) {
      unsigned char* h = rt.pinned(0, x_bytes);
      memcpy(h, params->wdata, x_bytes);
      x_host = h;
    }
  }
  stat.phase(0);

  for (int g = 0; g < G; ++g) {
    Dev& d = rt.devs[g];
    HIPCHK(hipSetDevice(d.id));
    hipStream_t s = d.stream;
    int64_t r0 = 0, rows = M;
    if (G > 1) lamm_hip_shard_rows(M, G, g, 16, &r0, &rows);
    if (rows == 0) continue;
    WeightEntry* w = nullptr;
    void* a_dev;
    int64_t a_pitch;
    size_t a_s2, a_s3;
    if (weight) {
      w = &rt.weights(d, WeightKey{src0->data, t0, rows * ne02 * ne03, kb, src0->nb[1], src0->nb[2], src0->nb[3]}, a_row,
                      src0, r0, rows, fp);
      a_dev = w->dev;
      a_pitch = w->dev_pitch;
      a_s2 = (size_t)a_pitch * rows;
      a_s3 = a_s2 * ne02;
    } else {
      const Transient tr = upload_transient(d, src0, a_row);
      a_dev = tr.dev;
      a_pitch = tr.pitch;
      a_s2 = tr.s2;
      a_s3 = tr.s3;
    }
    stat.phase(1);
    // activations on (or mapped into) the device
    void* dB;
    if (zc_in) {
      dB = xv ? static_cast<void*>(xv) : rt.pinned_dev(0);
    } else if (hostq) {   // the pool's q8 rows
      dB = d.scratch(0, x_bytes + 64);
      HIPCHK(hipMemcpyAsync(dB, x_host, x_bytes, hipMemcpyHostToDevice, s));
      if (knobs().stats_sync) HIPCHK(hipStreamSynchronize(s));
      stat.phase(2);
    } else if (act == kFused || act == kGpuQuant) {
      float* dX = static_cast<float*>(d.scratch(2, x_bytes + 64));
      const bool dense = ldx == ne00 && src1->nb[1] == (size_t)ne00 * sizeof(float) &&
                         src1->nb[2] == src1->nb[1] * (size_t)N && src1->nb[3] == src1->nb[2] * (size_t)ne12;
      if (dense) {   // one linear copy (HIP's 2D path moves pageable rows one by one)
        HIPCHK(hipMemcpyAsync(dX, src1->data, x_bytes, hipMemcpyHostToDevice, s));
      } else {
        for (int64_t i13 = 0; i13 < ne13; ++i13)
          for (int64_t i12 = 0; i12 < ne12; ++i12) {
            const unsigned char* x =
                static_cast<const unsigned char*>(src1->data) + i12 * src1->nb[2] + i13 * src1->nb[3];
            HIPCHK(hipMemcpy2DAsync(dX + (i13 * ne12 + i12) * N * ldx, (size_t)ldx * sizeof(float), x, src1->nb[1],
                                    (size_t)ne00 * sizeof(float), (size_t)N, hipMemcpyHostToDevice, s));
          }
      }
      stat.phase(2);
      dB = dX;
      // q8_0 / q8_1 activations are quantized by the library inside the kernels that read them;
      // q8_K / f16 ones here
      if (act == kGpuQuant && (ref || (vdt != kQ8_0 && vdt != kQ8_1))) {
        void* dq = d.scratch(0, b_row * (size_t)(N * nslices) + 64);
        const int qrc = lamm_hip_quantize(vdt, /*AVX2 flavour*/ 1, dX, ldx, dq, kb, (int)ne00, (int)(N * nslices), s);
        if (qrc != LAMM_OK) {
          fprintf(stderr, "lamm_hip: lamm_hip_quantize failed (%d): %s\n", qrc, g_err.c_str());
          std::abort();
        }
        dB = dq;
      }
    } else if (use_wdata) {
      dB = d.scratch(0, x_bytes + 64);
      HIPCHK(hipMemcpyAsync(dB, x_host, x_bytes, hipMemcpyHostToDevice, s));
    } else {
      dB = d.scratch(0, x_bytes + 64);
      HIPCHK(hipMemcpy2DAsync(dB, b_row, src1->data, src1->nb[1], b_row, (size_t)(N * nslices), hipMemcpyHostToDevice,
                              s));
    }
    const bool b_f32 = act == kFused || (act == kGpuQuant && !hostq && !ref && (vdt == kQ8_0 || vdt == kQ8_1));
    const size_t b_pitch = b_f32 ? x_row : b_row;
    // C: zero-copy = this device's rows [r0, r0 + rows) of the pinned [slice][N][M] image; else a
    // dense [slice][N][rows] scratch copied into dst below
    const int64_t ldc = zc_out ? M : rows;
    const size_t c_slice = (size_t)ldc * N * sizeof(float);
    float* dC = zc_out ? static_cast<float*>((rt.pinned(1, c_bytes), rt.pinned_dev(1))) + r0
                       : static_cast<float*>(d.scratch(1, c_slice * (size_t)nslices + 64));

    lamm_matrix A{a_dev, t0, (int)rows, (int)kb, a_pitch / (int64_t)block_bytes(t0)};
    lamm_matrix B = b_f32 ? lamm_matrix{dB, kF32, (int)ne00, (int)N, ldx} : lamm_matrix{dB, vdt, (int)kb, (int)N, (int64_t)kb};
    lamm_matrix C{dC, kF32, (int)rows, (int)N, ldc};
    lamm_batch bt{ne02, ne03, ne12, ne13, a_s2, a_s3,
                  b_pitch * (size_t)N, b_pitch * (size_t)(N * ne12), c_slice, c_slice * (size_t)ne12};
    // prefill calls on the fp6 / super-block engines reuse the weights' packed form
    GemvArgs pa = weight_args(&A, ne02, ne03, bt.nba2, bt.nba3);
    pa.N = (int)N;
    pa.ne12 = (int)ne12;
    pa.ne13 = (int)ne13;
    pa.r2 = (int)(ne12 / ne02);
    pa.r3 = (int)(ne13 / ne03);
    const bool stationary = !ref && weight && N > gemv_max_n(t0) && (!b_f32 || N > 8) &&
                            ((gemm_fp6_supported(t0) && gemm_path(pa, true) == 0) ||
                             (gemm_kq_supported(t0) && knobs().kq_gemm));
    if (direct) {   // the direct queue runs beside d.stream: nothing may still be in flight there
      if (d.enqueued) HIPCHK(hipStreamSynchronize(s));
      d.enqueued = false;
      in_direct = lamm::direct_begin(d.id);
    }
    if (watch) {   // the sentinel in every word of C before the launch (watch_c)
      uint32_t* hc = reinterpret_cast<uint32_t*>(rt.pinned(1, c_bytes));
      std::fill(hc, hc + c_bytes / sizeof(float), kCSentinel);
    }
    Completion comp{d.done_ctr, d.flag_dev, 0, false};
    if (zc_out && spin_enabled() && kernel_signal_enabled() && !watch) {   // nothing is queued behind the matmul
      comp.seq = ++d.seq;
      g_completion = &comp;
    }
    // this call leads a learned group: its siblings' GEMVs on the same activation buffer, in the
    // same launch (lamm_hip_matmul_group) -- their results wait in pinned memory for their own calls
    lamm_matrix gA[LAMM_GROUP_MAX], gC[LAMM_GROUP_MAX];
    int ng = 0;
    if (sib_form && !in_direct && !stationary && comp.seq == 0 && zc_out && !watch) {
      // (not with a C watch: watch_c returns once the LEADER's words land, while the group's other
      // segments may still read the activations and write their pinned results -- ADVICE r5)
      auto fit = g_sib.followers.find(wkey);
      if (fit != g_sib.followers.end() && !fit->second.empty()) {
        size_t total = 0;
        for (const SibKey& f : fit->second) total += (size_t)f.M;
        g_sib.pending.clear();   // earlier results live in the buffer about to be rewritten (or regrown)
        rt.pinned(3, total * sizeof(float));
        float* dres = static_cast<float*>(rt.pinned_dev(3));
        gA[0] = A;
        gC[0] = C;
        ng = 1;
        size_t off = 0;
        for (const SibKey& f : fit->second) {
          auto ce = d.cache.find(f.key);
          if (ce == d.cache.end() || f.key.type != t0 || f.key.kb != kb || ng == LAMM_GROUP_MAX) continue;
          const WeightEntry& we = ce->second;
          gA[ng] = lamm_matrix{we.dev, t0, (int)f.M, (int)kb, we.dev_pitch / (int64_t)block_bytes(t0)};
          gC[ng] = lamm_matrix{dres + off, kF32, (int)f.M, 1, f.M};
          ++ng;
          SibResult r;
          r.key = f.key;
          r.x = src1->data;
          r.xbytes.assign(static_cast<const unsigned char*>(src1->data), static_cast<const unsigned char*>(src1->data) + xb);
          r.fp = we.fingerprint;
          r.slot = off;
          r.M = f.M;
          g_sib.pending[f.key.host] = std::move(r);
          ++g_sib.launched;
          off += (size_t)f.M;
        }
      }
    }
    const int flags = ref ? LAMM_ORDER_REFERENCE : 0;
    const int rc = ng > 1      ? lamm_hip_matmul_group(gA, ng, &B, gC, flags, s)
                   : stationary ? lamm_hip_matmul_weights(rt.prepared(d, *w, A, ne02, ne03), &B, &C, &bt, s)
                                : lamm_hip_matmul_ex(&A, &B, &C, &bt, flags, s);
    g_completion = nullptr;
    d.pending = comp.signaled ? comp.seq : 0;
    if (rc != LAMM_OK) {
      fprintf(stderr, "lamm_hip: lamm_hip_matmul_batched failed (%d): %s\n", rc, g_err.c_str());
      std::abort();
    }
    stat.phase(3);
    if (c_pool) {   // C down into pinned memory; the pool scatters it into dst below
      HIPCHK(hipMemcpyAsync(rt.pinned(1, c_bytes), dC, c_bytes, hipMemcpyDeviceToHost, s));
    } else if (!zc_out) {   // this device's rows straight into dst
      const bool dense = rows == M && dst->nb[1] == (size_t)M * sizeof(float) &&
                         dst->nb[2] == dst->nb[1] * (size_t)N && dst->nb[3] == dst->nb[2] * (size_t)ne12;
      if (dense) {
        HIPCHK(hipMemcpyAsync(dst->data, dC, c_bytes, hipMemcpyDeviceToHost, s));
      } else {
        for (int64_t i13 = 0; i13 < ne13; ++i13)
          for (int64_t i12 = 0; i12 < ne12; ++i12) {
            unsigned char* c_host =
                static_cast<unsigned char*>(dst->data) + i12 * dst->nb[2] + i13 * dst->nb[3] + r0 * sizeof(float);
            HIPCHK(hipMemcpy2DAsync(c_host, dst->nb[1], dC + (i13 * ne12 + i12) * rows * N,
                                    (size_t)rows * sizeof(float), (size_t)rows * sizeof(float), N,
                                    hipMemcpyDeviceToHost, s));
          }
      }
    }
    stat.phase(4);
  }
  if (in_direct && lamm::direct_end() > 0) {
    // completed on the direct queue (direct_end waited for its completion signal)
  } else if (watch) {
    watch_c(rt.devs[0], rt.pinned(1, c_bytes), c_bytes / sizeof(float));
  } else {
    for (int g = 0; g < G; ++g) {
      HIPCHK(hipSetDevice(rt.devs[g].id));
      wait_device(rt.devs[g]);
    }
  }
  stat.phase(5);
  if (c_pool) {
    RowJob jb;
    jb.src = rt.pinned(1, c_bytes);
    jb.dst = static_cast<unsigned char*>(dst->data);
    jb.bytes = (size_t)M * sizeof(float);
    jb.s1 = jb.bytes, jb.s2 = jb.bytes * (size_t)N, jb.s3 = jb.s2 * (size_t)ne12;
    jb.d1 = dst->nb[1], jb.d2 = dst->nb[2], jb.d3 = dst->nb[3];
    jb.n1 = N, jb.n2 = ne12, jb.rows = N * nslices;
    g_pool_last.store(dst, std::memory_order_release);
    pool_run(jb, params->nth);
  } else if (zc_out) {
    const unsigned char* hC = rt.pinned(1, c_bytes);
    const size_t c_slice = (size_t)M * N * sizeof(float);
    for (int64_t i13 = 0; i13 < ne13; ++i13)
      for (int64_t i12 = 0; i12 < ne12; ++i12) {
        unsigned char* c_host = static_cast<unsigned char*>(dst->data) + i12 * dst->nb[2] + i13 * dst->nb[3];
        const unsigned char* src = hC + (size_t)(i13 * ne12 + i12) * c_slice;
        for (int64_t j = 0; j < N; ++j)
          memcpy(c_host + j * dst->nb[1], src + (size_t)j * M * sizeof(float), M * sizeof(float));
      }
  }
  stat.phase(6);
}

}  // namespace

extern "C" void lamm_hip_cache_clear(void) {
  Runtime& rt = Runtime::get();
  std::lock_guard<std::mutex> lock(rt.mu);
  rt.clear();
  g_sib.clear();
}

extern "C" void lamm_hip_boundary_reset(void) {
  Runtime& rt = Runtime::get();
  std::lock_guard<std::mutex> lock(rt.mu);
  rt.reset();
  g_sib.clear();
  reload_knobs();   // the next call sees the environment as it is now
}

extern "C" void lamm_hip_sibling_stats(uint64_t* launched, uint64_t* taken) {
  Runtime& rt = Runtime::get();
  std::lock_guard<std::mutex> lock(rt.mu);
  if (launched) *launched = g_sib.launched;
  if (taken) *taken = g_sib.taken;
}

extern "C" size_t lamm_hip_cache_bytes(void) {
  Runtime& rt = Runtime::get();
  std::lock_guard<std::mutex> lock(rt.mu);
  return rt.cached_bytes();
}
