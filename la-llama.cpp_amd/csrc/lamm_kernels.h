// lamm_kernels.h -- internal launch interface of the lamm HIP kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lamm {

// All strides in BYTES for A/B and in floats for C.  K in elements.
// Row i of A starts at A + i*lda; column j of B at B + j*ldb; C[j*ldc + i].
// Batch dims follow ggml's mul_mat (src/loongarch_matmul.cpp:130-142): slice
// (i12, i13) uses A slice (i12/r2, i13/r3), B slice (i12, i13), C slice (i12, i13);
// one launch covers all ne12*ne13 slices (blockIdx.y) instead of a host loop.
struct GemvArgs {
  const unsigned char* A; int64_t lda;
  const unsigned char* B; int64_t ldb;
  float* C; int64_t ldc;
  int M, N, K, nblk;
  int ne12 = 1, ne13 = 1, r2 = 1, r3 = 1;
  int64_t sa2 = 0, sa3 = 0, sb2 = 0, sb3 = 0;   // bytes
  int64_t sc2 = 0, sc3 = 0;                     // floats
  // GEMV only, q8_0 / q8_1 activations: B holds F32 rows (ldb in bytes) that the kernel
  // quantizes while staging them (ggml's INIT fused into the launch, AVX2 flavour, bit-exact)
  int b_f32 = 0;
  // completion signal (row-per-wave GEMV only, the ggml boundary's decode calls): the last
  // workgroup to finish stores seq into *flag (host-mapped) -- no separate signal launch
  unsigned* done_ctr = nullptr;   // device counter, zero between launches
  unsigned* flag = nullptr;
  unsigned seq = 0;
};

hipError_t launch_gemv(int type, const GemvArgs& p, hipStream_t s);
// lamm_hip_profile_next: HIP events the next decode-GEMV launch on this thread records its own
// start / end in (hipExtLaunchKernel: the dispatch's timestamps, what a kernel tracer reports);
// taking them clears them
struct LaunchTiming {
  hipEvent_t start = nullptr, stop = nullptr;
};
LaunchTiming take_launch_timing();
// row-per-wave decode GEMV (lamm_gemv_rpw.hip): 32-element block formats, N <= 2, K <= 12288;
// `waves` per workgroup (4 / 8 / 16; 8 at most for K > 4096)
bool gemv_rpw_supported(int type, const GemvArgs& p);
int rpw_waves(const GemvArgs& p);   // 0: the wave-group kernels (lamm_gemv.hip) take the call
hipError_t launch_gemv_rpw(int type, const GemvArgs& p, hipStream_t s, int waves);
// q2_K / q4_K / q5_K single-column decode GEMV (lamm_gemv_rpw.hip): one slice, K <= 12288, q8_K
// activations
bool gemv_kq_supported(int type, const GemvArgs& p);
hipError_t launch_gemv_kq(int type, const GemvArgs& p, hipStream_t s);
size_t gemv_lds_bytes(int type, int nc);
hipError_t launch_gemv_dense(int type, const GemvArgs& p, hipStream_t s);   // F32 / F16 rows
// q4_K / q5_K / q6_K prefill GEMM (lamm_gemm_kq.hip); B rows (q8_K) 4-byte aligned
hipError_t launch_gemm_kq(int type, const GemvArgs& p, const void* prepA, void* workspace, hipStream_t s);
bool gemm_kq_supported(int type);
size_t gemm_kq_workspace_bytes(int type, const GemvArgs& p, bool prepared);
size_t gemm_kq_weight_bytes(int type, const GemvArgs& p);
hipError_t prepare_kq_weights(int type, const GemvArgs& p, void* wsA, hipStream_t s);
// F32 / F16 prefill GEMM on the matrix cores (lamm_gemm_dense.hip); split-K partials in the
// workspace for grids under 256 tiles
hipError_t launch_gemm_dense(int type, const GemvArgs& p, void* workspace, hipStream_t s);
size_t gemm_dense_workspace_bytes(int type, const GemvArgs& p);
bool gemm_dense_supported(int type);
bool gemm_dense_args_ok(const GemvArgs& p);   // strides the 32-bit tile offsets reach

// C (slice z, row j, col i) = sum_{s < nsplit} part[s][z][j][i] in split order (deterministic)
void launch_splitk_reduce(const GemvArgs& p, int nsplit, const float* part, hipStream_t s);

// weight quantizers (lamm_quantize_w.hip): ggml_quantize_chunk's *_reference row quantizers
bool quantize_weights_supported(int type);
hipError_t launch_quantize_weights(int type, const float* x, int64_t ldx, void* y, int64_t ldy_bytes, int K, int M,
                                   hipStream_t s);

// hipFuncSetAttribute(kernel, MaxDynamicSharedMemorySize, bytes) once per (device, kernel) and
// size: a launch path that set it every call would pay the runtime call on every launch
void set_max_lds(const void* kernel, int bytes);

// completion flag (lamm_signal.hip): stores seq into *flag_dev after everything queued on s
hipError_t launch_signal(unsigned* flag_dev, unsigned seq, hipStream_t s);

// mul_mat in the reference's x86 float order, bit for bit (lamm_ref.hip): q4_0 / q5_0 x q8_0,
// q4_1 / q5_1 x q8_1, q6_K x q8_K; any N, batch slices.  One-column calls of the 32-element formats
// (ref_gemv_supported) also take F32 activation rows (p.b_f32: ggml's AVX2 INIT quantization in
// the kernel's staging), honour lamm_hip_profile_next and can signal their own completion (p.flag)
bool ref_order_supported(int type, int btype);
bool ref_gemv_supported(int type, const GemvArgs& p);
hipError_t launch_ref(int type, const GemvArgs& p, hipStream_t s);
// up to kRefSegs weights of one type and row length times the same activation column in one launch
// of ref_gemv_kernel's body (lamm_hip_matmul_group); entry 0 repeats p.A / p.C / p.M
constexpr int kRefSegs = 4;
struct RefSegs {
  const unsigned char* A[kRefSegs];
  float* C[kRefSegs];
  int M[kRefSegs];
};
hipError_t launch_ref_group(int type, const GemvArgs& p, const RefSegs& sg, int nseg, hipStream_t s);
// the same group in the fast engines' order (lamm_gemv_rpw.hip gemv_flat_group_kernel): one column,
// K = 4096, every weight >= 2048 rows -- the weights whose single calls run gemv_flat1_kernel, whose
// per-row arithmetic the group kernel repeats, so each C[i] has its single call's bits
bool gemv_group_supported(int type, const GemvArgs& p, const RefSegs& sg, int nseg);
hipError_t launch_gemv_group(int type, const GemvArgs& p, const RefSegs& sg, int nseg, hipStream_t s);

hipError_t launch_gemm(int type, const GemvArgs& p, void* workspace, hipStream_t s);
size_t gemm_workspace_bytes(int type, const GemvArgs& p);   // device scratch launch_gemm needs
bool gemm_supported(int type);
bool gemm_args_ok(int type, const GemvArgs& p);   // B pitch/alignment the GEMM staging needs

// q4_0 / q4_1 / q5_0 (and q5_1 with prepared weights) prefill GEMM on the block-scaled fp6
// matrix path (lamm_gemm_fp6.hip)
// prepA: the weights' packed form from prepare_fp6_weights (weight-stationary callers), or
// null to pack A into the workspace on every call
hipError_t launch_gemm_fp6(int type, const GemvArgs& p, const void* prepA, void* workspace, hipStream_t s);
size_t gemm_fp6_workspace_bytes(int type, const GemvArgs& p, bool prepared);
// packed weights: depends on M, K and the A slices (p.ne12/p.r2 x p.ne13/p.r3), not on N or B
size_t gemm_fp6_weight_bytes(int type, const GemvArgs& p);
// in_range (q5_1): false when a block scale is past what the packed form holds (use dq16)
hipError_t prepare_fp6_weights(int type, const GemvArgs& p, void* wsA, hipStream_t s, bool* in_range = nullptr);
bool gemm_fp6_supported(int type);   // q4_0 / q4_1 / q5_0 / q5_1 / q8_0 (q5_1, q8_0: prepared weights only)
// the call runs on the 128 x 64 K-group plan (gemm_fp6_kv_kernel) -- the only one q8_0's two weight
// code planes have
bool gemm_fp6_kv_plan(const GemvArgs& p);
int gemm_fp6_tiles(const GemvArgs& p);   // 256x128 output tiles of the fp6 GEMM (before K-splits)
int gemm_fp6_grid(const GemvArgs& p);    // its main-kernel workgroups (tiles x K-splits)

// q4_0 / q4_1 / q5_0 / q5_1 / q8_0 prefill GEMM on f16 MFMAs with the block scales folded into the
// operands as the raw blocks are unpacked (lamm_gemm_dq.hip): one launch, no workspace, 1e-3 bar
hipError_t launch_gemm_dq(int type, const GemvArgs& p, void* workspace, hipStream_t s);
size_t gemm_dq_workspace_bytes(const GemvArgs& p);   // 0: no workspace (the one-launch forms)
bool gemm_dq_supported(int type);
bool gemm_dq_args_ok(const GemvArgs& p);
int gemm_dq_tiles(const GemvArgs& p);   // its workgroups (128 x 64 output tiles over all slices)

// host side: ggml's AVX2 from_float for q8_0 / q8_1 activations (lamm_host_quant.cpp)
bool host_quant_supported(int type);
void host_quantize_row(int type, const float* x, void* y, int64_t nblk);
void host_stream_copy(void* dst, const void* src, size_t n);   // non-temporal stores (AVX2 hosts)

}  // namespace lamm
