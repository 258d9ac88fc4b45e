/*
 * lamm_hip.h -- C ABI of the MI355X (gfx950) lamm backend: liblamm_hip.so
 *
 * Two entry layers, both plain C (no HIP / torch types in any signature):
 *
 *  1. The ggml operator boundary -- a drop-in for the reference plug-in
 *     (AyiStar/la-llama.cpp src/loongarch_matmul.h:18-24), called from
 *     ggml_compute_forward_mul_mat under #ifdef LA_LLAMA
 *     (llama.cpp-b2430 ggml.c:10858-10863):
 *
 *        if (lamm_can_mul_mat(params, dst)) { lamm_mul_mat(params, dst); return; }
 *
 *     Same names, same argument meaning, same error behaviour: can_mul_mat returning
 *     false is the only "error" (ggml falls back to its own CPU loop); lamm_mul_mat
 *     aborts with a message on an internal failure (src/lamm_impl.hpp:100-103).
 *     The structs are ggml's (b2430 layout); they stay opaque here.
 *
 *  2. The plug-in operator API on DEVICE memory, mirroring the reference's internal
 *     interface LAMMImpl<T>::matmul(const Matrix &A, const Matrix &B, const Matrix &C)
 *     (src/lamm_impl.hpp:20, Matrix = src/lamm_common.h:87-93): same struct layout,
 *     same units (A.col = K in blocks, ld in elements of the matrix's own type,
 *     C element (i,j) at c[j*ldc + i]).  Runs asynchronously on `hip_stream`.
 */
#ifndef LAMM_HIP_H
#define LAMM_HIP_H

#include <stdbool.h>
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- 1. ggml boundary (replaces src/loongarch_matmul.h:18-24) ---------------- */
struct ggml_compute_params;
struct ggml_tensor;

/* Replaces src/loongarch_matmul.cpp:10-62.  False outside the COMPUTE phase, for
 * unsupported (src0, vec_dot_type) pairs, non-contiguous quantized src1, non-F32 dst,
 * LAMM_OPT_LEVEL=0 in the environment, or when no gfx950 device is present.
 * Accepts the reference's 7 pairs plus f16 / q4_K / q5_K / q6_K;
 * LAMM_HIP_EXTRA_TYPES=0 restricts it to the reference's exact set. */
bool lamm_can_mul_mat(const struct ggml_compute_params *params,
                      const struct ggml_tensor *dst);

/* Replaces src/loongarch_matmul.cpp:64-143.  Thread ith==0 of the ggml pool owns
 * the GPU work (weights cached device-resident, B uploaded, C downloaded into
 * dst with its strides, stream synchronised before return); other threads return
 * at once and meet thread 0 at ggml's post-COMPUTE barrier.  Computes all M rows
 * (the reference drops M % nth rows: SURVEY §8a defect 1). */
void lamm_mul_mat(const struct ggml_compute_params *params,
                  struct ggml_tensor *dst);

/* Replaces src/loongarch_matmul.cpp:145.  3 when the GPU path is active,
 * 0 when disabled by LAMM_OPT_LEVEL=0. */
int lamm_get_opt_level(void);

/* ---- 2. operator API on device memory ------------------------------------- */
typedef struct lamm_matrix {   /* == struct Matrix, src/lamm_common.h:87-93 */
  void *data;                  /* device pointer */
  int type;                    /* ggml_type id: 0 f32, 2 q4_0, 3 q4_1, 6 q5_0,
                                  7 q5_1, 8 q8_0, 9 q8_1, 10 q2_K, 15 q8_K;
                                  SURVEY §8f additions: 1 f16, 12 q4_K, 13 q5_K, 14 q6_K */
  int row;
  int col;
  int64_t ld;                  /* leading dimension, in blocks of `type` */
} lamm_matrix;

enum lamm_status {
  LAMM_OK = 0,
  LAMM_ERR_TYPE = 1,   /* unsupported (A.type, B.type, C.type) combination */
  LAMM_ERR_SHAPE = 2,  /* M/N/K or leading dimensions inconsistent */
  LAMM_ERR_ALIGN = 3,  /* A.data or A row pitch not 16-byte aligned */
  LAMM_ERR_HIP = 4,    /* HIP runtime error (see lamm_hip_last_error) */
  LAMM_ERR_NODEV = 5   /* no gfx950 device */
};

/* C[j*C.ld + i] = sum_k A[i,k] * B[k,j] for i < C.row (=A.row), j < C.col (=B.col).
 * A: weights (f32/q4_0/q4_1/q5_0/q5_1/q8_0/q2_K, + f16/q4_K/q5_K/q6_K), A.col = K/blck,
 *    A.ld >= A.col.
 * B: activations of type vec_dot_type(A.type) (f32/q8_0/q8_1/q8_K/f16), column j at
 *    B.data + j*B.ld blocks, B.row = A.col.  For A in q4_0/q4_1/q5_0/q5_1/q8_0 and
 *    B.col <= 8, B may instead be the F32 rows (B.row = K elements, B.ld in floats): the
 *    decode GEMV quantizes them while staging (ggml's INIT with the AVX2 from_float
 *    rounding), giving exactly the C of lamm_hip_quantize(.., flavour 1, ..) + matmul.
 * C: f32, C.ld >= C.row.   Returns a lamm_status.  Asynchronous on hip_stream.
 * Loads are range-checked per dword: A and B must be readable up to the next
 * 4-byte boundary past their last byte (always true for hipMalloc / torch memory). */
int lamm_hip_matmul(const lamm_matrix *A, const lamm_matrix *B, const lamm_matrix *C,
                    void *hip_stream);

/* Batched form: the reference's per-slice loop over ne12 x ne13 with broadcast
 * r2 = ne12/ne02, r3 = ne13/ne03 (src/loongarch_matmul.cpp:130-142) as ONE launch.
 * Slice (i12, i13) multiplies A slice (i12/r2, i13/r3) by B slice (i12, i13) into
 * C slice (i12, i13).  Strides are in bytes, like ggml's nb[2], nb[3].
 * lamm_hip_matmul(A, B, C, s) == lamm_hip_matmul_batched(A, B, C, NULL, s). */
typedef struct lamm_batch {
  int64_t ne02, ne03;          /* A slices */
  int64_t ne12, ne13;          /* B and C slices; multiples of ne02, ne03 */
  size_t nba2, nba3;           /* A slice strides (bytes, multiples of 16) */
  size_t nbb2, nbb3;           /* B slice strides (bytes) */
  size_t nbc2, nbc3;           /* C slice strides (bytes, multiples of 4) */
} lamm_batch;

int lamm_hip_matmul_batched(const lamm_matrix *A, const lamm_matrix *B, const lamm_matrix *C,
                            const lamm_batch *batch, void *hip_stream);

/* lamm_hip_matmul_batched with flags.  LAMM_ORDER_REFERENCE: compute every output in the
 * reference's own x86 float order -- the lamm opt-3 AVX2 kernels' eight fp32 FMA lanes per output
 * and reduce_sum's tree (src/lamm_kernel_q4_0.hpp:59-128, src/lamm_simd_avx2.h:117-127; q2_K's
 * block kernel src/lamm_kernel_q2_k.hpp:163-307 with its mins term), ggml's AVX2
 * ggml_vec_dot_q{4,5,6}_K_q8_K for q4_K / q5_K / q6_K (LC/ggml-quants.c:7082-7145, :7696-7777,
 * :8305-8385) -- so C is bit-identical to the reference's CPU build on the same blocks (VALU
 * kernels, slower than the default engines).  Supported: q4_0 / q5_0 with q8_0 B, q4_1 / q5_1 with
 * q8_1 B, q2_K / q4_K / q5_K / q6_K with q8_K B (quantized B only); others (q8_0: SURVEY §8a
 * defect 2's order) return LAMM_ERR_TYPE.  The ggml boundary uses it under LAMM_HIP_ORDER=reference (its
 * default until round 5; since round 6 the boundary runs the fast engines unless asked). */
#define LAMM_ORDER_REFERENCE 1
int lamm_hip_matmul_ex(const lamm_matrix *A, const lamm_matrix *B, const lamm_matrix *C,
                       const lamm_batch *batch, int flags, void *hip_stream);

/* n (1..LAMM_GROUP_MAX) weights times the same activation B: C[i] = A[i] * B, each exactly as
 * lamm_hip_matmul_ex(&A[i], B, &C[i], NULL, flags, s) computes it (the same bits).  A one-column
 * B with LAMM_ORDER_REFERENCE and weights of one 32-element type sharing col and ld runs as one
 * launch (the reference-order GEMV over all of them); anything else as n calls.  No reference
 * interface corresponds: llama.cpp multiplies wq / wk / wv (and ffn gate / up) by the same normed
 * activation as separate mul_mat nodes (LC/llama.cpp:5738-5752 in build_llama), one lamm_mul_mat
 * call each (LC/ggml.c:10858-10862); the ggml boundary's sibling calls batch them through here. */
#define LAMM_GROUP_MAX 4
int lamm_hip_matmul_group(const lamm_matrix *A, int n, const lamm_matrix *B, const lamm_matrix *C,
                          int flags, void *hip_stream);

/* Activation quantizer on device (ggml INIT phase, LC/ggml.c:10865-10887, run on
 * the GPU): x[N][K] f32 (row j at x + j*ldx floats) -> y, N rows of `vec_type`
 * blocks (row j at y + j*ldy blocks).  flavour 0 = *_reference rounding
 * (roundf), 1 = the AVX2 from_float rounding (nearest-even, id = 127/amax).
 * vec_type: q8_0, q8_1, q8_K, or f16 (ggml_fp32_to_fp16_row, nearest-even).
 * Weight types (src0 side, ggml_quantize_chunk LC/ggml.c:20413 with no importance
 * matrix): q4_0, q4_1, q5_0, q5_1, q2_K, q4_K, q5_K, q6_K reproduce the bytes of the
 * *_reference row quantizers (flavour ignored); q8_0 weights = q8_0 with flavour 0. */
int lamm_hip_quantize(int vec_type, int flavour, const float *x, int64_t ldx, void *y,
                      int64_t ldy, int K, int N, void *hip_stream);

/* The same AVX2-flavour activation quantizer on the host (no device needed): one row of k
 * floats (k a multiple of 32) -> k/32 q8_0 or q8_1 blocks, byte for byte what ggml's x86
 * INIT writes (LC/ggml-quants.c:1277-1330 quantize_row_q8_0, :1505-1575 quantize_row_q8_1,
 * AVX2 branches) and lamm_hip_quantize(.., flavour 1, ..) writes on the device.  The boundary
 * runs it on ggml's pool threads for prefill-sized calls (LAMM_HIP_POOL).  Other vec types:
 * LAMM_ERR_TYPE; k not a multiple of 32: LAMM_ERR_SHAPE. */
int lamm_hip_quantize_host(int vec_type, const float *x, void *y, int64_t k);

/* Weight-stationary form (weight residency).  Inference multiplies the
 * same weights by new activations on every call; a lamm_weights handle records A (whose
 * device blocks must stay valid and unchanged while the handle lives) and its ggml slice
 * dims, and for the formats the prefill GEMM repacks (q4_0 / q4_1 / q5_0 / q5_1) keeps that
 * packed form device-resident (lamm_hip_weights_bytes), so a call skips the per-call weight
 * repack.  q5_1 is packed (and then runs on the fp6 engine) only while every block scale is
 * <= 2047 and every block min <= 32752 in magnitude (round 6: 32 d and 2 m must stay exact in fp16);
 * creation synchronises hip_stream for that check, and a tensor past it keeps no packed
 * form (lamm_hip_weights_bytes 0).  lamm_hip_matmul_weights(W, B, C, batch, s) computes exactly what
 * lamm_hip_matmul_batched(&A, B, C, batch, s) computes; batch may be NULL (one slice per A
 * slice) and, if given, must repeat W's ne02 / ne03 / nba2 / nba3.  Creation runs on
 * hip_stream; destroy synchronises the device before freeing. */
typedef struct lamm_weights lamm_weights;
int lamm_hip_weights_create(const lamm_matrix *A, int64_t ne02, int64_t ne03, size_t nba2, size_t nba3,
                            void *hip_stream, lamm_weights **out);
int lamm_hip_matmul_weights(const lamm_weights *W, const lamm_matrix *B, const lamm_matrix *C,
                            const lamm_batch *batch, void *hip_stream);
size_t lamm_hip_weights_bytes(const lamm_weights *W);
void lamm_hip_weights_destroy(lamm_weights *W);

/* Which engine lamm_hip_matmul* (stationary = 0) or lamm_hip_matmul_weights (stationary = 1)
 * runs an M x N x K call of weight type `type` over `slices` A slices on, under the current
 * LAMM_* switches: "gemv" (decode GEMV), "gemv-groups" (GEMV launches of 8 columns), "dense"
 * (F32 / F16 GEMM), "superblock" (k-quant GEMM), "fp6" (block-scaled fp6 MFMA GEMM), "i8"
 * (MFMA-i8 GEMM), "dq16" (dequantizing f16 MFMA GEMM); "" for an unsupported type or shape.
 * b_f32: B holds F32 rows (q8_0 / q8_1 activation types).  Host-only: no device is touched.
 * The answer is for a call with flags = 0 (LAMM_ORDER_REFERENCE calls always run lamm_ref.hip's
 * kernels), contiguous rows and a 4-byte aligned B (an unaligned q8_K B skips "superblock", an
 * unaligned q8 B skips "dq16"): the engine an aligned, default-order call takes.
 *
 * Accuracy of the engines: every one computes each 32-element block dot exactly in integers and
 * scales it in fp32 (the reference's arithmetic, its own order only under LAMM_ORDER_REFERENCE),
 * except "dq16", which rounds each operand to f16 with its block scale folded in (<= 2^-10 relative
 * per product, within the 1e-3 bar); its range guard recomputes, with exact block dots, every tile
 * whose scales leave f16's normal range or whose operands overflow f16. */
const char *lamm_hip_engine(int type, int64_t M, int N, int K, int slices, int stationary, int b_f32);

/* Measurement hook: the next lamm_hip_matmul* call on this thread records the start and end of
 * its decode-GEMV dispatch (one column, K = 4096: BASELINE config 2's kernel) in these two HIP
 * events (hipEvent_t, created by the caller), from the dispatch's own timestamps
 * (hipExtLaunchKernel) -- the duration a kernel tracer reports, with no event packets of their own
 * around it.  The one-column decode kernels take it this way (the block-format GEMV, the k-quant
 * GEMV, the reference-order GEMV); for every other engine the two events are recorded on the
 * stream around the call's launches.  The request expires with that call either way. */
int lamm_hip_profile_next(void *start_event, void *stop_event);

/* Direct dispatch (round 5): between lamm_hip_direct_begin(device) and lamm_hip_direct_end() the
 * one-kernel decode GEMVs this thread launches (the block-format flat GEMV of config 2 and the
 * reference-order GEMV) are written as AQL packets into the library's own user-mode queue on that
 * device instead of going through HIP -- no hipLaunchKernel, no signal launch; the stream argument
 * of the calls in between is not used for them, and any other kernel still goes to its stream.
 * Inputs must be ready when the region opens (drain the streams that produced them).  end waits
 * until every dispatched kernel completed (the command processor's completion signal) and returns
 * how many were dispatched directly (0: every launch went through HIP); begin returns LAMM_OK,
 * LAMM_ERR_NODEV for a device index out of range, or LAMM_ERR_HIP when the queue is not available
 * (ROCr's loader extension missing, a region already open on this thread); end without an open
 * region returns -LAMM_ERR_HIP.  The ggml boundary can use it for decode-sized calls
 * (LAMM_HIP_DIRECT=1; off by default, it measured no faster there).  Round 6: a region in which
 * some calls had to launch through HIP sets lamm_hip_last_error() to the reason (as a failed begin
 * does), and a kernarg block the queue has written before (same kernel, arguments and grid) is
 * dispatched from its cached slot without rewriting it. */
int lamm_hip_direct_begin(int device);
int lamm_hip_direct_end(void);

/* ggml boundary diagnostics (round 5): how many sibling decode calls -- same activation row, another
 * weight (llama.cpp's wq / wk / wv, ffn_gate / ffn_up) -- were computed ahead in an earlier call's
 * device round trip, and how many of those results a later call took (its src1 bytes and weight
 * fingerprint unchanged; LAMM_HIP_SIBLINGS=0 turns the prediction off).  Either pointer may be NULL. */
void lamm_hip_sibling_stats(uint64_t *launched, uint64_t *taken);

const char *lamm_hip_last_error(void);
int lamm_hip_device_count(void);
/* Provenance: hash (sha256, 16 hex digits) of the sources this library was built from. */
const char *lamm_hip_build_id(void);

/* ggml type traits for the supported types (LC/ggml.c:477-775). */
int lamm_blck_size(int type);
size_t lamm_type_size(int type);
int lamm_vec_dot_type(int type);

/* ---- 3. multi-GPU row sharding (the reference's row split over threads,
 *         src/lamm_impl.hpp:38-43 / :107-112, mapped onto GPUs) -------------------------
 * Every rank of a communicator owns a contiguous slab of A's rows, computes its slab of C with
 * the calls above (A.data / C.data offset to its rows), and lamm_hip_allgather_rows gives every
 * rank the whole C through one RCCL all-gather over xGMI.  RCCL is loaded at the first
 * communicator (dlopen); all calls return a lamm_status (lamm_hip_comm_last_error explains). */
typedef struct lamm_comm lamm_comm;
#define LAMM_COMM_ID_BYTES 128
/* Rows [*r0, *r0 + *rows) of rank `rank` of `world`: whole `align`-row tiles, the tile remainder
 * spread over the first ranks -- every row exactly once, for any M (the reference's M / nth
 * split drops M % nth rows: SURVEY §8a defect 1). */
void lamm_hip_shard_rows(int64_t M, int world, int rank, int align, int64_t *r0, int64_t *rows);
/* One process per GPU: rank 0 makes the id (LAMM_COMM_ID_BYTES) and shares it (e.g. over
 * torch.distributed); every rank then joins with its own device. */
int lamm_hip_comm_unique_id(void *id);
int lamm_hip_comm_init_rank(lamm_comm **out, int world, int rank, const void *id, int device);
/* One process driving `ndev` devices (ncclCommInitAll).  Ranks that share a device (a rehearsal
 * on a one-GPU box; RCCL refuses duplicates) exchange slabs with device copies instead. */
int lamm_hip_comm_init_all(lamm_comm **out, int ndev, const int *devices);
int lamm_hip_comm_size(const lamm_comm *c);
int lamm_hip_comm_local_ranks(const lamm_comm *c);      /* ranks driven by this process */
int lamm_hip_comm_rank(const lamm_comm *c, int local);   /* global rank of local rank `local` */
void lamm_hip_comm_destroy(lamm_comm *c);
const char *lamm_hip_comm_last_error(void);
/* For each local rank i (arrays of lamm_hip_comm_local_ranks entries): slabs[i] holds its C slab
 * (N columns of its rows, column stride ld_slab[i] floats, on its device); C[i] receives the
 * whole C (C[j*ldc + row], ldc >= M) on that device.  Enqueued on streams[i]; the slab may
 * alias C[i] + r0. */
int lamm_hip_allgather_rows(lamm_comm *c, const float *const *slabs, const int64_t *ld_slab, float *const *C,
                            int64_t ldc, int64_t M, int N, int align, void *const *streams);

/* Device weight residency used by the ggml boundary (keyed by src0->data/type/
 * shape/strides plus a sampled fingerprint of the bytes). */
void lamm_hip_cache_clear(void);
size_t lamm_hip_cache_bytes(void);
/* The boundary's devices: LAMM_HIP_DEVICES unset = one device (LAMM_HIP_DEVICE or the first
 * gfx950); "all" = every gfx950 device; "0,1,2,3" = that list.  With several, each weight's rows
 * are split over them (lamm_hip_shard_rows) and every device copies its rows of C straight into
 * dst -- the host consumes C, no collective.  Read at the first call; reset drops
 * every device's cache and stream so the next call reads the environment again. */
void lamm_hip_boundary_reset(void);

/* Every LAMM_* environment switch (engine/plan overrides for A/B runs and tests, the boundary's
 * policies) is read once, at the first call that needs it; this re-reads them all.
 * lamm_hip_boundary_reset() re-reads them too. */
void lamm_hip_reload_env(void);

#ifdef __cplusplus
}
#endif
#endif /* LAMM_HIP_H */
