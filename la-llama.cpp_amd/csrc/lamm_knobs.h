// lamm_knobs.h -- every LAMM_* environment switch of liblamm_hip.so, read ONCE: at the first
// call that needs one, again only at lamm_hip_reload_env() (and lamm_hip_boundary_reset()).
// No launch path calls getenv.  The production defaults are the zero / -1 values; every switch
// only forces an alternative engine, plan or boundary policy (A/B measurements, tests).
#pragma once

namespace lamm {

struct Knobs {
  // ---- operator API: engine and plan selection
  int gemm_path = -1;          // LAMM_GEMM_PATH: fp6|0 / i8|1 forces the exact q4_0/q4_1/q5_0 prefill engine,
                               // dq16|2 the dequantizing f16 one (every 32-element format)
  int gemv_max_n = -1;         // LAMM_GEMV_MAX_N: widest N on the decode GEMV (-1 unset: per-type default;
                               // 0 and 1 both mean N = 1 only, the floor)
  bool dense_gemm = true;      // LAMM_DENSE_GEMM=0: F32/F16 prefill on the grouped GEMV instead
  bool kq_gemm = true;         // LAMM_KQ_GEMM=0: k-quant prefill on the grouped GEMV / i8 engine
  int fp6_split = 0;           // LAMM_FP6_SPLIT=n: split-K plan with n splits
  int fp6_sub = -1;            // LAMM_FP6_SUB: 0 split-K plan, 1 4-group K-group plan, 2 2-group plan
  bool fp6_fused_reduce = false;   // LAMM_FP6_FUSED_REDUCE=1: split-K partials summed in-launch
  int fp6_wj = 2;              // LAMM_FP6_WJ=1: 16 waves of 32x64 on the 256x128 plan
  int fp6_kv_p = 0;            // LAMM_FP6_KV_P=3: three blocks in flight per wave of gemm_fp6_kv_kernel
                               // (A/B, q4_0 / q5_0; default two)
  bool fp6_av = true;          // LAMM_FP6_AV=0: the K-group plan's barrier-staged LDS form instead
  int i8_split = 0;            // LAMM_I8_SPLIT=n
  int dense_split = 0;         // LAMM_DENSE_SPLIT=n
  int kq_split = 0;            // LAMM_KQ_SPLIT=n
  int kq_variant = 0;          // LAMM_KQ_VARIANT=1: single-pass super-block kernel
  int gemv_variant = 0;        // LAMM_GEMV_VARIANT: 7 segmented, 8 DMA 4x4, 10 VGPR stream, 12 flat, 13 staged seg
  int gemv_rpw = -1;           // LAMM_GEMV_RPW: 0 off, 4 / 8 / 16 waves forced
  bool gemv_laneb = false;     // LAMM_GEMV_LANEB=1: per-lane activation blocks in the row-per-wave GEMV
  // ---- ggml boundary
  int opt_level = 3;           // LAMM_OPT_LEVEL=0: lamm_can_mul_mat always false
  int device = -1;             // LAMM_HIP_DEVICE: the boundary's device (-1: first gfx950)
  char devices[256] = {0};     // LAMM_HIP_DEVICES: "all" or "0,1,2,3" (empty: one device)
  bool stats = false;          // LAMM_HIP_STATS=1 (=2: also synchronise after each upload, so "B up"
  bool stats_sync = false;     // holds the transfer itself, not only its issue)
  double cache_gb = 64.0;      // LAMM_HIP_CACHE_GB
  bool pinned = true;          // LAMM_HIP_PINNED=0: no pinned staging (and no zero copy)
  int views = -1;              // LAMM_HIP_VIEWS: 0 never, 1 always, -1 prefill only
  bool extra_types = true;     // LAMM_HIP_EXTRA_TYPES=0: only the reference's 7 pairs
  int gpu_quant = -1;          // LAMM_HIP_GPU_QUANT: 0 CPU INIT, 1 GPU for every row count
  bool fused = false;          // LAMM_HIP_FUSED=1: the decode GEMV quantizes the F32 row itself (INIT claimed)
  bool spin = true;            // LAMM_HIP_SPIN=0: hipStreamSynchronize instead of the flag spin
  bool siblings = true;        // LAMM_HIP_SIBLINGS=0: no sibling decode calls computed ahead (lamm_hip.cpp Siblings)
  bool signal_write = false;   // LAMM_HIP_SIGNAL_WRITE=1: completion flag by hipStreamWriteValue32 (A/B)
  bool vram_x = true;          // LAMM_HIP_VRAM_X=0: decode activations zero-copy from pinned host memory
                               // instead of written into device memory through the BAR
  bool aql_host_karg = false;  // LAMM_AQL_HOSTKARG=1: the direct queue's kernargs in host memory (A/B)
  bool direct = false;         // LAMM_HIP_DIRECT=1: decode-sized boundary calls dispatch on the library's
                               // own AQL queue (lamm_aql.cpp) instead of launching through HIP
  int c_watch = 0;             // LAMM_HIP_C_WATCH=1|2: decode-sized zero-copy calls learn completion from
                               // C's own words (lamm_hip.cpp watch_c; 1 coherent C, 2 non-coherent)
                               // instead of from a signal launch behind the GEMV
  bool kernel_signal = false;  // LAMM_HIP_KERNEL_SIGNAL=1: the GEMV writes the completion flag
  int zero_copy = 3;           // LAMM_HIP_ZERO_COPY: 0 off, 1 in, 2 out, 3 both
  bool zero_copy_split = false;   // LAMM_HIP_ZERO_COPY_SPLIT=1: zero copy also when rows split over devices
  int helpers = 0;             // LAMM_HIP_HELPERS: ggml's other pool threads during thread 0's device work:
                               // 0 return at once (ggml's barrier spins on them), 1 wait here yielding,
                               // 2 wait here asleep (futex)
  int ref_mfma = -1;           // LAMM_REF_MFMA: reference-order prefill kernel (1: ref_mfma_kernel, 2 / 3 / 4: ref_mfma2
                               // with 2 / 1 / 4 column groups, 5: 2 groups + swizzled image, 6: 5 with the chain
                               // steps interleaved with the next group's MFMAs; unset: per format)
  int ref_gemv_bpt = 2;        // LAMM_REF_GEMV_BPT: blocks per producer thread of ref_gemv_kernel (2: 512
                               // threads per workgroup, 4: 256)
  bool aql_eager = true;       // LAMM_AQL_EAGER=0: direct-dispatch packets held until the next call (round 5)
  bool aql_fence_none = false; // LAMM_AQL_FENCE=none: a region's inner packets carry no acquire / release fence
                               // (probe: what the agent-scope fences between back-to-back kernels cost)
  bool ref_order = false;      // LAMM_HIP_ORDER=reference: the boundary computes in the reference's own float
                               // order (lamm_ref.hip, bit-identical to the lamm opt-3 AVX2 build) instead of
                               // the fast engines (the default since round 6: within the north star's 1e-3
                               // per node)
  int pool = 5;                // LAMM_HIP_POOL: what ggml's pool threads do for prefill-sized calls (bits):
                               // 1 quantize the F32 activations to q8_0 / q8_1 rows in pinned memory (the
                               // upload moves those instead of F32), 2 scatter C out of pinned memory
                               // (else HIP's pageable copy), 4 a reference-order call as two pipelined
                               // column chunks on two streams; 0: thread 0 alone, as before
};

// The current switches (read from the environment at the first call).
const Knobs& knobs();
// Re-read the environment (tests, A/B tools); earlier references stay valid.
void reload_knobs();

}  // namespace lamm
