// gemm_stream_probe.hip -- how fast can a CU pull BASELINE config 3's packed GEMM operands out of
// L2 / MALL, by which mechanism?  The operand stream of the fp6 K-group GEMM (csrc/lamm_gemm_fp6.hip,
// 128 x 64 output tile per workgroup, full K): per K-step (2 blocks) 8 KiB of A planes (128 rows)
// and 8 KiB of B planes (64 rows x hi/lo), 64 K-steps = 1 MiB per CU; all 256 workgroups at once
// (32 i-tiles x 8 j-tiles, XCD-aware order as the GEMM).  No arithmetic: every loaded dword is
// folded into an XOR that is stored only if impossible.  Per-launch time, hipGraph replay.
//   dma<S>     : LDS-DMA (buffer_load ... lds, 1 KiB per wave instruction) as the GEMM does:
//                stages of 4 K-steps (64 KiB), S stages, wait + barrier per stage; fragments read
//                back from LDS by ds_read_b128 like the MFMA operands
//   vgpr<D>    : every wave loads its own operands straight into VGPRs (global b128), no LDS:
//                wave (group g, half wi) takes K-steps g, g+4, ...: its 64 A rows (4 KiB) and all 64
//                B rows (8 KiB) per K-step, D K-steps in flight
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -I la-llama.cpp_amd/csrc tools/gemm_stream_probe.hip -o tools/gemm_stream_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <functional>

#include "lamm_device.h"

using namespace lamm;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

constexpr int NIT = 32, NJT = 8, NSTEP = 64;      // 4096 / 128, 512 / 64, 128 blocks / 2
constexpr int CHUNK = 8192;                        // bytes per (tile, K-step), A and B alike
constexpr size_t A_BYTES = (size_t)NIT * NSTEP * CHUNK, B_BYTES = (size_t)NJT * NSTEP * CHUNK;
constexpr int KG = 4, NW = 8;

__device__ __forceinline__ void tile_of(int& it, int& jt, int mode) {
  // XCD-aware order of the real kernel: one XCD's 32 workgroups = 8 i-tiles x 4 j-tiles
  // mode 1: every workgroup streams tile (0, 0) (L2-resident after the first touch);
  // mode 2: the workgroups of an XCD share one tile, XCDs differ (a per-XCD working set of 1 tile)
  const int id = blockIdx.x, x = id & 7, k = id >> 3, q = 256 >> 3;
  if (mode == 1) { it = jt = 0; return; }
  if (mode == 2) { it = x; jt = 0; return; }
  const int wv = x * q + k, per = NIT * NJT;
  const int ws_ = wv % per, ib = ws_ / (8 * NJT), rem = ws_ % (8 * NJT);
  jt = rem / 8;
  it = ib * 8 + rem % 8;
}

template <int NBUF>
__global__ __launch_bounds__(512) void k_dma(const unsigned char* A, const unsigned char* B, unsigned* out, int mode) {
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  constexpr int STAGE = KG * 2 * CHUNK;   // 64 KiB
  int it, jt;
  tile_of(it, jt, mode);
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const auto ra = make_rsrc(A + (size_t)it * NSTEP * CHUNK, NSTEP * CHUNK);
  const auto rb = make_rsrc(B + (size_t)jt * NSTEP * CHUNK, NSTEP * CHUNK);
  auto issue = [&](int ss) {
    unsigned char* dst = smem + (ss % NBUF) * STAGE;
#pragma unroll
    for (int k = 0; k < 8; ++k) {   // 64 pieces per stage over 8 waves
      const int pc = k * NW + w, g = pc / 16, q = pc % 16, ks = ss * KG + g;
      auto* d = (__attribute__((address_space(3))) void*)(dst + pc * 1024);
      if (q < 8)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, d, 16, lane * 16, ks * CHUNK + q * 1024, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rb, d, 16, lane * 16, ks * CHUNK + (q - 8) * 1024, 0, 0);
    }
  };
  const int nst = NSTEP / KG;   // 16 stages
  for (int k = 0; k < NBUF - 1 && k < nst; ++k) issue(k);
  u32x4 x = {0, 0, 0, 0};
  const int g = w / 2;
  for (int ss = 0; ss < nst; ++ss) {
    if (ss + NBUF - 1 < nst) {
      __builtin_amdgcn_s_waitcnt((8 * (NBUF - 2) & 0xF) | (((8 * (NBUF - 2)) >> 4) << 14) | (0x7 << 4) | (0xF << 8));
    } else {
      __builtin_amdgcn_s_waitcnt((0 & 0xF) | (0x7 << 4) | (0xF << 8));
    }
    __syncthreads();
    if (ss + NBUF - 1 < nst) issue(ss + NBUF - 1);
    // the fragments the MFMAs would read: this wave's 2 x (A 2 planes x 2 blocks x 2 subtiles) +
    // (B 2 planes x 2 blocks x 2 subtiles) ds_read_b128 per K-step
    const unsigned char* sg = smem + (ss % NBUF) * STAGE + g * 2 * CHUNK;
#pragma unroll
    for (int f = 0; f < 16; ++f) {
      const int off = (f * 1024 + (w & 1) * 512 + (lane & 31) * 16) % (2 * CHUNK);
      x ^= *reinterpret_cast<const u32x4*>(sg + off);
    }
  }
  if ((x[0] ^ x[1] ^ x[2] ^ x[3]) == 0x9e3779b9u) out[blockIdx.x] = x[0];
}

template <int D>
__global__ __launch_bounds__(512) void k_vgpr(const unsigned char* A, const unsigned char* B, unsigned* out, int mode) {
  int it, jt;
  tile_of(it, jt, mode);
  const int t = threadIdx.x, lane = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int g = w / 2, wi = w % 2;
  const auto ra = make_rsrc(A + (size_t)it * NSTEP * CHUNK, NSTEP * CHUNK);
  const auto rb = make_rsrc(B + (size_t)jt * NSTEP * CHUNK, NSTEP * CHUNK);
  u32x4 buf[D][12];
  auto issue = [&](int slot, int ks) {
#pragma unroll
    for (int k = 0; k < 4; ++k)   // A: planes x blocks, this wave's 64 rows (1 KiB each)
      buf[slot][k] = __builtin_amdgcn_raw_buffer_load_b128(ra, ks * CHUNK + k * 2048 + wi * 1024 + lane * 16, 0, 0);
#pragma unroll
    for (int k = 0; k < 8; ++k)   // B: planes x blocks x hi/lo, all 64 rows
      buf[slot][4 + k] = __builtin_amdgcn_raw_buffer_load_b128(rb, ks * CHUNK + k * 1024 + lane * 16, 0, 0);
  };
  const int n = NSTEP / KG;   // this wave's K-steps: g, g + 4, ...
#pragma unroll
  for (int d = 0; d < D - 1; ++d) issue(d, g + KG * d);
  u32x4 x = {0, 0, 0, 0};
  for (int i = 0; i < n; i += D) {
#pragma unroll
    for (int d = 0; d < D; ++d) {
      const int ii = i + d;
      if (ii + D - 1 < n) issue((d + D - 1) % D, g + KG * (ii + D - 1));
      if (ii + D - 1 < n)
        __builtin_amdgcn_s_waitcnt(((12 * (D - 1)) & 0xF) | (((12 * (D - 1)) >> 4) << 14) | (0x7 << 4) | (0xF << 8));
      else
        __builtin_amdgcn_s_waitcnt((0x7 << 4) | (0xF << 8));
#pragma unroll
      for (int k = 0; k < 12; ++k) x ^= buf[d][k];
    }
  }
  if ((x[0] ^ x[1] ^ x[2] ^ x[3]) == 0x9e3779b9u) out[blockIdx.x] = x[0];
}

int main() {
  unsigned char *A, *B;
  unsigned* out;
  CK(hipMalloc(&A, A_BYTES + 4096));
  CK(hipMalloc(&B, B_BYTES + 4096));
  CK(hipMalloc(&out, 4096));
  CK(hipMemset(A, 0x5a, A_BYTES));
  CK(hipMemset(B, 0x3c, B_BYTES));
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_graph = [&](const std::function<void()>& L) {
    constexpr int REPS = 200;
    hipGraph_t g;
    hipGraphExec_t ge;
    L();
    CK(hipStreamSynchronize(s));
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int r = 0; r < REPS; ++r) L();
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    float best = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      CK(hipEventRecord(e0, s));
      CK(hipGraphLaunch(ge, s));
      CK(hipEventRecord(e1, s));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      best = ms < best ? ms : best;
    }
    CK(hipGraphExecDestroy(ge));
    CK(hipGraphDestroy(g));
    return best * 1000.0 / REPS;
  };
  const double per_cu = (double)NSTEP * 2 * CHUNK;
  bool first = true;
  auto report = [&](const char* name, double us) {
    printf("%s\"%s\": {\"us\": %.2f, \"GBs_per_CU\": %.1f}", first ? "{" : ", ", name, us, per_cu / us / 1e3);
    first = false;
    fflush(stdout);
  };
  constexpr int lds = 2 * 65536;
  CK(hipFuncSetAttribute((const void*)k_dma<2>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  const char* mname[3] = {"", "-same", "-xcd"};
  for (int mode = 0; mode < 3; ++mode) {
    char n[32];
    snprintf(n, sizeof n, "dma2%s", mname[mode]);
    report(n, time_graph([&] { k_dma<2><<<256, 512, lds, s>>>(A, B, out, mode); }));
    snprintf(n, sizeof n, "vgpr2%s", mname[mode]);
    report(n, time_graph([&] { k_vgpr<2><<<256, 512, 0, s>>>(A, B, out, mode); }));
    if (mode == 0) {
      report("vgpr3", time_graph([&] { k_vgpr<3><<<256, 512, 0, s>>>(A, B, out, 0); }));
      report("vgpr4", time_graph([&] { k_vgpr<4><<<256, 512, 0, s>>>(A, B, out, 0); }));
    }
  }
  printf(", \"bytes_per_cu\": %.0f}\n", per_cu);
  return 0;
}
