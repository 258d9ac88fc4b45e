// prep_probe.hip -- where do the ~6.5 us of config 3's activation prep go?  The fp6 GEMM's
// q8 -> hi/lo fp6 plane kernel (prep_b_fp6_tile, csrc/lamm_gemm_fp6.hip, compiled into this TU)
// on config 3's B (512 x 4096 q8_0 = 2.2 MB in, 4.2 MB of planes out), beside copy kernels that
// move the same bytes: read-only, write-only, read+write; and the whole GEMM call vs its main
// kernel alone ("GBs" of the gemm lines = GFLOP/s / 1000 = TFLOP/s).  hipGraph replay, per-launch us.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -DLAMM_AB_VARIANTS -I la-llama.cpp_amd/csrc \
//         tools/prep_probe.hip la-llama.cpp_amd/csrc/lamm_knobs.cpp -o tools/prep_probe
// (-fno-slp-vectorize as the library's Makefile builds this TU: without it the K-group kernels spill)
#include "../la-llama.cpp_amd/csrc/lamm_gemm_fp6.hip"

#include <cstdio>
#include <cstring>
#include <functional>
#include <vector>

namespace lamm {
void set_max_lds(const void* kernel, int bytes) {
  (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}
}  // namespace lamm

using namespace lamm;

#define CK(x)                                                                              \
  do {                                                                                     \
    hipError_t e_ = (x);                                                                   \
    if (e_ != hipSuccess) {                                                                \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));    \
      exit(1);                                                                             \
    }                                                                                      \
  } while (0)

// MODE 1 read (xor, stored only if impossible), 2 write, 3 copy in -> out (out 2x in)
template <int MODE>
__global__ __launch_bounds__(256) void k_move(const u32x4* in, size_t nin, u32x4* out, size_t nout) {
  const size_t t = blockIdx.x * (size_t)blockDim.x + threadIdx.x, n = gridDim.x * (size_t)blockDim.x;
  u32x4 x = {0, 0, 0, 0};
  if constexpr (MODE & 1)
    for (size_t i = t; i < nin; i += n) x ^= __builtin_nontemporal_load(in + i);
  if constexpr (MODE & 2) {
    for (size_t i = t; i < nout; i += n) out[i] = x + (uint32_t)i;
  } else {
    if ((x[0] ^ x[1] ^ x[2] ^ x[3]) == 0x9e3779b9u) out[t] = x;
  }
}

int main(int argc, char** argv) {
  const char* only = argc > 1 ? argv[1] : nullptr;   // run only the lines whose name contains it
  const int M = 4096, K = 4096, nb = K / 32;
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto time_graph = [&](const std::function<void()>& L) {
    constexpr int REPS = 100;
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
  bool first = true;
  auto run = [&](const char* name, double bytes, const std::function<void()>& L) {
    if (only && !strstr(name, only)) return;
    const double us = time_graph(L);
    printf("%s\"%s\": {\"us\": %.2f, \"GBs\": %.0f}", first ? "{" : ", ", name, us, bytes / us / 1e3);
    first = false;
    fflush(stdout);
  };
  run("empty", 0, [&] { k_move<0><<<1, 64, 0, s>>>(nullptr, 0, nullptr, 0); });
  for (int N : {512, 2048}) {
    const size_t brow = (size_t)nb * 34, bbytes = (size_t)N * brow;
    std::vector<unsigned char> hb(bbytes);
    for (size_t i = 0; i < bbytes; ++i) hb[i] = (unsigned char)(i * 2654435761u >> 13);
    for (int j = 0; j < N; ++j)
      for (int b = 0; b < nb; ++b) { hb[j * brow + b * 34] = 0x00; hb[j * brow + b * 34 + 1] = 0x3c; }
    unsigned char *dB, *ws;
    GemvArgs p{};
    p.M = M; p.N = N; p.K = K; p.nblk = nb; p.ldb = (int64_t)brow; p.lda = nb * 18; p.ldc = M;
    const F6Layout L = F6Layout::of(p);
    const size_t wsb = (size_t)L.b_slice;
    CK(hipMalloc(&dB, bbytes + 256));
    CK(hipMalloc(&ws, wsb + 256));
    CK(hipMemcpy(dB, hb.data(), bbytes, hipMemcpyHostToDevice));
    p.B = dB;
    const int rg = (int)((L.njt * F6_TJ + PB_ROWS - 1) / PB_ROWS), nbg = (L.nsteps * F6_KB + PB_NB - 1) / PB_NB;
    // the whole fp6 GEMM call on stationary weights (prep + K-group main) and its main kernel alone
    unsigned char *dA, *wA, *wsAll;
    float* dC;
    const size_t arow = (size_t)nb * 18;
    std::vector<unsigned char> ha((size_t)M * arow);
    for (size_t i = 0; i < ha.size(); ++i) ha[i] = (unsigned char)(i * 2246822519u >> 11);
    for (int i = 0; i < M; ++i)
      for (int b = 0; b < nb; ++b) { ha[i * arow + b * 18] = 0x00; ha[i * arow + b * 18 + 1] = 0x2c; }
    CK(hipMalloc(&dA, ha.size() + 256));
    CK(hipMemcpy(dA, ha.data(), ha.size(), hipMemcpyHostToDevice));
    p.A = dA;
    CK(hipMalloc(&wA, gemm_fp6_weight_bytes(kQ4_0, p) + 256));
    const size_t wsn = gemm_fp6_workspace_bytes(kQ4_0, p, true);
    CK(hipMalloc(&wsAll, wsn));
    CK(hipMalloc(&dC, (size_t)M * N * 4 + 256));
    p.C = dC;
    CK(prepare_fp6_weights(kQ4_0, p, wA, s));
    CK(hipStreamSynchronize(s));
    char n[64];
    snprintf(n, sizeof n, "gemm_whole_N%d", N);
    run(n, 2.0 * M * N * K / 1e3, [&] { CK(launch_gemm_fp6(kQ4_0, p, wA, wsAll, s)); });
    if (N == 512) {
      constexpr size_t lds = (size_t)4 * 64 * (128 + 8) * 4;
      const int grid = (M / 128) * (N / 64);
#define KV(NAME, PP, AB, AD)                                                                          \
  set_max_lds((const void*)gemm_fp6_kv_kernel<kQ4_0, PP, AB, AD>, (int)lds);                          \
  snprintf(n, sizeof n, NAME "_N%d", N);                                                              \
  run(n, 2.0 * M * N * K / 1e3, [&] { gemm_fp6_kv_kernel<kQ4_0, PP, AB, AD><<<grid, 512, lds, s>>>(p, wA, wsAll); });
      KV("gemm_kvmain_p3", 3, 0, 0)
      KV("gemm_kvmain_p2", 2, 0, 0)
      KV("gemm_kvmain_ad_p3", 3, 0, 1)
      KV("gemm_kvmain_ad_p2", 2, 0, 1)
      KV("gemm_kvmain_ad_p4", 4, 0, 1)
      KV("gemm_kvmain_loadsonly_p3", 3, 1, 0)
      KV("gemm_kvmain_ad_loadsonly_p3", 3, 1, 1)
      KV("gemm_kvmain_computeonly_p3", 3, 2, 0)
      KV("gemm_kvmain_ad_computeonly_p3", 3, 2, 1)
      KV("gemm_kvmain_co_halffma_p3", 3, 3, 0)
      KV("gemm_kvmain_co_1fma_p3", 3, 4, 0)
      KV("gemm_kvmain_noactp1_p2", 2, 5, 0)
      KV("gemm_kvmain_nowp1_p2", 2, 6, 0)
      KV("gemm_kvmain_nop1_p2", 2, 7, 0)
      KV("gemm_kvmain_p2_again", 2, 0, 0)
      {   // the AD variant's C against the production kernel's, bit for bit
        std::vector<float> c0((size_t)M * N), c1((size_t)M * N);
        CK(hipMemset(dC, 0, (size_t)M * N * 4));
        gemm_fp6_kv_kernel<kQ4_0, 3, 0, 0><<<grid, 512, lds, s>>>(p, wA, wsAll);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(c0.data(), dC, c0.size() * 4, hipMemcpyDeviceToHost));
        CK(hipMemset(dC, 0, (size_t)M * N * 4));
        gemm_fp6_kv_kernel<kQ4_0, 3, 0, 1><<<grid, 512, lds, s>>>(p, wA, wsAll);
        CK(hipStreamSynchronize(s));
        CK(hipMemcpy(c1.data(), dC, c1.size() * 4, hipMemcpyDeviceToHost));
        size_t bad = 0;
        for (size_t i = 0; i < c0.size(); ++i) bad += memcmp(&c0[i], &c1[i], 4) != 0;
        printf(", \"ad_vs_production_mismatches\": %zu", bad);
      }
    }
    CK(hipFree(dA));
    CK(hipFree(wA));
    CK(hipFree(wsAll));
    CK(hipFree(dC));
    snprintf(n, sizeof n, "prep_tile_N%d", N);
    run(n, (double)bbytes + wsb, [&] { prep_b_fp6_tile<kQ4_0><<<dim3(rg * nbg, 1), PB_NT, 0, s>>>(p, ws); });
    const int grid = 1024;
    snprintf(n, sizeof n, "read_N%d", N);
    run(n, (double)bbytes, [&] { k_move<1><<<grid, 256, 0, s>>>((const u32x4*)dB, bbytes / 16, (u32x4*)ws, 0); });
    snprintf(n, sizeof n, "write_N%d", N);
    run(n, (double)wsb, [&] { k_move<2><<<grid, 256, 0, s>>>((const u32x4*)dB, 0, (u32x4*)ws, wsb / 16); });
    snprintf(n, sizeof n, "copy_N%d", N);
    run(n, (double)bbytes + wsb, [&] { k_move<3><<<grid, 256, 0, s>>>((const u32x4*)dB, bbytes / 16, (u32x4*)ws, wsb / 16); });
    CK(hipFree(dB));
    CK(hipFree(ws));
  }
  printf("}\n");
  return 0;
}
