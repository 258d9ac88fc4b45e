// mfma_probe.hip -- gfx950 micro-probes that size the quantized-GEMM epilogue design.
//
//  layout : checks the lane/element map of v_mfma_scale_f32_32x32x64_f8f6f4 with fp6 (e2m3)
//           operands against a host fp64 reference under several hypotheses;
//  timing : cycles per iteration (s_memtime) of MFMA / epilogue mixes at 1 and 2 waves/SIMD.
//
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_probe tools/mfma_probe.hip
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x16 __attribute__((ext_vector_type(16)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef _Float16 half4 __attribute__((ext_vector_type(4)));
typedef _Float16 half8 __attribute__((ext_vector_type(8)));

#define CHECK(x)                                                                  \
  do {                                                                            \
    hipError_t e_ = (x);                                                          \
    if (e_ != hipSuccess) {                                                       \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                    \
    }                                                                             \
  } while (0)

// ---------------------------------------------------------------- layout check
// in: per lane 6 dwords A, 6 dwords B, 1 dword scale A, 1 dword scale B
__global__ void fp6_layout(const uint32_t* in, float* out) {
  const int l = threadIdx.x;
  const uint32_t* p = in + l * 14;
  i32x8 a = {(int)p[0], (int)p[1], (int)p[2], (int)p[3], (int)p[4], (int)p[5], 0, 0};
  i32x8 b = {(int)p[6], (int)p[7], (int)p[8], (int)p[9], (int)p[10], (int)p[11], 0, 0};
  f32x16 c = {};
  c = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a, b, c, 2, 2, 0, (int)p[12], 0, (int)p[13]);
  for (int e = 0; e < 16; ++e) out[l * 16 + e] = c[e];
}

static double e2m3(uint32_t code) {
  const int s = (code >> 5) & 1, ex = (code >> 3) & 3, m = code & 7;
  const double v = ex == 0 ? m / 8.0 : std::ldexp(1.0 + m / 8.0, ex - 1);
  return s ? -v : v;
}

static int layout_check() {
  std::vector<uint32_t> in(64 * 14);
  srand(12345);
  std::vector<uint32_t> codeA(64 * 32), codeB(64 * 32), sa(64), sb(64);
  for (int l = 0; l < 64; ++l) {
    for (int e = 0; e < 32; ++e) { codeA[l * 32 + e] = rand() & 63; codeB[l * 32 + e] = rand() & 63; }
    sa[l] = 124 + rand() % 7;   // E8M0: 2^(s-127)
    sb[l] = 124 + rand() % 7;
    uint32_t wa[7] = {}, wb[7] = {};
    for (int e = 0; e < 32; ++e) {
      const int bit = 6 * e;
      wa[bit / 32] |= codeA[l * 32 + e] << (bit % 32);
      if (bit % 32 > 26) wa[bit / 32 + 1] |= codeA[l * 32 + e] >> (32 - bit % 32);
      wb[bit / 32] |= codeB[l * 32 + e] << (bit % 32);
      if (bit % 32 > 26) wb[bit / 32 + 1] |= codeB[l * 32 + e] >> (32 - bit % 32);
    }
    for (int k = 0; k < 6; ++k) { in[l * 14 + k] = wa[k]; in[l * 14 + 6 + k] = wb[k]; }
    in[l * 14 + 12] = sa[l];
    in[l * 14 + 13] = sb[l];
  }
  uint32_t* din;
  float* dout;
  CHECK(hipMalloc(&din, in.size() * 4));
  CHECK(hipMalloc(&dout, 64 * 16 * 4));
  CHECK(hipMemcpy(din, in.data(), in.size() * 4, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(fp6_layout, dim3(1), dim3(64), 0, 0, din, dout);
  CHECK(hipDeviceSynchronize());
  std::vector<float> got(64 * 16);
  CHECK(hipMemcpy(got.data(), dout, got.size() * 4, hipMemcpyDeviceToHost));
  // hypotheses for k(lane-half h, element e)
  const char* names[] = {"k=32h+e", "k=2e+h", "k=16*(e/16)*2+16h+e%16", "k=8*(e/8)*2+8h+e%8", "k=4*(e/4)*2+4h+e%4"};
  int best = -1;
  for (int hyp = 0; hyp < 5; ++hyp) {
    // A[row r][k], B[k][col c]; scales by (row, k/32) and (col, k/32)
    std::vector<double> A(32 * 64), B(64 * 32), SA(32 * 2), SB(32 * 2);
    for (int l = 0; l < 64; ++l) {
      const int r = l & 31, h = l >> 5;
      for (int e = 0; e < 32; ++e) {
        int k;
        switch (hyp) {
          case 0: k = 32 * h + e; break;
          case 1: k = 2 * e + h; break;
          case 2: k = (e / 16) * 32 + 16 * h + e % 16; break;
          case 3: k = (e / 8) * 16 + 8 * h + e % 8; break;
          default: k = (e / 4) * 8 + 4 * h + e % 4; break;
        }
        A[r * 64 + k] = e2m3(codeA[l * 32 + e]);
        B[k * 32 + r] = e2m3(codeB[l * 32 + e]);
      }
      SA[r * 2 + h] = std::ldexp(1.0, (int)sa[l] - 127);
      SB[r * 2 + h] = std::ldexp(1.0, (int)sb[l] - 127);
    }
    int bad = 0;
    double maxerr = 0;
    for (int l = 0; l < 64; ++l)
      for (int e = 0; e < 16; ++e) {
        const int col = l & 31, row = (e & 3) + 8 * (e >> 2) + 4 * (l >> 5);
        double ref = 0;
        for (int k = 0; k < 64; ++k) ref += SA[row * 2 + k / 32] * A[row * 64 + k] * B[k * 32 + col] * SB[col * 2 + k / 32];
        const double err = std::fabs(ref - got[l * 16 + e]);
        maxerr = std::fmax(maxerr, err / (std::fabs(ref) + 1e-6));
        if (err > 1e-5 * (std::fabs(ref) + 1)) ++bad;
      }
    printf("layout hypothesis %-28s mismatches %4d / 1024  max rel err %.3g\n", names[hyp], bad, maxerr);
    if (bad == 0 && best < 0) best = hyp;
  }
  CHECK(hipFree(din));
  CHECK(hipFree(dout));
  printf("layout: %s\n", best >= 0 ? names[best] : "NO HYPOTHESIS MATCHES");
  return best;
}

// ---------------------------------------------------------------- timing
#define KEEP(x) asm volatile("" : "+v"(x))

template <int MODE, int W>
__global__ __launch_bounds__(256 * W) void timing(int iters, const int* src, float* sink, long long* cyc) {
  const int lane = threadIdx.x & 63;
  i32x4 a4 = {src[lane], src[lane + 1], src[lane + 2], src[lane + 3]};
  i32x4 b4 = {src[lane + 4], src[lane + 5], src[lane + 6], src[lane + 7]};
  i32x8 a8 = {src[lane], src[lane + 1], src[lane + 2], src[lane + 3], src[lane + 4], src[lane + 5], 0, 0};
  i32x8 b8 = {src[lane + 6], src[lane + 7], src[lane + 8], src[lane + 9], src[lane + 10], src[lane + 11], 0, 0};
  half4 h4 = {(_Float16)0.01f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
  half8 h8 = {(_Float16)0.01f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f,
              (_Float16)0.f,   (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
  const i32x16 iz = {};
  const f32x16 fz = {};
  f32x16 acc[4];
  i32x16 iacc[4];
  for (int t = 0; t < 4; ++t) { acc[t] = fz; iacc[t] = iz; }
  float dbv[16];
  for (int e = 0; e < 16; ++e) dbv[e] = 1e-3f * (float)src[e];
  float da = 1e-2f * (float)src[lane + 3];

  __syncthreads();
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    KEEP(a4); KEEP(b4); KEEP(a8); KEEP(b8); KEEP(h4); KEEP(h8);
    if constexpr (MODE == 0) {          // 4 x i8 32x32x32, independent chains
      for (int t = 0; t < 4; ++t) iacc[t] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, iacc[t], 0, 0, 0);
    } else if constexpr (MODE == 1) {   // 4 x f16 32x32x8
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x8f16(h4, h4, acc[t], 0, 0, 0);
    } else if constexpr (MODE == 2) {   // 4 x fp6 scaled 32x32x64
      for (int t = 0; t < 4; ++t)
        acc[t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, acc[t], 2, 2, 0, 127, 0, 127);
    } else if constexpr (MODE == 3) {   // 4 x f16 32x32x16
      for (int t = 0; t < 4; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(h8, h8, acc[t], 0, 0, 0);
    } else if constexpr (MODE == 4) {   // i8 S + f16 P + cvt + fma
      for (int t = 0; t < 4; ++t) {
        KEEP(a4);
        const i32x16 s = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, iz, 0, 0, 0);
        const f32x16 p = __builtin_amdgcn_mfma_f32_32x32x8f16(h4, h4, fz, 0, 0, 0);
        for (int e = 0; e < 16; ++e) acc[t][e] = __builtin_fmaf((float)s[e], p[e], acc[t][e]);
      }
    } else if constexpr (MODE == 5) {   // fp6 S + f16 P + fma
      for (int t = 0; t < 4; ++t) {
        KEEP(a8);
        const f32x16 s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, fz, 2, 2, 0, 127, 0, 127);
        const f32x16 p = __builtin_amdgcn_mfma_f32_32x32x8f16(h4, h4, fz, 0, 0, 0);
        for (int e = 0; e < 16; ++e) acc[t][e] = __builtin_fmaf(s[e], p[e], acc[t][e]);
      }
    } else if constexpr (MODE == 6) {   // fp6 S + VALU P (16 mul) + fma
      for (int t = 0; t < 4; ++t) {
        KEEP(a8); KEEP(da);
        const f32x16 s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, fz, 2, 2, 0, 127, 0, 127);
        for (int e = 0; e < 16; ++e) acc[t][e] = __builtin_fmaf(s[e], da * dbv[e], acc[t][e]);
      }
    } else if constexpr (MODE == 7) {   // VALU only: 64 fma
      for (int t = 0; t < 4; ++t) {
        KEEP(da);
        for (int e = 0; e < 16; ++e) acc[t][e] = __builtin_fmaf(da, dbv[e], acc[t][e]);
      }
    } else if constexpr (MODE == 8) {   // fp6 S + fma with a register-resident P (P free)
      for (int t = 0; t < 4; ++t) {
        KEEP(a8);
        const f32x16 s = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, fz, 2, 2, 0, 127, 0, 127);
        for (int e = 0; e < 16; ++e) acc[t][e] = __builtin_fmaf(s[e], dbv[e], acc[t][e]);
      }
    } else if constexpr (MODE == 9) {   // i8 S + cvt + fma with register P
      for (int t = 0; t < 4; ++t) {
        KEEP(a4);
        const i32x16 s = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, iz, 0, 0, 0);
        for (int e = 0; e < 16; ++e) acc[t][e] = __builtin_fmaf((float)s[e], dbv[e], acc[t][e]);
      }
    } else if constexpr (MODE >= 11 && MODE <= 14) {
      // software-pipelined: the MFMA of block t+1 is issued before block t's VALU epilogue,
      // and sched_group_barrier interleaves them (1 MFMA : n VALU).
      //   11: fp6 S + fma (P in regs)        12: fp6 S + VALU P (mul) + fma
      //   13: fp6 S + f16 P MFMA + fma        14: i8 S + cvt + fma (P in regs)
      constexpr bool I8 = MODE == 14;
      f32x16 s[2];
      i32x16 si[2];
      f32x16 p[2];
      auto issue = [&](int t) {
        KEEP(a8); KEEP(a4);
        if constexpr (I8) si[t & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, iz, 0, 0, 0);
        else s[t & 1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, fz, 2, 2, 0, 127, 0, 127);
        if constexpr (MODE == 13) p[t & 1] = __builtin_amdgcn_mfma_f32_32x32x8f16(h4, h4, fz, 0, 0, 0);
      };
      auto epi = [&](int t) {
        KEEP(da);
        for (int e = 0; e < 16; ++e) {
          float pe;
          if constexpr (MODE == 12) pe = da * dbv[e];
          else if constexpr (MODE == 13) pe = p[t & 1][e];
          else pe = dbv[e];
          const float se = I8 ? (float)si[t & 1][e] : s[t & 1][e];
          acc[t][e] = __builtin_fmaf(se, pe, acc[t][e]);
        }
      };
      constexpr int NV = (MODE == 12 || MODE == 14) ? 32 : 16;
      constexpr int NM = MODE == 13 ? 2 : 1;
      issue(0);
      for (int t = 0; t < 4; ++t) {
        if (t < 3) issue(t + 1);
        __builtin_amdgcn_sched_barrier(0);
        epi(t);
        if constexpr (NM == 2) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, NV / 2, 0);
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, NV / 2, 0);
        } else {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);
        }
      }
    } else if constexpr (MODE >= 15 && MODE <= 17) {
      // packed-f32 epilogues (v_pk_fma_f32 / v_pk_mul_f32 via 2-wide vectors), pipelined
      //   15: fp6 S + f16 P MFMA + 8 pk_fma      16: fp6 S + 8 pk_mul P + 8 pk_fma
      //   17: i8 S + f16 P MFMA + 16 cvt + 8 pk_fma
      typedef float f32x2 __attribute__((ext_vector_type(2)));
      constexpr bool I8 = MODE == 17;
      f32x16 s[2], p[2];
      i32x16 si[2];
      auto issue = [&](int t) {
        KEEP(a8); KEEP(a4);
        if constexpr (I8) si[t & 1] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a4, b4, iz, 0, 0, 0);
        else s[t & 1] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(a8, b8, fz, 2, 2, 0, 127, 0, 127);
        if constexpr (MODE != 16) p[t & 1] = __builtin_amdgcn_mfma_f32_32x32x8f16(h4, h4, fz, 0, 0, 0);
      };
      auto epi = [&](int t) {
        KEEP(da);
        for (int e = 0; e < 16; e += 2) {
          f32x2 se, pe;
          if constexpr (I8) se = f32x2{(float)si[t & 1][e], (float)si[t & 1][e + 1]};
          else se = f32x2{s[t & 1][e], s[t & 1][e + 1]};
          if constexpr (MODE == 16) pe = f32x2{da, da} * f32x2{dbv[e], dbv[e + 1]};
          else pe = f32x2{p[t & 1][e], p[t & 1][e + 1]};
          f32x2 ac = {acc[t][e], acc[t][e + 1]};
          ac = __builtin_elementwise_fma(se, pe, ac);
          acc[t][e] = ac[0];
          acc[t][e + 1] = ac[1];
        }
      };
      issue(0);
      for (int t = 0; t < 4; ++t) {
        if (t < 3) issue(t + 1);
        __builtin_amdgcn_sched_barrier(0);
        epi(t);
      }
    } else if constexpr (MODE == 10) {  // 4 x f16 16x16x16 (P for a 32x32 tile as 4 quarter tiles)
      for (int t = 0; t < 4; ++t) {
        typedef float f32x4 __attribute__((ext_vector_type(4)));
        f32x4 q = {acc[t][0], acc[t][1], acc[t][2], acc[t][3]};
        q = __builtin_amdgcn_mfma_f32_16x16x16f16(h4, h4, q, 0, 0, 0);
        acc[t][0] = q[0]; acc[t][1] = q[1]; acc[t][2] = q[2]; acc[t][3] = q[3];
      }
    }
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int t = 0; t < 4; ++t)
    for (int e = 0; e < 16; ++e) s += acc[t][e] + (float)iacc[t][e];
  if (s == 1.2345f) sink[threadIdx.x] = s;
  if (lane == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

template <int MODE, int W>
static void run_timing1(const char* name, int waves_per_simd, int* src, float* sink, long long* cyc, int ncu) {
  const int iters = 2000;
  const int threads = 256 * waves_per_simd;
  const int blocks = ncu;
  hipLaunchKernelGGL((timing<MODE, W>), dim3(blocks), dim3(threads), 0, 0, 10, src, sink, cyc);
  CHECK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  CHECK(hipEventRecord(e0));
  hipLaunchKernelGGL((timing<MODE, W>), dim3(blocks), dim3(threads), 0, 0, iters, src, sink, cyc);
  CHECK(hipEventRecord(e1));
  CHECK(hipDeviceSynchronize());
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const int nw = blocks * threads / 64;
  std::vector<long long> c(nw);
  CHECK(hipMemcpy(c.data(), cyc, nw * 8, hipMemcpyDeviceToHost));
  double avg = 0;
  for (long long v : c) avg += (double)v;
  avg /= nw;
  const double cyc_it = avg / iters;
  printf("%-44s waves/SIMD=%d  cycles/iter/wave=%7.1f  per-SIMD cycles/iter=%7.1f  clk=%.2f GHz  wall ns/iter/SIMD=%6.1f\n",
         name, waves_per_simd, cyc_it, cyc_it / waves_per_simd, avg / (ms * 1e-3) / 1e9,
         ms * 1e6 / iters / waves_per_simd);
  CHECK(hipEventDestroy(e0));
  CHECK(hipEventDestroy(e1));
}

template <int MODE>
static void run_timing(const char* name, int w, int* src, float* sink, long long* cyc, int ncu) {
  if (w == 1) run_timing1<MODE, 1>(name, 1, src, sink, cyc, ncu);
  else if (w == 2) run_timing1<MODE, 2>(name, 2, src, sink, cyc, ncu);
  else run_timing1<MODE, 4>(name, 4, src, sink, cyc, ncu);
}

int main() {
  int ncu = 0;
  hipDeviceProp_t prop;
  CHECK(hipGetDeviceProperties(&prop, 0));
  ncu = prop.multiProcessorCount;
  printf("device %s, %d CUs\n", prop.gcnArchName, ncu);
  layout_check();
  int* src;
  float* sink;
  long long* cyc;
  CHECK(hipMalloc(&src, 4096 * 4));
  std::vector<int> h(4096);
  for (int i = 0; i < 4096; ++i) h[i] = (int)(((unsigned)i * 2654435761u) >> 7) & 0x3f3f3f3f;
  CHECK(hipMemcpy(src, h.data(), 4096 * 4, hipMemcpyHostToDevice));
  CHECK(hipMalloc(&sink, 4096 * 4));
  CHECK(hipMalloc(&cyc, ncu * 8 * 8));
  for (int w : {1, 2, 4}) {
    run_timing<0>("4x i8 32x32x32", w, src, sink, cyc, ncu);
    run_timing<1>("4x f16 32x32x8", w, src, sink, cyc, ncu);
    run_timing<3>("4x f16 32x32x16", w, src, sink, cyc, ncu);
    run_timing<2>("4x fp6 scaled 32x32x64", w, src, sink, cyc, ncu);
    run_timing<10>("4x f16 16x16x16", w, src, sink, cyc, ncu);
    run_timing<7>("64 v_fma (VALU only)", w, src, sink, cyc, ncu);
    run_timing<4>("4x [i8 S + f16 P + cvt + fma]", w, src, sink, cyc, ncu);
    run_timing<9>("4x [i8 S + cvt + fma, P in regs]", w, src, sink, cyc, ncu);
    run_timing<5>("4x [fp6 S + f16 P + fma]", w, src, sink, cyc, ncu);
    run_timing<6>("4x [fp6 S + VALU P + fma]", w, src, sink, cyc, ncu);
    run_timing<8>("4x [fp6 S + fma, P in regs]", w, src, sink, cyc, ncu);
    run_timing<11>("pipelined 4x [fp6 S + fma, P regs]", w, src, sink, cyc, ncu);
    run_timing<12>("pipelined 4x [fp6 S + VALU P + fma]", w, src, sink, cyc, ncu);
    run_timing<13>("pipelined 4x [fp6 S + f16 P + fma]", w, src, sink, cyc, ncu);
    run_timing<14>("pipelined 4x [i8 S + cvt + fma, P regs]", w, src, sink, cyc, ncu);
    run_timing<15>("pipelined 4x [fp6 S + f16 P + pk_fma]", w, src, sink, cyc, ncu);
    run_timing<16>("pipelined 4x [fp6 S + pk_mul P + pk_fma]", w, src, sink, cyc, ncu);
    run_timing<17>("pipelined 4x [i8 S + f16 P + cvt + pk_fma]", w, src, sink, cyc, ncu);
  }
  return 0;
}
