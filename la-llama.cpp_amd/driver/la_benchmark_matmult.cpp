// la-benchmark-matmult for the MI355X lamm backend.
//
// The reference's benchmark (AyiStar/la-llama.cpp src/la-benchmark-matmult.cpp) builds
// ggml_mul_mat graphs and times ggml_graph_compute on the CPU.  This driver keeps its
// command line (-t/-i/-d, test/utils.py:21-24), its shapes (K=11008, M=4096, N=128; the
// LAMM_DEBUG shape K=4096, M=33, N=18 with --debug, :173-183), its inputs (constant 1.0 /
// 1.5 / 2.0, or srand(0) uniform values under --debug, :220-251), its result check (the
// sum of C within 1e-2 of the analytic sum, else "ABORT" and exit 1, :369-381) and its
// output (per-iteration table and the "Average <gflops>" line that
// test/test_matmult_performance.py:42 parses, :334-391) -- and runs the timed step on the
// GPU through liblamm_hip.so's C ABI:
//   one step = quantize the F32 activations on the GPU (ggml's INIT phase, the AVX2
//   from_float flavour, LC/ggml.c:10865-10887) + lamm_hip_matmul (the COMPUTE phase),
//   timed with HIP events on the stream (inputs resident in HBM, as the reference's are in
//   host RAM).
// The reference alternates two weight matrices (g1 timed, g2 untimed) to push g1 out of
// the CPU caches (:311-316, :383-385); here the timed step rotates over R device copies of
// the quantized weights (default: enough copies for 512 MiB, twice the 256 MiB Infinity
// Cache) and the untimed g2 step multiplies the second matrix, so each timed call reads its
// weights from HBM.
// Extra flags: -M/-N/-K (shape), -r R (weight copies), -s (weight-stationary handles:
// lamm_hip_weights_create once, lamm_hip_matmul_weights per step).
// -t is accepted and printed for compatibility; the GPU does not use host threads.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <strings.h>
#include <vector>

#include "lamm_hip.h"

namespace {

struct DType { const char* name; int type; };
// the reference's dtype table (:26-36); f16 is one of this backend's extra weight types
const DType kTypes[] = {{"f32", 0},  {"f16", 1},  {"q2_k", 10}, {"q4_0", 2},  {"q4_1", 3},
                        {"q4_k", 12}, {"q5_0", 6}, {"q5_1", 7},  {"q5_k", 13}, {"q6_k", 14}, {"q8_0", 8}};

const char* type_name(int t) {
  for (const DType& d : kTypes)
    if (d.type == t) return d.name;
  return "?";
}

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    fprintf(stderr, "la-benchmark-matmult: %s: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}
void lamm_ok(int rc, const char* what) {
  if (rc != LAMM_OK) {
    fprintf(stderr, "la-benchmark-matmult: %s failed (%d): %s\n", what, rc, lamm_hip_last_error());
    exit(1);
  }
}

struct Params {
  int n_threads = 1, n_iterations = 10, type = 0, copies = 0;
  int M = -1, N = -1, K = -1;
  bool debug = false, stationary = false;
};

void usage(const char* argv0, const Params& p) {
  fprintf(stderr, "usage: %s [options]\n\noptions:\n", argv0);
  fprintf(stderr, "  -h, --help            show this help message and exit\n");
  fprintf(stderr, "  -t N, --threads N     number of threads (accepted, unused by the GPU) (default: %d)\n", p.n_threads);
  fprintf(stderr, "  -i N, --iter N        number of iterations (default: %d)\n", p.n_iterations);
  fprintf(stderr, "  -d T, --dtype T       weight type: f32 f16 q2_k q4_0 q4_1 q4_k q5_0 q5_1 q5_k q6_k q8_0 (default: f32)\n");
  fprintf(stderr, "  --debug               LAMM_DEBUG shape (K=4096 M=33 N=18) with random inputs\n");
  fprintf(stderr, "  -M m -N n -K k        override the shape (K: multiple of 256 for k-quants, 32 otherwise)\n");
  fprintf(stderr, "  -r R                  device copies of the weights rotated by the timed step\n");
  fprintf(stderr, "  -s                    weight-stationary handles (lamm_hip_weights_*)\n\n");
}

int parse_type(const char* s) {
  for (const DType& d : kTypes)
    if (strcasecmp(s, d.name) == 0) return d.type;
  printf("Unknonw type name: %s\n", s);   // the reference's message (:81)
  exit(1);
}

// one weight matrix on the device: R row-padded copies of the quantized rows
struct Weights {
  int type = 0, kb = 0;
  int64_t ld = 0;             // row pitch in blocks (16-byte aligned rows)
  size_t bytes = 0;           // one copy
  std::vector<void*> copy;
  std::vector<lamm_weights*> handle;
};

// f32 host rows (M x K) -> `copies` device copies of `type` rows, quantized on the GPU
// (ggml_quantize_chunk, :294-303: the reference quantizes outside the timed loop too)
Weights make_weights(const std::vector<float>& host, int type, int M, int K, int copies, bool stationary,
                     hipStream_t s) {
  Weights w;
  w.type = type;
  const int bl = lamm_blck_size(type);
  const size_t bpb = lamm_type_size(type);
  w.kb = K / bl;
  w.ld = w.kb;
  while ((w.ld * bpb) % 16) ++w.ld;   // device rows need 16-byte pitches (q2_K, q6_K rows are not)
  w.bytes = (size_t)w.ld * bpb * M;
  float* dx = nullptr;
  hip_ok(hipMalloc(&dx, host.size() * sizeof(float)), "hipMalloc(f32 weights)");
  hip_ok(hipMemcpy(dx, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice), "upload weights");
  void* first = nullptr;
  hip_ok(hipMalloc(&first, w.bytes + 256), "hipMalloc(weights)");
  // on s, like the copy / quantizer that fill it: a null-stream hipMemset is not ordered with a
  // non-blocking stream and could land after them (it once zeroed part of the F32 weights)
  hip_ok(hipMemsetAsync(first, 0, w.bytes + 256, s), "hipMemsetAsync");
  if (type == 0) {
    hip_ok(hipMemcpy2DAsync(first, w.ld * 4, dx, (size_t)K * 4, (size_t)K * 4, M, hipMemcpyDeviceToDevice, s), "copy f32");
  } else {
    lamm_ok(lamm_hip_quantize(type, 0, dx, K, first, w.ld, K, M, s), "lamm_hip_quantize(weights)");
  }
  hip_ok(hipStreamSynchronize(s), "quantize weights");
  hip_ok(hipFree(dx), "hipFree");
  w.copy.push_back(first);
  for (int r = 1; r < copies; ++r) {
    void* p = nullptr;
    hip_ok(hipMalloc(&p, w.bytes + 256), "hipMalloc(weight copy)");
    hip_ok(hipMemcpyAsync(p, first, w.bytes, hipMemcpyDeviceToDevice, s), "copy weights");
    w.copy.push_back(p);
  }
  if (stationary) {
    for (void* p : w.copy) {
      lamm_matrix A{p, type, M, w.kb, w.ld};
      lamm_weights* h = nullptr;
      lamm_ok(lamm_hip_weights_create(&A, 1, 1, 0, 0, s, &h), "lamm_hip_weights_create");
      w.handle.push_back(h);
    }
  }
  hip_ok(hipStreamSynchronize(s), "weight copies");
  return w;
}

struct Activations {
  int vtype = 0, N = 0, K = 0;
  int64_t ld = 0;   // blocks
  float* x = nullptr;
  void* q = nullptr;
};

Activations make_activations(const std::vector<float>& host, int wtype, int N, int K) {
  Activations b;
  b.vtype = lamm_vec_dot_type(wtype);
  b.N = N;
  b.K = K;
  b.ld = K / lamm_blck_size(b.vtype);
  hip_ok(hipMalloc(&b.x, host.size() * sizeof(float)), "hipMalloc(f32 activations)");
  hip_ok(hipMemcpy(b.x, host.data(), host.size() * sizeof(float), hipMemcpyHostToDevice), "upload activations");
  if (b.vtype != 0) hip_ok(hipMalloc(&b.q, (size_t)b.ld * lamm_type_size(b.vtype) * N + 256), "hipMalloc(q8)");
  return b;
}

// one ggml_graph_compute of mul_mat(A, B): INIT (quantize src1 on the GPU, AVX2 flavour) +
// COMPUTE (lamm_hip_matmul)
void step(const Weights& w, int r, Activations& b, float* C, int M, hipStream_t s) {
  void* bdata = b.x;
  if (b.vtype != 0) {
    lamm_ok(lamm_hip_quantize(b.vtype, 1, b.x, b.K, b.q, b.ld, b.K, b.N, s), "lamm_hip_quantize(activations)");
    bdata = b.q;
  }
  lamm_matrix Bm{bdata, b.vtype, w.kb, b.N, b.ld};
  lamm_matrix Cm{C, 0, M, b.N, M};
  if (!w.handle.empty()) {
    lamm_ok(lamm_hip_matmul_weights(w.handle[r], &Bm, &Cm, nullptr, s), "lamm_hip_matmul_weights");
  } else {
    lamm_matrix Am{w.copy[r], w.type, M, w.kb, w.ld};
    lamm_ok(lamm_hip_matmul(&Am, &Bm, &Cm, s), "lamm_hip_matmul");
  }
}

double sum_device(const float* C, size_t n) {
  std::vector<float> h(n);
  hip_ok(hipMemcpy(h.data(), C, n * sizeof(float), hipMemcpyDeviceToHost), "download C");
  double sum = 0;   // tensor_sum_elements (:50-60)
  for (float v : h) sum += v;
  return sum;
}

}  // namespace

int main(int argc, char** argv) {
  Params p;
  bool invalid = false;
  std::string arg;
  for (int i = 1; i < argc; i++) {
    arg = argv[i];
    auto next = [&](int& dst) {
      if (++i >= argc) { invalid = true; return; }
      dst = std::stoi(argv[i]);
    };
    if (arg == "-t" || arg == "--threads") next(p.n_threads);
    else if (arg == "-i" || arg == "--iter") next(p.n_iterations);
    else if (arg == "-M") next(p.M);
    else if (arg == "-N") next(p.N);
    else if (arg == "-K") next(p.K);
    else if (arg == "-r") next(p.copies);
    else if (arg == "-s") p.stationary = true;
    else if (arg == "--debug") p.debug = true;
    else if (arg == "-h" || arg == "--help") { usage(argv[0], p); exit(1); }
    else if (arg == "-d" || arg == "--dtype") {
      if (++i >= argc) { invalid = true; break; }
      p.type = parse_type(argv[i]);
    }
    if (invalid) break;
  }
  if (invalid) {
    fprintf(stderr, "error: invalid parameter for argument: %s\n", arg.c_str());
    usage(argv[0], p);
    exit(1);
  }

  if (lamm_hip_device_count() <= 0) {
    fprintf(stderr, "la-benchmark-matmult: no gfx950 device (%s)\n", lamm_hip_last_error());
    return 1;
  }
  hipDeviceProp_t prop;
  hip_ok(hipGetDeviceProperties(&prop, 0), "hipGetDeviceProperties");
  printf("device: %s (%s), %d CUs\n", prop.name, prop.gcnArchName, prop.multiProcessorCount);
  printf("LAMM optimization level = %d\n", lamm_get_opt_level());
  printf("Starting Test\n");
  if (p.debug) printf("Debugging the correctness\n");

  const int sizey = p.M > 0 ? p.M : (p.debug ? 33 : 4096);     // M, rows of A
  const int sizex = p.K > 0 ? p.K : (p.debug ? 4096 : 11008);  // K
  const int sizez = p.N > 0 ? p.N : (p.debug ? 18 : 128);      // N, columns of B
  const int type = p.type;
  const int qk = lamm_blck_size(type);
  if (qk <= 0 || sizex % qk || sizex % 32 || sizey <= 0 || sizez <= 0) {
    fprintf(stderr, "la-benchmark-matmult: K=%d must be a multiple of %d (and 32) for %s\n", sizex, qk > 32 ? qk : 32,
            type_name(type));
    return 1;
  }

  // inputs in ggml's layout: m11/m12 are sizey rows of sizex, m2 is sizez rows of sizex
  std::vector<float> m11((size_t)sizex * sizey), m12((size_t)sizex * sizey), m2((size_t)sizex * sizez);
  double correct = 0.0;
  if (p.debug) {
    std::srand(0);   // the reference's fill order (:221-236): for each k, A rows then B rows
    for (int i = 0; i < sizex; i++) {
      for (int j = 0; j < sizey; j++) {
        m11[(size_t)j * sizex + i] = 1 + static_cast<float>(std::rand() / static_cast<float>(RAND_MAX));
        m12[(size_t)j * sizex + i] = 1.5 + static_cast<float>(std::rand() / static_cast<float>(RAND_MAX));
      }
      for (int j = 0; j < sizez; j++)
        m2[(size_t)j * sizex + i] = 2 + static_cast<float>(std::rand() / static_cast<float>(RAND_MAX));
    }
    // sum_{i,j,k} m11[j][i] * m2[k][i] (:237-245), factorised per k-index in double
    for (int i = 0; i < sizex; i++) {
      double sa = 0, sb = 0;
      for (int j = 0; j < sizey; j++) sa += m11[(size_t)j * sizex + i];
      for (int k = 0; k < sizez; k++) sb += m2[(size_t)k * sizex + i];
      correct += sa * sb;
    }
  } else {
    std::fill(m11.begin(), m11.end(), 1.0f);
    std::fill(m12.begin(), m12.end(), 1.5f);
    std::fill(m2.begin(), m2.end(), 2.0f);
    correct = (sizex * (1.0f * 2.0f)) * ((double)sizey * sizez);
  }
  printf("Theoretical sum of m11xm2 = %6.2f\n", correct);

  hipStream_t s;
  hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  float* C = nullptr;
  hip_ok(hipMalloc(&C, (size_t)sizey * sizez * sizeof(float)), "hipMalloc(C)");

  // ------ F32 demo test (:255-276): the same mul_mat through the F32 path
  printf("\n------ Demo Test - Matrix Mult via F32 code\n");
  printf("n_threads=%i\n", p.n_threads);
  {
    Weights wf = make_weights(m11, 0, sizey, sizex, 1, false, s);
    Activations bf = make_activations(m2, 0, sizez, sizex);
    step(wf, 0, bf, C, sizey, s);
    hip_ok(hipStreamSynchronize(s), "F32 demo");
    const double sum = sum_device(C, (size_t)sizey * sizez);
    printf("%15s: type = %i (%5s) ne = %5d x %5d - Sum of tensor %s is %6.2f\n", "m11xm2", 0, "f32", sizey, sizez,
           "m11xm2", sum);
    if (std::abs(sum - correct) / std::abs(correct) > 1e-4) {
      printf("\nABORT - ERROR in F32 Matrix Multiplication result - expected %6.2f, got %6.2f\n", correct, sum);
      exit(1);
    }
    hip_ok(hipFree(wf.copy[0]), "hipFree");
    hip_ok(hipFree(bf.x), "hipFree");
  }

  // ------ Test - Matrix Mult via <type> code (:282-320)
  printf("\n------ Test - Matrix Mult via %s code\n", type_name(type));
  int copies = p.copies;
  {
    const size_t bpb = lamm_type_size(type);
    int64_t ld = sizex / qk;
    while ((ld * bpb) % 16) ++ld;
    const size_t one = (size_t)ld * bpb * sizey;
    if (copies <= 0) copies = (int)std::min<size_t>(64, std::max<size_t>(1, ((size_t)512 << 20) / one + 1));
  }
  Weights w1 = make_weights(m11, type, sizey, sizex, copies, p.stationary, s);
  Weights w2 = make_weights(m12, type, sizey, sizex, 1, p.stationary, s);
  Activations b = make_activations(m2, type, sizez, sizex);
  printf("weights: %d device copies of %.2f MB (%s rows of %lld blocks)%s\n", copies, w1.bytes / 1e6,
         type_name(type), (long long)w1.ld, p.stationary ? ", weight-stationary handles" : "");

  // ------ do_benchmark (:322-392)
  printf("n_threads=%i\n", p.n_threads);
  const long long flops_per_matrix = (long long)(sizey + sizey) * sizex * sizez;
  printf("Matrix Multiplication of (%i,%i,%i) x (%i,%i,%i) - about %6.2f gFLOPS\n\n", sizex, sizey, 1, sizex, sizez,
         1, 1.0f * flops_per_matrix / 1000 / 1000 / 1000);
  printf("Iteration;NThreads; SizeX; SizeY; SizeZ; Required_FLOPS; Elapsed_u_Seconds; gigaFLOPS\n");
  printf("=====================================================================================\n");

  hipEvent_t e0, e1;
  hip_ok(hipEventCreate(&e0), "hipEventCreate");
  hip_ok(hipEventCreate(&e1), "hipEventCreate");
  step(w1, 0, b, C, sizey, s);   // warm-up: code objects loaded, workspaces allocated
  step(w2, 0, b, C, sizey, s);
  hip_ok(hipStreamSynchronize(s), "warm-up");
  double gflops_sum = 0;
  for (int i = 0; i < p.n_iterations; i++) {
    hip_ok(hipEventRecord(e0, s), "hipEventRecord");
    step(w1, i % copies, b, C, sizey, s);
    hip_ok(hipEventRecord(e1, s), "hipEventRecord");
    hip_ok(hipEventSynchronize(e1), "hipEventSynchronize");
    float ms = 0;
    hip_ok(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
    const double usec = ms * 1e3;
    const double gflops = (double)flops_per_matrix / usec / 1000.0;
    gflops_sum += gflops;
    printf("%9i;%8i;%6i;%6i;%6i;%15lli;%18.2f;%10.2f\n", i, p.n_threads, sizex, sizey, sizez, flops_per_matrix, usec,
           gflops);

    // the result must be in the right ballpark (:369-381)
    const double sum = sum_device(C, (size_t)sizey * sizez);
    const double delta = std::abs(sum - correct) / std::abs(correct);
    const double allowed = 1e-2;
    if (delta > allowed) {
      printf("\nABORT - ERROR in Matrix Multiplication result - expected %6.2f, got %6.2f (delta %.3f%% > allowed_delta %.3f%%)\n",
             correct, sum, delta * 100, allowed * 100);
      exit(1);
    }
    step(w2, 0, b, C, sizey, s);   // the untimed g2 graph (:383-385)
    hip_ok(hipStreamSynchronize(s), "g2");
  }
  printf("\n");
  printf("Average%78.2f\n", gflops_sum / ((double)p.n_iterations));
  printf("=====================================================================================\n");

  for (lamm_weights* h : w1.handle) lamm_hip_weights_destroy(h);
  for (lamm_weights* h : w2.handle) lamm_hip_weights_destroy(h);
  for (void* q : w1.copy) hip_ok(hipFree(q), "hipFree");
  for (void* q : w2.copy) hip_ok(hipFree(q), "hipFree");
  hip_ok(hipFree(b.x), "hipFree");
  if (b.q) hip_ok(hipFree(b.q), "hipFree");
  hip_ok(hipFree(C), "hipFree");
  hip_ok(hipStreamDestroy(s), "hipStreamDestroy");
  return 0;
}
