// llama-matmul-bench: the weight-matmul workload of one Llama-7B step (BASELINE config 5's
// model) through liblamm_hip.so, on one GPU.
//
// What llama.cpp-b2430 sends to the lamm hook per token step (build_llama
// LC/llama.cpp:5708-5830): per layer wq, wk, wv, wo (4096 x 4096), ffn_gate, ffn_up
// (11008 x 4096), ffn_down (4096 x 11008), each preceded by the INIT quantization of its F32
// activations (LC/ggml.c:10865-10887; wq/wk/wv share one, as do gate/up), and per step the
// Q6_K output.weight (32000 x 4096: llama.cpp's quant policy for Q4_0 models,
// LC/llama.cpp:11731-11742).  This tool runs exactly that sequence of lamm_hip_quantize +
// lamm_hip_matmul calls over 32 layers of distinct synthetic weights (quantized on the GPU
// from random F32 values), captured once into a hipGraph and replayed.  It is NOT the whole
// model: attention (F16 KV-cache matmuls, softmax), RMSNorm, RoPE, SiLU and the residual adds
// are left out, so the result is an upper bound on tok/s set by the weight matmuls (which
// the reference's profiling puts at > 90 % of CPU inference time, README.md:150).
// Each matmul's input is the previous matmul's output (re-quantized), as in the model.
//
// usage: llama-matmul-bench [-d q4_0] [-n tokens per step] [-i replays] [-l layers]
//                           [--no-graph] [-s] [--output-type q6_k] [--unfused] [--batch-proj]
// --batch-proj stores wq|wk|wv and ffn_gate|ffn_up as slices of one tensor each and runs each
// group as ONE lamm_hip_matmul_batched launch against the shared input (B slice stride 0):
// 4 launches per layer instead of 7 (a GPU-native layout; llama.cpp-b2430 issues 7 mul_mats).
// --chain runs the 7 x 32 single-token GEMVs as ONE lamm_hip_chain launch (lamm_chain.hip: a
// persistent kernel whose waves stream the next op's weight rows while its input is produced;
// ops wait inside the launch only for the op that produces their input), then the output
// projection as its own launch; each layer gets its own output buffers (a chain's outputs may
// not overlap) and layer 0 reads a fixed input.
// --concurrent keeps llama.cpp's 7 separate tensors but forks wk / wv and ffn_up onto side
// streams (parallel branches of the captured graph) -- measured SLOWER (decode 1.88 -> 2.14
// ms): each GEMV grid wants every CU (one 149 KiB-LDS workgroup per CU), so concurrent
// branches only contend; batching (--batch-proj) is the way to share the launch cost.
// Single-token decode steps (N = 1) hand the F32 activations of q8_0/q8_1-typed weights straight to the
// GEMV, which quantizes them while staging (bit-exact with the separate quantizer), and prefill
// steps (N > 8) to the GEMMs, which quantize them in their activation prep;
// --unfused runs the separate lamm_hip_quantize launches instead.
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

void hip_ok(hipError_t e, const char* what) {
  if (e != hipSuccess) {
    fprintf(stderr, "llama-matmul-bench: %s: %s\n", what, hipGetErrorString(e));
    exit(1);
  }
}
void lamm_ok(int rc, const char* what) {
  if (rc != LAMM_OK) {
    fprintf(stderr, "llama-matmul-bench: %s failed (%d): %s\n", what, rc, lamm_hip_last_error());
    exit(1);
  }
}

struct DType { const char* name; int type; };
const DType kTypes[] = {{"f16", 1},  {"q2_k", 10}, {"q4_0", 2},  {"q4_1", 3}, {"q4_k", 12},
                        {"q5_0", 6}, {"q5_1", 7},  {"q5_k", 13}, {"q6_k", 14}, {"q8_0", 8}};
const char* type_name(int t) {
  for (const DType& d : kTypes)
    if (d.type == t) return d.name;
  return "?";
}
int parse_type(const char* s) {
  for (const DType& d : kTypes)
    if (strcasecmp(s, d.name) == 0) return d.type;
  fprintf(stderr, "llama-matmul-bench: unknown type %s\n", s);
  exit(1);
}

// one weight tensor on the device (rows of `type` blocks, 16-byte aligned pitch)
struct Tensor {
  int type = 0, M = 0, K = 0, kb = 0, slices = 1;   // slices: projections sharing one input
  int64_t ld = 0;
  void* data = nullptr;
  lamm_weights* handle = nullptr;
  size_t bytes() const { return (size_t)ld * lamm_type_size(type) * M; }   // one slice
};

// random F32 values (fixed LCG) quantized on the GPU into `copies` distinct tensors
std::vector<Tensor> make_weights(int type, int M, int K, int copies, bool stationary, hipStream_t s,
                                 int slices = 1) {
  std::vector<float> h((size_t)M * K);
  uint32_t st = 0x9e3779b9u ^ (uint32_t)(M * 131 + K);
  for (float& v : h) {
    st = st * 1664525u + 1013904223u;
    v = ((int)(st >> 9) - (1 << 22)) * (1.0f / (1 << 22));   // uniform in [-1, 1)
  }
  const float amp = std::sqrt(3.0f / K);   // unit gain per matmul: activations stay O(1) over 32 layers
  for (float& v : h) v *= amp;
  float* dx = nullptr;
  hip_ok(hipMalloc(&dx, h.size() * 4), "hipMalloc");
  hip_ok(hipMemcpy(dx, h.data(), h.size() * 4, hipMemcpyHostToDevice), "upload");
  std::vector<Tensor> out;
  for (int c = 0; c < copies; ++c) {
    Tensor t;
    t.type = type;
    t.M = M;
    t.K = K;
    t.slices = slices;
    t.kb = K / lamm_blck_size(type);
    t.ld = t.kb;
    while ((t.ld * lamm_type_size(type)) % 16) ++t.ld;
    hip_ok(hipMalloc(&t.data, t.bytes() * slices + 256), "hipMalloc(weights)");
    for (int z = 0; z < slices; ++z)
      lamm_ok(lamm_hip_quantize(type, 0, dx, K, (char*)t.data + z * t.bytes(), t.ld, K, M, s),
              "lamm_hip_quantize(weights)");
    if (stationary) {
      lamm_matrix A{t.data, type, M, t.kb, t.ld};
      lamm_ok(lamm_hip_weights_create(&A, slices, 1, t.bytes(), 0, s, &t.handle), "lamm_hip_weights_create");
    }
    out.push_back(t);
  }
  hip_ok(hipStreamSynchronize(s), "quantize weights");
  hip_ok(hipFree(dx), "hipFree");
  return out;
}

struct Act {   // F32 activations [N][K] and their vec_dot-typed copy
  float* x = nullptr;
  void* q = nullptr;
  int K = 0;
};

struct Model {
  int N = 1;
  // --concurrent: projections that share an input run on forked streams (graph branches)
  hipStream_t side[2] = {nullptr, nullptr};
  hipEvent_t fork = nullptr, join[2] = {nullptr, nullptr};
  std::vector<Tensor> wq, wk, wv, wo, w1, w3, w2, out;
  Act a4096, b4096, c4096, a11008;
  float *q, *k, *v, *o, *g, *u, *d, *logits;
  lamm_chain* chain = nullptr;   // --chain: every layer's 7 GEMVs as one launch
  Act last;                      // --chain: the output projection's input (last layer's down)
};

bool g_fused = true;   // decode (N <= 8): F32 activations straight into the GEMV (INIT fused)

bool fused(int wtype, int N) {
  const int vt = lamm_vec_dot_type(wtype);
  // GEMV: one column only -- with 8 columns every workgroup re-quantizes 8 rows before its
  // first dot and the step gets slower (3.87 -> 4.66 ms at N = 8; N = 1: 2.05 -> 1.89 ms).
  // GEMM (N > 8): the engines quantize F32 rows inside their activation prep, one pass fewer.
  return g_fused && (N == 1 || N > 8) && (vt == 8 || vt == 9);
}

void quantize(int wtype, Act& a, int N, hipStream_t s) {
  const int vt = lamm_vec_dot_type(wtype);
  if (vt == 0 || fused(wtype, N)) return;
  lamm_ok(lamm_hip_quantize(vt, 1, a.x, a.K, a.q, a.K / lamm_blck_size(vt), a.K, N, s), "lamm_hip_quantize(act)");
}

void matmul(const Tensor& w, const Act& a, float* C, int N, hipStream_t s) {
  const int vt = lamm_vec_dot_type(w.type);
  lamm_matrix B{vt == 0 ? (void*)a.x : a.q, vt, w.kb, N, (int64_t)(a.K / lamm_blck_size(vt))};
  if (fused(w.type, N)) B = lamm_matrix{a.x, 0, a.K, N, (int64_t)a.K};
  lamm_matrix Cm{C, 0, w.M, N, w.M};
  // slices > 1: one batched launch, every weight slice against the same B (B slice stride 0)
  const lamm_batch bt{w.slices, 1, w.slices, 1, w.bytes(), 0, 0, 0, (size_t)N * w.M * 4, 0};
  if (w.handle) {
    lamm_ok(lamm_hip_matmul_weights(w.handle, &B, &Cm, &bt, s), "lamm_hip_matmul_weights");
  } else {
    lamm_matrix A{w.data, w.type, w.M, w.kb, w.ld};
    lamm_ok(lamm_hip_matmul_batched(&A, &B, &Cm, &bt, s), "lamm_hip_matmul_batched");
  }
}

// one token step: the mul_mat nodes of build_llama in graph order
void step(Model& m, int layers, hipStream_t s) {
  const int N = m.N;
  if (m.chain) {
    lamm_ok(lamm_hip_chain_run(m.chain, s), "lamm_hip_chain_run");
    quantize(m.out[0].type, m.last, N, s);
    matmul(m.out[0], m.last, m.logits, N, s);
    return;
  }
  for (int l = 0; l < layers; ++l) {
    quantize(m.wq[l].type, m.a4096, N, s);           // attn_norm output -> wq / wk / wv
    if (m.side[0] && m.wq[l].slices == 1) {          // wk / wv on forked streams, joined before wo
      hip_ok(hipEventRecord(m.fork, s), "hipEventRecord");
      for (int b = 0; b < 2; ++b) hip_ok(hipStreamWaitEvent(m.side[b], m.fork, 0), "hipStreamWaitEvent");
      matmul(m.wk[l], m.a4096, m.k, N, m.side[0]);
      matmul(m.wv[l], m.a4096, m.v, N, m.side[1]);
      matmul(m.wq[l], m.a4096, m.q, N, s);
      for (int b = 0; b < 2; ++b) {
        hip_ok(hipEventRecord(m.join[b], m.side[b]), "hipEventRecord");
        hip_ok(hipStreamWaitEvent(s, m.join[b], 0), "hipStreamWaitEvent");
      }
    } else {
      matmul(m.wq[l], m.a4096, m.q, N, s);           // --batch-proj: wq holds wq | wk | wv
      if (m.wq[l].slices == 1) {
        matmul(m.wk[l], m.a4096, m.k, N, s);
        matmul(m.wv[l], m.a4096, m.v, N, s);
      }
    }
    quantize(m.wo[l].type, m.b4096, N, s);           // kqv_out (here: the q projection) -> wo
    matmul(m.wo[l], m.b4096, m.o, N, s);
    quantize(m.w1[l].type, m.c4096, N, s);           // ffn_norm output (here: wo's) -> gate / up
    if (m.side[0] && m.w1[l].slices == 1) {          // ffn_up on a forked stream
      hip_ok(hipEventRecord(m.fork, s), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(m.side[0], m.fork, 0), "hipStreamWaitEvent");
      matmul(m.w3[l], m.c4096, m.u, N, m.side[0]);
      matmul(m.w1[l], m.c4096, m.g, N, s);
      hip_ok(hipEventRecord(m.join[0], m.side[0]), "hipEventRecord");
      hip_ok(hipStreamWaitEvent(s, m.join[0], 0), "hipStreamWaitEvent");
    } else {
      matmul(m.w1[l], m.c4096, m.g, N, s);           // --batch-proj: w1 holds gate | up
      if (m.w1[l].slices == 1) matmul(m.w3[l], m.c4096, m.u, N, s);
    }
    quantize(m.w2[l].type, m.a11008, N, s);          // silu(gate) * up (here: up) -> ffn_down
    matmul(m.w2[l], m.a11008, m.d, N, s);
  }
  quantize(m.out[0].type, m.a4096, N, s);            // result_norm -> output.weight
  matmul(m.out[0], m.a4096, m.logits, N, s);
}

}  // namespace

int main(int argc, char** argv) {
  int type = 2, N = 1, iters = 20, layers = 32, out_type = 14;
  bool graph = true, stationary = false, batch_proj = false, concurrent = false, chain = false;
  for (int i = 1; i < argc; ++i) {
    const std::string a = argv[i];
    auto next = [&]() -> const char* {
      if (++i >= argc) { fprintf(stderr, "missing value for %s\n", a.c_str()); exit(1); }
      return argv[i];
    };
    if (a == "-d") type = parse_type(next());
    else if (a == "-n") N = atoi(next());
    else if (a == "-i") iters = atoi(next());
    else if (a == "-l") layers = atoi(next());
    else if (a == "--output-type") out_type = parse_type(next());
    else if (a == "--no-graph") graph = false;
    else if (a == "-s") stationary = true;
    else if (a == "--unfused") g_fused = false;
    else if (a == "--batch-proj") batch_proj = true;
    else if (a == "--concurrent") concurrent = true;
    else if (a == "--chain") chain = true;
    else {
      fprintf(stderr, "usage: %s [-d q4_0] [-n tokens] [-i replays] [-l layers] [--no-graph] [-s] [--output-type q6_k] [--unfused] [--batch-proj] [--concurrent] [--chain]\n",
              argv[0]);
      return 1;
    }
  }
  if (lamm_hip_device_count() <= 0) {
    fprintf(stderr, "llama-matmul-bench: no gfx950 device (%s)\n", lamm_hip_last_error());
    return 1;
  }
  constexpr int H = 4096, F = 11008, V = 32000;
  hipStream_t s;
  hip_ok(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
  Model m;
  m.N = N;
  if (concurrent) {
    for (int b = 0; b < 2; ++b) {
      hip_ok(hipStreamCreateWithFlags(&m.side[b], hipStreamNonBlocking), "hipStreamCreate");
      hip_ok(hipEventCreateWithFlags(&m.join[b], hipEventDisableTiming), "hipEventCreate");
    }
    hip_ok(hipEventCreateWithFlags(&m.fork, hipEventDisableTiming), "hipEventCreate");
  }
  if (batch_proj) {   // q|k|v and gate|up as slices of one tensor each: 4 launches per layer
    m.wq = make_weights(type, H, H, layers, stationary, s, 3);
    m.w1 = make_weights(type, F, H, layers, stationary, s, 2);
  } else {
    m.wq = make_weights(type, H, H, layers, stationary, s);
    m.wk = make_weights(type, H, H, layers, stationary, s);
    m.wv = make_weights(type, H, H, layers, stationary, s);
    m.w1 = make_weights(type, F, H, layers, stationary, s);
    m.w3 = make_weights(type, F, H, layers, stationary, s);
  }
  m.wo = make_weights(type, H, H, layers, stationary, s);
  m.w2 = make_weights(type, H, F, layers, stationary, s);
  m.out = make_weights(out_type, V, H, 1, stationary, s);
  size_t wbytes = 0;
  double params = 0;
  for (auto* v : {&m.wq, &m.wk, &m.wv, &m.wo, &m.w1, &m.w3, &m.w2, &m.out})
    for (const Tensor& t : *v) {
      wbytes += (size_t)t.kb * lamm_type_size(t.type) * t.M * t.slices;
      params += (double)t.M * t.K * t.slices;
    }

  // activations: F32 rows + a vec_dot-typed buffer large enough for any of the formats
  auto mk_act = [&](Act& a, int K, float* alias) {
    a.K = K;
    a.x = alias;
    hip_ok(hipMalloc(&a.q, (size_t)N * K * 2 + 4096), "hipMalloc(q act)");
  };
  auto mk_out = [&](float*& p, int M) {
    hip_ok(hipMalloc(&p, (size_t)N * M * 4 + 256), "hipMalloc(out)");
    hip_ok(hipMemsetAsync(p, 0, (size_t)N * M * 4 + 256, s), "hipMemsetAsync");   // ordered on s
  };
  mk_out(m.q, 3 * H); mk_out(m.k, H); mk_out(m.v, H); mk_out(m.o, H);
  mk_out(m.g, 2 * F); mk_out(m.u, F); mk_out(m.d, H); mk_out(m.logits, V);
  {   // the first layer's input: random values in the ffn_down output buffer
    std::vector<float> h((size_t)N * H);
    for (size_t i = 0; i < h.size(); ++i) h[i] = std::sin(0.37f * (float)i);
    hip_ok(hipStreamSynchronize(s), "memsets");
    hip_ok(hipMemcpy(m.d, h.data(), h.size() * 4, hipMemcpyHostToDevice), "upload x");
  }
  mk_act(m.a4096, H, m.d);    // layer input = previous layer's ffn_down output
  mk_act(m.b4096, H, m.q);
  mk_act(m.c4096, H, m.o);
  mk_act(m.a11008, F, batch_proj ? m.g + (size_t)N * F : m.u);   // the up projection's output

  std::vector<void*> chain_bufs;
  if (chain) {   // per-layer outputs; layer 0 reads a copy of the first input
    if (batch_proj || N != 1) {
      fprintf(stderr, "llama-matmul-bench: --chain is a single-token path of separate tensors (no --batch-proj, -n 1)\n");
      return 1;
    }
    auto buf = [&](int M) {
      float* p = nullptr;
      hip_ok(hipMalloc(&p, (size_t)M * 4 + 256), "hipMalloc(chain)");
      hip_ok(hipMemset(p, 0, (size_t)M * 4 + 256), "hipMemset(chain)");
      chain_bufs.push_back(p);
      return p;
    };
    float* x = buf(H);
    hip_ok(hipMemcpy(x, m.d, (size_t)H * 4, hipMemcpyDeviceToDevice), "copy x");
    std::vector<lamm_chain_op> ops;
    auto op = [&](const Tensor& w, const float* in, float* out) {
      ops.push_back(lamm_chain_op{lamm_matrix{w.data, w.type, w.M, w.kb, w.ld}, in, out});
    };
    for (int l = 0; l < layers; ++l) {
      float *q = buf(H), *k = buf(H), *v = buf(H), *o = buf(H), *g = buf(F), *u = buf(F), *d = buf(H);
      op(m.wq[l], x, q);
      op(m.wk[l], x, k);
      op(m.wv[l], x, v);
      op(m.wo[l], q, o);
      op(m.w1[l], o, g);
      op(m.w3[l], o, u);
      op(m.w2[l], u, d);
      x = d;
    }
    lamm_ok(lamm_hip_chain_create(ops.data(), (int)ops.size(), &m.chain), "lamm_hip_chain_create");
    mk_act(m.last, H, x);
  }

  printf("llama-matmul-bench: Llama-7B weight matmuls, %d layers, weights %s, output.weight %s, "
         "%.2f GB of weight blocks, %d token(s) per step, %s%s%s\n",
         layers, type_name(type), type_name(out_type), wbytes / 1e9, N, graph ? "hipGraph" : "stream",
         stationary ? ", weight-stationary handles" : "", chain ? ", one chain launch for the layers" : "");

  // warm-up (workspaces reach their final size before capture), then capture one step
  for (int w = 0; w < 2; ++w) step(m, layers, s);
  hip_ok(hipStreamSynchronize(s), "warm-up");
  hipGraphExec_t exec = nullptr;
  if (graph) {
    hipGraph_t g;
    hip_ok(hipStreamBeginCapture(s, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
    step(m, layers, s);
    hip_ok(hipStreamEndCapture(s, &g), "hipStreamEndCapture");
    hip_ok(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0), "hipGraphInstantiate");
    hip_ok(hipGraphDestroy(g), "hipGraphDestroy");
    hip_ok(hipGraphLaunch(exec, s), "hipGraphLaunch");
    hip_ok(hipStreamSynchronize(s), "graph warm-up");
  }
  hipEvent_t e0, e1;
  hip_ok(hipEventCreate(&e0), "hipEventCreate");
  hip_ok(hipEventCreate(&e1), "hipEventCreate");
  hip_ok(hipEventRecord(e0, s), "hipEventRecord");
  for (int it = 0; it < iters; ++it) {
    if (graph) hip_ok(hipGraphLaunch(exec, s), "hipGraphLaunch");
    else step(m, layers, s);
  }
  hip_ok(hipEventRecord(e1, s), "hipEventRecord");
  hip_ok(hipEventSynchronize(e1), "hipEventSynchronize");
  float ms = 0;
  hip_ok(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
  const double t = ms * 1e-3 / iters;
  std::vector<float> lg((size_t)N * V);
  hip_ok(hipMemcpy(lg.data(), m.logits, lg.size() * 4, hipMemcpyDeviceToHost), "download logits");
  double cs = 0;
  for (float v : lg) cs += std::fabs(v);
  if (!std::isfinite(cs)) {
    fprintf(stderr, "llama-matmul-bench: non-finite logits\n");
    return 1;
  }
  if (m.chain) lamm_ok(lamm_hip_chain_status(m.chain), "lamm_hip_chain_status");
  if (m.chain && lamm_hip_chain_trace(m.chain, nullptr, 0)) {   // LAMM_CHAIN_TRACE=1: last launch's phase timeline
    const int nph = lamm_hip_chain_phases(m.chain), w = 2 * nph + 2;
    std::vector<uint64_t> tr(lamm_hip_chain_trace(m.chain, nullptr, 0));
    lamm_hip_chain_trace(m.chain, tr.data(), tr.size());
    const int grid = (int)(tr.size() / w);
    uint64_t t0 = ~0ull;
    for (int g = 0; g < grid; ++g) t0 = std::min(t0, tr[(size_t)g * w]);
    auto col = [&](int k, std::vector<double>& v) {
      v.clear();
      for (int g = 0; g < grid; ++g) v.push_back((tr[(size_t)g * w + k] - t0) * 0.01);   // 100 MHz -> us
      std::sort(v.begin(), v.end());
    };
    std::vector<double> b, e;
    printf("chain trace (us from the first workgroup's start; staging begin min/max, end min/max):\n");
    for (int p = 0; p < nph; ++p) {
      col(1 + 2 * p, b);
      col(2 + 2 * p, e);
      if (p < 8 || p >= nph - 4)
        printf("  phase %3d: begin %8.2f %8.2f  end %8.2f %8.2f\n", p, b.front(), b.back(), e.front(), e.back());
    }
    col(w - 1, e);
    printf("  end: %8.2f %8.2f\n", e.front(), e.back());
  }
  const int launches = m.chain ? 2 : (batch_proj ? 4 : 7) * layers + 1;
  printf("step %.3f ms  |  %.1f tok/s  |  weight stream %.1f GB/s  |  %.1f TFLOP/s  |  %d matmul launches + %d quantizations per step  |  logits |sum| %.4g\n",
         t * 1e3, N / t, wbytes / t / 1e9, 2.0 * params * N / t / 1e12, launches,
         m.chain ? 1 : fused(type, N) ? 1 : 4 * layers + 1, cs);
  printf("{\"tool\": \"llama-matmul-bench\", \"layers\": %d, \"tokens_per_step\": %d, \"ms_per_step\": %.4f, \"tok_per_s\": %.2f, "
         "\"weight_GBps\": %.1f, \"TFLOPs\": %.2f, \"graph\": %s, \"stationary\": %s, \"type\": \"%s\", "
         "\"mode\": \"%s\", \"launches\": %d}\n",
         layers, N, t * 1e3, N / t, wbytes / t / 1e9, 2.0 * params * N / t / 1e12, graph ? "true" : "false",
         stationary ? "true" : "false", type_name(type),
         m.chain ? "chain" : batch_proj ? "batch-proj" : concurrent ? "concurrent" : "separate", launches);
  return 0;
}
