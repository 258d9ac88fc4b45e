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
// Row-sharded multi-GPU form (BASELINE config 5: "weight rows sharded 8xMI355X + RCCL
// all-gather"; the reference's row split over threads, src/lamm_impl.hpp:38-43 / :107-112,
// mapped onto GPUs): every weight's rows split over the ranks (lamm_hip_shard_rows),
// each rank computes its rows of every projection into its full-size output and one
// lamm_hip_allgather_rows per projection gives every rank the whole vector for the next matmul.
//   --shard G [--devices 0,1,..]   one process, G local ranks (lamm_hip_comm_init_all; device ids
//                                  may repeat: the loopback rehearsal on one GPU)
//   --rank r --world w --comm-id HEX [--device d]   one process per GPU (lamm_hip_comm_init_rank)
// --batch-proj in the sharded form stores q|k|v and gate|up as ONE tall weight each (12288 and
// 22016 rows) so their rows shard like any other weight.  The whole step (matmuls + all-gathers)
// is captured into one hipGraph per process.  --dump FILE writes rank 0's logits (f32) after
// the timed replays (bit-for-bit comparison of a sharded run against one GPU).
// --concurrent keeps llama.cpp's 7 separate tensors but forks wk / wv and ffn_up onto side
// streams (parallel branches of the captured graph) -- measured SLOWER (decode 1.88 -> 2.14
// ms): each GEMV grid wants every CU (one 149 KiB-LDS workgroup per CU), so concurrent
// branches only contend; batching (--batch-proj) is the way to share the launch cost.
// Single-token decode steps (N = 1) hand the F32 activations of q8_0/q8_1-typed weights straight to the
// GEMV, which quantizes them while staging (bit-exact with the separate quantizer), and prefill
// steps (N > 8) to the GEMMs, which quantize them in their activation prep;
// --unfused runs the separate lamm_hip_quantize launches instead.
// --ctx P (single GPU, -n 1): a decode step with the attention matmuls too -- per layer the token's
// K row / V column appended to a device-resident F16 KV cache of P cells, KQ and KQV over all P
// cells as batched F16 GEMVs (32 heads per launch), the F32 -> F16 conversions of their src1
// (ggml's INIT) on the GPU: every mul_mat of a llama.cpp decode step, with nothing crossing
// PCIe.  Softmax / RoPE / norms are llama.cpp ops outside the hook and stay out.  --check
// recomputes the last layer's attention on the host from the device buffers after the replays.
#include <execinfo.h>
#include <pthread.h>
#include <hip/hip_runtime.h>
#include <signal.h>
#include <unistd.h>

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
  int64_t r0 = 0, Mfull = 0;   // sharded form: this slab is rows [r0, r0 + M) of a Mfull-row weight
  void* data = nullptr;
  lamm_weights* handle = nullptr;
  size_t bytes() const { return (size_t)ld * lamm_type_size(type) * M; }   // one slice
};

// random F32 values (fixed LCG, seeded by the shape) of an M x K weight
std::vector<float> host_weights(int M, int K) {
  std::vector<float> h((size_t)M * K);
  uint32_t st = 0x9e3779b9u ^ (uint32_t)(M * 131 + K);
  for (float& v : h) {
    st = st * 1664525u + 1013904223u;
    v = ((int)(st >> 9) - (1 << 22)) * (1.0f / (1 << 22));   // uniform in [-1, 1)
  }
  const float amp = std::sqrt(3.0f / K);   // unit gain per matmul: activations stay O(1) over 32 layers
  for (float& v : h) v *= amp;
  return h;
}

// host_weights(M, K) quantized on the GPU into `copies` distinct tensors
std::vector<Tensor> make_weights(int type, int M, int K, int copies, bool stationary, hipStream_t s,
                                 int slices = 1) {
  const std::vector<float> h = host_weights(M, K);
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
  // --ctx P: the attention matmuls over a device-resident F16 KV cache of P cells per layer
  int ctx = 0;
  std::vector<void*> kc, vt;   // per layer: K [head][P][128], V transposed [head][128][P] (b2430)
  void *qh = nullptr, *probs = nullptr, *vrow = nullptr;
  float *scores = nullptr, *kqv = nullptr;
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

// Decode attention of layer l on the device (N = 1, the token at cache cell P - 1): what
// llm_build_kqv sends to the mul_mat hook (LC/llama.cpp:5322-5372) with the KV cache resident on
// the GPU instead of in host memory -- this token's K row and V column appended to the F16 cache
// (the ggml_cpy of k_cur / v_cur, LC/llama.cpp:5252-5270), q to F16 (ggml's INIT of the F16
// matmul), KQ = K . q per head, then KQV = V^T . p per head.  Scale, mask and softmax between
// the two are llama.cpp ops, not mul_mats: the scores go to KQV as its src1 unchanged.
void attention(Model& m, int l, hipStream_t s) {
  constexpr int NH = 32, D = 128, F16 = 1;
  const int P = m.ctx;
  const bool tall = m.wq[l].slices == 3;   // --batch-proj: q | k | v in one output
  const float* k = tall ? m.q + NH * D : m.k;
  const float* v = tall ? m.q + 2 * NH * D : m.v;
  lamm_ok(lamm_hip_quantize(F16, 0, k, D, (char*)m.kc[l] + (size_t)(P - 1) * D * 2, (int64_t)P * D, D, NH, s),
          "K append");
  // V^T column P - 1: the row converted once, then scattered at the cache's row pitch (a strided
  // device copy; ggml's cpy into the transposed view)
  lamm_ok(lamm_hip_quantize(F16, 0, v, NH * D, m.vrow, NH * D, NH * D, 1, s), "V -> f16");
  hip_ok(hipMemcpy2DAsync((char*)m.vt[l] + (size_t)(P - 1) * 2, (size_t)P * 2, m.vrow, 2, 2, NH * D,
                          hipMemcpyDeviceToDevice, s),
         "V append");
  lamm_ok(lamm_hip_quantize(F16, 0, m.q, D, m.qh, D, D, NH, s), "q -> f16");
  const lamm_matrix A{m.kc[l], F16, P, D, D}, B{m.qh, F16, D, 1, D}, C{m.scores, 0, P, 1, P};
  const lamm_batch bt{NH, 1, NH, 1, (size_t)P * D * 2, 0, (size_t)D * 2, 0, (size_t)P * 4, 0};
  lamm_ok(lamm_hip_matmul_batched(&A, &B, &C, &bt, s), "KQ");
  lamm_ok(lamm_hip_quantize(F16, 0, m.scores, P, m.probs, P, P, NH, s), "kq -> f16");
  const lamm_matrix A2{m.vt[l], F16, D, P, P}, B2{m.probs, F16, P, 1, P}, C2{m.kqv, 0, D, 1, D};
  const lamm_batch bt2{NH, 1, NH, 1, (size_t)D * P * 2, 0, (size_t)P * 2, 0, (size_t)D * 4, 0};
  lamm_ok(lamm_hip_matmul_batched(&A2, &B2, &C2, &bt2, s), "KQV");
}

// --check: the last layer's attention of the last replay recomputed on the host from the device
// buffers it used -- the appended K row / V column equal this token's k / v in F16, every score is
// K . q and every kqv value V^T . p (F16 products summed in double), within 1e-3 of sum |a b|
bool check_attention(const Model& m, int l) {
  constexpr int NH = 32, D = 128, H = NH * D;
  const int P = m.ctx;
  auto down = [](const void* src, size_t bytes) {
    std::vector<unsigned char> v(bytes);
    hip_ok(hipMemcpy(v.data(), src, bytes, hipMemcpyDeviceToHost), "download (check)");
    return v;
  };
  auto h2f = [](const unsigned char* p) {
    _Float16 h;
    memcpy(&h, p, 2);
    return (double)h;
  };
  const bool tall = m.wq[l].slices == 3;
  const auto kc = down(m.kc[l], (size_t)H * P * 2), vt = down(m.vt[l], (size_t)H * P * 2);
  const auto qh = down(m.qh, (size_t)H * 2), pr = down(m.probs, (size_t)NH * P * 2);
  const auto sc = down(m.scores, (size_t)NH * P * 4), kqv = down(m.kqv, (size_t)H * 4);
  const auto kv = down(tall ? m.q + H : m.k, (size_t)H * 4), vv = down(tall ? m.q + 2 * H : m.v, (size_t)H * 4);
  const auto qf = down(m.q, (size_t)H * 4);
  auto f32 = [](const std::vector<unsigned char>& v, size_t i) {
    float f;
    memcpy(&f, &v[4 * i], 4);
    return f;
  };
  double worst = 0;
  int bad_cells = 0;
  for (int h = 0; h < NH; ++h) {
    for (int d = 0; d < D; ++d) {   // the appended cell and q, as F16 of this token's values
      const size_t i = (size_t)h * D + d;
      bad_cells += h2f(&kc[(((size_t)h * P + P - 1) * D + d) * 2]) != (double)(_Float16)f32(kv, i);
      bad_cells += h2f(&vt[(((size_t)h * D + d) * P + P - 1) * 2]) != (double)(_Float16)f32(vv, i);
      bad_cells += h2f(&qh[i * 2]) != (double)(_Float16)f32(qf, i);
    }
    for (int p = 0; p < P; ++p) {   // KQ
      double s = 0, a = 0;
      for (int d = 0; d < D; ++d) {
        const double x = h2f(&kc[(((size_t)h * P + p) * D + d) * 2]) * h2f(&qh[((size_t)h * D + d) * 2]);
        s += x;
        a += std::fabs(x);
      }
      worst = std::max(worst, std::fabs(f32(sc, (size_t)h * P + p) - s) / (a + 1e-30));
      bad_cells += h2f(&pr[((size_t)h * P + p) * 2]) != (double)(_Float16)f32(sc, (size_t)h * P + p);
    }
    for (int d = 0; d < D; ++d) {   // KQV
      double s = 0, a = 0;
      for (int p = 0; p < P; ++p) {
        const double x = h2f(&vt[(((size_t)h * D + d) * P + p) * 2]) * h2f(&pr[((size_t)h * P + p) * 2]);
        s += x;
        a += std::fabs(x);
      }
      worst = std::max(worst, std::fabs(f32(kqv, (size_t)h * D + d) - s) / (a + 1e-30));
    }
  }
  const bool ok = bad_cells == 0 && worst < 1e-3;
  printf("attention check (layer %d, %d cells): %s, max rel err %.3e, F16 conversions off %d\n", l, P,
         ok ? "ok" : "FAILED", worst, bad_cells);
  return ok;
}

// one token step: the mul_mat nodes of build_llama in graph order
void step(Model& m, int layers, hipStream_t s) {
  const int N = m.N;
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
    if (m.ctx > 0) attention(m, l, s);               // kqv_out -> wo
    quantize(m.wo[l].type, m.b4096, N, s);           // kqv_out (without --ctx: the q projection) -> wo
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

// ---------------------------------------------------------------- row-sharded form
constexpr int kShardAlign = 16;   // row granularity of the split (lamm_hip_shard_rows)

// rows [r0, r0 + rows) of a `rep` x M-row weight stacked from host_weights(M, K) (rep = 3: q|k|v,
// 2: gate|up), quantized on this device into `copies` distinct slabs
std::vector<Tensor> make_slabs(int type, int M, int K, int rep, int64_t r0, int64_t rows, int copies, bool stationary,
                               hipStream_t s) {
  const std::vector<float> h = host_weights(M, K);
  std::vector<float> part((size_t)std::max<int64_t>(rows, 1) * K);
  for (int64_t i = 0; i < rows; ++i)
    memcpy(&part[(size_t)i * K], &h[(size_t)((r0 + i) % M) * K], (size_t)K * 4);
  float* dx = nullptr;
  hip_ok(hipMalloc(&dx, part.size() * 4), "hipMalloc");
  hip_ok(hipMemcpy(dx, part.data(), part.size() * 4, hipMemcpyHostToDevice), "upload");
  std::vector<Tensor> out;
  for (int c = 0; c < copies; ++c) {
    Tensor t;
    t.type = type;
    t.M = (int)rows;
    t.K = K;
    t.kb = K / lamm_blck_size(type);
    t.ld = t.kb;
    while ((t.ld * lamm_type_size(type)) % 16) ++t.ld;
    t.r0 = r0;
    t.Mfull = (int64_t)rep * M;
    hip_ok(hipMalloc(&t.data, t.bytes() + 256), "hipMalloc(weights)");
    if (rows > 0) {
      lamm_ok(lamm_hip_quantize(type, 0, dx, K, t.data, t.ld, K, (int)rows, s), "lamm_hip_quantize(weights)");
      if (stationary) {
        lamm_matrix A{t.data, type, (int)rows, t.kb, t.ld};
        lamm_ok(lamm_hip_weights_create(&A, 1, 1, 0, 0, s, &t.handle), "lamm_hip_weights_create");
      }
    }
    out.push_back(t);
  }
  hip_ok(hipStreamSynchronize(s), "quantize weights");
  hip_ok(hipFree(dx), "hipFree");
  return out;
}

// one local rank of a sharded run: its device, stream, weight slabs, and full-size vectors
struct Rank {
  int dev = 0, grank = 0;
  hipStream_t s = nullptr;
  std::vector<Tensor> wq, wk, wv, wo, w1, w3, w2, out;   // tall form: wq = q|k|v, w1 = gate|up
  float *q = nullptr, *k = nullptr, *v = nullptr, *o = nullptr, *g = nullptr, *u = nullptr, *d = nullptr,
        *logits = nullptr;
  Act a4096, b4096, c4096, a11008;
};

// this rank's rows of C = w . a, written at their place in the full output C (column stride Mfull)
void matmul_rows(const Tensor& w, Act& a, float* C, int N, hipStream_t s) {
  if (w.M == 0) return;
  quantize(w.type, a, N, s);
  const int vt = lamm_vec_dot_type(w.type);
  lamm_matrix B{vt == 0 ? (void*)a.x : a.q, vt, w.kb, N, (int64_t)(a.K / lamm_blck_size(vt))};
  if (fused(w.type, N)) B = lamm_matrix{a.x, 0, a.K, N, (int64_t)a.K};
  lamm_matrix Cm{C + w.r0, 0, w.M, N, w.Mfull};
  if (w.handle) {
    lamm_ok(lamm_hip_matmul_weights(w.handle, &B, &Cm, nullptr, s), "lamm_hip_matmul_weights");
  } else {
    lamm_matrix A{w.data, w.type, w.M, w.kb, w.ld};
    lamm_ok(lamm_hip_matmul(&A, &B, &Cm, s), "lamm_hip_matmul");
  }
}

// every local rank: its rows of one projection; then one all-gather of that output
template <class W, class In, class Out>
void project(std::vector<Rank>& R, lamm_comm* comm, int N, W wsel, In insel, Out outsel) {
  std::vector<const float*> slabs;
  std::vector<int64_t> ld;
  std::vector<float*> Cs;
  std::vector<void*> streams;
  int64_t Mfull = 0;
  for (Rank& r : R) {
    hip_ok(hipSetDevice(r.dev), "hipSetDevice");
    const Tensor& w = wsel(r);
    float* C = outsel(r);
    matmul_rows(w, insel(r), C, N, r.s);
    Mfull = w.Mfull;
    slabs.push_back(C + w.r0);
    ld.push_back(w.Mfull);
    Cs.push_back(C);
    streams.push_back(r.s);
  }
  lamm_ok(lamm_hip_allgather_rows(comm, slabs.data(), ld.data(), Cs.data(), Mfull, Mfull, N, kShardAlign,
                                  streams.data()),
          "lamm_hip_allgather_rows");
}

void step_sharded(std::vector<Rank>& R, lamm_comm* comm, int layers, int N, bool tall) {
  for (int l = 0; l < layers; ++l) {
    project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.wq[l]; }, [](Rank& r) -> Act& { return r.a4096; },
            [](Rank& r) { return r.q; });
    if (!tall) {
      project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.wk[l]; }, [](Rank& r) -> Act& { return r.a4096; },
              [](Rank& r) { return r.k; });
      project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.wv[l]; }, [](Rank& r) -> Act& { return r.a4096; },
              [](Rank& r) { return r.v; });
    }
    project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.wo[l]; }, [](Rank& r) -> Act& { return r.b4096; },
            [](Rank& r) { return r.o; });
    project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.w1[l]; }, [](Rank& r) -> Act& { return r.c4096; },
            [](Rank& r) { return r.g; });
    if (!tall)
      project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.w3[l]; }, [](Rank& r) -> Act& { return r.c4096; },
              [](Rank& r) { return r.u; });
    project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.w2[l]; }, [](Rank& r) -> Act& { return r.a11008; },
            [](Rank& r) { return r.d; });
  }
  project(R, comm, N, [](Rank& r) -> const Tensor& { return r.out[0]; }, [](Rank& r) -> Act& { return r.a4096; },
          [](Rank& r) { return r.logits; });
}

struct ShardOpts {
  int world = 0;            // > 0: sharded
  std::vector<int> devices; // local ranks' devices (--shard / --devices), or the one device (--rank)
  int rank = -1;            // >= 0: one rank per process
  std::string comm_id;      // hex (2 * LAMM_COMM_ID_BYTES digits) or "auto" (world 1 only)
  std::string dump;
  std::string dump_q;       // the first projection's gathered output (identical inputs at any G)
  bool graph = true;        // --no-graph: eager replays
};

int run_sharded(const ShardOpts& o, int type, int out_type, int N, int iters, int layers, bool stationary, bool tall) {
  constexpr int H = 4096, F = 11008, V = 32000;
  lamm_comm* comm = nullptr;
  std::vector<Rank> R(o.devices.size());
  if (o.rank >= 0) {
    unsigned char id[LAMM_COMM_ID_BYTES] = {0};
    if (o.comm_id == "auto") {
      if (o.world != 1) { fprintf(stderr, "llama-matmul-bench: --comm-id auto needs --world 1\n"); return 1; }
      lamm_ok(lamm_hip_comm_unique_id(id), "lamm_hip_comm_unique_id");
    } else {
      if (o.comm_id.size() != 2 * LAMM_COMM_ID_BYTES) { fprintf(stderr, "llama-matmul-bench: bad --comm-id\n"); return 1; }
      for (int i = 0; i < LAMM_COMM_ID_BYTES; ++i) id[i] = (unsigned char)std::stoi(o.comm_id.substr(2 * i, 2), nullptr, 16);
    }
    if (lamm_hip_comm_init_rank(&comm, o.world, o.rank, id, o.devices[0]) != LAMM_OK) {
      fprintf(stderr, "llama-matmul-bench: lamm_hip_comm_init_rank: %s\n", lamm_hip_comm_last_error());
      return 1;
    }
    R[0].grank = o.rank;
  } else {
    if (lamm_hip_comm_init_all(&comm, (int)o.devices.size(), o.devices.data()) != LAMM_OK) {
      fprintf(stderr, "llama-matmul-bench: lamm_hip_comm_init_all: %s\n", lamm_hip_comm_last_error());
      return 1;
    }
    for (size_t i = 0; i < R.size(); ++i) R[i].grank = (int)i;
  }
  const int world = o.world;
  size_t wbytes = 0;
  double params = 0;
  for (size_t i = 0; i < R.size(); ++i) {
    Rank& r = R[i];
    r.dev = o.devices[i];
    hip_ok(hipSetDevice(r.dev), "hipSetDevice");
    hip_ok(hipStreamCreateWithFlags(&r.s, hipStreamNonBlocking), "hipStreamCreate");
    auto slabs = [&](int ty, int M, int K, int rep, int copies) {
      int64_t r0, rows;
      lamm_hip_shard_rows((int64_t)rep * M, world, r.grank, kShardAlign, &r0, &rows);
      auto v = make_slabs(ty, M, K, rep, r0, rows, copies, stationary, r.s);
      if (i == 0) {   // whole-model bytes / params (every rank's slabs add up to one model)
        wbytes += (size_t)v.size() * (size_t)(K / lamm_blck_size(ty)) * lamm_type_size(ty) * (size_t)rep * M;
        params += (double)v.size() * rep * M * K;
      }
      return v;
    };
    if (tall) {
      r.wq = slabs(type, H, H, 3, layers);
      r.w1 = slabs(type, F, H, 2, layers);
    } else {
      r.wq = slabs(type, H, H, 1, layers);
      r.wk = slabs(type, H, H, 1, layers);
      r.wv = slabs(type, H, H, 1, layers);
      r.w1 = slabs(type, F, H, 1, layers);
      r.w3 = slabs(type, F, H, 1, layers);
    }
    r.wo = slabs(type, H, H, 1, layers);
    r.w2 = slabs(type, H, F, 1, layers);
    r.out = slabs(out_type, V, H, 1, 1);
    auto mk_out = [&](float*& p, int M) {
      hip_ok(hipMalloc(&p, (size_t)N * M * 4 + 256), "hipMalloc(out)");
      hip_ok(hipMemsetAsync(p, 0, (size_t)N * M * 4 + 256, r.s), "hipMemsetAsync");
    };
    mk_out(r.q, 3 * H); mk_out(r.k, H); mk_out(r.v, H); mk_out(r.o, H);
    mk_out(r.g, 2 * F); mk_out(r.u, F); mk_out(r.d, H); mk_out(r.logits, V);
    std::vector<float> x((size_t)N * H);
    for (size_t j = 0; j < x.size(); ++j) x[j] = std::sin(0.37f * (float)j);   // the single-GPU run's input
    hip_ok(hipStreamSynchronize(r.s), "memsets");
    hip_ok(hipMemcpy(r.d, x.data(), x.size() * 4, hipMemcpyHostToDevice), "upload x");
    auto mk_act = [&](Act& a, int K, float* alias) {
      a.K = K;
      a.x = alias;
      hip_ok(hipMalloc(&a.q, (size_t)N * K * 2 + 4096), "hipMalloc(q act)");
    };
    // tall form at N > 1: q|k|v rows interleave per column ([N][12288]), so wo's input is not the
    // first N x 4096 block -- the bench only needs a well-formed input, so it reads those floats
    mk_act(r.a4096, H, r.d);
    mk_act(r.b4096, H, r.q);
    mk_act(r.c4096, H, r.o);
    mk_act(r.a11008, F, tall ? r.g + (size_t)F : r.u);
  }
  printf("llama-matmul-bench: Llama-7B weight matmuls, %d layers, weights %s, output.weight %s, %.2f GB of weight "
         "blocks, %d token(s) per step, rows sharded over %d rank(s) (%s; this process: %zu), hipGraph%s%s\n",
         layers, type_name(type), type_name(out_type), wbytes / 1e9, N, world,
         o.rank >= 0 ? "one process per GPU, RCCL" : (lamm_hip_comm_local_ranks(comm) > 1 ? "one process" : "one rank"),
         R.size(), stationary ? ", weight-stationary handles" : "", tall ? ", q|k|v and gate|up as tall weights" : "");
  for (int w = 0; w < 2; ++w) step_sharded(R, comm, layers, N, tall);
  for (Rank& r : R) {
    hip_ok(hipSetDevice(r.dev), "hipSetDevice");
    hip_ok(hipStreamSynchronize(r.s), "warm-up");
  }
  // one graph: the step on rank 0's stream, the other local ranks' streams forked from it (any number
  // of local ranks: the loopback all-gather joins the streams by fan-in / fan-out through rank 0's
  // stream, every event waited on as soon as it is recorded -- round 4's all-pairs waits on reused
  // events sent HIP's graph code into unbounded recursion at 8 ranks and forced eager replays there).
  // --no-graph: eager replays.
  const bool graphed = o.graph;
  if (!graphed) {
    printf("llama-matmul-bench: %zu local ranks: eager replays (no hipGraph)\n", R.size());
    step_sharded(R, comm, layers, N, tall);
    for (Rank& r : R) {
      hip_ok(hipSetDevice(r.dev), "hipSetDevice");
      hip_ok(hipStreamSynchronize(r.s), "eager warm-up");
    }
  }
  hip_ok(hipSetDevice(R[0].dev), "hipSetDevice");
  hipEvent_t fork;
  std::vector<hipEvent_t> join(R.size());
  hip_ok(hipEventCreateWithFlags(&fork, hipEventDisableTiming), "hipEventCreate");
  for (size_t i = 1; i < R.size(); ++i) {
    hip_ok(hipSetDevice(R[i].dev), "hipSetDevice");
    hip_ok(hipEventCreateWithFlags(&join[i], hipEventDisableTiming), "hipEventCreate");
  }
  hip_ok(hipSetDevice(R[0].dev), "hipSetDevice");
  hipGraph_t g;
  hipGraphExec_t exec = nullptr;
  if (graphed) {
  hip_ok(hipStreamBeginCapture(R[0].s, hipStreamCaptureModeRelaxed), "hipStreamBeginCapture");
  hip_ok(hipEventRecord(fork, R[0].s), "hipEventRecord");
  for (size_t i = 1; i < R.size(); ++i) hip_ok(hipStreamWaitEvent(R[i].s, fork, 0), "hipStreamWaitEvent");
  step_sharded(R, comm, layers, N, tall);
  for (size_t i = 1; i < R.size(); ++i) {
    hip_ok(hipSetDevice(R[i].dev), "hipSetDevice");
    hip_ok(hipEventRecord(join[i], R[i].s), "hipEventRecord");
    hip_ok(hipSetDevice(R[0].dev), "hipSetDevice");
    hip_ok(hipStreamWaitEvent(R[0].s, join[i], 0), "hipStreamWaitEvent");
  }
  hip_ok(hipStreamEndCapture(R[0].s, &g), "hipStreamEndCapture");
  hip_ok(hipGraphInstantiate(&exec, g, nullptr, nullptr, 0), "hipGraphInstantiate");
  hip_ok(hipGraphDestroy(g), "hipGraphDestroy");
  hip_ok(hipGraphLaunch(exec, R[0].s), "hipGraphLaunch");
  hip_ok(hipStreamSynchronize(R[0].s), "graph warm-up");
  }
  hipEvent_t e0, e1;
  hip_ok(hipEventCreate(&e0), "hipEventCreate");
  hip_ok(hipEventCreate(&e1), "hipEventCreate");
  hip_ok(hipEventRecord(e0, R[0].s), "hipEventRecord");
  for (int it = 0; it < iters; ++it) {
    if (graphed) {
      hip_ok(hipGraphLaunch(exec, R[0].s), "hipGraphLaunch");
      continue;
    }
    hip_ok(hipEventRecord(fork, R[0].s), "hipEventRecord");
    for (size_t i = 1; i < R.size(); ++i) {
      hip_ok(hipSetDevice(R[i].dev), "hipSetDevice");
      hip_ok(hipStreamWaitEvent(R[i].s, fork, 0), "hipStreamWaitEvent");
    }
    step_sharded(R, comm, layers, N, tall);
    for (size_t i = 1; i < R.size(); ++i) {
      hip_ok(hipSetDevice(R[i].dev), "hipSetDevice");
      hip_ok(hipEventRecord(join[i], R[i].s), "hipEventRecord");
      hip_ok(hipSetDevice(R[0].dev), "hipSetDevice");
      hip_ok(hipStreamWaitEvent(R[0].s, join[i], 0), "hipStreamWaitEvent");
    }
  }
  hip_ok(hipEventRecord(e1, R[0].s), "hipEventRecord");
  hip_ok(hipEventSynchronize(e1), "hipEventSynchronize");
  float ms = 0;
  hip_ok(hipEventElapsedTime(&ms, e0, e1), "hipEventElapsedTime");
  const double t = ms * 1e-3 / iters;
  std::vector<float> lg((size_t)N * V);
  hip_ok(hipMemcpy(lg.data(), R[0].logits, lg.size() * 4, hipMemcpyDeviceToHost), "download logits");
  double cs = 0;
  for (float v : lg) cs += std::fabs(v);
  if (!std::isfinite(cs)) {
    fprintf(stderr, "llama-matmul-bench: non-finite logits\n");
    return 1;
  }
  auto dump = [](const std::string& path, const std::vector<float>& v) {
    FILE* f = fopen(path.c_str(), "wb");
    const bool ok = f && fwrite(v.data(), 4, v.size(), f) == v.size();
    if (f) fclose(f);
    if (!ok) fprintf(stderr, "llama-matmul-bench: writing %s failed\n", path.c_str());
    return ok;
  };
  if (!o.dump.empty() && !dump(o.dump, lg)) return 1;
  if (!o.dump_q.empty()) {   // layer 0's q|k|v (tall) or q projection, from the input every G shares
    std::vector<float> x((size_t)N * H);
    for (size_t j = 0; j < x.size(); ++j) x[j] = std::sin(0.37f * (float)j);
    for (Rank& r : R) {
      hip_ok(hipSetDevice(r.dev), "hipSetDevice");
      hip_ok(hipMemcpy(r.d, x.data(), x.size() * 4, hipMemcpyHostToDevice), "upload x");
    }
    project(R, comm, N, [&](Rank& r) -> const Tensor& { return r.wq[0]; }, [](Rank& r) -> Act& { return r.a4096; },
            [](Rank& r) { return r.q; });
    for (Rank& r : R) {
      hip_ok(hipSetDevice(r.dev), "hipSetDevice");
      hip_ok(hipStreamSynchronize(r.s), "first projection");
    }
    std::vector<float> q((size_t)N * R[0].wq[0].Mfull);
    hip_ok(hipSetDevice(R[0].dev), "hipSetDevice");
    hip_ok(hipMemcpy(q.data(), R[0].q, q.size() * 4, hipMemcpyDeviceToHost), "download q");
    if (!dump(o.dump_q, q)) return 1;
  }
  const int projections = (tall ? 4 : 7) * layers + 1;
  printf("step %.3f ms  |  %.1f tok/s  |  weight stream %.1f GB/s (whole model)  |  %d matmuls + %d all-gathers per rank "
         "per step  |  logits |sum| %.6g\n",
         t * 1e3, N / t, wbytes / t / 1e9, projections, projections, cs);
  printf("{\"tool\": \"llama-matmul-bench\", \"layers\": %d, \"tokens_per_step\": %d, \"ms_per_step\": %.4f, "
         "\"tok_per_s\": %.2f, \"weight_GBps\": %.1f, \"TFLOPs\": %.2f, \"graph\": %s, \"stationary\": %s, "
         "\"type\": \"%s\", \"mode\": \"%s\", \"launches\": %d, \"world\": %d, \"rank\": %d, \"local_ranks\": %zu, "
         "\"allgathers\": %d, \"logits_abs_sum\": %.9g}\n",
         layers, N, t * 1e3, N / t, wbytes / t / 1e9, 2.0 * params * N / t / 1e12, graphed ? "true" : "false", stationary ? "true" : "false",
         type_name(type), tall ? "sharded-batch-proj" : "sharded", projections, world, o.rank >= 0 ? o.rank : 0,
         R.size(), projections, cs);
  lamm_hip_comm_destroy(comm);
  return 0;
}

}  // namespace

// a host-side fault prints its call stack before the process ends (the tests see only the exit code)
void on_fault(int sig) {
  void* frames[64];
  const int n = backtrace(frames, 64);
  const char msg[] = "llama-matmul-bench: fatal signal, call stack:\n";
  (void)!write(2, msg, sizeof msg - 1);
  backtrace_symbols_fd(frames, n, 2);
  _exit(128 + sig);
}

int real_main(int argc, char** argv);

// The HIP runtime walks a captured graph's dependencies recursively: the 8-rank sharded step (8
// streams joined by events at every all-gather) took it past the default 8 MiB main-thread stack
// (call stack of the fault: libamdhip64 recursing in one frame).  The whole program runs on a
// thread with a 1 GiB stack (address space; only the pages it touches are committed).
int main(int argc, char** argv) {
  struct Args {
    int argc;
    char** argv;
    int rc;
  } a{argc, argv, 1};
  pthread_attr_t attr;
  pthread_attr_init(&attr);
  pthread_attr_setstacksize(&attr, (size_t)1 << 30);
  pthread_t th;
  if (pthread_create(&th, &attr, [](void* p) -> void* {
        auto* x = static_cast<Args*>(p);
        x->rc = real_main(x->argc, x->argv);
        return nullptr;
      }, &a) != 0) {
    return real_main(argc, argv);
  }
  pthread_join(th, nullptr);
  return a.rc;
}

int real_main(int argc, char** argv) {
  setvbuf(stdout, nullptr, _IOLBF, 0);
  int type = 2, N = 1, iters = 20, layers = 32, out_type = 14, ctx = 0;
  bool graph = true, stationary = false, batch_proj = false, concurrent = false, check = false;
  ShardOpts so;
  int shard = 0;
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
    else if (a == "--no-graph") graph = false, so.graph = false;
    else if (a == "-s") stationary = true;
    else if (a == "--unfused") g_fused = false;
    else if (a == "--batch-proj") batch_proj = true;
    else if (a == "--concurrent") concurrent = true;
    else if (a == "--shard") shard = atoi(next());
    else if (a == "--devices") {
      so.devices.clear();
      for (const char* c = next(); *c;) {
        char* end = nullptr;
        so.devices.push_back((int)strtol(c, &end, 10));
        if (end == c) break;
        c = *end == ',' ? end + 1 : end;
      }
    }
    else if (a == "--rank") so.rank = atoi(next());
    else if (a == "--world") so.world = atoi(next());
    else if (a == "--comm-id") so.comm_id = next();
    else if (a == "--device") so.devices = {atoi(next())};
    else if (a == "--dump") so.dump = next();
    else if (a == "--dump-q") so.dump_q = next();
    else if (a == "--ctx") ctx = atoi(next());
    else if (a == "--check") check = true;
    else {
      fprintf(stderr, "usage: %s [-d q4_0] [-n tokens] [-i replays] [-l layers] [--no-graph] [-s] [--output-type q6_k] "
                      "[--unfused] [--batch-proj] [--concurrent] [--shard G [--devices 0,1,..]] "
                      "[--rank r --world w --comm-id HEX|auto [--device d]] [--dump FILE] [--ctx P [--check]]\n",
              argv[0]);
      return 1;
    }
  }
  if (lamm_hip_device_count() <= 0) {
    fprintf(stderr, "llama-matmul-bench: no gfx950 device (%s)\n", lamm_hip_last_error());
    return 1;
  }
  // after the HIP runtime's own start-up (it installs handlers of its own)
  static char altstack[1 << 16];   // the handler also runs when the fault is a stack overflow
  stack_t ss = {};
  ss.ss_sp = altstack;
  ss.ss_size = sizeof altstack;
  sigaltstack(&ss, nullptr);
  struct sigaction sa = {};
  sa.sa_handler = on_fault;
  sa.sa_flags = SA_ONSTACK;
  sigaction(SIGSEGV, &sa, nullptr);
  sigaction(SIGBUS, &sa, nullptr);
  if (so.rank >= 0 || shard > 0 || !so.devices.empty() || !so.dump.empty() || !so.dump_q.empty()) {   // the row-sharded form
    if (so.rank >= 0) {
      if (so.world < 1 || so.rank >= so.world || so.comm_id.empty()) {
        fprintf(stderr, "llama-matmul-bench: --rank needs --world > rank and --comm-id\n");
        return 1;
      }
      if (so.devices.empty()) so.devices = {so.rank % lamm_hip_device_count()};
    } else {
      if (so.devices.empty()) {   // G local ranks on devices 0..G-1 (repeating when fewer: loopback)
        const int G = shard > 0 ? shard : 1;
        for (int i = 0; i < G; ++i) so.devices.push_back(i % lamm_hip_device_count());
      }
      so.world = (int)so.devices.size();
    }
    if (concurrent || !graph) {
      fprintf(stderr, "llama-matmul-bench: the sharded form is graph-captured, without --concurrent\n");
      return 1;
    }
    if (ctx > 0) {
      fprintf(stderr, "llama-matmul-bench: --ctx runs in the single-GPU form\n");
      return 1;
    }
    return run_sharded(so, type, out_type, N, iters, layers, stationary, batch_proj);
  }
  if (ctx > 0 && (N != 1 || ctx % 8 || concurrent)) {
    fprintf(stderr, "llama-matmul-bench: --ctx P needs -n 1, P a multiple of 8, no --concurrent\n");
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
  m.ctx = ctx;
  size_t kv_bytes = 0;
  if (ctx > 0) {   // the F16 KV cache (random contents), q / scores / probs / kqv buffers
    const size_t cell = (size_t)H * 2;   // one token's K row (or V column) over all heads, bytes
    float* r = nullptr;
    hip_ok(hipMalloc(&r, (size_t)ctx * H * 4), "hipMalloc");
    {
      std::vector<float> h((size_t)ctx * H);
      for (size_t i = 0; i < h.size(); ++i) h[i] = std::sin(0.011f * (float)i) * 0.5f;
      hip_ok(hipMemcpy(r, h.data(), h.size() * 4, hipMemcpyHostToDevice), "upload kv");
    }
    for (int l = 0; l < layers; ++l)
      for (auto* v : {&m.kc, &m.vt}) {
        void* p = nullptr;
        hip_ok(hipMalloc(&p, cell * ctx + 256), "hipMalloc(kv)");
        lamm_ok(lamm_hip_quantize(1, 0, r, H, p, H, H, ctx, s), "kv init");
        v->push_back(p);
      }
    hip_ok(hipStreamSynchronize(s), "kv init");
    hip_ok(hipFree(r), "hipFree");
    kv_bytes = 2 * cell * ctx * layers;
    hip_ok(hipMalloc(&m.qh, (size_t)H * 2 + 256), "hipMalloc");
    hip_ok(hipMalloc(&m.vrow, (size_t)H * 2 + 256), "hipMalloc");
    hip_ok(hipMalloc(&m.scores, (size_t)32 * ctx * 4 + 256), "hipMalloc");
    hip_ok(hipMalloc(&m.probs, (size_t)32 * ctx * 2 + 256), "hipMalloc");
    mk_out(m.kqv, H);
  }
  mk_act(m.b4096, H, ctx > 0 ? m.kqv : m.q);
  mk_act(m.c4096, H, m.o);
  mk_act(m.a11008, F, batch_proj ? m.g + (size_t)N * F : m.u);   // the up projection's output

  printf("llama-matmul-bench: Llama-7B weight matmuls, %d layers, weights %s, output.weight %s, "
         "%.2f GB of weight blocks, %d token(s) per step, %s%s\n",
         layers, type_name(type), type_name(out_type), wbytes / 1e9, N, graph ? "hipGraph" : "stream",
         stationary ? ", weight-stationary handles" : "");

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
  if (ctx > 0 && check && !check_attention(m, layers - 1)) return 1;
  const int launches = (batch_proj ? 4 : 7) * layers + 1 + (ctx > 0 ? 7 * layers : 0);
  printf("step %.3f ms  |  %.1f tok/s  |  weight stream %.1f GB/s  |  %.1f TFLOP/s  |  %d matmul launches + %d quantizations per step  |  logits |sum| %.4g\n",
         t * 1e3, N / t, wbytes / t / 1e9, 2.0 * params * N / t / 1e12, launches,
         fused(type, N) ? 1 : 4 * layers + 1, cs);
  printf("{\"tool\": \"llama-matmul-bench\", \"layers\": %d, \"tokens_per_step\": %d, \"ms_per_step\": %.4f, \"tok_per_s\": %.2f, "
         "\"weight_GBps\": %.1f, \"TFLOPs\": %.2f, \"graph\": %s, \"stationary\": %s, \"type\": \"%s\", "
         "\"mode\": \"%s\", \"launches\": %d, \"ctx\": %d, \"kv_cache_GB\": %.3f, \"bytes_GBps\": %.1f}\n",
         layers, N, t * 1e3, N / t, wbytes / t / 1e9, 2.0 * params * N / t / 1e12, graph ? "true" : "false",
         stationary ? "true" : "false", type_name(type),
         batch_proj ? "batch-proj" : concurrent ? "concurrent" : "separate", launches, ctx, kv_bytes / 1e9,
         (wbytes + kv_bytes) / t / 1e9);
  return 0;
}
