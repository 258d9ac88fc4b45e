/*
 * ref_driver.c -- TEST INFRASTRUCTURE ONLY (never shipped, never the product path).
 *
 * A tiny C driver around the *real* reference (AyiStar/la-llama.cpp @ b2430 ggml +
 * the lamm plug-in), compiled out-of-tree from the sources where they lie under
 * /root/reference by oracle/Makefile into oracle/_ref/.  It is used for two jobs:
 *
 *   gen   : produce golden vectors (quantized A, quantized B, C) exactly the way
 *           la-benchmark-matmult does it (src/la-benchmark-matmult.cpp:294-316):
 *             A  <- ggml_quantize_chunk(type, A_f32)            (LC/ggml.c ggml_quantize_chunk)
 *             Bq <- traits[vec_dot_type].from_float(B_f32)      (INIT phase, LC/ggml.c:10865-10887)
 *             Br <- traits[vec_dot_type].from_float_reference   (scalar reference quantizer)
 *             C  <- ggml_graph_compute(ggml_mul_mat(A, B))       (hook LC/ggml.c:10858-10863)
 *   bench : time ggml_graph_compute of one mul_mat node the way la-benchmark-matmult
 *           does (src/la-benchmark-matmult.cpp:345-386: timed region = graph compute,
 *           which includes the INIT src1 quantization; a second graph on another A
 *           copy runs between timed iterations to evict caches).  Used only as the
 *           cpu_baseline leg of bench.py ("kind": "reference").
 *
 * Usage:
 *   ref_driver gen   <type> <M> <N> <K> <nthreads> <A_f32.bin> <B_f32.bin> <out_prefix>
 *   ref_driver bench <type> <M> <N> <K> <nthreads> <iters> <budget_seconds>
 *   ref_driver quant <type> <rows> <K> <x_f32.bin> <out.bin>
 *         (quant: the type's from_float on each row -- the INIT quantizer of this build, e.g.
 *         the AVX2 quantize_row_q8_0 / _q8_1 in the lamm3 build; pins the oracle's restatement
 *         on edge inputs, tools/gen_golden_quant.py)
 * type is a ggml type name: f32 q4_0 q4_1 q5_0 q5_1 q8_0 q2_k (+ q4_k q5_k q6_k)
 */
#include "ggml.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <strings.h>
#include <time.h>

static enum ggml_type parse_type(const char *s) {
  if (!strcasecmp(s, "f32")) return GGML_TYPE_F32;
  if (!strcasecmp(s, "f16")) return GGML_TYPE_F16;   /* SURVEY §8f */
  if (!strcasecmp(s, "q4_0")) return GGML_TYPE_Q4_0;
  if (!strcasecmp(s, "q4_1")) return GGML_TYPE_Q4_1;
  if (!strcasecmp(s, "q5_0")) return GGML_TYPE_Q5_0;
  if (!strcasecmp(s, "q5_1")) return GGML_TYPE_Q5_1;
  if (!strcasecmp(s, "q8_0")) return GGML_TYPE_Q8_0;
  if (!strcasecmp(s, "q8_1")) return GGML_TYPE_Q8_1;   /* activation type (quant mode) */
  if (!strcasecmp(s, "q2_k")) return GGML_TYPE_Q2_K;
  if (!strcasecmp(s, "q4_k")) return GGML_TYPE_Q4_K;   /* SURVEY §8f "next" formats */
  if (!strcasecmp(s, "q5_k")) return GGML_TYPE_Q5_K;
  if (!strcasecmp(s, "q6_k")) return GGML_TYPE_Q6_K;
  fprintf(stderr, "unknown type %s\n", s);
  exit(2);
}

static void *read_file(const char *path, size_t expect) {
  FILE *f = fopen(path, "rb");
  if (!f) { perror(path); exit(2); }
  void *buf = malloc(expect);
  if (fread(buf, 1, expect, f) != expect) { fprintf(stderr, "short read %s\n", path); exit(2); }
  fclose(f);
  return buf;
}

static void write_file(const char *prefix, const char *suffix, const void *p, size_t n) {
  char path[4096];
  snprintf(path, sizeof path, "%s%s", prefix, suffix);
  FILE *f = fopen(path, "wb");
  if (!f) { perror(path); exit(2); }
  fwrite(p, 1, n, f);
  fclose(f);
}

static void compute_graph(struct ggml_cgraph *g, int nth, uint8_t **work, size_t *work_sz) {
  struct ggml_cplan plan = ggml_graph_plan(g, nth);
  if (plan.work_size > *work_sz) {
    *work = realloc(*work, plan.work_size);
    *work_sz = plan.work_size;
  }
  plan.work_data = *work;
  ggml_graph_compute(g, &plan);
}

static int do_gen(int argc, char **argv) {
  if (argc < 10) { fprintf(stderr, "gen: bad args\n"); return 2; }
  enum ggml_type type = parse_type(argv[2]);
  int M = atoi(argv[3]), N = atoi(argv[4]), K = atoi(argv[5]), nth = atoi(argv[6]);
  float *af = read_file(argv[7], (size_t)M * K * sizeof(float));
  float *bf = read_file(argv[8], (size_t)N * K * sizeof(float));
  const char *out = argv[9];

  ggml_type_traits_t tr = ggml_internal_get_type_traits(type);
  enum ggml_type vdt = tr.vec_dot_type;
  ggml_type_traits_t vtr = ggml_internal_get_type_traits(vdt);

  size_t ctx_size = 3 * ((size_t)M * K + (size_t)N * K + (size_t)M * N) * sizeof(float) + (64u << 20);
  struct ggml_init_params ip = {ctx_size, NULL, false};
  struct ggml_context *ctx = ggml_init(ip);

  struct ggml_tensor *a = ggml_new_tensor_2d(ctx, type, K, M);
  if (type == GGML_TYPE_F32) {
    memcpy(a->data, af, (size_t)M * K * sizeof(float));
  } else {
    ggml_quantize_chunk(type, af, a->data, 0, M, K, NULL);
  }
  struct ggml_tensor *b = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, N);
  memcpy(b->data, bf, (size_t)N * K * sizeof(float));

  struct ggml_tensor *c = ggml_mul_mat(ctx, a, b);
  struct ggml_cgraph *g = ggml_new_graph(ctx);
  ggml_build_forward_expand(g, c);
  uint8_t *work = NULL;
  size_t work_sz = 0;
  compute_graph(g, nth, &work, &work_sz);

  size_t arow = ggml_row_size(type, K);
  size_t brow = ggml_row_size(vdt, K);
  write_file(out, ".A.bin", a->data, arow * M);
  write_file(out, ".C.bin", c->data, (size_t)M * N * sizeof(float));

  uint8_t *bq = malloc(brow * N);
  uint8_t *br = malloc(brow * N);
  for (int j = 0; j < N; j++) {
    if (vdt == GGML_TYPE_F32) {
      memcpy(bq + j * brow, bf + (size_t)j * K, brow);
      memcpy(br + j * brow, bf + (size_t)j * K, brow);
    } else {
      vtr.from_float(bf + (size_t)j * K, bq + j * brow, K);
      /* q8_K has no from_float_reference: its from_float IS the reference
       * quantizer (LC/ggml.c:768-774, LC/ggml-quants.c:4031-4033) */
      (vtr.from_float_reference ? vtr.from_float_reference : vtr.from_float)(
          bf + (size_t)j * K, br + j * brow, K);
    }
  }
  write_file(out, ".Bq.bin", bq, brow * N);
  write_file(out, ".Br.bin", br, brow * N);

  /* stock vec_dot on the *from_float* B, row by row (ggml's own non-lamm loop) */
  float *cv = malloc((size_t)M * N * sizeof(float));
  for (int j = 0; j < N; j++)
    for (int i = 0; i < M; i++)
      tr.vec_dot(K, &cv[(size_t)j * M + i], 0, (const char *)a->data + (size_t)i * arow, 0,
                 bq + j * brow, 0, 1);
  write_file(out, ".Cv.bin", cv, (size_t)M * N * sizeof(float));

  free(cv); free(bq); free(br); free(work); free(af); free(bf);
  ggml_free(ctx);
  return 0;
}

static double now_us(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

static int cmp_d(const void *x, const void *y) {
  double a = *(const double *)x, b = *(const double *)y;
  return (a > b) - (a < b);
}

static int do_bench(int argc, char **argv) {
  if (argc < 9) { fprintf(stderr, "bench: bad args\n"); return 2; }
  enum ggml_type type = parse_type(argv[2]);
  int M = atoi(argv[3]), N = atoi(argv[4]), K = atoi(argv[5]), nth = atoi(argv[6]);
  int iters = atoi(argv[7]);
  double budget_s = atof(argv[8]);

  size_t arow = ggml_row_size(type, K);
  size_t ctx_size = 2 * arow * M + 2 * (size_t)N * K * 4 + 2 * (size_t)M * N * 4 + (64u << 20);
  struct ggml_init_params ip = {ctx_size, NULL, false};
  struct ggml_context *ctx = ggml_init(ip);

  /* synthetic N(0,1)-ish data via a fixed LCG + Box-Muller; two A copies (g1/g2) */
  float *tmp = malloc((size_t)M * K * sizeof(float));
  uint64_t st = 0x9E3779B97F4A7C15ull;
  struct ggml_tensor *a[2];
  for (int r = 0; r < 2; r++) {
    for (size_t i = 0; i < (size_t)M * K; i++) {
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      double u1 = ((st >> 11) + 1.0) / 9007199254740993.0;
      st = st * 6364136223846793005ull + 1442695040888963407ull;
      double u2 = (st >> 11) / 9007199254740992.0;
      tmp[i] = (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
    }
    a[r] = ggml_new_tensor_2d(ctx, type, K, M);
    if (type == GGML_TYPE_F32) memcpy(a[r]->data, tmp, (size_t)M * K * 4);
    else ggml_quantize_chunk(type, tmp, a[r]->data, 0, M, K, NULL);
  }
  struct ggml_tensor *b = ggml_new_tensor_2d(ctx, GGML_TYPE_F32, K, N);
  for (size_t i = 0; i < (size_t)N * K; i++) ((float *)b->data)[i] = tmp[i % ((size_t)M * K)];
  free(tmp);

  struct ggml_cgraph *g[2];
  for (int r = 0; r < 2; r++) {
    struct ggml_tensor *c = ggml_mul_mat(ctx, a[r], b);
    g[r] = ggml_new_graph(ctx);
    ggml_build_forward_expand(g[r], c);
  }
  uint8_t *work = NULL;
  size_t work_sz = 0;
  compute_graph(g[1], nth, &work, &work_sz); /* warm-up */

  double *t = malloc(sizeof(double) * (iters > 0 ? iters : 1));
  int done = 0;
  double t_start = now_us();
  for (int i = 0; i < iters; i++) {
    double t0 = now_us();
    compute_graph(g[0], nth, &work, &work_sz);
    t[done++] = now_us() - t0;
    compute_graph(g[1], nth, &work, &work_sz); /* evict, as la-benchmark-matmult */
    if ((now_us() - t_start) * 1e-6 > budget_s) break;
  }
  qsort(t, done, sizeof(double), cmp_d);
  double med = t[done / 2];
  double flops = 2.0 * M * N * (double)K;
  printf("{\"type\": \"%s\", \"M\": %d, \"N\": %d, \"K\": %d, \"threads\": %d, \"iters\": %d, "
         "\"median_us\": %.3f, \"gflops\": %.4f}\n",
         argv[2], M, N, K, nth, done, med, flops / med * 1e-3);
  free(t); free(work);
  ggml_free(ctx);
  return 0;
}

static int do_quant(int argc, char **argv) {
  if (argc < 7) { fprintf(stderr, "quant: bad args\n"); return 2; }
  enum ggml_type type = parse_type(argv[2]);
  int rows = atoi(argv[3]), K = atoi(argv[4]);
  float *x = read_file(argv[5], (size_t)rows * K * sizeof(float));
  ggml_type_traits_t tr = ggml_internal_get_type_traits(type);
  size_t row = ggml_row_size(type, K);
  uint8_t *y = calloc((size_t)rows, row);
  for (int r = 0; r < rows; r++) tr.from_float(x + (size_t)r * K, y + (size_t)r * row, K);
  write_file(argv[6], "", y, (size_t)rows * row);
  free(x);
  free(y);
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) { fprintf(stderr, "usage: ref_driver gen|bench ...\n"); return 2; }
  ggml_time_init();
  if (!strcmp(argv[1], "gen")) return do_gen(argc, argv);
  if (!strcmp(argv[1], "bench")) return do_bench(argc, argv);
  if (!strcmp(argv[1], "quant")) return do_quant(argc, argv);
  fprintf(stderr, "unknown mode %s\n", argv[1]);
  return 2;
}
