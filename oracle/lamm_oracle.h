/*
 * lamm_oracle.h -- TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference
 * arithmetic for the lamm_* mul_mat hot path.  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may load this; the product path never does.
 *
 * Parity is PINNED: tests/test_oracle_golden.py checks every function here
 * bit-for-bit against golden vectors produced by the real reference built from
 * /root/reference (oracle/Makefile, oracle/ref_driver.c, tools/gen_golden.py).
 */
#ifndef LAMM_ORACLE_H
#define LAMM_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Type ids are ggml's enum values (LC/ggml.h:341-368). */
enum {
  LO_F32 = 0, LO_F16 = 1, LO_Q4_0 = 2, LO_Q4_1 = 3, LO_Q5_0 = 6, LO_Q5_1 = 7,
  LO_Q8_0 = 8, LO_Q8_1 = 9, LO_Q2_K = 10, LO_Q4_K = 12, LO_Q5_K = 13, LO_Q6_K = 14, LO_Q8_K = 15
};

/* Activation-quantizer flavour.  ggml's INIT phase calls traits.from_float
 * (LC/ggml.c:10865-10887); on an AVX2 build that is the SIMD quantizer
 * (id = 127/amax, round-half-even: LC/ggml-quants.c:1290-1311), on a scalar
 * build it is the *_reference one (d = amax/127, id = 1/d, roundf: :1182-1205). */
enum { LO_QUANT_REF = 0, LO_QUANT_AVX = 1 };

float    lo_fp16_to_fp32(uint16_t h);
uint16_t lo_fp32_to_fp16(float f);

int    lo_block_elems(int type);     /* 32, or 256 for k-quants, 1 for f32 */
size_t lo_block_bytes(int type);     /* 18/20/22/24/34/36/84/292, 4 for f32 */
int    lo_vec_dot_type(int type);    /* LC/ggml.c:477-615 vec_dot_type */
size_t lo_row_bytes(int type, int k);

/* quantize k floats (k % block_elems == 0) into blocks of `type`. */
void lo_quantize_row(int type, int flavour, const float *x, void *y, int k);
void lo_dequantize_row(int type, const void *x, float *y, int k);

/* ggml's scalar vec_dot for (type, vec_dot_type(type)) over k elements. */
float lo_vec_dot(int type, int k, const void *a, const void *b);

/* C[j*ldc + i] = vec_dot(A row i, B column j) for i<M, j<N (lamm layout,
 * src/lamm_kernel_q4_0.hpp:36).  lda/ldb are in BYTES here. */
void lo_mul_mat(int type, int M, int N, int K, const void *A, size_t lda_bytes,
                const void *B, size_t ldb_bytes, float *C, size_t ldc);

/* The reference's x86 CPU float order (the lamm opt-3 AVX2 kernels; ggml's AVX2 q6_K): eight
 * fp32 FMA chains per output, one per __m256 lane, then reduce_sum's fixed tree.  Types f32, q4_0,
 * q4_1, q5_0, q5_1, q6_K (0 for the others).  Pinned bit-for-bit to the golden C_lamm3.
 * f16 (x f16): ggml's AVX2 ggml_vec_dot_f16 -- 32 FMA chains, GGML_F32x8_REDUCE's tree, the
 * n % 32 leftovers in double -- pinned to the reference's own attention nodes (tests/golden/ref_nodes/f16_attention.npz). */
float lo_vec_dot_avx(int type, int k, const void *a, const void *b);
void lo_mul_mat_avx(int type, int M, int N, int K, const void *A, size_t lda_bytes,
                    const void *B, size_t ldb_bytes, float *C, size_t ldc);

#ifdef __cplusplus
}
#endif
#endif
