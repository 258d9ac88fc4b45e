/*
 * loongarch_matmul.h -- drop-in replacement header for the reference plug-in.
 *
 * llama.cpp-b2430's ggml.c includes "loongarch_matmul.h" under #ifdef LA_LLAMA
 * (LC/ggml.c:115-117) and calls lamm_can_mul_mat / lamm_mul_mat from
 * ggml_compute_forward_mul_mat (LC/ggml.c:10858-10863).  Putting this directory on
 * the include path instead of la-llama.cpp's src/ and linking liblamm_hip.so (instead
 * of src/loongarch_matmul.o) routes those calls to the MI355X backend unchanged.
 * Declarations: include/lamm_hip.h (same names and signatures as
 * src/loongarch_matmul.h:18-24).
 */
#ifndef LOONGARCH_MATMUL_H
#define LOONGARCH_MATMUL_H

#ifdef _MSC_VER
#define LA_INLINE __forceinline
#define LA_NOINLINE __declspec(noinline)
#else
#define LA_INLINE inline __attribute__((always_inline))
#define LA_NOINLINE __attribute__((__noinline__))
#endif

#include "lamm_hip.h"

#endif /* LOONGARCH_MATMUL_H */
