// lamm_formats.h -- the block-format contract of the lamm_* mul_mat path.
//
// Byte layouts restate LC/ggml-common.h:144-225 (q4_0..q8_1), :199-209 (q2_K) and
// :316-321 (q8_K) of llama.cpp-b2430; type ids are ggml's enum values
// (LC/ggml.h:341-368) so a ggml tensor's `type` field can be used unchanged.
// The (weight type -> activation "vec_dot" type) pairing is the reference's
// supported set, src/loongarch_matmul.cpp:37-52 / src/lamm_ggml_type_trait.h:8-56.
#pragma once
#include <stddef.h>
#include <stdint.h>

namespace lamm {

enum Type : int {
  kF32 = 0, kF16 = 1, kQ4_0 = 2, kQ4_1 = 3, kQ5_0 = 6, kQ5_1 = 7,
  kQ8_0 = 8, kQ8_1 = 9, kQ2_K = 10, kQ4_K = 12, kQ5_K = 13, kQ6_K = 14, kQ8_K = 15,
};

struct block_q4_0 { uint16_t d; uint8_t qs[16]; };
struct block_q4_1 { uint16_t d, m; uint8_t qs[16]; };
struct block_q5_0 { uint16_t d; uint8_t qh[4]; uint8_t qs[16]; };
struct block_q5_1 { uint16_t d, m; uint8_t qh[4]; uint8_t qs[16]; };
struct block_q8_0 { uint16_t d; int8_t qs[32]; };
struct block_q8_1 { uint16_t d, s; int8_t qs[32]; };
struct block_q2_K { uint8_t scales[16]; uint8_t qs[64]; uint16_t d, dmin; };
struct block_q8_K { float d; int8_t qs[256]; int16_t bsums[16]; };
// SURVEY §8f "next" formats (LC/ggml-common.h:263-313, QK_K = 256, K_SCALE_SIZE = 12);
// not lamm formats in the reference, which leaves them to stock ggml
struct block_q4_K { uint16_t d, dmin; uint8_t scales[12]; uint8_t qs[128]; };
struct block_q5_K { uint16_t d, dmin; uint8_t scales[12]; uint8_t qh[32]; uint8_t qs[128]; };
struct block_q6_K { uint8_t ql[128]; uint8_t qh[64]; int8_t scales[16]; uint16_t d; };

static_assert(sizeof(block_q4_0) == 18, "q4_0");
static_assert(sizeof(block_q4_1) == 20, "q4_1");
static_assert(sizeof(block_q5_0) == 22, "q5_0");
static_assert(sizeof(block_q5_1) == 24, "q5_1");
static_assert(sizeof(block_q8_0) == 34, "q8_0");
static_assert(sizeof(block_q8_1) == 36, "q8_1");
static_assert(sizeof(block_q2_K) == 84, "q2_K");
static_assert(sizeof(block_q8_K) == 292, "q8_K");
static_assert(offsetof(block_q5_0, qs) == 6 && offsetof(block_q5_1, qs) == 8, "q5 qs");
static_assert(offsetof(block_q2_K, d) == 80 && offsetof(block_q8_K, bsums) == 260, "k-quant");
static_assert(sizeof(block_q4_K) == 144 && sizeof(block_q5_K) == 176 && sizeof(block_q6_K) == 210, "k-quants");
static_assert(offsetof(block_q5_K, qs) == 48 && offsetof(block_q6_K, d) == 208, "k-quant fields");

// Host-side traits, indexed by ggml type id.
inline bool is_kquant256(int t) { return t == kQ2_K || t == kQ4_K || t == kQ5_K || t == kQ6_K || t == kQ8_K; }
inline int block_elems(int t) { return (t == kF32 || t == kF16) ? 1 : is_kquant256(t) ? 256 : 32; }
inline size_t block_bytes(int t) {
  switch (t) {
    case kF32: return 4;   case kF16: return 2;   case kQ4_0: return 18; case kQ4_1: return 20;
    case kQ5_0: return 22; case kQ5_1: return 24; case kQ8_0: return 34;
    case kQ8_1: return 36; case kQ2_K: return 84; case kQ8_K: return 292;
    case kQ4_K: return 144; case kQ5_K: return 176; case kQ6_K: return 210;
    default: return 0;
  }
}
inline int vec_dot_type(int t) {
  switch (t) {
    case kF32: return kF32;
    case kF16: return kF16;   // F16 weights (KV cache) x F16 rows, ggml_vec_dot_f16
    case kQ4_0: case kQ5_0: case kQ8_0: return kQ8_0;
    case kQ4_1: case kQ5_1: return kQ8_1;
    case kQ2_K: case kQ4_K: case kQ5_K: case kQ6_K: return kQ8_K;
    default: return -1;
  }
}
inline bool is_weight_type(int t) { return vec_dot_type(t) >= 0; }

}  // namespace lamm
