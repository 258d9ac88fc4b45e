// lamm_rowdot.h -- the row-per-wave block-dot pieces of the decode GEMV (lamm_gemv_rpw.hip) and
// the fp6 GEMM's activation prep (lamm_gemm_fp6.hip): block layouts, wide buffer loads
// with realignment, the A-block unpack and the activation staging (ggml's AVX2 from_float for
// F32 rows, bit for bit).  The arithmetic is the reference's lamm_kernel_q*.hpp block dot:
// exact int32 dots, d_a*d_b*S [+ m_a*s_b] in fp32.
#pragma once
#include "lamm_device.h"
#include "lamm_kernels.h"

namespace lamm {
namespace {

// Completion signal (LAMM_HIP_KERNEL_SIGNAL=1, see GemvArgs): every workgroup releases its C
// stores to system scope before it counts itself in; the last one to arrive acquires the others'
// releases and only then stores the flag the host spins on (a relaxed counter alone
// let the host see the flag before other workgroups' C reached host memory).
__device__ __forceinline__ void signal_done(const GemvArgs& p) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's C stores have completed
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence_system();
    if (atomicAdd(p.done_ctr, 1u) == gridDim.x * gridDim.y - 1) {
      __threadfence_system();
      __hip_atomic_store(p.done_ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(p.flag, p.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

template <int T> struct RFmt;
template <> struct RFmt<kQ4_0> { static constexpr int BPB = 18, VBPB = 34; };
template <> struct RFmt<kQ4_1> { static constexpr int BPB = 20, VBPB = 36; };
template <> struct RFmt<kQ5_0> { static constexpr int BPB = 22, VBPB = 34; };
template <> struct RFmt<kQ5_1> { static constexpr int BPB = 24, VBPB = 36; };
template <> struct RFmt<kQ8_0> { static constexpr int BPB = 34, VBPB = 34; };

// NW consecutive dwords at byte offset `off` (dword aligned) of a buffer resource, as wide
// buffer loads (b128 / b64 / b32); out-of-range dwords read as 0.
template <int NW, int AUX>
__device__ __forceinline__ void load_words(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t (&w)[NW]) {
  unroll<NW / 4>([&](auto I) {
    constexpr int i = I;
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(r, off + 16 * i, 0, AUX);
    w[4 * i] = v[0]; w[4 * i + 1] = v[1]; w[4 * i + 2] = v[2]; w[4 * i + 3] = v[3];
  });
  constexpr int b = NW / 4 * 4;
  if constexpr (NW - b >= 2) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(r, off + 4 * b, 0, AUX);
    w[b] = (uint32_t)v[0];
    w[b + 1] = (uint32_t)v[1];
    if constexpr (NW - b == 3) w[b + 2] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * b + 8, 0, AUX);
  } else if constexpr (NW - b == 1) {
    w[b] = __builtin_amdgcn_raw_buffer_load_b32(r, off + 4 * b, 0, AUX);
  }
}

// One weight block's dwords from the dword below its start, into NWA = (BPB + 3) / 4 + 1 words (the
// realignment's input).  Every block size is even, so a block starts at a shift of 0 or 2 bytes
// (always 0 when BPB % 4 == 0): ceil((BPB + 2) / 4) dwords hold it, one fewer than NWA -- q4_0
// 20 bytes (b128 + b32) instead of 24 (b128 + b64).  The spare word is 0; realign never needs its
// bytes (config 2 probe: G8-n5 vs G8, profiles/r03/gemv_probe_15.json; library A/B
// profiles/r03/block_words/: q4_0 3.65 -> 3.61 us, q8_0 5.85 -> 5.76, decode step -1.3 %).  q5_0
// (22 bytes) keeps b128 + b64 + b32: its 6-dword form measured 4.01 -> 4.11 us.
template <int BPB>
constexpr int block_dwords() { return BPB % 4 == 0 ? BPB / 4 : BPB == 22 ? (BPB + 3) / 4 + 1 : (BPB + 2 + 3) / 4; }
template <int BPB, int AUX, int NWA>
__device__ __forceinline__ void load_block_words(__amdgpu_buffer_rsrc_t r, uint32_t off, uint32_t (&w)[NWA]) {
  constexpr int NL = block_dwords<BPB>();
  static_assert(NL <= NWA, "fits the realignment input");
  static_assert(BPB % 2 == 0 && 4 * NL >= BPB + (BPB % 4 ? 2 : 0), "covers the block at its largest shift");
  uint32_t t[NL];
  load_words<NL, AUX>(r, off, t);
#pragma unroll
  for (int k = 0; k < NWA; ++k) w[k] = k < NL ? t[k] : 0u;
}

// bytes [sh, sh + 4*(NW-1)) of w as NW-1 dwords (sh in {0, 1, 2, 3} bytes)
template <int NW>
__device__ __forceinline__ void realign(const uint32_t (&w)[NW], uint32_t (&m)[NW - 1], int sh) {
  unroll<NW - 1>([&](auto K) {
    constexpr int k = K;
    m[k] = __builtin_amdgcn_alignbit(w[k + 1], w[k], sh * 8);
  });
}

// A 32-element block as the dot needs it: 8 int8 quads (the 4-bit / 5-bit formats unpacked to
// unsigned bytes) + d (+ m for q4_1 / q5_1)
template <int T, int NW>
__device__ __forceinline__ void unpack_a(const uint32_t (&m)[NW], uint32_t (&q)[8], float& da, float& ma) {
  ma = 0.f;
  if constexpr (T == kQ8_0) {
    da = h2f(get16<0>(m));
    unroll<8>([&](auto K) { q[K] = get32<2 + 4 * K>(m); });
  } else {
    constexpr bool AFF = (T == kQ4_1 || T == kQ5_1);
    constexpr bool FIVE = (T == kQ5_0 || T == kQ5_1);
    constexpr int QS = (AFF ? 4 : 2) + (FIVE ? 4 : 0);
    da = h2f(get16<0>(m));
    if constexpr (AFF) ma = h2f(get16<2>(m));
    uint32_t qh = 0;
    if constexpr (FIVE) qh = get32<AFF ? 4 : 2>(m);
    unroll<4>([&](auto K) {
      constexpr int k = K;
      const uint32_t x = get32<QS + 4 * k>(m);
      q[k] = x & 0x0f0f0f0fu;
      q[4 + k] = (x >> 4) & 0x0f0f0f0fu;
      if constexpr (FIVE) {
        q[k] |= spread4_hi((qh >> (4 * k)) & 0xf);
        q[4 + k] |= spread4_hi((qh >> (16 + 4 * k)) & 0xf);
      }
      // q4_0 / q5_0 quants stay unsigned: their offset is applied to the dot in the integer
      // domain, sum (q - c) b = sum q b - c sum b, with sum b precomputed per activation block
    });
  }
}

// One 32-element F32 block -> q8_0 / q8_1 the way ggml's AVX2 from_float rounds it
// (LC/ggml-quants.c quantize_row_q8_0 / _q8_1 AVX2 branches: id = 127/amax, nearest-even,
// d and s = d * sum as fp16), bit-identical to lamm_hip_quantize(.., flavour 1, ..):
// q = the 32 int8 quants as 8 little-endian dwords, dh / sh = fp16 bits of d / s.
template <bool WITH_S>
__device__ __forceinline__ void q8_from_f32(const uint32_t (&w)[32], uint32_t (&q)[8], uint16_t& dh, uint16_t& sh) {
  float amax = 0.f;
#pragma unroll
  for (int k = 0; k < 32; ++k) amax = fmaxf(amax, fabsf(__builtin_bit_cast(float, w[k])));
  const float dd = amax / 127.f;
  const float id = amax != 0.0f ? 127.f / amax : 0.0f;
  int sum = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    uint32_t qw = 0;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      int v = avx_cvt_i32(__builtin_rintf(__builtin_bit_cast(float, w[4 * k + e]) * id));
      sum = (int)((uint32_t)sum + (uint32_t)v);   // before the saturation, wrapping (AVX2 q8_1's s)
      v = v > 127 ? 127 : (v < -128 ? -128 : v);
      qw |= (uint32_t)(v & 0xff) << (8 * e);
    }
    q[k] = qw;
  }
  float dv = dd;
  asm volatile("" : "+v"(dv));   // no contraction of the d*sum product below into the division
  dh = __builtin_bit_cast(uint16_t, (_Float16)dv);
  sh = 0;
  if constexpr (WITH_S) {
    float sd = (float)sum * dd;
    asm volatile("" : "+v"(sd));
    sh = __builtin_bit_cast(uint16_t, (_Float16)sd);
  }
}

// The activation rows, decoded once per workgroup: per column j and block b, the 8 int8 quads
// as two 16-byte halves (lanes read consecutive 16-byte slots: conflict-free ds_read_b128),
// fp32(fp16 d) and, for q8_1, fp32(fp16 s).  F32 rows are quantized here (ggml's AVX2
// from_float, bit for bit as stage_b_f32 in lamm_gemv.hip).  Split in two so a thread's
// activation loads can be issued BEFORE its wave's A loads: waiting for them then does not wait
// for the HBM stream (vmcnt retires in order).
template <int T, bool BF32>
struct ActStage {
  using F = RFmt<T>;
  static constexpr int NWB = (F::VBPB + 3) / 4 + 1;
  static constexpr int NW = BF32 ? 32 : NWB;
  uint32_t w[NW];
  uint32_t off = 0;

  template <int NC>
  __device__ __forceinline__ void load(const GemvArgs& p, __amdgpu_buffer_rsrc_t rb, int it) {
    static_assert(NC <= 2, "column by comparison, not division");
    const int ncols = p.N < NC ? p.N : NC;
    const int j = NC > 1 && it >= p.nblk ? 1 : 0, b = it - j * p.nblk;
    const bool ok = j < ncols && it < NC * p.nblk;
    if constexpr (BF32) {
      off = ok ? (uint32_t)(j * p.ldb + (int64_t)b * 128) : 0x7ffffff0u;
      load_words<32, 0>(rb, off, w);
    } else {
      off = ok ? (uint32_t)(j * p.ldb + (int64_t)b * F::VBPB) : 0x7ffffff0u;
      load_words<NWB, 0>(rb, off & ~3u, w);
    }
  }

  // the loaded words as an opaque definition here: the decode cannot be hoisted above this point
  // (behind a branch around the loads the compiler otherwise moves it -- and its wait for the
  // activation -- in front of the row's A loads)
  __device__ __forceinline__ void pin() {
#pragma unroll
    for (int i = 0; i < NW; ++i) asm volatile("" : "+v"(w[i]));
  }

  __device__ __forceinline__ void store(int it, u32x4* q0, u32x4* q1, float* bd, float* bs) const {
    uint32_t q[8];
    float d, sx;
    decode(q, d, sx);
    q0[it] = u32x4{q[0], q[1], q[2], q[3]};
    q1[it] = u32x4{q[4], q[5], q[6], q[7]};
    bd[it] = d;
    bs[it] = sx;
  }

  // the block as the dot needs it: 8 quads, d, and s (q8_1) or the bit pattern of sum b (q4_0 / q5_0)
  __device__ __forceinline__ void decode(uint32_t (&q)[8], float& d, float& sx) const {
    d = 0.f;
    sx = 0.f;
    if constexpr (BF32) {
      uint16_t dh, sh;
      q8_from_f32<F::VBPB == 36>(w, q, dh, sh);
      d = h2f(dh);
      if constexpr (F::VBPB == 36) sx = h2f(sh);
    } else {
      uint32_t m[NWB - 1];
      realign(w, m, (int)(off & 3u));
      constexpr int VQS = F::VBPB == 36 ? 4 : 2;
      unroll<8>([&](auto K) { q[K] = get32<VQS + 4 * K>(m); });
      d = h2f(m[0] & 0xffff);
      if constexpr (VQS == 4) sx = h2f(m[0] >> 16);
    }
    if constexpr (T == kQ4_0 || T == kQ5_0) {   // sum b (exact int) for the offset term
      int sb = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) sb = dot4(q[k], 0x01010101u, sb);
      sx = __builtin_bit_cast(float, sb);
    }
  }
};

// F32 activation rows staged by L lanes per 32-element block (L = 2 or 4; 32 / L values each):
// the block's |max| and sum of quants are combined across the L lanes with DPP, every value is
// rounded by the lane that holds it -- the same bytes as ActStage<T, true> / q8_from_f32 (max
// and integer sums do not depend on the order), with 1 / L of the latency per block.  Thread t
// handles block t / L, values (32 / L) (t % L) ..; all L lanes of a block must call store()
// together (they do: t runs over whole groups).
template <int T, int L>
struct ActStageL {
  static_assert(L == 2 || L == 4, "lanes per block");
  using F = RFmt<T>;
  static constexpr int NV = 32 / L;   // values per lane
  uint32_t w[NV];

  template <int NC>
  __device__ __forceinline__ void load(const GemvArgs& p, __amdgpu_buffer_rsrc_t rb, int t) {
    static_assert(NC <= 2, "column by comparison, not division");
    const int ncols = p.N < NC ? p.N : NC;
    const int it = t / L, part = t % L;
    const int j = NC > 1 && it >= p.nblk ? 1 : 0, b = it - j * p.nblk;
    const bool ok = j < ncols && it < NC * p.nblk;
    load_words<NV, 0>(rb, ok ? (uint32_t)(j * p.ldb + (int64_t)b * 128 + 4 * NV * part) : 0x7ffffff0u, w);
  }

  __device__ __forceinline__ void store(int t, u32x4* q0, u32x4* q1, float* bd, float* bs) const {
    const int it = t / L, part = t % L;
    float amax = 0.f;
#pragma unroll
    for (int k = 0; k < NV; ++k) amax = fmaxf(amax, fabsf(__builtin_bit_cast(float, w[k])));
    amax = fmaxf(amax, dpp_get<0xB1>(amax));                  // quad_perm [1,0,3,2]
    if constexpr (L == 4) amax = fmaxf(amax, dpp_get<0x4E>(amax));   // quad_perm [2,3,0,1]
    const float dd = amax / 127.f;
    const float id = amax != 0.0f ? 127.f / amax : 0.0f;
    int sum = 0;
    uint32_t q[NV / 4];
#pragma unroll
    for (int k = 0; k < NV / 4; ++k) {
      uint32_t qw = 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        int v = avx_cvt_i32(__builtin_rintf(__builtin_bit_cast(float, w[4 * k + e]) * id));
        sum = (int)((uint32_t)sum + (uint32_t)v);   // before the saturation, wrapping (AVX2 q8_1's s)
        v = v > 127 ? 127 : (v < -128 ? -128 : v);
        qw |= (uint32_t)(v & 0xff) << (8 * e);
      }
      q[k] = qw;
    }
    sum += __builtin_bit_cast(int, dpp_get<0xB1>(__builtin_bit_cast(float, sum)));
    if constexpr (L == 4) sum += __builtin_bit_cast(int, dpp_get<0x4E>(__builtin_bit_cast(float, sum)));
    // quad words (NV / 4 per lane) of the block: words 0-3 in q0, 4-7 in q1
    const int w0 = (NV / 4) * part;
    uint32_t* dst = reinterpret_cast<uint32_t*>(w0 < 4 ? &q0[it] : &q1[it]) + (w0 & 3);
#pragma unroll
    for (int k = 0; k < NV / 4; ++k) dst[k] = q[k];
    if (part == 0) {
      float dv = dd;
      asm volatile("" : "+v"(dv));
      bd[it] = h2f(__builtin_bit_cast(uint16_t, (_Float16)dv));
      float sx = 0.f;
      if constexpr (F::VBPB == 36) {
        float sd = (float)sum * dd;
        asm volatile("" : "+v"(sd));
        sx = h2f(__builtin_bit_cast(uint16_t, (_Float16)sd));
      }
      if constexpr (T == kQ4_0 || T == kQ5_0) sx = __builtin_bit_cast(float, sum);   // sum b, exact
      bs[it] = sx;
    }
  }
};

template <int T, int NC, bool BF32>
__device__ __forceinline__ __amdgpu_buffer_rsrc_t act_rsrc(const GemvArgs& p, const unsigned char* Bz) {
  using F = RFmt<T>;
  const int ncols = p.N < NC ? p.N : NC;
  const int64_t bbytes = BF32 ? (int64_t)(ncols - 1) * p.ldb + (int64_t)p.K * 4
                              : (int64_t)(ncols - 1) * p.ldb + (int64_t)p.nblk * F::VBPB;
  return make_rsrc(Bz, (uint32_t)min((bbytes + 3) & ~int64_t(3), (int64_t)0x7fffffff));
}

}  // namespace
}  // namespace lamm
