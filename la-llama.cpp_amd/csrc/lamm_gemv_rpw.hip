// lamm_gemv_rpw.hip -- row-per-wave decode GEMV for the 32-element block formats
// (q4_0, q4_1, q5_0, q5_1, q8_0 against q8_0 / q8_1 or F32 activations), N <= 2.
//
// The per-block arithmetic of lamm_gemv.hip's block_dot (the reference's lamm_kernel_q*.hpp:
// exact int32 block dots, d_a*d_b*S [+ m_a*s_b] in fp32), laid out for ONE call that is too
// small to fill the chip with the wave-group kernel: a 4096 x 4096 q4_0 GEMV (BASELINE config
// 2) is 1024 four-row groups there -- 128 workgroups of 8 waves, half the CUs.  Here:
//   * a wave owns a whole row at a time; lane l takes blocks l, l+64, l+128, ... (each block
//     whole in one lane: no cross-lane unpacking), all of the row's loads in flight at once,
//     and the wave's NEXT row (rows strided over the grid) is issued before the current one
//     is computed;
//   * the activation row(s) are decoded once per workgroup into LDS (quads, d, s or sum b);
//     those loads are issued before the row stream so waiting for them does not wait for HBM;
//   * the q4_0 / q5_0 offset is applied in the integer domain (sum (q-c) b = sum q b - c sum b);
//   * the 64 lane partials reduce through DPP + readlane in a fixed order (deterministic).
// Bytes per call are the algorithmic A + B + C (A streamed once, non-temporal).
#include <hip/hip_ext.h>

#include "lamm_aql.h"
#include "lamm_rowdot.h"

#include <cstdlib>
#include "lamm_knobs.h"

namespace lamm {
namespace {

// One wave per row: the row's loads for ITER blocks per lane (K <= ITER * 2048) go out at once;
// each wave also issues its NEXT row's loads before computing the current one (rows strided by
// the grid), so a persistent grid keeps HBM busy across rows.
template <int T, int NC, int WAVES, bool BF32, int ITER, bool LB>
__global__ __launch_bounds__(64 * WAVES) void gemv_rpw_kernel(GemvArgs p) {
  using F = RFmt<T>;
  constexpr int NWA = (F::BPB + 3) / 4 + 1;     // A dwords per block incl. realignment slack
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nb = p.nblk;
  u32x4* sq0 = reinterpret_cast<u32x4*>(smem_raw);
  u32x4* sq1 = sq0 + NC * nb;
  float* sbd = reinterpret_cast<float*>(sq1 + NC * nb);
  float* sbs = sbd + NC * nb;

  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // The prologue is on the critical path of a ~4 us launch: the first loads wait for every
  // instruction before them, so nothing here divides unless the launch has several slices
  // (round 2's prologue -- four runtime divisions, ~220 instructions before the first load --
  // cost ~0.5 us per config-2 call, profiles/r03/gemv_probe_*.json: lib vs R16)
  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if (gridDim.y > 1) {
    const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  const int ncols = p.N < NC ? p.N : NC;
  const uint32_t row_bytes = (uint32_t)((nb * F::BPB + 3) & ~3);
  const int stride = gridDim.x * WAVES;

  auto issue = [&](int64_t row, uint32_t (&wa)[ITER][NWA]) {
    const auto ra = make_rsrc(Az + row * p.lda, row_bytes);
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int b = lane + 64 * it;
      const uint32_t off = b < nb ? (uint32_t)(b * F::BPB) & ~3u : 0x7ffffff0u;
      load_block_words<F::BPB, 2>(ra, off, wa[it]);   // non-temporal: A is read once
    }
  };
  // LANEB (q8 activations, one column, K <= 4096): each lane holds the two activation blocks its
  // own weight blocks meet, loaded straight from L2 -- no LDS staging, no workgroup barrier
  // (profiles/r02/rpw_probe.txt: the staging + barrier cost 0.36 us of a 3.6 us launch, per-lane
  // loads 0.2).  Same bytes, same block arithmetic: C is bit-identical either way.
  constexpr bool LANEB = LB && !BF32 && NC == 1 && ITER == 2;
  uint32_t lq[ITER][8];
  float ld[ITER], ls[ITER];
  // ITER = 2 (64 < nblk <= 128): each 64-block run reduces on its own and the two run sums add in
  // run order -- gemv_flat_kernel's order, so a row's value does not depend on which of the two
  // kernels the launch's row count picks (a sharded weight's 1024-row slab vs the whole 4096)
  constexpr int NR = ITER == 2 ? 2 : 1;
  auto compute = [&](int64_t row, const uint32_t (&wa)[ITER][NWA]) {
    float accr[NR][NC];
#pragma unroll
    for (int r = 0; r < NR; ++r)
#pragma unroll
      for (int j = 0; j < NC; ++j) accr[r][j] = 0.f;
#pragma unroll
    for (int it = 0; it < ITER; ++it) {
      const int b = lane + 64 * it;
      float (&acc)[NC] = accr[NR == 2 ? it : 0];
      if (b < nb) {
        uint32_t m[NWA - 1];
        realign(wa[it], m, (int)((uint32_t)(b * F::BPB) & 3u));
        uint32_t q[8];
        float da, ma;
        unpack_a<T>(m, q, da, ma);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          u32x4 b0, b1;
          float db, bsv;
          if constexpr (LANEB) {
            b0 = u32x4{lq[it][0], lq[it][1], lq[it][2], lq[it][3]};
            b1 = u32x4{lq[it][4], lq[it][5], lq[it][6], lq[it][7]};
            db = ld[it];
            bsv = ls[it];
          } else {
            b0 = sq0[j * nb + b];
            b1 = sq1[j * nb + b];
            db = sbd[j * nb + b];
            bsv = sbs[j * nb + b];
          }
          int s = 0;
          s = dot4(q[0], b0[0], s); s = dot4(q[1], b0[1], s); s = dot4(q[2], b0[2], s); s = dot4(q[3], b0[3], s);
          s = dot4(q[4], b1[0], s); s = dot4(q[5], b1[1], s); s = dot4(q[6], b1[2], s); s = dot4(q[7], b1[3], s);
          if constexpr (T == kQ4_0) s -= 8 * __builtin_bit_cast(int, bsv);
          if constexpr (T == kQ5_0) s -= 16 * __builtin_bit_cast(int, bsv);
          if constexpr (T == kQ4_1 || T == kQ5_1)
            acc[j] = __builtin_fmaf(da * db, (float)s, __builtin_fmaf(ma, bsv, acc[j]));
          else
            acc[j] = __builtin_fmaf(da * db, (float)s, acc[j]);
        }
      }
    }
    float acc[NC];
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      acc[j] = wave_sum(accr[0][j]);   // 64-lane reduction, fixed order
      if constexpr (NR == 2) acc[j] += wave_sum(accr[1][j]);
    }
    if (lane == 0) {
#pragma unroll
      for (int j = 0; j < NC; ++j)
        if (j < ncols) Cz[(int64_t)j * p.ldc + row] = acc[j];
    }
  };

  int64_t row = (int64_t)blockIdx.x * WAVES + wave;
  uint32_t wa0[ITER][NWA], wa1[ITER][NWA];
  const auto rb = act_rsrc<T, NC, BF32>(p, Bz);
  const int nact = NC * nb;
  ActStage<T, BF32> st;
  const int t0 = threadIdx.x;
  if constexpr (LANEB) {
    ActStage<T, BF32> st1;
    st.template load<NC>(p, rb, lane);        // this lane's activation blocks lane, lane + 64
    st1.template load<NC>(p, rb, lane + 64);
    __builtin_amdgcn_sched_barrier(0);   // ahead of the row's HBM stream in the vmcnt order
    issue(row < p.M ? row : 0, wa0);
    __builtin_amdgcn_sched_barrier(0);
    st.decode(lq[0], ld[0], ls[0]);
    st1.decode(lq[1], ld[1], ls[1]);
  } else if (BF32 && 2 * nact <= (int)blockDim.x) {
    // F32 rows in one pass, several lanes per block (ActStageL): 4 when the threads cover it
    // (4096 x 4096 F32 5.12 -> 4.41 us), else 2.  (Three passes with every load up front
    // measured slower on every shape, profiles/r02/ab_gemv_f32_staging.txt.)
    auto stage = [&](auto lanes) {
      constexpr int LN = decltype(lanes)::value;
      ActStageL<T, LN> sl;
      sl.template load<NC>(p, rb, t0);
      __builtin_amdgcn_sched_barrier(0);   // keep the activation loads first in the vmcnt order
      issue(row < p.M ? row : 0, wa0);
      __builtin_amdgcn_sched_barrier(0);
      if (t0 < LN * nact) sl.store(t0, sq0, sq1, sbd, sbs);
    };
    if (4 * nact <= (int)blockDim.x)
      stage(std::integral_constant<int, 4>{});
    else
      stage(std::integral_constant<int, 2>{});
    __syncthreads();
  } else {
    // the activation loads ahead of the row's HBM stream (the sched barriers keep them first in
    // the vmcnt order and the decode behind the A loads), issued only by the waves that hold a
    // block: a scalar branch -- letting every wave issue them with out-of-range offsets (zeros)
    // cost 0.16 us per config-2 launch (tools/gemv_probe.hip G8 vs G8-allstage,
    // profiles/r03/gemv_probe_11.json)
    if (wave * 64 < nact) st.template load<NC>(p, rb, t0);
    __builtin_amdgcn_sched_barrier(0);   // keep the activation loads first in the vmcnt order
    issue(row < p.M ? row : 0, wa0);
    __builtin_amdgcn_sched_barrier(0);
    if (t0 < nact) {
      st.pin();
      st.store(t0, sq0, sq1, sbd, sbs);
    }
    for (int it = t0 + blockDim.x; it < nact; it += blockDim.x) {
      st.template load<NC>(p, rb, it);
      st.store(it, sq0, sq1, sbd, sbs);
    }
    __syncthreads();
  }
  while (row < p.M) {
    int64_t next = row + stride;
    if (next < p.M) issue(next, wa1);
    compute(row, wa0);
    row = next;
    if (row >= p.M) break;
    next = row + stride;
    if (next < p.M) issue(next, wa0);
    compute(row, wa1);
    row = next;
  }
  if (p.flag) signal_done(p);
}

// Single-column decode, 64 (ITER - 1) < nblk <= 64 ITER blocks per row (ITER = 2, K = 4096: config
// 2 and every Llama-7B projection but ffn_down -- a 6-run instance for ffn_down's K = 11008 measured
// no faster than gemv_rpw_kernel in the decode step, profiles/r03/decode_step/): the workgroup's WAVES
// rows as ONE flat list of WAVES * ITER runs of 64 blocks, wave w's load k taking run
// m = k WAVES + w (row m / ITER, blocks (m % ITER) 64 + lane) -- so the workgroup's first loads
// cover contiguous bytes (the fastest read order on this chip: profiles/r03/gemv_probe_4.json
// rw8x8 2.75 us vs 3.41 row by row) -- each run lies in one row; a wave reduces each run (fixed
// DPP order), the runs of a row are summed in LDS in run order (deterministic), one store per
// row.  Blocks past nblk (the last run of a ragged row) and rows past M load zeros and store
// nothing.
// The body takes plain values: the slice offsets (SL) and the completion signal (gemv_flat_kernel's
// SIG) stay outside it, so a one-slice launch without a signal reads nothing but its scalar
// arguments (gemv_flat1_kernel: preloaded into SGPRs, no kernarg load before the first A load and
// none after the last one).
template <int T, int WAVES, bool BF32, int ITER>
__device__ __forceinline__ void flat_body(const unsigned char* Az, uint32_t lda, const unsigned char* Bz, float* Cz,
                                          int M, int nblk, int group) {
  using F = RFmt<T>;
  constexpr int NWA = (F::BPB + 3) / 4 + 1;
  constexpr int NB = 64 * ITER, NT = 64 * WAVES;
  __shared__ u32x4 sq0[NB], sq1[NB];
  __shared__ float sbd[NB], sbs[NB];
  __shared__ float part[WAVES * ITER];
  const int lane = threadIdx.x & 63, t0 = threadIdx.x;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row0 = group * WAVES;
  const int nrows = M - row0 < WAVES ? M - row0 : WAVES;
  // A resource over this workgroup's rows, ending at its last row's last block byte
  const auto ra = make_rsrc(Az + (int64_t)row0 * lda, (uint32_t)(nrows - 1) * lda + ((nblk * F::BPB + 3) & ~3));
  uint32_t wa[ITER][NWA];
  auto issue = [&]() {
#pragma unroll
    for (int k = 0; k < ITER; ++k) {
      const int m = k * WAVES + w, r = m / ITER, bi = (m % ITER) * 64 + lane;   // wave-uniform run m
      const uint32_t off = bi < nblk ? (uint32_t)r * lda + ((uint32_t)(bi * F::BPB) & ~3u) : 0x7ffffff0u;
      load_block_words<F::BPB, 2>(ra, off, wa[k]);
    }
  };
  const auto rb = make_rsrc(Bz, BF32 ? (uint32_t)nblk * 128 : (uint32_t)(nblk * F::VBPB + 3) & ~3u);
  GemvArgs p{};   // what the staging reads of it: one column of nblk blocks at B
  p.N = 1;
  p.nblk = nblk;
  if constexpr (BF32) {   // F32 rows: four (or two) lanes per block, one pass
    constexpr int LB = 4 * NB <= NT ? 4 : 2;
    static_assert(LB * NB <= NT, "one staging pass");
    ActStageL<T, LB> sl;
    sl.template load<1>(p, rb, t0);
    __builtin_amdgcn_sched_barrier(0);
    issue();
    __builtin_amdgcn_sched_barrier(0);
    if (t0 < LB * NB) sl.store(t0, sq0, sq1, sbd, sbs);
  } else {
    static_assert(NB <= NT, "one staging pass");
    ActStage<T, false> st;
    if (w * 64 < NB) st.template load<1>(p, rb, t0);   // the two waves that hold a block (scalar branch)
    __builtin_amdgcn_sched_barrier(0);
    issue();
    __builtin_amdgcn_sched_barrier(0);
    if (t0 < NB) {
      st.pin();
      st.store(t0, sq0, sq1, sbd, sbs);
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < ITER; ++k) {
    const int m = k * WAVES + w, bi = (m % ITER) * 64 + lane;
    uint32_t mm[NWA - 1];
    realign(wa[k], mm, (int)((uint32_t)(bi * F::BPB) & 3u));
    uint32_t q[8];
    float da, ma;
    unpack_a<T>(mm, q, da, ma);   // blocks past nblk: all-zero bytes -> d = 0, no contribution
    const u32x4 b0 = sq0[bi], b1 = sq1[bi];
    const float db = sbd[bi], bsv = sbs[bi];
    int sdot = 0;
    sdot = dot4(q[0], b0[0], sdot); sdot = dot4(q[1], b0[1], sdot); sdot = dot4(q[2], b0[2], sdot);
    sdot = dot4(q[3], b0[3], sdot); sdot = dot4(q[4], b1[0], sdot); sdot = dot4(q[5], b1[1], sdot);
    sdot = dot4(q[6], b1[2], sdot); sdot = dot4(q[7], b1[3], sdot);
    if constexpr (T == kQ4_0) sdot -= 8 * __builtin_bit_cast(int, bsv);
    if constexpr (T == kQ5_0) sdot -= 16 * __builtin_bit_cast(int, bsv);
    float acc;
    if constexpr (T == kQ4_1 || T == kQ5_1)
      acc = __builtin_fmaf(da * db, (float)sdot, ma * bsv);
    else
      acc = da * db * (float)sdot;
    acc = wave_sum(acc);
    if (lane == 0) part[m] = acc;
  }
  __syncthreads();
  if (t0 < nrows) {
    float c = part[t0 * ITER];
#pragma unroll
    for (int k = 1; k < ITER; ++k) c += part[t0 * ITER + k];
    Cz[row0 + t0] = c;   // (a write-through store here measured no faster, profiles/r03/write_through/)
  }
}

// SL: more than one slice; SIG: the launch carries the boundary's completion signal
template <int T, int WAVES, bool BF32, int ITER, bool SL, bool SIG>
__global__ __launch_bounds__(64 * WAVES) void gemv_flat_kernel(GemvArgs p) {
  const unsigned char* Az = p.A;
  const unsigned char* Bz = p.B;
  float* Cz = p.C;
  if constexpr (SL) {
    const int z = blockIdx.y, i12 = z % p.ne12, i13 = z / p.ne12;
    Az += (int64_t)(i12 / p.r2) * p.sa2 + (int64_t)(i13 / p.r3) * p.sa3;
    Bz += (int64_t)i12 * p.sb2 + (int64_t)i13 * p.sb3;
    Cz += (int64_t)i12 * p.sc2 + (int64_t)i13 * p.sc3;
  }
  flat_body<T, WAVES, BF32, ITER>(Az, (uint32_t)p.lda, Bz, Cz, p.M, p.nblk, blockIdx.x);   // lda < 2^16: nb <= 64 ITER
  if constexpr (SIG) signal_done(p);
}

// One slice, no signal, K = 4096 (BASELINE config 2 as bench.py and the device API launch it)
template <int T, bool BF32>
__global__ __launch_bounds__(512) void gemv_flat1_kernel(const unsigned char* A, const unsigned char* B, float* C,
                                                         uint32_t lda, int M) {
  // XCD-aware row groups: workgroup b runs on XCD b % 8 (round-robin dispatch); give each XCD a
  // contiguous range of groups, so its rows' C lines are written from one L2 (probe G8-xcd vs G8,
  // profiles/r03/gemv_probe_12/13.json)
  const int n = gridDim.x, x = blockIdx.x & 7, k = blockIdx.x >> 3, q = n >> 3, r = n & 7;
  const int group = x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
  flat_body<T, 8, BF32, 2>(A, lda, B, C, M, 128, group);
}

// Several weights times the same activation column in one launch (lamm_hip_matmul_group in the fast
// order: llama.cpp's wq / wk / wv and ffn gate / up decode calls, the ggml boundary's sibling calls):
// blockIdx.y picks the weight, blockIdx.x its 8-row group in gemv_flat1_kernel's XCD-aware order over
// the longest weight's groups (groups past a shorter weight's rows return at once).  Each row runs
// flat_body exactly as in gemv_flat1_kernel, so every C[i] has the bits of its own single call.
template <int T, bool BF32>
__global__ __launch_bounds__(512) void gemv_flat_group_kernel(RefSegs sg, const unsigned char* B, uint32_t lda) {
  const int z = blockIdx.y, M = sg.M[z];
  const int n = gridDim.x, x = blockIdx.x & 7, k = blockIdx.x >> 3, q = n >> 3, r = n & 7;
  const int group = x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
  if (group * 8 >= M) return;
  flat_body<T, 8, BF32, 2>(sg.A[z], lda, B, sg.C[z], M, 128, group);
}

// The k-quant formats against q8_K, one column, K <= 12288 (the reference's Q2_K kernel,
// src/lamm_kernel_q2_k.hpp, whose block dot is LC/ggml-quants.c ggml_vec_dot_q2_K_q8_K; q4_K /
// q5_K, SURVEY §8f: ggml_vec_dot_q4_K_q8_K / _q5_K_q8_K): one wave per row, lane l on super-block
// 16 c + l / 4 (c < ITER) and its quarter qq = l % 4 = 64 consecutive elements; the activation row
// staged once per workgroup in LDS (q8_K: d, 256 quants, 16 bsums; 80 dwords per super-block so a
// quarter's 64 quants are four aligned ds_read_b128).  A super-block's four quarters meet in their
// quad by DPP on the integer sums (exact), then the reference's
//   d_b (d_a sum_s sc_s sum q b - dmin sum_s mn_s bsums_s)
// runs once per super-block; the wave's super-blocks reduce in a fixed DPP order.  Per quarter:
//   q2_K: sub-blocks 4qq..4qq+3 (16 elements each): 32 bytes of qs read at two shifts, 4 scale
//         bytes (4-bit scale | 4-bit min), d / dmin
//   q4_K: sub-blocks 2qq, 2qq+1 (32 elements each): 32 bytes of qs (low / high nibbles), the
//         6-bit scales / mins of both (LC/ggml-quants.c's utmp shuffle), d / dmin
//   q5_K: as q4_K, plus bit sb of qh[l] as the 5th bit
template <int T> struct KQ;
template <> struct KQ<kQ2_K> { static constexpr int BPB = 84; };
template <> struct KQ<kQ4_K> { static constexpr int BPB = 144; };
template <> struct KQ<kQ5_K> { static constexpr int BPB = 176; };
template <> struct KQ<kQ6_K> { static constexpr int BPB = 210; };

#ifndef KQ_WAVES
#define KQ_WAVES 8   // rows (waves) per workgroup (probe builds: 4, 16)
#endif
template <int T, int ITER>
__global__ __launch_bounds__(64 * KQ_WAVES) void gemv_kq_kernel(const unsigned char* A, int64_t lda, const unsigned char* B,
                                                                float* C, int M, int nsb) {
  constexpr int WAVES = KQ_WAVES, NSB = 16 * ITER, SBW = 80, SDW = NSB * 73, PASS = (SDW + 64 * WAVES - 1) / (64 * WAVES);
  constexpr int BPB = KQ<T>::BPB;
  __shared__ __attribute__((aligned(16))) uint32_t act[NSB * SBW];
  const int lane = threadIdx.x & 63, t0 = threadIdx.x, qq = lane & 3;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int row = blockIdx.x * WAVES + w;
  const auto rb = make_rsrc(B, (uint32_t)nsb * 292);
  uint32_t sv[PASS];
#pragma unroll
  for (int k = 0; k < PASS; ++k) {
    const int idx = t0 + 64 * WAVES * k;
    sv[k] = bload4(rb, idx < SDW ? (uint32_t)idx * 4 : 0x7ffffff0u);   // past the row: zeros
  }
  __builtin_amdgcn_sched_barrier(0);   // the activation loads first in the vmcnt order
  const auto ra = make_rsrc(A + (int64_t)(row < M ? row : 0) * lda, ((uint32_t)nsb * BPB + 3) & ~3u);
  // this lane's bytes of each of its super-blocks: qs (32 B), the header, and for q5_K qh (32 B);
  // q6_K: ql (2 x 16 B) and qh (16 B) of its 64 elements, 2-byte aligned (210-byte super-blocks)
  u32x4 qa[ITER][2], hd[ITER], qh[ITER][2];
  uint32_t sc[ITER], sc6[ITER][2];
#pragma unroll
  for (int c = 0; c < ITER; ++c) {
    const int sb = 16 * c + (lane >> 2);
    const uint32_t base = sb < nsb ? (uint32_t)sb * BPB : 0x7fff0000u;
    if constexpr (T == kQ6_K) {
      // quarter qq = (half j, 16-element column t): elements 128 j + 32 g + 16 t + i (g < 4, i < 16):
      // ql[64 j + 16 t ..] (g = 0, 2: low / high nibbles), ql[64 j + 32 + 16 t ..] (g = 1, 3),
      // qh[32 j + 16 t ..] (bits 2 g), scales sc[8 j + 2 g + t], d at 208
      const int j = qq >> 1, t = qq & 1;
      const uint32_t b4 = base & ~3u;
      const int shb = (int)(base & 3u) * 8;
      auto chunk16 = [&](uint32_t o) {   // 16 bytes at base + o (o a multiple of 4)
        const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(ra, b4 + o, 0, 2);
        const uint32_t w4 = __builtin_amdgcn_raw_buffer_load_b32(ra, b4 + o + 16, 0, 2);
        return u32x4{__builtin_amdgcn_alignbit(v[1], v[0], shb), __builtin_amdgcn_alignbit(v[2], v[1], shb),
                     __builtin_amdgcn_alignbit(v[3], v[2], shb), __builtin_amdgcn_alignbit(w4, v[3], shb)};
      };
      qa[c][0] = chunk16(64 * j + 16 * t);
      qa[c][1] = chunk16(64 * j + 32 + 16 * t);
      qh[c][0] = chunk16(128 + 32 * j + 16 * t);
      // scales 8 j .. 8 j + 7 and d (bytes 192 + 8 j .., 208): three dwords from the dword below
      const uint32_t s0 = __builtin_amdgcn_raw_buffer_load_b32(ra, b4 + 192 + 8 * j, 0, 2);
      const uint32_t s1 = __builtin_amdgcn_raw_buffer_load_b32(ra, b4 + 196 + 8 * j, 0, 2);
      const uint32_t s2 = __builtin_amdgcn_raw_buffer_load_b32(ra, b4 + 200 + 8 * j, 0, 2);
      sc6[c][0] = __builtin_amdgcn_alignbit(s1, s0, shb);
      sc6[c][1] = __builtin_amdgcn_alignbit(s2, s1, shb);
      hd[c][0] = __builtin_amdgcn_raw_buffer_load_b32(ra, b4 + 208, 0, 2);   // d = bits [shb, shb + 16)
    } else if constexpr (T == kQ2_K) {
      const uint32_t qo = base + 16 + 32 * (qq >> 1);
      qa[c][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, qo, 0, 2);
      qa[c][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, qo + 16, 0, 2);
      sc[c] = __builtin_amdgcn_raw_buffer_load_b32(ra, base + 4 * qq, 0, 2);
      hd[c][0] = __builtin_amdgcn_raw_buffer_load_b32(ra, base + 80, 0, 2);   // d | dmin
    } else {
      constexpr int QS = T == kQ5_K ? 48 : 16;
      hd[c] = __builtin_amdgcn_raw_buffer_load_b128(ra, base, 0, 2);   // d | dmin, scales[12]
      qa[c][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + QS + 32 * qq, 0, 2);
      qa[c][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + QS + 32 * qq + 16, 0, 2);
      if constexpr (T == kQ5_K) {
        qh[c][0] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + 16, 0, 2);
        qh[c][1] = __builtin_amdgcn_raw_buffer_load_b128(ra, base + 32, 0, 2);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int k = 0; k < PASS; ++k) {   // dword k of a 73-dword super-block: d -> 0, quants / bsums -> 3 + k
    const int idx = t0 + 64 * WAVES * k;
    if (idx < SDW) {
      const int sb = idx / 73, kk = idx % 73;
      act[sb * SBW + (kk ? 3 + kk : 0)] = sv[k];
    }
  }
  __syncthreads();
  float acc = 0.f;
#pragma unroll
  for (int c = 0; c < ITER; ++c) {
    const int sb = 16 * c + (lane >> 2);
    const uint32_t* a = &act[sb * SBW];
    u32x4 b[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) b[i] = *reinterpret_cast<const u32x4*>(a + 4 + 16 * qq + 4 * i);
    const uint2 bsw = *reinterpret_cast<const uint2*>(a + 68 + 2 * qq);   // bsums 4qq .. 4qq + 3 (int16)
    auto bsum = [&](int i) { return (int)(int16_t)(((i < 2 ? bsw.x : bsw.y) >> (16 * (i & 1))) & 0xffffu); };
    const float yd = __builtin_bit_cast(float, a[0]);
    int isum = 0, summs = 0;
    uint32_t dd;
    if constexpr (T == kQ6_K) {
      // (q - 32) b = q b - 32 b: the sum of b per 16 elements is the q8_K bsum of that group
      const int j = qq >> 1, t = qq & 1;
      dd = (hd[c][0] >> (((uint32_t)(16 * c + (lane >> 2)) * 210u & 3u) * 8)) & 0xffffu;
      const u32x4 bj[4] = {*reinterpret_cast<const u32x4*>(a + 4 + 32 * j + 4 * t),
                           *reinterpret_cast<const u32x4*>(a + 4 + 32 * j + 8 + 4 * t),
                           *reinterpret_cast<const u32x4*>(a + 4 + 32 * j + 16 + 4 * t),
                           *reinterpret_cast<const u32x4*>(a + 4 + 32 * j + 24 + 4 * t)};
      const uint32_t* bs = a + 68;   // 16 int16 bsums, two per dword
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        int part = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t lo = (qa[c][g & 1][k] >> (g >= 2 ? 4 : 0)) & 0x0f0f0f0fu;
          const uint32_t q = lo | (((qh[c][0][k] >> (2 * g)) & 0x03030303u) << 4);
          part = dot4(q, bj[g][k], part);
        }
        const int bi = 8 * j + 2 * g + t;
        const int bsum = (int)(int16_t)((bs[bi >> 1] >> (16 * (bi & 1))) & 0xffffu);
        const int scv = (int)(int8_t)((sc6[c][g >> 1] >> (8 * (2 * (g & 1) + t))) & 0xffu);
        isum += scv * (part - 32 * bsum);
      }
    } else if constexpr (T == kQ2_K) {
      dd = hd[c][0];
#pragma unroll
      for (int i = 0; i < 4; ++i) {   // sub-block s = 4 qq + i: half i & 1 of the qs run, shift 2 jj
        const int sh = 2 * (2 * (qq & 1) + (i >> 1));
        const int scv = (int)((sc[c] >> (8 * i)) & 0xffu);
        int part = 0;
#pragma unroll
        for (int k = 0; k < 4; ++k) part = dot4((qa[c][i & 1][k] >> sh) & 0x03030303u, b[i][k], part);
        isum += (scv & 0xf) * part;
        summs += bsum(i) * (scv >> 4);
      }
    } else {
      dd = hd[c][0];
      // the 6-bit scales / mins of the 8 sub-blocks (LC/ggml-quants.c:7324-7330's utmp shuffle),
      // then this quarter's two: sub-blocks 2 qq, 2 qq + 1
      uint32_t u0 = hd[c][1], u1 = hd[c][2], u2 = hd[c][3];
      const uint32_t u3 = ((u2 >> 4) & 0x0f0f0f0fu) | (((u1 >> 6) & 0x03030303u) << 4);
      const uint32_t uaux = u1 & 0x3f3f3f3fu;
      u1 = (u2 & 0x0f0f0f0fu) | (((u0 >> 6) & 0x03030303u) << 4);
      u2 = uaux;
      u0 &= 0x3f3f3f3fu;
      const uint32_t scw = qq < 2 ? u0 : u1, mnw = qq < 2 ? u2 : u3;
      const int sh = 16 * (qq & 1);
#pragma unroll
      for (int h = 0; h < 2; ++h) {   // sub-block 2 qq + h: nibble h of the 32 qs bytes
        const int scv = (int)((scw >> (sh + 8 * h)) & 0xffu), mnv = (int)((mnw >> (sh + 8 * h)) & 0xffu);
        int part = 0;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          uint32_t q = (qa[c][k >> 2][k & 3] >> (4 * h)) & 0x0f0f0f0fu;
          if constexpr (T == kQ5_K) q |= ((qh[c][k >> 2][k & 3] >> (2 * qq + h)) & 0x01010101u) << 4;
          part = dot4(q, b[2 * h + (k >> 2)][k & 3], part);
        }
        isum += scv * part;
        summs += mnv * (bsum(2 * h) + bsum(2 * h + 1));
      }
    }
    // the quad's four quarters of one super-block (integer: exact)
    isum += __builtin_amdgcn_update_dpp(0, isum, 0xB1, 0xF, 0xF, false);
    isum += __builtin_amdgcn_update_dpp(0, isum, 0x4E, 0xF, 0xF, false);
    summs += __builtin_amdgcn_update_dpp(0, summs, 0xB1, 0xF, 0xF, false);
    summs += __builtin_amdgcn_update_dpp(0, summs, 0x4E, 0xF, 0xF, false);
    if (qq == 0 && sb < nsb) {
      if constexpr (T == kQ6_K) {
        acc += (yd * h2f(dd)) * (float)isum;
      } else {
        const float da = h2f(dd & 0xffffu), dm = h2f(dd >> 16);
        acc += (yd * da) * (float)isum - (yd * dm) * (float)summs;
      }
    }
  }
  acc = wave_sum(acc);
  if (lane == 0 && row < M) C[row] = acc;
}

template <int T, int NC, int WAVES, bool BF32, int ITER>
hipError_t launch_rpw_k(const GemvArgs& p, hipStream_t s) {
  // LAMM_GEMV_LANEB=1: per-lane activation blocks for q8 single-column calls (A/B)
  const bool laneb = !BF32 && NC == 1 && ITER == 2 && knobs().gemv_laneb;
  const size_t lds = laneb ? 0 : (size_t)NC * p.nblk * 40;
  const int slices = p.ne12 * p.ne13;
  const int gmax = (p.M + WAVES - 1) / WAVES;
  // one round of workgroups over the chip: ~2 per CU in total across the slices
  int gx = (512 + slices - 1) / slices;
  gx = gx < 1 ? 1 : (gx > gmax ? gmax : gx);
  if (lds > 64 * 1024) return hipErrorInvalidValue;
  if (laneb)
    hipLaunchKernelGGL((gemv_rpw_kernel<T, NC, WAVES, BF32, ITER, true>), dim3(gx, slices), dim3(64 * WAVES), lds, s, p);
  else
    hipLaunchKernelGGL((gemv_rpw_kernel<T, NC, WAVES, BF32, ITER, false>), dim3(gx, slices), dim3(64 * WAVES), lds, s,
                       p);
  return hipGetLastError();
}

template <int T, int NC>
hipError_t launch_rpw_nc(const GemvArgs& p, hipStream_t s, int waves) {
  const bool bf = p.b_f32 != 0;
  // one column, K = 4096 (128 blocks): the flat-run kernel, 8 waves
  if constexpr (NC == 1) {
    if (p.nblk == 128 && waves == 8 && !knobs().gemv_laneb) {
      const dim3 g((unsigned)((p.M + 7) / 8), (unsigned)(p.ne12 * p.ne13));
      const bool sl = g.y > 1, sig = p.flag != nullptr;
      if (!sl && !sig) {
        const uint32_t lda = (uint32_t)p.lda;
        const LaunchTiming tm = take_launch_timing();
        if (tm.start) {   // lamm_hip_profile_next: the dispatch records its own start / end
          if (bf) hipExtLaunchKernelGGL((gemv_flat1_kernel<T, true>), g, dim3(512), 0, s, tm.start, tm.stop, 0, p.A, p.B,
                                        p.C, lda, p.M);
          else hipExtLaunchKernelGGL((gemv_flat1_kernel<T, false>), g, dim3(512), 0, s, tm.start, tm.stop, 0, p.A, p.B,
                                     p.C, lda, p.M);
          return hipGetLastError();
        }
        // direct region open (lamm_aql.cpp): the library's own queue; the explicit arguments as the
        // kernel declares them
        struct {
          const unsigned char* A;
          const unsigned char* B;
          float* C;
          uint32_t lda;
          int M;
        } a{p.A, p.B, p.C, lda, p.M};
        const void* fn = bf ? reinterpret_cast<const void*>(gemv_flat1_kernel<T, true>)
                            : reinterpret_cast<const void*>(gemv_flat1_kernel<T, false>);
        if (direct_launch(fn, g, dim3(512), 0, &a, sizeof a)) return hipSuccess;
        if (bf) hipLaunchKernelGGL((gemv_flat1_kernel<T, true>), g, dim3(512), 0, s, p.A, p.B, p.C, lda, p.M);
        else hipLaunchKernelGGL((gemv_flat1_kernel<T, false>), g, dim3(512), 0, s, p.A, p.B, p.C, lda, p.M);
        return hipGetLastError();
      }
      auto go = [&](auto bfc, auto slc, auto sgc) {
        hipLaunchKernelGGL((gemv_flat_kernel<T, 8, decltype(bfc)::value, 2, decltype(slc)::value, decltype(sgc)::value>),
                           g, dim3(512), 0, s, p);
      };
      using t_ = std::true_type;
      using f_ = std::false_type;
      if (bf) {
        if (sl) sig ? go(t_{}, t_{}, t_{}) : go(t_{}, t_{}, f_{});
        else go(t_{}, f_{}, t_{});
      } else {
        if (sl) sig ? go(f_{}, t_{}, t_{}) : go(f_{}, t_{}, f_{});
        else go(f_{}, f_{}, t_{});
      }
      return hipGetLastError();
    }
  }
  if (p.nblk <= 128) {
    if (waves >= 16) return bf ? launch_rpw_k<T, NC, 16, true, 2>(p, s) : launch_rpw_k<T, NC, 16, false, 2>(p, s);
    if (waves >= 8) return bf ? launch_rpw_k<T, NC, 8, true, 2>(p, s) : launch_rpw_k<T, NC, 8, false, 2>(p, s);
    return bf ? launch_rpw_k<T, NC, 4, true, 2>(p, s) : launch_rpw_k<T, NC, 4, false, 2>(p, s);
  }
  if (waves >= 16 && bf) return launch_rpw_k<T, NC, 16, true, 6>(p, s);   // F32: staging in one pass
  if (waves >= 8) return bf ? launch_rpw_k<T, NC, 8, true, 6>(p, s) : launch_rpw_k<T, NC, 8, false, 6>(p, s);
  return bf ? launch_rpw_k<T, NC, 4, true, 6>(p, s) : launch_rpw_k<T, NC, 4, false, 6>(p, s);
}

template <int T>
hipError_t launch_rpw_t(const GemvArgs& p, hipStream_t s, int waves) {
  if (p.N <= 1) return launch_rpw_nc<T, 1>(p, s, waves);
  return launch_rpw_nc<T, 2>(p, s, waves);
}

}  // namespace

// Up to which row count the row-per-wave form beats the wave-group kernels (single calls, K = 4096,
// profiles/r03/gemv_kq/): q2_K / q4_K faster at 4096 and 11008 rows, slower at 32000 (the
// wave-group stream wins once the grid is long); q5_K (each lane also reads the whole 32-byte qh)
// faster at 4096 only.
bool gemv_kq_supported(int type, const GemvArgs& p) {
  // q6_K: every row count (a Q4_0 model's 32000-row output.weight, llama.cpp:11731-11742)
  const int max_rows = type == kQ6_K ? (1 << 30) : type == kQ5_K ? 6144 : 16384;
  return (type == kQ2_K || type == kQ4_K || type == kQ5_K || type == kQ6_K) && p.N == 1 && p.ne12 * p.ne13 == 1 &&
         p.nblk <= 48 && p.M <= max_rows && p.flag == nullptr && p.b_f32 == 0;
}

hipError_t launch_gemv_kq(int type, const GemvArgs& p, hipStream_t s) {
  const dim3 g((unsigned)((p.M + KQ_WAVES - 1) / KQ_WAVES));
  auto go = [&](auto tc) {
    constexpr int T = decltype(tc)::value;
    const LaunchTiming tm = take_launch_timing();
    auto go = [&](auto kern) {
      if (tm.start)
        hipExtLaunchKernelGGL(kern, g, dim3(64 * KQ_WAVES), 0, s, tm.start, tm.stop, 0, p.A, p.lda, p.B, p.C, p.M, p.nblk);
      else hipLaunchKernelGGL(kern, g, dim3(64 * KQ_WAVES), 0, s, p.A, p.lda, p.B, p.C, p.M, p.nblk);
    };
    if (p.nblk <= 16) go(gemv_kq_kernel<T, 1>);
    else if (p.nblk <= 32) go(gemv_kq_kernel<T, 2>);
    else go(gemv_kq_kernel<T, 3>);
  };
  switch (type) {
    case kQ2_K: go(std::integral_constant<int, kQ2_K>{}); break;
    case kQ4_K: go(std::integral_constant<int, kQ4_K>{}); break;
    case kQ5_K: go(std::integral_constant<int, kQ5_K>{}); break;
    case kQ6_K: go(std::integral_constant<int, kQ6_K>{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

bool gemv_group_supported(int type, const GemvArgs& p, const RefSegs& sg, int nseg) {
  if (nseg < 1 || nseg > kRefSegs || p.N != 1 || p.nblk != 128 || p.ne12 * p.ne13 != 1 || p.flag ||
      (p.lda & 15) || p.lda >= (1 << 16) || !gemv_rpw_supported(type, p) || knobs().gemv_rpw >= 0 || knobs().gemv_laneb)
    return false;
  for (int i = 0; i < nseg; ++i) {   // the rows whose single calls are gemv_flat1_kernel (rpw_waves: 8 waves)
    GemvArgs q = p;
    q.M = sg.M[i];
    if (sg.M[i] < 2048 || rpw_waves(q) != 8) return false;
  }
  return true;
}

hipError_t launch_gemv_group(int type, const GemvArgs& p, const RefSegs& sg, int nseg, hipStream_t s) {
  if (!gemv_group_supported(type, p, sg, nseg)) return hipErrorInvalidValue;
  int mmax = 0;
  for (int i = 0; i < nseg; ++i) mmax = sg.M[i] > mmax ? sg.M[i] : mmax;
  const dim3 g((unsigned)((mmax + 7) / 8), (unsigned)nseg);
  const bool bf = p.b_f32 != 0;
  auto go = [&](auto tc) {
    constexpr int T = decltype(tc)::value;
    if (bf) hipLaunchKernelGGL((gemv_flat_group_kernel<T, true>), g, dim3(512), 0, s, sg, p.B, (uint32_t)p.lda);
    else hipLaunchKernelGGL((gemv_flat_group_kernel<T, false>), g, dim3(512), 0, s, sg, p.B, (uint32_t)p.lda);
  };
  switch (type) {
    case kQ4_0: go(std::integral_constant<int, kQ4_0>{}); break;
    case kQ4_1: go(std::integral_constant<int, kQ4_1>{}); break;
    case kQ5_0: go(std::integral_constant<int, kQ5_0>{}); break;
    case kQ5_1: go(std::integral_constant<int, kQ5_1>{}); break;
    case kQ8_0: go(std::integral_constant<int, kQ8_0>{}); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

bool gemv_rpw_supported(int type, const GemvArgs& p) {
  return p.N <= 2 && p.nblk <= 6 * 64 &&
         (type == kQ4_0 || type == kQ4_1 || type == kQ5_0 || type == kQ5_1 || type == kQ8_0);
}

hipError_t launch_gemv_rpw(int type, const GemvArgs& p, hipStream_t s, int waves) {
  switch (type) {
    case kQ4_0: return launch_rpw_t<kQ4_0>(p, s, waves);
    case kQ4_1: return launch_rpw_t<kQ4_1>(p, s, waves);
    case kQ5_0: return launch_rpw_t<kQ5_0>(p, s, waves);
    case kQ5_1: return launch_rpw_t<kQ5_1>(p, s, waves);
    case kQ8_0: return launch_rpw_t<kQ8_0>(p, s, waves);
    default: return hipErrorInvalidValue;
  }
}

}  // namespace lamm
