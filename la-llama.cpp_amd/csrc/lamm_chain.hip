// lamm_chain.hip -- a decode chain: a sequence of single-token GEMVs (per Llama layer
// wq|wk|wv -> wo -> ffn_gate|ffn_up -> ffn_down, layer after layer) as ONE persistent launch.
//
// Why.  One token of Llama-7B is 225 GEMVs of 9-50 MB (build_llama
// LC/llama.cpp:5708-5830); as separate launches each pays the ramp of an empty chip (the first
// row's HBM latency, the activation staging) and drains before the next may start, so the step
// streams weights at ~3 TB/s although one long launch reaches ~6 (profiles/r02/prof_bp_*.txt).
// Weights do not depend on activations: a wave can have the next op's rows in flight while the
// op's input is still being produced.
//
// Structure.
//  * grid = one workgroup per CU, 8 waves each; every phase's rows (the concatenated rows of
//    the ops that share one input) are strided over all waves of the grid, wave w taking rows
//    w, w + S, ... -- the row-per-wave block dot of lamm_gemv_rpw.hip (lamm_rowdot.h), so each
//    op's y is bit-identical to lamm_hip_matmul(A, F32 x);
//  * a wave issues the loads of its next row before computing the current one, across phase
//    boundaries, so while it waits for a phase's input its first row of that phase is landing;
//  * outputs are published as 8-byte {value, tag} granules, one write-through (sc1) store per
//    row; tag = launch sequence * 1024 + phase + 1.  The data is its own flag: a workgroup
//    stages a phase's input by reading the producer's granules with sc1 loads (L1 bypassed) and
//    re-reading until every tag matches -- no counters, fences or grid barriers
//    (MI355X_MICROARCH.md, visibility: R2 granules);
//  * every wait is bounded: a thread that gives up sets the chain's error word and carries on
//    with what it read, so the launch always drains (lamm_hip_chain_status reports it);
//  * the launch sequence number lives in device memory and is advanced by the last workgroup
//    to finish (a kernel argument would be frozen by graph capture), so a replayed graph never
//    mistakes the previous launch's granules for this one's.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "../../include/lamm_hip.h"
#include "lamm_rowdot.h"

namespace lamm {
namespace {

struct ChainOp {
  const unsigned char* A;   // weight rows (lda bytes apart)
  float* y;                 // plain output (read by the caller after the launch)
  uint64_t* g;              // granule output (read by later phases inside the launch)
  int64_t lda;
  int row0, M;              // first row of this op inside its phase, rows
};
struct ChainPhase {
  const float* x;           // external input (src < 0)
  const uint64_t* gx;       // producer's granules (src >= 0)
  int op0, nops, M, nblk, src, npc;   // npc: pieces per row
};
struct ChainArgs {
  const ChainOp* ops;
  const ChainPhase* ph;
  unsigned* ctl;            // [0] launch sequence, [1] finished workgroups, [2] error word
  int nph, nbmax, nops, pad;
  uint64_t* trace;          // LAMM_CHAIN_TRACE: per workgroup [start, (stage begin, end) x nph, end]
};

constexpr int kChainIter = 6;             // blocks per lane: K <= 6 * 64 * 32 = 12288
constexpr int kChainWaves = 8;
constexpr int kPieceBlocks = 128;         // a row streams in pieces of 128 blocks (2 per lane)
#ifndef LAMM_CHAIN_DEPTH
#define LAMM_CHAIN_DEPTH 8
#endif
constexpr int kChainDepth = LAMM_CHAIN_DEPTH;   // pieces in flight per wave
constexpr unsigned kChainPolls = 1u << 19;   // x s_sleep 4 (~256 clk): ~50 ms before giving up
constexpr int kChainMaxPhases = 1023;        // tags: phase + 1 in the low 10 bits
constexpr int kAuxSc1 = 16;                  // buffer cache policy bit: sc1 (write-through / L1 bypass)

// The op / phase tables are copied into LDS at the start: read from there (ds_read, counted by
// lgkmcnt) they never make a wave wait for its in-flight weight rows, which a vector load of the
// table would (vmcnt retires in order), and they stay wave-uniform (readfirstlane).
constexpr int kOpWords = sizeof(ChainOp) / 4, kPhWords = sizeof(ChainPhase) / 4;
static_assert(sizeof(ChainOp) % 8 == 0 && sizeof(ChainPhase) % 8 == 0, "table records are 8-byte aligned");

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
template <class P>
__device__ __forceinline__ P* uni_ptr(const uint32_t* w) {
  const uint64_t v = (uint64_t)(uint32_t)uni((int)w[0]) | ((uint64_t)(uint32_t)uni((int)w[1]) << 32);
  return reinterpret_cast<P*>(v);
}

template <int T, int WAVES>
__global__ __launch_bounds__(64 * WAVES) void gemv_chain_kernel(ChainArgs a) {
  using F = RFmt<T>;
  constexpr int NWA = (F::BPB + 3) / 4 + 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem_raw[];
  const int nbm = a.nbmax;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int gw = blockIdx.x * WAVES + wave;
  const int S = gridDim.x * WAVES;
  const unsigned seq =
      __builtin_amdgcn_readfirstlane(__hip_atomic_load(a.ctl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
  const unsigned tagbase = seq << 10;

  // LDS: [staging buffer 0][staging buffer 1][phase table][op table]
  uint32_t* tph = reinterpret_cast<uint32_t*>(smem_raw + (size_t)2 * nbm * 40);
  uint32_t* top = tph + a.nph * kPhWords;
  {
    const uint32_t* gph = reinterpret_cast<const uint32_t*>(a.ph);
    const uint32_t* gop = reinterpret_cast<const uint32_t*>(a.ops);
    for (int i = threadIdx.x; i < a.nph * kPhWords; i += blockDim.x) tph[i] = gph[i];
    for (int i = threadIdx.x; i < a.nops * kOpWords; i += blockDim.x) top[i] = gop[i];
    __syncthreads();
  }
  // field accessors (word offsets of ChainPhase / ChainOp)
  auto ph_M = [&](int p) { return uni((int)tph[p * kPhWords + 6]); };
  auto ph_nblk = [&](int p) { return uni((int)tph[p * kPhWords + 7]); };
  auto ph_src = [&](int p) { return uni((int)tph[p * kPhWords + 8]); };
  auto ph_op0 = [&](int p) { return uni((int)tph[p * kPhWords + 4]); };
  auto ph_nops = [&](int p) { return uni((int)tph[p * kPhWords + 5]); };
  auto op_row0 = [&](int o) { return uni((int)top[o * kOpWords + 8]); };
  auto op_M = [&](int o) { return uni((int)top[o * kOpWords + 9]); };
  auto op_lda = [&](int o) { return uni((int)top[o * kOpWords + 6]); };

  struct Buf { u32x4* q0; u32x4* q1; float* bd; float* bs; };
  auto buf = [&](int p) {
    unsigned char* base = smem_raw + (size_t)(p & 1) * nbm * 40;
    Buf b;
    b.q0 = reinterpret_cast<u32x4*>(base);
    b.q1 = b.q0 + nbm;
    b.bd = reinterpret_cast<float*>(b.q1 + nbm);
    b.bs = b.bd + nbm;
    return b;
  };
  // op of row r of phase p (ops of a phase are concatenated in order)
  auto locate = [&](int p, int r) {
    const int op0 = ph_op0(p), nops = ph_nops(p);
    int o = op0;
    for (int k = 1; k < nops; ++k)
      if (r >= op_row0(op0 + k)) o = op0 + k;
    return o;
  };
  auto first_from = [&](int p) {
    while (p < a.nph && gw >= ph_M(p)) ++p;
    return p;
  };


  auto ph_npc = [&](int p) { return uni((int)tph[p * kPhWords + 9]); };

  // A wave's work is a sequence of row pieces: phase by phase, its rows w, w + S, ..., each row
  // in pieces of 128 blocks (lane l: blocks 128k + l and 128k + 64 + l -- the order the
  // single-launch kernel adds them in, so sums stay bit-identical).
  struct Cur { int p, r, k; };
  auto next = [&](Cur& c) {
    if (c.p >= a.nph) return;
    if (++c.k < ph_npc(c.p)) return;
    c.k = 0;
    c.r += S;
    if (c.r >= ph_M(c.p)) {
      c.p = first_from(c.p + 1);
      c.r = gw;
    }
  };
  // EVERY call issues the same 4 load instructions (pieces past the chain's end and blocks past
  // a row's end read zeros through an empty / short resource and move no bytes), so the
  // compiler's vmcnt waits stay exact whatever the row's K
  auto issue = [&](const Cur& c, uint32_t (&wa)[2][NWA]) {
    const unsigned char* A = nullptr;
    uint32_t bytes = 0;
    int nb = 0;
    if (c.p < a.nph) {
      const int o = locate(c.p, c.r);
      nb = min(kPieceBlocks, ph_nblk(c.p) - kPieceBlocks * c.k);
      A = uni_ptr<const unsigned char>(top + o * kOpWords) + (int64_t)(c.r - op_row0(o)) * op_lda(o) +
          (int64_t)kPieceBlocks * c.k * F::BPB;
      bytes = (uint32_t)((nb * F::BPB + 3) & ~3);
    }
    const auto ra = make_rsrc(A, bytes);
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int b = lane + 64 * it;
      const uint32_t off = b < nb ? (uint32_t)(b * F::BPB) & ~3u : 0x7ffffff0u;
      load_words<NWA, 2>(ra, off, wa[it]);   // non-temporal: each weight row is read once
    }
  };
  float acc = 0.f;   // the current row's lane partial, carried over its pieces
  auto compute = [&](const Cur& c, const uint32_t (&wa)[2][NWA]) {
    const int nbr = ph_nblk(c.p);
    const Buf B = buf(c.p);
    if (c.k == 0) acc = 0.f;
#pragma unroll
    for (int it = 0; it < 2; ++it) {
      const int b = kPieceBlocks * c.k + lane + 64 * it;
      if (b < nbr) {
        uint32_t m[NWA - 1];
        realign(wa[it], m, (int)((uint32_t)(b * F::BPB) & 3u));
        uint32_t q[8];
        float da, ma;
        unpack_a<T>(m, q, da, ma);
        const u32x4 b0 = B.q0[b], b1 = B.q1[b];
        int s = 0;
        s = dot4(q[0], b0[0], s); s = dot4(q[1], b0[1], s); s = dot4(q[2], b0[2], s); s = dot4(q[3], b0[3], s);
        s = dot4(q[4], b1[0], s); s = dot4(q[5], b1[1], s); s = dot4(q[6], b1[2], s); s = dot4(q[7], b1[3], s);
        const float db = B.bd[b];
        if constexpr (T == kQ4_0) s -= 8 * __builtin_bit_cast(int, B.bs[b]);
        if constexpr (T == kQ5_0) s -= 16 * __builtin_bit_cast(int, B.bs[b]);
        if constexpr (T == kQ4_1 || T == kQ5_1)
          acc = __builtin_fmaf(da * db, (float)s, __builtin_fmaf(ma, B.bs[b], acc));
        else
          acc = __builtin_fmaf(da * db, (float)s, acc);
      }
    }
    if (c.k + 1 < ph_npc(c.p)) return;
    const float v = wave_sum(acc);
    // stored by lane 0; the other lanes' offsets fall outside the resource (dropped)
    const int o = locate(c.p, c.r);
    const uint32_t ri = (uint32_t)(c.r - op_row0(o)), M = (uint32_t)op_M(o);
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v),
                                          make_rsrc(uni_ptr<float>(top + o * kOpWords + 2), M * 4u),
                                          lane == 0 ? ri * 4u : 0x7ffffff0u, 0, 0);
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const u32x2 gv = {__builtin_bit_cast(uint32_t, v), tagbase + (unsigned)c.p + 1u};
    __builtin_amdgcn_raw_buffer_store_b64(gv, make_rsrc(uni_ptr<uint64_t>(top + o * kOpWords + 4), M * 8u),
                                          lane == 0 ? ri * 8u : 0x7ffffff0u, 0, kAuxSc1);
  };

  auto stamp = [&](int k) {   // RTC (100 MHz) for the trace, by one lane of the workgroup
    if (a.trace && threadIdx.x == 0) a.trace[(size_t)blockIdx.x * (2 * a.nph + 2) + k] = __builtin_amdgcn_s_memrealtime();
  };
  auto stage = [&](int p) {
    stamp(1 + 2 * p);
    const int nb = ph_nblk(p), src = ph_src(p);
    const Buf B = buf(p);
    for (int t = threadIdx.x; t < nb; t += blockDim.x) {
      ActStage<T, true> st;
      if (src < 0) {
        load_words<32, 0>(make_rsrc(uni_ptr<const float>(tph + p * kPhWords), (uint32_t)nb * 128u), (uint32_t)t * 128u,
                          st.w);
      } else {
        const unsigned want = tagbase + (unsigned)src + 1u;
        const auto rg = make_rsrc(uni_ptr<const uint64_t>(tph + p * kPhWords + 2), (uint32_t)nb * 256u);
        for (unsigned polls = 0;; ++polls) {
          bool ok = true;
#pragma unroll
          for (int k = 0; k < 16; ++k) {
            const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rg, (uint32_t)t * 256u + 16u * k, 0, kAuxSc1);
            st.w[2 * k] = v[0];
            st.w[2 * k + 1] = v[2];
            ok &= v[1] == want && v[3] == want;
          }
          if (ok) break;
          if (polls >= kChainPolls) {   // give up: flag it, carry on so the launch drains
            atomicOr(&a.ctl[2], 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(4);
          asm volatile("" ::: "memory");   // re-read the granules
        }
      }
      st.store(t, B.q0, B.q1, B.bd, B.bs);
    }
    __syncthreads();
    stamp(2 + 2 * p);
  };

  // kChainDepth pieces in flight per wave, in a ring of register slots named statically (the
  // loop is unrolled over the ring: no branch between slots, exact vmcnt waits).  Phases are
  // staged in order by every wave -- the staging ends in a workgroup barrier -- before the
  // wave's first piece of that phase, and the phases it has no row in are staged too.
  stamp(0);
  constexpr int D = kChainDepth;
  uint32_t wa[D][2][NWA];
  Cur cc{first_from(0), gw, 0};   // next piece to compute
  Cur ic = cc;                    // next piece to issue
  int staged = 0;                 // phases staged so far
  unroll<D>([&](auto K) {
    issue(ic, wa[K]);
    next(ic);
  });
  bool done = false;
  while (!done) {
    unroll<D>([&](auto K) {
      if (done) return;
      if (cc.p >= a.nph) {
        done = true;
        return;
      }
      while (staged <= cc.p) stage(staged++);
      compute(cc, wa[K]);
      next(cc);
      issue(ic, wa[K]);
      next(ic);
    });
  }
  while (staged < a.nph) stage(staged++);

  // the last workgroup to finish advances the launch sequence for the next launch
  __syncthreads();
  stamp(2 * a.nph + 1);
  if (threadIdx.x == 0) {
    const unsigned done = atomicAdd(&a.ctl[1], 1u);
    if (done == gridDim.x - 1) {
      __hip_atomic_store(&a.ctl[1], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(&a.ctl[0], seq + 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

}  // namespace

int report_error(int code, const char* msg);   // lamm_hip.cpp: sets lamm_hip_last_error()

}  // namespace lamm

using namespace lamm;

struct lamm_chain {
  int type = 0, device = 0, nops = 0, nph = 0, nbmax = 0, grid = 0;
  ChainOp* ops = nullptr;
  ChainPhase* ph = nullptr;
  unsigned* ctl = nullptr;
  uint64_t* gran = nullptr;
  uint64_t* trace = nullptr;   // LAMM_CHAIN_TRACE=1 at create
};

namespace {

int chain_fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));
int chain_fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  return report_error(code, buf);
}

void chain_free(lamm_chain* c) {
  if (!c) return;
  if (c->ops) (void)hipFree(c->ops);
  if (c->ph) (void)hipFree(c->ph);
  if (c->ctl) (void)hipFree(c->ctl);
  if (c->gran) (void)hipFree(c->gran);
  if (c->trace) (void)hipFree(c->trace);
  delete c;
}

size_t chain_lds(const lamm_chain* c) {
  return (size_t)2 * c->nbmax * 40 + (size_t)c->nph * sizeof(ChainPhase) + (size_t)c->nops * sizeof(ChainOp);
}
constexpr size_t kChainLdsMax = 160 * 1024;

int row_bytes(int type) {
  switch (type) {
    case kQ4_0: return 18;
    case kQ4_1: return 20;
    case kQ5_0: return 22;
    case kQ5_1: return 24;
    case kQ8_0: return 34;
    default: return 0;
  }
}

}  // namespace

extern "C" int lamm_hip_chain_create(const lamm_chain_op* ops, int nops, lamm_chain** out) {
  if (!out) return chain_fail(LAMM_ERR_SHAPE, "null output handle");
  *out = nullptr;
  if (!ops || nops < 1) return chain_fail(LAMM_ERR_SHAPE, "empty chain");
  const int type = ops[0].A.type;
  const int bpb = row_bytes(type);
  if (!bpb) return chain_fail(LAMM_ERR_TYPE, "chain weights must be q4_0/q4_1/q5_0/q5_1/q8_0 (got %d)", type);
  // y ranges must not overlap one another, nor any external input
  std::vector<std::pair<uintptr_t, uintptr_t>> ys;
  for (int i = 0; i < nops; ++i) {
    const lamm_chain_op& o = ops[i];
    if (o.A.type != type) return chain_fail(LAMM_ERR_TYPE, "op %d: every op of a chain has one weight type", i);
    if (!o.A.data || !o.x || !o.y || o.A.row < 1 || o.A.col < 1 || o.A.ld < o.A.col)
      return chain_fail(LAMM_ERR_SHAPE, "op %d: bad matrix", i);
    if (o.A.col > kChainIter * 64) return chain_fail(LAMM_ERR_SHAPE, "op %d: K > %d", i, kChainIter * 64 * 32);
    if (((uintptr_t)o.A.data & 15) || (o.A.ld * bpb) % 16)
      return chain_fail(LAMM_ERR_ALIGN, "op %d: weights and their row pitch must be 16-byte aligned", i);
    if (((uintptr_t)o.x & 3) || ((uintptr_t)o.y & 3)) return chain_fail(LAMM_ERR_ALIGN, "op %d: x / y not 4-byte aligned", i);
    ys.push_back({(uintptr_t)o.y, (uintptr_t)o.y + (uintptr_t)o.A.row * 4});
  }
  {
    std::vector<std::pair<uintptr_t, uintptr_t>> s = ys;
    std::sort(s.begin(), s.end());
    for (size_t i = 1; i < s.size(); ++i)
      if (s[i].first < s[i - 1].second) return chain_fail(LAMM_ERR_SHAPE, "outputs of two ops overlap");
  }
  // phases: consecutive ops on the same input whose input no op of the phase produces
  std::vector<ChainOp> hops(nops);
  std::vector<ChainPhase> hph;
  std::vector<int> phase_of(nops, -1);
  std::vector<size_t> goff(nops);
  size_t gtot = 0;
  for (int i = 0; i < nops; ++i) {
    const lamm_chain_op& o = ops[i];
    const int K = o.A.col * 32;
    int src = -1;
    for (int j = i - 1; j >= 0; --j)
      if (ops[j].y == o.x) { src = j; break; }
    if (src >= 0) {
      if (ops[src].A.row != K) return chain_fail(LAMM_ERR_SHAPE, "op %d: input has %d rows, K is %d", i, ops[src].A.row, K);
    } else {
      const uintptr_t x0 = (uintptr_t)o.x, x1 = x0 + (uintptr_t)K * 4;
      for (const auto& y : ys)
        if (x0 < y.second && y.first < x1)
          return chain_fail(LAMM_ERR_SHAPE, "op %d: input overlaps an output without being one", i);
    }
    const bool same = !hph.empty() && ops[hph.back().op0].x == o.x && (src < 0 || phase_of[src] != (int)hph.size() - 1);
    if (!same) {
      if ((int)hph.size() >= kChainMaxPhases) return chain_fail(LAMM_ERR_SHAPE, "more than %d phases", kChainMaxPhases);
      ChainPhase P{};
      P.x = o.x;
      P.op0 = i;
      P.nops = 0;
      P.M = 0;
      P.nblk = o.A.col;
      P.src = src >= 0 ? phase_of[src] : -1;
      P.npc = (o.A.col + kPieceBlocks - 1) / kPieceBlocks;
      P.gx = reinterpret_cast<const uint64_t*>((intptr_t)src);   // producing op, resolved below
      hph.push_back(P);
    }
    ChainPhase& P = hph.back();
    phase_of[i] = (int)hph.size() - 1;
    hops[i].A = static_cast<const unsigned char*>(o.A.data);
    hops[i].y = o.y;
    hops[i].lda = o.A.ld * bpb;
    hops[i].row0 = P.M;
    hops[i].M = o.A.row;
    P.M += o.A.row;
    P.nops += 1;
    goff[i] = gtot;
    gtot += (size_t)o.A.row;
  }
  auto* c = new lamm_chain;
  c->type = type;
  c->nops = nops;
  c->nph = (int)hph.size();
  for (const auto& P : hph) c->nbmax = std::max(c->nbmax, P.nblk);
  if (chain_lds(c) > kChainLdsMax) {
    delete c;
    return chain_fail(LAMM_ERR_SHAPE, "chain tables do not fit in LDS (%d ops, %d phases)", nops, (int)hph.size());
  }
  hipError_t e = hipGetDevice(&c->device);
  int cus = 0;
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
  c->grid = cus > 0 ? cus : 256;
  if (e == hipSuccess) e = hipMalloc(&c->gran, gtot * 8 + 64);
  if (e == hipSuccess) e = hipMemset(c->gran, 0, gtot * 8 + 64);
  for (int i = 0; i < nops; ++i) hops[i].g = c->gran + goff[i];
  for (auto& P : hph) {   // gx held the producing op's index
    const intptr_t src = reinterpret_cast<intptr_t>(P.gx);
    P.gx = src >= 0 ? c->gran + goff[src] : nullptr;
  }
  if (e == hipSuccess) e = hipMalloc(&c->ops, sizeof(ChainOp) * nops);
  if (e == hipSuccess) e = hipMemcpy(c->ops, hops.data(), sizeof(ChainOp) * nops, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMalloc(&c->ph, sizeof(ChainPhase) * hph.size());
  if (e == hipSuccess) e = hipMemcpy(c->ph, hph.data(), sizeof(ChainPhase) * hph.size(), hipMemcpyHostToDevice);
  const unsigned ctl0[4] = {1u, 0u, 0u, 0u};   // sequence starts at 1: a zeroed granule never matches
  if (e == hipSuccess) e = hipMalloc(&c->ctl, 64);
  if (e == hipSuccess) e = hipMemcpy(c->ctl, ctl0, sizeof ctl0, hipMemcpyHostToDevice);
  const char* tr = getenv("LAMM_CHAIN_TRACE");
  if (e == hipSuccess && tr && tr[0] == '1')
    e = hipMalloc(&c->trace, (size_t)c->grid * (2 * c->nph + 2) * sizeof(uint64_t));
  if (e != hipSuccess) {
    chain_free(c);
    return chain_fail(LAMM_ERR_HIP, "chain setup: %s", hipGetErrorString(e));
  }
  *out = c;
  return LAMM_OK;
}

extern "C" int lamm_hip_chain_run(lamm_chain* c, void* stream) {
  if (!c) return chain_fail(LAMM_ERR_SHAPE, "null chain");
  ChainArgs a{c->ops, c->ph, c->ctl, c->nph, c->nbmax, c->nops, 0, c->trace};
  const size_t lds = chain_lds(c);
  const auto s = static_cast<hipStream_t>(stream);
  const dim3 grid(c->grid), block(64 * kChainWaves);
  auto go = [&](auto kern) {
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(kern, grid, block, lds, s, a);
  };
  switch (c->type) {
    case kQ4_0: go(gemv_chain_kernel<kQ4_0, kChainWaves>); break;
    case kQ4_1: go(gemv_chain_kernel<kQ4_1, kChainWaves>); break;
    case kQ5_0: go(gemv_chain_kernel<kQ5_0, kChainWaves>); break;
    case kQ5_1: go(gemv_chain_kernel<kQ5_1, kChainWaves>); break;
    case kQ8_0: go(gemv_chain_kernel<kQ8_0, kChainWaves>); break;
    default: return chain_fail(LAMM_ERR_TYPE, "chain type %d", c->type);
  }
  const hipError_t e = hipGetLastError();
  return e == hipSuccess ? LAMM_OK : chain_fail(LAMM_ERR_HIP, "chain launch: %s", hipGetErrorString(e));
}

extern "C" int lamm_hip_chain_status(lamm_chain* c) {
  if (!c) return chain_fail(LAMM_ERR_SHAPE, "null chain");
  unsigned err = 0;
  hipError_t e = hipMemcpy(&err, c->ctl + 2, 4, hipMemcpyDeviceToHost);
  if (e == hipSuccess && err) e = hipMemset(c->ctl + 2, 0, 4);
  if (e != hipSuccess) return chain_fail(LAMM_ERR_HIP, "chain status: %s", hipGetErrorString(e));
  if (err) return chain_fail(LAMM_ERR_HIP, "a chain launch gave up waiting for a phase input (results invalid)");
  return LAMM_OK;
}

extern "C" int lamm_hip_chain_phases(const lamm_chain* c) { return c ? c->nph : 0; }

extern "C" size_t lamm_hip_chain_trace(const lamm_chain* c, uint64_t* out, size_t n) {
  if (!c || !c->trace) return 0;
  const size_t all = (size_t)c->grid * (2 * c->nph + 2);
  if (out && n >= all && hipMemcpy(out, c->trace, all * sizeof(uint64_t), hipMemcpyDeviceToHost) != hipSuccess) return 0;
  return all;
}

extern "C" void lamm_hip_chain_destroy(lamm_chain* c) { chain_free(c); }
