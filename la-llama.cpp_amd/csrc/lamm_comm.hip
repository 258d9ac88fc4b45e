// lamm_comm.hip -- multi-GPU row sharding of the lamm operator.
//
// Output rows are independent (src/lamm_impl.hpp:50-53: C[i,:] needs only row i of A and all
// of B), and the reference already splits rows over threads (job_size = M / nth,
// src/lamm_impl.hpp:38-43, :107-112 -- dropping the M % nth tail rows, SURVEY §8a defect 1).
// Here the ranks of a communicator own contiguous slabs of A's rows (lamm_hip_shard_rows: every
// row exactly once, slab boundaries on the kernels' row tile), each rank computes its slab of C
// with the single-GPU kernels, and one all-gather over RCCL (xGMI) gives every rank the whole C:
//
//   pack   : slab [N][rows_r] -> the rank's segment of a [world][N][maxrows] gather buffer
//            (skipped when N == 1 and the slabs are equal: C itself is the gather buffer)
//   gather : ncclAllGather (in place)
//   unpack : one kernel scatters [world][N][maxrows] into C[N][M] (ldc)
//
// RCCL is loaded with dlopen at the first communicator (a process that already holds it --
// PyTorch's copy -- shares that one; liblamm_hip.so itself has no link-time dependency on it).
// Ranks that share ONE device (a rehearsal on a one-GPU box; RCCL refuses duplicate devices)
// run in loopback mode: the same pack / unpack kernels, the exchange done by device copies whose
// ordering is expressed with events only (no host synchronisation), so a loopback all-gather
// can be captured into a hipGraph like the RCCL one.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/lamm_hip.h"

namespace {

struct Rccl {
  bool ok = false;
  std::string err;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

const Rccl& rccl() {
  static Rccl r = [] {
    Rccl x;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("librccl.so", RTLD_NOW | RTLD_GLOBAL);
    if (!h) {
      x.err = std::string("dlopen librccl: ") + dlerror();
      return x;
    }
    auto sym = [&](auto& fn, const char* name) {
      fn = reinterpret_cast<std::remove_reference_t<decltype(fn)>>(dlsym(h, name));
      return fn != nullptr;
    };
    x.ok = sym(x.GetUniqueId, "ncclGetUniqueId") && sym(x.CommInitRank, "ncclCommInitRank") &&
           sym(x.CommInitAll, "ncclCommInitAll") && sym(x.CommDestroy, "ncclCommDestroy") &&
           sym(x.AllGather, "ncclAllGather") && sym(x.GroupStart, "ncclGroupStart") &&
           sym(x.GroupEnd, "ncclGroupEnd") && sym(x.GetErrorString, "ncclGetErrorString");
    if (!x.ok) x.err = "librccl lacks an nccl* entry point";
    return x;
  }();
  return r;
}

thread_local std::string g_comm_err;
int cfail(int code, const std::string& msg) {
  g_comm_err = msg;
  return code;
}

// Rows [r0, r0 + rows) of rank `rank`: whole `align`-row tiles, the tile remainder spread over
// the first ranks, the ragged tail (M % align) on the rank holding the last tile.
__host__ __device__ inline void shard_rows(int64_t M, int world, int rank, int align, int64_t* r0, int64_t* rows) {
  if (align < 1) align = 1;
  const int64_t tiles = (M + align - 1) / align;
  const int64_t base = tiles / world, extra = tiles % world;
  const int64_t t0 = rank * base + (rank < extra ? rank : extra);
  const int64_t nt = base + (rank < extra ? 1 : 0);
  int64_t a = t0 * align, b = (t0 + nt) * align;
  if (a > M) a = M;
  if (b > M) b = M;
  *r0 = a;
  *rows = b - a;
}

// [world][N][maxrows] -> C[N][M]: rank r's rows land at [r0_r, r0_r + rows_r) of every column
__global__ void unshard_rows_kernel(const float* __restrict__ g, float* __restrict__ C, int64_t ldc, int64_t M,
                                    int N, int world, int align, int64_t maxrows) {
  const int64_t total = (int64_t)world * N * maxrows;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total;
       idx += (int64_t)gridDim.x * blockDim.x) {
    const int64_t k = idx % maxrows;
    const int64_t rj = idx / maxrows;
    const int j = (int)(rj % N), r = (int)(rj / N);
    int64_t r0, rows;
    shard_rows(M, world, r, align, &r0, &rows);
    if (k < rows) C[(int64_t)j * ldc + r0 + k] = g[idx];
  }
}

// Loopback exchange (ranks sharing a device): destination rank `self` copies every other rank's
// segment [k * count, (k + 1) * count) of its gather buffer from that rank's buffer -- one launch
// per rank instead of world - 1 copies (a graph-captured step with G ranks would otherwise hold
// G (G - 1) copy nodes per all-gather: 56 at G = 8, which the HIP runtime's graph code does not
// survive -- tests/test_benchmark_driver.py::test_llama_bench_sharded_decode_bitexact)
constexpr int kLoopbackMax = 64;
struct LoopbackSrcs {
  const float* p[kLoopbackMax];
};
__global__ void loopback_gather_kernel(LoopbackSrcs src, float* __restrict__ dst, int64_t count, int nl, int rank0,
                                       int self) {
  const int64_t per = (int64_t)(nl - 1) * count;
  for (int64_t idx = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; idx < per; idx += (int64_t)gridDim.x * blockDim.x) {
    int k = (int)(idx / count);
    k += k >= self ? 1 : 0;   // skip this rank's own segment
    const int64_t e = (int64_t)(rank0 + k) * count + idx % count;
    dst[e] = src.p[k][e];
  }
}

}  // namespace

struct lamm_comm {
  int world = 1;
  int rank0 = 0;                    // global rank of local index 0
  bool loopback = false;
  std::vector<int> devices;         // per local rank
  std::vector<ncclComm_t> comms;    // per local rank (empty in loopback mode)
  std::vector<float*> gbuf;         // per local rank: [world][N][maxrows] gather buffer
  std::vector<size_t> gcap;
  // loopback: per local rank i >= 1, "my segment is packed" / "my reads of the others are done"
  // (recorded on rank i's stream, waited on by rank 0's); [0]: rank 0's fan-out of each
  std::vector<hipEvent_t> packed, done;
  std::mutex mu;
};

extern "C" void lamm_hip_shard_rows(int64_t M, int world, int rank, int align, int64_t* r0, int64_t* rows) {
  shard_rows(M, world, rank, align, r0, rows);
}

extern "C" const char* lamm_hip_comm_last_error(void) { return g_comm_err.c_str(); }

extern "C" int lamm_hip_comm_unique_id(void* id) {
  const Rccl& r = rccl();
  if (!r.ok) return cfail(LAMM_ERR_HIP, r.err);
  ncclUniqueId u;
  const ncclResult_t e = r.GetUniqueId(&u);
  if (e != ncclSuccess) return cfail(LAMM_ERR_HIP, std::string("ncclGetUniqueId: ") + r.GetErrorString(e));
  memcpy(id, &u, sizeof u);
  return LAMM_OK;
}

extern "C" int lamm_hip_comm_init_rank(lamm_comm** out, int world, int rank, const void* id, int device) {
  *out = nullptr;
  if (world < 1 || rank < 0 || rank >= world) return cfail(LAMM_ERR_SHAPE, "bad world / rank");
  const Rccl& r = rccl();
  if (!r.ok) return cfail(LAMM_ERR_HIP, r.err);
  if (hipSetDevice(device) != hipSuccess) return cfail(LAMM_ERR_NODEV, "hipSetDevice failed");
  auto* c = new lamm_comm;
  c->world = world;
  c->rank0 = rank;
  c->devices = {device};
  c->comms.resize(1);
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  const ncclResult_t e = r.CommInitRank(&c->comms[0], world, u, rank);
  if (e != ncclSuccess) {
    delete c;
    return cfail(LAMM_ERR_HIP, std::string("ncclCommInitRank: ") + r.GetErrorString(e));
  }
  c->gbuf.assign(1, nullptr);
  c->gcap.assign(1, 0);
  *out = c;
  return LAMM_OK;
}

extern "C" int lamm_hip_comm_init_all(lamm_comm** out, int ndev, const int* devices) {
  *out = nullptr;
  if (ndev < 1) return cfail(LAMM_ERR_SHAPE, "ndev < 1");
  auto* c = new lamm_comm;
  c->world = ndev;
  c->devices.assign(devices, devices + ndev);
  std::vector<int> sorted(c->devices);
  std::sort(sorted.begin(), sorted.end());
  c->loopback = std::adjacent_find(sorted.begin(), sorted.end()) != sorted.end();
  if (!c->loopback && ndev > 1) {
    const Rccl& r = rccl();
    if (!r.ok) {
      delete c;
      return cfail(LAMM_ERR_HIP, r.err);
    }
    c->comms.resize(ndev);
    const ncclResult_t e = r.CommInitAll(c->comms.data(), ndev, devices);
    if (e != ncclSuccess) {
      delete c;
      return cfail(LAMM_ERR_HIP, std::string("ncclCommInitAll: ") + r.GetErrorString(e));
    }
  } else {
    c->loopback = true;   // one rank, or ranks sharing a device
  }
  c->gbuf.assign(ndev, nullptr);
  c->gcap.assign(ndev, 0);
  *out = c;
  return LAMM_OK;
}

extern "C" int lamm_hip_comm_size(const lamm_comm* c) { return c ? c->world : 0; }
extern "C" int lamm_hip_comm_local_ranks(const lamm_comm* c) { return c ? (int)c->devices.size() : 0; }
extern "C" int lamm_hip_comm_rank(const lamm_comm* c, int local) { return c ? c->rank0 + local : -1; }

extern "C" void lamm_hip_comm_destroy(lamm_comm* c) {
  if (!c) return;
  for (size_t i = 0; i < c->devices.size(); ++i) {
    (void)hipSetDevice(c->devices[i]);
    (void)hipDeviceSynchronize();
    if (c->gbuf[i]) (void)hipFree(c->gbuf[i]);
    if (i < c->packed.size()) (void)hipEventDestroy(c->packed[i]);
    if (i < c->done.size()) (void)hipEventDestroy(c->done[i]);
  }
  if (!c->comms.empty() && rccl().ok)
    for (ncclComm_t k : c->comms) rccl().CommDestroy(k);
  delete c;
}

extern "C" int lamm_hip_allgather_rows(lamm_comm* c, const float* const* slabs, const int64_t* ld_slab,
                                       float* const* C, int64_t ldc, int64_t M, int N, int align,
                                       void* const* streams) {
  if (!c) return cfail(LAMM_ERR_SHAPE, "null communicator");
  if (M < 0 || N < 1 || ldc < M) return cfail(LAMM_ERR_SHAPE, "bad M / N / ldc");
  std::lock_guard<std::mutex> lock(c->mu);
  const int nl = (int)c->devices.size();
  int64_t r00, maxrows;
  lamm_hip_shard_rows(M, c->world, 0, align, &r00, &maxrows);   // rank 0 holds the most rows
  if (maxrows == 0) return LAMM_OK;
  bool equal = true;
  for (int r = 0; r < c->world; ++r) {
    int64_t a, n;
    lamm_hip_shard_rows(M, c->world, r, align, &a, &n);
    equal = equal && n == maxrows;
  }
  const size_t count = (size_t)N * maxrows;
  const bool direct = N == 1 && equal;   // C is already [world][maxrows]: gather into it
  auto st = [&](int i) { return static_cast<hipStream_t>(streams[i]); };

  // 1. pack each local rank's slab into its segment of the gather buffer (or of C)
  for (int i = 0; i < nl; ++i) {
    if (hipSetDevice(c->devices[i]) != hipSuccess) return cfail(LAMM_ERR_NODEV, "hipSetDevice");
    const int g = c->rank0 + i;
    int64_t r0, rows;
    lamm_hip_shard_rows(M, c->world, g, align, &r0, &rows);
    float* seg;
    if (direct) {
      seg = C[i] + r0;
    } else {
      const size_t need = (size_t)c->world * count;
      if (c->gcap[i] < need) {
        if (c->gbuf[i]) {
          (void)hipStreamSynchronize(st(i));
          (void)hipFree(c->gbuf[i]);
        }
        c->gbuf[i] = nullptr;
        c->gcap[i] = 0;
        if (hipMalloc(&c->gbuf[i], need * sizeof(float)) != hipSuccess) return cfail(LAMM_ERR_HIP, "hipMalloc gather");
        c->gcap[i] = need;
      }
      seg = c->gbuf[i] + (size_t)g * count;
    }
    if (rows > 0 && seg != slabs[i]) {
      const hipError_t e = hipMemcpy2DAsync(seg, (size_t)(direct ? maxrows : maxrows) * sizeof(float), slabs[i],
                                            (size_t)ld_slab[i] * sizeof(float), (size_t)rows * sizeof(float), (size_t)N,
                                            hipMemcpyDeviceToDevice, st(i));
      if (e != hipSuccess) return cfail(LAMM_ERR_HIP, std::string("pack: ") + hipGetErrorString(e));
    }
  }
  // 2. exchange
  if (c->loopback && nl > 1) {
    // events only (graph-capturable): every stream copies the other ranks' segments once they are
    // packed, then every stream waits until all the others have finished reading ITS buffers --
    // the caller's next matmul on stream k overwrites C[k] / gbuf[k] (without that
    // wait a reader of the previous contents could race it)
    if (c->packed.empty()) {
      // created into locals and handed to the communicator only once all exist (a
      // failure half-way used to leave null handles that later calls recorded and destroyed)
      std::vector<hipEvent_t> packed(nl, nullptr), done(nl, nullptr);
      bool made = true;
      for (int i = 0; i < nl && made; ++i) {
        (void)hipSetDevice(c->devices[i]);
        made = hipEventCreateWithFlags(&packed[i], hipEventDisableTiming) == hipSuccess &&
               hipEventCreateWithFlags(&done[i], hipEventDisableTiming) == hipSuccess;
      }
      if (!made) {
        for (int i = 0; i < nl; ++i) {
          if (packed[i]) (void)hipEventDestroy(packed[i]);
          if (done[i]) (void)hipEventDestroy(done[i]);
        }
        return cfail(LAMM_ERR_HIP, "hipEventCreate");
      }
      c->packed.swap(packed);
      c->done.swap(done);
    }
    auto ok = [](hipError_t e) { return e == hipSuccess; };
    // Fan in to local rank 0's stream and back out (2 (nl - 1) waits per phase instead of nl (nl - 1),
    // VERDICT r4 item 7): every event is waited on right after it is recorded, before the stream
    // that recorded it enqueues anything else, so a captured graph never sees an event whose
    // recording stream has moved on (the old all-pairs form, with every stream waiting on every
    // other stream's reused event, sent HIP's graph code into unbounded recursion at 8 ranks).
    auto barrier = [&](std::vector<hipEvent_t>& ev) -> bool {
      for (int i = 1; i < nl; ++i) {
        (void)hipSetDevice(c->devices[i]);
        if (!ok(hipEventRecord(ev[i], st(i)))) return false;
        (void)hipSetDevice(c->devices[0]);
        if (!ok(hipStreamWaitEvent(st(0), ev[i], 0))) return false;
      }
      (void)hipSetDevice(c->devices[0]);
      if (!ok(hipEventRecord(ev[0], st(0)))) return false;
      for (int i = 1; i < nl; ++i) {
        (void)hipSetDevice(c->devices[i]);
        if (!ok(hipStreamWaitEvent(st(i), ev[0], 0))) return false;
      }
      return true;
    };
    if (!barrier(c->packed)) return cfail(LAMM_ERR_HIP, "loopback barrier (packed)");
    // every rank on ONE device (the one-GPU rehearsal): one gather launch per rank; ranks on
    // several devices (some of them shared): device copies, which cross devices
    const bool one_dev = std::all_of(c->devices.begin(), c->devices.end(), [&](int d) { return d == c->devices[0]; });
    LoopbackSrcs srcs{};
    if (one_dev && nl <= kLoopbackMax)
      for (int k = 0; k < nl; ++k) srcs.p[k] = direct ? C[k] : c->gbuf[k];
    for (int i = 0; i < nl; ++i) {
      (void)hipSetDevice(c->devices[i]);
      float* dst = direct ? C[i] : c->gbuf[i];
      if (one_dev && nl <= kLoopbackMax) {
        const int64_t per = (int64_t)(nl - 1) * (int64_t)count;
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((per + 255) / 256, 2048));
        hipLaunchKernelGGL(loopback_gather_kernel, dim3(grid), dim3(256), 0, st(i), srcs, dst, (int64_t)count, nl,
                           c->rank0, i);
        if (!ok(hipGetLastError())) return cfail(LAMM_ERR_HIP, "loopback gather launch");
      } else {
        for (int k = 0; k < nl; ++k) {
          if (k == i) continue;
          const float* src = direct ? C[k] : c->gbuf[k];
          const size_t off = (size_t)(c->rank0 + k) * count;
          if (!ok(hipMemcpyAsync(dst + off, src + off, count * sizeof(float), hipMemcpyDeviceToDevice, st(i))))
            return cfail(LAMM_ERR_HIP, "loopback copy");
        }
      }
    }
    // no stream goes on (and overwrites its own buffers) until every stream has read them
    if (!barrier(c->done)) return cfail(LAMM_ERR_HIP, "loopback barrier (done)");
  } else if (!c->loopback) {
    const Rccl& r = rccl();
    r.GroupStart();
    for (int i = 0; i < nl; ++i) {
      (void)hipSetDevice(c->devices[i]);
      float* buf = direct ? C[i] : c->gbuf[i];
      const ncclResult_t e =
          r.AllGather(buf + (size_t)(c->rank0 + i) * count, buf, count, ncclFloat32, c->comms[i], st(i));
      if (e != ncclSuccess) {
        r.GroupEnd();
        return cfail(LAMM_ERR_HIP, std::string("ncclAllGather: ") + r.GetErrorString(e));
      }
    }
    const ncclResult_t e = r.GroupEnd();
    if (e != ncclSuccess) return cfail(LAMM_ERR_HIP, std::string("ncclGroupEnd: ") + r.GetErrorString(e));
  }
  // 3. unpack into C[N][M]
  if (!direct) {
    for (int i = 0; i < nl; ++i) {
      (void)hipSetDevice(c->devices[i]);
      const int64_t total = (int64_t)c->world * count;
      const int grid = (int)std::min<int64_t>((total + 255) / 256, 4096);
      hipLaunchKernelGGL(unshard_rows_kernel, dim3(grid), dim3(256), 0, st(i), c->gbuf[i], C[i], ldc, M, N, c->world,
                         align, maxrows);
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return cfail(LAMM_ERR_HIP, std::string("unshard: ") + hipGetErrorString(e));
    }
  }
  return LAMM_OK;
}
