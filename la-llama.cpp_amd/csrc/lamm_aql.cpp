// lamm_aql.cpp -- the library's own AQL queue: direct dispatch of the one-kernel decode GEMVs.
//
// A decode-sized call is one kernel of a few microseconds, and HIP's launch path costs about as
// much on the host (hipLaunchKernel ~3 us per call through llama.cpp, a graph replay ~22 us of
// start-up) plus a signal launch for completion.  Here the library writes the
// AQL kernel-dispatch packet itself into a user-mode queue of its own on the same GPU agent and
// rings the doorbell; the command processor decrements a completion signal when the kernel is
// done (after its system-scope release, so C in host memory is visible), and the host spins on it.
//
// The kernels are the library's own, as HIP loaded them: the code object is found through ROCr's
// loader extension (every executable the process loaded), the kernel by its name
// (hipKernelNameRefByPtr), and its kernarg layout is checked against the code object v5 rule the
// compiler follows -- explicit arguments, then the 256-byte implicit block at the next 8-byte
// boundary (block counts, group sizes, remainders, grid dims, dynamic LDS size), which is filled
// here as HIP fills it.  Anything that does not check out (no ROCr entry, name not found, another
// kernarg size) leaves the call on HIP's launch path: direct_launch returns false.
//
// Kernarg blocks are content-addressed (round 6): a block whose bytes were written before (the same
// kernel, arguments and grid: a decode step's call on the same weight, every step of a benchmark that
// rotates over a fixed set of weights) is dispatched from its cached slot -- immutable once written,
// so any packet may point at it at any time -- with no BAR writes and no HDP flush + read-back (two
// PCIe round trips that set the host's cost per dispatch).  Blocks the cache cannot hold go through
// the ring of reusable slots as before.
//
// Every reason the queue or a kernel is unusable is recorded (Aql::why, direct_reason()): round 5's
// driver box dispatched nothing directly and said nothing about why.  Several GPU agents can share
// one PCI function's address (a partitioned device); the queue is created on the agent the library's
// kernels were loaded for, found when the first kernel is looked up.
//
// Ordering: the queue is a second queue beside the HIP stream.  A direct region (lamm_hip_direct_
// begin / end, or the boundary's decode call) must not mix with work on the HIP stream: callers
// drain the stream before it (cold weight uploads) and the region ends with every packet complete.
#include <hip/hip_runtime.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <hsa/hsa_ven_amd_loader.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "lamm_aql.h"
#include "lamm_knobs.h"

namespace lamm {
namespace {

constexpr uint32_t kQueueSize = 256;       // packets
constexpr uint32_t kSlots = 2 * kQueueSize;  // kernarg slots (a slot is reused only once its packet completed)
constexpr uint32_t kSlotBytes = 1024;
constexpr uint32_t kImplicitBytes = 256;   // code object v5 implicit kernarg block
constexpr uint32_t kCached = 512;          // content-addressed kernarg slots (never rewritten)

struct AqlKernel {
  uint64_t object = 0;
  uint32_t kernarg = 0, group = 0, priv = 0;
  bool ok = false;
};

void queue_error(hsa_status_t st, hsa_queue_t*, void*) {
  const char* msg = nullptr;
  hsa_status_string(st, &msg);
  fprintf(stderr, "lamm_hip: direct-dispatch queue error: %s\n", msg ? msg : "?");
  std::abort();
}

class Aql {
 public:
  bool init(int device) {
    if (hsa_init() != HSA_STATUS_SUCCESS) return no("hsa_init failed");
    hsa_inited_ = true;
    int bus = -1, dev = -1, dom = -1;
    if (hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) != hipSuccess ||
        hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) != hipSuccess)
      return no("HIP reports no PCI address for the device");
    want_bdf_ = (uint32_t)((bus << 8) | (dev << 3));
    want_dom_ = (uint32_t)dom;
    hsa_iterate_agents(
        [](hsa_agent_t a, void* d) {
          Aql* self = static_cast<Aql*>(d);
          hsa_device_type_t t;
          hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
          if (t == HSA_DEVICE_TYPE_CPU && !self->cpu_.handle) self->cpu_ = a;
          if (t == HSA_DEVICE_TYPE_GPU) {
            uint32_t bdf = 0, dom = 0;
            hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
            hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
            if ((bdf & ~7u) == self->want_bdf_ && dom == self->want_dom_) self->cands_.push_back(a);
          }
          return HSA_STATUS_SUCCESS;
        },
        this);
    if (cands_.empty()) {
      char b[96];
      snprintf(b, sizeof b, "no HSA GPU agent at PCI %04x:%02x:%02x", want_dom_, (unsigned)bus, (unsigned)dev);
      return no(b);
    }
    if (!cpu_.handle) return no("no HSA CPU agent");
    // kernarg memory: the host pool that carries the kernarg flag
    hsa_amd_agent_iterate_memory_pools(
        cpu_,
        [](hsa_amd_memory_pool_t p, void* d) {
          hsa_amd_segment_t seg;
          hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
          if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
          uint32_t fl = 0;
          hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
          if (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT) *static_cast<hsa_amd_memory_pool_t*>(d) = p;
          return HSA_STATUS_SUCCESS;
        },
        &karg_pool_);
    if (!karg_pool_.handle) return no("no host kernarg memory pool");
    if (hsa_system_get_major_extension_table(HSA_EXTENSION_AMD_LOADER, 1, sizeof(loader_), &loader_) !=
        HSA_STATUS_SUCCESS)
      return no("no ROCr loader extension");
    return true;
  }

  // the queue, its kernarg memory and completion signal on agent `gpu` (the agent the first kernel
  // looked up was loaded for)
  bool create_queue(hsa_agent_t gpu) {
    gpu_ = gpu;
    // The kernarg ring in the GPU's fine-grained memory, written by the host through the BAR and
    // made visible by an HDP flush + read-back before the doorbell (as HIP does for its device
    // kernargs): the kernels' scalar loads of their arguments stay on the device.  With the ring in
    // host memory each of them crossed PCIe -- through llama.cpp's decode a boundary call took
    // 47-50 us instead of 22-23 (profiles/r05/direct/).  LAMM_AQL_HOSTKARG=1: the host ring (A/B).
    hsa_agent_get_info(gpu_, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &hdp_);
    if (!knobs().aql_host_karg && hdp_.HDP_MEM_FLUSH_CNTL) {
      hsa_amd_memory_pool_t vp{0};
      hsa_amd_agent_iterate_memory_pools(
          gpu_,
          [](hsa_amd_memory_pool_t p, void* d) {
            hsa_amd_segment_t seg;
            hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
            if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
            uint32_t fl = 0;
            hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &fl);
            if (fl & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_FINE_GRAINED) *static_cast<hsa_amd_memory_pool_t*>(d) = p;
            return HSA_STATUS_SUCCESS;
          },
          &vp);
      if (vp.handle) {
        karg_pool_ = vp;
        dev_karg_ = true;
      }
    }
    void* k = nullptr;
    const size_t bytes = (size_t)(kSlots + kCached) * kSlotBytes;
    if (hsa_amd_memory_pool_allocate(karg_pool_, bytes, 0, &k) != HSA_STATUS_SUCCESS)
      return no(dev_karg_ ? "kernarg allocation in device fine-grained memory failed" : "kernarg allocation failed");
    karg_ = static_cast<unsigned char*>(k);
    const hsa_agent_t both[2] = {gpu_, cpu_};
    if (hsa_amd_agents_allow_access(2, both, nullptr, karg_) != HSA_STATUS_SUCCESS) return no("kernarg access grant failed");
    memset(karg_, 0, bytes);
    if (hsa_queue_create(gpu_, kQueueSize, HSA_QUEUE_TYPE_SINGLE, queue_error, nullptr, UINT32_MAX, UINT32_MAX, &q_) !=
        HSA_STATUS_SUCCESS)
      return no("hsa_queue_create failed");
    // a busy-wait completion signal (no interrupt behind each completion: the host spins anyway)
    if (hsa_amd_signal_create(0, 0, nullptr, HSA_AMD_SIGNAL_AMD_GPU_ONLY, &done_) != HSA_STATUS_SUCCESS)
      return no("completion signal creation failed");
    return true;
  }

  const AqlKernel& kernel(const void* fn, size_t explicit_bytes) {
    auto it = cache_.find(fn);
    if (it != cache_.end()) return it->second;
    AqlKernel k;
    hipFuncAttributes fa;
    const char* name = hipFuncGetAttributes(&fa, fn) == hipSuccess ? hipKernelNameRefByPtr(fn, nullptr) : nullptr;
    hsa_agent_t found{0};
    if (!name) {
      no("HIP gives no name for a kernel");
    } else {
      struct Find {
        Aql* self;
        std::string name;
        AqlKernel* k;
        hsa_agent_t* found;
      } f{this, name, &k, &found};
      loader_.hsa_ven_amd_loader_iterate_executables(
          [](hsa_executable_t ex, void* d) {
            Find* f = static_cast<Find*>(d);
            if (f->k->object) return HSA_STATUS_SUCCESS;
            // the queue's agent once there is one, else every agent at the device's PCI address
            std::vector<hsa_agent_t> agents = f->self->q_ ? std::vector<hsa_agent_t>{f->self->gpu_} : f->self->cands_;
            for (hsa_agent_t a : agents)
              for (const std::string& n : {f->name, f->name + ".kd"}) {
                hsa_executable_symbol_t sym;
                if (hsa_executable_get_symbol_by_name(ex, n.c_str(), &a, &sym) != HSA_STATUS_SUCCESS) continue;
                hsa_symbol_kind_t kind;
                hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_TYPE, &kind);
                if (kind != HSA_SYMBOL_KIND_KERNEL) continue;
                hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &f->k->object);
                hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &f->k->kernarg);
                hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &f->k->group);
                hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &f->k->priv);
                *f->found = a;
                return HSA_STATUS_SUCCESS;
              }
            return HSA_STATUS_SUCCESS;
          },
          &f);
      // the code object v5 layout this file fills: explicit args, then the implicit block at the next
      // 8-byte boundary; any other size (an older code object, a kernel whose hidden args differ)
      // stays on HIP's launch path
      const size_t want = ((explicit_bytes + 7) & ~size_t(7)) + kImplicitBytes;
      char b[256];
      if (!k.object) {
        snprintf(b, sizeof b, "kernel %.120s not found in any loaded executable for the device's %zu agent(s)", name,
                 cands_.size());
        no(b);
      } else if (k.priv) {
        snprintf(b, sizeof b, "kernel %.120s needs %u B of scratch", name, k.priv);
        no(b);
      } else if (k.kernarg != want || k.kernarg > kSlotBytes) {
        snprintf(b, sizeof b, "kernel %.120s: kernarg segment %u B, expected %zu", name, k.kernarg, want);
        no(b);
      } else if (!q_ && !create_queue(found)) {
        // (create_queue recorded why)
      } else {
        k.ok = true;
      }
    }
    return cache_.emplace(fn, k).first->second;
  }

  // Round 6 (default, eager_): every packet is published as soon as it is written, the region's
  // first with a system-scope acquire, all with agent-scope releases, and the region ends with a
  // barrier packet carrying the completion signal and the system-scope release -- the first kernel
  // no longer waits for the second call.  Round 5 (LAMM_AQL_EAGER=0):
  // a packet is written at once but published (header + doorbell) only when the next one arrives or
  // the region ends, so the last packet of a region is known when it is published: only it carries
  // the completion signal and a system-scope release; the first carries a system-scope acquire
  // (inputs the host wrote), the others agent scope on both sides (probe, profiles/r05/direct/:
  // system fences and a signal on every packet cost 1.5-3 us per kernel back to back).
  bool dispatch(const AqlKernel& k, dim3 g, dim3 b, uint32_t dyn_lds, const void* args, size_t bytes) {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q_, 1);
    // queue space (and with it the ring's kernarg slot: packets run in order behind their barrier
    // bits, so packet idx - kSlots completed before packet idx - kSlots + 1 was launched)
    const auto t0 = std::chrono::steady_clock::now();
    while (idx - hsa_queue_load_read_index_scacquire(q_) >= kQueueSize) {
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(2)) {
        fprintf(stderr, "lamm_hip: direct-dispatch queue full for 2 s\n");
        std::abort();
      }
      __builtin_ia32_pause();
    }
    // the whole kernarg block, explicit arguments + implicit block, built on the host first
    const size_t ibase = (bytes + 7) & ~size_t(7), total = ibase + kImplicitBytes;
    unsigned char blk[kSlotBytes];
    memset(blk, 0, total);
    memcpy(blk, args, bytes);
    unsigned char* im = blk + ibase;
    const uint32_t bc[3] = {g.x, g.y, g.z};
    const uint16_t gs[3] = {(uint16_t)b.x, (uint16_t)b.y, (uint16_t)b.z};
    memcpy(im + 0, bc, 12);    // hidden_block_count_x/y/z
    memcpy(im + 12, gs, 6);    // hidden_group_size_x/y/z (remainders 0: whole workgroups)
    const uint16_t dims = g.z > 1 ? 3 : g.y > 1 ? 2 : 1;
    memcpy(im + 64, &dims, 2);       // hidden_grid_dims
    memcpy(im + 120, &dyn_lds, 4);   // hidden_dynamic_lds_size
    // a block written before: its cached slot; a new one: a fresh cached slot while there are any,
    // else the ring
    std::string key(reinterpret_cast<const char*>(blk), total);
    key.append(reinterpret_cast<const char*>(&k.object), sizeof k.object);
    unsigned char* ka;
    bool written = false;
    auto hit = slots_.find(key);
    if (hit != slots_.end()) {
      ka = karg_ + (size_t)(kSlots + hit->second) * kSlotBytes;
      ++hits_;
    } else {
      if (slots_.size() < kCached) {
        const uint32_t c = (uint32_t)slots_.size();
        slots_.emplace(std::move(key), c);
        ka = karg_ + (size_t)(kSlots + c) * kSlotBytes;
      } else {
        ka = karg_ + (idx % kSlots) * kSlotBytes;
      }
      memcpy(ka, blk, total);
      written = true;
    }
    hsa_kernel_dispatch_packet_t* p = packet(idx);
    p->workgroup_size_x = (uint16_t)b.x;
    p->workgroup_size_y = (uint16_t)b.y;
    p->workgroup_size_z = (uint16_t)b.z;
    p->reserved0 = 0;
    p->grid_size_x = g.x * b.x;
    p->grid_size_y = g.y * b.y;
    p->grid_size_z = g.z * b.z;
    p->private_segment_size = k.priv;
    p->group_segment_size = k.group + dyn_lds;
    p->kernel_object = k.object;
    p->kernarg_address = ka;
    p->reserved2 = 0;
    if (dev_karg_ && written) {   // the BAR writes above reach device memory before the packet can be read
      *hdp_.HDP_MEM_FLUSH_CNTL = 1u;
      (void)*reinterpret_cast<volatile uint32_t*>(hdp_.HDP_MEM_FLUSH_CNTL);
      (void)*reinterpret_cast<volatile uint32_t*>(ka + ibase + 120);
    }
    if (pending_) publish(false);
    pending_ = true;
    pend_idx_ = idx;
    pend_setup_ = (uint16_t)(dims << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS);
    pend_first_ = first_;
    first_ = false;
    if (eager_) {   // published at once; the region's end adds a barrier packet for completion
      publish(false);
      dispatched_ = true;
    }
    return true;
  }

  // every packet dispatched so far has completed; false after `seconds` without that.  The next
  // packet opens a new region (system-scope acquire).
  bool wait(double seconds) {
    if (pending_) publish(true);
    if (dispatched_) {   // eager packets: a barrier-AND packet behind them carries the completion
      barrier_packet();
      dispatched_ = false;
    }
    first_ = true;
    const auto t0 = std::chrono::steady_clock::now();
    for (unsigned it = 0;; ++it) {
      if (hsa_signal_load_scacquire(done_) == 0) return true;
      if ((it & 1023) == 1023 &&
          std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > seconds)
        return false;
      __builtin_ia32_pause();
    }
  }

  std::mutex mu;
  std::string why;        // the first reason this queue (or a kernel on it) cannot dispatch
  uint64_t hits_ = 0;     // dispatches from a cached kernarg slot

 private:
  bool no(const char* reason) {
    if (why.empty()) why = reason;
    return false;
  }
  hsa_kernel_dispatch_packet_t* packet(uint64_t idx) {
    return static_cast<hsa_kernel_dispatch_packet_t*>(q_->base_address) + (idx % kQueueSize);
  }
  void publish(bool last) {
    hsa_kernel_dispatch_packet_t* p = packet(pend_idx_);
    if (last) hsa_signal_add_relaxed(done_, 1);
    p->completion_signal = last ? done_ : hsa_signal_t{0};
    const uint32_t inner = knobs().aql_fence_none ? HSA_FENCE_SCOPE_NONE : HSA_FENCE_SCOPE_AGENT;
    const uint32_t acq = pend_first_ ? HSA_FENCE_SCOPE_SYSTEM : inner;
    const uint32_t rel = last ? HSA_FENCE_SCOPE_SYSTEM : inner;
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                                       (1u << HSA_PACKET_HEADER_BARRIER) | (acq << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (rel << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    __atomic_store_n(reinterpret_cast<uint32_t*>(p), (uint32_t)header | ((uint32_t)pend_setup_ << 16), __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q_->doorbell_signal, (hsa_signal_value_t)pend_idx_);
    pending_ = false;
  }

  // a barrier-AND packet (no dependencies) behind the region's kernels: it completes once they have
  // (barrier bit), then its system-scope release makes their stores visible to the host and it
  // decrements the completion signal
  void barrier_packet() {
    const uint64_t idx = hsa_queue_add_write_index_relaxed(q_, 1);
    while (idx - hsa_queue_load_read_index_scacquire(q_) >= kQueueSize) __builtin_ia32_pause();
    hsa_barrier_and_packet_t* p = reinterpret_cast<hsa_barrier_and_packet_t*>(packet(idx));
    p->reserved0 = 0;
    p->reserved1 = 0;
    for (auto& d : p->dep_signal) d = hsa_signal_t{0};
    p->reserved2 = 0;
    hsa_signal_add_relaxed(done_, 1);
    p->completion_signal = done_;
    const uint16_t header = (uint16_t)((HSA_PACKET_TYPE_BARRIER_AND << HSA_PACKET_HEADER_TYPE) |
                                       (1u << HSA_PACKET_HEADER_BARRIER) |
                                       (HSA_FENCE_SCOPE_NONE << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                                       (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE));
    __atomic_store_n(reinterpret_cast<uint32_t*>(p), (uint32_t)header, __ATOMIC_RELEASE);
    hsa_signal_store_screlease(q_->doorbell_signal, (hsa_signal_value_t)idx);
  }

  // LAMM_AQL_EAGER (default 1): publish every kernel packet as it is written (agent-scope release) and
  // close the region with a barrier packet; 0: hold each packet until the next arrives (round 5)
  const bool eager_ = knobs().aql_eager;
  bool dispatched_ = false;
  bool hsa_inited_ = false, dev_karg_ = false;
  hsa_amd_hdp_flush_t hdp_{};
  bool pending_ = false, pend_first_ = false, first_ = true;
  uint64_t pend_idx_ = 0;
  uint16_t pend_setup_ = 0;
  uint32_t want_bdf_ = 0, want_dom_ = 0;
  hsa_agent_t gpu_{0}, cpu_{0};
  std::vector<hsa_agent_t> cands_;   // GPU agents at the device's PCI address
  hsa_amd_memory_pool_t karg_pool_{0};
  unsigned char* karg_ = nullptr;
  hsa_queue_t* q_ = nullptr;
  hsa_signal_t done_{0};
  hsa_ven_amd_loader_1_03_pfn_t loader_{};
  std::unordered_map<const void*, AqlKernel> cache_;
  std::unordered_map<std::string, uint32_t> slots_;   // kernarg block bytes -> cached slot
};

std::mutex g_mu;
std::unordered_map<int, Aql*> g_queues;   // per HIP device; nullptr: unavailable
std::unordered_map<int, std::string> g_unavailable;   // why a device has no queue

thread_local Aql* t_direct = nullptr;
thread_local int t_launches = 0, t_fallbacks = 0;
thread_local std::string t_reason;

Aql* queue_for(int device) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_queues.find(device);
  if (it != g_queues.end()) return it->second;
  Aql* q = new Aql();
  if (!q->init(device)) {
    g_unavailable[device] = q->why;
    delete q;   // (init creates no queue: nothing to tear down)
    q = nullptr;
  }
  g_queues[device] = q;
  return q;
}

// HIP device -> its HSA GPU agent (PCI bus / device / domain) and the HDP flush register ROCr maps
struct HdpEntry {
  uint32_t* reg = nullptr;
  bool host_access = false;   // the host can store into the agent's local memory (large BAR)
};
std::unordered_map<int, HdpEntry> g_hdp;

uint32_t* hdp_register(int device) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_hdp.find(device);
  if (it != g_hdp.end()) return it->second.reg;
  HdpEntry e;
  int bus = -1, dev = -1, dom = -1;
  if (hsa_init() == HSA_STATUS_SUCCESS && hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, device) == hipSuccess &&
      hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, device) == hipSuccess &&
      hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainID, device) == hipSuccess) {
    struct Want {
      uint32_t bdf, dom;
      hsa_agent_t gpu;
    } w{(uint32_t)((bus << 8) | (dev << 3)), (uint32_t)dom, {0}};
    hsa_iterate_agents(
        [](hsa_agent_t a, void* d) {
          Want* w = static_cast<Want*>(d);
          hsa_device_type_t t;
          hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
          if (t != HSA_DEVICE_TYPE_GPU) return HSA_STATUS_SUCCESS;
          uint32_t bdf = 0, dom = 0;
          hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
          hsa_agent_get_info(a, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
          if ((bdf & ~7u) == w->bdf && dom == w->dom) w->gpu = a;
          return HSA_STATUS_SUCCESS;
        },
        &w);
    hsa_amd_hdp_flush_t h{};
    if (w.gpu.handle && hsa_agent_get_info(w.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_HDP_FLUSH, &h) == HSA_STATUS_SUCCESS)
      e.reg = h.HDP_MEM_FLUSH_CNTL;
    bool direct = false;
    if (w.gpu.handle &&
        hsa_agent_get_info(w.gpu, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_SVM_DIRECT_HOST_ACCESS, &direct) == HSA_STATUS_SUCCESS)
      e.host_access = direct;
  }
  g_hdp[device] = e;
  return e.reg;
}

}  // namespace

bool hdp_flush_available(int device) { return hdp_register(device) != nullptr; }

bool vram_host_writable(int device) {
  if (!hdp_register(device)) return false;
  std::lock_guard<std::mutex> lock(g_mu);
  return g_hdp[device].host_access;
}

void hdp_flush(int device, const void* last_written) {
  uint32_t* r = hdp_register(device);
  if (r) {
    *r = 1u;
    (void)*reinterpret_cast<volatile uint32_t*>(r);
  }
  if (last_written) (void)*reinterpret_cast<const volatile uint32_t*>(last_written);
}

bool direct_begin(int device) {
  t_reason.clear();
  if (t_direct) {
    t_reason = "a direct region is already open on this thread";
    return false;
  }
  Aql* q = queue_for(device);
  if (!q) {
    std::lock_guard<std::mutex> lock(g_mu);
    t_reason = g_unavailable[device];
    return false;
  }
  q->mu.lock();
  t_direct = q;
  t_launches = t_fallbacks = 0;
  return true;
}

int direct_end(double seconds) {
  Aql* q = t_direct;
  if (!q) return -1;
  t_direct = nullptr;
  const bool ok = t_launches == 0 || q->wait(seconds);
  q->mu.unlock();
  if (!ok) {
    fprintf(stderr, "lamm_hip: direct-dispatch kernels not complete after %.1f s\n", seconds);
    std::abort();
  }
  return t_launches;
}

bool direct_active() { return t_direct != nullptr; }

int direct_fallbacks() { return t_fallbacks; }

int direct_launches() { return t_launches; }

void direct_note(const std::string& why) {
  ++t_fallbacks;
  if (t_reason.empty()) t_reason = why;
}

const std::string& direct_reason() { return t_reason; }

uint64_t direct_cache_hits(int device) {
  std::lock_guard<std::mutex> lock(g_mu);
  auto it = g_queues.find(device);
  return it != g_queues.end() && it->second ? it->second->hits_ : 0;
}

bool direct_launch(const void* fn, dim3 grid, dim3 block, uint32_t dyn_lds, const void* args, size_t bytes) {
  Aql* q = t_direct;
  if (!q) return false;
  const AqlKernel& k = q->kernel(fn, bytes);
  if (!k.ok) {
    ++t_fallbacks;
    t_reason = q->why;
    return false;
  }
  q->dispatch(k, grid, block, dyn_lds, args, bytes);
  ++t_launches;
  return true;
}

}  // namespace lamm
