// lamm_aql.h -- direct dispatch on the library's own AQL queue (lamm_aql.cpp)
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <string>

namespace lamm {

// Open a direct region on this thread for HIP device `device` (false: no queue, or one is open).
bool direct_begin(int device);
// Close it: wait until every kernel dispatched in it completed (abort after `seconds`); returns
// the number of direct launches the region made (0: everything went through HIP).
int direct_end(double seconds = 1.0);
bool direct_active();
// calls of the open (or last) region that fell back to HIP, and why the last fallback, or the last
// direct_begin, could not use the queue
int direct_fallbacks();
// direct launches so far in the open region; a call made in the region whose kernel did not go onto
// the queue for a reason of the caller's (another engine, a pending profiling request) notes why
int direct_launches();
void direct_note(const std::string& why);
const std::string& direct_reason();
// dispatches that found their kernarg block already in a cached slot (this device's queue)
uint64_t direct_cache_hits(int device);
// Dispatch kernel `fn` (its host stub) with explicit arguments [args, args + bytes) when a region
// is open and the kernel's layout checks out; false: the caller launches through HIP.
bool direct_launch(const void* fn, dim3 grid, dim3 block, uint32_t dyn_lds, const void* args, size_t bytes);

// Host writes into device memory through the BAR reach it only through the HDP: flush it (ROCr's
// mapped flush register) and read `last_written` back, so a kernel launched next sees the bytes.
bool hdp_flush_available(int device);
// the host can store straight into this device's memory (large BAR) and flush the HDP after it
bool vram_host_writable(int device);
void hdp_flush(int device, const void* last_written);

}  // namespace lamm
