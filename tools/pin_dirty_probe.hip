// pin_dirty_probe.hip -- does a host buffer that CPU threads have just written (its lines dirty
// in their caches) upload more slowly than one that sits in memory?  H2D of 2.2 MiB (q8_0 rows of
// a 512 x 4096 prefill) and 8 MiB (its F32 rows) from pinned and pageable memory, after: nothing
// ("idle"), a 16-thread rewrite ("dirty"), a 16-thread rewrite + clflushopt of every line
// ("flushed"), a 16-thread rewrite with non-temporal stores ("streamed").  Median of 15, us
// (only the copy + synchronise is timed).
#include <hip/hip_runtime.h>
#include <immintrin.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e = (x);                                                                            \
    if (e != hipSuccess) {                                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                       \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

__attribute__((target("avx2,clflushopt"))) static void touch(unsigned char* p, size_t n, int mode, int seed) {
  if (mode == 3) {
    const __m256i v = _mm256_set1_epi8((char)seed);
    for (size_t i = 0; i + 32 <= n; i += 32) _mm256_stream_si256((__m256i*)(p + i), v);
    _mm_sfence();
    return;
  }
  for (size_t i = 0; i < n; i += 8) *(volatile uint64_t*)(p + i) = seed + i;
  if (mode == 2) {
    for (size_t i = 0; i < n; i += 64) _mm_clflushopt(p + i);
    _mm_sfence();
  }
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t sizes[] = {(size_t)2228224, (size_t)8 << 20};
  const char* modes[] = {"idle", "dirty", "flushed", "streamed"};
  const int T = 16;
  printf("{");
  bool first = true;
  for (size_t n : sizes) {
    void* d;
    CK(hipMalloc(&d, n));
    unsigned char* pin;
    CK(hipHostMalloc((void**)&pin, n, hipHostMallocPortable));
    unsigned char* page = (unsigned char*)aligned_alloc(4096, n);
    for (int pinned = 1; pinned >= 0; --pinned) {
      unsigned char* h = pinned ? pin : page;
      for (int m = 0; m < 4; ++m) {
        std::vector<double> t;
        for (int r = 0; r < 18; ++r) {
          if (m > 0) {
            std::vector<std::thread> th;
            const size_t per = (n / T + 63) & ~size_t(63);
            for (int i = 0; i < T; ++i) {
              const size_t a = i * per, b = std::min(n, a + per);
              if (a < b) th.emplace_back(touch, h + a, b - a, m, r);
            }
            for (auto& x : th) x.join();
          }
          const auto t0 = std::chrono::steady_clock::now();
          CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
          CK(hipStreamSynchronize(s));
          if (r >= 3) t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(t.begin(), t.end());
        printf("%s\"h2d_%zuK_%s_%s\": %.1f", first ? "" : ", ", n >> 10, pinned ? "pinned" : "pageable", modes[m], t[t.size() / 2]);
        first = false;
        fflush(stdout);
      }
    }
    free(page);
    CK(hipHostFree(pin));
    CK(hipFree(d));
  }
  printf("}\n");
  return 0;
}
