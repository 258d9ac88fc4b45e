// pin_flags_probe.hip -- H2D / D2H of a prefill upload (2.2 MiB of q8_0 rows, 8 MiB of F32) from
// pinned host buffers allocated with the flags the boundary uses: mapped + non-coherent (its
// zero-copy activation buffer), mapped coherent (its zero-copy C), plain portable; and pageable.
// Median of 20 hipMemcpyAsync + hipStreamSynchronize, us.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                      \
  do {                                                                                             \
    hipError_t e = (x);                                                                            \
    if (e != hipSuccess) {                                                                         \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                                       \
      exit(1);                                                                                     \
    }                                                                                              \
  } while (0)

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  const size_t sizes[] = {(size_t)2228224, (size_t)8 << 20};
  struct K { const char* name; unsigned flags; };
  const K kinds[] = {{"mapped_noncoherent", hipHostMallocMapped | hipHostMallocPortable | hipHostMallocNonCoherent},
                     {"mapped_coherent", hipHostMallocMapped | hipHostMallocPortable},
                     {"portable", hipHostMallocPortable},
                     {"default", hipHostMallocDefault}};
  printf("{");
  bool first = true;
  for (size_t n : sizes) {
    void* d;
    CK(hipMalloc(&d, n));
    std::vector<unsigned char> page(n, 1);
    for (int k = -1; k < 4; ++k) {
      void* h = page.data();
      if (k >= 0) CK(hipHostMalloc(&h, n, kinds[k].flags));
      for (int dir = 0; dir < 2; ++dir) {
        std::vector<double> t;
        for (int r = 0; r < 23; ++r) {
          const auto t0 = std::chrono::steady_clock::now();
          if (dir) CK(hipMemcpyAsync(h, d, n, hipMemcpyDeviceToHost, s));
          else CK(hipMemcpyAsync(d, h, n, hipMemcpyHostToDevice, s));
          CK(hipStreamSynchronize(s));
          if (r >= 3) t.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(t.begin(), t.end());
        printf("%s\"%s_%zuK_%s\": %.1f", first ? "" : ", ", dir ? "d2h" : "h2d", n >> 10, k < 0 ? "pageable" : kinds[k].name,
               t[t.size() / 2]);
        first = false;
      }
      if (k >= 0) CK(hipHostFree(h));
    }
    CK(hipFree(d));
  }
  printf("}\n");
  return 0;
}
