// xfer_probe.hip -- prefill-sized host<->device transfers through the ggml boundary: the
// activations (512 x 4096 F32 = 8 MiB) up and C (8 MiB) down, from / to ordinary (pageable)
// host memory as ggml hands it over.  Median of 20 of each, us:
//   pageable      : hipMemcpyAsync straight from / to the pageable buffer + sync
//   reg_per_call  : hipHostRegister, hipMemcpyAsync, hipHostUnregister (pinned for the call only)
//   registered    : hipMemcpyAsync on an already registered buffer (the transfer alone)
//   via_pinned    : host memcpy into / out of a pinned staging buffer + DMA
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#define CK(x)                                                          \
  do {                                                                 \
    hipError_t e = (x);                                                \
    if (e != hipSuccess) {                                             \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));           \
      exit(1);                                                         \
    }                                                                  \
  } while (0)

template <class F>
double med(F&& f) {
  std::vector<double> t;
  for (int r = 0; r < 23; ++r) {
    const auto t0 = std::chrono::steady_clock::now();
    f();
    const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count();
    if (r >= 3) t.push_back(us);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main() {
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  printf("{");
  const size_t sizes[] = {(size_t)512 << 10, (size_t)8 << 20};
  for (size_t n : sizes) {
    void* d;
    CK(hipMalloc(&d, n));
    std::vector<unsigned char> page(n + 4096, 1);
    unsigned char* h = page.data();
    void* pin;
    CK(hipHostMalloc(&pin, n, hipHostMallocDefault));
    for (int dir = 0; dir < 2; ++dir) {
      const hipMemcpyKind k = dir ? hipMemcpyDeviceToHost : hipMemcpyHostToDevice;
      auto cp = [&](void* host) {
        if (dir) CK(hipMemcpyAsync(host, d, n, k, s));
        else CK(hipMemcpyAsync(d, host, n, k, s));
        CK(hipStreamSynchronize(s));
      };
      const char* name = dir ? "d2h" : "h2d";
      printf("%s\"%s_%zuK_pageable\": %.1f", (n == sizes[0] && !dir) ? "" : ", ", name, n >> 10, med([&] { cp(h); }));
      printf(", \"%s_%zuK_reg_per_call\": %.1f", name, n >> 10, med([&] {
               CK(hipHostRegister(h, n, hipHostRegisterDefault));
               cp(h);
               CK(hipHostUnregister(h));
             }));
      CK(hipHostRegister(h, n, hipHostRegisterDefault));
      printf(", \"%s_%zuK_registered\": %.1f", name, n >> 10, med([&] { cp(h); }));
      CK(hipHostUnregister(h));
      printf(", \"%s_%zuK_via_pinned\": %.1f", name, n >> 10, med([&] {
               if (!dir) memcpy(pin, h, n);
               cp(pin);
               if (dir) memcpy(h, pin, n);
             }));
    }
    CK(hipHostFree(pin));
    CK(hipFree(d));
  }
  // 2D copies from / to pageable memory, as the boundary issues them: 512 rows x 16 KiB with the
  // pitch equal to the width (a dense F32 activation / C block), and 4096 rows x 1 KiB at a
  // 1280-byte pitch (b2430's transposed V-cache view at n_kv = 512, n_ctx = 640); "lin" = the
  // same bytes as one linear copy of the whole span
  struct R2 { const char* name; size_t rows, width, pitch; };
  const R2 shapes[] = {{"dense_512x16K", 512, 16384, 16384}, {"vview_4096x1K_p1280", 4096, 1024, 1280}};
  for (const R2& r : shapes) {
    const size_t span = r.rows * r.pitch;
    void* d;
    CK(hipMalloc(&d, span));
    std::vector<unsigned char> page(span + 4096, 1);
    unsigned char* h = page.data();
    printf(", \"h2d_2d_%s\": %.1f", r.name, med([&] {
             CK(hipMemcpy2DAsync(d, r.pitch, h, r.pitch, r.width, r.rows, hipMemcpyHostToDevice, s));
             CK(hipStreamSynchronize(s));
           }));
    printf(", \"d2h_2d_%s\": %.1f", r.name, med([&] {
             CK(hipMemcpy2DAsync(h, r.pitch, d, r.pitch, r.width, r.rows, hipMemcpyDeviceToHost, s));
             CK(hipStreamSynchronize(s));
           }));
    printf(", \"h2d_lin_%s\": %.1f", r.name, med([&] {
             CK(hipMemcpyAsync(d, h, span, hipMemcpyHostToDevice, s));
             CK(hipStreamSynchronize(s));
           }));
    CK(hipFree(d));
  }
  // Overlap of the two directions, as a pipelined prefill call would use them: 8 MiB up from one
  // pageable buffer and 8 MiB down into another, one after the other on one stream ("seq"), on two
  // streams issued back to back ("2s"), and in 4 chunks alternating between the streams ("4c")
  {
    const size_t n = (size_t)8 << 20, nc = n / 4;
    void *du, *dd;
    CK(hipMalloc(&du, n));
    CK(hipMalloc(&dd, n));
    std::vector<unsigned char> up(n + 4096, 1), dn(n + 4096, 2);
    hipStream_t s2;
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    printf(", \"updown_seq\": %.1f", med([&] {
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
             CK(hipMemcpyAsync(dn.data(), dd, n, hipMemcpyDeviceToHost, s));
             CK(hipStreamSynchronize(s));
           }));
    printf(", \"updown_2s\": %.1f", med([&] {
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
             CK(hipMemcpyAsync(dn.data(), dd, n, hipMemcpyDeviceToHost, s2));
             CK(hipStreamSynchronize(s));
             CK(hipStreamSynchronize(s2));
           }));
    printf(", \"updown_4c\": %.1f", med([&] {
             for (int c = 0; c < 4; ++c) {
               CK(hipMemcpyAsync((char*)du + c * nc, up.data() + c * nc, nc, hipMemcpyHostToDevice, s));
               CK(hipMemcpyAsync(dn.data() + c * nc, (char*)dd + c * nc, nc, hipMemcpyDeviceToHost, s2));
             }
             CK(hipStreamSynchronize(s));
             CK(hipStreamSynchronize(s2));
           }));
    // the host-side cost of issuing the 8 MiB pageable upload alone (does the call return before
    // the bytes have moved?)
    printf(", \"h2d_issue_only\": %.1f", med([&] {
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
           }));
    CK(hipStreamSynchronize(s));
    // the same with both host buffers registered: for the whole run ("reg"), or around each call
    // ("regpc": register, move, unregister -- what a boundary call could do with ggml's buffers)
    CK(hipHostRegister(up.data(), n, hipHostRegisterDefault));
    CK(hipHostRegister(dn.data(), n, hipHostRegisterDefault));
    printf(", \"updown_reg_seq\": %.1f", med([&] {
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
             CK(hipMemcpyAsync(dn.data(), dd, n, hipMemcpyDeviceToHost, s));
             CK(hipStreamSynchronize(s));
           }));
    printf(", \"updown_reg_2s\": %.1f", med([&] {
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
             CK(hipMemcpyAsync(dn.data(), dd, n, hipMemcpyDeviceToHost, s2));
             CK(hipStreamSynchronize(s));
             CK(hipStreamSynchronize(s2));
           }));
    printf(", \"updown_reg_4c\": %.1f", med([&] {
             for (int c = 0; c < 4; ++c) {
               CK(hipMemcpyAsync((char*)du + c * nc, up.data() + c * nc, nc, hipMemcpyHostToDevice, s));
               CK(hipMemcpyAsync(dn.data() + c * nc, (char*)dd + c * nc, nc, hipMemcpyDeviceToHost, s2));
             }
             CK(hipStreamSynchronize(s));
             CK(hipStreamSynchronize(s2));
           }));
    printf(", \"h2d_reg_issue_only\": %.1f", med([&] {
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
           }));
    CK(hipStreamSynchronize(s));
    CK(hipHostUnregister(up.data()));
    CK(hipHostUnregister(dn.data()));
    printf(", \"updown_regpc_2s\": %.1f", med([&] {
             CK(hipHostRegister(up.data(), n, hipHostRegisterDefault));
             CK(hipHostRegister(dn.data(), n, hipHostRegisterDefault));
             CK(hipMemcpyAsync(du, up.data(), n, hipMemcpyHostToDevice, s));
             CK(hipMemcpyAsync(dn.data(), dd, n, hipMemcpyDeviceToHost, s2));
             CK(hipStreamSynchronize(s));
             CK(hipStreamSynchronize(s2));
             CK(hipHostUnregister(up.data()));
             CK(hipHostUnregister(dn.data()));
           }));
    // registering a range that overlaps a registered one (two tensors sharing a page)
    CK(hipHostRegister(up.data(), n / 2 + 100, hipHostRegisterDefault));
    const hipError_t eo = hipHostRegister(up.data() + n / 2, n / 2, hipHostRegisterDefault);
    printf(", \"overlapping_register\": \"%s\"", hipGetErrorString(eo));
    if (eo == hipSuccess) CK(hipHostUnregister(up.data() + n / 2));
    (void)hipGetLastError();
    CK(hipHostUnregister(up.data()));
    CK(hipStreamDestroy(s2));
    CK(hipFree(du));
    CK(hipFree(dd));
  }
  printf("}\n");
  return 0;
}
