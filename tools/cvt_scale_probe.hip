// Probe: what v_cvt_scalef32_pk_f16_fp8 does with a non-power-of-two f32 scale (all of it, or only
// its exponent?), on e4m3 codes of the small integers a 4- / 5-bit weight quant takes.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
__global__ void k(const unsigned* in, float* out, float s) {
  const unsigned x = in[threadIdx.x];
  const h2 a = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(x, s, false);
  const h2 b = __builtin_amdgcn_cvt_scalef32_pk_f16_fp8(x, s, true);
  out[4 * threadIdx.x + 0] = (float)a[0];
  out[4 * threadIdx.x + 1] = (float)a[1];
  out[4 * threadIdx.x + 2] = (float)b[0];
  out[4 * threadIdx.x + 3] = (float)b[1];
}
int main() {
  // e4m3 (OCP): 1.0 = 0x38, 2 = 0x40, 3 = 0x44, 5 = 0x4A, 7 = 0x4E, -8 = 0xD0, 15 = 0x57, -16 = 0xD8
  unsigned h[2] = {0x4A443840u, 0xD857D04Eu};
  unsigned* d;
  float* o;
  hipMalloc(&d, sizeof h);
  hipMalloc(&o, 8 * sizeof(float));
  hipMemcpy(d, h, sizeof h, hipMemcpyHostToDevice);
  const float scales[3] = {1.0f, 0.3f, 0.0123456f * 256.f};
  for (float s : scales) {
    hipLaunchKernelGGL(k, dim3(1), dim3(2), 0, 0, d, o, s);
    float r[8];
    hipMemcpy(r, o, sizeof r, hipMemcpyDeviceToHost);
    printf("scale %.9g:", s);
    for (float v : r) printf(" %.9g", v);
    printf("   expect x:");
    const float x[8] = {1, 2, 3, 5, 7, -8, 15, -16};
    for (float v : x) printf(" %.9g", (float)(_Float16)(v * s));
    printf("\n");
  }
  return 0;
}
