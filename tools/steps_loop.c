/* steps_loop.c -- a C caller of the plug-in API that issues K lamm_hip_matmul calls back to back
 * (what a C host such as llama.cpp does per token), so bench.py can time K steps without
 * Python/ctypes submission (~5 us per call) or a hipGraph replay's start-up in the timed region.
 *   gcc -O2 -shared -fPIC -I include tools/steps_loop.c -L la-llama.cpp_amd -llamm_hip ... */
#include "lamm_hip.h"

/* step s multiplies A[(first + s) % nA] by B into C; returns the first non-OK status */
int lamm_steps_matmul(const lamm_matrix *A, int nA, const lamm_matrix *B, const lamm_matrix *C, int first,
                      int steps, void *stream) {
  for (int s = 0; s < steps; ++s) {
    int rc = lamm_hip_matmul(&A[(first + s) % nA], B, C, stream);
    if (rc != LAMM_OK) return rc;
  }
  return LAMM_OK;
}
