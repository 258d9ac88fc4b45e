"""Config 3 (q4_0 4096 x 512 x 4096) per-call GEMM under whatever LAMM_GEMM_PATH says: 50 graph-replayed
launches (the PMC passes of tools/gpu_dq7.sh attribute counters per kernel)."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "la-llama.cpp_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import lamm_amd as la  # noqa: E402
from bench import make_weights, make_activations  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "q4_0"
M, N, K = 4096, 512, 4096
t = la.BY_NAME[fmt]
gen = torch.Generator(device="cuda")
gen.manual_seed(21)
A, rb = make_weights(torch, la, fmt, 1, M, K, gen)
B = make_activations(torch, la, fmt, N, K, gen)
C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
for _ in range(50):
    la.mul_mat_torch(t, A, B, C, M, N, K)
torch.cuda.synchronize()
print(la.gemm_engine(fmt, M, N, K), "ok")
