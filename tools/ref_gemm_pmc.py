#!/usr/bin/env python3
"""Launch only the reference-order prefill GEMM (q4_0 4096 x 512 x 4096, ref_mfma2_kernel) and the
F16 attention kernel 10 times each -- the program rocprofv3 --pmc passes count (tools/gpu_pmc_ref.sh)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402

gen = torch.Generator(device="cuda")
gen.manual_seed(7)
t, M, N, K = la.Q4_0, 4096, 512, 4096
A, _ = bench.make_weights(torch, la, "q4_0", 1, M, K, gen)
x = torch.randn(N, K, device="cuda", generator=gen)
B = torch.zeros(N * la.row_bytes(la.Q8_0, K) + 64, dtype=torch.uint8, device="cuda")
la.quantize_torch(la.Q8_0, x, B, flavour=1)
C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
for _ in range(10):
    la.mul_mat_torch(t, A, B, C, M, N, K, flags=la.ORDER_REFERENCE)
H, M2, N2, K2 = 32, 512, 512, 128
A2 = (torch.randn(H * M2 * K2, device="cuda", generator=gen) * 0.3).half().view(torch.uint8)
B2 = torch.randn(H * N2 * K2, device="cuda", generator=gen).half().view(torch.uint8)
C2 = torch.zeros(H * N2 * M2, dtype=torch.float32, device="cuda")
bt = la.Batch(H, 1, H, 1, 2 * M2 * K2, 2 * M2 * K2 * H, 2 * N2 * K2, 2 * N2 * K2 * H, 4 * M2 * N2, 4 * M2 * N2 * H)
for _ in range(10):
    la.mul_mat_torch(la.F16, A2, B2, C2, M2, N2, K2, batch=bt, flags=la.ORDER_REFERENCE)
torch.cuda.synchronize()
print("done")
