#!/usr/bin/env python3
"""Workload for the PMC passes of config 3's fp6 GEMM (tools/pmc_config3.sh):
Q4_0 x Q8_0 M=4096 N=512 K=4096 with stationary weights (the packed fp6 form resident, as bench.py's
config 3), 30 calls = 30 x (prep_b_fp6_tile + gemm_fp6_kv_kernel)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402

fmt = sys.argv[1] if len(sys.argv) > 1 else "q4_0"
M, N, K = 4096, 512, 4096
t = la.BY_NAME[fmt]
gen = torch.Generator(device="cuda")
gen.manual_seed(21)
A, arow = bench.make_weights(torch, la, fmt, 1, M, K, gen)
B = bench.make_activations(torch, la, fmt, N, K, gen)
C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
W = la.Weights(t, A, M, K)
s = torch.cuda.current_stream().cuda_stream
for _ in range(30):
    W.matmul_torch(B, C, N, stream=s)
torch.cuda.synchronize()
W.close()
print("ok", la.gemm_engine(fmt, M, N, K, 1, stationary=True))
