#!/usr/bin/env python3
"""Workload for the PMC passes of the config-2 GEMV (tools/pmc_flat1.sh): 20 single 4096x4096 q4_0
calls rotating over 33 weight copies -- gemv_flat1_kernel, the kernel bench.py's headline times --
then 5 launches over all 33 copies at once (gemv_flat_kernel with the slice offsets: the same body
and access pattern, 312 MB > MALL read once -- the FETCH_SIZE calibration)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402

M = K = 4096
t = la.Q4_0
kb = K // 32
sl = 33
gen = torch.Generator(device="cuda")
gen.manual_seed(3)
A, arow = bench.make_weights(torch, la, "q4_0", sl, M, K, gen)
B = bench.make_activations(torch, la, "q4_0", sl, K, gen)
C = torch.zeros(sl * M, dtype=torch.float32, device="cuda")
s = torch.cuda.current_stream().cuda_stream
Bm = la.Matrix(B.data_ptr(), la.Q8_0, kb, 1, kb)
for r in range(20):
    la.matmul(la.Matrix(A.data_ptr() + (r % sl) * M * arow, t, M, kb, kb), Bm, la.Matrix(C.data_ptr(), la.F32, M, 1, M), s)
torch.cuda.synchronize()
os.environ["LAMM_GEMV_RPW"] = "8"   # the flat kernel (8 waves) over the 33 slices, not the wave-group stream
bt = la.Batch(sl, 1, sl, 1, M * arow, sl * M * arow, 34 * kb, sl * 34 * kb, 4 * M, 4 * M * sl)
for _ in range(5):
    la.matmul_batched(la.Matrix(A.data_ptr(), t, M, kb, kb), Bm, la.Matrix(C.data_ptr(), la.F32, M, 1, M), bt, s)
torch.cuda.synchronize()
print("ok")
