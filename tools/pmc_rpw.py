#!/usr/bin/env python3
"""Workload for the PMC passes of the config-2 GEMV (tools/pmc_gemv_single.sh): 20 single
4096x4096 q4_0 calls rotating over 33 weight copies (the row-per-wave kernel bench.py's headline
times), then 5 launches of the same kernel over all 33 copies at once (312 MB > MALL: the
calibration run -- same access pattern, a byte count no cache can absorb)."""
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
os.environ["LAMM_GEMV_RPW"] = "16"   # the same kernel (16 waves, as the single calls) over 33 slices in one launch
bt = la.Batch(sl, 1, sl, 1, M * arow, sl * M * arow, 34 * kb, sl * 34 * kb, 4 * M, 4 * M * sl)
for _ in range(5):
    la.matmul_batched(la.Matrix(A.data_ptr(), t, M, kb, kb), Bm, la.Matrix(C.data_ptr(), la.F32, M, 1, M), bt, s)
torch.cuda.synchronize()
print("ok")
