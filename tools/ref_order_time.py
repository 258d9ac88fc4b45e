#!/usr/bin/env python3
"""Per-launch time of the reference-order kernels (csrc/lamm_ref.hip) against the fast engines on
the shapes the ggml boundary sends them: Llama-7B decode (N = 1) and prefill (N = 64 / 512)
projections, and the q6_K output.weight.  HIP events over 20 launches each (after 3 warm-up)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def timed(fn, n=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / n


out = {}
for fmt, M, K, Ns in (("q4_0", 4096, 4096, (1, 64, 512)), ("q4_0", 11008, 4096, (1, 512)), ("q4_0", 4096, 11008, (1, 512)),
                      ("q6_k", 32000, 4096, (1, 64))):
    t = la.BY_NAME[fmt]
    vt = la.vec_dot_type(t)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(5)
    A, _ = bench.make_weights(torch, la, fmt, 1, M, K, gen)
    for N in Ns:
        x = torch.randn(N, K, device="cuda", generator=gen)
        B = torch.zeros(N * la.row_bytes(vt, K) + 64, dtype=torch.uint8, device="cuda")
        la.quantize_torch(vt, x, B, flavour=1)
        C = torch.zeros(N * M, dtype=torch.float32, device="cuda")
        ref = timed(lambda: la.mul_mat_torch(t, A, B, C, M, N, K, flags=la.ORDER_REFERENCE))
        fast = timed(lambda: la.mul_mat_torch(t, A, B, C, M, N, K))
        out[f"{fmt}_{M}x{N}x{K}"] = {"reference_order_us": round(ref, 2), "fast_us": round(fast, 2),
                                     "fast_engine": la.gemm_engine(fmt, M, N, K)}
        print(f"{fmt} {M}x{N}x{K}: reference order {ref:.2f} us, fast {fast:.2f} us", flush=True)
print(json.dumps(out))
