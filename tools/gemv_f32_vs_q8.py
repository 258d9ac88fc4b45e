#!/usr/bin/env python3
"""One q4_0 decode GEMV per step at the Llama-7B projection sizes, graph-replayed over weight
copies beyond the MALL: activations given as q8_0 rows vs as F32 (quantized inside the GEMV, the
decode step's fused form).  Per-launch us; one JSON line.
usage: python tools/gemv_f32_vs_q8.py [M,K M,K ...]"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def run(M, K, act):
    ctx = bench.Ctx(torch, la)
    t = la.Q4_0
    kb = K // 32
    rb = la.row_bytes(t, K)
    R = max(8, -(-int(1.15 * bench.MALL_BYTES) // (M * rb)))
    gen = torch.Generator(device="cuda")
    gen.manual_seed(11)
    A, _ = bench.make_weights(torch, la, "q4_0", R, M, K, gen)
    x = torch.randn(1, K, device="cuda", generator=gen)
    if act == "q8":
        B = torch.zeros(la.row_bytes(la.Q8_0, K) + 16, dtype=torch.uint8, device="cuda")
        la.quantize_torch(la.Q8_0, x, B, flavour=1)
        Bm = la.Matrix(B.data_ptr(), la.Q8_0, kb, 1, kb)
    else:
        B = x.contiguous()
        Bm = la.Matrix(B.data_ptr(), la.F32, K, 1, K)
    C = torch.zeros(M, dtype=torch.float32, device="cuda")
    Cm = la.Matrix(C.data_ptr(), la.F32, M, 1, M)
    mats = [la.Matrix(A.data_ptr() + c * M * rb, t, M, kb, kb) for c in range(R)]

    def step(i):
        la.matmul(mats[i % R], Bm, Cm, torch.cuda.current_stream().cuda_stream)

    _, ev, _ = bench.time_steps(ctx, step, 200, 5)
    return round(ev * 1e6, 3)


def main():
    shapes = [tuple(int(v) for v in a.split(",")) for a in sys.argv[1:]] or [(4096, 4096), (12288, 4096),
                                                                               (22016, 4096), (4096, 11008)]
    out = {}
    for M, K in shapes:
        out[f"{M}x{K}"] = {"q8_us": run(M, K, "q8"), "f32_us": run(M, K, "f32")}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
