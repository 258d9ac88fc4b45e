#!/usr/bin/env python3
"""Timing of the F32 / F16 prefill GEMM (lamm_gemm_dense.hip) on a few shapes, with torch's
own matmul (hipBLASLt) on the same shape as a yardstick.  Prints one JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
import lamm_amd as la  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    out = {}
    shapes = [("f32", 512, 512, 512, 1), ("f32", 4096, 512, 4096, 1), ("f16", 4096, 512, 4096, 1),
              ("f16", 4096, 4096, 4096, 1), ("f16", 512, 512, 128, 32), ("f16", 4096, 512, 128, 32)]
    for name, M, N, K, S in shapes:
        t = la.BY_NAME[name]
        dt = torch.float32 if name == "f32" else torch.float16
        a = torch.randn(S, M, K, device="cuda").to(dt)
        b = torch.randn(S, N, K, device="cuda").to(dt)
        c = torch.empty(S, N, M, device="cuda", dtype=torch.float32)
        eb = a.element_size()
        bt = la.Batch(S, 1, S, 1, M * K * eb, S * M * K * eb, N * K * eb, S * N * K * eb, 4 * M * N, 4 * M * N * S)
        us = timeit(lambda: la.mul_mat_torch(t, a.view(torch.uint8), b.view(torch.uint8), c, M, N, K, batch=bt))
        ref = torch.bmm(b.float(), a.float().transpose(1, 2))
        err = ((c - ref).abs().max() / ref.abs().max()).item()
        us_t = timeit(lambda: torch.bmm(b, a.transpose(1, 2)))
        fl = 2.0 * M * N * K * S
        out[f"{name}_{M}x{N}x{K}x{S}"] = {"us": round(us, 2), "TFLOPs": round(fl / us / 1e6, 1),
                                          "torch_us": round(us_t, 2), "torch_TFLOPs": round(fl / us_t / 1e6, 1),
                                          "max_err_rel": err}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
