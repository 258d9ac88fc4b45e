#!/usr/bin/env python3
"""Whole-launch time (hipGraph-replayed, bench.config3_gemm) of the non-fp6 prefill engines at
N = 512: q6_k 32000 x 4096 (Llama's output.weight, super-block engine), q4_k 4096 x 4096
(super-block), q8_0 4096 x 4096 (MFMA-i8).  Run once per library (LAMM_HIP_LIB) to A/B a build
variant; prints one JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402

SHAPES = [("q6_k", 32000, 512, 4096), ("q4_k", 4096, 512, 4096), ("q8_0", 4096, 512, 4096)]


def main():
    ctx = bench.Ctx(torch, la)
    out = {"lib": os.environ.get("LAMM_HIP_LIB", "default")}
    for fmt, M, N, K in SHAPES:
        _, kern, _, _, _ = bench.config3_gemm(ctx, fmt, M, N, K, 1, 20)
        out[f"{fmt}_{M}x{N}x{K}"] = {"us": round(kern * 1e6, 2), "engine": la.gemm_engine(fmt, M, N, K, 1, stationary=True),
                                     "TOPs": round(2.0 * M * N * K / kern / 1e12, 1)}
        print(fmt, out[f"{fmt}_{M}x{N}x{K}"], flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
