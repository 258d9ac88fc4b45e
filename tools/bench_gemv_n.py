#!/usr/bin/env python3
"""GEMV (decode) timing vs the number of activation rows N = 1..8 per weight format:
algorithmic bytes (A + B + C) / kernel time, weights > MALL per launch.  One JSON line."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "la-llama.cpp_amd"))
sys.path.insert(0, ROOT)
import lamm_amd as la  # noqa: E402
import bench  # noqa: E402


def main():
    fmts = (sys.argv[1] if len(sys.argv) > 1 else "q4_0,q8_0,q4_k,q6_k,f16").split(",")
    M = K = 4096
    out = {}
    for f in fmts:
        out[f] = {}
        for N in [int(n) for n in os.environ.get("NS", "1,2,4,8").split(",")]:
            u = bench.gemv_bytes(la, f, M, K, N)
            sl = max(4, -(-int(1.15 * bench.MALL_BYTES) // u))
            _, _, kk = bench.run_case(torch, la, None, f, M, N, K, sl, 10, 2, 1)
            out[f][N] = {"GBs": round(sl * u / kk / 1e9, 1), "us_per_slice": round(kk / sl * 1e6, 3)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
