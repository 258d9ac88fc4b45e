#!/usr/bin/env python3
"""Single-call decode GEMV per weight format (config 2's measurement: ONE M x 1 x K GEMV per step,
the steps rotating over weight copies > the 256 MiB MALL, the kernel alone over 1000
graph-replayed launches): algorithmic bytes (A + B + C) / per-launch time.  One JSON line.
usage: python tools/bench_gemv_n.py [fmt,fmt,...] [M] [K]"""
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
    fmts = (sys.argv[1] if len(sys.argv) > 1 else "q4_0,q4_k,q5_k,q6_k,f16").split(",")
    M = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    K = int(sys.argv[3]) if len(sys.argv) > 3 else 4096
    ctx = bench.Ctx(torch, la)
    out = {"M": M, "K": K}
    for f in fmts:
        g = bench.config2_gemv(ctx, f, M, K, 50, 5)
        out[f] = {"us": round(g["kern"] * 1e6, 3), "GBs": round(g["slab_bytes"] / g["kern"] / 1e9, 1),
                  "frac": round(g["slab_bytes"] / g["kern"] / 1e9 / bench.HBM_PEAK_GBS, 4)}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
